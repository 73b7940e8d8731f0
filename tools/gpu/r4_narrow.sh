#!/bin/bash
# round 4: the one-wave (narrow) kernel: exactness on several shapes with narrow forced,
# then the metric bench (narrow chosen automatically) against narrow=0, ABAB.
set -o pipefail
OUT=gpurun_out/${TAG:-r4_narrow}
mkdir -p $OUT
chk() { LVG_TUNING=narrow=2 timeout -k 10 ${CT:-180} python tools/variant_check.py "$@" > $OUT/chk_$(echo "$@" | tr ' ' _).txt 2>&1; rc=$?;
        echo "check $*: rc=$rc $(tail -1 $OUT/chk_$(echo "$@" | tr ' ' _).txt)"; return $rc; }
chk ch3oha256_4096 16 || exit 1
chk ch3oha256_4096 96 || exit 1
chk ch3oha256_4096 12 150 || exit 1
chk ch3oha256_4096 12 77 || exit 1
chk ch3ohe256_sweep 64 || exit 1
for rep in 1 2; do
  for v in n1 n0; do
    tun=""; [ $v = n0 ] && tun="narrow=0"
    LVG_TUNING=$tun timeout -k 10 300 python bench.py --no-cpu --no-host-entry --no-provenance --steps ${STEPS:-10} \
      > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || { tail -5 $OUT/bench_${v}_$rep.err; exit 3; }
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'kernel %.2f ms' % d['roofline']['kernel_ms'], d['roofline'].get('kernel'))"
  done
done
