#!/bin/bash
# Round 6 same-box A/B: the GPU suite on the library FULL (every variant switch on), an exactness
# check of each variant (tools/variant_check.py), then ABAB bench lines of the metric workload.
# usage: FULL=vall VARIANTS="prod vcd vcp vall" TAG=... bash tools/gpu/ab_r6b.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r6_ab}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
libof() { if [ "$1" = prod ]; then echo $L/liblvg_amd.so; else echo $L/liblvg_amd_$1.so; fi; }
if [ -n "$FULL" ]; then
  LVG_LIB_PATH=$(libof $FULL) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $OUT/pytest_$FULL.log 2>&1 || { tail -40 $OUT/pytest_$FULL.log; exit 1; }
  tail -1 $OUT/pytest_$FULL.log
fi
for v in $VARIANTS; do
  [ $v = prod ] && continue
  LVG_LIB_PATH=$(libof $v) timeout -k 10 240 python tools/variant_check.py ch3oha256_4096 ${CHK:-48} > $OUT/check_$v.txt 2>&1
  rc=$?; echo "$v check rc=$rc: $(tail -1 $OUT/check_$v.txt)"
  [ $rc -le 1 ] || exit $rc
done
for rep in $(seq ${REPS:-2}); do
  for v in $VARIANTS; do
    LVG_LIB_PATH=$(libof $v) timeout -k 10 300 python bench.py --no-cpu --no-host-entry --no-provenance --steps ${STEPS:-10} \
      > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 3
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'kernel %.3f ms' % d['roofline']['kernel_ms'])"
  done
done
for v in $SHARD; do
  LVG_LIB_PATH=$(libof $v) timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8_$v.txt 2>&1 || exit 4
  echo "$v $(tail -1 $OUT/shard8_$v.txt)"
done
