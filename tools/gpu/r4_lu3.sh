#!/bin/bash
# round 4: exactness of a block-kernel variant on several shapes, then same-box ABAB bench and
# 8-way shares against the product. usage: V=lu3 bash tools/gpu/r4_lu3.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r4_lu3}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
lib=$L/liblvg_amd_v$V.so
chk() { LVG_LIB_PATH=$lib timeout -k 10 ${CT:-180} python tools/variant_check.py "$@" > $OUT/chk_$(echo "$@" | tr ' ' _).txt 2>&1; rc=$?;
        echo "check $*: rc=$rc $(tail -1 $OUT/chk_$(echo "$@" | tr ' ' _).txt)"; return $rc; }
chk ch3oha256_4096 4 || exit 1
chk ch3oha256_4096 96 || exit 1
chk ch3oha256_4096 12 150 || exit 1
chk ch3oha256_4096 12 77 || exit 1
chk ch3ohe256_sweep 64 || exit 1
chk ph2o45_1024 48 || exit 1
for rep in 1 2; do
  for v in prod $V; do
    l2=$L/liblvg_amd.so; [ $v = prod ] || l2=$lib
    LVG_LIB_PATH=$l2 timeout -k 10 300 python bench.py --no-cpu --no-host-entry --no-provenance --steps ${STEPS:-10} \
      > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 3
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'kernel %.2f ms' % d['roofline']['kernel_ms'])"
  done
done
for v in prod $V; do
  l2=$L/liblvg_amd.so; [ $v = prod ] || l2=$lib
  LVG_LIB_PATH=$l2 timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8_$v.txt 2>&1 || exit 4
  echo "$v $(tail -1 $OUT/shard8_$v.txt) $(grep '"rank": 6' $OUT/shard8_$v.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lu_alone_ms", round(d["ms_per_lu_alone"],4))')"
done
