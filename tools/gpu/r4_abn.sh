#!/bin/bash
# round 4: same-box ABAB bench (metric workload) and 8-way shares for several library variants
# (liblvg_amd_v<k>.so, tools/build_variant2.sh) against the product; an exactness check per variant
# first. usage: VS="lu3 lu3p1" bash tools/gpu/r4_abn.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r4_abn}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
lib() { [ $1 = prod ] && echo $L/liblvg_amd.so || echo $L/liblvg_amd_v$1.so; }
for v in $VS; do
  LVG_LIB_PATH=$(lib $v) timeout -k 10 180 python tools/variant_check.py ch3oha256_4096 ${CHK:-64} > $OUT/chk_$v.txt 2>&1 || { echo "$v check failed"; tail -3 $OUT/chk_$v.txt; exit 1; }
  echo "$v check: $(tail -1 $OUT/chk_$v.txt)"
done
for rep in $(seq ${REPS:-2}); do
  for v in prod $VS; do
    LVG_LIB_PATH=$(lib $v) timeout -k 10 300 python bench.py --no-cpu --no-host-entry --no-provenance --steps ${STEPS:-10} $BARGS \
      > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 3
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'kernel %.2f ms' % d['roofline']['kernel_ms'])"
  done
done
if [ -z "$NOSHARD" ]; then
for v in prod $VS; do
  LVG_LIB_PATH=$(lib $v) timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8_$v.txt 2>&1 || exit 4
  echo "$v $(tail -1 $OUT/shard8_$v.txt) $(grep '"rank": 6' $OUT/shard8_$v.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lu_alone_ms", round(d["ms_per_lu_alone"],4))')"
done
fi
