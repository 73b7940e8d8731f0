#!/bin/bash
# Same-box A/B (rounds 5-6): the GPU suite (TESTS), then for the metric workload an exactness check of
# every block-kernel variant (tools/variant_check.py) and ABAB bench lines (REPS x), the 8-way
# share of the 4096-layer cloud for SHARD variants, and the two wave-kernel workloads for WAVEV.
# usage: VARIANTS="prod vbase vX" SHARD="prod vbase" WAVEV="prod vbase" TESTS="tests -m gpu" TAG=... bash tools/gpu/r5_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r6_ab}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
libof() { if [ "$1" = prod ]; then echo $L/liblvg_amd.so; else echo $L/liblvg_amd_$1.so; fi; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
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
for wl in ph2o45_1024 oh24_overlap_2048; do
  for rep in 1 2; do
    for v in $WAVEV; do
      LVG_LIB_PATH=$(libof $v) timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-host-entry --no-provenance \
        --steps 5 > $OUT/bench_${wl}_${v}_$rep.json 2> $OUT/bench_${wl}_${v}_$rep.err || exit 7
      python -c "import json; d=json.loads(open('$OUT/bench_${wl}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$wl $v', round(d['value']), 'kernel %.3f ms' % d['roofline']['kernel_ms'])"
    done
  done
done
