#!/bin/bash
# round 4 A/B on one box: exactness of the product build (both block-kernel instantiations
# via the GPU tests), throughput ABAB against variant V (256-thread kernel), 8-way shares
# against variant VW (512-thread kernel). usage: V=o VW=ow TESTS="..." bash tools/gpu/r4_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r4_ab}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for rep in 1 2; do
  for v in prod $V; do
    lib=$L/liblvg_amd.so; [ $v = prod ] || lib=$L/liblvg_amd_v$v.so
    LVG_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu --no-host-entry --no-provenance --steps ${STEPS:-10} \
      > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 3
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'kernel %.2f ms' % d['roofline']['kernel_ms'])"
  done
done
for v in prod $VW; do
  lib=$L/liblvg_amd.so; [ $v = prod ] || lib=$L/liblvg_amd_v$v.so
  LVG_LIB_PATH=$lib timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8_$v.txt 2>&1 || exit 4
  echo "$v $(tail -1 $OUT/shard8_$v.txt) $(grep '"rank": 6' $OUT/shard8_$v.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lu_alone_ms", round(d["ms_per_lu_alone"],4))')"
done
# wave kernel (N <= 64): the two small BASELINE configs, prod vs WV, ABAB
if [ -n "$WV" ]; then
  for wl in ph2o45_1024 oh24_overlap_2048; do
    for rep in 1 2; do
      for v in prod $WV; do
        lib=$L/liblvg_amd.so; [ $v = prod ] || lib=$L/liblvg_amd_v$v.so
        LVG_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-host-entry --no-provenance \
          --steps 5 > $OUT/bench_${wl}_${v}_$rep.json 2> $OUT/bench_${wl}_${v}_$rep.err || exit 7
        python -c "import json; d=json.loads(open('$OUT/bench_${wl}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$wl $v', round(d['value']), 'kernel %.3f ms' % d['roofline']['kernel_ms'])"
      done
    done
  done
fi
if [ -n "$TIMERS" ]; then
  timeout -k 10 300 python tools/latency_timers.py ch3oha256_4096 > $OUT/timers_wide.txt 2>&1 || exit 5
  LVG_TUNING=wide=0 timeout -k 10 300 python tools/latency_timers.py ch3oha256_4096 > $OUT/timers_256.txt 2>&1 || exit 6
  head -1 $OUT/timers_wide.txt; head -1 $OUT/timers_256.txt
fi
