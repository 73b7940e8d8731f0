#!/bin/bash
# round 4: wave kernel (N <= 64) — GPU tests of the product, then same-box ABAB of the two small
# BASELINE configs against a variant library (V, default the previous product copy "head").
set -o pipefail
OUT=gpurun_out/${TAG:-r4_wave}
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
V=${V:-head}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_level_sweep.py tests/test_gpu_coverage.py tests/test_gpu_chains.py \
     -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for wl in ph2o45_1024 oh24_overlap_2048; do
  for rep in 1 2; do
    for v in prod $V; do
      lib=$L/liblvg_amd.so; [ $v = prod ] || lib=$L/liblvg_amd_v$v.so
      LVG_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-host-entry --no-provenance \
        --steps 5 > $OUT/bench_${wl}_${v}_$rep.json 2> $OUT/bench_${wl}_${v}_$rep.err || exit 7
      python -c "import json; d=json.loads(open('$OUT/bench_${wl}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$wl $v', round(d['value']), 'kernel %.3f ms' % d['roofline']['kernel_ms'])"
    done
  done
done
