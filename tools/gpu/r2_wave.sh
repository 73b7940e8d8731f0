#!/bin/bash
# Wave-kernel configs: parity subset, then bench lines and the slowest-layer latency.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2w}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chains.py tests/test_gpu_coverage.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in ph2o45_1024 oh24_overlap_2048; do
  timeout -k 10 200 python bench.py --workload $w --steps 3 --no-cpu --no-host-entry > $OUT/b_$w.json 2> $OUT/b_$w.err || exit 1
  python -c "import json; b=json.load(open('$OUT/b_$w.json')); print('$w', round(b['value']), round(b['roofline']['kernel_ms'],3))"
done
timeout -k 10 200 python tools/latency_probe.py ph2o45_1024 | head -2
