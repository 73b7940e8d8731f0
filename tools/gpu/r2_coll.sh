#!/bin/bash
# Collision operators built ahead (coll_kernel): GPU suite, then A/B bench lines on the
# headline workload (default vs LVG_COLL_AHEAD=0, the per-layer in-kernel build). Diagnostic.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2coll}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in ${WLS:-ch3oha256_4096}; do
  for v in on off on off; do
    if [ $v = on ]; then e=1; else e=0; fi
    LVG_COLL_AHEAD=$e timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-host-entry > $OUT/b_${w}_$v.json 2>> $OUT/bench.err || exit 1
    python -c "import json; d=json.load(open('$OUT/b_${w}_$v.json')); print('$w','$v', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['value']))"
  done
done
