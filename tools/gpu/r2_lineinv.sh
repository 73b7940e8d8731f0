#!/bin/bash
# Wave-kernel line invariants: GPU suite, then A/B bench lines (product vs v0 = per-iteration
# line data, -DLVG_WAVE_LINE_INV=0) on the two wave-kernel configs. Diagnostic.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2li}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in ph2o45_1024 oh24_overlap_2048; do
  for v in prod v0 prod v0; do
    if [ $v = prod ]; then lib=""; else lib=radiative_transfer_amd/_lib/liblvg_amd_$v.so; fi
    LVG_LIB_PATH=$lib timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu > $OUT/b_${w}_$v.json 2>> $OUT/bench.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b_${w}_$v.json')); print('$w','$v', round(d['ms_per_step'],3), d['roofline']['kernel_ms'])"
  done
done
