#!/bin/bash
# A/B of a library variant V (radiative_transfer_amd/_lib/liblvg_amd_v$V.so, tools/build_variants.sh)
# against the product library: the Python GPU parity suite on the variant, then alternating
# bench lines on the workloads in WLS. Diagnostic.
set -o pipefail
V=${V:?variant}
OUT=gpurun_out/${VOUT:-r2ab_v$V}
mkdir -p $OUT
VL=radiative_transfer_amd/_lib/liblvg_amd_v$V.so
LVG_LIB_PATH=$VL timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    --deselect tests/test_host_cpp.py::test_host_facade_bit_exact \
    --deselect tests/test_sanitizers_cpu.py::test_abi_host_code_under_asan_ubsan_on_gpu > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in ${WLS:-ph2o45_1024 oh24_overlap_2048}; do
  for v in prod v$V prod v$V; do
    if [ $v = prod ]; then lib=""; else lib=$VL; fi
    LVG_LIB_PATH=$lib timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-host-entry > $OUT/b_${w}_$v.json 2>> $OUT/bench.err || exit 1
    python -c "import json; d=json.load(open('$OUT/b_${w}_$v.json')); print('$w','$v', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
  done
done
