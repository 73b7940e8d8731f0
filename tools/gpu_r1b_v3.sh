# exactness on the parity cases that reach the two-wave range (N = 256 and N = 100) + timing
set -o pipefail
cd /root/repo
LVG_LIB_PATH=radiative_transfer_amd/_lib/liblvg_amd_vh.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_vh.log 2>&1 || { tail -30 gpurun_out/gpu_tests_vh.log; exit 1; }
tail -2 gpurun_out/gpu_tests_vh.log
bash tools/gpu_variants.sh
