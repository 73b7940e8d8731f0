set -o pipefail
cd /root/repo
LVG_BLOCK_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dbg1.log 2>&1; echo "block rc=$?"; tail -2 gpurun_out/dbg1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k device_resident > gpurun_out/dbg2.log 2>&1; echo "torch-only rc=$?"; tail -2 gpurun_out/dbg2.log
