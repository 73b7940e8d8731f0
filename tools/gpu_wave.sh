# wave kernel: parity tests, then a bench line for every BASELINE workload (1 GPU)
set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wave_parity.log 2>&1 || { tail -30 gpurun_out/wave_parity.log; exit 1; }
tail -3 gpurun_out/wave_parity.log
bash tools/gpu_configs.sh
