set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gpu_tests.log
exit $rc
