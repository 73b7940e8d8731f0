set -o pipefail
cd /root/repo
timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 4096 > gpurun_out/phase_4096.log 2>&1
rc=$?
cat gpurun_out/phase_4096.log
exit $rc
