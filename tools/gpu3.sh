set -o pipefail
cd /root/repo
timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_ch3oh.log 2>&1 && \
timeout -k 10 300 python tools/phase_timers.py ph2o45_1024 1024 > gpurun_out/phase_h2o.log 2>&1 && \
timeout -k 10 300 python tools/phase_timers.py ph2o45_1024 16 > gpurun_out/phase_h2o16.log 2>&1
echo rc=$?
cat gpurun_out/phase_*.log
