# occupancy experiment: phase timers at 1 and 2 workgroups per CU
set -o pipefail
cd /root/repo
LVG_BLOCKS_PER_CU=1 timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_1wg.log 2>&1 && \
LVG_BLOCKS_PER_CU=2 timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_2wg.log 2>&1
rc=$?
cat gpurun_out/phase_1wg.log gpurun_out/phase_2wg.log
exit $rc
