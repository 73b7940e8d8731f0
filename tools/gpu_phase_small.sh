set -o pipefail
cd /root/repo
timeout -k 10 200 python tools/phase_timers.py ph2o45_1024 1024 > gpurun_out/ph_ph2o.txt 2>&1 && timeout -k 10 200 python tools/phase_timers.py oh24_overlap_2048 2048 > gpurun_out/ph_oh.txt 2>&1
