# Round-1 (session b) measurement pass: smoke, full bench line with the CPU baseline,
# rocprofv3 kernel trace + PMC FETCH/WRITE passes, phase timers.
set -o pipefail
cd /root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
bash tools/profile.sh r1b || exit 1
timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_r1b.txt 2>&1 || { cat gpurun_out/phase_r1b.txt; exit 1; }
cat gpurun_out/phase_r1b.txt
