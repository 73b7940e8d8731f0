set -o pipefail
cd /root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-budget 10 > gpurun_out/bench1.log 2> gpurun_out/bench1.err
echo rc=$?
tail -3 gpurun_out/smoke.log; tail -3 gpurun_out/bench1.err; cat gpurun_out/bench1.log
