# final check of the committed product: full GPU suite, smoke, bench line
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { tail -40 gpurun_out/gpu_tests_final.log; exit 1; }
tail -2 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && cat gpurun_out/bench_final.json
