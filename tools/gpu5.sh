set -o pipefail
cd /root/repo
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err && \
bash tools/profile.sh r1
rc=$?
cat gpurun_out/bench_r1.json
exit $rc
