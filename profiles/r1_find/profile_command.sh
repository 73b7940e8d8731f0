set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_find
timeout -k 10 600 python tools/bench_find.py 4096 > gpurun_out/find.json 2> gpurun_out/find.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_find -o run -- python3 tools/bench_find.py 4096 > gpurun_out/find_prof.json 2> gpurun_out/find_prof.err
rc=$?
cat gpurun_out/find.json
find gpurun_out/prof_find -name "*kernel_stats.csv" -exec head -8 {} \;
exit $rc
