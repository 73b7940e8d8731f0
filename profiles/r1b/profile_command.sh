# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
#   1) kernel trace + stats          2) PMC FETCH_SIZE          3) PMC WRITE_SIZE
# PMC passes are separate (slot limits) and never combined with sys/runtime traces.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench_trace.json 2> $OUT/trace.err && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_fetch.json 2> $OUT/fetch.err && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_write.json 2> $OUT/write.err
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
