# rocprofv3 passes for one bench workload (run on the GPU box from the repo root):
#   1) kernel trace + stats          2) PMC FETCH_SIZE          3) PMC WRITE_SIZE
# PMC passes are separate (slot limits) and never combined with sys/runtime traces.
# usage: tools/profile.sh TAG [WORKLOAD]   -> gpurun_out/prof_TAG_WORKLOAD/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2}
WL=${2:-ch3oha256_4096}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
B="python3 bench.py --workload $WL --no-cpu --no-host-entry --no-provenance"   # no rocm-smi child under the profiler
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    $B --steps 3 --warmup 1 > $OUT/bench_trace.json 2> $OUT/trace.err && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    $B --steps 2 --warmup 1 > $OUT/bench_fetch.json 2> $OUT/fetch.err && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    $B --steps 2 --warmup 1 > $OUT/bench_write.json 2> $OUT/write.err
rc=$?
echo "profile $WL rc=$rc"
exit $rc
