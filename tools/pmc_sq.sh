# SQ / SQC counters for the solve kernel (separate passes, kernel-trace only)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_${1:-x}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_IFETCH SQ_INSTS --output-format csv -d $OUT/p1 -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --layers 2048 > $OUT/b1.json 2> $OUT/p1.err && \
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ --output-format csv -d $OUT/p2 -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --layers 2048 > $OUT/b2.json 2> $OUT/p2.err
rc=$?
python3 - <<PY
import csv, glob
for f in sorted(glob.glob("$OUT/p*/run_counter_collection.csv")):
    tot = {}
    for r in csv.DictReader(open(f)):
        if "solve_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(f, {k: f"{v:.4g}" for k, v in tot.items()})
PY
exit $rc
