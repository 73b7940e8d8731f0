# instruction mix of the solve kernel: available SQ counters, then one pass (kernel-trace only)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mix
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $OUT/avail.txt | sort -u > $OUT/sq_names.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --output-format csv -d $OUT/p1 -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/b1.json 2> $OUT/p1.err
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
