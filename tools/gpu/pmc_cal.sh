set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_cal
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_FMA_F64 --kernel-trace --output-format csv -d $OUT/p1 -o run -- tools/probe/rate_probe > $OUT/rate.txt 2> $OUT/p1.err
rc=$?
python3 - <<PY
import csv, glob
for f in sorted(glob.glob("$OUT/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    print(rows[0].keys())
    for r in rows:
        print(r.get("Dispatch_Id"), r["Kernel_Name"][:30], r["Counter_Name"], r["Counter_Value"])
for f in sorted(glob.glob("$OUT/p*/run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        print(r.get("Dispatch_Id"), r["Kernel_Name"][:30], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "ns")
PY
exit $rc
