#!/bin/bash
# Memory-side PMC of the metric launch (two passes, 4 TCC counters each, kernel trace only): fabric
# read / write requests and the part of them destined for DRAM (the rest are Infinity-Cache hits),
# then the DRAM-credit stall cycles, the L2 hit / miss counts and the GPU-active cycles.
# usage: bash tools/gpu/pmc_dram.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_dram_${1:-x}
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-host-entry --no-provenance"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum \
    --kernel-trace --output-format csv -d $OUT/p1 -o run -- $B > $OUT/b1.json 2> $OUT/p1.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $OUT/p2 -o run -- $B > $OUT/b2.json 2> $OUT/p2.err || exit 2
python3 - <<PY
import csv, glob
for p in ("p1", "p2"):
    f = glob.glob("$OUT/%s/**/*counter_collection.csv" % p, recursive=True)[0]
    tot = {}
    for r in csv.DictReader(open(f)):
        if "solve_kernel" in r["Kernel_Name"]:
            k = (r["Dispatch_Id"], r["Counter_Name"])
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
    for (d, c), v in sorted(tot.items()):
        print(p, d, c, "%.6g" % v)
PY
