#!/bin/bash
# Where the solve kernel's waves spend their cycles (SQ counters, quad-cycles, kernel-trace only,
# one pass): parked (s_waitcnt / barrier), issue-stalled, issuing, and per instruction type.
# usage: bash tools/gpu/pmc_wait.sh TAG [bench args]   (LVG_LIB_PATH selects a variant)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_wait_${1:-x}
shift
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS \
    --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-host-entry --no-provenance "$@" \
    > $OUT/b1.json 2> $OUT/p1.err
rc=$?
python3 - <<PY
import csv
rows = [r for r in csv.DictReader(open("$OUT/p1/run_counter_collection.csv")) if "solve" in r["Kernel_Name"]]
ids = sorted(set(r["Dispatch_Id"] for r in rows), key=int)
for i in ids:
    d = {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows if r["Dispatch_Id"] == i}
    wc = d["SQ_WAVE_CYCLES"]
    print(i, rows[[r["Dispatch_Id"] for r in rows].index(i)]["Kernel_Name"][:40],
          " ".join(f"{k[3:]}={v / wc:.3f}" for k, v in d.items() if k != "SQ_WAVE_CYCLES"), f"wave_quad={wc:.4g}")
PY
exit $rc
