#!/bin/bash
# Wave kernel (N <= 64): SQ wait/issue shares (tools/gpu/pmc_wait.sh) and the instruction mix of
# the two small BASELINE configs, one rocprofv3 --pmc pass each (kernel-trace only).
set -o pipefail
export TMPDIR=/tmp
for wl in ph2o45_1024 oh24_overlap_2048; do
  bash tools/gpu/pmc_wait.sh wave_$wl --workload $wl || exit 1
  OUT=gpurun_out/pmc_mix_$wl
  mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES \
      --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-host-entry \
      --no-provenance --workload $wl > $OUT/b1.json 2> $OUT/p1.err || exit 2
  python3 - <<PY
import csv
rows = [r for r in csv.DictReader(open("$OUT/p1/run_counter_collection.csv")) if "solve" in r["Kernel_Name"]]
i = sorted(set(r["Dispatch_Id"] for r in rows), key=int)[-1]
d = {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows if r["Dispatch_Id"] == i}
print("$wl", " ".join(f"{k}={v:.4g}" for k, v in d.items()))
PY
done
