#!/bin/bash
# Instruction-cache behaviour of the solve kernels (SQC counters, one rocprofv3 --pmc pass per
# workload, kernel-trace only): hits and misses of the shared instruction cache against the
# instructions fetched.
set -o pipefail
export TMPDIR=/tmp
for wl in ${WLS:-ch3oha256_4096 ph2o45_1024}; do
  OUT=gpurun_out/pmc_icache_$wl
  mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU \
      --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-host-entry \
      --no-provenance $BARGS --workload $wl > $OUT/b1.json 2> $OUT/p1.err || { tail -5 $OUT/p1.err; exit 2; }
  python3 - <<PY
import csv
rows = [r for r in csv.DictReader(open("$OUT/p1/run_counter_collection.csv")) if "solve" in r["Kernel_Name"]]
i = sorted(set(r["Dispatch_Id"] for r in rows), key=int)[-1]
d = {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows if r["Dispatch_Id"] == i}
print("$wl", " ".join(f"{k}={v:.4g}" for k, v in d.items()))
PY
done
