#!/bin/bash
# coll_kernel variants (VS="2 3 4": liblvg_amd_v<k>.so): exactness on 128 CH3OH-A layers
# vs the oracle, then rocprofv3 kernel stats of a short headline bench per library. Diagnostic.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${VOUT:-r2collvar}
mkdir -p $OUT
for v in prod ${VS:-2 3 4}; do
  if [ $v = prod ]; then lib=""; else lib=radiative_transfer_amd/_lib/liblvg_amd_v$v.so; fi
  if [ $v != prod ]; then LVG_LIB_PATH=$lib timeout -k 10 200 python tools/variant_check.py > $OUT/exact_$v.txt 2>&1 || exit 1; cat $OUT/exact_$v.txt; fi
  LVG_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$v -o run -- \
      python3 bench.py --no-cpu --no-host-entry --steps 3 --warmup 1 > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  f=$(find $OUT/t_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -E "coll_kernel|solve_kernel" $f | cut -d, -f1-4
done
