#!/bin/bash
# Underfilled launches (at most one workgroup per CU): product library vs a build of the
# N <= 256 kernel for one workgroup per CU (liblvg_amd_v<k>.so, -DLVG_OCC=1). Diagnostic.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2o}
mkdir -p $OUT
for k in prod "$@"; do
  if [ "$k" = prod ]; then L=""; else L=$PWD/radiative_transfer_amd/_lib/liblvg_amd_v$k.so; fi
  LVG_LIB_PATH=$L timeout -k 10 200 python bench.py --layers 512 --steps 3 --no-cpu --no-host-entry > $OUT/b_${k}_512.json 2> $OUT/b_${k}_512.err || exit 1
  LVG_LIB_PATH=$L timeout -k 10 300 python bench.py --workload ch3ohe256_sweep --chain-len 128 --steps 2 --no-cpu --no-host-entry > $OUT/b_${k}_sweepc.json 2> $OUT/b_${k}_sweepc.err || exit 1
  LVG_LIB_PATH=$L timeout -k 10 200 python bench.py --layers 256 --steps 3 --no-cpu --no-host-entry > $OUT/b_${k}_256.json 2> $OUT/b_${k}_256.err || exit 1
  for c in 512 sweepc 256; do
    python -c "import json; b=json.load(open('$OUT/b_${k}_$c.json')); print('$k', '$c', round(b['value']), round(b['roofline']['kernel_ms'],2))"
  done
done
