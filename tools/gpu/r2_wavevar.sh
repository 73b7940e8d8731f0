#!/bin/bash
# wave-kernel variants: bench ph2o45 / oh24 per library (product + liblvg_amd_v<k>.so), exactness on ph2o45.
set -o pipefail
OUT=gpurun_out/r2wv
mkdir -p $OUT
for k in prod "$@"; do
  if [ "$k" = prod ]; then L=""; else L=$PWD/radiative_transfer_amd/_lib/liblvg_amd_v$k.so; fi
  for w in ph2o45_1024 oh24_overlap_2048; do
    LVG_LIB_PATH=$L timeout -k 10 200 python bench.py --workload $w --steps 3 --no-cpu --no-host-entry > $OUT/b_${k}_$w.json 2> $OUT/b_${k}_$w.err || exit 1
    LVG_LIB_PATH=$L timeout -k 10 200 python tools/variant_check.py $w 256 > $OUT/x_${k}_$w.txt 2>&1 || { cat $OUT/x_${k}_$w.txt; exit 1; }
    python -c "import json; b=json.load(open('$OUT/b_${k}_$w.json')); print('$k', '$w', round(b['value']), round(b['roofline']['kernel_ms'],3), open('$OUT/x_${k}_$w.txt').read().strip())"
  done
done
