#!/bin/bash
# Per-GPU load of the strong-scaling runs (4096 layers / N GPUs): kernel time with 2 vs 1
# workgroups per CU. Diagnostic.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2u}
mkdir -p $OUT
for nl in 2048 1024 512; do
  for bpc in 2 1; do
    LVG_BLOCKS_PER_CU=$bpc timeout -k 10 200 python bench.py --layers $nl --steps 3 --no-cpu --no-host-entry > $OUT/b_${nl}_${bpc}.json 2> $OUT/b_${nl}_${bpc}.err || exit 1
    python -c "import json,sys; b=json.load(open('$OUT/b_${nl}_${bpc}.json')); print($nl, $bpc, round(b['value']), round(b['roofline']['kernel_ms'],2))"
  done
done
