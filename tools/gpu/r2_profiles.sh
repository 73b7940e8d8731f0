#!/bin/bash
# Bench lines (with CPU legs) and rocprofv3 stats + PMC traffic for the BASELINE workloads.
set -o pipefail
TAG=${TAG:-r2}
mkdir -p gpurun_out/lines_$TAG
for WL in ${WLS:-ch3oha256_4096 ph2o45_1024 ch3ohe256_sweep oh24_overlap_2048}; do
  timeout -k 10 400 python bench.py --workload $WL > gpurun_out/lines_$TAG/$WL.json 2> gpurun_out/lines_$TAG/$WL.err || exit 1
  bash tools/profile.sh $TAG $WL || exit 1
done
echo done
