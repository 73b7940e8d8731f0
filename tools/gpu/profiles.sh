#!/bin/bash
# Bench lines (with CPU legs) and rocprofv3 stats + PMC traffic for the BASELINE workloads,
# all on one box at one commit: gpurun_out/lines_$TAG/<workload>.json and
# gpurun_out/prof_$TAG_<workload>/ (tools/profile.sh). tools/update_profiles.py copies
# them into profiles/$TAG/ and refreshes profiles/pmc_traffic.json.
set -o pipefail
TAG=${TAG:-r3}
mkdir -p gpurun_out/lines_$TAG
git_rev=$(cat .commit 2>/dev/null || echo unknown)
for WL in ${WLS:-ch3oha256_4096 ph2o45_1024 ch3ohe256_sweep oh24_overlap_2048}; do
  timeout -k 10 400 python bench.py --workload $WL > gpurun_out/lines_$TAG/$WL.json 2> gpurun_out/lines_$TAG/$WL.err || exit 1
  bash tools/profile.sh $TAG $WL || exit 1
done
echo "done ($git_rev)"
