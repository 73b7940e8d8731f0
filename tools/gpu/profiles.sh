#!/bin/bash
# rocprofv3 stats + PMC traffic, then the bench line (with CPU legs) for the BASELINE
# workloads, all on one box at one commit (.commit, written before the gpurun call):
# gpurun_out/prof_$TAG_<workload>/ (tools/profile.sh) and gpurun_out/lines_$TAG/<workload>.json.
# The profile runs first and tools/update_profiles.py refreshes profiles/pmc_traffic.json on
# the box, so each bench line's roofline.traffic comes from the profile of the same run;
# that file is copied to gpurun_out/lines_$TAG/ and update_profiles.py rebuilds it locally
# from the merged CSVs.
set -o pipefail
TAG=${TAG:-r3}
mkdir -p gpurun_out/lines_$TAG
git_rev=$(cat .commit 2>/dev/null || echo unknown)
for WL in ${WLS:-ch3oha256_4096 ph2o45_1024 ch3ohe256_sweep oh24_overlap_2048}; do
  bash tools/profile.sh $TAG $WL || exit 1
  python tools/update_profiles.py $TAG $WL > gpurun_out/lines_$TAG/$WL.traffic.json || exit 1
  timeout -k 10 400 python bench.py --workload $WL > gpurun_out/lines_$TAG/$WL.json 2> gpurun_out/lines_$TAG/$WL.err || exit 1
done
cp profiles/pmc_traffic.json gpurun_out/lines_$TAG/pmc_traffic.json
echo "done ($git_rev)"
