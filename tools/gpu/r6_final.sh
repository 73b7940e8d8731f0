#!/bin/bash
# Round 6 profile set at one commit (.commit): the GPU suite and smoke on the product library, the
# GPU suite on the checked-glb library, rocprofv3 stats + PMC traffic + the bench line (CPU legs
# included) for the four BASELINE workloads (tools/gpu/profiles.sh), the strong-scaling shares of
# the 4096-layer cloud, and the timer build's phase split (block kernel) and slowest-layer phases
# (wave kernel). Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6_final
mkdir -p $OUT
L=$PWD/radiative_transfer_amd/_lib
if [ -z "$NOSUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $OUT/pytest_prod.txt 2>&1 || { tail -40 $OUT/pytest_prod.txt; exit 1; }
  tail -1 $OUT/pytest_prod.txt
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
  tail -1 $OUT/smoke.txt
  LVG_LIB_PATH=$L/liblvg_amd_checked.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
      --timeout-method thread > $OUT/pytest_checked_glb.txt 2>&1 || { tail -40 $OUT/pytest_checked_glb.txt; exit 1; }
  tail -1 $OUT/pytest_checked_glb.txt
fi
if [ -z "$NOPROF" ]; then
  TAG=r6 bash tools/gpu/profiles.sh || exit 2
fi
for G in 2 4 8; do
  timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 $G > $OUT/shard$G.txt 2>&1 || exit 3
  tail -1 $OUT/shard$G.txt
done
if [ -z "$NOTIMERS" ]; then
  timeout -k 10 300 python tools/phase_timers.py --v2 ch3oha256_4096 4096 > $OUT/phase_4096.txt 2>&1 || exit 4
  sed -n 1,12p $OUT/phase_4096.txt
  for wl in ph2o45_1024 oh24_overlap_2048; do
    timeout -k 10 300 python tools/latency_timers.py $wl > $OUT/wave_$wl.txt 2>&1 || exit 5
    tail -3 $OUT/wave_$wl.txt
  done
fi
echo "done ($(cat .commit 2>/dev/null || echo unknown))"
