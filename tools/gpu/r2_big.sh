#!/bin/bash
# N > 256: GPU parity of the 768-thread block kernel, then a bench line at the reference's 768 levels.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_chains.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -8 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --nb-lev 768 --layers 1024 --steps 2 --cpu-budget 10 > $OUT/bench_768.json 2> $OUT/bench_768.err || exit 1
cat $OUT/bench_768.json
