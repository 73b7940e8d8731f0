#!/bin/bash
# Warm-chain batching: GPU parity of lvg_solve_chains, then bench lines in chain mode.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --chain-len 8 --steps 3 > $OUT/bench_chains_ch3oha.json 2> $OUT/bench_chains_ch3oha.err || exit 1
cat $OUT/bench_chains_ch3oha.json
timeout -k 10 300 python bench.py --workload ph2o45_1024 --chain-len 8 --steps 3 > $OUT/bench_chains_ph2o.json 2> $OUT/bench_chains_ph2o.err || exit 1
cat $OUT/bench_chains_ph2o.json
