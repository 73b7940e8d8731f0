#!/bin/bash
# round 4 baseline on this box: the changed GPU tests, the default bench line, the 8-way shares
set -o pipefail
OUT=gpurun_out/r4_base
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_chains.py tests/test_gpu_wide.py -x -v \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 10 --no-cpu --no-host-entry > $OUT/bench.json 2> $OUT/bench.err || exit 3
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8.txt 2>&1 || exit 4
tail -1 $OUT/shard8.txt
