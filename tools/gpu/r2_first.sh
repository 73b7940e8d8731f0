#!/bin/bash
# Round-2 first check: GPU parity tests, smoke, and one bench line.
set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-budget 10 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err
