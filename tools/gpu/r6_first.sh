#!/bin/bash
# Round 6: the GPU suite on the product library and on the checked-glb build, the timer
# build's boundary / iteration LU split on the metric config, bench lines (plain, and with
# the RCCL process group at world size 1).
set -o pipefail
OUT=gpurun_out/${VOUT:-r6a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_prod.log 2>&1 || { tail -40 $OUT/pytest_prod.log; exit 1; }
tail -2 $OUT/pytest_prod.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
LVG_LIB_PATH=radiative_transfer_amd/_lib/liblvg_amd_timers.so timeout -k 10 300 \
    python -u tools/phase_timers.py ch3oha256_4096 4096 --v2 > $OUT/timers_4096.txt 2>&1 || { cat $OUT/timers_4096.txt; exit 1; }
cat $OUT/timers_4096.txt
LVG_LIB_PATH=radiative_transfer_amd/_lib/liblvg_amd_checked.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_checked.log 2>&1 || { tail -40 $OUT/pytest_checked.log; exit 1; }
tail -2 $OUT/pytest_checked.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python -u bench.py --process-group --no-cpu --no-host-entry > $OUT/bench_pg.json 2> $OUT/bench_pg.err || { tail -20 $OUT/bench_pg.err; exit 1; }
cat $OUT/bench_pg.json
