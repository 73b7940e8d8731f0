#!/bin/bash
# GPU parity suite, smoke, and the bench line with CPU legs. Diagnostic driver for a round.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2f}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
