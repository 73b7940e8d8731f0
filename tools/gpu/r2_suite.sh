#!/bin/bash
# Whole GPU suite (as the driver runs it) + smoke.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2s}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -3 $OUT/smoke.log
