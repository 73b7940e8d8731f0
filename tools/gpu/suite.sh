#!/bin/bash
# The GPU test suite and smoke as the driver runs them (round-end tiers), on the box.
set -o pipefail
OUT=gpurun_out/${VOUT:-suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -3 $OUT/smoke.log
