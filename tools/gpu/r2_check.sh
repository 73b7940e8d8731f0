#!/bin/bash
# exactness on CH3OH-A (oracle), GPU parity suite, bench line. Diagnostic.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2c}
mkdir -p $OUT
timeout -k 10 200 python tools/variant_check.py > $OUT/exact.txt 2>&1; rc=$?
cat $OUT/exact.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
if [ "${PYTEST:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; tail -3 $OUT/pytest.log
fi
