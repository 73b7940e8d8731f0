#!/bin/bash
# coll_kernel in temperature order (XCD chunks) vs index order: GPU suite, then rocprof kernel
# stats of a short headline bench for each, and bench lines. Diagnostic.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${VOUT:-r2corder}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in t i; do
  if [ $v = i ]; then export LVG_COLL_INDEX_ORDER=1; else unset LVG_COLL_INDEX_ORDER; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$v -o run -- \
      python3 bench.py --no-cpu --no-host-entry --steps 3 --warmup 1 > $OUT/p_$v.json 2> $OUT/p_$v.err || exit 1
  f=$(find $OUT/t_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -E "coll_kernel|solve_kernel" $f | cut -d, -f1-4
done
for v in t i t i; do
  if [ $v = i ]; then export LVG_COLL_INDEX_ORDER=1; else unset LVG_COLL_INDEX_ORDER; fi
  timeout -k 10 200 python bench.py --no-cpu --no-host-entry --steps 10 --warmup 2 > $OUT/b_$v.json 2>> $OUT/bench.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['roofline']['coll_kernel_ms'],3))"
done
