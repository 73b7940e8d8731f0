#!/bin/bash
# Round 6: the GPU suite + smoke on the product library, a bench line, the 8-way share, and
# optional PMC passes (PMC="pass1;pass2", each a counter list) on the metric workload.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${VOUT:-r6v}
mkdir -p $OUT
if [ -z "$NOSUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python -u bench.py --no-cpu --no-host-entry --steps 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), 'kernel %.3f ms' % d['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/shard_latency.py ch3oha256_4096 8 > $OUT/shard8.txt 2>&1 || exit 4
tail -1 $OUT/shard8.txt
i=0
IFS=';' read -ra PASSES <<< "${PMC:-}"
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-host-entry --no-provenance > $OUT/pmc$i.json 2> $OUT/pmc$i.err || exit 5
done
python3 - <<PY
import csv, glob
for f in sorted(glob.glob("$OUT/pmc*/**/*counter_collection.csv", recursive=True)):
    tot = {}
    for r in csv.DictReader(open(f)):
        if "solve_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(f.split("/")[2], {k: f"{v:.4g}" for k, v in tot.items()})
PY
