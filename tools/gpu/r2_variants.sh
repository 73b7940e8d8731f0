#!/bin/bash
# Time library variants liblvg_amd_v<k>.so (built by tools/build_variants.sh) with bench.py,
# plus the product library, and check each for exactness against the oracle. Diagnostic only.
set -o pipefail
OUT=gpurun_out/${VOUT:-r2v}
mkdir -p $OUT
if [ -x tools/probe/mfma_f64_probe ]; then
  timeout -k 10 60 tools/probe/mfma_f64_probe $OUT/mfma_f64_probe.bin > $OUT/mfma_probe.log 2>&1 || exit 1
fi
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/b_prod.json 2> $OUT/b_prod.err || exit 1
for k in "$@"; do
  lib=radiative_transfer_amd/_lib/liblvg_amd_v$k.so
  LVG_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/b_v$k.json 2> $OUT/b_v$k.err || exit 1
  LVG_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/variant_check.py > $OUT/x_v$k.txt 2>&1 || exit 1
done
python - "$OUT" "$@" <<'PY'
import json, sys
out = sys.argv[1]
for k in ["prod"] + ["v" + a for a in sys.argv[2:]]:
    b = json.load(open(f"{out}/b_{k}.json"))
    x = open(f"{out}/x_{k}.txt").read().strip() if k != "prod" else "-"
    print(k, round(b["value"]), "kernel_ms", round(b["roofline"]["kernel_ms"], 2), x)
PY
