#!/bin/bash
# Same-box A/B of library variants (tools/build_variants.sh): for each tag, an exactness
# check against the oracle on a layer subset (variant_check.py) and a bench line.
# REPS=k repeats the bench lines in ABAB order (checks run once).
# usage: VARIANTS="prod v0 vA" WL=ch3oha256_4096 CHK=48 bash tools/gpu/ab.sh   (OUT=gpurun_out/ab)
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
WL=${WL:-ch3oha256_4096}
mkdir -p $OUT
for rep in $(seq ${REPS:-1}); do
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then lib=$PWD/radiative_transfer_amd/_lib/liblvg_amd.so; else lib=$PWD/radiative_transfer_amd/_lib/liblvg_amd_$v.so; fi
  if [ $rep = 1 ] && [ "${CHK:-48}" != 0 ]; then
    LVG_LIB_PATH=$lib timeout -k 10 ${CHKT:-240} python tools/variant_check.py $WL ${CHK:-48} > $OUT/check_$v.txt 2>&1
    rc=$?; echo "$v check rc=$rc: $(tail -1 $OUT/check_$v.txt)"
    [ $rc -le 1 ] || exit $rc
  fi
  LVG_LIB_PATH=$lib timeout -k 10 ${BENCHT:-300} python bench.py --workload $WL --no-cpu --no-host-entry --no-provenance \
      --steps ${STEPS:-5} ${BENCH_ARGS} > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || exit 3
  python -c "import json,sys; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), 'ms/step %.2f kernel %.2f frac %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac']))"
done
done
