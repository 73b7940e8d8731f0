# bench + exactness probe for each library variant radiative_transfer_amd/_lib/liblvg_amd_v*.so
set -o pipefail
cd /root/repo
for f in radiative_transfer_amd/_lib/liblvg_amd_v*.so; do
  v=$(basename $f .so); v=${v#liblvg_amd_}
  LVG_LIB_PATH=$f timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b$v.json 2> gpurun_out/b$v.err || exit $?
  LVG_LIB_PATH=$f timeout -k 10 300 python tools/variant_check.py > gpurun_out/c$v.txt 2>&1; rc=$?
  python -c "import json;d=json.load(open('gpurun_out/b$v.json'));print('$v',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],2), open('gpurun_out/c$v.txt').read().strip().splitlines()[-1])"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
