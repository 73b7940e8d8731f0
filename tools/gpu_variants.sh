# bench each library variant (radiative_transfer_amd/_lib/liblvg_amd_v*.so)
set -o pipefail
cd /root/repo
for v in 0 1 2 3; do
  LVG_LIB_PATH=radiative_transfer_amd/_lib/liblvg_amd_v$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bv$v.json 2> gpurun_out/bv$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bv$v.json'));print('v$v',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],2))"
done
