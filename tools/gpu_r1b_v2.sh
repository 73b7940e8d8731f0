# variant timings only (product parity already checked this session) + one-WG-per-CU run
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
LVG_BLOCKS_PER_CU=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b_bpc1.json 2> gpurun_out/b_bpc1.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_bpc1.json'));print('1 WG/CU',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],2))"
bash tools/gpu_variants.sh
