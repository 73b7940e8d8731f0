# bench line for every BASELINE workload (1 GPU)
set -o pipefail
cd /root/repo
for w in ph2o45_1024 oh24_overlap_2048 ch3ohe256_sweep ch3oha256_4096; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --cpu-budget 5 > gpurun_out/cfg_$w.json 2> gpurun_out/cfg_$w.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/cfg_$w.json'));print('$w',round(d['value']),'ms',round(d['ms_per_step'],3),'units',d['config']['layer_iterations_per_step'],'frac',round(d['roofline']['frac'],4),'cpu',round(d['cpu_baseline']['value']))"
done
