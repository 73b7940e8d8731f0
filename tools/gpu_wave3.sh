# wave kernel: parity, timings, phase timers (timers: wave 0 of each block only -> x waves per block)
set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wave_parity.log 2>&1 || { tail -30 gpurun_out/wave_parity.log; exit 1; }
tail -1 gpurun_out/wave_parity.log
for w in ph2o45_1024 oh24_overlap_2048; do
  timeout -k 10 120 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu > gpurun_out/wv_$w.json 2>gpurun_out/wv_$w.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/wv_$w.json'));print('$w',round(d['value']),'ms',round(d['ms_per_step'],3))"
  timeout -k 10 120 python tools/phase_timers.py $w 1024 > gpurun_out/wph_$w.txt 2>&1 || exit 1
  head -9 gpurun_out/wph_$w.txt
done
