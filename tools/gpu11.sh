# parity tests + bench with and without the scheduling order
set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err && \
LVG_INDEX_ORDER=1 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_idx.json 2> gpurun_out/bench_idx.err
rc=$?
for f in bench bench_idx; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',round(d['value']),'ms_per_step',round(d['ms_per_step'],2),'kernel_ms',round(d['roofline']['kernel_ms'],2))"; done
exit $rc
