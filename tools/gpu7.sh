# GPU cycle: parity tests, phase timers (CH3OH), bench without CPU leg
set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_ch3oh.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/phase_ch3oh.log; python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('VALUE',d['value'],'kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])"
exit $rc
