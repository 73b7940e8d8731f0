# timer-overhead check: product vs timer build on the same 1024-layer run
set -o pipefail
cd /root/repo
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --layers 1024 > gpurun_out/b1024.json 2>gpurun_out/b1024.err && \
timeout -k 10 300 python tools/phase_timers.py ch3oha256_4096 1024 > gpurun_out/phase_ch3oh.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.json 2>gpurun_out/bench.err
rc=$?
python -c "import json;d=json.load(open('gpurun_out/b1024.json'));print('1024:',d['value'],'kernel_ms',d['roofline']['kernel_ms'])"
head -2 gpurun_out/phase_ch3oh.log
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('4096:',d['value'],'kernel_ms',d['roofline']['kernel_ms'])"
exit $rc
