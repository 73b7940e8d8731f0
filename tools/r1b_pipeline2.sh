# Unattended: product build (L11 from the fetched rows) + old-path variant v9, CPU tests, one gpurun.
cd /root/repo
echo "== build $(date)"
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build2.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build2.log; exit 1; }
bash tools/build_variants.sh "9:-DLVG_LA_TILE=0" > gpurun_out/variants_build2.log 2>&1 || { echo VARIANT BUILD FAILED; tail -30 gpurun_out/variants_build2.log; exit 1; }
echo "== cpu tests $(date)"
timeout 1500 python -m pytest tests -x -q -m "not gpu" > gpurun_out/cpu_tests2.log 2>&1; echo "cpu tests rc=$?"; tail -2 gpurun_out/cpu_tests2.log
echo "== gpurun $(date)"
/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_r1b.sh' > gpurun_out/gpurun2.log 2>&1; echo "gpurun rc=$?"
tail -8 gpurun_out/gpurun2.log
echo "== done $(date)"
