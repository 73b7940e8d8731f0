# Unattended: product build, CPU tests, variant builds + register report, one gpurun call.
cd /root/repo
echo "== build $(date)"
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
echo "== variants $(date)"
bash tools/build_variants.sh "1:-DLVG_PANEL_PRIO=1" "2:-DLVG_PANEL_W1=1" "3:-DLVG_PANEL_W1=1 -DLVG_PANEL_PRIO=1" "4:-DLVG_OCC=3" "5:-DLVG_PREFETCH_L=1" "6:-DLVG_PANEL_W1=1 -DLVG_PREFETCH_L=1" "7:-DLVG_L2_PREFETCH=1" > gpurun_out/variants_build.log 2>&1 &
VP=$!
for f in "" "-DLVG_PANEL_W1=1" "-DLVG_OCC=3"; do
  echo "-- resource usage, flags: $f"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off $f -c radiative_transfer_amd/csrc/lvg_kernels.hip -o /tmp/k_res.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A 14 "Function Name: _ZN3lvg12solve_kernel" | grep -E "VGPRs|AGPRs|Spill|LDS Size|Occupancy|SGPRs"
done
echo "== cpu tests $(date)"
timeout 1500 python -m pytest tests -x -q -m "not gpu" > gpurun_out/cpu_tests.log 2>&1; echo "cpu tests rc=$?"; tail -3 gpurun_out/cpu_tests.log
wait $VP; echo "variants build rc=$?"; ls radiative_transfer_amd/_lib/
echo "== gpurun $(date)"
/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_r1b.sh' > gpurun_out/gpurun1.log 2>&1; echo "gpurun rc=$?"
tail -40 gpurun_out/gpurun1.log
echo "== done $(date)"
