# Build library variants radiative_transfer_amd/_lib/liblvg_amd_v<k>.so, one per
# argument "k:FLAGS" (e.g. 0:"-DLVG_L2_PREFETCH=0"), in parallel: lvg_kernels.hip is
# recompiled with FLAGS, every other object comes from the product build
# (radiative_transfer_amd/_lib/obj, python -m radiative_transfer_amd.build). Timed by
# tools/gpu/r2_variants.sh on the GPU box. Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
O=radiative_transfer_amd/_lib/obj
pids=()
for spec in "$@"; do
  k=${spec%%:*}; flags=${spec#*:}
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags \
      -c radiative_transfer_amd/csrc/lvg_kernels.hip -o $O/var_$k.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so \
      $O/var_$k.o $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
