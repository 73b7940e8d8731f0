# Build library variants radiative_transfer_amd/_lib/liblvg_amd_v<k>.so, one per
# argument "k:FLAGS" (e.g. 0:"-DLVG_L2_PREFETCH=0"), in parallel. Timed by
# tools/gpu_variants.sh on the GPU box. Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
pids=()
for spec in "$@"; do
  k=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off $flags \
    radiative_transfer_amd/csrc/lvg_kernels.hip radiative_transfer_amd/csrc/lvg_transitions.hip \
    radiative_transfer_amd/csrc/lvg_sched.hip radiative_transfer_amd/csrc/lvg_abi.cpp \
    -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
