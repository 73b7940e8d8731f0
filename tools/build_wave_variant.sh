# Build radiative_transfer_amd/_lib/liblvg_amd_v<k>.so with lvg_wave.hip taken from SRC
# (default the tree's) and compiled with FLAGS; every other object from the product build.
# usage: bash tools/build_wave_variant.sh k "FLAGS" [SRC]. Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
O=radiative_transfer_amd/_lib/obj
k=$1; flags=$2; src=${3:-radiative_transfer_amd/csrc/lvg_wave.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I radiative_transfer_amd/csrc \
  $flags -c $src -o $O/var_${k}_wave.o &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so \
  $O/lvg_kernels.o $O/lvg_kernels_wide.o $O/var_${k}_wave.o $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o
