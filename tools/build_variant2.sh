# Build radiative_transfer_amd/_lib/liblvg_amd_v<k>.so with BOTH block-kernel instantiations
# (256-thread lvg_kernels.hip and 512-thread lvg_kernels_wide.hip) compiled with FLAGS; every
# other object from the product build. usage: bash tools/build_variant2.sh k "FLAGS". Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
O=radiative_transfer_amd/_lib/obj
k=$1; flags=$2
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I radiative_transfer_amd/csrc"
( $H $flags -c radiative_transfer_amd/csrc/lvg_kernels.hip -o $O/var_${k}_n.o &
  $H $flags -DLVG_WIDE=1 -c radiative_transfer_amd/csrc/lvg_kernels.hip -o $O/var_${k}_w.o & wait ) &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so \
  $O/var_${k}_n.o $O/var_${k}_w.o $O/lvg_wave.o $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o
