# Build radiative_transfer_amd/_lib/liblvg_amd_v<k>.so from a modified copy of the block-kernel
# sources in DIR (two levels below the repo root, e.g. radiative_transfer_amd/var_<k>/, so that
# its ../../include resolves): both N <= 256 instantiations (256- and 512-thread) from
# DIR/lvg_kernels.hip, the wave kernel from DIR/lvg_wave.hip when WAVE=1, every other object
# from the product build. usage: [WAVE=1] bash tools/build_srcvariant.sh k DIR. Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
O=radiative_transfer_amd/_lib/obj
k=$1; d=$2
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off"
wobj=$O/lvg_wave.o
( $H -c $d/lvg_kernels.hip -o $O/var_${k}_n.o &
  $H -DLVG_WIDE=1 -c $d/lvg_kernels.hip -o $O/var_${k}_w.o &
  if [ "${WAVE:-0}" = 1 ]; then $H -c $d/lvg_wave.hip -o $O/var_${k}_wv.o & fi
  wait ) || exit 1
[ "${WAVE:-0}" = 1 ] && wobj=$O/var_${k}_wv.o
for f in $O/var_${k}_n.o $O/var_${k}_w.o $wobj; do [ -s $f ] || { echo "missing $f"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so \
  $O/var_${k}_n.o $O/var_${k}_w.o $wobj $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o
