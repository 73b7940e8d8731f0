# Build library variants radiative_transfer_amd/_lib/liblvg_amd_v<k>.so for same-box A/B
# runs, one per argument "k:SOURCE:FLAGS" (SOURCE: a copy of lvg_kernels.hip or
# lvg_wave.hip, path relative to the repo root; FLAGS: extra hipcc flags), in parallel.
# The variant object replaces the product object of the same kind; every other object
# comes from the product build (python -m radiative_transfer_amd.build). Select a variant
# at run time with LVG_LIB_PATH. Diagnostic only.
cd "$(dirname "$0")/.." || exit 1
O=radiative_transfer_amd/_lib/obj
pids=()
for spec in "$@"; do
  k=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; flags=${rest#*:}
  [ "$src" = "$rest" ] && flags=""
  # the variant object replaces the product object of its kind: the wave kernel, the
  # 512-thread instantiation (flags with -DLVG_WIDE=1) or the 256-thread one
  case "$(basename $src) $flags" in
    *wave*)         objs="$O/lvg_kernels.o $O/lvg_kernels_wide.o $O/var_$k.o" ;;
    *LVG_WIDE=1*)   objs="$O/lvg_kernels.o $O/var_$k.o $O/lvg_wave.o" ;;
    *)              objs="$O/var_$k.o $O/lvg_kernels_wide.o $O/lvg_wave.o" ;;
  esac
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I radiative_transfer_amd/csrc $flags \
      -c $src -o $O/var_$k.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_v$k.so \
      $objs $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
