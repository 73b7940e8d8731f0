# diagnostic library with per-phase s_memtime counters (tools/phase_timers.py,
# tools/latency_timers.py): the block and wave kernels rebuilt with -DLVG_PHASE_TIMERS,
# every other object from the product build (radiative_transfer_amd/_lib/obj)
cd "$(dirname "$0")/.." && O=radiative_transfer_amd/_lib/obj && F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DLVG_PHASE_TIMERS -DLVG_CHECKED_GLB $EXTRA" && \
( /opt/rocm/bin/hipcc $F -c radiative_transfer_amd/csrc/lvg_kernels.hip -o $O/timers.o & \
  /opt/rocm/bin/hipcc $F -c radiative_transfer_amd/csrc/lvg_kernels_wide.hip -o $O/timers_wide.o & \
  /opt/rocm/bin/hipcc $F -c radiative_transfer_amd/csrc/lvg_wave.hip -o $O/timers_wave.o & wait ) && \
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o radiative_transfer_amd/_lib/liblvg_amd_timers.so \
  $O/timers.o $O/timers_wide.o $O/timers_wave.o $O/lvg_kernels_big.o $O/lvg_transitions.o $O/lvg_sched.o $O/lvg_abi.o
