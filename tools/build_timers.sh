# diagnostic library with per-phase s_memtime counters (tools/phase_timers.py)
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DLVG_PHASE_TIMERS $EXTRA \
  -I include -I radiative_transfer_amd/csrc radiative_transfer_amd/csrc/lvg_abi.cpp radiative_transfer_amd/csrc/lvg_kernels.hip \
  radiative_transfer_amd/csrc/lvg_transitions.hip radiative_transfer_amd/csrc/lvg_sched.hip -o radiative_transfer_amd/_lib/liblvg_amd_timers.so
