"""Diagnostic: per-phase cycle breakdown of the solve kernel (timer build)."""
import ctypes as C, os, sys, time, numpy as np
sys.path.insert(0, "/root/repo")
os.environ.setdefault("LVG_LIB_PATH", "/root/repo/radiative_transfer_amd/_lib/liblvg_amd_timers.so")
from radiative_transfer_amd import synth, abi, native
names = ["setup+coll", "boundary LU", "line terms", "assemble+resid", "LU panel", "LU swap+trsm", "LU gemm", "LU backsub", "ctl",
         " (layer_setup)", " (pair tiles)", " (B diagonal)", "LU block load",
         "clk", "clk", "rsv", " (trsm: L fetch+Ub)", " (trsm: solve+U st)", " (trsm: LT stage)", " (panel: reduce+bar)",
         " (panel: select+div+fma)", " (panel: write-back)"]
SHOW = list(range(13)) + list(range(16, 22))
if "--v2" in sys.argv:          # the N <= 256 kernel's column-owned LU (lvg_lu256.h); sums over its 4 waves
    sys.argv.remove("--v2")
    names[4], names[5], names[6] = "LU panel (owner)", "LU step-end barrier", "LU rank-16 updates"
    names[12], names[15], names[16], names[17], names[21] = "LU block load", "LU residual (4 bar)", \
        " (L fetch+stage+bar)", " (TRSM, U rows)", " (publish + 2 bar)"
    SHOW = list(range(13)) + [15, 16, 17, 21]
name = sys.argv[1] if len(sys.argv) > 1 else "ch3oha256_4096"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
P, L, o = synth.make_problem(name, nb_lay=nl)
s = native.LvgSolver(P)
lib = native.load()
buf = (C.c_ulonglong * 32)()


def read_counters(out, reset):
    """256- and 512-thread kernels' counters summed (one kind runs per launch)."""
    a, b = (C.c_ulonglong * 32)(), (C.c_ulonglong * 32)()
    lib.lvg_debug_phase_cycles(a, reset)
    lib.lvg_debug_phase_cycles_wide(b, reset)
    for i in range(32):
        out[i] = a[i] + b[i]


s.solve_layers(L, abi.default_opts(**o))
read_counters(buf, 1)
t = time.time(); pops, st = s.solve_layers(L, abi.default_opts(**o)); dt = time.time() - t
ms, _ = s.last_kernel_time()
read_counters(buf, 1)
cyc = np.array(buf[:32], dtype=np.float64)
clk = np.array(buf[13:15], dtype=np.float64)
its = st["iterations"].sum()
print(f"{name} layers={nl} kernel {ms:.2f} ms, iterations {its}, LUs {its + nl}")
tot = cyc[:9].sum() - cyc[1]   # boundary LU overlaps the LU phases
for i in SHOW:
    n, c = names[i], cyc[i]
    print(f"  {n:16s} {c/1e6:10.2f} Mcyc  {100*c/tot:5.1f}%   per-LU {c/(its+nl):10.0f} cyc   per-layer {c/nl:10.0f} cyc")
print(f"  in-kernel clock (sum memtime / sum realtime x 100 MHz): {clk[0] / max(clk[1], 1) * 0.1:.3f} GHz; busy WG-time {clk[1] / 1e8:.3f} s")
np.savez(f"/root/repo/gpurun_out/dump_{name}_{nl}.npz", pops=pops, iters=st["iterations"], conv=st["converged"])
