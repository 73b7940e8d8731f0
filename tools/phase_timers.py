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
    names += [" (backsub: diag solve)", " (backsub: row updates)", " (wait before backsub)"]
    SHOW = list(range(13)) + [15, 16, 17, 21, 22, 23, 24]
name = sys.argv[1] if len(sys.argv) > 1 else "ch3oha256_4096"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
P, L, o = synth.make_problem(name, nb_lay=nl)
s = native.LvgSolver(P)
lib = native.load()
NS = 64                      # counters per kernel (PH_SLOTS): boundary-LU sub-phases at +32
buf = (C.c_ulonglong * NS)()


def read_counters(out, reset):
    """256- and 512-thread kernels' counters summed (one kind runs per launch)."""
    a, b = (C.c_ulonglong * NS)(), (C.c_ulonglong * NS)()
    lib.lvg_debug_phase_cycles(a, reset)
    lib.lvg_debug_phase_cycles_wide(b, reset)
    for i in range(NS):
        out[i] = a[i] + b[i]


s.solve_layers(L, abi.default_opts(**o))
read_counters(buf, 1)
t = time.time(); pops, st = s.solve_layers(L, abi.default_opts(**o)); dt = time.time() - t
ms, _ = s.last_kernel_time()
read_counters(buf, 1)
cyc = np.array(buf[:NS], dtype=np.float64)
clk = np.array(buf[13:15], dtype=np.float64)
its = st["iterations"].sum()
print(f"{name} layers={nl} kernel {ms:.2f} ms, iterations {its}, LUs {its + nl}")
tot = cyc[13]                 # wave-cycles: every wave's memtime over its solve_layer calls
if cyc[26] > 0:
    # the honest split (round 6): wall wave-cycles of each part over the total wave-cycles
    rows = [("setup + collision build (per layer)", cyc[0], nl),
            ("boundary LU (per layer)", cyc[1], nl),
            ("iteration, all of it (per iteration)", cyc[26], its),
            ("  of which the iteration LU", cyc[25], its),
            ("  of which line terms", cyc[2], its),
            ("  of which column diagonals", cyc[3], its)]
    print(f"  total {tot/1e6:.1f} M wave-cycles (memtime summed over waves)")
    for n, c, u in rows:
        print(f"  {n:40s} {c/1e6:10.2f} Mcyc  {100*c/tot:5.1f}%   per unit {c/max(u,1):10.0f} cyc")
    print(f"  boundary LU / iteration LU (per LU, wall wave-cycles): {cyc[1]/nl / max(cyc[25]/max(its,1), 1):.3f}")
    print("  LU sub-phases per LU, iteration | boundary:")
    for i in SHOW:
        if i in (0, 1, 2, 3, 8, 9, 10, 11, 13, 14):
            continue
        n = names[i]
        ci, cb = cyc[i], cyc[i + 32]
        print(f"    {n:24s} {ci/max(its,1):10.0f} | {cb/max(nl,1):10.0f} cyc")
else:
    tot = cyc[:9].sum() - cyc[1]   # boundary LU overlaps the LU phases
    for i in SHOW:
        n, c = names[i], cyc[i]
        print(f"  {n:16s} {c/1e6:10.2f} Mcyc  {100*c/tot:5.1f}%   per-LU {c/(its+nl):10.0f} cyc   per-layer {c/nl:10.0f} cyc")
print(f"  in-kernel clock (sum memtime / sum realtime x 100 MHz): {clk[0] / max(clk[1], 1) * 0.1:.3f} GHz; busy WG-time {clk[1] / 1e8:.3f} s")
np.savez(f"/root/repo/gpurun_out/dump_{name}_{nl}.npz", pops=pops, iters=st["iterations"], conv=st["converged"])
