"""Diagnostic (timer build): phase cycles of the single slowest layer of a config, solved alone."""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, "/root/repo")
os.environ.setdefault("LVG_LIB_PATH", "/root/repo/radiative_transfer_amd/_lib/liblvg_amd_timers.so")
from radiative_transfer_amd import abi, synth, native

name = sys.argv[1] if len(sys.argv) > 1 else "ph2o45_1024"
P, L, o = synth.make_problem(name)
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
lib = native.load()
# the wave kernel (N <= 64) keeps its counters in its own translation unit (lvg_wave.hip)
buf = (C.c_ulonglong * 64)()


def read(out, reset):
    """The counters of every kernel that may have run, summed (one kind runs per launch)."""
    fns = [lib.lvg_debug_wave_phase_cycles] if P.mol.nb_lev <= 64 else \
          [lib.lvg_debug_phase_cycles, lib.lvg_debug_phase_cycles_wide]
    tot = [0] * 64
    for f in fns:
        b = (C.c_ulonglong * 64)()
        f(b, reset)
        tot = [x + y for x, y in zip(tot, b)]
    for i in range(64):
        out[i] = tot[i]

_, st = s.solve_layers(L, opts)
k = int(np.argmax(st["iterations"]))
sub = L.subset(np.array([k]))
s.solve_layers(sub, opts)
read(buf, 1)
_, ss = s.solve_layers(sub, opts)
ms, _ = s.last_kernel_time()
read(buf, 1)
cyc = np.array(buf[:32], dtype=np.float64)
names = ["setup+coll", "boundary LU", "line terms", "assemble+resid", "LU panel", "LU swap+trsm", "LU gemm",
         "LU backsub", "ctl"]
it = int(ss["iterations"][0])
print(f"{name}: layer {k} alone, {it} iterations, kernel {ms:.3f} ms = {ms * 1e-3 * 2.3e9 / it:.0f} cyc/iteration at 2.3 GHz")
for i, n in enumerate(names):
    print(f"  {n:16s} {cyc[i] / it:10.0f} cyc/iteration")
for i, n in [(15, "  (residual hand-off)"), (12, "  (block load)"), (16, "  (L fetch+stage)"), (17, "  (TRSM)"),
             (21, "  (pre-panel bar+dump)"), (22, "  (bsub diag)"), (23, "  (bsub update)"), (24, "  (wait before bsub)")] \
        if P.mol.nb_lev > 64 else \
        [(16, "  (lines: record+opacity)"), (17, "  (lines: intervals)"), (18, "  (lines: tables+sums)"),
         (19, "  (lines: intensities)")]:
    print(f"  {n:22s} {cyc[i] / it:10.0f} cyc/iteration")
print(f"  sum of phases    {cyc[:9].sum() / it:10.0f} cyc/iteration; raw slots {buf[:32]}")
