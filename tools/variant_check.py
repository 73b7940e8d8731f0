"""Exactness probe for a library variant (LVG_LIB_PATH): a layer subset of a workload
(default 128 CH3OH-A layers; argv: workload, layers, levels) against the oracle."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from radiative_transfer_amd import synth, abi, native
from oracle import oracle

name = sys.argv[1] if len(sys.argv) > 1 else "ch3oha256_4096"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 128
nlev = int(sys.argv[3]) if len(sys.argv) > 3 else None
P, L, o = synth.make_problem(name, nb_lay=nl, nb_lev=nlev)
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
pg, sg = s.solve_layers(L, opts)
po, so = oracle.solve_layers(P, L, opts)
ok = np.array_equal(pg, po) and np.array_equal(sg["iterations"], so["iterations"])
print("exact" if ok else f"MISMATCH max|d|={np.max(np.abs(pg - po)):.3e}")
sys.exit(0 if ok else 1)
