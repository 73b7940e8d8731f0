"""Exactness probe for a library variant (LVG_LIB_PATH): 128 CH3OH-A layers against the oracle."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from radiative_transfer_amd import synth, abi, native
from oracle import oracle

P, L, o = synth.make_problem("ch3oha256_4096", nb_lay=128)
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
pg, sg = s.solve_layers(L, opts)
po, so = oracle.solve_layers(P, L, opts)
ok = np.array_equal(pg, po) and np.array_equal(sg["iterations"], so["iterations"])
print("exact" if ok else f"MISMATCH max|d|={np.max(np.abs(pg - po)):.3e}")
sys.exit(0 if ok else 1)
