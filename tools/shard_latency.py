"""Diagnostic: the strong-scaling shares of a config on one GPU (layers l*L/G .. (l+1)*L/G,
one launch each), their slowest layer alone, and its iteration count: how far the share's
time sits above the latency of its longest layer."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from radiative_transfer_amd import abi, synth, native

name = sys.argv[1] if len(sys.argv) > 1 else "ch3oha256_4096"
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
tuning = sys.argv[3] if len(sys.argv) > 3 else ""
P, L, o = synth.make_problem(name)
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
if tuning:
    s.set_tuning(tuning)
out = []
for r in range(G):
    lo, hi = r * L.nb_lay // G, (r + 1) * L.nb_lay // G
    sub = L.subset(np.arange(lo, hi))
    s.solve_layers(sub, opts)
    t = []
    for _ in range(3):
        _, st = s.solve_layers(sub, opts)
        t.append(s.last_kernel_time()[0])
    k = int(np.argmax(st["iterations"]))
    one = L.subset(np.array([lo + k]))
    s.solve_layers(one, opts)
    t1 = []
    for _ in range(3):
        s.solve_layers(one, opts)
        t1.append(s.last_kernel_time()[0])
    it = int(st["iterations"][k])
    out.append(dict(rank=r, layers=hi - lo, ms=min(t), its=int(st["iterations"].sum()), max_it=it,
                    slowest_alone_ms=min(t1), ms_per_lu_alone=min(t1) / (it + 1)))
    print(json.dumps(out[-1]), flush=True)
print(json.dumps(dict(config=name, G=G, tuning=tuning, step_ms=max(x["ms"] for x in out))))
