"""Diagnostic: kernel time of the slowest layers alone vs the whole config (is the launch
bound by its longest layer chain?). Prints ms for: all layers, the k slowest, the slowest."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from radiative_transfer_amd import abi, synth, native

name = sys.argv[1] if len(sys.argv) > 1 else "ph2o45_1024"
P, L, o = synth.make_problem(name)
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
s.solve_layers(L, opts)
_, st = s.solve_layers(L, opts)
ms_all, _ = s.last_kernel_time()
it = st["iterations"]
order = np.argsort(-it)
print(f"{name}: all {L.nb_lay} layers {ms_all:.2f} ms, iterations sum {it.sum()} max {it.max()}")
for k in (1, 4, 64, 256):
    sub = L.subset(np.sort(order[:k]))
    s.solve_layers(sub, opts)
    _, ss = s.solve_layers(sub, opts)
    ms, _ = s.last_kernel_time()
    print(f"  {k:4d} slowest layers: {ms:.3f} ms, max iterations {ss['iterations'].max()}, "
          f"{1e3 * ms / ss['iterations'].max():.2f} us per iteration of the longest")
