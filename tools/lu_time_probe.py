"""Diagnostic: kernel time per LU of a workload (kernel ms x resident slots / LUs), for
timing probes whose results are wrong on purpose (their iteration counts are not stable,
so bench.py's run-to-run check does not apply). argv: workload [layers]."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from radiative_transfer_amd import abi, synth, native

name = sys.argv[1] if len(sys.argv) > 1 else "ch3oha256_4096"
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 0
P, L, o = synth.make_problem(name, **({"nb_lay": nl} if nl else {}))
opts = abi.default_opts(**o)
s = native.LvgSolver(P)
for rep in range(3):
    _, st = s.solve_layers(L, opts)
    ms, _ = s.last_kernel_time()
    lus = int(st["iterations"].sum()) + L.nb_lay
    print(f"{name} rep {rep}: kernel {ms:.3f} ms, LUs {lus}, {ms * 1e3 * 512 / lus:.1f} us per LU-slot (512 slots)")
