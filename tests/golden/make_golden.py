"""Generate tests/golden/oracle_golden_v1.npz: small regression fixtures of the
CPU oracle on synth_v1 inputs (inputs are regenerated from seeds; only outputs
are stored). These are NOT reference outputs — the reference cannot be built
here (DESIGN.md "Parity") — they pin the oracle against accidental change.

    python -m tests.golden.make_golden
"""
import os

import numpy as np

from radiative_transfer_amd import abi, synth
from oracle import oracle

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_golden_v1.npz")


def compute():
    out = {}
    cases = [("oh24_single", 1, None), ("ph2o45_1024", 6, None), ("oh24_overlap_2048", 4, None),
             ("ch3oha256_4096", 2, 64)]
    for name, nl, nlev in cases:
        P, L, o = synth.make_problem(name, nb_lay=nl, nb_lev=nlev)
        pops, st = oracle.solve_layers(P, L, abi.default_opts(**o))
        out[f"{name}/pops"] = pops
        out[f"{name}/iterations"] = st["iterations"].astype(np.int32)
        out[f"{name}/converged"] = st["converged"].astype(np.int32)
        out[f"{name}/eq_error"] = st["eq_error"]
        bo = oracle.boundary_layer_populations(P, L)
        out[f"{name}/boundary"] = bo
        M, df, pn, eq = oracle.calc_new_pop(P, L, 0, bo[0], o.get("line_overlap", 0))
        out[f"{name}/matrix0"] = M
        out[f"{name}/newpop0"] = pn
    return out


if __name__ == "__main__":
    d = compute()
    np.savez_compressed(OUT, **d)
    print(OUT, sum(v.nbytes for v in d.values()), "bytes")
