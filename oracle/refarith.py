"""Distance between the bit-exact oracle and its reference-arithmetic build
(-DORACLE_REF_ARITH: glibc exp/log10/pow, LU without fma) on the BASELINE configs.

TEST INFRASTRUCTURE ONLY (tests/test_oracle_refarith_cpu.py).
SURVEY.md 8(c) tolerances:
  lockstep (same input populations, one calc_new_pop): |dn|/n <= 1e-9 for n >= 1e-30,
      |dn| <= 1e-39 below;
  converged populations, equal iteration counts: <= 1e-9 relative (same floor);
  iteration counts differing by +-1: <= 2e-5 relative;
  iteration counts identical on >= 99 % of layers.
"""
from __future__ import annotations

import numpy as np

from radiative_transfer_amd import abi, synth
from oracle import oracle

FLOOR = 1e-30


def rel_dev(a, b):
    """Per-entry relative deviation, with entries below FLOOR compared absolutely (scaled
    so that the 1e-39 absolute rule maps to 1e-9)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    big = np.abs(b) >= FLOOR
    out = np.zeros_like(a)
    out[big] = np.abs(a[big] - b[big]) / np.abs(b[big])
    out[~big] = np.abs(a[~big] - b[~big]) / 1e-30
    return out


# spread subsets: (config, layers drawn, stride) — sized so the whole table runs in ~1 min on 8 cores
SAMPLES = {
    "oh24_single": 1,
    "ph2o45_1024": 1024,
    "ch3oha256_4096": 256,
    "ch3ohe256_sweep": 256,
    "oh24_overlap_2048": 2048,
}


def compare(name: str, nb: int | None = None, nthreads: int = 0):
    prob, layers_all, o = synth.make_problem(name)
    L = layers_all.nb_lay
    nb = nb or SAMPLES[name]
    idx = np.unique(np.linspace(0, L - 1, min(nb, L)).round().astype(int))
    layers = layers_all.subset(idx)
    opts = abi.default_opts(**o)
    pe, se = oracle.solve_layers(prob, layers, opts, nthreads=nthreads)
    pr, sr = oracle.solve_layers(prob, layers, opts, nthreads=nthreads, ref=True)
    ie, ir = se["iterations"], sr["iterations"]
    same = ie == ir
    d = rel_dev(pe, pr).max(axis=1)
    # lockstep: one calc_new_pop from the same input (the reference-arith boundary populations)
    bp = oracle.boundary_layer_populations(prob, layers, ref=True)
    bpe = oracle.boundary_layer_populations(prob, layers)
    ov = o.get("line_overlap", 0)
    lock = []
    for j in range(min(8, layers.nb_lay)):
        _, _, p1, _ = oracle.calc_new_pop(prob, layers, j, bp[j], ov)
        _, _, p2, _ = oracle.calc_new_pop(prob, layers, j, bp[j], ov, ref=True)
        lock.append(rel_dev(p1, p2).max())
    return {
        "config": name, "layers": int(layers.nb_lay), "N": int(prob.mol.nb_lev),
        "iter_identical_frac": float(same.mean()),
        "iter_max_absdiff": int(np.abs(ie.astype(int) - ir.astype(int)).max()),
        "rel_max_same_iters": float(d[same].max()) if same.any() else 0.0,
        "rel_max_pm1_iters": float(d[~same].max()) if (~same).any() else 0.0,
        "rel_max_lockstep": float(max(lock)),
        "rel_max_boundary": float(rel_dev(bpe, bp).max()),
        "converged_exact": int(se["converged"].sum()), "converged_ref": int(sr["converged"].sum()),
    }


if __name__ == "__main__":
    import json
    print(json.dumps([compare(n) for n in SAMPLES], indent=1))
