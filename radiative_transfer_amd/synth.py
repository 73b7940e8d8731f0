"""synth_v1 — synthetic molecule, table and cloud generators.

The reference ships no input data (spectroscopy, collision, LVG escape and
dust tables are all read from an absent `input_data_path`), so
every configuration in BASELINE.json runs on synthetic inputs of the reference's
shapes, generated deterministically from a seed:

* level ladders with g = (2*spin+1)(2J+1) (spectroscopy.cpp:262, :360);
* Einstein A_ul = 3e-7 * dE^3 * U(0.1, 1) for dJ <= 1 (dK <= 1, same v);
  einst[l,u] = g_u/g_l * A_ul (spectroscopy.cpp:918-921);
* collision down-rates 1e-11 * (1 + T/100)^0.5 * exp(-dE/100) * U(0.5, 1.5)
  cm^3/s on each reference temperature grid, with the T = 0 K column zero;
* the LVG escape table ep = [1 - (1 - e^-tau)/tau] * delta/(1 + delta), tau = 1/gamma,
  on log grids gamma in [1e-6, 1e6] (81) and delta in [1e-4, 1e8] (41);
* one silicate-like dust component, a = 0.5e-5 cm, concentration 1.23e-11 * 2 n_H2;
* layer parameters drawn log-uniformly per layer.
"""
from __future__ import annotations

import numpy as np

from .abi import (Collisions, CollTable, DustComponent, EscTable, Layers, Molecule,
                  OverlapTable, Problem, LVG_COLL_CH3OH, LVG_COLL_H2O, LVG_COLL_OH_HF,
                  LVG_SP_E)

AMU = 1.66053906660e-24
HE_TO_H2 = 0.18          # n_He = 0.09 n_H (radiative_transfer.cpp:31) = 0.18 n_H2
V_TURB = 3.0e4           # MICROTURBULENT_SPEED (radiative_transfer.cpp:33)


# ---- shared tables -----------------------------------------------------------

def _esc_fn(gamma, delta):
    tau = 1.0 / np.asarray(gamma, dtype=np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        beta = np.where(tau > 1e-5, (1.0 - np.exp(-tau)) / np.maximum(tau, 1e-300),
                        1.0 - 0.5 * tau)
    return (1.0 - beta) * (delta / (1.0 + delta))


def esc_table() -> EscTable:
    gamma = np.logspace(-6, 6, 81)
    delta = np.logspace(-4, 8, 41)
    p = _esc_fn(gamma[None, :], delta[:, None])
    return EscTable(delta=delta, gamma=gamma, p=np.ascontiguousarray(p))


def overlap_tables():
    """Synthetic 4-D tables p1 (own line) and p2 (cross term) on the
    (log10 delta, dx, gamma ratio, gamma) grids of lvg_line_overlap_data."""
    ld = np.linspace(-4, 8, 13)
    dx = np.linspace(-4, 4, 17)
    gr = np.array([0.01, 0.03, 0.1, 0.3, 1.0, 3.0, 10.0, 30.0, 100.0])
    gm = np.logspace(-6, 6, 41)
    D, X, R, G = np.meshgrid(10.0 ** ld, dx, gr, gm, indexing="ij")
    w = np.exp(-0.5 * X * X) / (1.0 + R)
    base = _esc_fn(G, D)
    p1 = base * (1.0 - 0.3 * w)
    p2 = 0.3 * w * base
    shp = (ld.size * dx.size, gr.size * gm.size)
    t1 = OverlapTable(ld, dx, gr, gm, np.ascontiguousarray(p1.reshape(shp)))
    t2 = OverlapTable(ld, dx, gr, gm, np.ascontiguousarray(p2.reshape(shp)))
    return t1, t2


def dust_components():
    a = 0.5e-5
    e = np.logspace(-3, 5, 161)
    q = np.minimum(1.0, 1e-3 * (e / 100.0) ** 2)
    return [DustComponent(energy=e, abs_coeff=np.pi * a * a * q, wvl_exp=2.0)]


def _coll_table(rng, energy, tgrid, nb_lev=None, scale=1.0):
    n = energy.size if nb_lev is None else nb_lev
    f, s = np.tril_indices(n, -1)                  # f > s, row-major: f(f-1)/2 + s order
    order = np.lexsort((s, f))
    f, s = f[order], s[order]
    de = energy[f] - energy[s]
    amp = 1e-11 * scale * np.exp(-de / 100.0) * rng.uniform(0.5, 1.5, size=f.size)
    T = np.asarray(tgrid, dtype=np.float64)
    coeff = amp[:, None] * np.sqrt(1.0 + T[None, :] / 100.0)
    coeff[:, T == 0.0] = 0.0
    return CollTable(nb_lev=n, tgrid=T, coeff=np.ascontiguousarray(coeff))


def _einstein(rng, energy, g, allowed):
    N = energy.size
    A = np.zeros((N, N))
    u, l = np.nonzero(allowed)
    for ui, li in zip(u, l):
        if ui <= li:
            continue
        de = energy[ui] - energy[li]
        a = 3e-7 * de ** 3 * rng.uniform(0.1, 1.0)
        A[ui, li] = a
        A[li, ui] = g[ui] * a / float(g[li])
    return A


# ---- molecules ------------------------------------------------------------------

def ch3oh(rng, N=256, symmetry="A"):
    """Torsion-rotation ladder vt=0..2 (NB_VIBR_EXCIT_CH3OH_RABLI, coll_rates_ch3oh.h:7)."""
    spin = 1.5 if symmetry == "A" else 0.5
    B, Arot = 0.80, 4.25
    lev = []
    for v in range(3):
        for J in range(0, 40):
            for K in range(-min(J, 9), min(J, 9) + 1):
                e = 200.0 * v + B * J * (J + 1) + (Arot - B) * K * K + 0.37 * K + (0.9 if symmetry == "E" else 0.0) * v
                lev.append((e, v, J, K))
    lev.sort()
    lev = lev[:N]
    energy = np.array([x[0] for x in lev]) + rng.uniform(0, 1e-3, N)
    energy = np.maximum.accumulate(energy + np.arange(N) * 1e-9)
    v = np.array([x[1] for x in lev], dtype=np.int32)
    J = np.array([x[2] for x in lev], dtype=np.float64)
    K = np.array([x[3] for x in lev])
    g = ((2 * spin + 1) * (2 * J + 1)).astype(np.int32)
    allowed = ((v[:, None] == v[None, :]) & (np.abs(J[:, None] - J[None, :]) <= 1)
               & (np.abs(K[:, None] - K[None, :]) <= 1))
    np.fill_diagonal(allowed, False)
    A = _einstein(rng, energy, g, allowed)
    mol = Molecule(name="CH3OH" + ("a" if symmetry == "A" else "e"), mass=32.0 * AMU, energy=energy,
                   g=g, einst=A, v=v, j=J, spin=spin)
    he = _coll_table(rng, energy, np.arange(41) * 10.0)                       # coll_rates_ch3oh.cpp:40-44
    ph2 = _coll_table(rng, energy, np.concatenate([[0.0], np.arange(1, 21) * 10.0]))   # :242
    oh2 = _coll_table(rng, energy, np.concatenate([[0.0], np.arange(1, 21) * 10.0]))   # :352
    coll = Collisions(rule=LVG_COLL_CH3OH, neutral=[he, ph2, oh2])
    return mol, coll


def para_h2o(rng, N=45):
    lev = []
    for J in range(0, 16):
        for tau in range(-J, J + 1):
            e = 9.0 * J * (J + 1) + 8.5 * tau * tau / (J + 1.0) + 5.0 * tau
            lev.append((e, J, tau))
    lev.sort()
    lev = lev[:N]
    energy = np.array([x[0] for x in lev]) + rng.uniform(0, 0.05, N)
    energy = energy - energy[0]
    energy = np.maximum.accumulate(energy + np.arange(N) * 1e-6)
    J = np.array([x[1] for x in lev], dtype=np.float64)
    tau = np.array([x[2] for x in lev])
    g = (2 * J + 1).astype(np.int32)
    allowed = (np.abs(J[:, None] - J[None, :]) <= 1) & (np.abs(tau[:, None] - tau[None, :]) <= 2)
    allowed &= rng.uniform(size=allowed.shape) < 0.7
    allowed = allowed | allowed.T
    np.fill_diagonal(allowed, False)
    A = _einstein(rng, energy, g, allowed)
    mol = Molecule(name="pH2O", mass=18.0 * AMU, energy=energy, g=g, einst=A,
                   v=np.zeros(N, np.int32), j=J, spin=0.0)
    grid = lambda pts: np.concatenate([[0.0], np.asarray(pts, dtype=np.float64)])
    tabs = [
        _coll_table(rng, energy, grid([20, 50, 100, 200, 300, 500, 1000, 2000]), nb_lev=min(45, N)),       # He (coll_rates_h2o.cpp:35-37)
        _coll_table(rng, energy, grid(np.linspace(100, 2000, 11))),                                        # He rovib
        _coll_table(rng, energy, grid([20, 40, 60, 80, 100, 200, 400, 800, 1000, 1500]), nb_lev=min(45, N)),  # pH2
        _coll_table(rng, energy, grid([20, 40, 60, 80, 100, 200, 400, 800, 1000, 1500]), nb_lev=min(45, N)),  # oH2
        _coll_table(rng, energy, grid(np.linspace(200, 2000, 11))),                                        # H2 rovib
        _coll_table(rng, energy, grid(np.linspace(5, 1500, 14)), nb_lev=min(45, N)),                        # H
    ]
    etab = _coll_table(rng, energy, grid(np.linspace(200, 4000, 11)), scale=1e4)                           # e-
    etab.species = LVG_SP_E
    coll = Collisions(rule=LVG_COLL_H2O, neutral=tabs, electron=[etab])
    return mol, coll


def oh_hf(rng, N=24):
    """12 parent levels, each split into two hyperfine components (2p, 2p+1)."""
    assert N % 2 == 0
    npar = N // 2
    Jvals = [1.5, 1.5, 2.5, 2.5, 0.5, 0.5, 3.5, 3.5, 1.5, 1.5, 4.5, 4.5, 2.5, 2.5, 5.5, 5.5]
    base = [0.0, 0.0556, 83.72, 83.84, 126.29, 126.45, 187.49, 187.70, 188.45, 188.79,
            289.16, 289.48, 288.60, 289.0, 415.5, 416.0]
    for p in range(16, npar):          # more Lambda doublets for larger N (the reference's OH-HF has 56 levels)
        Jvals.append(Jvals[p - 8] + 2.0)
        base.append(base[p - 2] + 130.0 + (0.3 if p % 2 else 0.0))
    par_e = np.sort(np.array(base[:npar]) + rng.uniform(0, 0.02, npar) * (np.arange(npar) % 2))
    par_e = np.maximum.accumulate(par_e + np.arange(npar) * 1e-3)
    Jp = np.array(Jvals[:npar])
    hf = rng.uniform(1e-5, 5e-4, npar)
    energy = np.empty(N)
    energy[0::2] = par_e
    energy[1::2] = par_e + hf
    J = np.repeat(Jp, 2)
    g = np.empty(N, np.int32)
    g[0::2] = (2 * Jp).astype(np.int32)
    g[1::2] = (2 * Jp + 2).astype(np.int32)
    A = np.zeros((N, N))
    for p in range(1, npar):
        for q in range(p):
            if abs(Jp[p] - Jp[q]) > 1.0 or rng.uniform() > 0.75:
                if not (p == q + 1 and p % 2 == 1):
                    continue
            comps = [(0, 0), (1, 1)] + [c for c in [(0, 1), (1, 0)] if rng.uniform() < 0.6]
            for m, l in comps:
                u, lo = 2 * p + m, 2 * q + l
                de = energy[u] - energy[lo]
                a = 3e-7 * de ** 3 * rng.uniform(0.1, 1.0) * (1.0 if m == l else 0.2)
                A[u, lo] = a
                A[lo, u] = g[u] * a / float(g[lo])
    mol = Molecule(name="OH", mass=17.0 * AMU, energy=energy, g=g, einst=A,
                   v=np.zeros(N, np.int32), j=J, spin=0.5)
    grid = np.concatenate([[0.0], np.linspace(10, 300, 10)])
    coll = Collisions(rule=LVG_COLL_OH_HF, neutral=[_coll_table(rng, energy, grid),
                                                    _coll_table(rng, energy, grid),
                                                    _coll_table(rng, energy, grid)])
    return mol, coll


# ---- layers ------------------------------------------------------------------------

def _loguni(rng, lo, hi, n):
    return 10.0 ** rng.uniform(np.log10(lo), np.log10(hi), n)


def make_layers(T, nh2, x, dvdz) -> Layers:
    T = np.asarray(T, dtype=np.float64)
    nh2 = np.asarray(nh2, dtype=np.float64)
    n = T.size
    return Layers(
        temp_n=T.copy(), temp_el=T.copy(), el_conc=1e-7 * nh2, h_conc=1e-3 * nh2,
        ph2_conc=0.25 * nh2, oh2_conc=0.75 * nh2, he_conc=HE_TO_H2 * nh2,
        mol_conc=np.asarray(x, dtype=np.float64) * nh2, vel_turb=np.full(n, V_TURB),
        vel_grad=np.asarray(dvdz, dtype=np.float64),
        dust_conc=(1.23e-11 * 2.0 * nh2)[:, None].copy())


def random_layers(rng, n, T, nh2, x, dvdz):
    sign = np.where(rng.uniform(size=n) < 0.5, -1.0, 1.0)
    return make_layers(_loguni(rng, *T, n), _loguni(rng, *nh2, n), _loguni(rng, *x, n),
                       sign * _loguni(rng, *dvdz, n))


# ---- BASELINE.json configurations ---------------------------------------------------

CONFIGS = {
    # name: (molecule, N, layers, seed)
    "oh24_single": ("oh_hf", 24, 1, 24),
    "ph2o45_1024": ("ph2o", 45, 1024, 45),
    "ch3oha256_4096": ("ch3oh_a", 256, 4096, 256),
    "ch3ohe256_sweep": ("ch3oh_e", 256, 128 * 128, 257),
    "oh24_overlap_2048": ("oh_hf", 24, 2048, 2048),
}


def make_problem(name: str, nb_lay: int | None = None, nb_lev: int | None = None):
    """Return (Problem, Layers, opts_overrides) for a BASELINE configuration.
    nb_lay / nb_lev shrink the case for CPU-sized parity tests (same generator)."""
    kind, N, L, seed = CONFIGS[name]
    N = nb_lev or N
    L = nb_lay or L
    rng = np.random.default_rng(seed)
    esc = esc_table()
    dust = dust_components()
    ov1 = ov2 = None
    opts = {}
    if kind == "ch3oh_a" or kind == "ch3oh_e":
        mol, coll = ch3oh(rng, N, "A" if kind == "ch3oh_a" else "E")
        opts["allow_plain_retry"] = 0           # radiative_transfer.cpp:259
    elif kind == "ph2o":
        mol, coll = para_h2o(rng, N)
    else:
        mol, coll = oh_hf(rng, N)
        opts["acceleration"] = 0                # radiative_transfer.cpp:440, :571
    lrng = np.random.default_rng(seed + 1000)
    if name == "oh24_single":
        layers = make_layers(np.full(L, 50.0), np.full(L, 1e6), np.full(L, 1e-6), np.full(L, 1e-9))
    elif name == "ph2o45_1024":
        layers = random_layers(lrng, L, (20, 1000), (1e4, 1e8), (1e-7, 1e-4), (1e-10, 1e-7))
    elif name == "ch3oha256_4096":
        layers = random_layers(lrng, L, (20, 300), (1e4, 1e8), (1e-9, 1e-6), (1e-10, 1e-7))
    elif name == "ch3ohe256_sweep":
        side = int(round(np.sqrt(L)))
        nh = np.logspace(3, 9, side)
        T = np.logspace(1, np.log10(400.0), side)
        NH, TT = np.meshgrid(nh, T, indexing="ij")
        nh, T = NH.reshape(-1)[:L], TT.reshape(-1)[:L]
        layers = make_layers(T, nh, np.full(T.size, 1e-7), np.full(T.size, 1e-9))
    else:
        ov1, ov2 = overlap_tables()
        opts["line_overlap"] = 1
        layers = random_layers(lrng, L, (20, 200), (1e4, 1e8), (1e-8, 1e-5), (1e-10, 1e-7))
    prob = Problem(mol=mol, coll=coll, dust=dust, esc=esc, overlap1=ov1, overlap2=ov2)
    return prob, layers, opts


def geometry(nb_lay: int, seed: int = 7, v_shock: float = 2.0e6, dz: float = 1.0e13):
    """Synthetic cloud geometry for the post-processing (synth_v1): layer thickness
    dz (cm, +-20 %), gas velocity decreasing from v_shock to 0 across the layers as in
    a C-shock profile (cm/s); height = zu(last) - zl(first) = sum of dz."""
    from .abi import Geometry
    rng = np.random.default_rng(seed)
    d = dz * rng.uniform(0.8, 1.2, nb_lay)
    vel = v_shock * (1. - np.linspace(0., 1., nb_lay)) ** 2
    return Geometry(d, vel, float(d.sum()))

