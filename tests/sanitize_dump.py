"""Dump a Problem + Layers (+ geometry, solve options) as manifest.txt + <name>.bin, the
input of tests/cpp/oracle_driver.c (test infrastructure, tests/test_sanitizers_cpu.py)."""
import os

import numpy as np


def _put(d, man, name, a, dt):
    a = np.ascontiguousarray(a, dtype=np.float64 if dt == "f8" else np.int32).reshape(-1)
    a.tofile(os.path.join(d, name + ".bin"))
    man.append(f"{name} {dt} {a.size}")


def dump_problem(d, P, L, geo, opts):
    os.makedirs(d, exist_ok=True)
    man = []
    m = P.mol
    N = m.nb_lev
    _put(d, man, "mol_mass", [m.mass], "f8")
    _put(d, man, "mol_energy", m.energy, "f8")
    _put(d, man, "mol_g", m.g, "i4")
    _put(d, man, "mol_v", m.v if m.v is not None else np.zeros(N), "i4")
    _put(d, man, "mol_j", m.j if m.j is not None else np.zeros(N), "f8")
    _put(d, man, "mol_einst", m.einst, "f8")
    tabs = list(P.coll.neutral) + list(P.coll.electron)
    _put(d, man, "coll_meta", [P.coll.rule, len(P.coll.neutral), len(P.coll.electron)], "i4")
    for t, T in enumerate(tabs):
        _put(d, man, f"coll_t{t}_meta", [T.nb_lev, len(T.tgrid), T.species], "i4")
        _put(d, man, f"coll_t{t}_tgrid", T.tgrid, "f8")
        _put(d, man, f"coll_t{t}_coeff", T.coeff, "f8")
    _put(d, man, "dust_meta", [len(P.dust)], "i4")
    for c, dc in enumerate(P.dust):
        _put(d, man, f"dust_c{c}_energy", dc.energy, "f8")
        _put(d, man, f"dust_c{c}_abs", dc.abs_coeff, "f8")
        _put(d, man, f"dust_c{c}_wvl_exp", [dc.wvl_exp], "f8")
    _put(d, man, "esc_delta", P.esc.delta, "f8")
    _put(d, man, "esc_gamma", P.esc.gamma, "f8")
    _put(d, man, "esc_p", P.esc.p, "f8")
    for q, t in ((1, P.overlap1), (2, P.overlap2)):
        if t is not None:
            for f, a in (("ld", t.log10_delta), ("dx", t.dx), ("gr", t.gratio), ("g", t.gamma), ("p", t.p)):
                _put(d, man, f"ov{q}_{f}", a, "f8")
    for f in ("temp_n", "temp_el", "el_conc", "h_conc", "ph2_conc", "oh2_conc", "he_conc", "mol_conc", "vel_turb",
              "vel_grad"):
        _put(d, man, "lay_" + f, getattr(L, f), "f8")
    _put(d, man, "lay_dust_conc", L.dust_conc if L.dust_conc is not None else np.zeros(1), "f8")
    _put(d, man, "geo_dz", geo.dz, "f8")
    _put(d, man, "geo_vel_n", geo.vel_n, "f8")
    _put(d, man, "geo_height", [geo.height], "f8")
    _put(d, man, "opts_i", [opts.acceleration, opts.allow_plain_retry, opts.max_iter_acc, opts.max_iter_plain], "i4")
    with open(os.path.join(d, "manifest.txt"), "w") as f:
        f.write("\n".join(man) + "\n")
