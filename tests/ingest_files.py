"""Writers of synthetic input directories in the reference's on-disk formats
(test infrastructure for tests/test_ingest_cpu.py).

The reference ships no data files, so each file is written from a
seeded synthetic "truth" exactly in the layout its reader consumes:
spectroscopy.cpp:295-385 / :865-927 (CH3OH), :218-273 / :816-863 (H2O),
:560-608 / :1090-1131 (OH hyperfine); coll_rates_ch3oh.cpp:27-441,
coll_rates_h2o.cpp:28-484, coll_rates_oh.cpp:129-293; cloud_data.cpp:228-472.
The truth is returned alongside, for oracle/ingest.py to derive the expected tables.
"""
from __future__ import annotations

import os

import numpy as np

def R(x):
    """Shortest round-trip text of a float: the C++ reader gets the same double."""
    return repr(float(x))


def _w(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


# ---- CH3OH ------------------------------------------------------------------------------
def ch3oh_levels_truth(rng, nb_ang_mom=22):
    """Rows of levels_ch3oh.txt per J block: A rows (K >= 0 with a sign), then E rows."""
    blocks = []
    for J in range(nb_ang_mom + 1):
        rows = []
        a_keys = [(0, "+")] + [(K, s) for K in range(1, J + 1) for s in "+-"]
        for K, s in a_keys:
            e = [100.0 + 150.0 * vt + 0.8 * J * (J + 1) + 3.45 * K * K + (0.013 * K if s == "+" else -0.011 * K)
                 + float(rng.uniform(0, 0.05)) for vt in range(9)]
            rows.append(("A", s, J, K, e))
        for K in range(-J, J + 1):
            e = [107.0 + 151.0 * vt + 0.8 * J * (J + 1) + 3.4 * K * K + 0.2 * K + float(rng.uniform(0, 0.05))
                 for vt in range(9)]
            rows.append(("E", " ", J, K, e))
        blocks.append(rows)
    return blocks


def write_ch3oh_levels(d, blocks):
    out = ["! synthetic CH3OH torsion-rotation levels\n", "! columns: sym J K E(vt=0..8)\n"]
    for J, rows in enumerate(blocks):
        out += [f"! J = {J}\n", "!\n", "!\n", "!\n"]
        for ch1, ch2, JJ, K, e in rows:
            lab = f"{ch1}{ch2}" if ch1 == "A" else f"{ch1}"
            out.append(f"{lab} {JJ} {K} " + " ".join(R(x) for x in e) + "\n")
    _w(os.path.join(d, "spectroscopy", "levels_ch3oh.txt"), "".join(out))


def a_levels(blocks, nb_vibr=2, ang_mom_max=99):
    """(vt, J, signed K) of the A-species rows, as the reader keeps them (unsorted)."""
    out = []
    for rows in blocks:
        for ch1, ch2, J, K, e in rows:
            if ch1 != "A":
                continue
            for vt in range(9):
                if vt <= nb_vibr and J <= ang_mom_max:
                    out.append((vt, J, -K if ch2 == "-" else K, e[vt]))
    return out


def write_ch3oh_radiative(d, lines):
    """lines: (vt_u, J_u, K_u, vt_l, J_l, K_l, S) with signed K (A species)."""
    out = ["! synthetic\n", "!\n", "!\n", "!\n", f"{len(lines)}\n"]
    for vu, ju, ku, vl, jl, kl, S in lines:
        su, sl = ("-" if ku < 0 else "+"), ("-" if kl < 0 else "+")
        out.append(f" {vu} {ju} {abs(ku)}{su} {vl} {jl} {abs(kl)}{sl} 12.5 0.0 {R(S)} 0 0 0 0 0 0\n")
    _w(os.path.join(d, "spectroscopy", "radiative_ch3oh_a.txt"), "".join(out))


def _rate_token(rng, x):
    """A rate value, sometimes in the reference's broken forms: 'a.b-dfg' (dropped)
    or negative (clipped to 0) -> (text, value the reader keeps)."""
    u = rng.uniform()
    if u < 0.03:
        return "2.5-13", 0.0
    if u < 0.05:
        return R(-abs(x)), 0.0
    return R(x), x


def ch3oh_coll_file(rng, levels, nT, tgrid, with_vt):
    """levels: (vt, J, K) listed at the head of the file; per temperature a full
    final x initial rate matrix. Returns (text, kept values [nT][n][n])."""
    n = len(levels)
    out = ["! synthetic CH3OH collision rates\n", "!\n", "!\n", "!\n"]
    for idx, (vt, J, K) in enumerate(levels):
        s = "-" if K < 0 else "+"
        out.append(f"{idx + 1} " + (f"{vt} " if with_vt else "") + f"A {s} {J} {abs(K)} 1.0\n")
    out += ["!\n", "!\n", "!\n"]
    vals = np.zeros((nT, n, n))
    for j in range(nT):
        out.append(R(float(tgrid[j])) + "\n")
        for i in range(n):
            toks = []
            for k in range(n):
                x = 0.0 if i == k else float(1e-11 * rng.uniform(0.1, 2.0))
                t, v = _rate_token(rng, x)
                toks.append(t)
                vals[j, i, k] = v
            out.append(f"{i + 1} " + " ".join(toks) + "\n")
    return "".join(out), vals


def write_ch3oh_coll(d, rng, pool, file_levels, file_levels_rovibr, file_levels_oh2):
    """pool: [(vt, J, K)] candidate levels (some absent from the diagram). Returns the truth."""
    truth = {}
    tg20 = np.arange(1, 21) * 10.0
    tg40 = np.arange(1, 41) * 10.0
    for part in ("he", "ph2"):
        for vt in range(3):
            cand = [x for x in pool if x[0] == vt]
            pick = [cand[i] for i in rng.choice(len(cand), size=min(file_levels, len(cand)), replace=False)]
            text, vals = ch3oh_coll_file(rng, pick, 20, tg20, False)
            _w(os.path.join(d, "coll_ch3oh", f"coll_ch3oh_a{vt}_{part}.txt"), text)
            truth[(part, vt)] = (pick, tg20, vals)
    pick = [pool[i] for i in rng.choice(len(pool), size=min(file_levels_rovibr, len(pool)), replace=False)]
    text, vals = ch3oh_coll_file(rng, pick, 40, tg40, True)
    _w(os.path.join(d, "coll_ch3oh", "coll_ch3oh_a_he_rovibr.txt"), text)
    truth[("he", "rovibr")] = (pick, tg40, vals)
    cand = [x for x in pool if x[0] == 0]
    pick = [cand[i] for i in rng.choice(len(cand), size=min(file_levels_oh2, len(cand)), replace=False)]
    text, vals = ch3oh_coll_file(rng, pick, 20, tg20, False)
    _w(os.path.join(d, "coll_ch3oh", "coll_ch3oh_a0_oh2.txt"), text)
    truth[("oh2", 0)] = (pick, tg20, vals)
    return truth


# ---- H2O --------------------------------------------------------------------------------------
def h2o_levels_truth(rng, n_rows=140):
    """(v1, v2, v3, J, ka, kc, E) rows of levels_h2o16.txt, both spin isomers, some excited."""
    rows = []
    vib = [(0, 0, 0), (0, 1, 0), (0, 2, 0), (1, 0, 0), (0, 0, 1), (0, 3, 0)]
    for J in range(0, 12):
        for ka in range(0, J + 1):
            for kc in (J - ka, J - ka + 1):
                if kc > J or kc < 0:
                    continue
                for vi, (v1, v2, v3) in enumerate(vib):
                    if vi and rng.uniform() > 0.08:
                        continue
                    e = 1595.0 * v2 + 3657.0 * v1 + 3756.0 * v3 + 9.3 * J * (J + 1) + 6.1 * ka * ka + float(rng.uniform(0, 1))
                    rows.append((v1, v2, v3, J, ka, kc, e))
    rows.sort(key=lambda r: r[6])
    return rows[:n_rows]


def write_h2o_levels(d, rows):
    out = ["! synthetic H2O levels\n", "! v1 v2 v3 J ka kc E\n", f"{len(rows)}\n"]
    out += [f"{a} {b} {c} {J} {ka} {kc} {R(e)}\n" for a, b, c, J, ka, kc, e in rows]
    _w(os.path.join(d, "spectroscopy", "levels_h2o16.txt"), "".join(out))


def write_h2o_radiative(d, lines):
    """lines: ((v1,v2,v3,J,ka,kc) up, (..) low, A)."""
    out = ["! synthetic\n", "!\n", f"{len(lines)}\n"]
    for u, l, a in lines:
        out.append(" ".join(str(x) for x in u) + "  " + " ".join(str(x) for x in l) + f" {R(a)} 100.0\n")
    _w(os.path.join(d, "spectroscopy", "radiative_h2o16.txt"), "".join(out))


def write_h2o_coll(d, rng, labels):
    """labels: (v, J, tau) of the diagram's levels in order, plus a few absent ones.
    Returns the truth of the seven files (coll_rates_h2o.cpp:28-484)."""
    t = {}
    n45 = 45
    imax = n45 * (n45 - 1) // 2
    r = lambda: float(1e-11 * rng.uniform(0.1, 2.0))
    # packed 45-level tables with "l li lf"
    for name, nT in (("oh2", 8), ("ph2", 8)):
        tg = np.sort(rng.uniform(10, 1500, nT))
        nb_lines = imax - 7
        vals = np.array([[r() for _ in range(nT)] for _ in range(nb_lines)])
        out = ["! synthetic\n", f"{nb_lines}\n", " ".join(R(float(x)) for x in tg) + "\n"]
        out += [f"{i + 1} 0 0 " + " ".join(R(x) for x in vals[i]) + "\n" for i in range(nb_lines)]
        _w(os.path.join(d, "coll_h2o", f"coll_ph2o_{name}.txt"), "".join(out))
        t[name] = (tg, vals)
    # H: "li lf x x", 14 temperatures, two comment lines
    tg = np.sort(rng.uniform(5, 1500, 14))
    nb_lines = imax
    vals = np.array([[r() for _ in range(14)] for _ in range(nb_lines)])
    out = ["! synthetic\n", "!\n", f"{nb_lines}\n", " ".join(R(float(x)) for x in tg) + "\n"]
    out += [f"0 0 0 0 " + " ".join(R(x) for x in vals[i]) + "\n" for i in range(nb_lines)]
    _w(os.path.join(d, "coll_h2o", "coll_ph2o_h.txt"), "".join(out))
    t["h"] = (tg, vals)
    # He: both directions of every pair, 10 temperatures
    tg = np.sort(rng.uniform(20, 2000, 10))
    nb_lines = 2 * imax
    vals = np.array([[r() for _ in range(10)] for _ in range(nb_lines)])
    out = ["! synthetic\n", f"{nb_lines}\n", " ".join(R(float(x)) for x in tg) + "\n"]
    out += [f"1 2 0 0 " + " ".join(R(x) for x in vals[i]) + "\n" for i in range(nb_lines)]
    _w(os.path.join(d, "coll_h2o", "coll_ph2o_he.txt"), "".join(out))
    t["he"] = (tg, vals)
    # labelled rovibrational tables (v J tau of both levels)
    pairs = [(u, l) for u in range(len(labels)) for l in range(u) if rng.uniform() < 0.4]
    extra = [((3, 30, 1), (0, 0, 0)), ((0, 1, 1), (5, 9, 9))]   # levels the diagram does not have
    for name, nT, ncom, header_jm in (("h2_rovibr", 11, 2, False), ("e_rovibr", 11, 2, False),
                                      ("he_rovibr", 9, 1, True)):
        tg = np.sort(rng.uniform(100, 4000, nT))
        rows = [(labels[u], labels[l]) for u, l in pairs] + extra
        vals = np.array([[r() for _ in range(nT)] for _ in range(len(rows))])
        out = ["! synthetic\n"] * ncom
        out.append(f"{len(rows)} {nT}\n" if header_jm else f"{len(rows)}\n")
        out.append(" ".join(R(float(x)) for x in tg) + "\n")
        for (a, b), v in zip(rows, vals):
            out.append(" ".join(str(x) for x in a) + " " + " ".join(str(x) for x in b) + " "
                       + " ".join(R(x) for x in v) + "\n")
        _w(os.path.join(d, "coll_h2o", f"coll_ph2o_{name}.txt"), "".join(out))
        t[name] = (tg, rows, vals)
    return t


# ---- OH hyperfine ---------------------------------------------------------------------------------
def oh_levels_truth(rng, n=24):
    rows = []
    e = 0.0
    for p in range(n // 2):
        J = 1.5 + (p // 2)
        e += float(rng.uniform(5, 60))
        for m in range(2):
            F = int(J - 0.5 + m)
            rows.append((0, J, 1.5 if p % 2 == 0 else 0.5, 1 if (p + m) % 2 == 0 else -1, F,
                         e + m * float(rng.uniform(1e-5, 5e-4))))
    return rows


def write_oh_levels(d, rows):
    out = ["! synthetic OH hyperfine levels\n", "!\n", "! v J omega parity F E\n", f"{len(rows)}\n"]
    out += [f"{v} {R(J)} {R(om)} {p} {F} {R(e)}\n" for v, J, om, p, F, e in rows]
    _w(os.path.join(d, "spectroscopy", "levels_oh_hf.txt"), "".join(out))


def write_oh_radiative(d, lines):
    out = ["! synthetic\n", "!\n", f"{len(lines)}\n"]
    for u, l, a in lines:
        out.append(f"{u[0]} {R(u[1])} {R(u[2])} {u[3]} {u[4]} {l[0]} {R(l[1])} {R(l[2])} {l[3]} {l[4]} {R(a)} 1.0\n")
    _w(os.path.join(d, "spectroscopy", "radiative_oh_hf.txt"), "".join(out))


def write_oh_coll(d, rng, nb):
    imax = nb * (nb - 1) // 2
    r = lambda: float(1e-11 * rng.uniform(0.1, 2.0))
    t = {}
    jm = 10
    tg = np.sort(rng.uniform(10, 300, jm))
    pairs = [(li, lf) for li in range(2, nb + 1) for lf in range(1, li)]
    order = rng.permutation(len(pairs))
    vals = {}
    out = ["!\n", "!\n", "!\n", f"{nb} {jm}\n", " ".join(R(float(x)) for x in tg) + "\n"]
    for o in order:
        li, lf = pairs[o]
        v = [r() for _ in range(jm)]
        vals[(li, lf)] = v
        out.append(f"{li} {lf} 0 0 " + " ".join(R(x) for x in v) + "\n")
    _w(os.path.join(d, "coll_oh", "coll_oh_hf_he.txt"), "".join(out))
    t["he"] = (tg, vals)
    for name in ("ph2", "oh2"):
        tg = np.sort(rng.uniform(10, 300, jm))
        vals = {}
        out = ["!\n", "!\n", "!\n", f"{nb} {jm}\n"]
        for j in range(jm):
            out.append(R(float(tg[j])) + "\n")
            allp = pairs + [(k, k) for k in range(1, nb + 1)]
            for o in rng.permutation(len(allp)):
                li, lf = allp[o]
                v = r()
                if li > lf:
                    vals[(li, lf, j)] = v
                out.append(f"{li} {lf} {R(v)}\n")
        _w(os.path.join(d, "coll_oh", f"coll_oh_hf_{name}_ext.txt"), "".join(out))
        t[name] = (tg, vals)
    assert imax == len(pairs)
    return t


# ---- cloud (cloud_data.cpp:228-472) ----------------------------------------------------------------
def write_cloud(d, rng, npts=13, ncomp=2):
    z = np.cumsum(rng.uniform(1e13, 5e13, npts))
    phys = np.zeros((npts, 13))
    phys[:, 0] = z
    phys[:, 2] = rng.uniform(20, 2000, npts)        # T_n
    phys[:, 4] = rng.uniform(20, 3000, npts)        # T_e
    phys[:, 5] = rng.uniform(1e5, 3e6, npts)        # v_n
    phys[:, 7] = 10 ** rng.uniform(4, 7, npts)      # n_H
    phys[:, 9] = 10 ** rng.uniform(-8, -6, npts)    # x_e
    phys[:, 12] = rng.uniform(-1e-8, 1e-8, npts)    # velocity gradient
    phys[3, 12] = 1e-15                             # below MIN_VELOCITY_GRADIENT
    phys[4, 12] = -2e-15
    for c in (1, 3, 6, 8, 10, 11):
        phys[:, c] = rng.uniform(0, 1, npts)
    opr = rng.uniform(0.1, 3.0, npts)
    names = ["H", "H2", "He", "CH3OH", "OH"]
    ab = np.zeros((npts, len(names)))
    ab[:, 0] = 10 ** rng.uniform(-4, -1, npts)
    ab[:, 1] = rng.uniform(0.3, 0.5, npts)
    ab[:, 2] = 0.09
    ab[:, 3] = 10 ** rng.uniform(-9, -6, npts)
    ab[:, 4] = 10 ** rng.uniform(-8, -6, npts)
    dust = rng.uniform(1, 100, (npts, ncomp + 1, 16))
    dust[:, :, 1] = 10 ** rng.uniform(-12, -10, (npts, ncomp + 1))
    row = lambda xs: " ".join(R(float(x)) for x in xs)
    _w(os.path.join(d, "sim_phys_param.txt"), "! phys\n# more\n" + "".join(row(r) + "\n" for r in phys) + "\n")
    _w(os.path.join(d, "sim_data_h2_chemistry.txt"), "! h2\n" + "".join(f"{R(float(a))} {R(float(b))}\n" for a, b in zip(z, opr)) + "\n")
    _w(os.path.join(d, "sim_specimen_abund.txt"), "! abundances\n!z " + " ".join(names) + "\n"
       + "".join(row([a] + list(b)) + "\n" for a, b in zip(z, ab)) + "\n")
    _w(os.path.join(d, "sim_dust_data.txt"), "! dust\n" + "".join(row([a] + list(b.reshape(-1))) + "\n" for a, b in zip(z, dust)) + "\n")
    return dict(z=z, phys=phys, opr=opr, names=names, ab=ab, dust=dust)
