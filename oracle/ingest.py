"""Expected results of the input-file readers (radiative_transfer_amd/host/lvg_ingest.cpp),
derived in numpy from the synthetic "truth" that tests/ingest_files.py wrote to disk.

TEST INFRASTRUCTURE ONLY: imported by tests/test_ingest_cpu.py, never by the product.
Each function restates the reference reader named in its docstring on the values the
file holds (not on the file text), so a parse error in the C++ reader — a skipped line,
a token read into the wrong field, a lost sign — shows up as a mismatch.
Parity unpinned: the reference ships no data files; the formats are
read off the reference's parsing code.
"""
from __future__ import annotations

import math

import numpy as np

CM_INVERSE_TO_KELVINS = 1.438776877   # lvg_ingest.hpp (CODATA 2018, as the oracle)
PLANCK_CONSTANT = 6.62607015e-27
DEBYE = 1.e-18
MIN_VELOCITY_GRADIENT = 3.e-14        # cloud_data.cpp:13
SP_HE, SP_PH2, SP_OH2, SP_H, SP_E = 0, 1, 2, 3, 4   # include/lvg_amd.h


def rounding(x):
    return math.floor(x + 0.5)


def pair(u, l):
    """Packed index of the pair u > l (collision_data row order)."""
    return u * (u - 1) // 2 + l


class Diagram:
    def __init__(self, levels):
        """levels: dicts with v, j, k1, k2, hf, syminv, g, energy (reference order)."""
        self.lev = levels
        self.n = len(levels)
        self.g = np.array([l["g"] for l in levels], dtype=np.float64)
        self.e = np.array([l["energy"] for l in levels], dtype=np.float64)

    def arrays(self):
        f = lambda k: np.array([l[k] for l in self.lev])
        return dict(energy=f("energy").astype(np.float64), j=f("j").astype(np.float64),
                    k1=f("k1").astype(np.float64), k2=f("k2").astype(np.float64),
                    hf=f("hf").astype(np.float64), g=f("g").astype(np.int32), v=f("v").astype(np.int32),
                    syminv=f("syminv").astype(np.int32))


def _level(**kw):
    d = dict(v=0, j=0., k1=0., k2=0., hf=0., syminv=0, g=1, energy=0.)
    d.update(kw)
    return d


# ---- CH3OH (spectroscopy.cpp:295-394, :865-927; coll_rates_ch3oh.cpp:27-441) -------------------
def ch3oh_diagram(blocks, spin, n_l, nb_vibr=2, ang_mom_max=22):
    """Levels of one symmetry species: energies relative to the J=0 K=0 vt=0 A row,
    sorted by energy, cut to n_l (spectroscopy.cpp:321-385)."""
    a_type = rounding(2 * spin) == 3
    e_min = blocks[0][0][4][0]
    out = []
    for rows in blocks:
        for ch1, ch2, J, K, e in rows:
            if (ch1 == "A") != a_type:
                continue
            for vt in range(9):
                if vt <= nb_vibr and J <= ang_mom_max:
                    out.append(_level(v=vt, j=float(J), k1=float(-K if ch2 == "-" else K),
                                      g=rounding(2 * spin + 1) * (2 * J + 1), energy=e[vt] - e_min))
    out.sort(key=lambda l: l["energy"])
    return Diagram(out[:n_l])


def ch3oh_get_nb(di, v, j, k):   # spectroscopy.cpp:387-394
    for i, l in enumerate(di.lev):
        if l["v"] == v and rounding(l["j"]) == rounding(j) and rounding(l["k1"]) == rounding(k):
            return i
    return -1


def ch3oh_einstein(di, lines):
    """lines: (vt_u, J_u, K_u, vt_l, J_l, K_l, S); A from the line strength
    (spectroscopy.cpp:893-923); later lines overwrite earlier ones."""
    a = np.zeros((di.n, di.n))
    for vu, ju, ku, vl, jl, kl, S in lines:
        up, low = ch3oh_get_nb(di, vu, ju, ku), ch3oh_get_nb(di, vl, jl, kl)
        if up < 0 or low < 0:
            continue
        de = di.e[up] - di.e[low]
        a[up, low] = 64. * S * DEBYE * DEBYE * math.pi * math.pow(math.pi * de, 3.) / (
            3. * PLANCK_CONSTANT * (2. * di.lev[up]["j"] + 1.))
        a[low, up] = di.g[up] * a[up, low] / di.g[low]
    return a


def _ch3oh_accumulate(coeff, di, nb_arr, vals, tg, j, reset_same_v):
    """coll_rates_ch3oh.cpp:93-124 / :179-216 for one temperature block:
    vals[final][initial] in the file's level order."""
    n = len(nb_arr)
    for i in range(n):
        for k in range(n):
            i1, i2 = nb_arr[k], nb_arr[i]
            if i1 < 0 or i2 < 0 or i1 == i2:
                continue
            rate = vals[i, k]
            reset = reset_same_v and k > i and di.lev[i1]["v"] == di.lev[i2]["v"]
            if i1 > i2:
                p = pair(i1, i2)
                if reset:
                    coeff[p, j] = 0.
                coeff[p, j] += 0.5 * rate
            else:
                p = pair(i2, i1)
                if reset:
                    coeff[p, j] = 0.
                coeff[p, j] += 0.5 * rate * di.g[i1] / di.g[i2] * math.exp(
                    (di.e[i2] - di.e[i1]) * CM_INVERSE_TO_KELVINS / tg[j])


def ch3oh_collisions(di, truth):
    """He (41-point grid, vt files then the rovibrational file), pH2, oH2 tables."""
    imax = di.n * (di.n - 1) // 2
    tables = []
    # He: coll_rates_ch3oh.cpp:27-226
    tg = np.arange(41) * 10.
    c = np.zeros((imax, 41))
    for vt in range(3):
        pick, tgf, vals = truth[("he", vt)]
        nb_arr = [ch3oh_get_nb(di, vt, J, K) for _, J, K in pick]
        for j in range(1, 21):
            tg[j] = tgf[j - 1]
            _ch3oh_accumulate(c, di, nb_arr, vals[j - 1], tg, j, False)
    c[:, 21:] = c[:, 20:21]
    pick, tgf, vals = truth[("he", "rovibr")]
    nb_arr = [ch3oh_get_nb(di, v, J, K) for v, J, K in pick]
    for j in range(1, 41):
        tg[j] = tgf[j - 1]
        _ch3oh_accumulate(c, di, nb_arr, vals[j - 1], tg, j, True)
    tables.append((tg.copy(), c, SP_HE, di.n))
    # pH2 (vt files, :228-333), oH2 (vt = 0, :335-441)
    for part, vts, sp in (("ph2", range(3), SP_PH2), ("oh2", [0], SP_OH2)):
        tg = np.zeros(21)
        c = np.zeros((imax, 21))
        for vt in vts:
            pick, tgf, vals = truth[(part, vt)]
            nb_arr = [ch3oh_get_nb(di, vt, J, K) for _, J, K in pick]
            for j in range(1, 21):
                tg[j] = tgf[j - 1]
                _ch3oh_accumulate(c, di, nb_arr, vals[j - 1], tg, j, False)
        tables.append((tg, c, sp, di.n))
    return dict(nb1=3, nb2=3, tables=tables)


# ---- H2O (spectroscopy.cpp:218-293, :816-863; coll_rates_h2o.cpp:28-513) --------------------------
def vibr_nb(v1, v2, v3):   # spectroscopy.cpp:284-293
    return {(0, 0, 0): 0, (0, 1, 0): 1, (0, 2, 0): 2, (1, 0, 0): 3, (0, 0, 1): 4}.get((v1, v2, v3), 5)


def h2o_diagram(rows, spin, n_l, nb_vibr=4):
    out = []
    for v1, v2, v3, J, ka, kc, e in rows:
        if len(out) >= n_l:
            break
        v = vibr_nb(v1, v2, v3)
        if abs(ka + kc + v3) % 2 == rounding(spin) and v <= nb_vibr:
            out.append(_level(v=v, j=float(J), k1=float(ka), k2=float(kc), g=rounding(2 * spin + 1) * (2 * J + 1),
                              energy=e))
    return Diagram(out)


def h2o_get_nb(di, v, j, tau):   # spectroscopy.cpp:275-282
    for i, l in enumerate(di.lev):
        if l["v"] == v and rounding(l["j"]) == rounding(j) and rounding(l["k1"] - l["k2"]) == rounding(tau):
            return i
    return -1


def h2o_label(di, i):
    l = di.lev[i]
    return (l["v"], int(l["j"]), int(l["k1"] - l["k2"]))


def h2o_einstein(di, lines):
    a = np.zeros((di.n, di.n))
    for u, l, coeff in lines:
        up = h2o_get_nb(di, vibr_nb(*u[:3]), u[3], u[4] - u[5])
        low = h2o_get_nb(di, vibr_nb(*l[:3]), l[3], l[4] - l[5])
        if up < 0 or low < 0:
            continue
        a[up, low] = coeff
        a[low, up] = di.g[up] * coeff / di.g[low]
    return a


def h2o_collisions(di, t):
    """Tables in the rule's slot order (coll_rates_h2o.cpp:494-503):
    He, He rovibr, pH2, oH2, H2 rovibr, H | e rovibr."""
    n45 = 45
    im45 = n45 * (n45 - 1) // 2
    imax = di.n * (di.n - 1) // 2

    def packed(name, sp):
        tg, vals = t[name]
        c = np.zeros((im45, len(tg) + 1))
        m = min(len(vals), im45)
        c[:m, 1:] = vals[:m]
        return (np.concatenate([[0.], tg]), c, sp, n45)

    def labelled(name, sp):
        tg, rows, vals = t[name]
        c = np.zeros((imax, len(tg) + 1))
        for (a, b), v in zip(rows, vals):
            up, low = h2o_get_nb(di, *a), h2o_get_nb(di, *b)
            if up >= 0 and low >= 0:
                c[pair(up, low), 1:] = v
        return (np.concatenate([[0.], tg]), c, sp, di.n)

    # He, both directions (coll_rates_h2o.cpp:246-271)
    tg, vals = t["he"]
    tgf = np.concatenate([[0.], tg])
    c = np.zeros((im45, len(tgf)))
    for li in range(1, n45):
        for lf in range(li):
            if li >= di.n:
                continue
            i, f = li * (n45 - 1) + lf, lf * (n45 - 1) + li - 1
            for j in range(1, len(tgf)):
                c[pair(li, lf), j] = 0.5 * (vals[i, j - 1] + vals[f, j - 1] * di.g[lf] / di.g[li] * math.exp(
                    (di.e[li] - di.e[lf]) * CM_INVERSE_TO_KELVINS / tgf[j]))
    he = (tgf, c, SP_HE, n45)
    tables = [he, labelled("he_rovibr", SP_HE), packed("ph2", SP_PH2), packed("oh2", SP_OH2),
              labelled("h2_rovibr", SP_PH2), packed("h", SP_H), labelled("e_rovibr", SP_E)]
    return dict(nb1=6, nb2=7, tables=tables)


# ---- OH hyperfine (spectroscopy.cpp:560-619, :1090-1131; coll_rates_oh.cpp:129-378) -----------------
def oh_diagram(rows, n_l):
    return Diagram([_level(v=v, j=J, k1=om, syminv=p, hf=float(F), g=2 * F + 1, energy=e)
                    for v, J, om, p, F, e in rows[:n_l]])


def oh_get_nb(di, parity, v, j, omega, hf):
    for i, l in enumerate(di.lev):
        if (l["v"] == v and rounding(2 * l["j"]) == rounding(2 * j) and rounding(2 * l["k1"]) == rounding(2 * omega)
                and rounding(2 * l["hf"]) == rounding(2 * hf) and l["syminv"] == parity):
            return i
    return -1


def oh_einstein(di, lines):
    a = np.zeros((di.n, di.n))
    for u, l, coeff in lines:
        up = oh_get_nb(di, u[3], u[0], u[1], u[2], u[4])
        low = oh_get_nb(di, l[3], l[0], l[1], l[2], l[4])
        if up < 0 or low < 0:
            continue
        a[up, low] = coeff
        a[low, up] = di.g[up] * coeff / di.g[low]
    return a


def oh_collisions(nb, t):
    """He (coll_rates_oh.cpp:250-293) then the extended pH2 / oH2 tables (:196-248)."""
    imax = nb * (nb - 1) // 2
    tables = []
    tg, vals = t["he"]
    c = np.zeros((imax, len(tg) + 1))
    for (li, lf), v in vals.items():
        c[pair(li - 1, lf - 1), 1:] = v
    tables.append((np.concatenate([[0.], tg]), c, SP_HE, nb))
    for name, sp in (("ph2", SP_PH2), ("oh2", SP_OH2)):
        tg, vals = t[name]
        c = np.zeros((imax, len(tg) + 1))
        for (li, lf, j), v in vals.items():
            c[pair(li - 1, lf - 1), j + 1] = v
        tables.append((np.concatenate([[0.], tg]), c, sp, nb))
    return dict(nb1=3, nb2=3, tables=tables)


# ---- cloud profiles (cloud_data.cpp:143-472) ---------------------------------------------------------
FIELDS = ["zl", "zu", "dz", "zm", "temp_n", "temp_el", "av_temp_d", "vel_n", "velg_n", "tot_h_conc", "he_conc",
          "h_conc", "oh2_conc", "ph2_conc", "el_conc", "mol_conc", "h2_opr", "vel_turb"]
AVERAGED = ["temp_n", "temp_el", "av_temp_d", "vel_n", "velg_n", "tot_h_conc", "he_conc", "h_conc", "oh2_conc",
            "ph2_conc", "el_conc", "mol_conc", "h2_opr", "vel_turb"]


def cloud_points(t):
    """Per-point values as set_physical_parameters reads them (cloud_data.cpp:269-345)."""
    phys, ab, dust, opr = t["phys"], t["ab"], t["dust"], t["opr"]
    pts = []
    for p in range(len(phys)):
        th = phys[p, 7]
        h2 = ab[p, 1] * th
        ph2 = h2 / (1. + opr[p])
        pts.append(dict(zl=phys[p, 0], zu=0., dz=0., zm=0., temp_n=phys[p, 2], temp_el=phys[p, 4],
                        vel_n=phys[p, 5], tot_h_conc=th, el_conc=phys[p, 9] * th, velg_n=phys[p, 12],
                        h2_opr=opr[p], h_conc=ab[p, 0] * th, he_conc=ab[p, 2] * th, ph2_conc=ph2,
                        oh2_conc=h2 - ph2, mol_conc=0., vel_turb=0., av_temp_d=dust[p, -1, 0],
                        dust_temp=list(dust[p, :-1, 0]), dust_conc=list(dust[p, :-1, 1] * th)))
    return pts


def set_physical_parameters(t):
    pts = cloud_points(t)
    lays = []
    for i in range(len(pts) - 1):
        c, n = dict(pts[i]), pts[i + 1]
        c["zu"] = n["zl"]
        c["dz"] = c["zu"] - c["zl"]
        c["zm"] = c["zl"] + 0.5 * c["dz"]
        for f in AVERAGED:
            c[f] = 0.5 * (c[f] + n[f])
        c["dust_temp"] = [0.5 * (a + b) for a, b in zip(c["dust_temp"], n["dust_temp"])]
        c["dust_conc"] = [0.5 * (a + b) for a, b in zip(c["dust_conc"], n["dust_conc"])]
        if abs(c["velg_n"]) < MIN_VELOCITY_GRADIENT:
            c["velg_n"] = MIN_VELOCITY_GRADIENT if c["velg_n"] > 0. else -MIN_VELOCITY_GRADIENT
        lays.append(c)
    return lays


def set_molecular_conc(lays, t, mol_name, f):
    z = list(t["phys"][:, 0])
    col = t["names"].index(mol_name)
    conc = [t["ab"][p, col] * t["phys"][p, 7] for p in range(len(z))]
    nz = len(z)
    for c in lays:
        j = 0
        while j < nz - 1 and z[j] < c["zl"]:
            j += 1
        k = j
        while k < nz - 1 and z[k] < c["zu"]:
            k += 1
        m = 0.
        if j > 0 and z[j] > c["zl"]:
            m += 0.5 * (z[j] - c["zl"]) * (conc[j] + conc[j - 1] + (conc[j] - conc[j - 1]) * (c["zl"] - z[j - 1])
                                           / (z[j] - z[j - 1]))
        while j < k:
            m += 0.5 * (z[j + 1] - z[j]) * (conc[j] + conc[j + 1])
            j += 1
        if k > 0 and z[k] > c["zu"]:
            m -= 0.5 * (z[k] - c["zu"]) * (conc[k] + conc[k - 1] + (conc[k] - conc[k - 1]) * (c["zu"] - z[k - 1])
                                           / (z[k] - z[k - 1]))
        c["mol_conc"] = m * (f / (c["zu"] - c["zl"]))
    return lays


def join_layers(lays, nb):
    """dz-weighted merge of every nb consecutive layers; the remainder is dropped."""
    out = []
    for i in range(0, nb * (len(lays) // nb), nb):
        grp = lays[i:i + nb]
        tot = 0.
        for g in grp:
            tot += g["dz"]
        x = [g["dz"] / tot for g in grp]
        c = dict(grp[0])
        c["zu"] = grp[-1]["zu"]
        c["dz"] = c["zu"] - c["zl"]
        c["zm"] = c["zl"] + 0.5 * c["dz"]
        for f in AVERAGED:
            s = grp[0][f] * x[0]
            for j in range(1, nb):
                s += grp[j][f] * x[j]
            c[f] = s
        for key in ("dust_temp", "dust_conc"):
            vals = []
            for q in range(len(grp[0][key])):
                s = grp[0][key][q] * x[0]
                for j in range(1, nb):
                    s += grp[j][key][q] * x[j]
                vals.append(s)
            c[key] = vals
        out.append(c)
    return out


def cloud_arrays(lays):
    """The layout tests/cpp/test_ingest.cpp dumps: FIELDS rows + the dust vector sizes
    (flattened field-major), the dust vectors, the cloud height."""
    fields = np.array([[c[f] for c in lays] for f in FIELDS] +
                      [[float(len(c["dust_temp"])) for c in lays], [float(len(c["dust_conc"])) for c in lays]])
    dt = np.array([v for c in lays for v in c["dust_temp"]])
    dc = np.array([v for c in lays for v in c["dust_conc"]])
    height = lays[-1]["zu"] - lays[0]["zl"]
    return fields.reshape(-1), dt, dc, height
