"""CPU checks of the oracle (oracle/lvg_oracle.c) against independent numpy
restatements of the reference functions. The reference itself cannot be built
or run here (its numerics library is absent; DESIGN.md "Parity"), so these tests
pin each oracle building block to a second, vectorised implementation written
directly from the reference source lines cited below."""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from oracle import oracle

C2 = 1.438776877  # CM_INVERSE_TO_KELVINS


# ---- absent numerics library ---------------------------------------------------

def test_lu_solve_matches_numpy():
    rng = np.random.default_rng(1)
    for n in (1, 2, 4, 17, 45, 64):
        a = rng.normal(size=(n, n)) + n * np.eye(n)
        b = rng.normal(size=n)
        x = oracle.lu_solve(a, b)
        np.testing.assert_allclose(x, np.linalg.solve(a, b), rtol=1e-12, atol=1e-14)


def test_lu_partial_pivoting_takes_first_maximum():
    # column 0 has a tie between rows 1 and 2; a first-maximum rule pivots on row 1
    a = np.array([[1.0, 2.0, 3.0], [4.0, 1.0, 0.0], [-4.0, 5.0, 1.0]])
    b = np.array([1.0, 2.0, 3.0])
    np.testing.assert_allclose(oracle.lu_solve(a, b), np.linalg.solve(a, b), rtol=1e-14)


def test_portable_exp_log10_within_ulps_of_libm():
    rng = np.random.default_rng(2)
    L = oracle.lib()
    xs = rng.uniform(-700, 700, 20000)
    ex = np.array([L.oracle_exp(float(x)) for x in xs])
    ref = np.exp(xs)
    ulp = np.abs(ex - ref) / np.spacing(ref)
    assert ulp.max() <= 1.0
    ys = 10.0 ** rng.uniform(-300, 300, 20000)
    lg = np.array([L.oracle_log10(float(y)) for y in ys])
    ref = np.log10(ys)
    ok = np.abs(ref) > 1e-3
    assert (np.abs(lg - ref)[ok] / np.spacing(np.abs(ref[ok]))).max() <= 4.0
    assert L.oracle_exp(0.0) == 1.0 and L.oracle_log10(1000.0) == 3.0


# ---- tables ----------------------------------------------------------------------

def _bilinear_clamped(delta_grid, gamma_grid, p, gamma, delta):
    """lvg_method_functions.cpp:74-110, vectorised independently."""
    def idx_w(g, x):
        k = np.searchsorted(g, x, side="right") - 1
        below, above = x < g[0], x > g[-1]
        k = np.clip(k, 0, g.size - 2)
        w = (x - g[k]) / (g[k + 1] - g[k])
        w = np.where(below, 0.0, np.where(above, 1.0, w))
        return k, w
    k, t = idx_w(delta_grid, delta)
    l, u = idx_w(gamma_grid, gamma)
    e = (p[k, l] * (1 - t) * (1 - u) + p[k + 1, l] * t * (1 - u) + p[k, l + 1] * (1 - t) * u
         + p[k + 1, l + 1] * u * t)
    return np.clip(e, 0.0, 1.0)


def test_esc_func_bilinear_with_clamping():
    P, _, _ = synth.make_problem("oh24_single")
    rng = np.random.default_rng(3)
    g = 10.0 ** rng.uniform(-8, 8, 400)
    d = 10.0 ** rng.uniform(-6, 10, 400)
    got = np.array([oracle.esc_func(P, a, b) for a, b in zip(g, d)])
    ref = _bilinear_clamped(P.esc.delta, P.esc.gamma, P.esc.p, g, d)
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=1e-15)


def test_overlap_esc_func_multilinear():
    """lvg_method_functions.cpp:324-392 against scipy's regular-grid interpolator on clamped inputs."""
    from scipy.interpolate import RegularGridInterpolator
    P, _, _ = synth.make_problem("oh24_overlap_2048", nb_lay=2)
    T = P.overlap1
    grid4 = T.p.reshape(T.log10_delta.size, T.dx.size, T.gratio.size, T.gamma.size)
    f = RegularGridInterpolator((T.log10_delta, T.dx, T.gratio, T.gamma), grid4)
    rng = np.random.default_rng(4)
    for _ in range(300):
        g, d = 10.0 ** rng.uniform(-7, 7), 10.0 ** rng.uniform(-5, 9)
        gr, dx = 10.0 ** rng.uniform(-3, 3), rng.uniform(-5, 5)
        got = oracle.overlap_esc_func(P, 0, g, d, gr, dx)
        q = [np.clip(np.log10(d), T.log10_delta[0], T.log10_delta[-1]), np.clip(dx, T.dx[0], T.dx[-1]),
             np.clip(gr, T.gratio[0], T.gratio[-1]), np.clip(g, T.gamma[0], T.gamma[-1])]
        assert abs(got - float(np.clip(f(q)[0], 0, 1))) < 1e-12


# ---- collision rules -----------------------------------------------------------------

def _table_rate(tab, f, s, T):
    """collision_data::locate + get_rate (coll_rates.cpp:54-82), T clamped to max_temp."""
    tg = tab.tgrid
    lo = 0
    hi = tg.size - 1
    while hi - lo > 1:
        m = (lo + hi) // 2
        if tg[m] < T:
            lo = m
        else:
            hi = m
    Tc = min(T, tg[-1])
    i = f * (f - 1) // 2 + s
    c = tab.coeff[i]
    return c[lo] + (c[lo + 1] - c[lo]) / (tg[lo + 1] - tg[lo]) * (Tc - tg[lo])


def _up(mol, f, s, down, T):
    return down * np.exp((mol.energy[s] - mol.energy[f]) * C2 / T) * mol.g[f] / mol.g[s]


@pytest.mark.parametrize("name", ["ch3oha256_4096", "ph2o45_1024", "oh24_overlap_2048"])
def test_collision_rules(name):
    """ch3oh (coll_rates_ch3oh.cpp:484-533), h2o (coll_rates_h2o.cpp:530-548),
    oh_hf (coll_rates_oh.cpp:392-407), electrons (coll_rates.cpp:199-217)."""
    P, L, _ = synth.make_problem(name, nb_lay=3, nb_lev=40 if name.startswith("ch3oh") else None)
    mol, tabs, etabs = P.mol, P.coll.neutral, P.coll.electron
    lay = 1
    T, Te = L.temp_n[lay], L.temp_el[lay]
    he, ph2, oh2, h, e = L.he_conc[lay], L.ph2_conc[lay], L.oh2_conc[lay], L.h_conc[lay], L.el_conc[lay]
    dn, un, de, ue = oracle.coll_rates(P, L, lay)
    N = mol.nb_lev
    rng = np.random.default_rng(5)
    pairs = [(f, s) for f in range(1, N) for s in range(f)]
    for f, s in [pairs[i] for i in rng.choice(len(pairs), 150, replace=False)]:
        k = lambda t: _table_rate(tabs[t], f, s, T)
        if name.startswith("ch3oh"):
            if mol.v[f] == mol.v[s]:
                d = (k(1) * ph2 + k(2) * oh2) if (mol.v[f] == 0 and mol.j[f] <= 9 and mol.j[s] <= 9) else k(1) * (ph2 + oh2)
                d += k(0) * he
            else:
                d = k(0) * (he + ph2 + 3 * oh2)
        elif name.startswith("ph2o"):
            d = k(0) * he + k(2) * ph2 + k(3) * oh2 + k(5) * h if f < 45 else k(1) * (he + 0.2 * h) + k(4) * (ph2 + oh2)
        else:
            d = (k(0) * he if f < tabs[0].nb_lev else 0.0)
            if f < tabs[1].nb_lev:
                d += k(1) * ph2 + k(2) * oh2
        np.testing.assert_allclose(dn[f, s], d, rtol=1e-13)
        np.testing.assert_allclose(un[f, s], _up(mol, f, s, d, T), rtol=1e-13)
        if etabs:
            ed = _table_rate(etabs[0], f, s, Te) * e
            np.testing.assert_allclose(de[f, s], ed, rtol=1e-13)
            np.testing.assert_allclose(ue[f, s], _up(mol, f, s, ed, Te), rtol=1e-13)
        else:
            assert de[f, s] == 0.0 and ue[f, s] == 0.0


# ---- scheme ---------------------------------------------------------------------------

def test_boundary_layer_populations_matches_numpy():
    """iteration_control.cpp:52-91: neutral collisions + A/2, row 0 <- 1."""
    P, L, _ = synth.make_problem("ph2o45_1024", nb_lay=4)
    got = oracle.boundary_layer_populations(P, L)
    A = P.mol.einst
    N = P.mol.nb_lev
    for lay in range(4):
        dn, un, _, _ = oracle.coll_rates(P, L, lay)
        M = np.zeros((N, N))
        for f in range(1, N):
            for s in range(f):
                M[s, f] = 0.5 * A[f, s] + dn[f, s]
                M[f, s] = un[f, s]
        M -= np.diag(M.sum(axis=0))
        M[0, :] = 1.0
        b = np.zeros(N); b[0] = 1.0
        np.testing.assert_allclose(got[lay], np.linalg.solve(M, b), rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("name,overlap", [("ph2o45_1024", 0), ("oh24_overlap_2048", 1)])
def test_calc_new_pop_structure(name, overlap):
    """iteration_lvg.cpp:87-161: row 0 of ones, conservation in the other rows,
    the new populations solve M n = e0 and sum to one."""
    P, L, _ = synth.make_problem(name, nb_lay=2)
    bo = oracle.boundary_layer_populations(P, L)
    M, df, pn, eq = oracle.calc_new_pop(P, L, 0, bo[0], overlap)
    N = P.mol.nb_lev
    assert np.all(M[0] == 1.0)
    off = M - np.diag(np.diag(M))
    assert np.all(off[1:] >= 0.0)
    # columns d >= 1 conserve: sum_{r>=1} M[r][d] = -(rate d -> 0) <= 0 (row 0 was overwritten);
    # column 0 sums to the total outflow of level 0 (its diagonal sat in row 0)
    colsum = M[1:].sum(axis=0)
    assert np.all(colsum[1:] <= 1e-12 * np.abs(np.diag(M)).max())
    assert colsum[0] > 0.0
    np.testing.assert_allclose(M @ pn, np.eye(N)[0], atol=1e-12)
    assert abs(pn.sum() - 1.0) < 1e-12
    np.testing.assert_allclose(df, np.eye(N)[0] - M @ bo[0], rtol=1e-9, atol=1e-15)
    assert eq == np.abs(df).max()


def test_line_groups_follow_hfs_sort_quirk():
    """hfs_lines::sort (iteration_lvg.cpp:259-290): the 'closest pair' search never
    updates its running minimum, so the LAST gap smaller than the FIRST wins."""
    P, _, _ = synth.make_problem("oh24_overlap_2048", nb_lay=1)
    g = oracle.line_groups(P)
    assert g.shape[0] > 0 and set(np.unique(g[:, 0])) <= {1, 2}
    # every A > 1e-99 line between two different doublets appears exactly once
    N = P.mol.nb_lev
    lines = set()
    for row in g:
        lines.add((row[1], row[2]))
        if row[0] == 2:
            lines.add((row[3], row[4]))
    expect = {(u, l) for u in range(2, N) for l in range(N) if (l // 2) < (u // 2) and P.mol.einst[u, l] > 1e-99}
    assert lines == expect


def test_hfs_grouping_handmade():
    """init_molecule_data + hfs_lines::sort/split (iteration_lvg.cpp:259-346) on one
    doublet pair with exact binary energies: lines sorted by energy, reordered
    around the first line, the first two split off as an overlapping pair."""
    from radiative_transfer_amd.abi import Collisions, Molecule, Problem
    P, _, _ = synth.make_problem("oh24_overlap_2048", nb_lay=1)
    E = np.array([0.0, 0.5, 100.0, 100.25])
    A = np.zeros((4, 4))
    for u in (2, 3):
        for l in (0, 1):
            A[u, l] = A[l, u] = 1e-3
    mol = Molecule("t", P.mol.mass, E, np.full(4, 2, np.int32), A, np.zeros(4, np.int32), np.ones(4))
    tg = np.array([0.0, 10.0, 100.0, 300.0])
    rng = np.random.default_rng(0)
    coll = Collisions(P.coll.rule, [synth._coll_table(rng, E, tg) for _ in range(3)])
    g = oracle.line_groups(Problem(mol, coll, P.dust, P.esc, P.overlap1, P.overlap2))
    # line energies 99.5 (2,1), 99.75 (3,1), 100 (2,0), 100.25 (3,0): equal gaps -> centre 99.5
    assert g.tolist() == [[2, 2, 1, 3, 1], [2, 2, 0, 3, 0]]


# ---- iteration_control ---------------------------------------------------------------

def test_solve_is_deterministic_and_normalised():
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=12)
    opts = abi.default_opts(**o)
    p1, s1 = oracle.solve_layers(P, L, opts)
    p2, s2 = oracle.solve_layers(P, L, opts, nthreads=1)
    assert np.array_equal(p1, p2) and np.array_equal(s1, s2)
    assert np.all(s1["converged"] == 1)
    assert np.all(np.abs(p1.sum(axis=1) - 1.0) < 1e-10)
    assert (s1["iterations"] > 40).any(), "no layer exercised the Ng acceleration"


def test_iteration_cap_returns_best_eq_iterate():
    """iteration_control.h:128-135: at the cap the lowest-eq_error iterate is returned and
    is_found reflects the last step only; the plain retry then runs (radiative_transfer.cpp:258-276)."""
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=12)
    base, sb = oracle.solve_layers(P, L, abi.default_opts(**o))
    slow = int(np.argmax(sb["iterations"]))
    Ls = L.subset([slow])
    capped, sc = oracle.solve_layers(P, Ls, abi.default_opts(max_iter_acc=3, allow_plain_retry=0, **o))
    assert sc["converged"][0] == 0 and sc["iterations"][0] == 3
    assert sc["eq_error"][0] <= 1.0
    retry, sr = oracle.solve_layers(P, Ls, abi.default_opts(max_iter_acc=3, allow_plain_retry=1, **o))
    assert sr["used_plain_retry"][0] == 1 and sr["iterations"][0] > 3


def test_init_modes():
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=6)
    opts = abi.default_opts(**o)
    bl, _ = oracle.solve_layers(P, L, opts)
    warm, sw = oracle.solve_layers(P, L, abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o))
    assert np.array_equal(warm[0], bl[0])            # layer 0 has no predecessor
    given, sg = oracle.solve_layers(P, L, abi.default_opts(init=abi.LVG_INIT_GIVEN, **o), pops=bl)
    assert np.all(sg["iterations"] <= 3)            # restarting from the solution converges at once
    np.testing.assert_allclose(given, bl, rtol=1e-4)


def test_golden_fixtures_reproduce():
    """Regression fixtures (tests/golden, made by tests/golden/make_golden.py from this oracle)."""
    import os
    from tests.golden import make_golden
    path = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden_v1.npz")
    ref = np.load(path, allow_pickle=False)
    cur = make_golden.compute()
    assert set(ref.files) == set(cur)
    for k in ref.files:
        assert np.array_equal(ref[k], cur[k]), k
