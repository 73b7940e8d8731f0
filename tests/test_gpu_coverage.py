"""GPU parity beyond the BASELINE cases of test_gpu_parity.py (tolerance: none).

- The option paths of the N > 64 block kernel: iteration caps with
  the best-iterate substitution (q3, iteration_control.h:128-135), the plain retry
  (radiative_transfer.cpp:258-276), Ng acceleration actually running at N = 256
  (accel_step, iteration_control.h:139-193, whose sums share the panel LDS union), and
  the init modes — on CH3OH-A (N = 256) and on p-H2O forced onto the block kernel.
- The reference's own level counts and the kernel instantiations they select (item 6,
  ADVICE): N = 12 / 64 (wave kernel NM = 16 / 64), OH-HF N = 56 (radiative_transfer.cpp
  :419, wave NM = 56), H2O N = 150 (:901), CH3OH N = 160 (block kernel, 129..255 rows);
  N = 33 for the NM = 40 instantiation (OH-HF 24 and p-H2O 45 cover NM = 24 and 48).
- The OH (non-HF) rule, q10 (coll_rates_oh.cpp:334-347), and the GENERIC base-class
  rule (coll_rates.cpp:181-217, q5 first electron set) (item 8).
- The three |dx| regions of the overlap scheme (iteration_lvg.cpp:461-500): pure
  4-D table, the 3.5 < |dx| < 4 blend, single-line beyond 4 (item 8).
- NaN inputs: the pivot rule follows oracle_lu_solve for NaN.
- An asynchronous device-entry solve on a caller stream followed at once by a host
  entry call on the same handle (the handle orders them).
"""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgError, LvgSolver
from oracle import oracle
from parity_helpers import assert_same, overlap_dx

pytestmark = pytest.mark.gpu

# The block kernel comes in two instantiations for N <= 256 (lvg_kernels.hip): the
# 256-thread one (kind 0, launches that fill the chip) and the 512-thread one (kind 2,
# picked automatically for launches of at most two layers per CU — every small test
# here). `wide=0` / `wide=2` pin each one; the tests assert the kind that ran.
BLOCK_KINDS = [pytest.param(0, id="bt256"), pytest.param(2, id="bt512")]


def _block_tuning(kind, *extra):
    return ",".join(("block_kernel=1", f"wide={kind}") + extra)


def _cmp(s, P, L, opts, pops=None, equal_nan=False):
    pg, sg = s.solve_layers(L, opts, pops=pops)
    po, so = oracle.solve_layers(P, L, opts, pops=pops)
    assert_same(pg, sg, po, so, equal_nan=equal_nan)
    return po, so


@pytest.mark.parametrize("kind", BLOCK_KINDS)
@pytest.mark.parametrize("name,nl", [("ch3oha256_4096", 6), ("ph2o45_1024", 12)])
def test_block_kernel_option_paths(name, nl, kind):
    P, L, o = synth.make_problem(name, nb_lay=nl)
    s = LvgSolver(P)
    s.set_tuning(_block_tuning(kind))
    variants = [{"accel_start": 2, "accel_nb": 2, "accel_period": 1},                 # Ng from iteration 2
                {"accel_start": 3, "accel_nb": 3, "accel_period": 2, "max_iter_acc": 9},
                {"max_iter_acc": 2, "allow_plain_retry": 0},                          # cap -> best iterate
                {"max_iter_acc": 2, "allow_plain_retry": 1, "max_iter_plain": 3},      # forced plain retry
                {"acceleration": 0, "max_iter_plain": 2}]
    ran_accel = False
    for kw in variants:
        opts = abi.default_opts(**{**o, **kw})
        po, so = _cmp(s, P, L, opts)
        assert s.last_kernel_kind() == kind
        if opts.acceleration and (so["iterations"] > opts.accel_start).any():
            ran_accel = True
    assert ran_accel, "no layer reached the Ng step"
    # init modes
    base = abi.default_opts(**o)
    p0, _ = oracle.solve_layers(P, L, base)
    guess = 0.5 * p0 + 0.5 / P.mol.nb_lev
    _cmp(s, P, L, abi.default_opts(init=abi.LVG_INIT_GIVEN, **o), pops=guess)
    assert s.last_kernel_kind() == kind
    _cmp(s, P, L, abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o))
    assert s.last_kernel_kind() == kind
    s.close()


@pytest.mark.parametrize("name,nlev", [("ph2o45_1024", 12), ("ph2o45_1024", 33), ("ph2o45_1024", 64),
                                       ("oh24_overlap_2048", 56), ("ph2o45_1024", 150), ("ch3oha256_4096", 160)])
def test_reference_level_counts(name, nlev):
    P, L, o = synth.make_problem(name, nb_lay=8, nb_lev=nlev)
    s = LvgSolver(P)
    _cmp(s, P, L, abi.default_opts(**o))
    if o.get("line_overlap"):
        _cmp(s, P, L, abi.default_opts(**{**o, "line_overlap": 0}))
    bo = oracle.boundary_layer_populations(P, L)
    assert np.array_equal(s.boundary_layer_populations(L), bo)
    Mg, dfg, pg, eg = s.debug_calc_new_pop(L, 3, bo[3], o.get("line_overlap", 0))
    Mo, dfo, po, eo = oracle.calc_new_pop(P, L, 3, bo[3], o.get("line_overlap", 0))
    assert np.array_equal(Mg, Mo) and np.array_equal(dfg, dfo) and np.array_equal(pg, po) and eg == eo
    s.close()


def _oh_nonhf_problem():
    P, L, o = synth.make_problem("oh24_overlap_2048", nb_lay=8)
    rng = np.random.default_rng(33)
    E = P.mol.energy
    grid = np.concatenate([[0.0], np.linspace(10, 300, 10)])
    # He table over all levels (q10 reads it without a level bound); the H2 tables shorter,
    # so their bound check (coll_rates_oh.cpp:340) cuts pairs with up >= 16
    P.coll = abi.Collisions(rule=abi.LVG_COLL_OH, neutral=[synth._coll_table(rng, E, grid),
                                                         synth._coll_table(rng, E, grid, nb_lev=16),
                                                         synth._coll_table(rng, E, grid, nb_lev=16)])
    o.pop("line_overlap", None)
    return P, L, o


def _generic_problem():
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=8)
    rng = np.random.default_rng(34)
    E = P.mol.energy
    g1 = np.concatenate([[0.0], np.linspace(20, 1000, 9)])
    he = synth._coll_table(rng, E, g1)
    ph2 = synth._coll_table(rng, E, g1, nb_lev=30)
    h = synth._coll_table(rng, E, g1, nb_lev=20)
    e1 = synth._coll_table(rng, E, g1, nb_lev=20, scale=1e4)
    e2 = synth._coll_table(rng, E, g1, scale=1e4)
    he.species, ph2.species, h.species = abi.LVG_SP_HE, abi.LVG_SP_PH2, abi.LVG_SP_H
    e1.species = e2.species = abi.LVG_SP_E
    P.coll = abi.Collisions(rule=abi.LVG_COLL_GENERIC, neutral=[he, ph2, h], electron=[e1, e2])
    return P, L, o


@pytest.mark.parametrize("kind", BLOCK_KINDS)
def test_pipelined_collision_build_with_electrons(kind):
    """The block kernels' pipelined collision build (build_collision_pipe: no boundary matrix
    written, at most three neutral terms) with its electron slot: the GENERIC rule's electron
    tables (coll_rates.cpp:181-217) on layers started from given populations and on warm
    chains, where no boundary matrix is built. Bit-exact against the oracle."""
    P, L, o = _generic_problem()
    s = LvgSolver(P)
    s.set_tuning(_block_tuning(kind))
    p0, _ = oracle.solve_layers(P, L, abi.default_opts(**o))
    guess = 0.5 * p0 + 0.5 / P.mol.nb_lev
    _cmp(s, P, L, abi.default_opts(init=abi.LVG_INIT_GIVEN, **o), pops=guess)
    assert s.last_kernel_kind() == kind
    _cmp(s, P, L, abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o))
    assert s.last_kernel_kind() == kind
    off = np.array([0, 3, 8], dtype=np.int32)
    wopts = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    pg, sg = s.solve_chains(L, off, wopts)
    po, so = oracle.solve_chains(P, L, off, wopts)
    assert_same(pg, sg, po, so)
    assert s.last_kernel_kind() == kind
    s.close()


@pytest.mark.parametrize("make", [_oh_nonhf_problem, _generic_problem], ids=["oh_nonhf_q10", "generic_q5"])
@pytest.mark.parametrize("kind", [pytest.param(1, id="wave")] + BLOCK_KINDS)
def test_collision_rules(make, kind):
    P, L, o = make()
    s = LvgSolver(P)
    s.set_tuning("" if kind == 1 else _block_tuning(kind))
    _cmp(s, P, L, abi.default_opts(**o))
    assert s.last_kernel_kind() == kind
    bo = oracle.boundary_layer_populations(P, L)
    Mg, dfg, pg, eg = s.debug_calc_new_pop(L, 0, bo[0], 0)
    Mo, dfo, po, eo = oracle.calc_new_pop(P, L, 0, bo[0], 0)
    assert np.array_equal(Mg, Mo) and np.array_equal(pg, po)
    # the rule matters: the rates differ from a 3-table OH-HF / base reading of the same tables
    for lay in (0, 5):
        d, u, de, ue = oracle.coll_rates(P, L, lay)
        assert np.count_nonzero(d) > 0
    s.close()


def test_overlap_dx_regions():
    """Each |dx| branch of intensity_calc(u1, l1, u2, l2) is taken, and the GPU matches the
    oracle on the layers where it is."""
    P, L, o = synth.make_problem("oh24_overlap_2048")
    pairs, dx = overlap_dx(P, L)
    regions = {"table": dx < 3.5, "blend": (dx > 3.5) & (dx < 4.0), "single": dx > 4.0}
    pick = []
    for name, m in regions.items():
        lay = np.nonzero(m.any(axis=1))[0]
        assert lay.size > 0, f"no layer takes the {name} branch"
        pick += list(lay[:6])
    idx = np.unique(pick)
    sub = L.subset(idx)
    _, dsub = overlap_dx(P, sub)
    assert ((dsub > 3.5) & (dsub < 4.0)).sum() >= 6
    s = LvgSolver(P)
    _cmp(s, P, sub, abi.default_opts(**o))
    s.close()


def _swap_grid_entries(P, field, i):
    """Entries i and i+1 of one overlap grid swapped, identically in both tables (the
    device keeps one copy of the grids): a non-monotone grid."""
    for t in (P.overlap1, P.overlap2):
        g = np.array(getattr(t, field), dtype=np.float64, copy=True)
        g[i], g[i + 1] = g[i + 1], g[i]
        setattr(t, field, g)


@pytest.mark.parametrize("field", ["gamma", "gratio"])
def test_overlap_nonmonotone_grid(field):
    """the wave kernel's grid-interval hints fall back to plain bisection when its
    LDS grid copies are not non-decreasing (lvg_wave.hip, the per-block check). A gamma or
    gamma-ratio grid with two entries swapped takes that branch; the result is still the
    oracle's locate_index on the same grid, bit for bit."""
    P, L, o = synth.make_problem("oh24_overlap_2048", nb_lay=24)
    g = getattr(P.overlap1, field)
    _swap_grid_entries(P, field, len(g) // 2)
    assert (np.diff(getattr(P.overlap1, field)) < 0).any()
    s = LvgSolver(P)
    _cmp(s, P, L, abi.default_opts(**o))
    assert s.last_kernel_kind() == 1
    s.close()


def test_overlap_tables_must_share_grid_values():
    """The device keeps overlap1's grids for both tables, so lvg_create rejects a second
    table whose grids differ in value (not only in size)."""
    P, L, o = synth.make_problem("oh24_overlap_2048", nb_lay=2)
    g = np.array(P.overlap2.gamma, dtype=np.float64, copy=True)
    g[-1] *= 1.5
    P.overlap2.gamma = g
    with pytest.raises(LvgError, match="share grids"):
        LvgSolver(P)


@pytest.mark.parametrize("name", ["ph2o45_1024", "ch3oha256_4096"])
def test_nan_inputs_follow_oracle(name):
    """NaN in a layer (molecule concentration -> NaN line terms, velocity gradient) gives
    the oracle's result, NaN for NaN, including its pivot choices."""
    P, L, o = synth.make_problem(name, nb_lay=4)
    L.mol_conc[1] = np.nan
    L.vel_grad[2] = np.nan
    s = LvgSolver(P)
    _cmp(s, P, L, abi.default_opts(**{**o, "max_iter_acc": 6, "max_iter_plain": 6}), equal_nan=True)
    s.close()


def test_async_device_solve_then_host_entry_on_same_handle():
    import torch
    P, L, o = synth.make_problem("ch3oha256_4096", nb_lay=64)
    opts = abi.default_opts(**o)
    s = LvgSolver(P)
    dev = torch.device("cuda", 0)
    A, B = L.subset(np.arange(0, 48)), L.subset(np.arange(48, 64))
    soa = torch.from_numpy(A.soa()).to(dev)
    pops = torch.zeros((A.nb_lay, P.mol.nb_lev), dtype=torch.float64, device=dev)
    st = torch.zeros((A.nb_lay, abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    side = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    s.solve_layers_device(A.nb_lay, soa.data_ptr(), pops.data_ptr(), st.data_ptr(), opts,
                          stream_ptr=side.cuda_stream)
    pb, sb = s.solve_layers(B, opts)            # the handle's own stream, right away
    torch.cuda.synchronize()
    pa = pops.cpu().numpy()
    sa = np.frombuffer(st.cpu().numpy().tobytes(), dtype=abi.STATUS_DTYPE)
    poa, soa_ = oracle.solve_layers(P, A, opts)
    pob, sob = oracle.solve_layers(P, B, opts)
    assert_same(pa, sa, poa, soa_)
    assert_same(pb, sb, pob, sob)
    s.close()


@pytest.mark.parametrize("kind", BLOCK_KINDS)
@pytest.mark.parametrize("make", [lambda: synth.make_problem("ch3oha256_4096", nb_lay=12), _generic_problem],
                         ids=["ch3oha256", "generic_electrons"])
def test_collision_build_paths(make, kind):
    """Independent layers on the block kernel with the collision operators built in the
    solve kernel (the default), built ahead by coll_kernel (B formed from K without
    electron tables, B stored with them), and with coll_kernel asked for but over its
    memory budget (the fallback to the in-kernel build): all bit-exact against the
    oracle (coll_rates.cpp:152-174 per layer, iteration_lvg.cpp:118-131)."""
    P, L, o = make()
    s = LvgSolver(P)
    opts = abi.default_opts(**o)
    po, so = oracle.solve_layers(P, L, opts)
    for extra, ahead in (((), False), (("coll_ahead=1",), True), (("coll_ahead=1", "coll_order=0"), True),
                         (("coll_ahead=1", "coll_mem=0"), False)):
        spec = _block_tuning(kind, *extra)
        s.set_tuning("")                         # set_tuning merges: start from the defaults
        s.set_tuning(spec)
        pg, sg = s.solve_layers(L, opts)
        assert_same(pg, sg, po, so)
        assert (s.last_coll_time() > 0) == ahead, spec
        assert s.last_kernel_kind() == kind, spec
    with pytest.raises(Exception):
        s.set_tuning("no_such_key=1")
    s.close()
