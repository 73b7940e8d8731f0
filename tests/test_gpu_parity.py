"""GPU parity: the HIP path through the C ABI against the CPU oracle on the same
synth_v1 inputs. Tolerance: NONE — the kernels are built to reproduce the
oracle's floating-point operation sequence (DESIGN.md "Parity"), so populations,
iteration counts and every status field must be bitwise identical. Full-size
BASELINE configurations are checked through size-independent properties plus
bit-exact subsets."""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgError, LvgSolver
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu

_solvers = {}


def solver_for(name, nb_lay=None, nb_lev=None):
    key = (name, nb_lev)
    P, L, o = synth.make_problem(name, nb_lay=nb_lay, nb_lev=nb_lev)
    if key not in _solvers:
        _solvers[key] = LvgSolver(P)
    return _solvers[key], P, L, o


CASES = [("oh24_single", 1, None), ("ph2o45_1024", 48, None), ("oh24_overlap_2048", 24, None),
         ("ch3oha256_4096", 6, None), ("ch3ohe256_sweep", 6, None), ("ch3oha256_4096", 24, 100)]


@pytest.mark.parametrize("name,nl,nlev", CASES)
def test_solve_bit_exact(name, nl, nlev):
    s, P, L, o = solver_for(name, nl, nlev)
    opts = abi.default_opts(**o)
    pg, sg = s.solve_layers(L, opts)
    po, so = oracle.solve_layers(P, L, opts)
    assert_same(pg, sg, po, so)


@pytest.mark.parametrize("name,nl,nlev", CASES)
def test_calc_new_pop_and_boundary_bit_exact(name, nl, nlev):
    """calc_new_pop (iteration_lvg.cpp:87-161): assembled matrix, residual, new pops."""
    s, P, L, o = solver_for(name, nl, nlev)
    ov = o.get("line_overlap", 0)
    bg = s.boundary_layer_populations(L)
    bo = oracle.boundary_layer_populations(P, L)
    assert np.array_equal(bg, bo)
    for lay in sorted({0, L.nb_lay - 1}):
        Mg, dfg, pg, eg = s.debug_calc_new_pop(L, lay, bo[lay], ov)
        Mo, dfo, po, eo = oracle.calc_new_pop(P, L, lay, bo[lay], ov)
        assert np.array_equal(Mg, Mo)
        assert np.array_equal(dfg, dfo)
        assert np.array_equal(pg, po)
        assert eg == eo


def test_init_given_and_warm_chain():
    s, P, L, o = solver_for("ph2o45_1024", 16)
    base = abi.default_opts(**o)
    p0, _ = oracle.solve_layers(P, L, base)
    guess = 0.5 * p0 + 0.5 / P.mol.nb_lev
    og = abi.default_opts(init=abi.LVG_INIT_GIVEN, **o)
    pg, sg = s.solve_layers(L, og, pops=guess)
    po, so = oracle.solve_layers(P, L, og, pops=guess)
    assert_same(pg, sg, po, so)
    ow = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    pg, sg = s.solve_layers(L, ow)
    po, so = oracle.solve_layers(P, L, ow)
    assert_same(pg, sg, po, so)


def test_iteration_cap_best_iterate_and_plain_retry():
    """iteration_control.h:128-135 (cap -> best eq_error iterate) and the plain retry
    of radiative_transfer.cpp:258-276, forced with small caps."""
    s, P, L, o = solver_for("ph2o45_1024", 16)
    for kw in ({"max_iter_acc": 44, "allow_plain_retry": 0},
               {"max_iter_acc": 44, "allow_plain_retry": 1, "max_iter_plain": 30},
               {"acceleration": 0, "max_iter_plain": 7},
               {"accel_start": 6, "accel_period": 3, "accel_nb": 4}):
        opts = abi.default_opts(**{**o, **kw})
        pg, sg = s.solve_layers(L, opts)
        po, so = oracle.solve_layers(P, L, opts)
        assert_same(pg, sg, po, so)
    assert (so["converged"] == 1).any()


def test_device_resident_entry_matches_host_entry():
    import torch
    s, P, L, o = solver_for("ph2o45_1024", 32)
    opts = abi.default_opts(**o)
    ph, sh = s.solve_layers(L, opts)
    dev = torch.device("cuda", 0)
    soa = torch.from_numpy(L.soa()).to(dev)
    pops = torch.zeros((L.nb_lay, P.mol.nb_lev), dtype=torch.float64, device=dev)
    st = torch.zeros((L.nb_lay, abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    s.solve_layers_device(L.nb_lay, soa.data_ptr(), pops.data_ptr(), st.data_ptr(), opts,
                          stream_ptr=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(pops.cpu().numpy(), ph)
    sd = np.frombuffer(st.cpu().numpy().tobytes(), dtype=abi.STATUS_DTYPE)
    assert np.array_equal(sd, sh)
    ms, n = s.last_kernel_time()
    assert ms > 0 and n == 1


def test_empty_and_error_paths():
    s, P, L, o = solver_for("ph2o45_1024", 4)
    pg, sg = s.solve_layers(L.subset(np.arange(0)), abi.default_opts(**o))
    assert pg.shape == (0, P.mol.nb_lev)
    with pytest.raises(LvgError):
        s.solve_layers(L, abi.default_opts(line_overlap=1, **o))   # no overlap tables in this problem
    with pytest.raises(LvgError):
        s.solve_layers(L, abi.default_opts(accel_nb=1, **o))


# ---- full BASELINE sizes ---------------------------------------------------------------

@pytest.mark.parametrize("name", ["ph2o45_1024", "oh24_overlap_2048", "ch3oha256_4096", "ch3ohe256_sweep"])
def test_full_size(name):
    """The four BASELINE configurations at full size (1024 / 2048 / 4096 layers, 16,384
    sweep cells): every layer converges, populations are normalised and non-negative,
    results are identical run to run, and EVERY layer is bit-exact against the oracle
    (the oracle runs on the box's OpenMP threads: 4096 CH3OH-A layers in ~2 s on 16,
    the 16,384 CH3OH-E cells in ~8 s)."""
    s, P, L, o = solver_for(name)
    opts = abi.default_opts(**o)
    p1, s1 = s.solve_layers(L, opts)
    p2, s2 = s.solve_layers(L, opts)
    assert np.array_equal(p1, p2) and np.array_equal(s1, s2)
    assert np.all(s1["converged"] == 1)
    assert np.all(np.abs(p1.sum(axis=1) - 1.0) < 1e-9)
    assert p1.min() > -1e-12
    po, so = oracle.solve_layers(P, L, opts)
    assert_same(p1, s1, po, so)
