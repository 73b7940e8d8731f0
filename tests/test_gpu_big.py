"""GPU parity above 256 levels: the 768-thread instantiation of the
block kernel (lvg_kernels_big.hip) that lvg_create selects for 256 < N <= 768 — the
reference's CH3OH callers use nb_lev_ch3oh = 768 (radiative_transfer.cpp:647, :773).
Tolerance: none, as everywhere (same operation order as the oracle).

Covers N = 768 (the reference's count, 24 full 32-column blocks), N = 300 (a ragged
last block column, odd rows of the panel's last wave) and N = 257 (one row past the
256-thread kernel), with the iteration-cap / plain-retry / Ng option paths, the init
modes, warm chains, the calc_new_pop probe and boundary-layer populations.
"""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgSolver
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu


def _cmp(s, P, L, opts, pops=None):
    pg, sg = s.solve_layers(L, opts, pops=pops)
    po, so = oracle.solve_layers(P, L, opts, pops=pops)
    assert_same(pg, sg, po, so)
    return po, so


@pytest.mark.parametrize("nlev,nl", [(768, 4), (300, 6), (257, 3)])
def test_big_n_bit_exact(nlev, nl):
    P, L, o = synth.make_problem("ch3oha256_4096", nb_lay=nl, nb_lev=nlev)
    s = LvgSolver(P)
    po, so = _cmp(s, P, L, abi.default_opts(**o))
    assert np.all(so["converged"] == 1)
    bo = oracle.boundary_layer_populations(P, L)
    assert np.array_equal(s.boundary_layer_populations(L), bo)
    Mg, dfg, pg, eg = s.debug_calc_new_pop(L, nl - 1, bo[nl - 1])
    Mo, dfo, pe, eo = oracle.calc_new_pop(P, L, nl - 1, bo[nl - 1])
    assert np.array_equal(Mg, Mo) and np.array_equal(dfg, dfo) and np.array_equal(pg, pe) and eg == eo
    s.close()


def test_big_n_option_paths_and_init_modes():
    P, L, o = synth.make_problem("ch3oha256_4096", nb_lay=4, nb_lev=768)
    s = LvgSolver(P)
    ran_accel = False
    for kw in ({"accel_start": 2, "accel_nb": 2, "accel_period": 1},
               {"max_iter_acc": 2, "allow_plain_retry": 1, "max_iter_plain": 3},
               {"acceleration": 0, "max_iter_plain": 2}):
        opts = abi.default_opts(**{**o, **kw})
        _, so = _cmp(s, P, L, opts)
        ran_accel |= bool(opts.acceleration and (so["iterations"] > opts.accel_start).any())
    assert ran_accel
    p0, _ = oracle.solve_layers(P, L, abi.default_opts(**o))
    guess = 0.5 * p0 + 0.5 / P.mol.nb_lev
    _cmp(s, P, L, abi.default_opts(init=abi.LVG_INIT_GIVEN, **o), pops=guess)
    ow = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    _cmp(s, P, L, ow)
    pg, sg = s.solve_chains(L, [0, 1, 4], ow)
    pc, sc = oracle.solve_chains(P, L, [0, 1, 4], ow)
    assert_same(pg, sg, pc, sc)
    s.close()
