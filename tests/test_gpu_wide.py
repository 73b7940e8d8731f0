"""The 512-thread block kernel (lvg_kernels_wide.hip) for underfilled launches — tolerance:
none, bit for bit against the oracle and against the 256-thread kernel.

The per-GPU share of a strongly scaled cloud (radiative_transfer.cpp:236-256, 4096 layers
over 8 GPUs = 512) and warm chains with at most one cloud per CU leave CUs to spare; the
ABI then runs each N <= 256 layer on eight waves (128-column LU blocks, lvg_lu256.h).
Covered: the automatic choice and its limits (two layers per CU; one chain per CU), the
forced and disabled settings, acceleration and plain-retry paths, and warm chains.
"""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgSolver
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ch3():
    P, L, o = synth.make_problem("ch3oha256_4096")
    return P, L, o


def test_wide_auto_choice_and_exactness(ch3):
    P, L, o = ch3
    opts = abi.default_opts(**o)
    sub = L.subset(np.arange(0, 4096, 64))                 # 64 layers: underfilled
    s = LvgSolver(P)
    pg, sg = s.solve_layers(sub, opts)
    assert s.last_kernel_kind() == 2
    po, so = oracle.solve_layers(P, sub, opts)
    assert_same(pg, sg, po, so)
    s.set_tuning("wide=0")
    p0, s0 = s.solve_layers(sub, opts)
    assert s.last_kernel_kind() == 0
    assert_same(p0, s0, po, so)
    s.close()


def test_wide_threshold(ch3):
    """Automatic: at most 2 layers per CU; above that the 256-thread kernel."""
    P, L, o = ch3
    opts = abi.default_opts(**o)
    s = LvgSolver(P)
    s.solve_layers(L.subset(np.arange(512)), opts)
    assert s.last_kernel_kind() == 2                        # <= 2 per CU on a 256-CU MI355X
    s.solve_layers(L.subset(np.arange(2048)), opts)
    assert s.last_kernel_kind() == 0
    s.close()


def test_wide_forced_accel_and_retry(ch3):
    P, L, o = ch3
    opts = abi.default_opts(**{**o, "accel_nb": 3, "accel_start": 3, "accel_period": 2,
                                "allow_plain_retry": 1, "max_iter_acc": 6})
    sub = L.subset(np.arange(7, 4096, 331))
    s = LvgSolver(P)
    s.set_tuning("wide=2")
    pg, sg = s.solve_layers(sub, opts)
    assert s.last_kernel_kind() == 2
    po, so = oracle.solve_layers(P, sub, opts)
    assert_same(pg, sg, po, so)
    assert sg["used_plain_retry"].any()                     # the plain retry ran (1 of 13)
    s.close()


def test_wide_chains(ch3):
    P, L, o = ch3
    opts = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    sub = L.subset(np.arange(0, 96))
    off = np.array([0, 10, 11, 40, 40, 96], dtype=np.int32)    # ragged, one empty chain
    s = LvgSolver(P)
    pg, sg = s.solve_chains(sub, off, opts)
    assert s.last_kernel_kind() == 2
    po, so = oracle.solve_chains(P, sub, off, opts)
    assert_same(pg, sg, po, so)
    s.close()
