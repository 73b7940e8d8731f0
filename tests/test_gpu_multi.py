"""Several GPUs behind ONE handle (lvg_create_multi / lvg_create_devices; SURVEY 8b's
device_mask): the batch is split into contiguous layer blocks (whole clouds for chains), one
host thread and stream per device, no exchange. On the one-GPU box the split runs as several
handles on device 0 (lvg_create_devices([0, 0, 0])), which exercises the partition, the
threads and the per-device streams; a mask naming an absent device fails cleanly. Bit-exact
against the oracle and against the single-device handle (radiative_transfer.cpp:236-256 is
the serial layer loop the split replaces)."""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgError, LvgSolver
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,nl", [("ph2o45_1024", 50), ("ch3oha256_4096", 10), ("oh24_overlap_2048", 7)])
def test_mask_one_equals_single_handle(name, nl):
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    one = LvgSolver(P)
    multi = LvgSolver(P, device_mask=0b1)
    assert multi.nb_devices() == 1
    p1, s1 = one.solve_layers(L, opts)
    pm, sm = multi.solve_layers(L, opts)
    assert np.array_equal(p1, pm) and np.array_equal(s1, sm)
    po, so = oracle.solve_layers(P, L, opts)
    assert_same(pm, sm, po, so)
    one.close(); multi.close()


@pytest.mark.parametrize("name,nl,devs", [("ph2o45_1024", 50, [0, 0, 0]), ("ch3oha256_4096", 10, [0, 0]),
                                          ("ch3oha256_4096", 1, [0, 0, 0]), ("oh24_overlap_2048", 7, [0, 0])])
def test_split_over_handles_bit_exact(name, nl, devs):
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    s = LvgSolver(P, devices=devs)
    assert s.nb_devices() == len(devs)
    pg, sg = s.solve_layers(L, opts)
    po, so = oracle.solve_layers(P, L, opts)
    assert_same(pg, sg, po, so)
    ms, n = s.last_kernel_time()
    assert ms > 0 and 1 <= n <= len(devs)
    # init = given, split the same way
    og = abi.default_opts(init=abi.LVG_INIT_GIVEN, **o)
    guess = 0.5 * po + 0.5 / P.mol.nb_lev
    pg, sg = s.solve_layers(L, og, pops=guess)
    po2, so2 = oracle.solve_layers(P, L, og, pops=guess)
    assert_same(pg, sg, po2, so2)
    # boundary_layer_populations, split
    assert np.array_equal(s.boundary_layer_populations(L), oracle.boundary_layer_populations(P, L))
    s.close()


def test_chains_split_and_whole_cloud_chain():
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=40)
    off = np.array([0, 7, 7, 15, 16, 31, 40], dtype=np.int32)     # ragged, one empty cloud
    ow = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    s = LvgSolver(P, devices=[0, 0, 0])
    pg, sg = s.solve_chains(L, off, ow)
    po, so = oracle.solve_chains(P, L, off, ow)
    assert_same(pg, sg, po, so)
    # one chain over the whole cloud: sequential, first device
    pg, sg = s.solve_layers(L, ow)
    po, so = oracle.solve_layers(P, L, ow)
    assert_same(pg, sg, po, so)
    s.close()


def test_absent_device_fails_cleanly():
    import torch
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    n = torch.cuda.device_count()
    with pytest.raises(LvgError):
        LvgSolver(P, device_mask=1 << n)
    with pytest.raises(LvgError):
        LvgSolver(P, devices=[0, n])
