"""C-ABI checks that need no GPU: the library loads, exports every entry point
include/lvg_amd.h declares, and rejects malformed descriptions with an error
code and message before touching a device (never exit(), unlike the reference's
loaders, e.g. lvg_method_functions.cpp:32-35)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from radiative_transfer_amd import abi, build, native, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    build.build()
    return native.load()


def header_functions():
    src = open(os.path.join(ROOT, "include", "lvg_amd.h")).read()
    return sorted(set(re.findall(r"^(?:int|void|const char \*)\s*(lvg_\w+)\(", src, re.M)))


def test_exports_every_declared_symbol(lib):
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(native.EXPORTS)


def test_abi_version_and_defaults(lib):
    assert lib.lvg_abi_version() == 1
    o = abi.c_solve_opts()
    lib.lvg_solve_opts_default(C.byref(o))
    # radiative_transfer.cpp:26-27, :45; iteration_control.h:71
    assert (o.min_error, o.max_iter_acc, o.max_iter_plain) == (1e-5, 150, 15000)
    assert (o.accel_start, o.accel_period, o.accel_nb, o.acceleration) == (40, 5, 5, 1)
    assert (o.allow_plain_retry, o.init, o.line_overlap) == (1, abi.LVG_INIT_BOUNDARY_LAYER, 0)


def _create(lib, prob):
    cp = prob.to_c()
    h = C.c_void_p()
    rc = lib.lvg_create(cp.ptr, 0, C.byref(h))
    msg = lib.lvg_last_error(None).decode()
    if rc == 0:
        lib.lvg_destroy(h)
    return rc, msg


def _mutate(**kw):
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    for k, v in kw.items():
        setattr(P.mol, k, v)
    return P


def test_rejects_malformed_problems(lib):
    P = _mutate(energy=np.arange(45, dtype=float)[::-1].copy())
    rc, msg = _create(lib, P)
    assert rc == -1 and "ascending" in msg
    P = _mutate(g=np.zeros(45, np.int32))
    rc, msg = _create(lib, P)
    assert rc == -1 and "g[" in msg
    # a radiative line between degenerate levels (intensity_calc divides by E^3)
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    P.mol.energy = P.mol.energy.copy()
    P.mol.energy[5] = P.mol.energy[4]
    P.mol.einst = P.mol.einst.copy()
    P.mol.einst[5, 4] = 1e-3
    rc, msg = _create(lib, P)
    assert rc == -1 and "non-positive energy" in msg
    # unsorted collision temperature grid
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    P.coll.neutral[0].tgrid = P.coll.neutral[0].tgrid[::-1].copy()
    rc, msg = _create(lib, P)
    assert rc == -1 and "tgrid" in msg
    # only one overlap table
    P, _, _ = synth.make_problem("oh24_overlap_2048", nb_lay=1)
    P.overlap2 = None
    rc, msg = _create(lib, P)
    assert rc == -1 and "overlap" in msg
    # more levels than this build's largest kernel (768, the reference's CH3OH count)
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    N = 769
    P.mol.energy = np.arange(N, dtype=float)
    P.mol.g = np.ones(N, np.int32)
    P.mol.einst = np.zeros((N, N))
    P.mol.v = np.zeros(N, np.int32)
    P.mol.j = np.zeros(N)
    rc, msg = _create(lib, P)
    assert rc == -4 and "exceeds" in msg


def test_valid_problem_without_device_fails_cleanly(lib):
    """On a host with no GPU the library reports a device error (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    rc, msg = _create(lib, P)
    assert rc == -2 and msg
    with pytest.raises(native.LvgError):
        native.LvgSolver(P)


def test_partition_rules_match_dist(lib):
    """lvg_shard_range / lvg_chain_shard (the multi-device handle's split, no device) are
    dist.shard_range / dist.chain_shard, the rules of the one-process-per-GPU path."""
    from radiative_transfer_amd import dist
    lo, hi = C.c_int(), C.c_int()
    for n in (0, 1, 7, 512, 4096, 4097, 16384):
        for g in (1, 2, 3, 4, 8):
            for r in range(g):
                assert lib.lvg_shard_range(n, g, r, C.byref(lo), C.byref(hi)) == 0
                assert (lo.value, hi.value) == dist.shard_range(n, g, r)
    assert lib.lvg_shard_range(4, 0, 0, C.byref(lo), C.byref(hi)) == -1
    assert lib.lvg_shard_range(4, 2, 2, C.byref(lo), C.byref(hi)) == -1
    rng = np.random.default_rng(6)
    for trial in range(40):
        lens = rng.integers(0, 9, size=int(rng.integers(1, 30)))
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        for g in (1, 2, 3, 8):
            for r in range(g):
                assert lib.lvg_chain_shard(len(off) - 1, off.ctypes.data_as(C.POINTER(C.c_int)), g, r,
                                           C.byref(lo), C.byref(hi)) == 0
                assert (lo.value, hi.value) == dist.chain_shard(off, g, r), (off, g, r)


def test_multi_device_create_rejects_without_touching_a_device(lib):
    P, _, _ = synth.make_problem("ph2o45_1024", nb_lay=1)
    cp = P.to_c()
    h = C.c_void_p()
    assert lib.lvg_create_multi(cp.ptr, 0, C.byref(h)) == -1
    assert "empty" in lib.lvg_last_error(None).decode() and not h.value
    assert lib.lvg_create_devices(cp.ptr, 0, None, C.byref(h)) == -1
    assert lib.lvg_nb_devices(None) == 0


def test_rejects_null_table_arrays(lib):
    """NULL arrays fail with LVG_E_ARG in validation (they used to reach memcmp / hipMemcpy)."""
    P, _, _ = synth.make_problem("oh24_overlap_2048", nb_lay=1)
    cp = P.to_c()
    cp.ov[1].gratio = None
    h = C.c_void_p()
    assert lib.lvg_create(cp.ptr, 0, C.byref(h)) == -1
    assert "overlap table arrays missing" in lib.lvg_last_error(None).decode()
