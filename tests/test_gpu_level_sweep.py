"""GPU parity across level counts (tolerance: none — bit for bit against the oracle).

The kernel selected and its register tiling depend on N: the wave kernel's NM = 16..64
instantiations (one per 8 levels, lvg_wave.h), the 256-thread block kernel's panel paths
around its 64- and 128-column block boundaries, both the 256-thread instantiation (4 waves,
64-column blocks) and the 512-thread one (8 waves, 128-column blocks; lvg_kernels_wide.hip,
lvg_lu256.h), and the 768-thread instantiation for 256 < N <= 768 (lvg_kernels_big.hip). Each N here is solved on a few layers from the
boundary-layer start (radiative_transfer.cpp:236-288) with acceleration on, and the
boundary-layer solve (iteration_control.cpp:52-91) is compared on its own.
"""
import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from radiative_transfer_amd.native import LvgSolver
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu

WAVE_N = [20, 28, 40, 52, 60]                       # NM = 24, 32, 40, 56, 64
BLOCK_N = [65, 96, 128, 129, 192, 193, 240, 255]    # 64-row slot and 64/128-column block boundaries
BIG_N = [320, 385, 512, 640]                        # 768-thread kernel


def _run(name, nlev, nl, tuning="", kind=None, thin=False):
    P, L, o = synth.make_problem(name, nb_lay=nl, nb_lev=nlev)
    if thin:
        # lines with i - j <= 3 only, so that the wave kernel's LDS line-term buffer holds them
        i, j = np.indices(P.mol.einst.shape)
        P.mol.einst[np.abs(i - j) > 3] = 0.
    opts = abi.default_opts(**{**o, "accel_nb": 3, "accel_start": 3, "accel_period": 2})
    s = LvgSolver(P)
    if tuning:
        s.set_tuning(tuning)
    pg, sg = s.solve_layers(L, opts)
    if kind is not None:
        assert s.last_kernel_kind() == kind
    po, so = oracle.solve_layers(P, L, opts)
    assert_same(pg, sg, po, so)
    assert np.array_equal(s.boundary_layer_populations(L), oracle.boundary_layer_populations(P, L))
    s.close()


@pytest.mark.parametrize("nlev", WAVE_N)
def test_wave_level_counts(nlev):
    _run("ph2o45_1024", nlev, 8, "", 1, thin=nlev > 52)


# the overlap scheme (OH hyperfine pairs, 4-D table, single lines) across the NM classes 16-48,
# each case asserting the kernel that solves it against the oracle: up to 40 levels the wave
# kernel (every lane runs the single / near / far paths with clamped indices, lvg_wave.hip); at
# 48 levels the overlap line terms no longer fit the wave kernel's LDS (2 x lines > WYCAP, the
# host plan lvg_wave_plan rejects it) and the block kernel takes the solve, its 512-thread
# instantiation since 8 layers leave CUs to spare (lvg_last_kernel_kind 2)
WAVE_OV_N = [(12, 1), (22, 1), (32, 1), (40, 1), (48, 2)]   # NM = 16, 24, 32, 40, 48


@pytest.mark.parametrize("nlev,kind", WAVE_OV_N)
def test_wave_overlap_level_counts(nlev, kind):
    _run("oh24_overlap_2048", nlev, 8, "", kind)


@pytest.mark.parametrize("nlev", BLOCK_N)
@pytest.mark.parametrize("wide", [0, 2])
def test_block_level_counts(nlev, wide):
    _run("ch3oha256_4096", nlev, 4, f"wide={wide}", 2 if wide else 0)


@pytest.mark.parametrize("nlev", BIG_N)
def test_big_level_counts(nlev):
    _run("ch3oha256_4096", nlev, 2, kind=3)
