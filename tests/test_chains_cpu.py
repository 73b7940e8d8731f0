"""The oracle's batched warm chains (oracle_solve_chains) equal one warm-chain
oracle_solve_layers per cloud (radiative_transfer.cpp:219-289 run once per cloud) —
this pins the checker that tests/test_gpu_chains.py compares the HIP path against."""
import numpy as np

from radiative_transfer_amd import abi, synth
from oracle import oracle


def test_oracle_chains_equal_per_cloud_solves():
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=24)
    off = [0, 7, 7, 8, 16, 24]
    for kw in ({}, {"max_iter_acc": 3, "allow_plain_retry": 0}, {"max_iter_acc": 3, "max_iter_plain": 4}):
        opts = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **{**o, **kw})
        pc, sc = oracle.solve_chains(P, L, off, opts, nthreads=4)
        for a, b in zip(off[:-1], off[1:]):
            if a == b:
                continue
            pl, sl = oracle.solve_layers(P, L.subset(np.arange(a, b)), opts)
            assert np.array_equal(pc[a:b], pl)
            assert np.array_equal(sc[a:b], sl)
        if kw:
            assert (sc["converged"] == 0).any()
