"""The multi-GPU path (radiative_transfer_amd/dist.py) on CPU with gloo, world
size 2: contiguous layer shards, the status all-reduce and the population
all_gather reproduce the single-process solve bit for bit. The per-rank solver
here is the CPU oracle (test infrastructure); on MI355X it is LvgSolver."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from radiative_transfer_amd import abi, dist, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, nl, out):
    import torch.distributed as td
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    pops, st, totals = dist.solve_sharded(L, lambda sub: oracle.solve_layers(P, sub, opts, nthreads=1),
                                          P.mol.nb_lev, gather=True)
    # bench.py's per-step reduction of a device-layout status tensor (here on the CPU)
    import torch
    lo, hi = dist.shard_range(nl, world, rank)
    raw = np.frombuffer(st[lo:hi].tobytes(), dtype=np.float64).reshape(hi - lo, abi.STATUS_DTYPE.itemsize // 8)
    dev_tot = dist.reduce_status_device(torch.from_numpy(raw.copy())).numpy()
    if rank == 0:
        np.savez(out, pops=pops, iters=st["iterations"], conv=st["converged"],
                 totals=np.array([totals[0], totals[1]]), relmax=np.array([totals[2]]), dev_tot=dev_tot)
    td.barrier()
    td.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 4096):
        for w in (1, 2, 3, 8):
            spans = [dist.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


# nl=1 < world: rank 1's block is empty (it must neither crash nor hang the all_gather)
@pytest.mark.parametrize("name,nl", [("ph2o45_1024", 10), ("oh24_overlap_2048", 6), ("ph2o45_1024", 1)])
def test_gloo_world2_matches_single_process(tmp_path, name, nl):
    from oracle import oracle
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), name, nl, out), nprocs=2, join=True)
    got = np.load(out)
    P, L, o = synth.make_problem(name, nb_lay=nl)
    ref, st = oracle.solve_layers(P, L, abi.default_opts(**o))
    assert np.array_equal(got["pops"], ref)
    assert np.array_equal(got["iters"], st["iterations"])
    assert got["totals"][0] == st["iterations"].sum()
    assert got["totals"][1] == (st["converged"] == 0).sum()
    assert got["relmax"][0] == st["rel_error"].max()
    assert np.array_equal(got["dev_tot"], [st["iterations"].sum(), (st["converged"] == 0).sum(), st["rel_error"].max()])
