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


def test_chain_shard_whole_clouds_balanced():
    off = np.array([0, 5, 5, 9, 30, 31, 40, 64])
    for w in (1, 2, 3, 4, 8):
        spans = [dist.chain_shard(off, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == len(off) - 1
        assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def _chain_worker(rank, world, port, out):
    import torch.distributed as td
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=20)
    opts = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    off = [0, 3, 9, 9, 14, 20]
    pops, st, (lo, hi), totals = dist.solve_chains_sharded(
        L, off, lambda sub, loff: oracle.solve_chains(P, sub, loff, opts, nthreads=1), P.mol.nb_lev)
    np.savez(out + f".{rank}.npz", pops=pops, iters=st["iterations"], lo=lo, hi=hi, tot=np.array(totals[:2]))
    td.barrier()
    td.destroy_process_group()


def test_gloo_world2_warm_chains_match_single_process(tmp_path):
    """Whole clouds per rank reproduce the single-process chains bit for bit."""
    from oracle import oracle
    out = str(tmp_path / "c")
    mp.spawn(_chain_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=20)
    opts = abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN, **o)
    ref, st = oracle.solve_chains(P, L, [0, 3, 9, 9, 14, 20], opts)
    r = [np.load(out + f".{k}.npz") for k in range(2)]
    assert r[0]["lo"] == 0 and r[0]["hi"] == r[1]["lo"] and r[1]["hi"] == 20
    assert np.array_equal(np.concatenate([r[0]["pops"], r[1]["pops"]]), ref)
    assert np.array_equal(np.concatenate([r[0]["iters"], r[1]["iters"]]), st["iterations"])
    assert r[0]["tot"][0] == st["iterations"].sum()
