"""The multi-GPU path (radiative_transfer_amd/dist.py) wrapping the HIP solver — tolerance:
none, bit for bit against the single-process HIP solve and the oracle.

torch.distributed world size 2 on the one GPU of the box (each rank its own LvgSolver
handle on cuda:0, gloo for the collectives: RCCL does not take two ranks on one device).
The ranks solve their contiguous layer blocks (dist.shard_range), the populations come back
through all_gather and the per-step status reduction (dist.reduce_status_device, bench.py's
collective) sums iterations and non-converged layers and takes the max rel_error. This is
the reference's parallel axis, the loop over shock models of radiative_transfer.cpp:152-216,
spread over ranks; tests/test_distributed_cpu.py covers the same code with the oracle as the
per-rank solver.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from radiative_transfer_amd import abi, dist, synth

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, nl, out):
    import torch
    import torch.distributed as td
    from radiative_transfer_amd.native import LvgSolver
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    s = LvgSolver(P)
    pops, st, totals = dist.solve_sharded(L, lambda sub: s.solve_layers(sub, opts), P.mol.nb_lev, gather=True)
    lo, hi = dist.shard_range(nl, world, rank)
    raw = np.frombuffer(st[lo:hi].tobytes(), dtype=np.float64).reshape(hi - lo, abi.STATUS_DTYPE.itemsize // 8)
    dev_tot = dist.reduce_status_device(torch.from_numpy(raw.copy())).numpy()
    s.close()
    if rank == 0:
        np.savez(out, pops=pops, iters=st["iterations"], conv=st["converged"], rel=st["rel_error"],
                 totals=np.array([totals[0], totals[1]]), relmax=np.array([totals[2]]), dev_tot=dev_tot)
    td.barrier()
    td.destroy_process_group()


@pytest.mark.parametrize("name,nl", [("ph2o45_1024", 24), ("ch3oha256_4096", 6), ("oh24_overlap_2048", 1)])
def test_sharded_hip_solver_world2(tmp_path, name, nl):
    from oracle import oracle
    from radiative_transfer_amd.native import LvgSolver
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), name, nl, out), nprocs=2, join=True)
    got = np.load(out)
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    s = LvgSolver(P)
    p1, s1 = s.solve_layers(L, opts)
    s.close()
    po, so = oracle.solve_layers(P, L, opts)
    assert np.array_equal(got["pops"], p1) and np.array_equal(p1, po)
    assert np.array_equal(got["iters"], s1["iterations"]) and np.array_equal(s1["iterations"], so["iterations"])
    assert np.array_equal(got["conv"], s1["converged"])
    assert got["totals"][0] == s1["iterations"].sum()
    assert got["totals"][1] == (s1["converged"] == 0).sum()
    assert got["relmax"][0] == s1["rel_error"].max()
    assert np.array_equal(got["dev_tot"], [s1["iterations"].sum(), (s1["converged"] == 0).sum(), s1["rel_error"].max()])
