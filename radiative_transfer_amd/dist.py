"""Multi-GPU layer sharding.

Layers are independent once every layer starts from its own
boundary_layer_populations guess, so a cloud shards into contiguous layer
blocks, one per rank (one process per GPU). There is no data-path collective:
the only exchange is the per-solve status reduction below (total
layer-iterations, non-converged layers, max rel_error), plus an optional
all_gather of the populations when the caller wants them on every rank.
The backend is whatever torch.distributed was initialised with: "nccl" (RCCL
over xGMI) on MI355X nodes, "gloo" in the CPU tests.
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of rank `rank`: layer l goes to rank floor(l*world/n)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lo = (n_total * rank) // world
    hi = (n_total * (rank + 1)) // world
    return lo, hi


def reduce_status(status: np.ndarray, device=None):
    """All-reduce of (sum iterations, sum non-converged, max rel_error) over ranks."""
    import torch
    import torch.distributed as td
    dev = device if device is not None else torch.device("cpu")
    s = torch.tensor([float(status["iterations"].sum()), float((status["converged"] == 0).sum())],
                     dtype=torch.float64, device=dev)
    m = torch.tensor([float(status["rel_error"].max()) if status.size else 0.0], dtype=torch.float64, device=dev)
    if td.is_available() and td.is_initialized():
        td.all_reduce(s, op=td.ReduceOp.SUM)
        td.all_reduce(m, op=td.ReduceOp.MAX)
    return int(s[0].item()), int(s[1].item()), float(m[0].item())


def solve_sharded(layers, solve_fn: Callable, n_lev: int, gather: bool = True, device=None):
    """Solve this rank's layer block with `solve_fn(layers_subset) -> (pops, status)`.

    Returns (pops, status, totals) where pops/status are the full cloud when
    `gather` (all_gather over ranks) and the local block otherwise.
    """
    import torch
    import torch.distributed as td
    world = td.get_world_size() if td.is_initialized() else 1
    rank = td.get_rank() if td.is_initialized() else 0
    lo, hi = shard_range(layers.nb_lay, world, rank)
    pops, status = solve_fn(layers.subset(np.arange(lo, hi)))
    totals = reduce_status(status, device)
    if not gather or world == 1:
        return pops, status, totals
    dev = device if device is not None else torch.device("cpu")
    counts = [shard_range(layers.nb_lay, world, r) for r in range(world)]
    maxn = max(h - l for l, h in counts)
    buf = torch.zeros((maxn, n_lev), dtype=torch.float64, device=dev)
    buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(pops)).to(dev)
    raw = np.frombuffer(status.tobytes(), dtype=np.float64).reshape(hi - lo, -1)
    sbuf = torch.zeros((maxn, raw.shape[1]), dtype=torch.float64, device=dev)
    sbuf[: hi - lo] = torch.from_numpy(raw.copy()).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    souts = [torch.zeros_like(sbuf) for _ in range(world)]
    td.all_gather(outs, buf)
    td.all_gather(souts, sbuf)
    full = np.concatenate([o[: h - l].cpu().numpy() for o, (l, h) in zip(outs, counts)])
    sfull = np.concatenate([s[: h - l].cpu().numpy() for s, (l, h) in zip(souts, counts)])
    st = np.frombuffer(np.ascontiguousarray(sfull).tobytes(), dtype=status.dtype).copy()
    return full, st, totals
