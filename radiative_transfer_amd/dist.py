"""Multi-GPU layer sharding.

Layers are independent once every layer starts from its own
boundary_layer_populations guess, so a cloud shards into contiguous layer
blocks, one per rank (one process per GPU). There is no data-path collective:
the only exchange is the per-solve status reduction below (total
layer-iterations, non-converged layers, max rel_error), plus an optional
all_gather of the populations when the caller wants them on every rank.
Warm chains (the reference's default start rule) are sequential within a cloud, so
there whole clouds go to ranks (`chain_shard`), contiguous and balanced by layer count.
The backend is whatever torch.distributed was initialised with: "nccl" (RCCL
over xGMI) on MI355X nodes, "gloo" in the CPU tests. Collective tensors live on
the current GPU under nccl (RCCL takes device tensors only) and on the CPU
otherwise, unless the caller names a device.
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np

from . import abi

_STATUS_WORDS = abi.STATUS_DTYPE.itemsize // 8          # lvg_layer_status as float64 words
_ITER_WORD = abi.STATUS_DTYPE.fields["iterations"][1] // 4   # int32 index of `iterations`
_CONV_WORD = abi.STATUS_DTYPE.fields["converged"][1] // 4
_REL_WORD = abi.STATUS_DTYPE.fields["rel_error"][1] // 8     # float64 index of `rel_error`


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of rank `rank`: layer l goes to rank floor(l*world/n)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lo = (n_total * rank) // world
    hi = (n_total * (rank + 1)) // world
    return lo, hi


def chain_shard(chain_off, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous range [c_lo, c_hi) of clouds of rank `rank` for warm chains
    (chain c = layers [chain_off[c], chain_off[c+1])): cloud c goes to the rank whose
    layer block (shard_range over all layers) holds the cloud's first layer, so ranks get
    whole clouds and about the same number of layers."""
    off = np.asarray(chain_off, dtype=np.int64)
    n = int(off[-1])
    lo, hi = shard_range(n, world, rank)
    starts = off[:-1]
    c_lo = int(np.searchsorted(starts, lo, side="left"))
    c_hi = int(np.searchsorted(starts, hi, side="left")) if rank < world - 1 else len(starts)
    return c_lo, c_hi


def solve_chains_sharded(layers, chain_off, solve_fn: Callable, n_lev: int, device=None):
    """Warm chains over ranks: this rank solves its clouds (chain_shard) with
    `solve_fn(layers_subset, local_chain_off) -> (pops, status)`; returns
    (pops, status, (first layer, last layer + 1), totals) for the local block."""
    import torch.distributed as td
    world = td.get_world_size() if td.is_initialized() else 1
    rank = td.get_rank() if td.is_initialized() else 0
    off = np.asarray(chain_off, dtype=np.int64)
    c_lo, c_hi = chain_shard(off, world, rank)
    l_lo, l_hi = int(off[c_lo]), int(off[c_hi])
    if l_hi > l_lo:
        pops, status = solve_fn(layers.subset(np.arange(l_lo, l_hi)), (off[c_lo:c_hi + 1] - l_lo).astype(np.int32))
    else:
        pops, status = np.zeros((0, n_lev)), np.zeros(0, dtype=abi.STATUS_DTYPE)
    return pops, status, (l_lo, l_hi), reduce_status(status, device)


def _default_device(device):
    import torch
    import torch.distributed as td
    if device is not None:
        return torch.device(device)
    if td.is_available() and td.is_initialized() and td.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def reduce_status(status: np.ndarray, device=None):
    """All-reduce of (sum iterations, sum non-converged, max rel_error) over ranks.
    `status` is this rank's host lvg_layer_status array (may be empty)."""
    import torch
    import torch.distributed as td
    dev = _default_device(device)
    s = torch.tensor([float(status["iterations"].sum()), float((status["converged"] == 0).sum())],
                     dtype=torch.float64, device=dev)
    m = torch.tensor([float(status["rel_error"].max()) if status.size else 0.0], dtype=torch.float64, device=dev)
    if td.is_available() and td.is_initialized():
        td.all_reduce(s, op=td.ReduceOp.SUM)
        td.all_reduce(m, op=td.ReduceOp.MAX)
    return int(s[0].item()), int(s[1].item()), float(m[0].item())


def reduce_status_device(status_t):
    """The same reduction on a device-resident status tensor [n, 5] float64 (the raw
    lvg_layer_status words written by lvg_solve_layers_device), without a host copy:
    returns a float64 tensor (sum iterations, sum non-converged, max rel_error) on the
    tensor's device, all-reduced over ranks when a process group is up."""
    import torch
    import torch.distributed as td
    words = status_t.reshape(-1, _STATUS_WORDS)
    if words.shape[0]:
        ints = words.contiguous().view(torch.int32)
        s = torch.stack([ints[:, _ITER_WORD].to(torch.float64).sum(),
                         (ints[:, _CONV_WORD] == 0).to(torch.float64).sum()])
        m = words[:, _REL_WORD].max().reshape(1).clone()
    else:                                   # an empty layer block (fewer layers than ranks)
        s = torch.zeros(2, dtype=torch.float64, device=words.device)
        m = torch.zeros(1, dtype=torch.float64, device=words.device)
    if td.is_available() and td.is_initialized():
        td.all_reduce(s, op=td.ReduceOp.SUM)
        td.all_reduce(m, op=td.ReduceOp.MAX)
    return torch.cat([s, m])


def status_numpy(status_t) -> np.ndarray:
    """Device status tensor [n, 5] float64 -> host lvg_layer_status array."""
    raw = status_t.detach().cpu().numpy()
    return np.frombuffer(np.ascontiguousarray(raw).tobytes(), dtype=abi.STATUS_DTYPE).copy()


def solve_sharded(layers, solve_fn: Callable, n_lev: int, gather: bool = True, device=None):
    """Solve this rank's layer block with `solve_fn(layers_subset) -> (pops, status)`.

    Returns (pops, status, totals) where pops/status are the full cloud when
    `gather` (all_gather over ranks) and the local block otherwise. A rank whose
    block is empty (fewer layers than ranks) does not call solve_fn.
    """
    import torch
    import torch.distributed as td
    world = td.get_world_size() if td.is_initialized() else 1
    rank = td.get_rank() if td.is_initialized() else 0
    lo, hi = shard_range(layers.nb_lay, world, rank)
    if hi > lo:
        pops, status = solve_fn(layers.subset(np.arange(lo, hi)))
    else:
        pops, status = np.zeros((0, n_lev)), np.zeros(0, dtype=abi.STATUS_DTYPE)
    totals = reduce_status(status, device)
    if not gather or world == 1:
        return pops, status, totals
    dev = _default_device(device)
    counts = [shard_range(layers.nb_lay, world, r) for r in range(world)]
    maxn = max(max(h - l for l, h in counts), 1)
    buf = torch.zeros((maxn, n_lev), dtype=torch.float64, device=dev)
    buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(pops).reshape(hi - lo, n_lev)).to(dev)
    raw = np.frombuffer(status.tobytes(), dtype=np.float64).reshape(hi - lo, _STATUS_WORDS)
    sbuf = torch.zeros((maxn, _STATUS_WORDS), dtype=torch.float64, device=dev)
    sbuf[: hi - lo] = torch.from_numpy(raw.copy()).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    souts = [torch.zeros_like(sbuf) for _ in range(world)]
    td.all_gather(outs, buf)
    td.all_gather(souts, sbuf)
    full = np.concatenate([o[: h - l].cpu().numpy() for o, (l, h) in zip(outs, counts)])
    sfull = np.concatenate([s[: h - l].cpu().numpy() for s, (l, h) in zip(souts, counts)])
    st = np.frombuffer(np.ascontiguousarray(sfull).tobytes(), dtype=abi.STATUS_DTYPE).copy()
    return full, st, totals
