#!/usr/bin/env python3
"""Benchmark: layer-iterations/s of the LVG level-population solve, CH3OH-A
256 levels x 4096 layers per GPU (BASELINE.json metric, configs[2]).

A "step" is one full batched solve of this rank's layers: per layer the
collision operator, boundary_layer_populations, and the iteration_control loop
(calc_new_pop = rate-matrix assembly + residual + LU, Ng acceleration) until
convergence — everything radiative_transfer.cpp:236-288 does per layer.
Units = calc_new_pop calls (layer-iterations), counted from the per-layer status.

Inputs (layer SoA) are resident in HBM before the timed region; the kernel runs
on torch's current stream. Multi-GPU: one process per GPU, layers sharded with
no data-path collective (weak scaling: 4096 layers per GPU); one RCCL
all-reduce per step exchanges the per-rank status (iteration total, non-
converged count, max residual) — the only cross-layer quantity of the path.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "layer-iterations/sec, CH3OH-A 256 lev × 4096 layers, 1/2/4/8 GPU"
UNIT = "layer-iterations/s"
PEAK_FP64_TFLOPS = 78.6      # MI355X FP64 (vector = dense matrix) peak, spec
PEAK_HBM_GBS = 8000.0


def flops_per_layer_iteration(N: int) -> float:
    """F_L = (2/3)N^3 + 4N^2."""
    return (2.0 / 3.0) * N ** 3 + 4.0 * N ** 2


def bytes_per_layer_iteration(N: int) -> float:
    """B_L = 8N^2 + 16N (dense-operand model)."""
    return 8.0 * N ** 2 + 16.0 * N


def load_pmc_traffic(N: int, workload: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc pass (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(workload)
        return float(e["hbm_bytes_per_launch"]) if e else None
    except Exception:
        return None


def cpu_baseline(prob, layers, opts, budget_s: float, threads: int):
    """Oracle (C restatement, OpenMP over layers) on a bounded sample of the same workload."""
    from oracle import oracle
    oracle.build()
    done_layers = 0
    its = 0
    t0 = time.perf_counter()
    chunk = 64
    while done_layers < layers.nb_lay and time.perf_counter() - t0 < budget_s:
        idx = np.arange(done_layers, min(done_layers + chunk, layers.nb_lay))
        _, st = oracle.solve_layers(prob, layers.subset(idx), opts, nthreads=threads)
        its += int(st["iterations"].sum())
        done_layers += idx.size
    dt = time.perf_counter() - t0
    return {"value": its / dt, "unit": UNIT, "cores": threads, "kind": "port",
            "sample": f"first {done_layers} of {layers.nb_lay} layers ({its} layer-iterations, {dt:.1f} s), "
                      f"oracle/lvg_oracle.c OpenMP schedule(dynamic,1)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="ch3oha256_4096")
    ap.add_argument("--layers", type=int, default=0, help="layers per GPU (default: the config's)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    from radiative_transfer_amd import abi, synth
    from radiative_transfer_amd.native import LvgSolver

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group(backend="nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    kind, N, L_cfg, seed = synth.CONFIGS[args.workload]
    per_gpu = args.layers or L_cfg
    # the global cloud: world x per_gpu layers from the config's generator; rank r owns a contiguous block
    prob, layers_all, o = synth.make_problem(args.workload, nb_lay=per_gpu * world)
    opts = abi.default_opts(**o)
    mine = layers_all.subset(np.arange(rank * per_gpu, (rank + 1) * per_gpu))

    solver = LvgSolver(prob, device=dev.index)
    soa = torch.from_numpy(mine.soa()).to(dev)
    pops = torch.zeros((per_gpu, N), dtype=torch.float64, device=dev)
    status = torch.zeros((per_gpu, abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        solver.solve_layers_device(per_gpu, soa.data_ptr(), pops.data_ptr(), status.data_ptr(), opts,
                                   stream_ptr=stream.cuda_stream)

    def status_np():
        raw = status.cpu().numpy().view(np.uint8).reshape(-1)
        return np.frombuffer(raw.tobytes(), dtype=abi.STATUS_DTYPE)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    st = status_np()
    units_local = int(st["iterations"].sum())

    # per-rank status exchange (the path's only collective)
    red = torch.tensor([float(units_local), float((st["converged"] == 0).sum()), float(st["rel_error"].max())],
                       dtype=torch.float64, device=dev)

    def reduce_status(t):
        if dist:
            import torch.distributed as td
            s = t[:2].clone()
            m = t[2:].clone()
            td.all_reduce(s, op=td.ReduceOp.SUM)
            td.all_reduce(m, op=td.ReduceOp.MAX)
            return torch.cat([s, m])
        return t

    if dist:
        import torch.distributed as td
        td.barrier()
    torch.cuda.synchronize()
    kern_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ms, _ = solver.last_kernel_time()
        kern_ms.append(ms)
        glob = reduce_status(red)
    torch.cuda.synchronize()
    if dist:
        td.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    st2 = status_np()
    assert int(st2["iterations"].sum()) == units_local, "iteration count changed between steps"
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        td.all_reduce(tt, op=td.ReduceOp.MAX)
        elapsed = float(tt.item())
    units_total = int(glob[0].item())
    nonconv = int(glob[1].item())

    if rank == 0:
        value = units_total * args.steps / elapsed
        kms = float(np.mean(kern_ms))
        per_launch_units = units_local
        achieved = flops_per_layer_iteration(N) * per_launch_units / (kms * 1e-3) / 1e12
        traffic = load_pmc_traffic(N, args.workload)
        out = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (synth_v1, SURVEY.md 8d)",
            "config": {"workload": args.workload, "nb_lev": N, "layers_per_gpu": per_gpu,
                       "layers_total": per_gpu * world, "layer_iterations_per_step": units_total,
                       "nonconverged_layers": nonconv, "parallelism": f"layers sharded x{world}",
                       "init": "boundary_layer", "acceleration": bool(opts.acceleration)},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic,
                         "kernel": "lvg::solve_kernel", "kernel_ms": kms,
                         "flops_per_unit": flops_per_layer_iteration(N), "units_per_launch": per_launch_units,
                         "hbm_model_bytes_per_unit": bytes_per_layer_iteration(N),
                         "hbm_model_frac": value / world * bytes_per_layer_iteration(N) / (PEAK_HBM_GBS * 1e9)},
        }
        if world == 1 and not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(prob, mine, opts, args.cpu_budget, threads)
        print(json.dumps(out))
    solver.close()
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
