#!/usr/bin/env python3
"""Benchmark: layer-iterations/s of the LVG level-population solve (BASELINE.json metric).

Default workload: CH3OH-A, 256 levels, ONE 4096-layer cloud (BASELINE.json configs[2]),
layer-sharded over the ranks with dist.shard_range — strong scaling: `--gpus N` splits
the same 4096 layers N ways (`--weak` keeps 4096 layers per GPU instead).
`--workload` selects the other BASELINE configs for their own lines: ph2o45_1024
(configs[1]), ch3ohe256_sweep (configs[3], 128x128 = 16384 cells), oh24_overlap_2048
(configs[4]). `--chain-len C` switches to the reference's default start rule
(LVG_INIT_WARM_CHAIN, radiative_transfer.cpp:247-252): the rank's layers become
independent clouds of C consecutive layers, each a warm chain, all solved in one
launch (lvg_solve_chains_device; one workgroup / wave per chain).

A "step" is one full batched solve of this rank's layers: per layer the collision
operator, boundary_layer_populations, and the iteration_control loop (calc_new_pop =
rate-matrix assembly + residual + LU, Ng acceleration) until convergence — everything
radiative_transfer.cpp:236-288 does per layer — followed by the per-step status
exchange (iteration total, non-converged count, max rel_error: dist.reduce_status_device,
one small RCCL all-reduce of this step's status tensor; the path's only collective).
Units = calc_new_pop calls (layer-iterations), counted from the per-layer status.

Inputs (layer SoA) are resident in HBM before the timed region; `value` never includes
PCIe. The host entry (lvg_solve_layers: layer upload + populations both ways) is timed
once after the timed region and reported as `host_entry_value`.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "layer-iterations/sec, CH3OH-A 256 lev × 4096 layers, 1/2/4/8 GPU"
UNIT = "layer-iterations/s"
PEAK_FP64_TFLOPS = 78.6      # MI355X FP64 peak (vector and matrix alike), spec
PEAK_HBM_GBS = 8000.0        # MI355X HBM3E, spec


def flops_per_layer_iteration(N: int) -> float:
    """F_L = (2/3)N^3 + 4N^2."""
    return (2.0 / 3.0) * N ** 3 + 4.0 * N ** 2


def bytes_per_layer_iteration(N: int) -> float:
    """B_L = 8N^2 + 16N (dense-operand model)."""
    return 8.0 * N ** 2 + 16.0 * N


def binding_roof(N: int) -> str:
    """the roof that binds R (min of HBM and FP64 bounds)."""
    hbm = PEAK_HBM_GBS * 1e9 / bytes_per_layer_iteration(N)
    fp64 = PEAK_FP64_TFLOPS * 1e12 / flops_per_layer_iteration(N)
    return "hbm" if hbm < fp64 else "fp64"


def load_pmc_traffic(workload: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (not measured in this run)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            e = json.load(f).get(workload)
        if not e:
            return None, None
        return float(e["hbm_bytes_per_launch"]), f"{e.get('source', p)} ({e.get('round', '?')}, " \
            f"{e.get('units_per_launch', '?')} units/launch)"
    except Exception:
        return None, None


def host_info() -> dict:
    """nproc, the CPUs this process may run on, model, SMT (for the cpu_baseline line)."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": platform.processor() or None, "smt": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            v = v.strip()
            if k.strip() == "Model name":
                info["model"] = v
            elif k.strip() == "Thread(s) per core":
                info["smt"] = f"{v} thread(s) per core"
    except Exception:
        pass
    return info


def cpu_leg(prob, layers, opts, budget_s: float, threads: int, chain_len: int = 0):
    """Oracle (C restatement, OpenMP schedule(dynamic,1) over layers, or over clouds for
    warm chains as the reference's shock-model loop) on a bounded sample."""
    from oracle import oracle
    oracle.build()
    done = its = 0
    chunk = max(8, 4 * threads)
    if chain_len:
        chunk = chain_len * max(1, threads)
    t0 = time.perf_counter()
    while done < layers.nb_lay and time.perf_counter() - t0 < budget_s:
        idx = np.arange(done, min(done + chunk, layers.nb_lay))
        sub = layers.subset(idx)
        if chain_len:
            _, st = oracle.solve_chains(prob, sub, chain_offsets(idx.size, chain_len), opts, nthreads=threads)
        else:
            _, st = oracle.solve_layers(prob, sub, opts, nthreads=threads)
        its += int(st["iterations"].sum())
        done += idx.size
    dt = time.perf_counter() - t0
    return its / dt, f"first {done} of {layers.nb_lay} layers ({its} layer-iterations, {dt:.1f} s)"


def chain_offsets(n: int, chain_len: int) -> np.ndarray:
    """Clouds of chain_len consecutive layers (the last one shorter)."""
    return np.unique(np.r_[np.arange(0, n, chain_len), n]).astype(np.int32)


def cpu_baseline(prob, layers, opts, budget_s: float, chain_len: int = 0):
    info = host_info()
    # all the CPUs this process may use; the GPU box caps a job's share (OMP_NUM_THREADS)
    threads = info["affinity_cpus"]
    if info["omp_num_threads"] and info["omp_num_threads"].isdigit():
        threads = min(threads, int(info["omp_num_threads"]))
    v_all, s_all = cpu_leg(prob, layers, opts, budget_s, threads, chain_len)
    v_one, s_one = cpu_leg(prob, layers, opts, budget_s, 1, chain_len)
    return {"value": v_all, "unit": UNIT, "cores": threads, "kind": "port",
            "sample": f"{s_all}, oracle/lvg_oracle.c -O3 OpenMP schedule(dynamic,1), {threads} threads",
            "one_thread": {"value": v_one, "unit": UNIT, "cores": 1, "sample": s_one},
            "host": info}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="ch3oha256_4096")
    ap.add_argument("--layers", type=int, default=0, help="cloud layers (default: the config's)")
    ap.add_argument("--nb-lev", type=int, default=0, help="levels (default: the config's; 768 = reference CH3OH)")
    ap.add_argument("--weak", action="store_true", help="config's layers PER GPU instead of one cloud")
    ap.add_argument("--chain-len", type=int, default=0,
                    help="warm chains of this many layers (LVG_INIT_WARM_CHAIN) instead of independent layers")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-entry", action="store_true")
    args = ap.parse_args()

    import torch
    from radiative_transfer_amd import abi, dist, synth
    from radiative_transfer_amd.native import LvgSolver

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    multi = world > 1
    if multi:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group(backend="nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    kind, N, L_cfg, seed = synth.CONFIGS[args.workload]
    N = args.nb_lev or N
    L_cloud = args.layers or L_cfg
    total = L_cloud * world if args.weak else L_cloud
    prob, layers_all, o = synth.make_problem(args.workload, nb_lay=total, nb_lev=N)
    opts = abi.default_opts(**o)
    if args.chain_len:
        opts.init = abi.LVG_INIT_WARM_CHAIN
    if args.chain_len:
        # clouds of chain_len consecutive layers; whole clouds per rank (dist.chain_shard)
        offs_all = chain_offsets(total, args.chain_len)
        c_lo, c_hi = dist.chain_shard(offs_all, world, rank)
        lo, hi = int(offs_all[c_lo]), int(offs_all[c_hi])
    else:
        lo, hi = dist.shard_range(total, world, rank)
    mine = layers_all.subset(np.arange(lo, hi))
    n_mine = hi - lo

    solver = LvgSolver(prob, device=dev.index)
    soa = torch.from_numpy(mine.soa()).to(dev)
    pops = torch.zeros((max(n_mine, 1), N), dtype=torch.float64, device=dev)
    status = torch.zeros((max(n_mine, 1), abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    offs = (offs_all[c_lo:c_hi + 1] - lo).astype(np.int32) if args.chain_len else None

    def step():
        if offs is not None:
            solver.solve_chains_device(n_mine, soa.data_ptr(), offs, pops.data_ptr(), status.data_ptr(), opts,
                                       stream_ptr=stream.cuda_stream)
        else:
            solver.solve_layers_device(n_mine, soa.data_ptr(), pops.data_ptr(), status.data_ptr(), opts,
                                       stream_ptr=stream.cuda_stream)
        return dist.reduce_status_device(status[:n_mine])

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    units_local = int(dist.status_numpy(status[:n_mine])["iterations"].sum())

    if multi:
        td.barrier()
    torch.cuda.synchronize()
    kern_ms, coll_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        glob = step()
        ms, _ = solver.last_kernel_time()
        kern_ms.append(ms)
        coll_ms.append(solver.last_coll_time())
    torch.cuda.synchronize()
    if multi:
        td.barrier()
    elapsed = time.perf_counter() - t0
    st2 = dist.status_numpy(status[:n_mine])
    assert int(st2["iterations"].sum()) == units_local, "iteration count changed between steps"
    if multi:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        td.all_reduce(tt, op=td.ReduceOp.MAX)
        elapsed = float(tt.item())
    units_total, nonconv, max_rel = int(glob[0].item()), int(glob[1].item()), float(glob[2].item())

    host_value = None
    if rank == 0 and world == 1 and not args.no_host_entry:
        th = time.perf_counter()
        if offs is not None:
            _, sh = solver.solve_chains(mine, offs, opts)
        else:
            _, sh = solver.solve_layers(mine, opts)
        host_value = int(sh["iterations"].sum()) / (time.perf_counter() - th)

    if rank == 0:
        value = units_total * args.steps / elapsed
        kms = float(np.mean(kern_ms))
        ms_step = 1e3 * elapsed / args.steps
        kernel = "lvg::solve_wave_kernel" if N <= 64 else "lvg::solve_kernel" if N <= 256 else "lvg_big::solve_kernel"
        bound = binding_roof(N)
        per_launch = units_local
        # committed PMC traffic applies only to the profiled configuration
        traffic, tsrc = load_pmc_traffic(args.workload) if (N, total) == (synth.CONFIGS[args.workload][1],
                                                                           L_cfg) and not args.chain_len else (None, None)
        if bound == "fp64":
            achieved = flops_per_layer_iteration(N) * per_launch / (kms * 1e-3) / 1e12
            roof = {"bound": "fp64", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_FP64_TFLOPS,
                    "peak_note": "MI355X FP64 peak 78.6 TF/s (vector FMA and v_mfma_f64 alike; not an MFMA claim)"}
        else:
            achieved = bytes_per_layer_iteration(N) * per_launch / (kms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": achieved / PEAK_HBM_GBS}
        roof.update({"traffic": traffic, "traffic_source": tsrc if traffic else None,
                     "kernel": kernel, "kernel_ms": kms,
                     # collision operators of the batch, built ahead by lvg::coll_kernel (in the
                     # step time, not in kernel_ms; 0 when each layer builds its own in-kernel)
                     "coll_kernel_ms": float(np.mean(coll_ms)),
                     # the same flops over the whole step (collision build, queue sort and the
                     # status reduction included)
                     "fp64_frac_step": flops_per_layer_iteration(N) * per_launch / (ms_step * 1e-3) / 1e12
                     / PEAK_FP64_TFLOPS,
                     "flops_per_unit": flops_per_layer_iteration(N),
                     "hbm_model_bytes_per_unit": bytes_per_layer_iteration(N), "units_per_launch": per_launch,
                     "fp64_frac": flops_per_layer_iteration(N) * per_launch / (kms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                     "hbm_model_frac": bytes_per_layer_iteration(N) * per_launch / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS})
        out = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (synth_v1, SURVEY.md 8d)",
            "config": {"workload": args.workload, "nb_lev": N, "layers_total": total,
                       "layers_per_gpu": hi - lo if world == 1 else f"{total // world}-{-(-total // world)}",
                       "layer_iterations_per_step": units_total, "nonconverged_layers": nonconv,
                       "max_rel_error": max_rel,
                       "parallelism": f"clouds sharded x{world} (dist.chain_shard)" if args.chain_len
                       else f"layers sharded x{world} (dist.shard_range)",
                       "init": f"warm_chain x{len(offs) - 1} clouds of {args.chain_len} layers" if offs is not None
                       else "boundary_layer", "acceleration": bool(opts.acceleration),
                       "line_overlap": bool(opts.line_overlap)},
            "roofline": roof,
        }
        if host_value is not None:
            out["host_entry_value"] = host_value
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(prob, mine, opts, args.cpu_budget, args.chain_len)
        print(json.dumps(out))
    solver.close()
    if multi:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
