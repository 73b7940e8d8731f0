#!/usr/bin/env python3
"""Benchmark: layer-iterations/s of the LVG level-population solve (BASELINE.json metric).

Default workload: CH3OH-A, 256 levels, ONE cloud of 4096 layers (BASELINE.json configs[2],
synth_v1) layer-sharded over the ranks with dist.shard_range — strong scaling, the metric's
"× 4096 layers, 1/2/4/8 GPU": with `--gpus N` every rank solves its contiguous block of
about 4096/N layers of the same cloud (the reference's serial layer loop,
radiative_transfer.cpp:236-256, split N ways). `--weak` gives every rank 4096 layers of a
4096·N-layer cloud instead (a diagnostic; BASELINE names no such config). The line reports
`layers_total` (4096 at every N), each rank's share (`shares`: layers, iterations, slowest
layer, kernel ms) and `max_share_ms`, the slowest rank's kernel time per step. `--workload` selects the other
BASELINE configs for their own lines: ph2o45_1024 (configs[1]), ch3ohe256_sweep
(configs[3], 128x128 = 16384 cells), oh24_overlap_2048 (configs[4]). `--chain-len C`
switches to the reference's default start rule (LVG_INIT_WARM_CHAIN,
radiative_transfer.cpp:247-252): the rank's layers become independent clouds of C
consecutive layers, each a warm chain, all solved in one launch (lvg_solve_chains_device;
one workgroup / wave per chain).

Launch. `python bench.py --gpus N` starts N rank processes itself (one per GPU, before
this process touches a GPU) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT set, waits for them and exits with the first failure's code; rank 0 prints
the line. Under torchrun (WORLD_SIZE already set) this process is one rank. `--gpus N`
with fewer than N visible GPUs fails before anything starts.

A "step" is one full batched solve of this rank's layers: per layer the collision
operator, boundary_layer_populations, and the iteration_control loop (calc_new_pop =
rate-matrix assembly + residual + LU, Ng acceleration) until convergence — everything
radiative_transfer.cpp:236-288 does per layer — followed by the per-step status
exchange (iteration total, non-converged count, max rel_error: dist.reduce_status_device,
one small RCCL all-reduce of this step's status tensor; the path's only collective).
Units = calc_new_pop calls (layer-iterations), counted from the per-layer status.

Inputs (layer SoA) are resident in HBM before the timed region; `value` never includes
PCIe (the task's measurement contract). The host entry (lvg_solve_layers:
layer upload + populations both ways) is timed over the same --steps after the timed region
and reported beside it as `host_entry_value` / `host_entry`.

CPU baseline (rank 0, N = 1): SURVEY 8(d)'s -O3 -march=native -fopenmp build of the oracle
(reference arithmetic, contraction allowed, compiled on this host) on the job's CPU share and
on one thread, and the bit-exact checker build on the job's share, each on a bounded sample.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
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
CLOCK_GHZ = 2.4              # MI355X max engine clock (MI355X_MICROARCH.md)


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


def latency_floor_cycles(N: int) -> float:
    """Dependent-chain floor of one calc_new_pop on one wave: the LU's N
    pivot columns are sequential, and each needs at least a 7-step DPP max reduction, a
    readlane broadcast and an fp64 division before the next column's key exists —
    about 10 dependent vector operations at >= 8 cycles each."""
    return 80.0 * N


def load_pmc_traffic(workload: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (not measured in this run)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            e = json.load(f).get(workload)
        if not e:
            return None, None
        return float(e["hbm_bytes_per_launch"]), f"{e.get('source', p)} ({e.get('round', '?')}, " \
            f"{e.get('units_per_launch', '?')} units/launch, commit {e.get('commit', '?')})"
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


# ---- GPU provenance (clock, power, identity), read by a child process ------------------

_SMI = ["rocm-smi", "--showclocks", "--showpower", "--showuniqueid", "--showserial", "--showproductname", "--json"]


def _smi_start():
    try:
        return subprocess.Popen(_SMI, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    except Exception:
        return None


def _smi_finish(p) -> dict:
    """Per card: sclk, mclk, socket power, unique id / serial, product (rocm-smi --json)."""
    if p is None:
        return {"error": "rocm-smi not runnable"}
    try:
        out, _ = p.communicate(timeout=30)
        raw = json.loads(out)
    except Exception as e:           # noqa: BLE001 - provenance is best effort, never fatal
        try:
            p.kill()
        except Exception:
            pass
        return {"error": f"rocm-smi: {type(e).__name__}"}
    cards = {}
    for card, d in raw.items():
        if not isinstance(d, dict):
            continue
        pick = {}
        for k, v in d.items():
            kl = k.lower()
            if "sclk" in kl or "mclk" in kl or "fclk" in kl:
                pick[k.strip().rstrip(":")] = v
            elif "power" in kl and "(w)" in kl:
                pick["power_w"] = v
            elif "unique id" in kl or "serial" in kl or kl.startswith("card series") or kl.startswith("card sku"):
                pick[k] = v
        cards[card] = pick
    return cards


class Provenance:
    """rocm-smi before the timed region (GPU idle), one started as the timed region
    begins (its sample lands inside it when the region outlasts the query), and one after."""

    def __init__(self, enabled: bool):
        self.enabled = enabled
        self.rec = {"host": socket.gethostname(), "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")}
        if enabled:
            self.rec["before"] = _smi_finish(_smi_start())
        self._during = None

    def timed_start(self):
        if self.enabled:
            self._during = _smi_start()

    def timed_end(self):
        if self.enabled:
            self.rec["during"] = _smi_finish(self._during)
            self.rec["after"] = _smi_finish(_smi_start())
        return self.rec


# ---- CPU baseline (the oracle: test infrastructure, timed beside the GPU) ---------------

def cpu_leg(prob, layers, opts, budget_s: float, threads: int, chain_len: int = 0, ref=False):
    """Oracle (C restatement, OpenMP schedule(dynamic,1) over layers, or over clouds for
    warm chains as the reference's shock-model loop) on a bounded sample. ref="native":
    the timing build (reference arithmetic, -O3 -march=native -fopenmp, contraction
    allowed); ref=False: the bit-exact checker build."""
    from oracle import oracle
    oracle.lib(ref)
    done = its = 0
    chunk = max(8, 4 * threads)
    if chain_len:
        chunk = chain_len * max(1, threads)
    t0 = time.perf_counter()
    while done < layers.nb_lay and time.perf_counter() - t0 < budget_s:
        idx = np.arange(done, min(done + chunk, layers.nb_lay))
        sub = layers.subset(idx)
        if chain_len:
            _, st = oracle.solve_chains(prob, sub, chain_offsets(idx.size, chain_len), opts, nthreads=threads, ref=ref)
        else:
            _, st = oracle.solve_layers(prob, sub, opts, nthreads=threads, ref=ref)
        its += int(st["iterations"].sum())
        done += idx.size
    dt = time.perf_counter() - t0
    return its / dt, f"first {done} of {layers.nb_lay} layers ({its} layer-iterations, {dt:.1f} s)"


def chain_offsets(n: int, chain_len: int) -> np.ndarray:
    """Clouds of chain_len consecutive layers (the last one shorter)."""
    return np.unique(np.r_[np.arange(0, n, chain_len), n]).astype(np.int32)


def cpu_baseline(prob, layers, opts, budget_s: float, chain_len: int = 0):
    """SURVEY 8(d)'s CPU baseline: the oracle's reference-arithmetic build compiled -O3
    -march=native -fopenmp on this host (contraction allowed; a timing leg, not a checker),
    on the job's CPU share; beside it the same build on one thread and the bit-exact checker
    build (-O3 -march=x86-64-v3 -ffp-contract=off) on the job's share."""
    from oracle import oracle
    info = host_info()
    # all the CPUs this process may use; the GPU box caps a job's share (OMP_NUM_THREADS)
    threads = info["affinity_cpus"]
    if info["omp_num_threads"] and info["omp_num_threads"].isdigit():
        threads = min(threads, int(info["omp_num_threads"]))
    v_all, s_all = cpu_leg(prob, layers, opts, budget_s, threads, chain_len, ref="native")
    v_one, s_one = cpu_leg(prob, layers, opts, budget_s, 1, chain_len, ref="native")
    v_chk, s_chk = cpu_leg(prob, layers, opts, budget_s, threads, chain_len, ref=False)
    sched = "OpenMP schedule(dynamic,1) over " + ("clouds" if chain_len else "layers")
    return {"value": v_all, "unit": UNIT, "cores": threads, "kind": "port",
            "sample": f"{s_all}; oracle/lvg_oracle.c {oracle.NATIVE_FLAGS}, {sched}, {threads} threads",
            "flags": oracle.NATIVE_FLAGS,
            "one_thread": {"value": v_one, "unit": UNIT, "cores": 1, "sample": s_one, "flags": oracle.NATIVE_FLAGS},
            "checker_build": {"value": v_chk, "unit": UNIT, "cores": threads, "sample": s_chk,
                              "flags": "-O3 -march=x86-64-v3 -fopenmp -ffp-contract=off (bit-exact checker)"},
            "host": info}


# ---- launcher -----------------------------------------------------------------------------

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus() -> int:
    """GPUs this process could use (torch.cuda.device_count() does not initialise the GPU
    on this image, so the launcher can ask before it starts the ranks)."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(args, argv) -> int:
    """One child per rank, each `bench.py <same args>` with the torch.distributed env.
    The children are killed when one of them fails (the others would wait at a barrier),
    when the launcher gets SIGINT/SIGTERM, and when `--launch-timeout` seconds pass (a rank
    hung at a rendezvous or a collective): the launcher then exits non-zero (124 on the
    deadline) and never leaves ranks holding GPUs behind."""
    import signal
    n = args.gpus
    if not args.stub:
        have = visible_gpus()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []

    def kill_all():
        for q in procs:
            if q.poll() is None:
                q.kill()
        for q in procs:
            try:
                q.wait(timeout=30)
            except Exception:
                pass

    def on_signal(signum, _frame):
        kill_all()
        sys.exit(128 + signum)

    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGINT, signal.SIGTERM)}
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
        rc = 0
        live = list(procs)
        deadline = time.monotonic() + args.launch_timeout
        while live:
            time.sleep(0.2)
            # poll first: ranks that finished just before the deadline are not killed
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    kill_all()          # a rank failed: the others would wait at a barrier
                    live = []
            if live and time.monotonic() > deadline:
                print(f"bench.py: ranks still running after {args.launch_timeout:.0f} s; killed", file=sys.stderr)
                kill_all()
                return 124
        return rc if rc >= 0 else 128 - rc
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)


# ---- one rank -----------------------------------------------------------------------------

class StubSolver:
    """CPU stand-in for the launcher test (--stub): no GPU, no oracle; every layer reports
    3 iterations. Exercises the rank setup, sharding, status reduction and reporting."""
    N = 0

    def __init__(self, N):
        self.N = N

    def solve_layers_device(self, n, soa, pops, status, opts, stream_ptr=0):
        pass

    def solve_chains_device(self, n, soa, offs, pops, status, opts, stream_ptr=0):
        pass

    def last_kernel_time(self):
        return 1.0, 1

    def last_coll_time(self):
        return 0.0

    def last_kernel_kind(self):
        return 0 if self.N else -1

    def close(self):
        pass


def run_rank(args) -> int:
    import torch
    from radiative_transfer_amd import abi, dist, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpus = args.gpus if args.gpus is not None else world
    if gpus != world:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE {world}", file=sys.stderr)
        return 2
    multi = world > 1
    stub = args.stub
    # a process group at world size 1 too (--process-group): the step's status all-reduce then
    # runs through RCCL on device tensors exactly as it does on every rank of an N-GPU run
    use_pg = multi or args.process_group
    backend = None
    if use_pg:
        import torch.distributed as td
        if not stub:
            torch.cuda.set_device(local)
        if not multi:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        td.init_process_group(backend="gloo" if stub else "nccl")
        backend = td.get_backend()
    elif not stub:
        torch.cuda.set_device(0)
    dev = torch.device("cpu") if stub else torch.device("cuda", torch.cuda.current_device())

    def sync():
        if not stub:
            torch.cuda.synchronize()

    kind, N, L_cfg, seed = synth.CONFIGS[args.workload]
    N = args.nb_lev or N
    L_cloud = args.layers or L_cfg
    total = L_cloud * world if args.weak else L_cloud
    prob, layers_all, o = synth.make_problem(args.workload, nb_lay=total, nb_lev=N)
    opts = abi.default_opts(**o)
    if args.chain_len:
        opts.init = abi.LVG_INIT_WARM_CHAIN
    offs_all = c_lo = c_hi = None
    if args.chain_len:
        # clouds of chain_len consecutive layers; whole clouds per rank (dist.chain_shard)
        offs_all = chain_offsets(total, args.chain_len)
        c_lo, c_hi = dist.chain_shard(offs_all, world, rank)
        lo, hi = int(offs_all[c_lo]), int(offs_all[c_hi])
    else:
        lo, hi = dist.shard_range(total, world, rank)
    mine = layers_all.subset(np.arange(lo, hi))
    n_mine = hi - lo

    if stub:
        solver = StubSolver(N)
        if args.stub_hang > 0:
            time.sleep(args.stub_hang)          # launcher test: a rank that does not finish
    else:
        from radiative_transfer_amd.native import LvgSolver
        solver = LvgSolver(prob, device=dev.index)
        if args.tuning:
            solver.set_tuning(args.tuning)
    soa = torch.from_numpy(mine.soa()).to(dev)
    pops = torch.zeros((max(n_mine, 1), N), dtype=torch.float64, device=dev)
    status = torch.zeros((max(n_mine, 1), abi.STATUS_DTYPE.itemsize // 8), dtype=torch.float64, device=dev)
    if stub:
        status.view(torch.int32)[:, abi.STATUS_DTYPE.fields["iterations"][1] // 4] = 3
        status.view(torch.int32)[:, abi.STATUS_DTYPE.fields["converged"][1] // 4] = 1
    stream_ptr = 0 if stub else torch.cuda.current_stream(dev).cuda_stream
    offs = (offs_all[c_lo:c_hi + 1] - lo).astype(np.int32) if args.chain_len else None

    def step():
        if n_mine > 0:                          # a rank may hold no clouds / layers at all
            if offs is not None:
                solver.solve_chains_device(n_mine, soa.data_ptr(), offs, pops.data_ptr(), status.data_ptr(), opts,
                                           stream_ptr=stream_ptr)
            else:
                solver.solve_layers_device(n_mine, soa.data_ptr(), pops.data_ptr(), status.data_ptr(), opts,
                                           stream_ptr=stream_ptr)
        return dist.reduce_status_device(status[:n_mine])

    for _ in range(max(1, args.warmup)):
        step()
    sync()
    st1 = dist.status_numpy(status[:n_mine])
    units_local = int(st1["iterations"].sum())
    max_layer_its = int(st1["iterations"].max()) if n_mine else 0

    prov = Provenance(enabled=(rank == 0 and not stub and not args.no_provenance))
    if use_pg:
        td.barrier()
    sync()
    prov.timed_start()
    kern_ms, coll_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        glob = step()
        ms, _ = solver.last_kernel_time()
        kern_ms.append(ms)
        coll_ms.append(solver.last_coll_time())
    sync()
    if use_pg:
        td.barrier()
    elapsed = time.perf_counter() - t0
    prov_rec = prov.timed_end()
    # the kernel the ABI chose; -1 (none) on a rank with no layers (the ABI reports -1 for
    # an empty launch too)
    kernel_kind = solver.last_kernel_kind() if n_mine > 0 else -1
    st2 = dist.status_numpy(status[:n_mine])
    assert int(st2["iterations"].sum()) == units_local, "iteration count changed between steps"
    # this rank's share: [lo, hi), iterations, slowest layer, mean kernel ms, step ms
    mine_rec = [float(lo), float(hi), float(units_local), float(max_layer_its),
                float(np.mean(kern_ms)) if n_mine else 0.0, 1e3 * elapsed / args.steps, float(kernel_kind)]
    shares = [mine_rec]
    if use_pg:
        rec = torch.tensor(mine_rec, dtype=torch.float64, device=dev)
        outs = [torch.zeros_like(rec) for _ in range(world)]
        td.all_gather(outs, rec)
        shares = [o.cpu().tolist() for o in outs]
        elapsed = max(r[5] for r in shares) * args.steps / 1e3          # max over ranks
        max_layer_its = int(max(r[3] for r in shares))
    units_total, nonconv, max_rel = int(glob[0].item()), int(glob[1].item()), float(glob[2].item())

    host_value = None
    if rank == 0 and world == 1 and not args.no_host_entry and not stub:
        # the host entry (lvg_solve_layers: layer upload, populations both ways over PCIe),
        # timed over the same --steps after the device-resident region
        its_h = 0
        th = time.perf_counter()
        for _ in range(args.steps):
            if offs is not None:
                _, sh = solver.solve_chains(mine, offs, opts)
            else:
                _, sh = solver.solve_layers(mine, opts)
            its_h += int(sh["iterations"].sum())
        dth = time.perf_counter() - th
        host_value = {"value": its_h / dth, "unit": UNIT, "steps": args.steps, "ms_per_step": 1e3 * dth / args.steps,
                      "entry": "lvg_solve_chains" if offs is not None else "lvg_solve_layers",
                      "note": "host buffers in and out (PCIe included); value is the device entry on HBM-resident buffers"}

    if rank == 0:
        print(json.dumps(report(args, world, N, total, L_cfg, lo, hi, units_total, units_local, nonconv, max_rel,
                                max_layer_its, elapsed, kern_ms, coll_ms, opts, offs, prov_rec, host_value,
                                prob, mine, stub, kernel_kind, shares, backend)), flush=True)
    solver.close()
    if use_pg:
        td.destroy_process_group()
    return 0


KERNELS = {-1: "none (empty launch)", 0: "lvg::solve_kernel", 1: "lvg::solve_wave_kernel",
           2: "lvg_wide::solve_kernel", 3: "lvg_big::solve_kernel"}


def report(args, world, N, total, L_cfg, lo, hi, units_total, units_local, nonconv, max_rel, max_layer_its,
           elapsed, kern_ms, coll_ms, opts, offs, prov_rec, host_value, prob, mine, stub, kernel_kind=0,
           shares=None, backend=None):
    from radiative_transfer_amd import synth
    value = units_total * args.steps / elapsed
    kms = float(np.mean(kern_ms))
    cms = float(np.mean(coll_ms))
    ms_step = 1e3 * elapsed / args.steps
    # the kernel the ABI chose for this launch (lvg_last_kernel_kind)
    kernel = KERNELS[kernel_kind]
    bound = binding_roof(N)
    per_launch = units_local
    F, B = flops_per_layer_iteration(N), bytes_per_layer_iteration(N)
    # committed PMC traffic applies only to the profiled configuration
    profiled = (N, hi - lo) == (synth.CONFIGS[args.workload][1], L_cfg) and not args.chain_len and not args.tuning
    traffic, tsrc = load_pmc_traffic(args.workload) if profiled else (None, None)
    if bound == "fp64":
        achieved = F * per_launch / (kms * 1e-3) / 1e12
        roof = {"bound": "fp64", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP64_TFLOPS,
                "peak_note": "MI355X FP64 peak 78.6 TF/s (vector FMA and v_mfma_f64 alike; not an MFMA claim)"}
    else:
        achieved = B * per_launch / (kms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS}
    roof.update({"traffic": traffic, "traffic_source": tsrc if traffic else None,
                 "kernel": kernel, "kernel_ms": kms,
                 # collision operators of the batch built ahead by lvg::coll_kernel (0 unless
                 # the tuning turns it on; not in kernel_ms)
                 "coll_kernel_ms": cms,
                 # the same flops over the whole step (queue sort, any collision pre-build and
                 # the status reduction included): the headline FP64 fraction
                 "fp64_frac_step": F * per_launch / (ms_step * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                 "flops_per_unit": F, "hbm_model_bytes_per_unit": B, "units_per_launch": per_launch,
                 "fp64_frac": F * per_launch / (kms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                 "hbm_model_frac": B * per_launch / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS})
    # When every layer of the launch is resident at once (the small-N configs), the launch
    # lasts as long as its slowest layer: a latency bound, stated against a chain floor.
    slowest = max_layer_its + 1                     # + the boundary-layer LU
    us_it = kms * 1e3 / slowest if slowest else 0.
    floor = latency_floor_cycles(N)
    roof["latency"] = {"slowest_layer_iterations": max_layer_its, "us_per_slowest_layer_iteration": us_it,
                       "cycles_per_iteration_at_2.4GHz": us_it * 1e-6 * CLOCK_GHZ * 1e9,
                       "floor_cycles_per_iteration": floor,
                       "floor_model": "N pivot columns x 80 cycles (7-step DPP max, readlane, fp64 division)",
                       "frac": floor / (us_it * 1e-6 * CLOCK_GHZ * 1e9) if us_it else None,
                       "binds": N <= 64}
    layers_rank = hi - lo
    out = {
        "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (synth_v1, SURVEY.md 8d)" + (" [STUB solver: launcher test]" if stub else ""),
        # a level or layer count other than the config's is named in the workload label
        "config": {"workload": args.workload + (f"_nblev{N}" if N != synth.CONFIGS[args.workload][1] else "")
                   + (f"_layers{args.layers}" if args.layers and args.layers != L_cfg else ""),
                   "nb_lev": N, "layers_total": total,
                   "layers_per_gpu": layers_rank if world == 1 or args.weak
                   else f"{total // world}-{-(-total // world)}",
                   "layer_iterations_per_step": units_total, "nonconverged_layers": nonconv,
                   "max_rel_error": max_rel,
                   "parallelism": f"clouds sharded x{world} (dist.chain_shard)" if args.chain_len
                   else f"layers sharded x{world} (dist.shard_range)",
                   "init": f"warm_chain x{len(offs) - 1} clouds of {args.chain_len} layers" if offs is not None
                   else "boundary_layer", "acceleration": bool(opts.acceleration),
                   "line_overlap": bool(opts.line_overlap), "tuning": args.tuning or None},
        "roofline": roof,
        # per rank: its layer block [lo, hi), layer-iterations, slowest layer's iterations,
        # mean kernel ms and timed ms per step, the kernel it ran; the step is the slowest share
        "shares": [{"rank": r, "lo": int(s[0]), "hi": int(s[1]), "layers": int(s[1] - s[0]),
                    "iterations": int(s[2]), "max_layer_iterations": int(s[3]), "kernel_ms": s[4],
                    "ms_per_step": s[5], "kernel": KERNELS[int(s[6])]} for r, s in enumerate(shares or [])],
        "max_share_ms": max((s[4] for s in shares), default=kms) if shares else kms,
        "provenance": prov_rec,
        # torch.distributed backend of the step's status all-reduce ("nccl" = RCCL over xGMI);
        # None: no process group (world size 1 without --process-group)
        "backend": backend,
    }
    if host_value is not None:
        out["host_entry_value"] = host_value["value"]
        out["host_entry"] = host_value
    if world == 1 and not args.no_cpu and not stub:
        out["cpu_baseline"] = cpu_baseline(prob, mine, opts, args.cpu_budget, args.chain_len)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default 1, or WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="ch3oha256_4096")
    ap.add_argument("--layers", type=int, default=0, help="layers of the cloud (--weak: per GPU); default the config's")
    ap.add_argument("--nb-lev", type=int, default=0, help="levels (default: the config's; 768 = reference CH3OH)")
    ap.add_argument("--strong", action="store_true",
                    help="split ONE cloud of the config's layers over the GPUs (the default; kept for old command lines)")
    ap.add_argument("--weak", action="store_true", help="every GPU solves the config's layers (a cloud N times larger)")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="seconds before the launcher kills ranks that have not finished")
    ap.add_argument("--chain-len", type=int, default=0,
                    help="warm chains of this many layers (LVG_INIT_WARM_CHAIN) instead of independent layers")
    ap.add_argument("--tuning", default="", help="lvg_set_tuning spec (diagnostics; results unchanged)")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-entry", action="store_true")
    ap.add_argument("--no-provenance", action="store_true")
    ap.add_argument("--process-group", action="store_true",
                    help="create the process group (RCCL) at world size 1 too; the status all-reduce goes through it")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)   # launcher test, CPU only
    ap.add_argument("--stub-hang", type=float, default=0.0, help=argparse.SUPPRESS)   # stub rank sleeps this long
    args = ap.parse_args(argv)
    if args.weak and args.strong:
        ap.error("--weak and --strong exclude each other")
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        return launch_ranks(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
