"""bench.py's own multi-rank launcher on the CPU (gloo, stub solver: no GPU, no oracle).

`python bench.py --gpus N` must start N ranks itself when WORLD_SIZE is unset, shard the
layers (strong scaling by default: ONE cloud of the config's layers split N ways, as
BASELINE configs[2] names it; --weak: N x the config's layers), reduce the per-step
status over the ranks and print ONE line from rank 0 with n_gpus == N, every rank's
share and the slowest share; it must refuse --gpus N when fewer than N GPUs are visible. The path the
line measures is BASELINE.json's 1/2/4/8-GPU axis (radiative_transfer.cpp:152-216 is the
reference's parallel loop it replaces)."""
import json
import os
import subprocess
import sys

import pytest

from radiative_transfer_amd import dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("gpus,mode", [(2, ""), (2, "--strong"), (2, "--weak"), (3, ""), (3, "--weak"), (1, "")])
def test_launcher_spawns_ranks(gpus, mode):
    args = ["--gpus", str(gpus), "--stub", "--steps", "2", "--warmup", "1", "--workload", "ph2o45_1024",
            "--layers", "8", "--no-cpu"] + ([mode] if mode else [])
    rc, lines, err = _run(*args)
    assert rc == 0, err
    assert len(lines) == 1, (lines, err)          # rank 0 only
    line = json.loads(lines[0])
    weak = mode == "--weak"
    total = 8 * gpus if weak else 8
    assert line["n_gpus"] == gpus
    assert line["scaling"] == ("weak" if weak else "strong")
    assert line["config"]["layers_total"] == total
    assert line["config"]["layer_iterations_per_step"] == 3 * total   # the stub's 3 per layer, all ranks
    assert line["value"] > 0 and line["steps"] == 2
    assert [(s["lo"], s["hi"]) for s in line["shares"]] == [dist.shard_range(total, gpus, r) for r in range(gpus)]


def test_default_is_the_metric_cloud_strong():
    """No flags but --gpus 2: BASELINE configs[2] as the metric names it — ONE cloud of
    4096 CH3OH-A layers split two ways: each rank's block is
    dist.shard_range(4096, 2, r), the reduced totals cover the 4096 layers once, and the
    line carries every rank's share and the slowest share's kernel time."""
    rc, lines, err = _run("--gpus", "2", "--stub", "--steps", "1", "--no-cpu")
    assert rc == 0, err
    line = json.loads(lines[0])
    assert line["scaling"] == "strong" and line["n_gpus"] == 2
    assert line["config"]["workload"] == "ch3oha256_4096"
    assert line["config"]["layers_total"] == 4096
    assert line["config"]["layer_iterations_per_step"] == 3 * 4096
    sh = line["shares"]
    assert [(s["lo"], s["hi"]) for s in sh] == [dist.shard_range(4096, 2, r) for r in range(2)] == [(0, 2048),
                                                                                                  (2048, 4096)]
    assert sum(s["iterations"] for s in sh) == 3 * 4096 and all(s["layers"] == 2048 for s in sh)
    assert line["max_share_ms"] == max(s["kernel_ms"] for s in sh)
    # the same with --strong (old command lines) and at 8 ranks: 512 layers each
    rc, lines, err = _run("--gpus", "8", "--strong", "--stub", "--steps", "1", "--no-cpu")
    assert rc == 0, err
    line = json.loads(lines[0])
    assert line["config"]["layers_total"] == 4096
    assert [s["layers"] for s in line["shares"]] == [512] * 8


def test_launcher_rank_without_clouds():
    """More ranks than warm-chain clouds: a rank with no clouds skips its solve and
    still joins the status reduction."""
    rc, lines, err = _run("--gpus", "2", "--stub", "--steps", "1", "--workload", "ph2o45_1024", "--layers", "4",
                          "--strong", "--chain-len", "8", "--no-cpu")
    assert rc == 0, err
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["layer_iterations_per_step"] == 12
    assert [s["layers"] for s in line["shares"]] == [4, 0]
    assert line["shares"][1]["kernel"].startswith("none")


def test_launcher_refuses_missing_gpus():
    """No GPU in this container: --gpus 2 (without the stub) fails before any rank starts."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible")
    rc, lines, err = _run("--gpus", "2", "--steps", "1", "--no-cpu")
    assert rc != 0 and not lines
    assert "visible GPUs" in err


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub", "--no-cpu"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_launcher_deadline_kills_ranks():
    """A rank that never finishes (the stub ranks sleep 120 s, far past the 3 s deadline)
    does not hang the launcher: it kills its ranks and exits 124."""
    rc, lines, err = _run("--gpus", "2", "--stub", "--steps", "1", "--workload", "ph2o45_1024", "--layers", "4",
                          "--no-cpu", "--launch-timeout", "3", "--stub-hang", "120", timeout=100)
    assert rc == 124 and not lines
    assert "killed" in err


def test_process_group_at_world_one():
    """--process-group builds the process group at world size 1 (gloo with the stub; RCCL on
    the GPU, tests/test_gpu_rccl.py) and the line names its backend; without it, no group."""
    rc, lines, err = _run("--stub", "--process-group", "--steps", "1", "--workload", "ph2o45_1024", "--layers", "8",
                          "--no-cpu")
    assert rc == 0, err
    line = json.loads(lines[0])
    assert line["backend"] == "gloo" and line["n_gpus"] == 1
    assert line["config"]["layer_iterations_per_step"] == 3 * 8
    rc, lines, err = _run("--stub", "--steps", "1", "--workload", "ph2o45_1024", "--layers", "8", "--no-cpu")
    assert rc == 0, err
    assert json.loads(lines[0])["backend"] is None
