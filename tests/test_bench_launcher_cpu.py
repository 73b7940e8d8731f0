"""bench.py's own multi-rank launcher on the CPU (gloo, stub solver: no GPU, no oracle).

`python bench.py --gpus N` must start N ranks itself when WORLD_SIZE is unset, shard the
layers (weak scaling by default: N x the config's layers; --strong: one cloud split N
ways), reduce the per-step status over the ranks and print ONE line from rank 0 with
n_gpus == N; it must refuse --gpus N when fewer than N GPUs are visible. The path the
line measures is BASELINE.json's 1/2/4/8-GPU axis (radiative_transfer.cpp:152-216 is the
reference's parallel loop it replaces)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("gpus,strong", [(2, False), (2, True), (3, False), (1, False)])
def test_launcher_spawns_ranks(gpus, strong):
    args = ["--gpus", str(gpus), "--stub", "--steps", "2", "--warmup", "1", "--workload", "ph2o45_1024",
            "--layers", "8", "--no-cpu"] + (["--strong"] if strong else [])
    rc, lines, err = _run(*args)
    assert rc == 0, err
    assert len(lines) == 1, (lines, err)          # rank 0 only
    line = json.loads(lines[0])
    total = 8 if strong else 8 * gpus
    assert line["n_gpus"] == gpus
    assert line["scaling"] == ("strong" if strong else "weak")
    assert line["config"]["layers_total"] == total
    assert line["config"]["layer_iterations_per_step"] == 3 * total   # the stub's 3 per layer, all ranks
    assert line["value"] > 0 and line["steps"] == 2


def test_launcher_rank_without_clouds():
    """More ranks than warm-chain clouds: a rank with no clouds skips its solve and
    still joins the status reduction."""
    rc, lines, err = _run("--gpus", "2", "--stub", "--steps", "1", "--workload", "ph2o45_1024", "--layers", "4",
                          "--strong", "--chain-len", "8", "--no-cpu")
    assert rc == 0, err
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["layer_iterations_per_step"] == 12


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
