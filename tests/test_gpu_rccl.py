"""The multi-GPU path on the RCCL backend, on one GPU: a world-size-1 "nccl" process group
(VERDICT r5 item 5). Each case runs in its own process (a fresh port before any GPU call),
so the test process itself never initialises RCCL. Bit-exact against the oracle, as every
GPU test. The layers shard as dist.shard_range (radiative_transfer.cpp:236-256 is the serial
layer loop this replaces; the all-reduce is the residual / status reduction of SURVEY 8e)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from radiative_transfer_amd import abi, synth
from oracle import oracle
from parity_helpers import assert_same

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
                LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")


@pytest.mark.parametrize("name,nl", [("ph2o45_1024", 24), ("ch3oha256_4096", 8)])
def test_rccl_world_size_one(tmp_path, name, nl):
    out = str(tmp_path / "r.npz")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_world1.py"), out, name, str(nl)],
                       env=_env(), cwd=ROOT, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    d = np.load(out)
    P, L, o = synth.make_problem(name, nb_lay=nl)
    opts = abi.default_opts(**o)
    po, so = oracle.solve_layers(P, L, opts)
    sg = np.frombuffer(d["status"].tobytes(), dtype=abi.STATUS_DTYPE)
    assert_same(d["pops"], sg, po, so)
    sd = np.frombuffer(d["status_d"].tobytes(), dtype=abi.STATUS_DTYPE)
    assert_same(d["pops_d"], sd, po, so)
    its, nonconv = int(so["iterations"].sum()), int((so["converged"] == 0).sum())
    assert d["totals"][0] == its and d["totals"][1] == nonconv and d["totals"][2] == so["rel_error"].max()
    assert d["tot_d"][0] == its and d["tot_d"][1] == nonconv and d["tot_d"][2] == so["rel_error"].max()


def test_bench_process_group_world_one():
    """bench.py --process-group: the step's status all-reduce through RCCL at world size 1;
    the line names the backend."""
    r = subprocess.run([sys.executable, "-u", "bench.py", "--process-group", "--workload", "ph2o45_1024",
                        "--layers", "64", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-host-entry",
                        "--no-provenance"], env=_env(), cwd=ROOT, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["backend"] == "nccl" and line["n_gpus"] == 1
    P, L, o = synth.make_problem("ph2o45_1024", nb_lay=64)
    _, so = oracle.solve_layers(P, L, abi.default_opts(**o))
    assert line["config"]["layer_iterations_per_step"] == int(so["iterations"].sum())
    assert line["config"]["nonconverged_layers"] == 0
