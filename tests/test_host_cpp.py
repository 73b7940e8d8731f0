"""C++ host surface (radiative_transfer_amd/host/lvg_host.hpp): the reference-shaped
classes (energy_diagram, einstein_coeff, collisional_transitions, dust_model,
lvg_method_data, cloud_data, iteration_scheme_lvg, iteration_control<T>,
boundary_layer_populations, calc_molecular_populations) driven from a C++ program
(tests/cpp/test_host_facade.cpp) and compared bit for bit with the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "test_host_facade")


def _build():
    from radiative_transfer_amd import build
    from oracle import oracle
    build.build_host()
    oracle.build()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])


def _run(tmp_path):
    _build()
    return subprocess.run([EXE, str(tmp_path) + "/"], capture_output=True, text=True, timeout=600)


def test_host_facade_without_device(tmp_path):
    """No GPU here: the table loader round trip still runs and the device error
    surfaces as lvg_error(LVG_E_DEVICE) -> exit code 3, never a CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present: covered by the gpu test")
    r = _run(tmp_path)
    assert "lvg_method_data save/load round trip (p)     equal" in r.stdout, r.stdout
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    assert "NO_DEVICE" in r.stdout


@pytest.mark.gpu
def test_host_facade_bit_exact(tmp_path):
    r = _run(tmp_path)
    print(r.stdout)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert "ALL EQUAL" in r.stdout
