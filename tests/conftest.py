import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


import pytest


@pytest.fixture(autouse=True, scope="session")
def _torch_hip_first():
    """On a GPU box, let torch initialise its HIP runtime before the first test loads
    liblvg_amd.so: torch's device init fails ("No HIP GPUs are available") once the
    library's runtime holds the device in the same process. device_count() does not
    initialise the GPU, so this is a no-op on the CPU container."""
    try:
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:
        pass
    yield
