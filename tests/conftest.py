import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through libcordagpu.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def engine():
    # torch ships its own HIP runtime (ROCm 7.0 libamdhip64.so) beside the system one the engine
    # links (/opt/rocm libamdhip64.so.7): with both in one process, torch's must open the device
    # first, or its later init reports "No HIP GPUs are available".
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    from corda_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()
