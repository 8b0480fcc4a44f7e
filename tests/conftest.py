import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def heartbeat(msg: str) -> None:
    """Progress of a long GPU test, appended to gpurun_out/heartbeat.log when
    that directory exists (pytest captures stdout; a GPU run whose outputs
    stay silent for minutes is taken to be hung)."""
    import time
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "heartbeat.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")
