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


@pytest.fixture(autouse=True)
def _release_cached_device_memory(request):
    """Before every device test: free what earlier tests left in torch's
    caching allocator, so the full-size tests (150-250 GB shards allocated by
    libcyclone's own hipMalloc) find the HBM free."""
    if "cuda" in request.fixturenames:
        import gc
        import torch
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    yield
