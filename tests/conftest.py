import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_sessionfinish(session, exitstatus):
    from tests import parity_log
    parity_log.write(os.environ.get("C2D_PARITY_LOG", str(ROOT / "gpurun_out" / "parity_metrics.tsv")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libc2d_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    from clap2diffusion_amd import _lib
    _lib.lib()  # loud failure if the library is missing
    return torch.device("cuda:0")


@pytest.fixture
def progress():
    """Append a line to gpurun_out/test_progress.log (long CPU-oracle legs of the GPU tests keep
    the GPU box's output alive: pytest captures stdout / stderr until a test ends)."""
    import time
    path = ROOT / "gpurun_out" / "test_progress.log"
    path.parent.mkdir(parents=True, exist_ok=True)

    def _log(msg: str) -> None:
        with open(path, "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {os.environ.get('PYTEST_CURRENT_TEST', '?').split(' ')[0]} {msg}\n")
    return _log
