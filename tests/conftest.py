import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libswifthip.so")


@pytest.fixture(scope="session")
def oracle32():
    import oracle_lib
    return oracle_lib.load("f32")


@pytest.fixture(scope="session")
def oracle64():
    import oracle_lib
    return oracle_lib.load("f64")


@pytest.fixture(scope="session")
def gpu_ctx():
    # torch's HIP runtime first, as bench.py does: a test that shares device
    # buffers through torch then finds the device whatever ran before it
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from swift_subtask_dev_amd import lib
    ctx = lib.Context(0, "f64")
    yield ctx
    ctx.close()
