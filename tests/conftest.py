import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libswifthip.so")


_torch_hip = []


def pytest_runtest_setup(item):
    # torch's HIP runtime first, before the first GPU test opens the library's
    # (as bench.py does): torch finds no device once the other runtime holds
    # it, so a test sharing buffers through torch must not depend on the order
    if _torch_hip or item.get_closest_marker("gpu") is None:
        return
    _torch_hip.append(True)
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


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
    from swift_subtask_dev_amd import lib
    ctx = lib.Context(0, "f64")
    yield ctx
    ctx.close()
