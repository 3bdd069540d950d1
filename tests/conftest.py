"""Test configuration: `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "esp32-wake-word_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def xiaoa_sd():
    from wakeword.onnx_reader import read_onnx, xiaoa_state_dict
    inits, _, _ = read_onnx(os.path.join(GOLDEN, "xiaoa.onnx"))
    return xiaoa_state_dict(inits)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch
