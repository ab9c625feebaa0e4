import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

REFERENCE = Path("/root/reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the in-tree native library exists (build() is cheap when up to date)."""
    from retina_amd import _build

    _build.build_library()
    yield


@pytest.fixture(scope="session")
def reference_dir():
    if not REFERENCE.exists():
        pytest.skip("reference tree not mounted")
    return REFERENCE


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no GPU visible")
    return 0


os.environ.setdefault("PYTHONHASHSEED", "0")
