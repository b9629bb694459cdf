import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _ensure_pkg():
    """Import the package from ``asr-rescoring_amd/`` (also when the symlink is absent)."""
    if "asr_rescoring_amd" in sys.modules:
        return
    try:
        import asr_rescoring_amd  # noqa: F401
    except ImportError:
        d = os.path.join(REPO, "asr-rescoring_amd")
        spec = importlib.util.spec_from_file_location("asr_rescoring_amd", os.path.join(d, "__init__.py"),
                                                      submodule_search_locations=[d])
        mod = importlib.util.module_from_spec(spec)
        sys.modules["asr_rescoring_amd"] = mod
        spec.loader.exec_module(mod)


_ensure_pkg()

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP) GPU and the built librescore.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
