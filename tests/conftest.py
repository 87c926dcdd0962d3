import os
import sys

import pytest

# librrt.so resolves its HIP symbols from the first HIP runtime in the global scope.  PyTorch
# bundles its own copy; when both are used in one process (GPU tests that hand torch device
# buffers to the C ABI), torch must be imported first so the two share ONE runtime.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU-side test")
