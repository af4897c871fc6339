import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle", ROOT / "tests" / "golden"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"

# torch's bundled HIP runtime is mapped before anything loads libdeepimpact_hip.so
# directly (ctypes.CDLL in test_boundary): _lib.lib() refuses a process where another
# libamdhip64 came first (_lib._guard_hip_runtime)
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def pytest_collection_modifyitems(config, items):
    # torch's HIP runtime first when GPU tests run: torch cannot initialise the GPU after
    # the library's own (newer) runtime has, and a module run alone (test_index_gpu.py)
    # may reach a torch-using test only after library calls
    if any(item.get_closest_marker("gpu") for item in items):
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
