import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librcgpu.so)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def native():
    """The native library, built in-tree if needed (no fallback). On a GPU
    box torch's HIP runtime (torch bundles its own libamdhip64) is brought up
    first: tests that hand CUDA tensors to the engine need both in one
    process, and torch's lazy init after the engine's own runtime was seen
    to find no device."""
    if gpu_available():
        import torch
        torch.cuda.init()
    from rna_clique_amd.build import build_native
    build_native()
    from rna_clique_amd import _native
    return _native.lib()
