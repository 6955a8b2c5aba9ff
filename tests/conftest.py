import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librcgpu.so)")
    config.addinivalue_line("markers", "heartbeat(seconds): how long the GPU heartbeat may keep a silent "
                                       "test alive (default HEARTBEAT_S)")


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


HEARTBEAT_S = 120


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """GPU tests: a line appended to gpurun_out/heartbeat.log every 30 s while
    the test runs. A GPU run is taken to be hung after 3 minutes with nothing
    new on stdout, stderr or under gpurun_out/, and pytest prints nothing
    during a test (-q) -- the full-size config tests (simulation, engine,
    oracle pairs) run longer than that. The beat stops after the test's
    `heartbeat` marker (about 2-3x its expected run time; HEARTBEAT_S when
    unmarked), so a test that hangs still goes silent and is caught."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    hb = request.node.get_closest_marker("heartbeat")
    limit = float(hb.args[0]) if hb else HEARTBEAT_S
    import threading
    import time
    stop = threading.Event()
    name = request.node.nodeid

    def beat():
        t0 = time.time()
        os.makedirs("gpurun_out", exist_ok=True)
        while not stop.wait(30) and time.time() - t0 < limit:
            with open(os.path.join("gpurun_out", "heartbeat.log"), "a") as f:
                f.write(f"{time.strftime('%H:%M:%S')} {name}: {time.time() - t0:.0f} s\n")

    t = threading.Thread(target=beat, daemon=True)
    t.start()
    try:
        yield
    finally:
        stop.set()
        t.join(timeout=5)
