import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: full-size cases")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    O.lib()
    return O


@pytest.fixture(autouse=True)
def _counter_trace(request):
    """Lab diagnostic (LK_DIAG_COUNTERS=<file>): the split-K counter sum after every GPU test, so the
    first test that leaves a counter armed is named. Off by default."""
    path = os.environ.get("LK_DIAG_COUNTERS")
    yield
    if not path or request.node.get_closest_marker("gpu") is None:
        return
    try:
        import torch
        if not torch.cuda.is_available():
            return
        import ggml_hip as G
        v = G.syncCountersSum()
    except Exception as e:  # noqa: BLE001 — diagnostic only
        v = f"error {e}"
    with open(path, "a") as f:
        f.write(f"{request.node.nodeid} {v}\n")


@pytest.fixture(scope="session")
def gpu():
    """Device + the HIP backend library; fails (not skips) when the library is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this environment")
    import ggml_hip
    ggml_hip.load_library()
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
