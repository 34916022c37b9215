"""The failure contract of the grid-synchronising kernels (include/lk_hip.h, lk_sync_timeouts):
the batched kernels reduce their split-K slabs inside the launch, workgroups waiting for each
other with a bounded wait. A wait that gives up must never turn into LK_OK — the synchronous
entry points return LK_ERR_DEVICE (HipDeviceError here; GGMLStatus.FAILED at backend level,
core/GGMLCpuBackend.kt:167-176) — and the arrival counters must re-arm inside every launch
(no counter survives a launch, so none can wrap however many calls a process makes)."""
import numpy as np
import pytest

from _util import random_acts, random_weights
from test_gpu_parity import gpu_matmul

pytestmark = pytest.mark.gpu

DEFAULT_BOUND = 20000000  # 200 ms at 100 MHz


@pytest.mark.parametrize("qt,M,K,N", [(2, 11008, 4096, 32), (2, 4096, 11008, 32), (3, 4096, 4096, 8), (2, 4096, 4096, 512)])
def test_split_k_counters_rearm_every_launch(gpu, oracle, qt, M, K, N):
    import ggml_hip as G
    q = oracle.quantize(qt, random_weights(M * K, 5))
    x = random_acts(K * N, 6).reshape(K, N)
    first = gpu_matmul(qt, q, M, K, N, x)
    assert G.syncCountersSum() == 0
    for _ in range(3):
        again = gpu_matmul(qt, q, M, K, N, x)
        assert np.array_equal(again.view(np.uint32), first.view(np.uint32))
        assert G.syncCountersSum() == 0
    assert G.syncTimeouts() == 0


def test_wait_that_gives_up_raises(gpu, oracle):
    """Wait bound 0: a workgroup that does not find its range's other K slices already arrived gives
    up at once. lk_mul_mat (host path) and lk_graph_compute must raise, not return wrong bytes with
    LK_OK; with the bound restored the same calls succeed bit-exactly and the counters are re-armed."""
    import ggml_hip as G
    qt, M, K, N = 2, 11008, 4096, 32
    q = oracle.quantize(qt, random_weights(M * K, 7))
    x = random_acts(K * N, 8).reshape(K, N)
    want = gpu_matmul(qt, q, M, K, N, x, host=True)
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=q.size + 4 * (K * N + M * N) + 4096)
    a = ga.allocateTensor(G.GGMLType.Q4_0, [K, M]); ga.setTensorBytes(a, q)
    b = ga.allocateTensor(G.GGMLType.F32, [N, K]); ga.setTensorBytes(b, np.ascontiguousarray(x))  # B(n, k) at k*4N + 4n
    d = ga.allocateTensor(G.GGMLType.F32, [N, M])
    g = G.ResidentGraph(ga, [(a, b, d)])
    g.compute()
    try:
        G.setSyncWaitBound(0)
        with pytest.raises(G.HipDeviceError, match="gave up"):
            G.computeMatMul(ga, ga.context, a, b, d)
        with pytest.raises(G.HipDeviceError, match="gave up"):
            g.compute()
    finally:
        G.setSyncWaitBound(DEFAULT_BOUND)
    assert G.syncTimeouts() > 0  # the device count saw them too (and is reset here)
    assert G.syncCountersSum() == 0
    G.computeMatMul(ga, ga.context, a, b, d)
    got = np.frombuffer(bytes(ga.tensorBytes(d)), np.float32).reshape(M, N)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    g.compute()
    assert bytes(ga.tensorBytes(d)) == got.tobytes()
    assert G.syncTimeouts() == 0
    g.close()
