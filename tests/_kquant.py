"""K-quant test helpers: random super-blocks with finite scales, and an independent numpy/Python
restatement of llama.kotlin's K-quant dots (core/GGMLComputeOps.kt:152-432) that cross-checks the
C oracle (oracle/lk_oracle.c). Test infrastructure only."""
import numpy as np

Q2_K, Q4_K, Q8_K = 8, 10, 13
BB = {Q2_K: 84, Q4_K: 144, Q8_K: 292}
QK_K = 256
f32 = np.float32


def random_kblocks(qt, nblk, seed):
    """nblk random super-blocks: random code bytes, finite scales (f16 d/dmin, f32 d for Q8_K)."""
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, size=(nblk, BB[qt]), dtype=np.uint8)
    if qt == Q2_K:
        raw[:, 80:82] = (rng.uniform(-0.05, 0.05, nblk).astype(np.float16)).view(np.uint8).reshape(nblk, 2)
        raw[:, 82:84] = (rng.uniform(-0.05, 0.05, nblk).astype(np.float16)).view(np.uint8).reshape(nblk, 2)
    elif qt == Q4_K:
        raw[:, 0:2] = (rng.uniform(-0.05, 0.05, nblk).astype(np.float16)).view(np.uint8).reshape(nblk, 2)
        raw[:, 2:4] = (rng.uniform(-0.05, 0.05, nblk).astype(np.float16)).view(np.uint8).reshape(nblk, 2)
    else:
        raw[:, 0:4] = (rng.uniform(-0.01, 0.01, nblk).astype(np.float32)).view(np.uint8).reshape(nblk, 4)
    return raw.reshape(-1)


def _h(b, o):
    return f32(np.frombuffer(bytes(b[o:o + 2]), dtype=np.float16)[0])


def _sb(v):  # Kotlin Byte.toInt(): sign-extended
    return int(v) - 256 if v >= 128 else int(v)


def _q2k_w(blk, item, d, dmin):
    sb = item // 16
    sm = _sb(blk[sb])
    scale = f32(f32(f32(sm & 0x0F) / f32(15.0)) * d)
    mn = f32(f32(f32((sm >> 4) & 0x0F) * d) + dmin)
    qb = _sb(blk[16 + sb * 4 + (item % 16) // 4])
    q = (qb >> (((item % 16) % 4) * 2)) & 0x03
    return f32(f32(f32(f32(q) / f32(3.0)) * scale) + mn)


def _q4k_w_full(blk, item, d, dmin):
    sb = item // 32
    sc = _sb(blk[4 + sb])
    qs, qml = sc & 0x3F, (sc >> 6) & 0x03
    qmh = (_sb(blk[4 + sb * 2 + 1]) & 0x0F) if sb * 2 + 1 < 12 else 0
    qm = qml | (qmh << 2)
    scale = f32(f32(f32(qs) / f32(63.0)) * d)
    mn = f32(f32(f32(f32(qm) / f32(63.0)) * d) + dmin)
    qb = _sb(blk[16 + sb * 16 + (item % 32) // 2])
    q = (qb & 0x0F) if item % 2 == 0 else ((qb >> 4) & 0x0F)
    return f32(f32(f32(f32(q) / f32(15.0)) * scale) + mn)


def _q4k_w_partial(blk, item, d, dmin):
    sb = item // 32
    sc = _sb(blk[4 + sb])
    scale = f32(f32(f32(sc & 0x3F) / f32(63.0)) * d)
    qb = _sb(blk[16 + sb * 16 + (item % 32) // 2])
    q = (qb & 0x0F) if (item % 32) % 2 == 0 else ((qb >> 4) & 0x0F)
    return f32(f32(f32(f32(q) / f32(15.0)) * scale) + dmin)


def weight(qt, raw, blk_index, item, full):
    blk = raw[blk_index * BB[qt]:(blk_index + 1) * BB[qt]]
    if qt == Q2_K:
        return _q2k_w(blk, item, _h(blk, 80), _h(blk, 82))
    if qt == Q4_K:
        return (_q4k_w_full if full else _q4k_w_partial)(blk, item, _h(blk, 0), _h(blk, 2))
    d = f32(np.frombuffer(bytes(blk[0:4]), dtype=np.float32)[0])
    return f32(f32(_sb(blk[4 + item])) * d)


def dequant_row_as_read(qt, raw, row, K):
    """The weight computeMatMul's K-quant dot uses for (row, k), k < K, including the full-block
    quirk (blockIndex = (row*K + blockStart)/256, items 0..255) and the flat-index partial path."""
    w = np.zeros(K, np.float32)
    for bs in range(0, K, QK_K):
        be = min(bs + QK_K, K)
        if be - bs == QK_K:
            blk = (row * K + bs) // QK_K
            for i in range(QK_K):
                w[bs + i] = weight(qt, raw, blk, i, True)
        else:
            for k in range(bs, be):
                flat = row * K + k
                w[k] = weight(qt, raw, flat // QK_K, flat % QK_K, False)
    return w


def mat_mul_kq_ref(qt, raw, M, K, x):
    """dst[M, N] with the weights as read and an f32 left-to-right accumulation."""
    x = np.asarray(x, np.float32)
    N = x.shape[1]
    out = np.zeros((M, N), np.float32)
    for i in range(M):
        w = dequant_row_as_read(qt, raw, i, K)
        for j in range(N):
            s = f32(0)
            for k in range(K):
                s = f32(s + f32(w[k] * x[k, j]))
            out[i, j] = s
    return out
