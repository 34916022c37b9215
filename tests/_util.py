"""Shared test helpers: deterministic inputs and the parity criterion (§8c)."""
from __future__ import annotations

import numpy as np

# parity bar for F32 results: normwise ||g-r||_inf/||r||_inf <= 1e-3 AND
# per element |g-r| <= 1e-3 * max(|r|, 1e-3*||r||_inf)
REL_TOL = 1e-3


# The batched (N > 1) MFMA path splits each activation as x = hi + lo in bf16, which represents
# x to within 2^-17·|x| (llama.kotlin_amd/csrc/lk_kernels.hpp, xsplit_kernel); products and
# sums are exact / f32, so its outputs are within 2^-17·Σ_k |w_ik|·|x_kj| of the exact product.
SPLIT_REL = 2.0 ** -17


def acc_noise(w_abs: np.ndarray, x_abs: np.ndarray, split: bool = False) -> np.ndarray:
    """Per-element allowance for the f32 accumulation noise of the reference's own sequential
    sum (and ours): 4·sqrt(K)·2^-24·Σ_k |w_ik|·|x_kj|. The reference (oracle) itself deviates
    from the exact product by up to ~3.6e-6·||r||_inf at K = 11008 (measured), which exceeds
    the fixed 1e-6·||r||_inf floor below on small outputs. split=True adds the bound of the
    batched path's activation split (SPLIT_REL·Σ|w||x|)."""
    K = w_abs.shape[1]
    s = w_abs.astype(np.float64) @ x_abs.astype(np.float64)
    return (4.0 * np.sqrt(K) * 2.0 ** -24 + (SPLIT_REL if split else 0.0)) * s


def parity_ok(g: np.ndarray, r: np.ndarray, rel: float = REL_TOL, noise: np.ndarray | None = None) -> tuple[bool, str]:
    g = np.asarray(g, np.float64)
    r = np.asarray(r, np.float64)
    if g.shape != r.shape:
        return False, f"shape {g.shape} != {r.shape}"
    if r.size == 0:
        return True, "empty"
    nan_r, nan_g = np.isnan(r), np.isnan(g)
    if not np.array_equal(nan_r, nan_g):
        return False, "NaN pattern differs"
    m = ~nan_r
    if not m.any():
        return True, "all NaN"
    g, r = g[m], r[m]
    inf = np.isinf(r)
    if not np.array_equal(r[inf], g[inf]):
        return False, "Inf pattern differs"
    g, r = g[~inf], r[~inf]
    if r.size == 0:
        return True, "all inf"
    rmax = np.max(np.abs(r))
    err = np.abs(g - r)
    normwise = err.max() / rmax if rmax > 0 else err.max()
    floor = rel * np.maximum(np.abs(r), rel * rmax)
    if noise is not None:
        floor = np.maximum(floor, np.asarray(noise, np.float64)[m][~inf])
    worst = np.max(err / np.maximum(floor, 1e-300)) if rmax > 0 else (0.0 if err.max() == 0 else np.inf)
    ok = (normwise <= rel) and bool(np.all(err <= floor)) if rmax > 0 else err.max() == 0
    return bool(ok), f"normwise={normwise:.3e} worst_elem_ratio={worst:.3f}"


def pattern_f32(n: int, seed: int) -> np.ndarray:
    """GGMLMatMulBenchmarkTest.kt:51-56: ((s+idx)%127 - 63)/10."""
    idx = np.arange(n, dtype=np.int64)
    return (((seed + idx) % 127 - 63).astype(np.float32) / np.float32(10.0)).astype(np.float32)


def pattern_src(qtype: int, n: int, seed: int) -> np.ndarray:
    """GGMLMatMulBenchmarkTest.kt:57-82 source values per quant type."""
    idx = np.arange(n, dtype=np.int64)
    if qtype == 6:  # Q8_0
        return ((seed + idx) % 254 - 127).astype(np.float32)
    if qtype == 2:  # Q4_0
        return ((seed + idx) % 16 - 8).astype(np.float32)
    if qtype == 3:  # Q4_1
        return ((seed + idx) % 20).astype(np.float32)
    return pattern_f32(n, seed)


def random_weights(n: int, seed: int = 0x5EED, std: float = 0.02) -> np.ndarray:
    return (np.random.default_rng(seed).standard_normal(n) * std).astype(np.float32)


def random_acts(n: int, seed: int = 0x5EED + 1) -> np.ndarray:
    return np.random.default_rng(seed).standard_normal(n).astype(np.float32)
