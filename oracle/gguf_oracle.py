"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of GGUF parsing, writing and
the upstream→llama.kotlin Q4 nibble repack. The checker for liblk_hip's GGUF
loader (llama.kotlin_amd/csrc/lk_gguf.cpp); the product never imports it.

Follows (paths under /root/reference):
  parse()           src/nativeMain/kotlin/ai/solace/llamakotlin/gguf/GGUFParser.kt:19-201
                    (header, readKeyValue :58-84, readTensorInfo :86-100, readArray
                    :102-126, alignOffset :199-201); tensor type ids decoded either as
                    upstream ggml_type (ggml/include/ggml.h:361-395) or, kotlin_ids=True,
                    as GGMLType.fromValue (core/GGMLTypes.kt:145-168) like GGUFParser.kt:93
  write_gguf()      the byte layout TestGGUFGenerator produces
                    (src/nativeTest/kotlin/ai/solace/llamakotlin/gguf/TestGGUFGenerator.kt:12-88)
  upstream_dequant  ggml/src/ggml-quants.c:1515-1553 (dequantize_row_q4_0 / _q4_1) and the
                    block_q8_0 layout (ggml/src/ggml-common.h:187-191)
  repack_to_kotlin  weight j low / j+16 high (upstream) -> 2j low / 2j+1 high
                    (core/GGMLTypes.kt:647-651)

Parity pinning: the reference's own GGUF known-answer tests (GGUFTest.kt,
GGUFIntegrationTest.kt) over TestGGUFGenerator's file, and the GGUF files the reference
ships under models/ (vocab-only, real llama.cpp output). Building the vendored upstream
ggml as a second oracle was denied in this environment ("Oracle").
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = b"GGUF"
DEFAULT_ALIGNMENT = 32

# GGUFType (gguf/GGUFTypes.kt:6-20)
UINT8, INT8, UINT16, INT16, UINT32, INT32, FLOAT32, BOOL, STRING, ARRAY, UINT64, INT64, FLOAT64 = range(13)
_SCALAR = {UINT8: "<B", INT8: "<b", UINT16: "<H", INT16: "<h", UINT32: "<I", INT32: "<i", FLOAT32: "<f",
           BOOL: "<?", UINT64: "<Q", INT64: "<q", FLOAT64: "<d"}

# upstream ggml_type id -> (lk_type or None, block weights, block bytes)
UPSTREAM_TYPES = {
    0: (0, 1, 4), 1: (1, 1, 2), 2: (2, 32, 18), 3: (3, 32, 20), 6: (4, 32, 22), 7: (5, 32, 24),
    8: (6, 32, 34), 9: (7, 32, 36), 10: (8, 256, 84), 11: (9, 256, 110), 12: (10, 256, 144),
    13: (11, 256, 176), 14: (12, 256, 210), 15: (13, 256, 292), 16: (None, 256, 66), 17: (None, 256, 74),
    18: (None, 256, 98), 19: (None, 256, 50), 20: (None, 32, 18), 21: (None, 256, 110), 22: (None, 256, 82),
    23: (None, 256, 136), 24: (15, 1, 1), 25: (16, 1, 2), 26: (17, 1, 4), 27: (18, 1, 8), 28: (None, 1, 8),
    29: (None, 256, 56), 30: (None, 1, 2), 31: (None, 32, 18), 32: (None, 32, 18), 33: (None, 32, 18),
}
# GGMLType.fromValue id -> (lk_type, block weights, block bytes)
KOTLIN_TYPES = {
    0: (0, 1, 4), 1: (1, 1, 2), 2: (2, 32, 18), 3: (3, 32, 20), 4: (4, 32, 22), 5: (5, 32, 24), 6: (6, 32, 34),
    7: (7, 32, 36), 8: (8, 256, 84), 9: (9, 256, 110), 10: (10, 256, 144), 11: (11, 256, 176),
    12: (12, 256, 210), 13: (13, 256, 292), 14: (14, 1, 0), 15: (15, 1, 1), 16: (16, 1, 2), 17: (17, 1, 4),
    18: (18, 1, 8),
}
# upstream ids of the Kotlin hot-path types
GGML_Q4_0, GGML_Q4_1, GGML_Q8_0 = 2, 3, 8


class GGUFError(Exception):
    def __init__(self, kind: str, msg: str):
        super().__init__(msg)
        self.kind = kind  # "IllegalArgument" | "IndexOutOfBounds"


class _R:
    def __init__(self, data: bytes):
        self.d = data
        self.p = 0

    def take(self, n: int) -> bytes:
        if n < 0 or self.p + n > len(self.d):
            raise GGUFError("IndexOutOfBounds", f"read of {n} at {self.p} exceeds {len(self.d)}")
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def scalar(self, t: int):
        f = _SCALAR[t]
        return struct.unpack(f, self.take(struct.calcsize(f)))[0]

    def string(self) -> str:
        n = self.scalar(UINT64)
        return self.take(n).decode("utf-8", errors="replace")  # Kotlin decodeToString


def _value(r: _R, t: int):
    if t == STRING:
        return r.string()
    if t == ARRAY:
        et = r.scalar(UINT32)
        if et not in _SCALAR and et != STRING:
            raise GGUFError("IllegalArgument", f"Unknown GGUF type: {et}")
        if et == ARRAY:
            raise GGUFError("IllegalArgument", "Nested arrays not supported")
        n = r.scalar(UINT64)
        return (et, [_value(r, et) for _ in range(n)])
    if t not in _SCALAR:
        raise GGUFError("IllegalArgument", f"Unknown GGUF type: {t}")
    return r.scalar(t)


def parse(data: bytes, kotlin_ids: bool = False) -> dict:
    """GGUFParser.parse: returns {version, metadata{key: (type, value)}, tensors[...], alignment, data_offset}."""
    r = _R(data)
    magic = r.take(4)
    if magic != MAGIC:
        raise GGUFError("IllegalArgument", f"Invalid GGUF magic: {magic!r}")
    version = r.scalar(UINT32)
    if version < 2:
        raise GGUFError("IllegalArgument", f"unsupported GGUF version {version}")
    n_t, n_kv = r.scalar(UINT64), r.scalar(UINT64)
    meta: dict = {}
    for _ in range(n_kv):
        key = r.string()
        t = r.scalar(UINT32)
        if t not in _SCALAR and t not in (STRING, ARRAY):
            raise GGUFError("IllegalArgument", f"Unknown GGUF type: {t}")
        meta[key] = (t, _value(r, t))  # dict: last value wins, first position kept
    table = KOTLIN_TYPES if kotlin_ids else UPSTREAM_TYPES
    tensors = []
    for _ in range(n_t):
        name = r.string()
        nd = r.scalar(UINT32)
        if not 1 <= nd <= 4:
            raise GGUFError("IllegalArgument", f"Unsupported tensor dimension count: {nd}")
        dims = [r.scalar(UINT64) for _ in range(nd)]
        nel = 1
        for v in dims:
            if v > 1 << 40 or (v and nel > (1 << 62) // v):
                raise GGUFError("IllegalArgument", f"{name}: dimension overflow")
            nel *= v
        ft = r.scalar(UINT32)
        if ft not in table:
            raise GGUFError("IllegalArgument", f"Unknown tensor type: {ft}")
        lk, blck, bb = table[ft]
        if dims[0] % blck:
            raise GGUFError("IllegalArgument", f"{name}: ne[0] not a multiple of {blck}")
        off = r.scalar(UINT64)
        if off > len(data):
            raise GGUFError("IndexOutOfBounds", f"{name}: offset beyond file")
        tensors.append(dict(name=name, dims=dims, file_type=ft, type=lk if lk is not None else -1,
                            repack=int(not kotlin_ids and ft in (GGML_Q4_0, GGML_Q4_1)),
                            offset=off, bytes=nel // blck * bb))
    alignment = DEFAULT_ALIGNMENT
    if "general.alignment" in meta:
        t, v = meta["general.alignment"]
        if t in (UINT8, INT8, UINT16, INT16, UINT32, INT32, UINT64, INT64):
            if v <= 0 or v > 1 << 62 or v & (v - 1):
                raise GGUFError("IllegalArgument", f"general.alignment {v} is not a power of two")
            alignment = v
    data_offset = (r.p + alignment - 1) // alignment * alignment
    return dict(version=version, metadata=meta, tensors=tensors, alignment=alignment, data_offset=data_offset,
                data_bytes=max([t["offset"] + t["bytes"] for t in tensors], default=0))


# -- writer ------------------------------------------------------------------

def _w_str(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    return struct.pack("<Q", len(b)) + b


def _w_value(t: int, v) -> bytes:
    if t == STRING:
        return _w_str(v)
    if t == ARRAY:
        et, items = v
        return struct.pack("<IQ", et, len(items)) + b"".join(_w_value(et, x) for x in items)
    return struct.pack(_SCALAR[t], v)


def write_gguf(metadata: list, tensors: list, version: int = 3, alignment: int = 32, pad_data: bool = True) -> bytes:
    """metadata: [(key, type, value)], tensors: [(name, dims, file_type, offset, payload bytes)].

    Header/KV/tensor-info layout as TestGGUFGenerator.kt:14-58, padded to `alignment`
    (:60-66), then each payload at data_offset + offset (zero gaps)."""
    out = bytearray(MAGIC + struct.pack("<IQQ", version, len(tensors), len(metadata)))
    for key, t, v in metadata:
        out += _w_str(key) + struct.pack("<I", t) + _w_value(t, v)
    for name, dims, ft, off, _ in tensors:
        out += _w_str(name) + struct.pack("<I", len(dims)) + b"".join(struct.pack("<Q", d) for d in dims)
        out += struct.pack("<IQ", ft, off)
    out += b"\0" * ((alignment - len(out) % alignment) % alignment)
    base = len(out)
    for _, _, _, off, payload in tensors:
        end = base + off + len(payload)
        if len(out) < end:
            out += b"\0" * (end - len(out))
        out[base + off:end] = payload
    if pad_data:
        out += b"\0" * ((alignment - len(out) % alignment) % alignment)
    return bytes(out)


def reference_test_file() -> bytes:
    """TestGGUFGenerator.generateTestFile (TestGGUFGenerator.kt:12-81): v3, 3 KVs, two F32
    tensors weight.0 [2,2] @0 = [1,2,3,4] and weight.1 [3,3] @16 = identity."""
    w0 = np.array([1, 2, 3, 4], np.float32).tobytes()
    w1 = np.eye(3, dtype=np.float32).reshape(-1).tobytes()
    return write_gguf(
        [("general.architecture", STRING, "test"), ("general.name", STRING, "test-model"),
         ("general.alignment", UINT64, 32)],
        [("weight.0", [2, 2], 0, 0, w0), ("weight.1", [3, 3], 0, 16, w1)], pad_data=False)


# -- upstream block semantics and the repack ---------------------------------

def _f16(b: np.ndarray) -> np.ndarray:
    return b.copy().view("<f2").astype(np.float32)


def upstream_dequant(ft: int, raw: bytes, n: int) -> np.ndarray:
    """dequantize_row_q4_0 / _q4_1 (ggml-quants.c:1515-1553) and q8_0 (d * q), in f32
    with one rounding per operation (mul, then add for Q4_1)."""
    bb = {GGML_Q4_0: 18, GGML_Q4_1: 20, GGML_Q8_0: 34}[ft]
    blk = np.frombuffer(raw, np.uint8)[: n // 32 * bb].reshape(-1, bb)
    d = _f16(blk[:, 0:2]).reshape(-1, 1)
    if ft == GGML_Q8_0:
        q = blk[:, 2:].view(np.int8).astype(np.float32)
        return (d * q).astype(np.float32).reshape(-1)
    qs = blk[:, 4:] if ft == GGML_Q4_1 else blk[:, 2:]
    w = np.concatenate([qs & 0xF, qs >> 4], axis=1).astype(np.float32)  # weight j, weight j+16
    if ft == GGML_Q4_0:
        return (d * (w - 8.0)).astype(np.float32).reshape(-1)
    m = _f16(blk[:, 2:4]).reshape(-1, 1)
    return ((d * w).astype(np.float32) + m).astype(np.float32).reshape(-1)


def repack_to_kotlin(ft: int, raw: bytes) -> bytes:
    """Upstream Q4_0/Q4_1 blocks -> llama.kotlin nibble order; other types unchanged."""
    if ft not in (GGML_Q4_0, GGML_Q4_1):
        return bytes(raw)
    bb, q0 = (18, 2) if ft == GGML_Q4_0 else (20, 4)
    blk = np.frombuffer(raw, np.uint8).reshape(-1, bb).copy()
    qs = blk[:, q0:]
    w = np.concatenate([qs & 0xF, qs >> 4], axis=1)  # w[:, k] = weight k
    blk[:, q0:] = (w[:, 0::2] | (w[:, 1::2] << 4)).astype(np.uint8)
    return blk.tobytes()


def upstream_quantize(ft: int, x: np.ndarray, seed: int = 0) -> bytes:
    """Synthetic upstream-layout blocks for x (valid scales, codes from x): the test
    inputs for the loader. Not a restatement of upstream quantize (unneeded: the loader
    is checked on the bytes it is given, whatever produced them)."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    nb = x.shape[0]
    if ft == GGML_Q8_0:
        amax = np.abs(x).max(axis=1)
        d = (amax / 127).astype(np.float16)
        inv = np.where(d != 0, 1 / d.astype(np.float32), 0).reshape(-1, 1)
        q = np.clip(np.rint(x * inv), -127, 127).astype(np.int8)
        return b"".join(d[i].tobytes() + q[i].tobytes() for i in range(nb))
    if ft == GGML_Q4_0:
        amax_i = np.abs(x).argmax(axis=1)
        mx = x[np.arange(nb), amax_i]
        d = (mx / -8).astype(np.float16)
        inv = np.where(d != 0, 1 / d.astype(np.float32), 0).reshape(-1, 1)
        q = np.clip(np.floor(x * inv + 8.5), 0, 15).astype(np.uint8)
        qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8)
        return b"".join(d[i].tobytes() + qs[i].tobytes() for i in range(nb))
    mn, mx = x.min(axis=1), x.max(axis=1)
    d = ((mx - mn) / 15).astype(np.float16)
    m = mn.astype(np.float16)
    inv = np.where(d != 0, 1 / d.astype(np.float32), 0).reshape(-1, 1)
    q = np.clip(np.floor((x - mn.reshape(-1, 1)) * inv + 0.5), 0, 15).astype(np.uint8)
    qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8)
    return b"".join(d[i].tobytes() + m[i].tobytes() + qs[i].tobytes() for i in range(nb))
