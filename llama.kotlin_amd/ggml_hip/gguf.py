"""GGUF loading for the MUL_MAT path: the reference's gguf package over liblk_hip's parser.

Mirrors (paths relative to src/nativeMain/kotlin/ai/solace/llamakotlin/):
  GGUFType / GGUFKeyValue / GGUFTensorInfo / GGUFConstants   gguf/GGUFTypes.kt:6-75
  GGUFParser(data).parse()                                    gguf/GGUFParser.kt:13-56
  GGUFContext (typed getters, findTensor, getTensorData)       gguf/GGUFContext.kt:6-152
  ModelLoader.loadFromBytes / loadFromFile                      gguf/ModelLoader.kt:6-25
  LoadedModel.getTensor / getTensorNames / getModelInfo         gguf/ModelLoader.kt:30-158

Parsing, bounds checks and the nibble repack run in the C-ABI (include/lk_gguf.h); this
module only shapes the results like the Kotlin classes. Differences from the reference,
all deliberate (see lk_gguf.h):
  * tensor type ids are upstream ggml_type by default (real llama.cpp files);
    ``kotlinIds=True`` reproduces GGMLType.fromValue;
  * getTensor loads every type llama.kotlin names, not F32 only, and Q4_0/Q4_1 land in
    llama.kotlin's nibble order (repacked on the GPU), so computeMatMul reads them as is;
  * loadFromFile memory-maps the file (the reference's is a stub);
  * LoadedModel.loadResident puts the whole data section in one HBM buffer (graph residency).
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import IllegalArgumentException, NotOffloadedError
from .tensor import GGMLGraphAllocator, GGMLTensor, GGMLType

KOTLIN_IDS = 1


class GGUFType(enum.IntEnum):
    """gguf/GGUFTypes.kt:6-20."""

    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


class GGUFConstants:
    MAGIC = "GGUF"
    DEFAULT_ALIGNMENT = 32


_NP = {GGUFType.UINT8: "<u1", GGUFType.INT8: "<i1", GGUFType.UINT16: "<u2", GGUFType.INT16: "<i2",
       GGUFType.UINT32: "<u4", GGUFType.INT32: "<i4", GGUFType.FLOAT32: "<f4", GGUFType.BOOL: "<u1",
       GGUFType.UINT64: "<u8", GGUFType.INT64: "<i8", GGUFType.FLOAT64: "<f8"}
_INTS = (GGUFType.UINT8, GGUFType.INT8, GGUFType.UINT16, GGUFType.INT16, GGUFType.UINT32, GGUFType.INT32,
         GGUFType.UINT64, GGUFType.INT64)


@dataclass
class GGUFKeyValue:
    """gguf/GGUFTypes.kt:25-29. ``arrayType`` is set for ARRAY values."""

    key: str
    type: GGUFType
    value: object
    arrayType: GGUFType | None = None


@dataclass
class GGUFTensorInfo:
    """gguf/GGUFTypes.kt:33-54 plus the stored size, file type id and repack flag."""

    name: str
    dimensions: list
    type: GGMLType | None
    offset: int
    fileType: int = 0
    nbytes: int = 0
    repack: bool = False
    index: int = field(default=-1, repr=False)


class LkGgufTensorInfo(ctypes.Structure):
    """``lk_gguf_tensor_info`` (include/lk_gguf.h)."""

    _fields_ = [
        ("name", ctypes.c_char_p),
        ("n_dims", ctypes.c_int32),
        ("file_type", ctypes.c_int32),
        ("type", ctypes.c_int32),
        ("repack", ctypes.c_int32),
        ("ne", ctypes.c_int64 * 4),
        ("offset", ctypes.c_uint64),
        ("bytes", ctypes.c_uint64),
    ]


def _decode(raw: bytes) -> str:
    return raw.decode("utf-8", errors="replace")  # Kotlin decodeToString replaces malformed input


class GGUFContext:
    """gguf/GGUFContext.kt:6-152, backed by an ``lk_gguf`` handle."""

    def __init__(self, handle, keepalive=None):
        self._h = handle
        self._keep = keepalive  # the borrowed image (loadFromBytes)
        L = _lib.load()
        self.version = int(L.lk_gguf_version(handle))
        self.alignment = int(L.lk_gguf_alignment(handle))
        self.dataOffset = int(L.lk_gguf_data_offset(handle))
        self.dataBytes = int(L.lk_gguf_data_bytes(handle))
        self.metadata: dict[str, GGUFKeyValue] = {}
        for i in range(int(L.lk_gguf_kv_count(handle))):
            kv = self._read_kv(L, i)
            self.metadata[kv.key] = kv
        self.tensors: list[GGUFTensorInfo] = []
        info = LkGgufTensorInfo()
        for i in range(int(L.lk_gguf_tensor_count(handle))):
            _lib.check(L.lk_gguf_get_tensor_info(handle, i, ctypes.byref(info)))
            self.tensors.append(GGUFTensorInfo(
                name=_decode(info.name), dimensions=[int(info.ne[d]) for d in range(info.n_dims)],
                type=GGMLType(info.type) if info.type >= 0 else None, offset=int(info.offset),
                fileType=int(info.file_type), nbytes=int(info.bytes), repack=bool(info.repack), index=i))

    def _read_kv(self, L, i) -> GGUFKeyValue:
        h = self._h
        key = _decode(L.lk_gguf_kv_key(h, i))
        t = GGUFType(L.lk_gguf_kv_type(h, i))
        s, n = ctypes.c_void_p(), ctypes.c_uint64()
        if t == GGUFType.STRING:
            _lib.check(L.lk_gguf_kv_get_string(h, i, -1, ctypes.byref(s), ctypes.byref(n)))
            return GGUFKeyValue(key, t, _decode(ctypes.string_at(s, n.value) if n.value else b""))
        if t == GGUFType.ARRAY:
            et, cnt = ctypes.c_int32(), ctypes.c_uint64()
            _lib.check(L.lk_gguf_kv_array_info(h, i, ctypes.byref(et), ctypes.byref(cnt)))
            et = GGUFType(et.value)
            if et == GGUFType.STRING:
                vals = []
                for e in range(cnt.value):
                    _lib.check(L.lk_gguf_kv_get_string(h, i, e, ctypes.byref(s), ctypes.byref(n)))
                    vals.append(_decode(ctypes.string_at(s, n.value) if n.value else b""))
            else:
                w = ctypes.c_uint64()
                _lib.check(L.lk_gguf_kv_array_data(h, i, ctypes.byref(s), ctypes.byref(w)))
                raw = ctypes.string_at(s, cnt.value * w.value) if cnt.value else b""
                arr = np.frombuffer(raw, _NP[et])
                vals = (arr != 0).tolist() if et == GGUFType.BOOL else arr.tolist()
            return GGUFKeyValue(key, t, vals, et)
        buf = ctypes.create_string_buffer(8)
        _lib.check(L.lk_gguf_kv_get(h, i, -1, buf, 8))
        v = np.frombuffer(buf.raw[:np.dtype(_NP[t]).itemsize], _NP[t])[0]
        return GGUFKeyValue(key, t, bool(v) if t == GGUFType.BOOL else v.item())

    # -- GGUFContext.kt:17-73 -------------------------------------------
    def getMetadataValue(self, key: str):
        kv = self.metadata.get(key)
        return None if kv is None else kv.value

    def getStringValue(self, key: str):
        kv = self.metadata.get(key)
        return kv.value if kv is not None and kv.type == GGUFType.STRING else None

    def getIntValue(self, key: str):
        v = self.getLongValue(key)
        if v is None:
            return None
        return (v + 2**31) % 2**32 - 2**31  # Kotlin toInt() truncation

    def getLongValue(self, key: str):
        kv = self.metadata.get(key)
        if kv is None or kv.type not in _INTS:
            return None
        return (kv.value + 2**63) % 2**64 - 2**63  # ULong.toLong()

    def getFloatValue(self, key: str):
        kv = self.metadata.get(key)
        if kv is None or kv.type not in (GGUFType.FLOAT32, GGUFType.FLOAT64):
            return None
        return float(np.float32(kv.value))

    def getBooleanValue(self, key: str):
        kv = self.metadata.get(key)
        return kv.value if kv is not None and kv.type == GGUFType.BOOL else None

    # -- GGUFContext.kt:78-95 -------------------------------------------
    def findTensor(self, name: str) -> GGUFTensorInfo | None:
        i = int(_lib.load().lk_gguf_find_tensor(self._h, name.encode()))
        return None if i < 0 else self.tensors[i]

    def getTensorData(self, info: GGUFTensorInfo) -> bytes:
        """The stored bytes (file layout), bounds-checked (IndexOutOfBoundsException)."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        _lib.check(_lib.load().lk_gguf_tensor_data(self._h, info.index, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p, n.value) if n.value else b""

    def getArchitecture(self):
        return self.getStringValue("general.architecture")

    def getModelName(self):
        return self.getStringValue("general.name")

    def printSummary(self):
        """GGUFContext.kt:122-152."""
        print("GGUF Model Summary:")
        print(f"  Version: {self.version}")
        print(f"  Architecture: {self.getArchitecture() or 'unknown'}")
        print(f"  Model Name: {self.getModelName() or 'unknown'}")
        print(f"  Tensors: {len(self.tensors)}")
        print(f"  Data Offset: {self.dataOffset}")
        print(f"  Alignment: {self.alignment}")
        print(f"\nMetadata ({len(self.metadata)} entries):")
        for k in sorted(self.metadata)[:10]:
            v = self.metadata[k].value
            vs = f'"{v}"' if isinstance(v, str) else (f"[{len(v)} items]" if isinstance(v, list) else str(v))
            print(f"  {k}: {vs}")
        if len(self.metadata) > 10:
            print(f"  ... and {len(self.metadata) - 10} more")
        print(f"\nTensors ({len(self.tensors)} entries):")
        for t in self.tensors[:10]:
            tn = t.type.name if t.type is not None else f"ggml_type {t.fileType}"
            print(f"  {t.name}: {tn} [{'×'.join(map(str, t.dimensions))}] @ {t.offset}")
        if len(self.tensors) > 10:
            print(f"  ... and {len(self.tensors) - 10} more")

    def close(self):
        if self._h:
            _lib.load().lk_gguf_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GGUFParser:
    """gguf/GGUFParser.kt:13: ``GGUFParser(data).parse()``."""

    def __init__(self, data: bytes, kotlinIds: bool = False):
        self.data = bytes(data)
        self.flags = KOTLIN_IDS if kotlinIds else 0

    def parse(self) -> GGUFContext:
        L = _lib.load()
        h = ctypes.c_void_p()
        buf = ctypes.c_char_p(self.data)  # borrowed: the context keeps self.data alive
        _lib.check(L.lk_gguf_open_memory(buf, len(self.data), self.flags, ctypes.byref(h)))
        return GGUFContext(h, keepalive=(self.data, buf))


class LoadedModel:
    """gguf/ModelLoader.kt:30-158."""

    def __init__(self, ggufContext: GGUFContext):
        self.ggufContext = ggufContext
        self._cache: dict[str, GGMLTensor] = {}
        self._resident: dict[int, int] = {}  # id(allocator) -> bufferId holding the data section

    def getTensorNames(self) -> list[str]:
        return [t.name for t in self.ggufContext.tensors]

    def getModelInfo(self) -> str:
        c = self.ggufContext
        return (f"Model: {c.getModelName() or 'Unknown'}\nArchitecture: {c.getArchitecture() or 'Unknown'}\n"
                f"Tensors: {len(c.tensors)}\nVersion: {c.version}\n")

    def loadResident(self, graphAllocator: GGMLGraphAllocator) -> int:
        """Copy the whole data section into one new device buffer of graphAllocator and
        repack every upstream Q4 tensor in place; later getTensor calls on that
        allocator return views into it. Returns the buffer id."""
        ga = graphAllocator
        if ga.device == "host":
            raise IllegalArgumentException("loadResident needs a device allocator")
        key = id(ga)
        if key in self._resident:
            return self._resident[key]
        c = self.ggufContext
        bid = ga.addBuffer(max(c.dataBytes, 1))
        from .ops import _OnStream
        with _OnStream(None) as sh:
            _lib.check(_lib.load().lk_gguf_load_all_device(c._h, ctypes.c_void_p(ga.dataPtr(bid)),
                                                             ga.bufferSize(bid), ctypes.c_void_p(sh)))
        ga._tops[bid] = c.dataBytes
        self._resident[key] = bid
        return bid

    def getTensor(self, name: str, graphAllocator: GGMLGraphAllocator) -> GGMLTensor | None:
        """ModelLoader.kt:40-48: cached per name; None if the file has no such tensor."""
        ga = graphAllocator
        key = (name, id(ga))
        if key in self._cache:
            return self._cache[key]
        info = self.ggufContext.findTensor(name)
        if info is None:
            return None
        t = self._create(info, ga)
        self._cache[key] = t
        return t

    def _create(self, info: GGUFTensorInfo, ga: GGMLGraphAllocator) -> GGMLTensor:
        if info.type is None:
            raise NotOffloadedError(f"tensor {info.name}: ggml_type {info.fileType} has no llama.kotlin GGMLType")
        if len(info.dimensions) not in (1, 2, 3, 4):  # ModelLoader.kt:61-67
            raise IllegalArgumentException(f"Unsupported tensor dimension count: {len(info.dimensions)}")
        bid = self._resident.get(id(ga))
        if bid is not None:
            return GGMLTensor(info.type, info.dimensions, name=info.name, bufferId=bid, dataOffset=info.offset)
        t = ga.allocateTensor(info.type, info.dimensions, name=info.name, nbytes=info.nbytes)
        L = _lib.load()
        ptr = ctypes.c_void_p(ga.dataPtr(t.bufferId) + t.dataOffset)
        room = ga.bufferSize(t.bufferId) - t.dataOffset
        if ga.device == "host":
            _lib.check(L.lk_gguf_load_tensor(self.ggufContext._h, info.index, ptr, room, 0, None))
        else:
            from .ops import _OnStream
            with _OnStream(None) as sh:
                _lib.check(L.lk_gguf_load_tensor(self.ggufContext._h, info.index, ptr, room, 1, ctypes.c_void_p(sh)))
        return t


class ModelLoader:
    """gguf/ModelLoader.kt:6-25."""

    def __init__(self, kotlinIds: bool = False):
        self.flags = KOTLIN_IDS if kotlinIds else 0

    def loadFromFile(self, filePath: str) -> LoadedModel:
        L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(L.lk_gguf_open_file(str(filePath).encode(), self.flags, ctypes.byref(h)))
        return LoadedModel(GGUFContext(h))

    def loadFromBytes(self, data: bytes) -> LoadedModel:
        return LoadedModel(GGUFParser(data, kotlinIds=bool(self.flags)).parse())


def repackQ4(ga: GGMLGraphAllocator, t: GGMLTensor, toKotlin: bool = True, stream=None):
    """In-place nibble-order conversion of a device Q4_0/Q4_1 tensor (lk_repack_q4_device)."""
    if ga.device == "host":
        raise IllegalArgumentException("repackQ4 needs a device tensor")
    from .ops import _OnStream
    nblk = t.numElements() // 32
    with _OnStream(stream) as sh:
        _lib.check(_lib.load().lk_repack_q4_device(ctypes.c_void_p(ga.dataPtr(t.bufferId) + t.dataOffset), nblk,
                                                   int(t.type), 0 if toKotlin else 1, ctypes.c_void_p(sh)))
