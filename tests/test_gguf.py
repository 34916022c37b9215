"""GGUF parsing and host-side loading (no GPU): liblk_hip's parser (include/lk_gguf.h)
through the Python mirror ggml_hip.gguf, checked against

  * the reference's own GGUF known-answer tests — GGUFTest.kt and GGUFIntegrationTest.kt
    (src/nativeTest/kotlin/ai/solace/llamakotlin/gguf/) over TestGGUFGenerator's file,
    which oracle/gguf_oracle.reference_test_file() reproduces byte for byte;
  * the GGUF files the reference ships (models/ggml-vocab-*.gguf, real llama.cpp output),
    parsed by the oracle restatement, when /root/reference is present;
  * the oracle on synthetic files with every value type and the quantized tensor types,
    and on truncated/corrupted images (same error class, or both succeed identically).
"""
import glob
import os
import struct

import numpy as np
import pytest

import gguf_oracle as GO

REF_MODELS = "/root/reference/models"


def _parse(data, kotlin_ids=False):
    from ggml_hip.gguf import GGUFParser
    return GGUFParser(data, kotlinIds=kotlin_ids).parse()


# --------------------------------------------------------------------------
# GGUFTest.kt / GGUFIntegrationTest.kt, assertion for assertion
# --------------------------------------------------------------------------

@pytest.fixture(scope="module")
def ref_file():
    return GO.reference_test_file()


def test_reference_file_layout(ref_file):
    # TestGGUFGenerator.kt: 24 B header, 3 KVs (44+42+37 B), 2 tensor infos (48 B each)
    # = 243 B, zero-padded to 256, then 16 + 36 B of F32 data.
    assert len(ref_file) == 308
    assert ref_file[:4] == b"GGUF" and ref_file[243:256] == b"\0" * 13
    assert struct.unpack("<4f", ref_file[256:272]) == (1.0, 2.0, 3.0, 4.0)


def test_gguf_parsing_basic(ref_file):  # GGUFTest.testGGUFParsingBasic
    c = _parse(ref_file)
    assert c.version == 3
    assert len(c.tensors) == 2
    assert len(c.metadata) == 3


def test_gguf_metadata(ref_file):  # GGUFTest.testGGUFMetadata
    c = _parse(ref_file)
    assert c.getStringValue("general.architecture") == "test"
    assert c.getStringValue("general.name") == "test-model"
    assert c.getLongValue("general.alignment") == 32


def test_gguf_tensors(ref_file):  # GGUFTest.testGGUFTensors
    from ggml_hip import GGMLType
    c = _parse(ref_file)
    t0 = c.findTensor("weight.0")
    assert t0 is not None and t0.name == "weight.0" and t0.type == GGMLType.F32
    assert t0.dimensions == [2, 2] and t0.offset == 0
    t1 = c.findTensor("weight.1")
    assert t1 is not None and t1.name == "weight.1" and t1.type == GGMLType.F32
    assert t1.dimensions == [3, 3] and t1.offset == 16
    assert c.findTensor("weight.2") is None


def test_gguf_tensor_data(ref_file):  # GGUFTest.testGGUFTensorData
    c = _parse(ref_file)
    data = c.getTensorData(c.findTensor("weight.0"))
    assert len(data) == 16
    assert struct.unpack("<4f", data) == (1.0, 2.0, 3.0, 4.0)
    assert len(c.getTensorData(c.findTensor("weight.1"))) == 36  # testTensorMetadataExtraction


def test_model_loader(ref_file):  # GGUFTest.testModelLoader
    from ggml_hip.gguf import ModelLoader
    m = ModelLoader().loadFromBytes(ref_file)
    info = m.getModelInfo()
    assert "test-model" in info and "test" in info
    names = m.getTensorNames()
    assert len(names) == 2 and "weight.0" in names and "weight.1" in names


def test_model_loader_tensor_creation(ref_file):  # GGUFTest.testModelLoaderTensorCreation + integration
    from ggml_hip import GGMLGraphAllocator, GGMLType
    from ggml_hip.gguf import ModelLoader
    m = ModelLoader().loadFromBytes(ref_file)
    ga = GGMLGraphAllocator(device="host", defaultBufferSize=1024)
    t = m.getTensor("weight.0", ga)
    assert t is not None and t.name == "weight.0" and t.type == GGMLType.F32
    assert t.ne[0] == 2 and t.ne[1] == 2
    assert [t.getFloat(ga, i, j) for j in range(2) for i in range(2)] == [1.0, 2.0, 3.0, 4.0]
    assert m.getTensor("weight.0", ga) is t  # tensorCache (ModelLoader.kt:40-48)
    t1 = m.getTensor("weight.1", ga)
    assert t1.ne[:2] == [3, 3]
    vals = np.frombuffer(ga.tensorBytes(t1), np.float32)
    assert vals.size == 9 and vals[0] == vals[4] == vals[8] == 1.0 and vals.sum() == 3.0
    assert m.getTensor("missing", ga) is None


def test_invalid_magic():  # GGUFTest.testInvalidMagic
    from ggml_hip import IllegalArgumentException
    with pytest.raises(IllegalArgumentException):
        _parse(b"XXXX")


def test_context_print_summary(ref_file, capsys):  # GGUFTest.testContextPrintSummary
    _parse(ref_file).printSummary()
    out = capsys.readouterr().out
    assert "Version: 3" in out and "weight.1: F32 [3×3] @ 16" in out


def test_version_and_alignment(ref_file):  # GGUFIntegrationTest.testGGUFVersionAndAlignment
    c = _parse(ref_file)
    assert c.version == 3 and c.alignment == 32
    assert c.dataOffset > 0 and c.dataOffset % c.alignment == 0
    assert c.dataOffset == 256


def test_load_from_file_matches_bytes(ref_file, tmp_path):
    from ggml_hip import IllegalStateException
    from ggml_hip.gguf import ModelLoader
    p = tmp_path / "t.gguf"
    p.write_bytes(ref_file)
    m = ModelLoader().loadFromFile(str(p))
    assert m.getTensorNames() == ["weight.0", "weight.1"]
    assert m.ggufContext.getTensorData(m.ggufContext.findTensor("weight.1")) == ref_file[272:308]
    with pytest.raises(IllegalStateException):
        ModelLoader().loadFromFile(str(tmp_path / "absent.gguf"))


# --------------------------------------------------------------------------
# C++ parser == oracle restatement
# --------------------------------------------------------------------------

def _mirror_summary(c):
    meta = {}
    for k, kv in c.metadata.items():
        v = kv.value
        if kv.arrayType is not None:
            v = (int(kv.arrayType), list(v))
        meta[k] = (int(kv.type), v)
    tensors = [dict(name=t.name, dims=t.dimensions, file_type=t.fileType,
                    type=int(t.type) if t.type is not None else -1, repack=int(t.repack), offset=t.offset,
                    bytes=t.nbytes) for t in c.tensors]
    return dict(version=c.version, metadata=meta, tensors=tensors, alignment=c.alignment,
                data_offset=c.dataOffset, data_bytes=c.dataBytes)


def _same_value(t, a, b):
    if t in (GO.FLOAT32, GO.FLOAT64):
        return np.array_equal(np.asarray(a, np.float64), np.asarray(b, np.float64), equal_nan=True)
    return a == b


def _assert_same(mine, ref):
    assert mine["version"] == ref["version"]
    assert mine["alignment"] == ref["alignment"] and mine["data_offset"] == ref["data_offset"]
    assert mine["data_bytes"] == ref["data_bytes"]
    assert list(mine["metadata"]) == list(ref["metadata"])  # same keys, same (first-insertion) order
    for k, (t, v) in ref["metadata"].items():
        mt, mv = mine["metadata"][k]
        assert mt == t, k
        if t == GO.ARRAY:
            assert mv[0] == v[0] and len(mv[1]) == len(v[1]), k
            assert _same_value(v[0], mv[1], v[1]), k
        else:
            assert _same_value(t, mv, v), k
    assert mine["tensors"] == ref["tensors"]


@pytest.mark.skipif(not glob.glob(os.path.join(REF_MODELS, "*.gguf")), reason="reference models/ absent")
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(REF_MODELS, "*.gguf"))),
                         ids=lambda p: os.path.basename(p))
def test_reference_vocab_files(path):
    """Real llama.cpp GGUF v3 files shipped with the reference: every key, type and value."""
    from ggml_hip.gguf import ModelLoader
    data = open(path, "rb").read()
    m = ModelLoader().loadFromFile(path)
    _assert_same(_mirror_summary(m.ggufContext), GO.parse(data))
    c = m.ggufContext
    assert c.getArchitecture() is not None
    toks = c.getMetadataValue("tokenizer.ggml.tokens")
    assert isinstance(toks, list) and len(toks) > 1000


def _all_types_file(**kw):
    meta = [
        ("general.architecture", GO.STRING, "llama"), ("u8", GO.UINT8, 200), ("i8", GO.INT8, -5),
        ("u16", GO.UINT16, 65535), ("i16", GO.INT16, -32768), ("u32", GO.UINT32, 4000000000),
        ("i32", GO.INT32, -7), ("f32", GO.FLOAT32, 1.5), ("b", GO.BOOL, True), ("b0", GO.BOOL, False),
        ("u64", GO.UINT64, 2**64 - 1), ("i64", GO.INT64, -(2**62)), ("f64", GO.FLOAT64, 0.1),
        ("empty", GO.STRING, ""), ("utf8", GO.STRING, "ñ→€"),
        ("arr.f32", GO.ARRAY, (GO.FLOAT32, [0.5, -2.0, 3.25])), ("arr.i32", GO.ARRAY, (GO.INT32, [1, -2, 3])),
        ("arr.str", GO.ARRAY, (GO.STRING, ["a", "", "xyz"])), ("arr.empty", GO.ARRAY, (GO.UINT8, [])),
        ("arr.bool", GO.ARRAY, (GO.BOOL, [True, False, True])), ("arr.u64", GO.ARRAY, (GO.UINT64, [2**63])),
        ("general.alignment", GO.UINT32, 64),
    ]
    rng = np.random.default_rng(11)
    tensors = []
    off = 0

    def add(name, dims, ft, nbytes):
        nonlocal off
        payload = rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes()
        tensors.append((name, dims, ft, off, payload))
        off = (off + nbytes + 63) // 64 * 64

    add("tok_embd.weight", [64, 3], 0, 64 * 3 * 4)          # F32
    add("norm.weight", [64], 1, 64 * 2)                      # F16
    add("blk.0.attn_q.weight", [128, 5], 2, 4 * 5 * 18)       # Q4_0 (upstream id 2)
    add("blk.0.ffn_up.weight", [96, 4], 3, 3 * 4 * 20)        # Q4_1
    add("blk.0.ffn_down.weight", [64, 7], 8, 2 * 7 * 34)      # Q8_0 (upstream id 8)
    add("blk.0.q6k", [256, 2], 14, 2 * 210)                   # Q6_K
    add("blk.0.bf16", [4, 4], 30, 32)                         # BF16: no llama.kotlin type
    add("t3d", [32, 2, 3], 2, 6 * 18)                         # 3-D Q4_0
    add("t4d", [32, 1, 2, 2], 8, 4 * 34)                      # 4-D Q8_0
    return GO.write_gguf(meta, tensors, alignment=64, **kw)


def test_all_value_types_and_tensor_types_match_oracle():
    data = _all_types_file()
    c = _parse(data)
    _assert_same(_mirror_summary(c), GO.parse(data))
    # typed getters (GGUFContext.kt:17-73)
    assert c.getIntValue("u8") == 200 and c.getIntValue("i8") == -5 and c.getIntValue("u32") == -294967296
    assert c.getLongValue("u32") == 4000000000 and c.getLongValue("u64") == -1  # ULong.toLong()
    assert c.getLongValue("f32") is None and c.getFloatValue("u8") is None
    assert c.getFloatValue("f32") == 1.5 and c.getFloatValue("f64") == np.float32(0.1)
    assert c.getBooleanValue("b") is True and c.getBooleanValue("b0") is False and c.getBooleanValue("u8") is None
    assert c.getStringValue("utf8") == "ñ→€" and c.getStringValue("empty") == "" and c.getStringValue("u8") is None
    assert c.getMetadataValue("arr.str") == ["a", "", "xyz"] and c.getMetadataValue("arr.bool") == [True, False, True]
    assert c.getMetadataValue("arr.u64") == [2**63] and c.getMetadataValue("arr.empty") == []
    assert c.alignment == 64 and c.dataOffset % 64 == 0
    from ggml_hip import GGMLType
    by = {t.name: t for t in c.tensors}
    assert by["blk.0.attn_q.weight"].type == GGMLType.Q4_0 and by["blk.0.attn_q.weight"].repack
    assert by["blk.0.ffn_up.weight"].type == GGMLType.Q4_1 and by["blk.0.ffn_up.weight"].repack
    assert by["blk.0.ffn_down.weight"].type == GGMLType.Q8_0 and not by["blk.0.ffn_down.weight"].repack
    assert by["blk.0.q6k"].type == GGMLType.Q6_K and by["blk.0.q6k"].nbytes == 420
    assert by["blk.0.bf16"].type is None and by["blk.0.bf16"].fileType == 30
    assert by["t3d"].dimensions == [32, 2, 3] and by["t4d"].dimensions == [32, 1, 2, 2]


def test_kotlin_ids_reading():
    """LK_GGUF_KOTLIN_IDS = GGUFParser.kt:93's GGMLType.fromValue: 6 is Q8_0, 8 is Q2_K, no repack."""
    from ggml_hip import GGMLType
    q = np.zeros(2 * 34, np.uint8).tobytes()
    data = GO.write_gguf([], [("a", [64], 6, 0, q), ("b", [256], 8, 96, np.zeros(84, np.uint8).tobytes()),
                              ("c", [32], 2, 192, np.zeros(18, np.uint8).tobytes())])
    c = _parse(data, kotlin_ids=True)
    _assert_same(_mirror_summary(c), GO.parse(data, kotlin_ids=True))
    assert [t.type for t in c.tensors] == [GGMLType.Q8_0, GGMLType.Q2_K, GGMLType.Q4_0]
    assert not any(t.repack for t in c.tensors)
    # the same file read with upstream ids: 6 is Q5_0, 8 is Q8_0
    u = _parse(data)
    assert [t.type for t in u.tensors] == [GGMLType.Q5_0, GGMLType.Q8_0, GGMLType.Q4_0]
    assert u.tensors[2].repack


def test_host_load_non_repacked_types_is_byte_copy():
    from ggml_hip import GGMLGraphAllocator, NotOffloadedError
    from ggml_hip.gguf import ModelLoader
    data = _all_types_file()
    ref = GO.parse(data)
    m = ModelLoader().loadFromBytes(data)
    ga = GGMLGraphAllocator(device="host", defaultBufferSize=1 << 12)
    for t in ref["tensors"]:
        raw = data[ref["data_offset"] + t["offset"]:][:t["bytes"]]
        if t["type"] < 0:
            with pytest.raises(NotOffloadedError):
                m.getTensor(t["name"], ga)
        elif not t["repack"]:
            x = m.getTensor(t["name"], ga)
            assert bytes(ga.tensorBytes(x, t["bytes"])) == raw, t["name"]
            assert x.ne[:len(t["dims"])] == t["dims"]


def test_load_tensor_checks_destination():
    import ctypes
    from ggml_hip import IllegalArgumentException, _lib
    data = _all_types_file()
    c = _parse(data)
    L = _lib.load()
    i = c.findTensor("tok_embd.weight").index
    buf = np.zeros(64 * 3 * 4, np.uint8)
    with pytest.raises(IllegalArgumentException):
        _lib.check(L.lk_gguf_load_tensor(c._h, i, buf.ctypes.data, buf.size - 1, 0, None))
    _lib.check(L.lk_gguf_load_tensor(c._h, i, buf.ctypes.data, buf.size, 0, None))
    assert L.lk_gguf_load_tensor(c._h, 99, buf.ctypes.data, buf.size, 0, None) == _lib.LK_ERR_OUT_OF_BOUNDS
    # kv accessors reject the wrong kind of value
    k = L.lk_gguf_find_key(c._h, b"u8")
    s, n = ctypes.c_void_p(), ctypes.c_uint64()
    assert L.lk_gguf_kv_get_string(c._h, k, -1, ctypes.byref(s), ctypes.byref(n)) == _lib.LK_ERR_INVALID_ARG
    out = ctypes.create_string_buffer(8)
    assert L.lk_gguf_kv_get(c._h, L.lk_gguf_find_key(c._h, b"arr.f32"), 3, out, 8) == _lib.LK_ERR_OUT_OF_BOUNDS
    assert L.lk_gguf_kv_get(c._h, k, -1, out, 0) == _lib.LK_ERR_INVALID_ARG
    assert L.lk_gguf_find_key(c._h, b"nope") == -1 and L.lk_gguf_kv_key(c._h, 10**6) is None


def _kind(fn):
    from ggml_hip import IllegalArgumentException, IndexOutOfBoundsException
    try:
        fn()
        return "ok"
    except IllegalArgumentException:
        return "IllegalArgument"
    except IndexOutOfBoundsException:
        return "IndexOutOfBounds"


def _oracle_kind(data, **kw):
    try:
        GO.parse(data, **kw)
        return "ok"
    except GGUFErrorAlias as e:
        return e.kind


GGUFErrorAlias = GO.GGUFError


@pytest.mark.parametrize("src", ["reference", "all_types"])
def test_truncated_images_match_oracle(ref_file, src):
    data = ref_file if src == "reference" else _all_types_file()
    ref = GO.parse(data)
    header_end = ref["data_offset"]
    for n in range(0, header_end, 1 if src == "reference" else 3):
        got = _kind(lambda: _parse(data[:n]))
        want = _oracle_kind(data[:n])
        assert got == want, (n, got, want)
    # a data section cut short parses, but getTensorData is bounds-checked (GGUFContext.kt:90-92)
    from ggml_hip import IndexOutOfBoundsException
    c = _parse(data[:-1])
    last = max(c.tensors, key=lambda t: t.offset + t.nbytes)
    if c.dataOffset + last.offset + last.nbytes > len(data) - 1:
        with pytest.raises(IndexOutOfBoundsException):
            c.getTensorData(last)


def test_corrupted_images_match_oracle(ref_file):
    rng = np.random.default_rng(5)
    base = bytearray(_all_types_file())
    hdr = GO.parse(bytes(base))["data_offset"]
    for trial in range(400):
        d = bytearray(base if trial % 2 else ref_file)
        lim = hdr if trial % 2 else 256
        for _ in range(int(rng.integers(1, 4))):
            d[int(rng.integers(4, lim))] = int(rng.integers(0, 256))
        d = bytes(d)
        want = _oracle_kind(d)
        got = _kind(lambda: _parse(d))
        assert got == want, (trial, got, want)
        if want == "ok":
            _assert_same(_mirror_summary(_parse(d)), GO.parse(d))


def test_structural_errors():
    from ggml_hip import IllegalArgumentException
    ok = [("general.alignment", GO.UINT32, 32)]
    bad = [
        GO.write_gguf(ok, [], version=1),                                             # v1 counts are u32
        GO.write_gguf([("k", 13, 0)] if False else ok, [("t", [3], 2, 0, b"")]),     # ne[0] % 32
        GO.write_gguf([("general.alignment", GO.UINT32, 48)], []),                   # not a power of two
        GO.write_gguf(ok, [("t", [32], 99, 0, b"")]),                                 # unknown tensor type
        GO.write_gguf(ok, [("t", [1, 1, 1, 1, 1], 0, 0, b"")]),                       # 5 dims
    ]
    nested = bytearray(GO.write_gguf([("a", GO.ARRAY, (GO.UINT8, []))], []))
    nested[24 + 8 + 1 + 4:24 + 8 + 1 + 8] = struct.pack("<I", GO.ARRAY)  # element type ARRAY
    bad.append(bytes(nested))
    for d in bad:
        assert _oracle_kind(d) == "IllegalArgument"
        with pytest.raises(IllegalArgumentException):
            _parse(d)


def test_duplicate_keys_last_value_first_position():
    d = GO.write_gguf([("a", GO.UINT32, 1), ("b", GO.STRING, "x"), ("a", GO.UINT32, 2)], [])
    c = _parse(d)
    assert list(c.metadata) == ["a", "b"] and c.getLongValue("a") == 2
    _assert_same(_mirror_summary(c), GO.parse(d))


def test_repack_oracle_is_a_permutation_of_weights():
    """repack_to_kotlin moves weight j of upstream to Kotlin position j: the Kotlin-order
    dequantization of the repacked bytes equals upstream dequantization of the original."""
    import oracle as O
    rng = np.random.default_rng(3)
    x = rng.standard_normal(32 * 40).astype(np.float32)
    for ft, lk in ((GO.GGML_Q4_0, O.Q4_0), (GO.GGML_Q4_1, O.Q4_1), (GO.GGML_Q8_0, O.Q8_0)):
        raw = GO.upstream_quantize(ft, x)
        kot = np.frombuffer(GO.repack_to_kotlin(ft, raw), np.uint8)
        a = O.dequantize(lk, kot, x.size)
        b = GO.upstream_dequant(ft, raw, x.size)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), ft
