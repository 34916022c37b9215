// lk_gguf.cpp — GGUF parsing and quantized-tensor loading (include/lk_gguf.h).
//
// Host code of liblk_hip.so. The parse follows the reference's GGUFParser
// (gguf/GGUFParser.kt:19-201) field for field — header, key/values, tensor infos,
// aligned data offset — with two deliberate differences, both documented in
// lk_gguf.h: tensor type ids are read as upstream ggml_type by default, and tensor
// sizes are per block (the reference multiplies elements by the per-block byte
// size, GGUFContext.kt:100-103, which is only right for F32/F16).
//
// The image is never copied: metadata values and tensor bytes are referenced in
// place (a caller buffer, or a read-only mmap of the file). Loading moves tensor
// bytes to HBM through pinned staging and runs the nibble repack on the GPU.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lk_gguf.h"
#include "../../include/lk_hip.h"

int lk_detail_fail(int st, const char *msg);  // lk_hip.hip: sets lk_last_error()

namespace {

int fail(int st, const std::string &msg) { return lk_detail_fail(st, msg.c_str()); }

struct ParseError {
  int st;
  std::string msg;
};

// GGUF value types (GGUFTypes.kt:6-20): payload width, 0 for STRING/ARRAY.
int value_width(int32_t t) {
  switch (t) {
    case LK_GGUF_UINT8: case LK_GGUF_INT8: case LK_GGUF_BOOL: return 1;
    case LK_GGUF_UINT16: case LK_GGUF_INT16: return 2;
    case LK_GGUF_UINT32: case LK_GGUF_INT32: case LK_GGUF_FLOAT32: return 4;
    case LK_GGUF_UINT64: case LK_GGUF_INT64: case LK_GGUF_FLOAT64: return 8;
    default: return 0;
  }
}
bool valid_value_type(int32_t t) { return t >= LK_GGUF_UINT8 && t <= LK_GGUF_FLOAT64; }

// Tensor storage per type id: lk_type, weights per block, bytes per block, repack.
struct TypeDesc {
  int32_t lk;
  int32_t blck;
  int32_t bytes;
  int32_t repack;
};

// Upstream ggml_type ids (ggml/include/ggml.h:361-395) with their block geometry
// (ggml/src/ggml.c type_traits, ggml-common.h block structs).
bool upstream_type(int32_t id, TypeDesc *d) {
  static const struct { int32_t id; TypeDesc d; } T[] = {
      {0, {LK_TYPE_F32, 1, 4, 0}},        {1, {LK_TYPE_F16, 1, 2, 0}},
      {2, {LK_TYPE_Q4_0, 32, 18, 1}},     {3, {LK_TYPE_Q4_1, 32, 20, 1}},
      {6, {LK_TYPE_Q5_0, 32, 22, 0}},     {7, {LK_TYPE_Q5_1, 32, 24, 0}},
      {8, {LK_TYPE_Q8_0, 32, 34, 0}},     {9, {LK_TYPE_Q8_1, 32, 36, 0}},
      {10, {LK_TYPE_Q2_K, 256, 84, 0}},   {11, {LK_TYPE_Q3_K, 256, 110, 0}},
      {12, {LK_TYPE_Q4_K, 256, 144, 0}},  {13, {LK_TYPE_Q5_K, 256, 176, 0}},
      {14, {LK_TYPE_Q6_K, 256, 210, 0}},  {15, {LK_TYPE_Q8_K, 256, 292, 0}},
      {16, {-1, 256, 66, 0}} /*IQ2_XXS*/, {17, {-1, 256, 74, 0}} /*IQ2_XS*/,
      {18, {-1, 256, 98, 0}} /*IQ3_XXS*/, {19, {-1, 256, 50, 0}} /*IQ1_S*/,
      {20, {-1, 32, 18, 0}} /*IQ4_NL*/,   {21, {-1, 256, 110, 0}} /*IQ3_S*/,
      {22, {-1, 256, 82, 0}} /*IQ2_S*/,   {23, {-1, 256, 136, 0}} /*IQ4_XS*/,
      {24, {LK_TYPE_I8, 1, 1, 0}},        {25, {LK_TYPE_I16, 1, 2, 0}},
      {26, {LK_TYPE_I32, 1, 4, 0}},       {27, {LK_TYPE_I64, 1, 8, 0}},
      {28, {-1, 1, 8, 0}} /*F64*/,        {29, {-1, 256, 56, 0}} /*IQ1_M*/,
      {30, {-1, 1, 2, 0}} /*BF16*/,       {31, {-1, 32, 18, 0}} /*Q4_0_4_4*/,
      {32, {-1, 32, 18, 0}} /*Q4_0_4_8*/, {33, {-1, 32, 18, 0}} /*Q4_0_8_8*/,
  };
  for (const auto &e : T)
    if (e.id == id) { *d = e.d; return true; }
  return false;
}

// GGMLType.fromValue ids (core/GGMLTypes.kt:145-168), the reference's reading of
// the same field (GGUFParser.kt:93-95). Files in these ids hold llama.kotlin's own
// block layout, so nothing is repacked. Q1_5_K has no defined storage (size 0).
bool kotlin_type(int32_t id, TypeDesc *d) {
  static const TypeDesc T[] = {
      {LK_TYPE_F32, 1, 4, 0},     {LK_TYPE_F16, 1, 2, 0},     {LK_TYPE_Q4_0, 32, 18, 0},
      {LK_TYPE_Q4_1, 32, 20, 0},  {LK_TYPE_Q5_0, 32, 22, 0},  {LK_TYPE_Q5_1, 32, 24, 0},
      {LK_TYPE_Q8_0, 32, 34, 0},  {LK_TYPE_Q8_1, 32, 36, 0},  {LK_TYPE_Q2_K, 256, 84, 0},
      {LK_TYPE_Q3_K, 256, 110, 0}, {LK_TYPE_Q4_K, 256, 144, 0}, {LK_TYPE_Q5_K, 256, 176, 0},
      {LK_TYPE_Q6_K, 256, 210, 0}, {LK_TYPE_Q8_K, 256, 292, 0}, {LK_TYPE_Q1_5_K, 1, 0, 0},
      {LK_TYPE_I8, 1, 1, 0},      {LK_TYPE_I16, 1, 2, 0},     {LK_TYPE_I32, 1, 4, 0},
      {LK_TYPE_I64, 1, 8, 0},
  };
  if (id < 0 || id >= (int32_t)(sizeof T / sizeof T[0])) return false;
  *d = T[id];
  return true;
}

struct KV {
  std::string key;
  int32_t type = 0;
  int32_t elem_type = -1;  // ARRAY
  uint64_t n = 0;          // ARRAY length
  uint64_t pos = 0;        // image offset of the payload (scalar / string bytes / first element)
  uint64_t len = 0;        // STRING byte length
  std::vector<std::pair<uint64_t, uint64_t>> strs;  // string ARRAY: (offset, length)
};

struct Tensor {
  std::string name;
  lk_gguf_tensor_info info;
};

}  // namespace

struct lk_gguf {
  const uint8_t *base = nullptr;
  uint64_t size = 0;
  void *map = nullptr;  // owned mmap (lk_gguf_open_file)
  uint64_t map_bytes = 0;
  int32_t flags = 0;
  uint32_t version = 0;
  std::vector<KV> kv;
  std::unordered_map<std::string, int64_t> kv_index;
  std::vector<Tensor> tensors;
  std::unordered_map<std::string, int64_t> tensor_index;
  uint64_t alignment = 32;
  uint64_t data_offset = 0;
  uint64_t data_bytes = 0;
};

namespace {

struct Reader {
  const uint8_t *p;
  uint64_t size, pos = 0;
  void need(uint64_t n, const char *what) {
    if (n > size || pos > size - n)
      throw ParseError{LK_ERR_OUT_OF_BOUNDS, std::string(what) + " exceeds available data at offset " +
                                                 std::to_string(pos)};
  }
  template <class T>
  T get(const char *what) {
    need(sizeof(T), what);
    T v;
    std::memcpy(&v, p + pos, sizeof(T));  // little-endian host (x86-64 / gfx950 hosts)
    pos += sizeof(T);
    return v;
  }
  // GGUF string: u64 length + bytes (GGUFParser.kt:59-60, :190-197)
  std::pair<uint64_t, uint64_t> str(const char *what) {
    const uint64_t n = get<uint64_t>(what);
    need(n, what);
    const uint64_t at = pos;
    pos += n;
    return {at, n};
  }
  void skip(uint64_t n, const char *what) {
    need(n, what);
    pos += n;
  }
};

// readKeyValue / readArray (GGUFParser.kt:58-126)
KV read_kv(Reader &r) {
  KV kv;
  auto k = r.str("key");
  kv.key.assign((const char *)r.p + k.first, k.second);
  kv.type = (int32_t)r.get<uint32_t>("value type");
  if (!valid_value_type(kv.type)) throw ParseError{LK_ERR_INVALID_ARG, "Unknown GGUF type: " + std::to_string(kv.type)};
  if (kv.type == LK_GGUF_STRING) {
    auto s = r.str("string value");
    kv.pos = s.first;
    kv.len = s.second;
  } else if (kv.type == LK_GGUF_ARRAY) {
    kv.elem_type = (int32_t)r.get<uint32_t>("array type");
    if (!valid_value_type(kv.elem_type))
      throw ParseError{LK_ERR_INVALID_ARG, "Unknown GGUF type: " + std::to_string(kv.elem_type)};
    if (kv.elem_type == LK_GGUF_ARRAY) throw ParseError{LK_ERR_INVALID_ARG, "Nested arrays not supported"};
    kv.n = r.get<uint64_t>("array length");
    kv.pos = r.pos;
    if (kv.elem_type == LK_GGUF_STRING) {
      if (kv.n > r.size / 8) throw ParseError{LK_ERR_OUT_OF_BOUNDS, "string array length exceeds available data"};
      kv.strs.reserve(kv.n);
      for (uint64_t e = 0; e < kv.n; e++) kv.strs.push_back(r.str("string array element"));
    } else {
      const uint64_t w = value_width(kv.elem_type);
      if (kv.n > r.size / w) throw ParseError{LK_ERR_OUT_OF_BOUNDS, "array exceeds available data"};
      r.skip(kv.n * w, "array");
    }
  } else {
    kv.pos = r.pos;
    r.skip(value_width(kv.type), "value");
  }
  return kv;
}

bool kv_integer(const lk_gguf *g, const KV &kv, uint64_t *v) {
  const uint8_t *p = g->base + kv.pos;
  switch (kv.type) {
    case LK_GGUF_UINT8: *v = p[0]; return true;
    case LK_GGUF_INT8: *v = (uint64_t)(int64_t)(int8_t)p[0]; return true;
    case LK_GGUF_UINT16: { uint16_t x; std::memcpy(&x, p, 2); *v = x; return true; }
    case LK_GGUF_INT16: { int16_t x; std::memcpy(&x, p, 2); *v = (uint64_t)(int64_t)x; return true; }
    case LK_GGUF_UINT32: { uint32_t x; std::memcpy(&x, p, 4); *v = x; return true; }
    case LK_GGUF_INT32: { int32_t x; std::memcpy(&x, p, 4); *v = (uint64_t)(int64_t)x; return true; }
    case LK_GGUF_UINT64: case LK_GGUF_INT64: std::memcpy(v, p, 8); return true;
    default: return false;
  }
}

// GGUFParser.parse (GGUFParser.kt:19-56) + readTensorInfo (:86-100)
void parse(lk_gguf *g) {
  Reader r{g->base, g->size};
  r.need(4, "magic");
  if (std::memcmp(g->base, "GGUF", 4) != 0) {
    std::string m((const char *)g->base, 4);
    throw ParseError{LK_ERR_INVALID_ARG, "Invalid GGUF magic: " + m};
  }
  r.pos = 4;
  g->version = r.get<uint32_t>("version");
  if (g->version < 2)  // v1 used 32-bit counts and lengths
    throw ParseError{LK_ERR_INVALID_ARG, "unsupported GGUF version " + std::to_string(g->version)};
  const uint64_t n_tensors = r.get<uint64_t>("tensor count");
  const uint64_t n_kv = r.get<uint64_t>("metadata count");
  // Counts are not checked up front: entries are read in order, so a bad count fails
  // exactly where the reference's sequential read would (each entry consumes >= 12 B).

  for (uint64_t i = 0; i < n_kv; i++) {
    KV kv = read_kv(r);
    auto it = g->kv_index.find(kv.key);
    if (it != g->kv_index.end()) {
      g->kv[it->second] = std::move(kv);  // metadata[kv.key] = kv: last value, first position
    } else {
      g->kv_index.emplace(kv.key, (int64_t)g->kv.size());
      g->kv.push_back(std::move(kv));
    }
  }

  const bool kotlin_ids = (g->flags & LK_GGUF_KOTLIN_IDS) != 0;
  g->tensors.reserve((size_t)std::min<uint64_t>(n_tensors, g->size / 24));
  for (uint64_t i = 0; i < n_tensors; i++) {
    Tensor t;
    auto nm = r.str("tensor name");
    t.name.assign((const char *)g->base + nm.first, nm.second);
    lk_gguf_tensor_info &ti = t.info;
    std::memset(&ti, 0, sizeof ti);
    const uint32_t nd = r.get<uint32_t>("tensor n_dims");
    // GGML_MAX_DIMS (ggml.h) / "Unsupported tensor dimension count" (ModelLoader.kt:210-216)
    if (nd < 1 || nd > 4)
      throw ParseError{LK_ERR_INVALID_ARG, "Unsupported tensor dimension count: " + std::to_string(nd)};
    ti.n_dims = (int32_t)nd;
    uint64_t nel = 1;
    for (int d = 0; d < 4; d++) ti.ne[d] = 1;
    for (uint32_t d = 0; d < nd; d++) {
      const uint64_t v = r.get<uint64_t>("tensor dim");
      if (v > (1ull << 40) || (v && nel > (1ull << 62) / v))
        throw ParseError{LK_ERR_INVALID_ARG, "tensor " + t.name + ": dimension overflow"};
      ti.ne[d] = (int64_t)v;
      nel *= v;
    }
    ti.file_type = (int32_t)r.get<uint32_t>("tensor type");
    TypeDesc td;
    if (!(kotlin_ids ? kotlin_type(ti.file_type, &td) : upstream_type(ti.file_type, &td)))
      throw ParseError{LK_ERR_INVALID_ARG, "Unknown tensor type: " + std::to_string(ti.file_type)};
    if (ti.ne[0] % td.blck != 0)
      throw ParseError{LK_ERR_INVALID_ARG, "tensor " + t.name + ": ne[0] = " + std::to_string(ti.ne[0]) +
                                               " is not a multiple of the block size " + std::to_string(td.blck)};
    ti.type = td.lk;
    ti.repack = td.repack;
    ti.bytes = nel / (uint64_t)td.blck * (uint64_t)td.bytes;
    ti.offset = r.get<uint64_t>("tensor offset");
    if (ti.offset > g->size) throw ParseError{LK_ERR_OUT_OF_BOUNDS, "tensor " + t.name + ": offset beyond file"};
    g->tensor_index.emplace(t.name, (int64_t)g->tensors.size());
    g->tensors.push_back(std::move(t));
  }
  for (auto &t : g->tensors) t.info.name = t.name.c_str();  // stable after the vector stops growing

  // general.alignment (GGUFParser.kt:45): any integer type; default 32.
  auto it = g->kv_index.find("general.alignment");
  uint64_t a;
  if (it != g->kv_index.end() && kv_integer(g, g->kv[it->second], &a)) {
    if (a == 0 || a > (1ull << 62) || (a & (a - 1)) != 0)  // negative signed values land above 2^62
      throw ParseError{LK_ERR_INVALID_ARG, "general.alignment " + std::to_string(a) + " is not a power of two"};
    g->alignment = a;
  }
  g->data_offset = (r.pos + g->alignment - 1) / g->alignment * g->alignment;  // alignOffset (:199-201)
  uint64_t end = 0;
  for (const auto &t : g->tensors) end = std::max(end, t.info.offset + t.info.bytes);
  g->data_bytes = end;
}

int open_image(lk_gguf *g, lk_gguf **out) {
  try {
    parse(g);
  } catch (const ParseError &e) {
    lk_gguf_close(g);
    return fail(e.st, e.msg);
  } catch (const std::bad_alloc &) {
    lk_gguf_close(g);
    return fail(LK_ERR_OUT_OF_BOUNDS, "GGUF metadata exceeds host memory");
  }
  *out = g;
  return LK_OK;
}

const KV *get_kv(const lk_gguf *g, int64_t i) {
  if (!g || i < 0 || i >= (int64_t)g->kv.size()) return nullptr;
  return &g->kv[i];
}

// --- host -> device streaming through pinned staging ------------------------
//
// hipMemcpy from pageable (or mmapped) memory runs at a fraction of PCIe rate;
// two pinned chunks alternate so the memcpy into one overlaps the DMA of the other.
constexpr uint64_t kStageBytes = 64ull << 20;

struct Staging {
  std::mutex mu;
  void *buf[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  int device = -1;
};
Staging &stage() {
  static Staging s;
  return s;
}

#define GG_HIP(expr)                                                                                 \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) return fail(LK_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int h2d(const uint8_t *src, uint8_t *dst, uint64_t n, hipStream_t st) {
  if (n == 0) return LK_OK;
  if (n <= (4ull << 20)) {  // small tensors: one synchronous copy
    GG_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st));
    GG_HIP(hipStreamSynchronize(st));
    return LK_OK;
  }
  Staging &s = stage();
  std::lock_guard<std::mutex> lock(s.mu);
  int dev = 0;
  GG_HIP(hipGetDevice(&dev));
  if (s.device != dev) {
    for (int k = 0; k < 2; k++) {
      if (s.buf[k]) { (void)hipHostFree(s.buf[k]); s.buf[k] = nullptr; }
      if (s.done[k]) { (void)hipEventDestroy(s.done[k]); s.done[k] = nullptr; }
    }
    for (int k = 0; k < 2; k++) {
      GG_HIP(hipHostMalloc(&s.buf[k], kStageBytes, hipHostMallocDefault));
      GG_HIP(hipEventCreateWithFlags(&s.done[k], hipEventDisableTiming));
    }
    s.device = dev;
  }
  bool used[2] = {false, false};
  for (uint64_t off = 0, c = 0; off < n; off += kStageBytes, c++) {
    const int k = (int)(c & 1);
    const uint64_t m = std::min(kStageBytes, n - off);
    if (used[k]) GG_HIP(hipEventSynchronize(s.done[k]));  // chunk k's previous DMA has drained
    std::memcpy(s.buf[k], src + off, m);
    GG_HIP(hipMemcpyAsync(dst + off, s.buf[k], m, hipMemcpyHostToDevice, st));
    GG_HIP(hipEventRecord(s.done[k], st));
    used[k] = true;
  }
  GG_HIP(hipStreamSynchronize(st));
  return LK_OK;
}

}  // namespace

extern "C" {

int lk_gguf_open_memory(const void *data, uint64_t bytes, int32_t flags, lk_gguf **out) {
  if (!out) return fail(LK_ERR_INVALID_ARG, "null out handle");
  *out = nullptr;
  if (!data && bytes) return fail(LK_ERR_NO_BUFFER, "null GGUF image");
  if (flags & ~LK_GGUF_KOTLIN_IDS) return fail(LK_ERR_INVALID_ARG, "unknown flags " + std::to_string(flags));
  lk_gguf *g = new lk_gguf;
  g->base = (const uint8_t *)data;
  g->size = bytes;
  g->flags = flags;
  return open_image(g, out);
}

int lk_gguf_open_file(const char *path, int32_t flags, lk_gguf **out) {
  if (!out || !path) return fail(LK_ERR_INVALID_ARG, "null path or out handle");
  *out = nullptr;
  if (flags & ~LK_GGUF_KOTLIN_IDS) return fail(LK_ERR_INVALID_ARG, "unknown flags " + std::to_string(flags));
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return fail(LK_ERR_NO_BUFFER, std::string("cannot open ") + path + ": " + std::strerror(errno));
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    ::close(fd);
    return fail(LK_ERR_NO_BUFFER, std::string("cannot stat ") + path);
  }
  lk_gguf *g = new lk_gguf;
  g->flags = flags;
  g->size = (uint64_t)sb.st_size;
  if (g->size) {
    void *m = mmap(nullptr, g->size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      delete g;
      return fail(LK_ERR_NO_BUFFER, std::string("cannot map ") + path + ": " + std::strerror(errno));
    }
    (void)madvise(m, g->size, MADV_SEQUENTIAL);
    g->map = m;
    g->map_bytes = g->size;
    g->base = (const uint8_t *)m;
  }
  ::close(fd);
  return open_image(g, out);
}

void lk_gguf_close(lk_gguf *g) {
  if (!g) return;
  if (g->map) munmap(g->map, g->map_bytes);
  delete g;
}

uint32_t lk_gguf_version(const lk_gguf *g) { return g ? g->version : 0; }
uint64_t lk_gguf_alignment(const lk_gguf *g) { return g ? g->alignment : 0; }
uint64_t lk_gguf_data_offset(const lk_gguf *g) { return g ? g->data_offset : 0; }
uint64_t lk_gguf_data_bytes(const lk_gguf *g) { return g ? g->data_bytes : 0; }

int64_t lk_gguf_kv_count(const lk_gguf *g) { return g ? (int64_t)g->kv.size() : 0; }

int64_t lk_gguf_find_key(const lk_gguf *g, const char *key) {
  if (!g || !key) return -1;
  auto it = g->kv_index.find(key);
  return it == g->kv_index.end() ? -1 : it->second;
}

const char *lk_gguf_kv_key(const lk_gguf *g, int64_t i) {
  const KV *kv = get_kv(g, i);
  return kv ? kv->key.c_str() : nullptr;
}

int32_t lk_gguf_kv_type(const lk_gguf *g, int64_t i) {
  const KV *kv = get_kv(g, i);
  return kv ? kv->type : -1;
}

int lk_gguf_kv_array_info(const lk_gguf *g, int64_t i, int32_t *elem_type, uint64_t *n) {
  const KV *kv = get_kv(g, i);
  if (!kv) return fail(LK_ERR_OUT_OF_BOUNDS, "metadata index " + std::to_string(i));
  if (kv->type != LK_GGUF_ARRAY) return fail(LK_ERR_INVALID_ARG, kv->key + " is not an array");
  if (elem_type) *elem_type = kv->elem_type;
  if (n) *n = kv->n;
  return LK_OK;
}

int lk_gguf_kv_get(const lk_gguf *g, int64_t i, int64_t elem, void *out, uint64_t out_bytes) {
  const KV *kv = get_kv(g, i);
  if (!kv) return fail(LK_ERR_OUT_OF_BOUNDS, "metadata index " + std::to_string(i));
  int32_t t = kv->type;
  uint64_t pos = kv->pos;
  if (elem >= 0) {
    if (t != LK_GGUF_ARRAY) return fail(LK_ERR_INVALID_ARG, kv->key + " is not an array");
    if ((uint64_t)elem >= kv->n) return fail(LK_ERR_OUT_OF_BOUNDS, kv->key + ": element " + std::to_string(elem));
    t = kv->elem_type;
    pos += (uint64_t)elem * (uint64_t)value_width(t);
  } else if (t == LK_GGUF_ARRAY) {
    return fail(LK_ERR_INVALID_ARG, kv->key + " is an array: pass an element index");
  }
  const int w = value_width(t);
  if (w == 0) return fail(LK_ERR_INVALID_ARG, kv->key + " is a string");
  if (!out || out_bytes < (uint64_t)w) return fail(LK_ERR_INVALID_ARG, kv->key + ": output too small");
  std::memcpy(out, g->base + pos, w);
  return LK_OK;
}

int lk_gguf_kv_array_data(const lk_gguf *g, int64_t i, const void **data, uint64_t *elem_bytes) {
  const KV *kv = get_kv(g, i);
  if (!kv) return fail(LK_ERR_OUT_OF_BOUNDS, "metadata index " + std::to_string(i));
  if (kv->type != LK_GGUF_ARRAY || kv->elem_type == LK_GGUF_STRING)
    return fail(LK_ERR_INVALID_ARG, kv->key + " is not a numeric array");
  if (data) *data = g->base + kv->pos;
  if (elem_bytes) *elem_bytes = (uint64_t)value_width(kv->elem_type);
  return LK_OK;
}

int lk_gguf_kv_get_string(const lk_gguf *g, int64_t i, int64_t elem, const char **s, uint64_t *len) {
  const KV *kv = get_kv(g, i);
  if (!kv) return fail(LK_ERR_OUT_OF_BOUNDS, "metadata index " + std::to_string(i));
  std::pair<uint64_t, uint64_t> at;
  if (elem < 0) {
    if (kv->type != LK_GGUF_STRING) return fail(LK_ERR_INVALID_ARG, kv->key + " is not a string");
    at = {kv->pos, kv->len};
  } else {
    if (kv->type != LK_GGUF_ARRAY || kv->elem_type != LK_GGUF_STRING)
      return fail(LK_ERR_INVALID_ARG, kv->key + " is not a string array");
    if ((uint64_t)elem >= kv->n) return fail(LK_ERR_OUT_OF_BOUNDS, kv->key + ": element " + std::to_string(elem));
    at = kv->strs[(size_t)elem];
  }
  if (s) *s = (const char *)g->base + at.first;
  if (len) *len = at.second;
  return LK_OK;
}

int64_t lk_gguf_tensor_count(const lk_gguf *g) { return g ? (int64_t)g->tensors.size() : 0; }

int64_t lk_gguf_find_tensor(const lk_gguf *g, const char *name) {
  if (!g || !name) return -1;
  auto it = g->tensor_index.find(name);  // first tensor of that name, as tensors.find (GGUFContext.kt:78-80)
  return it == g->tensor_index.end() ? -1 : it->second;
}

int lk_gguf_get_tensor_info(const lk_gguf *g, int64_t i, lk_gguf_tensor_info *out) {
  if (!g || i < 0 || i >= (int64_t)g->tensors.size())
    return fail(LK_ERR_OUT_OF_BOUNDS, "tensor index " + std::to_string(i));
  if (!out) return fail(LK_ERR_INVALID_ARG, "null info");
  *out = g->tensors[(size_t)i].info;
  return LK_OK;
}

// getTensorData (GGUFContext.kt:85-95): bounds-checked view of the stored bytes.
int lk_gguf_tensor_data(const lk_gguf *g, int64_t i, const void **data, uint64_t *bytes) {
  if (!g || i < 0 || i >= (int64_t)g->tensors.size())
    return fail(LK_ERR_OUT_OF_BOUNDS, "tensor index " + std::to_string(i));
  const lk_gguf_tensor_info &ti = g->tensors[(size_t)i].info;
  const uint64_t start = g->data_offset + ti.offset, end = start + ti.bytes;
  if (start < g->data_offset || end < start || end > g->size)
    return fail(LK_ERR_OUT_OF_BOUNDS,
                "Tensor data extends beyond file: " + std::to_string(end) + " > " + std::to_string(g->size));
  if (data) *data = g->base + start;
  if (bytes) *bytes = ti.bytes;
  return LK_OK;
}

// loadTensorData (ModelLoader.kt:78-96), for every stored type, into llama.kotlin's layout.
int lk_gguf_load_tensor(const lk_gguf *g, int64_t i, void *dst, uint64_t dst_bytes, int32_t dst_on_device,
                        void *stream) {
  const void *src;
  uint64_t n;
  int st = lk_gguf_tensor_data(g, i, &src, &n);
  if (st != LK_OK) return st;
  const lk_gguf_tensor_info &ti = g->tensors[(size_t)i].info;
  if (ti.type < 0)
    return fail(LK_ERR_NOT_IMPLEMENTED, "tensor " + g->tensors[(size_t)i].name + ": file type " +
                                            std::to_string(ti.file_type) + " has no llama.kotlin GGMLType");
  if (dst_bytes < n)
    return fail(LK_ERR_INVALID_ARG, "Tensor data size mismatch: expected " + std::to_string(n) + ", got " +
                                        std::to_string(dst_bytes));
  if (n && !dst) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  if (n == 0) return LK_OK;
  hipStream_t hs = (hipStream_t)stream;
  const int64_t nblk = (int64_t)(n / (ti.type == LK_TYPE_Q4_0 ? 18 : 20));
  if (dst_on_device) {
    if ((st = h2d((const uint8_t *)src, (uint8_t *)dst, n, hs)) != LK_OK) return st;
    if (ti.repack) {
      if ((st = lk_repack_q4_device(dst, nblk, ti.type, LK_REPACK_UPSTREAM_TO_KOTLIN, stream)) != LK_OK) return st;
      GG_HIP(hipStreamSynchronize(hs));
    }
    return LK_OK;
  }
  if (!ti.repack) {
    std::memcpy(dst, src, n);
    return LK_OK;
  }
  // host destination of an upstream Q4 tensor: the repack runs on the GPU
  void *tmp = nullptr;
  GG_HIP(hipMalloc(&tmp, n));
  st = h2d((const uint8_t *)src, (uint8_t *)tmp, n, hs);
  if (st == LK_OK) st = lk_repack_q4_device(tmp, nblk, ti.type, LK_REPACK_UPSTREAM_TO_KOTLIN, stream);
  if (st == LK_OK) {
    hipError_t e = hipMemcpyAsync(dst, tmp, n, hipMemcpyDeviceToHost, hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    if (e != hipSuccess) st = fail(LK_ERR_DEVICE, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
  }
  (void)hipFree(tmp);
  return st;
}

int lk_gguf_load_all_device(const lk_gguf *g, void *dev_base, uint64_t dev_bytes, void *stream) {
  if (!g) return fail(LK_ERR_INVALID_ARG, "null handle");
  if (dev_bytes < g->data_bytes)
    return fail(LK_ERR_INVALID_ARG, "device buffer " + std::to_string(dev_bytes) + " < data section " +
                                         std::to_string(g->data_bytes));
  if (g->data_bytes == 0) return LK_OK;
  if (!dev_base) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  if (g->data_offset + g->data_bytes > g->size)
    return fail(LK_ERR_OUT_OF_BOUNDS, "Tensor data extends beyond file: " +
                                          std::to_string(g->data_offset + g->data_bytes) + " > " +
                                          std::to_string(g->size));
  for (const auto &t : g->tensors)
    if (t.info.repack && ((uintptr_t)dev_base + t.info.offset) % 2)
      return fail(LK_ERR_INVALID_ARG, "tensor " + t.name + ": odd offset, cannot repack in place");
  hipStream_t hs = (hipStream_t)stream;
  int st = h2d(g->base + g->data_offset, (uint8_t *)dev_base, g->data_bytes, hs);
  if (st != LK_OK) return st;
  for (const auto &t : g->tensors) {
    if (!t.info.repack || t.info.bytes == 0) continue;
    const int64_t nblk = (int64_t)(t.info.bytes / (t.info.type == LK_TYPE_Q4_0 ? 18 : 20));
    st = lk_repack_q4_device((uint8_t *)dev_base + t.info.offset, nblk, t.info.type, LK_REPACK_UPSTREAM_TO_KOTLIN,
                             stream);
    if (st != LK_OK) return st;
  }
  GG_HIP(hipStreamSynchronize(hs));
  return LK_OK;
}

}  // extern "C"
