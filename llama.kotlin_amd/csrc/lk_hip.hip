// lk_hip.hip — host side of the C-ABI declared in include/lk_hip.h.
//
// Operator semantics and error behaviour mirror computeMatMul
// (core/GGMLComputeOps.kt:1435-1565) for the node types this backend offloads:
//   Q4_0 x F32 -> F32, Q4_1 x F32 -> F32, Q8_0 x F32 -> F32   (the hot path)
//   F32 x F32 -> F32, F16 x F16 -> F16                         (general fallback :1530-1556)
// Every other combination returns LK_ERR_NOT_IMPLEMENTED so the caller keeps it
// on the CPU path (GGMLHipBackend.supportsOp == false) — this library has no CPU
// compute of its own.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "lk_kernels.hpp"
#include "lk_skinny.hpp"
#include "lk_kpart.hpp"
#include "lk_wide32.hpp"
#include "../../include/lk_gguf.h"

using namespace lk;

namespace {

thread_local std::string g_err;
thread_local std::string g_route;  // lk_debug_route: kernels launched on this thread since the last clear

void note_route(const char *fmt, ...) {
  char buf[160];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (g_route.size() >= 4096) {  // bounded: keep the newest words (a caller that never clears)
    const size_t cut = g_route.find(' ', g_route.size() / 2);
    g_route.erase(0, cut == std::string::npos ? g_route.size() : cut + 1);
  }
  if (!g_route.empty()) g_route += ' ';
  g_route += buf;
}

int fail(int st, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(LK_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

}  // namespace

// shared with lk_gguf.cpp (one lk_last_error for the whole library)
int lk_detail_fail(int st, const char *msg) { return fail(st, "%s", msg); }

namespace {

// Per-device state of the host (ByteArray) path: one library stream, the weight
// residency cache and staging scratch. lk_mul_mat uses the current device;
// lk_mul_mat_sharded drives several from one host thread.
constexpr int kMaxDevices = 64;

// Device copies of A (weight mirrors, the host path's staging) carry this many bytes past the
// matrix: the wide and LDS GEMMs' last row windows read up to OVERREAD (< 64) bytes beyond it, and
// they take a matrix only when those bytes are inside its buffer (wide_eligible, gemm_lds_eligible).
constexpr uint64_t kASlack = 256;

// A device mirror of host bytes [lo, lo + bytes) of the ByteArray at `base`, as of weight
// generation `gen`. Shared: the cache holds one reference while the mirror is current, every
// lk_graph that bound it holds one, and an lk_mul_mat call holds one while it runs. A pin
// with another generation over overlapping bytes, lk_weights_evict* and lk_weights_evict_all
// drop the mirror from the cache and mark it stale; a graph that finds a stale mirror at its
// next compute re-binds its weights (and rebuilds its plans) from the current cache or the
// host bytes. The device memory is freed when the last reference goes.
struct Mirror {
  int dev = 0;
  uintptr_t base = 0;
  uint64_t lo = 0, bytes = 0, gen = 0;
  void *ptr = nullptr;
  std::atomic<bool> stale{false};
  ~Mirror() {
    if (!ptr) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
    (void)hipFree(ptr);  // implicitly synchronizing: in-flight readers finish first
    (void)hipSetDevice(prev);
  }
  bool covers(uintptr_t b, uint64_t l, uint64_t h) const { return b == base && lo <= l && h <= lo + bytes; }
  bool overlaps(uintptr_t b, uint64_t l, uint64_t h) const { return b == base && l < lo + bytes && lo < h; }
};
using MirrorRef = std::shared_ptr<Mirror>;

struct Dev {
  hipStream_t stream = nullptr;
  unsigned *fail_flag = nullptr;  // page-locked word behind lk_sync_fail_flag (lk_kernels.hpp)
  unsigned timeouts_seen = 0;     // lk_sync_timeout_count at the last lk_sync_timeouts
  // weight residency cache (host path): the current mirrors of this device (guarded by S().cache_mu)
  std::vector<MirrorRef> weights;
  uint64_t weight_bytes = 0;
  // scratch for the host path: A staging, B, dst span
  void *scratch[3] = {nullptr, nullptr, nullptr};
  size_t scratch_bytes[3] = {0, 0, 0};
};
struct State {
  std::mutex mu;
  std::mutex cache_mu;  // every Dev::weights / weight_bytes access
  int device = -1;  // the device lk_mul_mat / lk_weights_pin use
  Dev devs[kMaxDevices];
};
State &S() {
  static State s;
  return s;
}

int block_bytes(int32_t t) {
  switch (t) {
    case LK_TYPE_Q4_0: return LK_Q4_0_BLOCK_BYTES;
    case LK_TYPE_Q4_1: return LK_Q4_1_BLOCK_BYTES;
    case LK_TYPE_Q8_0: return LK_Q8_0_BLOCK_BYTES;
    default: return 0;
  }
}
bool is_q(int32_t t) { return block_bytes(t) != 0; }
// K-quant super-blocks of 256 weights (core/GGMLTypes.kt:117-122)
int kblock_bytes(int32_t t) {
  switch (t) {
    case LK_TYPE_Q2_K: return LK_Q2_K_BLOCK_BYTES;
    case LK_TYPE_Q4_K: return LK_Q4_K_BLOCK_BYTES;
    case LK_TYPE_Q8_K: return LK_Q8_K_BLOCK_BYTES;
    default: return 0;
  }
}
bool is_kq(int32_t t) { return kblock_bytes(t) != 0; }

// rank / numElements (core/GGMLTypes.kt:275-300), used by getNumBlocks' bound.
int t_rank(const lk_tensor *t) {
  bool all_le1 = true, any_gt0 = false;
  int last = -1;
  for (int i = 0; i < 4; i++) {
    if (t->ne[i] > 1) { all_le1 = false; last = i; }
    if (t->ne[i] > 0) any_gt0 = true;
  }
  if (all_le1) return any_gt0 ? 1 : 0;
  return last + 1;
}
int64_t t_num_elements(const lk_tensor *t) {
  int r = t_rank(t);
  bool all_le1 = true, any_eq0 = false;
  for (int i = 0; i < 4; i++) {
    if (t->ne[i] > 1) all_le1 = false;
    if (t->ne[i] == 0) any_eq0 = true;
  }
  if (r == 0 && all_le1) return 1;
  if (r == 0 && any_eq0) return 0;
  int64_t c = 1;
  for (int i = 0; i < std::max(r, 1); i++) {
    if (t->ne[i] == 0 && r > 1) return 0;
    if (t->ne[i] > 0) c *= t->ne[i];
  }
  return c;
}

// Byte footprint [lo, hi) of a 2-D strided element tensor read at (i0<n0, i1<n1).
void span2(const lk_tensor *t, int64_t n0, int64_t n1, uint64_t width, uint64_t *lo, uint64_t *hi) {
  *lo = t->data_offset;
  *hi = t->data_offset + (uint64_t)(n0 - 1) * t->nb[0] + (uint64_t)(n1 - 1) * t->nb[1] + width;
}

enum class Path { kQuantF32, kKQuantF32, kF32, kF16 };

struct Checked {
  Path path;
  int64_t M, N, K;
  uint64_t a_lo, a_hi, b_lo, b_hi, d_lo, d_hi; // byte footprints (absolute in the buffers)
  bool empty;                                   // M*N == 0: nothing is read or written
};

// computeMatMul's checks (core/GGMLComputeOps.kt:1436-1564) for what this backend offloads.
// Errors the Kotlin loop would raise on its first faulting access are reported up front
// (dst may then hold a partial result on the CPU path; here dst is left untouched).
int check(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, Checked *c) {
  if (!a || !b || !dst) return fail(LK_ERR_INVALID_ARG, "null tensor descriptor");
  const int64_t M = a->ne[1], K_a = a->ne[0], N = b->ne[0], K_b = b->ne[1];
  if (K_a != K_b) /* :1440 */
    return fail(LK_ERR_INVALID_ARG, "Dim mismatch K: a.ne[0](%lld) != b.ne[1](%lld)", (long long)K_a, (long long)K_b);
  const int64_t K = K_a;
  if (dst->ne[0] != N || dst->ne[1] != M) /* :1444-1446 */
    return fail(LK_ERR_INVALID_ARG,
                "Result tensor dimensions must match expected output size: expected [%lld, %lld], got [%lld, %lld]",
                (long long)N, (long long)M, (long long)dst->ne[0], (long long)dst->ne[1]);
  c->M = M; c->N = N; c->K = K;
  c->empty = (M <= 0 || N <= 0);
  if (is_q(a->type) && b->type == LK_TYPE_F32) {
    if (dst->type != LK_TYPE_F32) /* :1449, :1463, :1517 */
      return fail(LK_ERR_INVALID_ARG, "Result tensor type must be F32 for quantized x F32 matmul");
    c->path = Path::kQuantF32;
  } else if (is_kq(a->type) && b->type == LK_TYPE_F32) {
    if (dst->type != LK_TYPE_F32) /* :1484, :1495, :1506 */
      return fail(LK_ERR_INVALID_ARG, "Result tensor type must be F32 for K-quant x F32 matmul");
    c->path = Path::kKQuantF32;
  } else {
    if (dst->type != a->type) /* :1530 */
      return fail(LK_ERR_INVALID_ARG, "Result tensor type must match first input type for general matmul");
    if (a->type == LK_TYPE_F32 && b->type == LK_TYPE_F32) c->path = Path::kF32;
    else if (a->type == LK_TYPE_F16 && b->type == LK_TYPE_F16) c->path = Path::kF16;
    else return fail(LK_ERR_NOT_IMPLEMENTED, "type combination (%d x %d) is not offloaded (CPU path)", a->type, b->type);
  }
  if (c->empty) return LK_OK;
  if (!dst->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found (dst)");
  if (K > 0) {
    if (!a->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found (a)");
    if (!b->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found (b)");
  }
  const uint64_t ew = (c->path == Path::kF16) ? 2 : 4;
  // device loads need natural alignment of element tensors
  auto misaligned = [&](const lk_tensor *t) {
    return (((uintptr_t)t->data + t->data_offset) % ew) || (t->nb[0] % ew) || (t->nb[1] % ew);
  };
  if (K > 0) {
    if (c->path == Path::kQuantF32) {
      // getNumBlocks bound (core/GGMLTypes.kt:598-602): last block touched is (M*K-1)/32.
      const int64_t last_blk = (M * K - 1) / 32;
      const int64_t nblk = t_num_elements(a) / 32;
      if (last_blk >= nblk)
        return fail(LK_ERR_INVALID_ARG, "blockIndex %lld out of bounds for %lld blocks", (long long)last_blk, (long long)nblk);
      c->a_lo = a->data_offset;
      c->a_hi = a->data_offset + (uint64_t)(last_blk + 1) * block_bytes(a->type);
      if (c->a_hi > a->buf_bytes)
        return fail(LK_ERR_OUT_OF_BOUNDS, "quant block read ends at %llu, out of buffer bounds %llu",
                    (unsigned long long)c->a_hi, (unsigned long long)a->buf_bytes);
    } else if (c->path == Path::kKQuantF32) {
      // getNumBlocks = numElements / 256 (core/GGMLTypes.kt:518); the partial path reads the
      // block of flat index M*K-1; full blocks never reach past it
      const int64_t last_blk = (M * K - 1) / 256;
      const int64_t nblk = t_num_elements(a) / 256;
      if (last_blk >= nblk)
        return fail(LK_ERR_INVALID_ARG, "blockIndex %lld out of bounds for %lld blocks", (long long)last_blk, (long long)nblk);
      c->a_lo = a->data_offset;
      c->a_hi = a->data_offset + (uint64_t)(last_blk + 1) * kblock_bytes(a->type);
      if (c->a_hi > a->buf_bytes)
        return fail(LK_ERR_OUT_OF_BOUNDS, "K-quant block read ends at %llu, out of buffer bounds %llu",
                    (unsigned long long)c->a_hi, (unsigned long long)a->buf_bytes);
    } else {
      span2(a, K, M, ew, &c->a_lo, &c->a_hi);
      if (c->a_hi > a->buf_bytes)
        return fail(LK_ERR_OUT_OF_BOUNDS, "Calculated offset %llu is out of bounds for buffer size %llu",
                    (unsigned long long)(c->a_hi - ew), (unsigned long long)a->buf_bytes);
      if (misaligned(a)) return fail(LK_ERR_NOT_IMPLEMENTED, "unaligned element strides for a (CPU path)");
    }
    span2(b, N, K, ew, &c->b_lo, &c->b_hi);
    if (c->b_hi > b->buf_bytes)
      return fail(LK_ERR_OUT_OF_BOUNDS, "Calculated offset %llu is out of bounds for buffer size %llu",
                  (unsigned long long)(c->b_hi - ew), (unsigned long long)b->buf_bytes);
    if (misaligned(b)) return fail(LK_ERR_NOT_IMPLEMENTED, "unaligned element strides for b (CPU path)");
  } else {
    c->a_lo = c->a_hi = a->data_offset;
    c->b_lo = c->b_hi = b->data_offset;
  }
  span2(dst, N, M, ew, &c->d_lo, &c->d_hi);
  if (c->d_hi > dst->buf_bytes)
    return fail(LK_ERR_OUT_OF_BOUNDS, "Calculated offset %llu is out of bounds for buffer size %llu",
                (unsigned long long)(c->d_hi - ew), (unsigned long long)dst->buf_bytes);
  if (misaligned(dst)) return fail(LK_ERR_NOT_IMPLEMENTED, "unaligned element strides for dst (CPU path)");
  return LK_OK;
}

// Device entry points run on the caller's stream; NULL is the HIP null (default) stream,
// so they order with whatever the caller last enqueued there.
hipStream_t pick_stream(void *s) { return (hipStream_t)s; }

// Fast grouped GEMV eligibility: batch 1, K % 64 == 0, 4-byte aligned A, 16-byte
// aligned contiguous x, F32 dst with unit column stride irrelevant (N == 1).
// Q4_K rides the streaming kernel too (16-block units; K % 256 == 0), in plans and chains as
// well as single launches; the other K-quants keep their own kernels.
bool stream_kquant(const lk_tensor *a, const Checked &c) {
  return c.path == Path::kKQuantF32 && (a->type == LK_TYPE_Q4_K || a->type == LK_TYPE_Q2_K) && c.K % LK_QK_K == 0;
}

bool gemv_eligible(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const Checked &c) {
  if (!(c.path == Path::kQuantF32 || stream_kquant(a, c)) || c.N != 1 || c.K <= 0 || (c.K % 64) != 0) return false;
  if (c.M > (int64_t)INT32_MAX || c.K > (int64_t)INT32_MAX) return false;
  if (((uintptr_t)a->data + a->data_offset) % 4) return false;
  if (((uintptr_t)b->data + b->data_offset) % 16) return false;
  if (c.K > 1 && b->nb[1] != 4) return false; // x(k) = B(0,k) contiguous
  if (dst->nb[1] % 4) return false;
  return true;
}

constexpr int kRowsQ4 = 4;
constexpr int kRowsQ8 = 2;
int rows_per_wave(int32_t qt) { return qt == LK_TYPE_Q8_0 ? kRowsQ8 : kRowsQ4; }

GemvDesc make_desc(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const Checked &c) {
  GemvDesc d{};
  d.a = (const uint8_t *)a->data + a->data_offset;
  d.x = (const float *)((const uint8_t *)b->data + b->data_offset);
  d.dst = (float *)((uint8_t *)dst->data + dst->data_offset);
  d.dst_row_stride = (int64_t)(dst->nb[1] / 4);
  d.M = (int32_t)c.M;
  d.K = (int32_t)c.K;
  return d;
}

// LDS-DMA streaming kernel eligibility on top of gemv_eligible: at most kStreamMaxUnits
// units of 64 block pairs per row, rows a whole number of 16-byte DMA lanes, A 16-aligned.
// Returns the units-per-row class (1..kStreamMaxUnits) or 0.
// Bytes of A per 64 items as the streaming kernel cuts rows (a block pair; a quarter Q4_K block).
int stream_pair_bytes(int32_t t) {
  return is_q(t) ? 2 * block_bytes(t) : t == LK_TYPE_Q4_K ? LK_Q4_K_BLOCK_BYTES / 4 : t == LK_TYPE_Q2_K ? LK_Q2_K_BLOCK_BYTES / 4 : 0;
}

int stream_class(const lk_tensor *a, const Checked &c) {
  const int64_t np = c.K / 64;
  const int64_t nch = (np + 63) / 64;
  if (nch < 1 || nch > kStreamMaxUnits) return 0;
  if (!stream_pair_bytes(a->type) || (np * stream_pair_bytes(a->type)) % 16) return 0;
  if (((uintptr_t)a->data + a->data_offset) % 16) return 0;
  return (int)nch;
}

int cu_count() {
  static int cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <int QT, int CPL>
void launch_stream_t(int grid, const GemvDesc &single, const StreamWork *work, int spw, hipStream_t st, const PeerDesc *peer) {
#ifdef LK_PF
  constexpr size_t lds = StreamGeom<QT, CPL>::LDS + kStreamWaves * 1024;  // lab: the prefetch landing slots
#else
  constexpr size_t lds = StreamGeom<QT, CPL>::LDS;
#endif
  if (peer)
    hipLaunchKernelGGL((gemv_stream_peer_kernel<QT, CPL>), dim3(grid), dim3(kStreamWaves * 64), lds, st, work, spw, peer);
  else
    hipLaunchKernelGGL((gemv_stream_kernel<QT, CPL>), dim3(grid), dim3(kStreamWaves * 64), lds, st, work, spw, single.a, single.x,
                       single.dst, single.dst_row_stride, single.M, single.K);
}

int launch_stream(int32_t qt, int cpl, int grid, const GemvDesc &single, const StreamWork *work, int spw,
                  hipStream_t st, const PeerDesc *peer = nullptr) {
  if (grid <= 0) return LK_OK;
  note_route("stream<%d,%d>:g%d%s", qt, cpl, grid, peer ? "x" : work ? "p" : "");
#define LK_STREAM(T, C) \
  if (qt == T && cpl == C) { launch_stream_t<T, C>(grid, single, work, spw, st, peer); HIP_TRY(hipGetLastError()); return LK_OK; }
  LK_STREAM(LK_TYPE_Q4_0, 1) LK_STREAM(LK_TYPE_Q4_0, 2) LK_STREAM(LK_TYPE_Q4_0, 3)
  LK_STREAM(LK_TYPE_Q4_1, 1) LK_STREAM(LK_TYPE_Q4_1, 2) LK_STREAM(LK_TYPE_Q4_1, 3)
  LK_STREAM(LK_TYPE_Q8_0, 1) LK_STREAM(LK_TYPE_Q8_0, 2) LK_STREAM(LK_TYPE_Q8_0, 3)
  LK_STREAM(LK_TYPE_Q4_K, 1) LK_STREAM(LK_TYPE_Q4_K, 2) LK_STREAM(LK_TYPE_Q4_K, 3)
  LK_STREAM(LK_TYPE_Q2_K, 1) LK_STREAM(LK_TYPE_Q2_K, 2) LK_STREAM(LK_TYPE_Q2_K, 3)
#undef LK_STREAM
  return fail(LK_ERR_NOT_IMPLEMENTED, "stream gemv: type %d class %d", qt, cpl);
}

// Workgroups for `rows` rows: one per CU, but no fewer than ~kStreamWaves rows each.
int stream_grid(int64_t rows) {
  const int64_t g = (rows + kStreamWaves - 1) / kStreamWaves;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cu_count()));
}

int launch_gemv_v1(int32_t qt, const GemvDesc &d, hipStream_t st) {
  const int rpt = kGemvWaves * rows_per_wave(qt);
  const int64_t ntiles = ((int64_t)d.M + rpt - 1) / rpt;
  if (ntiles <= 0) return LK_OK;
  if (ntiles > INT32_MAX) return fail(LK_ERR_NOT_IMPLEMENTED, "too many rows");
  dim3 grid((unsigned)ntiles), block(256);
  note_route("gemv_v1<%d>", qt);
  switch (qt) {
    case LK_TYPE_Q4_0: hipLaunchKernelGGL((gemv_q_n1_kernel<LK_TYPE_Q4_0, kRowsQ4>), grid, block, 0, st, d); break;
    case LK_TYPE_Q4_1: hipLaunchKernelGGL((gemv_q_n1_kernel<LK_TYPE_Q4_1, kRowsQ4>), grid, block, 0, st, d); break;
    case LK_TYPE_Q8_0: hipLaunchKernelGGL((gemv_q_n1_kernel<LK_TYPE_Q8_0, kRowsQ8>), grid, block, 0, st, d); break;
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "gemv: type %d", qt);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// Batched quantized GEMM on MFMA: N >= 2, whole blocks per row (K % 32 == 0).
bool gemm_eligible(const Checked &c) {
  return c.path == Path::kQuantF32 && c.N >= 2 && c.K > 0 && (c.K % 32) == 0 && c.M <= INT32_MAX &&
         c.N <= INT32_MAX && c.K <= INT32_MAX;
}

// Device scratch for the GEMM (activation fragments, block sums, split-K partials, tile
// counters), per device and stream (gemm_scratch), grow-only. Counters are zeroed when allocated — on the launch's stream
// (hipMemsetAsync: stream-ordered before the launch that first uses them, and part of a capture
// that allocates them) — and re-armed by the kernels.
//
// Lifetime: launches captured into HIP graphs (lk_graph's replay, a caller's torch / HIP graph of
// lk_mul_mat_device or lk_plan_launch) bake these pointers in. A buffer outgrown by a later call is
// therefore never freed while the library lives: it is retired (kept allocated, untouched by any new
// launch) and released by lk_shutdown, so a replay captured before the growth still reads and writes
// memory that belongs to it. Growth doubles, so the retired bytes stay below the live ones.
// `epoch` counts reallocations (lk_graph records it; diagnostic).
struct GemmScratch {
  void *frag = nullptr; size_t frag_bytes = 0;
  void *partial = nullptr; size_t partial_bytes = 0;
  int32_t *counter = nullptr; size_t counter_n = 0;
  unsigned *tcnt = nullptr;  // split-K arrival counters, one word per output tile of a launch
  size_t tcnt_n = 0;
  std::vector<void *> retired;
  uint64_t retired_bytes = 0;
  uint64_t epoch = 0;
};

// One scratch per (device, stream): launches on different streams never share fragments, slabs or
// counters, so two streams may run batched MUL_MATs concurrently (a torch side stream and the
// library stream of the host path, say). A stream handle reused after hipStreamDestroy inherits the
// old stream's scratch, which its work no longer touches.
struct ScratchKey {
  int dev;
  hipStream_t st;
  bool operator<(const ScratchKey &o) const { return dev != o.dev ? dev < o.dev : (uintptr_t)st < (uintptr_t)o.st; }
};
std::mutex g_scratch_mu;
std::map<ScratchKey, GemmScratch> &scratch_map() {
  static std::map<ScratchKey, GemmScratch> m;  // node-based: references stay valid as it grows
  return m;
}

GemmScratch &gemm_scratch(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  return scratch_map()[ScratchKey{dev, st}];
}

// Grow *p to at least `want` bytes (at least double the old size); the old buffer is retired, not
// freed (see GemmScratch). zero: zero the new bytes on stream st (counters).
int grow_scratch(GemmScratch &S, void **p, size_t *have, size_t want, bool zero, hipStream_t st) {
  if (*have >= want) return LK_OK;
  const size_t bytes = std::max(want, 2 * *have);
  void *q = nullptr;
  if (hipMalloc(&q, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(LK_ERR_DEVICE, "scratch: hipMalloc of %zu B failed", bytes);
  }
  if (zero) HIP_TRY(hipMemsetAsync(q, 0, bytes, st));
  if (*p) { S.retired.push_back(*p); S.retired_bytes += *have; }
  *p = q;
  *have = bytes;
  S.epoch++;
  return LK_OK;
}
// Split-K fix-up by the last arriver (lk_kernels.hpp splitk_arrive): the per-tile arrival counters
// to pass (ntiles words, zero between launches: the last arrival of each tile re-arms its word), or
// null — then splitk_reduce_kernel sums the slabs after the GEMM (LK_SKP_UNFUSED=1, one slice, slabs
// beyond a 32-bit buffer offset, or more tiles per workgroup than its LDS list holds: list_ok false).
// No co-residency is assumed: nobody waits, so any grid size and any concurrent stream are safe.
// Per-tile arrival counters for the in-launch split-K fix-up by the last arriver, or null: the slabs
// are then summed by splitk_reduce_kernel launched after the GEMM (no waits either way). The default
// is per kernel family (`in_launch`), measured round 4: the last arriver wins for the
// wide kernel's two slices (C5 56.3 vs 56.2 µs: a launch saved at no cost) and loses for the skinny /
// pair / sk kernels' eight (Q8_0 N = 32 36.9 vs 27.8 µs, Q4_K 35.3 vs 26.8, the down projection
// 4096 x 11008 N = 32 on the pair kernel 43.7 vs 22.3): the slowest slice of a range ends up summing
// every tile of it. LK_SKP_UNFUSED=1 / LK_SKP_FUSED=1 force either form (A/B).
int splitk_counters(int slices, size_t slab_bytes, int64_t ntiles, bool list_ok, bool in_launch, hipStream_t st,
                    unsigned **out) {
  static const bool unfused = getenv("LK_SKP_UNFUSED") != nullptr, fused = getenv("LK_SKP_FUSED") != nullptr;
  *out = nullptr;
  if (!fused && (unfused || !in_launch)) return LK_OK;
  if (slices <= 1 || !list_ok || slab_bytes >= (1ull << 31) || ntiles <= 0) return LK_OK;
  GemmScratch &S = gemm_scratch(st);
  if (S.tcnt_n < (size_t)ntiles * kChainLine) {  // a 128-B line per tile
    const size_t want = std::max<size_t>((size_t)ntiles * kChainLine, 1 << 16);
    void *p = S.tcnt;
    size_t have = S.tcnt_n * sizeof(unsigned);
    if (int rc = grow_scratch(S, &p, &have, want * sizeof(unsigned), true, st)) return rc;
    S.tcnt = (unsigned *)p;
    S.tcnt_n = have / sizeof(unsigned);
  }
  // re-armed on the launch stream before every launch (stream-ordered, captured with it): a word left
  // non-zero by anything — a launch that failed part-way, a poke — cannot make a tile's last arrival
  // fire early or never (the kernels re-arm it too)
  HIP_TRY(hipMemsetAsync(S.tcnt, 0, (size_t)ntiles * kChainLine * sizeof(unsigned), st));
  *out = S.tcnt;
  return LK_OK;
}

// The per-tile counters of gemm_q_mfma_kernel / gemm_q_lds_kernel (zero between launches).
int gemm_counters(size_t tiles, hipStream_t st, int32_t **out) {
  GemmScratch &S = gemm_scratch(st);
  if (S.counter_n < tiles) {
    void *p = S.counter;
    size_t have = S.counter_n * sizeof(int32_t);
    if (int rc = grow_scratch(S, &p, &have, std::max<size_t>(tiles, 4096) * sizeof(int32_t), true, st)) return rc;
    S.counter = (int32_t *)p;
    S.counter_n = have / sizeof(int32_t);
  }
  // re-armed before every launch (see splitk_counters): round 4's resident-graph failure was a tile
  // whose counter was non-zero at entry, so its last arrival never fired and the tile stayed unwritten
  // (DESIGN §4); tests/test_scratch_gpu.py pokes a counter through lk_debug_poke_gemm_counter
  HIP_TRY(hipMemsetAsync(S.counter, 0, tiles * sizeof(int32_t), st));
  *out = S.counter;
  return LK_OK;
}

// Activation fragments for the batched kernels (xsplit_kernel: a wave per kXsItems (x-tile, block) items).
void launch_xsplit(const XSplitArgs &xa_in, hipStream_t st) {
  XSplitArgs xa = xa_in;
  const int64_t ntx = (xa.N + 15) / 16, nblk = xa.K / 32, waves = (ntx * nblk + kXsItems - 1) / kXsItems;
  xa.xblocks = (int32_t)((waves + 3) / 4);
  const int64_t zblocks = xa.zero ? ((int64_t)xa.zM * ((xa.zN + 3) / 4) + 255) / 256 : 0;
  hipLaunchKernelGGL(xsplit_kernel, dim3((unsigned)(xa.xblocks + zblocks)), dim3(256), 0, st, xa);
}

int grow(GemmScratch &S, void **p, size_t *have, size_t want) { return grow_scratch(S, p, have, want, false, nullptr); }

int gemm_waves() {  // LK_GEMM_WAVES = 4 or 8 waves per LDS-GEMM workgroup (tuning only)
  static int nw = [] {
    const char *e = getenv("LK_GEMM_WAVES");
    return (e && atoi(e) == 8) ? 8 : 4;
  }();
  return nw;
}

int gemm_occupancy() {  // LK_GEMM_OCC overrides (tuning only)
  static int occ = [] {
    const char *e = getenv("LK_GEMM_OCC");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 2;
  }();
  return occ;
}

template <int QT, int WM, int WN, int MT, int NT>
int launch_gemm_t(GemmArgs g, const XSplitArgs &xa, hipStream_t st) {
  constexpr int BM = WM * MT * 16, BN = WN * NT * 16;
  GemmScratch &S = gemm_scratch(st);
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  const int tiles = g.tiles_m * g.tiles_n;
  const int nblk = g.K / 32;
  // split K until the grid holds ~gemm_occupancy() workgroups per CU (latency hiding)
  int slices = std::max(1, std::min({(gemm_occupancy() * cu_count() + tiles - 1) / tiles, 32, nblk}));
  g.kslice = (nblk + slices - 1) / slices;
  slices = (nblk + g.kslice - 1) / g.kslice;
  if ((size_t)slices * tiles * BM * BN * sizeof(float) >= (1ull << 31)) {  // slabs through a 32-bit buffer offset
    g.kslice = nblk;
    slices = 1;
  }
  g.slices = slices;
  if (slices > 1) {
    int rc = grow(S, &S.partial, &S.partial_bytes, (size_t)slices * tiles * BM * BN * sizeof(float));
    if (rc) return rc;
    if ((rc = gemm_counters((size_t)tiles, st, &g.counter))) return rc;
    g.partial = (float *)S.partial;
  }
  note_route("gemm_q_mfma<%d>:t%ds%d", QT, tiles, slices);
  launch_xsplit(xa, st);
  hipLaunchKernelGGL((gemm_q_mfma_kernel<QT, WM, WN, MT, NT>), dim3((unsigned)(tiles * slices)), dim3(256), 0, st, g);
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// LDS-DMA pipelined GEMM (gemm_q_lds_kernel): K % 128 == 0 and weight rows aligned for its
// DMA pieces. One workgroup (4 waves, ~100-150 KB of LDS) per CU; split K to fill the grid.
bool gemm_lds_eligible(int32_t qt, const lk_tensor *a, const Checked &c) {
  if ((c.K / 32) % kLdsSB) return false;
  const uintptr_t base = (uintptr_t)a->data + a->data_offset;
  if (base % 8) return false;  // rows start 8-byte aligned for the 16-byte DMA pieces
  // the last row's last stage reads up to OVERREAD bytes past the matrix: they must be in the buffer
  const uint64_t over = qt == LK_TYPE_Q4_0 ? LdsGemmGeom<LK_TYPE_Q4_0, 2, 4>::OVERREAD
                       : qt == LK_TYPE_Q4_1 ? LdsGemmGeom<LK_TYPE_Q4_1, 2, 4>::OVERREAD
                                            : LdsGemmGeom<LK_TYPE_Q8_0, 2, 4>::OVERREAD;
  return c.a_hi + over <= a->buf_bytes;
}

template <int QT, int NT, int NW>
int launch_gemm_lds_t(GemmArgs g, const XSplitArgs &xa, hipStream_t st) {
  using GG = LdsGemmGeom<QT, NT, NW>;
  GemmScratch &S = gemm_scratch(st);
  g.tiles_m = (g.M + GG::BM - 1) / GG::BM;
  g.tiles_n = (g.N + GG::BN - 1) / GG::BN;
  const int tiles = g.tiles_m * g.tiles_n;
  const int nst = g.K / 32 / GG::SB;  // stages over the whole K
  int slices = std::max(1, std::min({(gemm_occupancy() * cu_count() / 4 + tiles - 1) / tiles, 32, nst}));
  g.kslice = ((nst + slices - 1) / slices) * GG::SB;
  slices = (g.K / 32 + g.kslice - 1) / g.kslice;
  if ((size_t)slices * tiles * GG::BM * GG::BN * sizeof(float) >= (1ull << 31)) {  // slabs through a 32-bit buffer offset
    g.kslice = g.K / 32;
    slices = 1;
  }
  g.slices = slices;
  if (slices > 1) {
    int rc = grow(S, &S.partial, &S.partial_bytes, (size_t)slices * tiles * GG::BM * GG::BN * sizeof(float));
    if (rc) return rc;
    if ((rc = gemm_counters((size_t)tiles, st, &g.counter))) return rc;
    g.partial = (float *)S.partial;
  }
  note_route("gemm_q_lds<%d,%d,%d>:t%ds%d", QT, NT, NW, tiles, slices);
  launch_xsplit(xa, st);
  constexpr size_t lds = GG::LDS;
  hipLaunchKernelGGL((gemm_q_lds_kernel<QT, NT, NW>), dim3((unsigned)(tiles * slices)), dim3(NW * 64), lds, st, g);
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

template <int QT>
int launch_gemm_qt(const GemmArgs &g, const XSplitArgs &xa, bool lds_ok, hipStream_t st) {
  if (lds_ok) {
    const int nw = gemm_waves();
    if (g.N <= 16) return nw == 8 ? launch_gemm_lds_t<QT, 1, 8>(g, xa, st) : launch_gemm_lds_t<QT, 1, 4>(g, xa, st);
    if (g.N <= 32) return nw == 8 ? launch_gemm_lds_t<QT, 2, 8>(g, xa, st) : launch_gemm_lds_t<QT, 2, 4>(g, xa, st);
    return nw == 8 ? launch_gemm_lds_t<QT, 4, 8>(g, xa, st) : launch_gemm_lds_t<QT, 4, 4>(g, xa, st);
  }
  if (g.N <= 16) return launch_gemm_t<QT, 4, 1, 2, 1>(g, xa, st);
  if (g.N <= 32) return launch_gemm_t<QT, 4, 1, 2, 2>(g, xa, st);
  return launch_gemm_t<QT, 2, 2, 2, 2>(g, xa, st);
}

// Skinny split-K GEMM (gemm_skinny_kernel): 2 <= N <= 32, whole blocks, weight rows and slice
// pieces 16-byte aligned (buffer offset % 16 == 0, row bytes % 16 == 0: every Llama shape).
bool skinny_eligible(const lk_tensor *a, const Checked &c) {
  static const bool off = getenv("LK_NO_SKINNY") != nullptr;  // tuning / A-B only
  if (off || c.N > 32) return false;
  const uint64_t bb = a->type == LK_TYPE_Q4_0 ? 18 : a->type == LK_TYPE_Q4_1 ? 20 : 34;
  const uint64_t rb = (uint64_t)(c.K / 32) * bb;
  const uintptr_t base = (uintptr_t)a->data + a->data_offset;
  return base % 16 == 0 && rb % 16 == 0 && rb * 16 < (1ull << 31);
}

template <int QT, int NT>
int launch_skinny_t(SkinnyArgs g, hipStream_t st) {
  using SG = SkinnyGeom<QT, NT>;
  GemmScratch &S = gemm_scratch(st);
  const int nblk = g.K / 32;
  const int slices = (nblk + SG::SB - 1) / SG::SB;
  const int ntile = (g.M + 15) / 16;
  // one workgroup per CU (LDS): about cu_count() workgroups in all; split-K fixed up by the last
  // arriver per tile unless LK_SKP_UNFUSED=1 (its list: 16 + NW·⌈tiles/NW⌉ ints in the staging area)
  const int cu = cu_count();
  int ranges = std::max(1, std::min(ntile, cu / slices));
  g.tiles_per_range = (ntile + ranges - 1) / ranges;
  ranges = (ntile + g.tiles_per_range - 1) / g.tiles_per_range;
  unsigned *rsync = nullptr;
  const bool list_ok = 1 + (g.tiles_per_range + SG::NW - 1) / SG::NW <= SG::D * SG::SLOT / 4;  // a wave's ring
  if (int rf = splitk_counters(slices, (size_t)slices * g.M * 16 * NT * sizeof(float), ntile, list_ok, false, st, &rsync)) return rf;
  g.slices = slices;
  if (slices > 1) {
    const int rc = grow(S, &S.partial, &S.partial_bytes, (size_t)slices * g.M * 16 * NT * sizeof(float));
    if (rc) return rc;
    g.partial = (float *)S.partial;
  }
  g.tasks = ranges * slices;
  g.rsync = rsync;
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("skinny<%d,%d>:s%dr%d%s", QT, NT, slices, ranges, rsync ? "f" : "");
  hipLaunchKernelGGL((gemm_skinny_kernel<QT, NT>), dim3(grid), dim3(SG::NW * 64), SG::LDS, st, g);
  if (slices > 1 && !rsync) {
    const int64_t threads = (int64_t)g.M * (16 * NT / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const float *)g.partial,
                       slices, g.M, g.N, 16 * NT, g.dst, g.d_nb0, g.d_nb1);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

bool getenv_flag(const char *name);

// gemm_skinny_pair_kernel's split-K tasks for g's shape: slices of SB blocks, row ranges filling the
// CUs; returns the slab bytes (0 for one slice). Shared by the single launch and a plan's grouped launch,
// so both compute the same bits.
template <int QT, int NT>
size_t pair_geometry(SkinnyArgs &g) {
  using SG = SkinnyPairGeom<QT, NT>;
  const int nblk = g.K / 32;
  const int slices = (nblk + SG::SB - 1) / SG::SB;
  const int ntile = (g.M + 15) / 16;
  // at least one tile per stream (4 wave pairs per workgroup): small matrices (a 1/8-row shard) otherwise
  // got one tile per workgroup, three of its four streams idle behind the full activation prologue.
  // Ranges only partition tiles among workgroups, so the bits do not depend on it.
  static const int min_tpr = [] { const char *e = getenv("LK_SKP_MIN_TPR"); return e ? std::max(1, atoi(e)) : 4; }();
  int ranges = std::max(1, std::min({ntile, cu_count() / slices, (ntile + min_tpr - 1) / min_tpr}));
  g.tiles_per_range = (ntile + ranges - 1) / ranges;
  ranges = (ntile + g.tiles_per_range - 1) / g.tiles_per_range;
  g.slices = slices;
  g.tasks = ranges * slices;
  return slices > 1 ? (size_t)slices * g.M * 16 * NT * sizeof(float) : 0;
}

// gemm_skinny_pair_kernel: the same split-K tasks, a wave pair per stream (8 waves).
template <int QT, int NT>
int launch_skinny_pair_t(SkinnyArgs g, hipStream_t st) {
  using SG = SkinnyPairGeom<QT, NT>;
  GemmScratch &S = gemm_scratch(st);
  (void)pair_geometry<QT, NT>(g);
  const int slices = g.slices, ntile = (g.M + 15) / 16, ranges = g.tasks / g.slices;
  // split-K fixed up by the last arriver per tile unless LK_SKP_UNFUSED=1 (splitk_counters)
  const size_t slab_bytes = (size_t)slices * g.M * 16 * NT * sizeof(float);
  unsigned *rsync = nullptr;
  const bool list_ok = 1 + (g.tiles_per_range + 3) / 4 <= NT * 64 * 4;  // parity 0 of a pair's hand-off
  if (int rc = splitk_counters(slices, slab_bytes, ntile, list_ok, false, st, &rsync)) return rc;
  const bool fuse = rsync != nullptr;
  if (slices > 1) {
    const int rc = grow(S, &S.partial, &S.partial_bytes, slab_bytes);
    if (rc) return rc;
    g.partial = (float *)S.partial;
  }
  g.rsync = rsync;
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("pair<%d,%d>:s%dr%d%s", QT, NT, slices, ranges, fuse ? "f" : "");
  hipLaunchKernelGGL((gemm_skinny_pair_kernel<QT, NT>), dim3(grid), dim3(SG::NW * 64), SG::LDS, st, g);
  if (slices > 1 && !fuse) {
    const int64_t threads = (int64_t)g.M * (16 * NT / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const float *)g.partial,
                       slices, g.M, g.N, 16 * NT, g.dst, g.d_nb0, g.d_nb1);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// gemm_sk_kernel (lk_skinny.hpp): Q4_K x F32, 16 <= N <= 32. Dense, 16-B aligned activations
// are split by the kernel itself; others go through xsplit_kernel first. Split-K slabs are
// fixed up inside the launch by the last arriver per tile (splitk_counters) or by splitk_reduce_kernel after it.
template <int QT, int NT>
int launch_sk_t(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  using SG = SkGeom<QT, NT>;
  GemmScratch &S = gemm_scratch(st);
  const int64_t nblk = c.K / 32, ntx = (c.N + 15) / 16;
  const size_t fb = (size_t)ntx * nblk * kXSplits * 64 * 16, sb = (size_t)nblk * ntx * 16 * sizeof(float);
  int rc = grow(S, &S.frag, &S.frag_bytes, fb + sb);
  if (rc) return rc;
  XSplitArgs xa{};
  xa.b = (const uint8_t *)b->data + b->data_offset;
  xa.b_nb0 = b->nb[0]; xa.b_nb1 = b->nb[1];
  xa.N = c.N; xa.K = c.K;
  xa.frag = (u32x4 *)S.frag;
  xa.xsum = (float *)((uint8_t *)S.frag + fb);
  xa.mult = 1.f;
  xa.q4_order = 2;
  SkArgs g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.frag = xa.frag;
  g.xsum = xa.xsum;
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  g.M = (int32_t)c.M; g.N = (int32_t)c.N; g.K = (int32_t)c.K;
  const int slices = (int)((nblk + SG::SB - 1) / SG::SB);
  const int ntile = (g.M + 15) / 16;
  const int cu = cu_count();
  int ranges = std::max(1, std::min(ntile, cu / slices));
  g.tiles_per_range = (ntile + ranges - 1) / ranges;
  ranges = (ntile + g.tiles_per_range - 1) / g.tiles_per_range;
  unsigned *rsync = nullptr;
  const bool list_ok = 1 + (g.tiles_per_range + 3) / 4 <= NT * 64 * 4;  // parity 0 of a pair's hand-off
  if (int rf = splitk_counters(slices, (size_t)slices * g.M * 16 * NT * sizeof(float), ntile, list_ok, false, st, &rsync)) return rf;
  g.slices = slices;
  if (slices > 1) {
    rc = grow(S, &S.partial, &S.partial_bytes, (size_t)slices * g.M * 16 * NT * sizeof(float));
    if (rc) return rc;
    g.partial = (float *)S.partial;
  }
  g.tasks = ranges * slices;
  g.rsync = rsync;
  g.b = xa.b;
  g.fx = b->nb[0] == 4 && b->nb[1] == 4 * (uint64_t)c.N && ((uintptr_t)xa.b & 15) == 0;
  if (!g.fx) launch_xsplit(xa, st);
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("sk<%d,%d>:s%dr%d%s", QT, NT, slices, ranges, rsync ? "f" : "");
  hipLaunchKernelGGL((gemm_sk_kernel<QT, NT>), dim3(grid), dim3(SG::NW * 64), SG::LDS, st, g);
  if (slices > 1 && !rsync) {
    const int64_t threads = (int64_t)g.M * (16 * NT / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const float *)g.partial,
                       slices, g.M, g.N, 16 * NT, g.dst, g.d_nb0, g.d_nb1);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// ---- a plan's grouped pair-kernel launch (round 6) ----------------------------------------------
// Independent 17 <= N <= 32 Q4 nodes of one type: one gemm_skinny_pair_group_kernel launch over all of
// them and one splitk_reduce_group_kernel launch of their slab sums, with the SkinnyArgs each node's
// single launch would use (pair_geometry: the same tasks, slices and summation order, so the same bits).
// The slabs are owned by the plan (one plan must not run on two streams at once).
struct PairNodeOps { const lk_tensor *a, *b, *d; const Checked *c; };
struct PairGroupLaunch { int32_t qt = 0; int nn = 0, nred = 0; unsigned grid = 0, rgrid = 0; SkinnyArgs *nodes = nullptr;
                         ReduceNode *red = nullptr; void *slabs = nullptr; };
SkinnyArgs skinny_args(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const Checked &c);

void free_pair_group(PairGroupLaunch &pg) {
  if (pg.nodes) (void)hipFree(pg.nodes);
  if (pg.red) (void)hipFree(pg.red);
  if (pg.slabs) (void)hipFree(pg.slabs);
  pg.nodes = nullptr; pg.red = nullptr; pg.slabs = nullptr;
}

int build_pair_group(int32_t qt, const std::vector<PairNodeOps> &ops, PairGroupLaunch &pg) {
  std::vector<SkinnyArgs> nodes;
  std::vector<ReduceNode> red;
  std::vector<size_t> slab_off;
  size_t slab_total = 0;
  int64_t tasks = 0, rthreads = 0;
  // heaviest tasks first (rows per task x blocks per slice): the dispatcher hands the light ones to the
  // CUs that finish early (largest-first list scheduling); a node's bits do not depend on the order
  std::vector<PairNodeOps> ord(ops);
  auto cost = [](const PairNodeOps &o) {
    SkinnyArgs g = skinny_args(o.a, o.b, o.d, *o.c);
    (void)pair_geometry<LK_TYPE_Q4_0, 2>(g);
    return (double)g.tiles_per_range * (double)std::min<int64_t>(16, o.c->K / 32);
  };
  std::stable_sort(ord.begin(), ord.end(), [&](const PairNodeOps &x, const PairNodeOps &y) { return cost(x) > cost(y); });
  for (const auto &o : ord) {
    SkinnyArgs g = skinny_args(o.a, o.b, o.d, *o.c);
    const size_t sb = qt == LK_TYPE_Q4_0 ? pair_geometry<LK_TYPE_Q4_0, 2>(g) : pair_geometry<LK_TYPE_Q4_1, 2>(g);
    slab_off.push_back(slab_total);
    slab_total += (sb + 255) / 256 * 256;
    tasks += g.tasks;
    nodes.push_back(g);
  }
  pg.qt = qt;
  if (slab_total && hipMalloc(&pg.slabs, slab_total) != hipSuccess) {
    (void)hipGetLastError();
    pg.slabs = nullptr;
    return fail(LK_ERR_DEVICE, "plan: pair group slabs (%zu B)", slab_total);
  }
  for (size_t k = 0; k < nodes.size(); k++) {
    SkinnyArgs &g = nodes[k];
    if (g.slices > 1) {
      g.partial = (float *)((uint8_t *)pg.slabs + slab_off[k]);
      ReduceNode r{};
      r.partial = g.partial; r.dst = g.dst; r.d_nb0 = g.d_nb0; r.d_nb1 = g.d_nb1;
      r.slices = g.slices; r.M = g.M; r.N = g.N; r.N16 = 32;
      r.threads = (int64_t)g.M * 8;  // one thread per 4 of the 32 padded columns of a row
      rthreads += (r.threads + 255) / 256 * 256;
      red.push_back(r);
    }
  }
  pg.nn = (int)nodes.size();
  pg.nred = (int)red.size();
  pg.grid = (unsigned)((tasks + 7) / 8 * 8);
  pg.rgrid = (unsigned)(rthreads / 256);
  const size_t nb = nodes.size() * sizeof(SkinnyArgs), rb = red.size() * sizeof(ReduceNode);
  if (hipMalloc((void **)&pg.nodes, nb) != hipSuccess || (rb && hipMalloc((void **)&pg.red, rb) != hipSuccess) ||
      hipMemcpy(pg.nodes, nodes.data(), nb, hipMemcpyHostToDevice) != hipSuccess ||
      (rb && hipMemcpy(pg.red, red.data(), rb, hipMemcpyHostToDevice) != hipSuccess)) {
    (void)hipGetLastError();
    return fail(LK_ERR_DEVICE, "plan: pair group upload");
  }
  return LK_OK;
}

int launch_pair_group(const PairGroupLaunch &pg, hipStream_t st) {
  note_route("pairgroup<%d,2>:n%dg%u", pg.qt, pg.nn, pg.grid);
  if (pg.qt == LK_TYPE_Q4_0)
    hipLaunchKernelGGL((gemm_skinny_pair_group_kernel<LK_TYPE_Q4_0, 2>), dim3(pg.grid), dim3(512),
                       (SkinnyPairGeom<LK_TYPE_Q4_0, 2>::LDS), st, (const SkinnyArgs *)pg.nodes, pg.nn);
  else
    hipLaunchKernelGGL((gemm_skinny_pair_group_kernel<LK_TYPE_Q4_1, 2>), dim3(pg.grid), dim3(512),
                       (SkinnyPairGeom<LK_TYPE_Q4_1, 2>::LDS), st, (const SkinnyArgs *)pg.nodes, pg.nn);
  if (pg.nred) hipLaunchKernelGGL(splitk_reduce_group_kernel, dim3(pg.rgrid), dim3(256), 0, st, (const ReduceNode *)pg.red, pg.nred);
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

bool getenv_flag(const char *name);

// True when p points into device memory of some HIP device (hipMalloc / torch tensors), false for
// page-locked or pageable host memory.
bool is_device_memory(const void *p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice;
}

// gemm_kpart_kernel (lk_kpart.hpp): Q4_0 / Q4_1 at 2 <= N <= 32, K split over the waves of a
// workgroup (8·KB blocks per workgroup) and over slices of that span; per-tile sums in LDS, the
// slices' slabs summed by the last arriver. One workgroup per CU (LDS); grids may exceed the CUs.
template <int QT, int NT>
int launch_kpart_t(const SkinnyArgs &s, hipStream_t st) {
  using KG = KpartGeom<QT, NT>;
  GemmScratch &S = gemm_scratch(st);
  // the activation fragments (xsplit_kernel) in the k order of QT's code decode, and T per (block,
  // column): Q4_0 −136·Σ(hi + lo) (codes 128 + n), Q4_1 Σx (codes n·2⁻⁹)
  const int64_t nblk = s.K / 32, ntx = (s.N + 15) / 16;
  const size_t fb = (size_t)ntx * nblk * kXSplits * 64 * 16, sb = (size_t)nblk * ntx * 16 * sizeof(float);
  if (int rc = grow(S, &S.frag, &S.frag_bytes, fb + sb)) return rc;
  XSplitArgs xa{};
  xa.b = s.b;
  xa.b_nb0 = s.b_nb0; xa.b_nb1 = s.b_nb1;
  xa.N = s.N; xa.K = s.K;
  xa.frag = (u32x4 *)S.frag;
  xa.xsum = (float *)((uint8_t *)S.frag + fb);
  xa.mult = QT == LK_TYPE_Q4_0 ? -136.f : 1.f;
  xa.q4_order = QT == LK_TYPE_Q4_0 ? 2 : 1;
  KpartArgs g{};
  g.a = s.a; g.frag = xa.frag; g.xsum = xa.xsum;
  g.dst = s.dst; g.d_nb0 = s.d_nb0; g.d_nb1 = s.d_nb1;
  g.M = s.M; g.N = s.N; g.K = s.K;
  const int slices = (int)((nblk + KG::SPAN - 1) / KG::SPAN);
  const int ntile = (g.M + 15) / 16;
  // one workgroup per CU (LDS); at most 64 tiles per range (the per-wave fix-up's lane mask)
  int ranges = std::max({1, std::min(ntile, cu_count() / slices), (ntile + 63) / 64});
  const int tpr = (ntile + ranges - 1) / ranges;
  ranges = (ntile + tpr - 1) / tpr;
  g.tiles_per_range = tpr;
  g.slices = slices;
  // two K slices (C3's N = 32 at K = 4096): each adds its tile sums into dst, zeroed by the xsplit
  // launch — a + b is b + a, so the result does not depend on which slice adds first, and equals the
  // slab sum s0 + s1 (only −0.0 + −0.0 becomes +0.0). More slices: slabs and the last arriver.
  // Only into device memory: float atomics on page-locked host memory (a resident graph's direct
  // output regions, a caller's mapped buffer) go over PCIe, where their atomicity is not promised.
  static const bool no_atomic = getenv_flag("LK_KPART_NO_ATOMIC");
  g.atomic_dst = slices == 2 && !no_atomic && is_device_memory(s.dst);
  if (g.atomic_dst) {
    xa.zero = s.dst; xa.z_nb0 = s.d_nb0; xa.z_nb1 = s.d_nb1; xa.zM = s.M; xa.zN = s.N;
  } else if (slices > 1) {
    const size_t slab_bytes = (size_t)slices * g.M * 16 * NT * sizeof(float);
    if (int rc = grow(S, &S.partial, &S.partial_bytes, slab_bytes)) return rc;
    g.partial = (float *)S.partial;
    if (int rc = splitk_counters(slices, slab_bytes, ntile, true, false, st, &g.tcnt)) return rc;
  }
  g.tasks = ranges * slices;
  launch_xsplit(xa, st);
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("kpart<%d,%d>:s%dr%d%s", QT, NT, slices, ranges, g.atomic_dst ? "a" : g.tcnt ? "f" : "");
  hipLaunchKernelGGL((gemm_kpart_kernel<QT, NT>), dim3(grid), dim3(KG::NW * 64), KG::LDS, st, g);
  if (slices > 1 && !g.tcnt && !g.atomic_dst) {
    const int64_t threads = (int64_t)g.M * (16 * NT / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const float *)g.partial,
                       slices, g.M, g.N, 16 * NT, g.dst, g.d_nb0, g.d_nb1);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

SkinnyArgs skinny_args(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const Checked &c) {
  SkinnyArgs g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.b = (const uint8_t *)b->data + b->data_offset;
  g.b_nb0 = b->nb[0]; g.b_nb1 = b->nb[1];
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  g.M = (int32_t)c.M; g.N = (int32_t)c.N; g.K = (int32_t)c.K;
  // the Q4_0 pair kernel's conflict-free LDS rows read up to 8 bytes past a row piece (SkinnyPairGeom::XC)
  // (opt-in: 2.0 -> 0.2 bank-conflict cycles per LDS instruction, but C3 Q4_0 21.27 -> 21.69 us per call,
  // A/B three rounds: the shifted rows touch one more line each)
  static const bool shift = getenv_flag("LK_SKP_SHIFT");
  g.shift8 = (shift && a->type == LK_TYPE_Q4_0 && c.a_hi + 8 <= a->buf_bytes) ? 8 : 0;
  return g;
}

int launch_skinny(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  static const bool no_kpart = getenv_flag("LK_KPART_OFF");  // A/B: the round-3 skinny / pair kernels
  static const bool kpart_all = getenv_flag("LK_KPART_ALL");  // A/B: every Q4 shape on the kpart kernel
  SkinnyArgs g = skinny_args(a, b, dst, c);
  // Q4_0 / Q4_1 at N <= 16 with at most two K slices (K <= 4096) on the K-partitioned kernel (round 4:
  // the slices add into dst); otherwise the skinny / pair kernels with the slab reduce launch
  // (measured round 4: N = 8 / 16 16.2 / 16.4 vs 17.5 / 17.7 µs; C3 N = 32 23.3 vs 23.0; the down
  // projection 4096 x 11008 N = 32 28.5 vs 22.3). Q8_0 one wave per stream.
  const bool one = c.N <= 16;
  const bool kp = !no_kpart && (kpart_all || (one && (c.K / 32 + 63) / 64 <= 2));
  if (kp && a->type == LK_TYPE_Q4_0) return one ? launch_kpart_t<LK_TYPE_Q4_0, 1>(g, st) : launch_kpart_t<LK_TYPE_Q4_0, 2>(g, st);
  if (kp && a->type == LK_TYPE_Q4_1) return one ? launch_kpart_t<LK_TYPE_Q4_1, 1>(g, st) : launch_kpart_t<LK_TYPE_Q4_1, 2>(g, st);
  switch (a->type) {
    case LK_TYPE_Q4_0: return one ? launch_skinny_t<LK_TYPE_Q4_0, 1>(g, st) : launch_skinny_pair_t<LK_TYPE_Q4_0, 2>(g, st);
    case LK_TYPE_Q4_1: return one ? launch_skinny_t<LK_TYPE_Q4_1, 1>(g, st) : launch_skinny_pair_t<LK_TYPE_Q4_1, 2>(g, st);
    case LK_TYPE_Q8_0: return one ? launch_skinny_t<LK_TYPE_Q8_0, 1>(g, st) : launch_skinny_t<LK_TYPE_Q8_0, 2>(g, st);
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "skinny gemm: type %d", a->type);
  }
}

// Wide GEMM (gemm_wide_kernel): N > 32, K % 128 == 0, weight rows 8-byte aligned, and the
// last row's 80-byte window may read OVERREAD bytes past the matrix: they must be in the buffer.
bool wide_eligible(const lk_tensor *a, const Checked &c) {
  static const bool off = getenv("LK_NO_WIDE") != nullptr;  // tuning / A-B only
  if (off || c.N <= 32 || (c.K / 32) % 4) return false;
  const uint64_t bb = block_bytes(a->type);
  const uintptr_t base = (uintptr_t)a->data + a->data_offset;
  const uint64_t over = a->type == LK_TYPE_Q4_0 ? WideGeom<LK_TYPE_Q4_0>::OVERREAD
                       : a->type == LK_TYPE_Q4_1 ? WideGeom<LK_TYPE_Q4_1>::OVERREAD
                                                 : WideGeom<LK_TYPE_Q8_0>::OVERREAD;
  const uint64_t rb = (uint64_t)(c.K / 32) * bb;
  return base % 8 == 0 && rb % 8 == 0 && (uint64_t)c.M * rb < (1ull << 31) && c.a_hi + over <= a->buf_bytes;
}

template <int QT>
int launch_wide_t(WideArgs g, XSplitArgs xa, hipStream_t st) {
  if (QT == LK_TYPE_Q4_0) {  // codes 128 + n against activations in k order (0,4,1,5,...), T = −136·Σ(hi + lo)
    xa.q4_order = 2;
    xa.mult = -136.f;
  }
  using WG = WideGeom<QT>;
  GemmScratch &S = gemm_scratch(st);
  g.tiles_m = (g.M + WG::BM - 1) / WG::BM;
  g.tiles_n = (g.N + WG::BN - 1) / WG::BN;
  const int tiles = g.tiles_m * g.tiles_n;
  const int nst = g.K / 32 / WG::SB;  // stages over the whole K
  int slices = std::max(1, std::min({(cu_count() + tiles - 1) / tiles, 16, nst}));
  g.kslice = ((nst + slices - 1) / slices) * WG::SB;
  slices = (g.K / 32 + g.kslice - 1) / g.kslice;
  g.slices = slices;
  const int npad = g.tiles_n * WG::BN;
  if (slices > 1) {
    const int rc = grow(S, &S.partial, &S.partial_bytes, (size_t)slices * g.M * npad * sizeof(float));
    if (rc) return rc;
    g.partial = (float *)S.partial;
  }
  // super-tile per XCD: sm x sn tiles (all slices), minimising the XCD's L2 footprint per k:
  // sn·BN·4 B of activation fragments + sm·BM·BB/32 B of weights
  const int per_xcd = (tiles + 7) / 8;
  int best = 1;
  double cost = 1e30;
  for (int sn = 1; sn <= g.tiles_n; sn++) {
    const int sm = std::min(g.tiles_m, (per_xcd + sn - 1) / sn);
    const double c = sn * WG::BN * 4.0 + sm * WG::BM * (WG::BB / 32.0);
    if (sm * sn >= per_xcd && c < cost) { cost = c; best = sn; }
  }
  g.sn = best;
  g.sm = std::min(g.tiles_m, (per_xcd + best - 1) / best);
  const int nsuper = ((g.tiles_m + g.sm - 1) / g.sm) * ((g.tiles_n + g.sn - 1) / g.sn);
  g.tasks = nsuper * g.sm * g.sn * slices;
  // split-K fixed up inside gemm_wide_kernel by the last arriver per tile (splitk_counters)
  g.rsync = nullptr;
  if (int rf = splitk_counters(slices, (size_t)slices * g.M * npad * sizeof(float), tiles, true, true, st, &g.rsync)) return rf;
  launch_xsplit(xa, st);
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("wide<%d>:t%ds%d%s", QT, tiles, slices, g.rsync ? "f" : "");
  hipLaunchKernelGGL((gemm_wide_kernel<QT>), dim3(grid), dim3(WG::NW * 64), WG::LDS, st, g);
  if (slices > 1 && !g.rsync) {
    const int64_t threads = (int64_t)g.M * (npad / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (const float *)g.partial,
                       slices, g.M, g.N, npad, g.dst, g.d_nb0, g.d_nb1);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// Q4_0 / Q4_1 at N > 16 on gemm_w32_kernel (round 6, lk_wide32.hpp): K % 128 == 0, rows 8-B aligned, the
// last row's last window (OVERREAD bytes past the matrix) inside A's buffer, 32-bit DMA and slab offsets.
bool w32_eligible(const lk_tensor *a, const Checked &c) {
  static const bool off = getenv("LK_W32_OFF") != nullptr;  // A/B only: back to the round-5 kernels
  // N <= 32 stays on the skinny / pair / kpart kernels: the w32 shape for C3 (<Q, 3, 1, 1>, two K slices)
  // measured 24.4-24.9 us against the pair kernel's 20.5-20.9 (A/B, two rounds);
  // LK_W32_SKINNY=1 routes 17 <= N <= 32 here anyway (A/B only)
  static const bool skinny = getenv("LK_W32_SKINNY") != nullptr;
  if (off || (a->type != LK_TYPE_Q4_0 && a->type != LK_TYPE_Q4_1) || c.N <= (skinny ? 16 : 32) || c.K % 128) return false;
  const uintptr_t base = (uintptr_t)a->data + a->data_offset;
  const uint64_t bb = a->type == LK_TYPE_Q4_1 ? 20 : 18;
  const uint64_t over = a->type == LK_TYPE_Q4_1 ? W32Geom<LK_TYPE_Q4_1, 2, 2, 2>::OVERREAD : W32Geom<LK_TYPE_Q4_0, 2, 2, 2>::OVERREAD;
  const uint64_t rb = (uint64_t)(c.K / 32) * bb, ntx = (uint64_t)(c.N + 31) / 32, nblk = (uint64_t)c.K / 32;
  return base % 8 == 0 && (uint64_t)c.M * rb < (1ull << 32) && ntx * nblk * 4096 < (1ull << 32) &&
         nblk * ntx * 32 * 4 < (1ull << 32) && c.a_hi + over <= a->buf_bytes;
}

template <int QT, int MT, int NT, int MH>
int launch_w32_t(W32Args g, hipStream_t st) {
  using W = W32Geom<QT, MT, NT, MH>;
  g.tiles_m = (g.M + W::BM - 1) / W::BM;
  g.tiles_n = (g.N + W::BN - 1) / W::BN;
  const int tiles = g.tiles_m * g.tiles_n, nst = g.K / 128, cus = cu_count();
  // one workgroup per CU (~132-140 KB of LDS): split K over workgroups only when the tiles leave CUs
  // idle, at most as many slices as fit the CUs, each at least 4 stages
  int slices = std::max(1, std::min({cus / std::max(tiles, 1), nst / 4, 16}));
  g.sstages = (nst + slices - 1) / slices;
  slices = (nst + g.sstages - 1) / g.sstages;
  g.slices = slices;
  g.tasks = tiles * slices;
  // column tiles per task group: an XCD's run of tasks (about tasks / 8) covers a block of row tiles x
  // bc column tiles (LK_W32_BC overrides; A/B only). C5, A/B three rounds on one box: bc = 1 / 2 / 4 / 8
  // 52.0-52.1 / 51.9-52.3 / 52.7-53.1 / 53.3-53.5 us per call; FETCH_SIZE x 2 of the GEMM 86.6 MB at
  // bc = 1, 53.6 MB at bc = 4
  static const int bc_env = [] { const char *e = getenv("LK_W32_BC"); return e ? atoi(e) : 0; }();
  g.bc = std::max(1, std::min(bc_env > 0 ? bc_env : 2, g.tiles_n));
  if (slices > 1) {
    GemmScratch &S = gemm_scratch(st);
    const size_t pb = (size_t)slices * tiles * W::BM * W::BN * sizeof(float);
    if (pb >= (1ull << 31)) { g.slices = 1; g.sstages = nst; g.tasks = tiles; slices = 1; }
    else {
      if (int rc = grow(S, &S.partial, &S.partial_bytes, pb)) return rc;
      g.partial = (float *)S.partial;
      if (int rc = splitk_counters(slices, pb, tiles, true, true, st, &g.tcnt)) return rc;
      if (!g.tcnt) return fail(LK_ERR_DEVICE, "w32: no split-K counters");
    }
  }
  const unsigned grid = (unsigned)((g.tasks + 7) / 8 * 8);
  note_route("w32<%d,%d,%d,%d>:t%ds%d", QT, MT, NT, MH, tiles, slices);
  w32_launch(QT, MT, NT, MH, g, grid, W::LDS, st);
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

int launch_w32(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  GemmScratch &S = gemm_scratch(st);
  const int64_t nblk = c.K / 32, ntx = (c.N + 31) / 32;
  const size_t fb = (size_t)ntx * nblk * 4 * 1024, tb = (size_t)nblk * ntx * 32 * sizeof(float);
  int rc = grow(S, &S.frag, &S.frag_bytes, fb + tb);
  if (rc) return rc;
  XSplit32Args xa{};
  xa.b = (const uint8_t *)b->data + b->data_offset;
  xa.b_nb0 = b->nb[0]; xa.b_nb1 = b->nb[1];
  xa.N = (int32_t)c.N; xa.K = (int32_t)c.K;
  xa.frag = (u32x4 *)S.frag;
  xa.tsum = (float *)((uint8_t *)S.frag + fb);
  xa.mult = a->type == LK_TYPE_Q4_1 ? -128.f : -136.f;
  W32Args g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.frag = xa.frag;
  g.tsum = xa.tsum;
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  g.M = (int32_t)c.M; g.N = (int32_t)c.N; g.K = (int32_t)c.K;
  w32_launch_xsplit(xa, (unsigned)(ntx * nblk), st);
  const bool q41 = a->type == LK_TYPE_Q4_1;
  static const int cfg = [] { const char *e = getenv("LK_W32_CFG"); return e ? atoi(e) : 0; }();  // A/B only
  if (c.N > 32) {
    if (cfg == 1) return q41 ? launch_w32_t<LK_TYPE_Q4_1, 4, 2, 1>(g, st) : launch_w32_t<LK_TYPE_Q4_0, 4, 2, 1>(g, st);
    return q41 ? launch_w32_t<LK_TYPE_Q4_1, 2, 2, 2>(g, st) : launch_w32_t<LK_TYPE_Q4_0, 2, 2, 2>(g, st);
  }
  return q41 ? launch_w32_t<LK_TYPE_Q4_1, 3, 1, 1>(g, st) : launch_w32_t<LK_TYPE_Q4_0, 3, 1, 1>(g, st);
}

int launch_gemm(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  GemmScratch &S = gemm_scratch(st);
  const int64_t nblk = c.K / 32, ntx = (c.N + 15) / 16;
  const size_t fb = (size_t)ntx * nblk * kXSplits * 64 * 16, sb = (size_t)nblk * ntx * 16 * sizeof(float);
  int rc = grow(S, &S.frag, &S.frag_bytes, fb + sb);
  if (rc) return rc;
  XSplitArgs xa{};
  xa.b = (const uint8_t *)b->data + b->data_offset;
  xa.b_nb0 = b->nb[0]; xa.b_nb1 = b->nb[1];
  xa.N = c.N; xa.K = c.K;
  xa.frag = (u32x4 *)S.frag;
  xa.xsum = (float *)((uint8_t *)S.frag + fb);
  xa.mult = a->type == LK_TYPE_Q4_0 ? GemmQ<LK_TYPE_Q4_0>::MULT : 1.f;
  xa.q4_order = a->type != LK_TYPE_Q8_0;
  if (wide_eligible(a, c)) {
    WideArgs w{};
    w.a = (const uint8_t *)a->data + a->data_offset;
    w.frag = xa.frag;
    w.xsum = xa.xsum;
    w.dst = (uint8_t *)dst->data + dst->data_offset;
    w.d_nb0 = dst->nb[0]; w.d_nb1 = dst->nb[1];
    w.M = (int32_t)c.M; w.N = (int32_t)c.N; w.K = (int32_t)c.K;
    switch (a->type) {
      case LK_TYPE_Q4_0: return launch_wide_t<LK_TYPE_Q4_0>(w, xa, st);
      case LK_TYPE_Q4_1: return launch_wide_t<LK_TYPE_Q4_1>(w, xa, st);
      case LK_TYPE_Q8_0: return launch_wide_t<LK_TYPE_Q8_0>(w, xa, st);
      default: break;
    }
  }
  const bool lds_ok = gemm_lds_eligible(a->type, a, c);
  GemmArgs g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.frag = xa.frag;
  g.xsum = xa.xsum;
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  g.M = (int32_t)c.M; g.N = (int32_t)c.N; g.K = (int32_t)c.K;
  switch (a->type) {
    case LK_TYPE_Q4_0: return launch_gemm_qt<LK_TYPE_Q4_0>(g, xa, lds_ok, st);
    case LK_TYPE_Q4_1: return launch_gemm_qt<LK_TYPE_Q4_1>(g, xa, lds_ok, st);
    case LK_TYPE_Q8_0: return launch_gemm_qt<LK_TYPE_Q8_0>(g, xa, lds_ok, st);
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "gemm: type %d", a->type);
  }
}

GenericArgs make_generic(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c) {
  GenericArgs g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.b = (const uint8_t *)b->data + b->data_offset;
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.M = c.M; g.N = c.N; g.K = c.K;
  g.a_nb0 = a->nb[0]; g.a_nb1 = a->nb[1];
  g.b_nb0 = b->nb[0]; g.b_nb1 = b->nb[1];
  g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  return g;
}

int launch_generic(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st);

bool getenv_flag(const char *name) {  // lab switches (A/B only): callers read them once into a static
  const char *e = getenv(name);
  return e && *e && *e != '0';
}

// F32 x F32 -> F32 on the f32 MFMA (f32_mfma_kernel): any strides; float4 loads of A's rows when
// they are contiguous and 16-byte aligned.
int launch_f32_mfma(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  static const bool f32_direct = getenv_flag("LK_F32_DIRECT");
  const GenericArgs g = make_generic(a, b, dst, c);
  const int64_t gx = (c.N + 31) / 32, gy = (c.M + 31) / 32;
  if (gx > 0x7FFFFFFF || gy > 65535) return launch_generic(a, b, dst, c, st);
  dim3 grid((unsigned)gx, (unsigned)gy), block(256);
  const bool v4 = g.a_nb0 == 4 && g.a_nb1 % 16 == 0 && ((uintptr_t)g.a & 15) == 0;
  const bool dense = v4 && g.b_nb0 == 4 && g.b_nb1 % 16 == 0 && ((uintptr_t)g.b & 15) == 0 && c.K % kF32Chunk == 0 &&
                     c.N % 4 == 0 && (c.M - 1) * g.a_nb1 + 4 * c.K < (1ll << 32) && c.K * g.b_nb1 < (1ll << 32) &&
                     !f32_direct;
  note_route(dense ? "f32_lds" : v4 ? "f32_mfma<1>" : "f32_mfma<0>");
  if (dense) hipLaunchKernelGGL(f32_lds_kernel, grid, block, 4 * 32768, st, g);
  else if (v4) hipLaunchKernelGGL(f32_mfma_kernel<true>, grid, block, 0, st, g);
  else hipLaunchKernelGGL(f32_mfma_kernel<false>, grid, block, 0, st, g);
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

int launch_generic(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  const GenericArgs g = make_generic(a, b, dst, c);
  const int64_t waves = c.M * c.N;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > (int64_t)INT32_MAX) return fail(LK_ERR_NOT_IMPLEMENTED, "output too large for the generic kernel");
  dim3 grid((unsigned)blocks), block(256);
  int32_t t = (c.path == Path::kQuantF32) ? a->type : (c.path == Path::kF32 ? LK_TYPE_F32 : LK_TYPE_F16);
  note_route("generic<%d>", t);
  switch (t) {
    case LK_TYPE_Q4_0: hipLaunchKernelGGL(mul_mat_generic_kernel<LK_TYPE_Q4_0>, grid, block, 0, st, g); break;
    case LK_TYPE_Q4_1: hipLaunchKernelGGL(mul_mat_generic_kernel<LK_TYPE_Q4_1>, grid, block, 0, st, g); break;
    case LK_TYPE_Q8_0: hipLaunchKernelGGL(mul_mat_generic_kernel<LK_TYPE_Q8_0>, grid, block, 0, st, g); break;
    case LK_TYPE_F32: hipLaunchKernelGGL(mul_mat_generic_kernel<LK_TYPE_F32>, grid, block, 0, st, g); break;
    case LK_TYPE_F16: hipLaunchKernelGGL(mul_mat_generic_kernel<LK_TYPE_F16>, grid, block, 0, st, g); break;
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "generic: type %d", t);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

template <int QT, int NC, bool VX, bool AL>
void launch_kq_gemv_t(const KQuantArgs &g, hipStream_t st) {
  dim3 grid((unsigned)((g.M + 3) / 4), (unsigned)((g.N + NC - 1) / NC)), block(256);
  hipLaunchKernelGGL((kquant_gemv_kernel<QT, NC, VX, AL>), grid, block, 0, st, g);
}

template <int QT>
void launch_kq_gemv(const KQuantArgs &g, bool vx, bool al, hipStream_t st) {
  if (g.N == 1) {
    if (vx) al ? launch_kq_gemv_t<QT, 1, true, true>(g, st) : launch_kq_gemv_t<QT, 1, true, false>(g, st);
    else al ? launch_kq_gemv_t<QT, 1, false, true>(g, st) : launch_kq_gemv_t<QT, 1, false, false>(g, st);
  } else {
    al ? launch_kq_gemv_t<QT, 4, false, true>(g, st) : launch_kq_gemv_t<QT, 4, false, false>(g, st);
  }
}

template <int QT>
void launch_kq_nc(int nc, dim3 grid, dim3 block, size_t lds, hipStream_t st, const KQuantArgs &g) {
  if (nc == 8) hipLaunchKernelGGL((kquant_nc_kernel<QT, 8, 16>), grid, block, lds, st, g);
  else if (nc == 4) hipLaunchKernelGGL((kquant_nc_kernel<QT, 4, 16>), grid, block, lds, st, g);
  else hipLaunchKernelGGL((kquant_nc_kernel<QT, 2, 16>), grid, block, lds, st, g);
}

// K-quant x F32. K % 256 == 0: kquant_gemv_kernel (a wave per row and 1 or 4 columns);
// otherwise (the Kotlin full-block quirk / flat partial path) kquant_mul_mat_kernel, one wave
// per output. LK_KQ_LEGACY (set) forces the latter (lab A/B).
int launch_kquant(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  note_route("kquant<%d>", a->type);
  KQuantArgs g{};
  g.a = (const uint8_t *)a->data + a->data_offset;
  g.b = (const uint8_t *)b->data + b->data_offset;
  g.dst = (uint8_t *)dst->data + dst->data_offset;
  g.b_nb0 = b->nb[0]; g.b_nb1 = b->nb[1]; g.d_nb0 = dst->nb[0]; g.d_nb1 = dst->nb[1];
  g.M = c.M; g.N = c.N; g.K = c.K;
  static const bool legacy = getenv("LK_KQ_LEGACY") != nullptr;  // A/B only
  if (!legacy && c.K % LK_QK_K == 0 && (c.M + 3) / 4 <= (int64_t)INT32_MAX && (c.N + 3) / 4 <= 65535) {
    const bool al = ((uintptr_t)g.a & 3) == 0;
    const bool vx = g.b_nb1 == 4 && ((uintptr_t)g.b & 15) == 0;
    static const bool no_n1 = getenv("LK_NO_KQ_N1") != nullptr;  // A/B only
    const size_t xlds = (size_t)(c.K / 32) * 36 * sizeof(float);
    const uintptr_t need = a->type == LK_TYPE_Q4_K ? 15 : 3;
    // Q4_K at batch 1 on the LDS-DMA stream kernel (a unit = 16 blocks = 64 lanes x 64 items,
    // the same 2304 B as a Q4_0 unit): rows split over one workgroup per CU, x staged once.
    // LK_KQ_STREAM=0 keeps kquant_n1_kernel (lab A/B).
    static const bool kq_stream = [] { const char *e = getenv("LK_KQ_STREAM"); return !e || atoi(e) != 0; }();
    // Q2_K between 2K and 6K rows stays on kquant_n1_kernel: its 1344-B units leave the stream
    // kernel two per wave there, and the one-shot latency wins (4096^2: 5.45 vs 5.86 us; from
    // 6144 rows on, and under 2K, the stream kernel is ahead: round-2 lab run q2k_run.sh)
    const bool q2k_mid = a->type == LK_TYPE_Q2_K && c.M > 2048 && c.M < 6144;
    if (kq_stream && !no_n1 && !q2k_mid && gemv_eligible(a, b, dst, c))
      if (const int cls = stream_class(a, c))
        return launch_stream(a->type, cls, stream_grid(c.M), make_desc(a, b, dst, c), nullptr, 0, st);
    if (!no_n1 && c.N == 1 && ((uintptr_t)g.a & need) == 0 && xlds <= 64 * 1024) {
      const dim3 grid((unsigned)((c.M + 15) / 16)), block(1024);
      switch (a->type) {
        case LK_TYPE_Q2_K: hipLaunchKernelGGL((kquant_n1_kernel<LK_TYPE_Q2_K, 16>), grid, block, xlds, st, g); break;
        case LK_TYPE_Q4_K: hipLaunchKernelGGL((kquant_n1_kernel<LK_TYPE_Q4_K, 16>), grid, block, xlds, st, g); break;
        default: hipLaunchKernelGGL((kquant_n1_kernel<LK_TYPE_Q8_K, 16>), grid, block, xlds, st, g); break;
      }
      HIP_TRY(hipGetLastError());
      return LK_OK;
    }
    // Q4_K at 16 <= N <= 32: the wave-pair MFMA kernel (lk_skinny.hpp; one Q4_K block per wave
    // and unit, affine weights within the F32 bar); smaller batches keep the exact-decode kernels
    // below (their weights are the Kotlin values bit for bit). LK_KQ_SK=0: lab A/B.
    static const bool kq_sk = [] { const char *e = getenv("LK_KQ_SK"); return !e || atoi(e) != 0; }();
    if (kq_sk && a->type == LK_TYPE_Q4_K && c.N >= 16 && c.N <= 32 && ((uintptr_t)g.a & 15) == 0 &&
        (uint64_t)(c.K / LK_QK_K) * LK_Q4_K_BLOCK_BYTES * 16 < (1ull << 31))
      return c.N <= 16 ? launch_sk_t<LK_TYPE_Q4_K, 1>(a, b, dst, c, st) : launch_sk_t<LK_TYPE_Q4_K, 2>(a, b, dst, c, st);
    // batch > 1: NC columns per workgroup staged in LDS (NC = 8 / 4 / 2 as K allows)
    const size_t col_lds = (size_t)(c.K / 32) * 36 * sizeof(float);
    int nc = 0;
    for (int cand : {8, 4, 2})
      if (nc == 0 && (int64_t)cand <= ((c.N + 1) / 2) * 2 && cand * col_lds <= 150 * 1024) nc = cand;
    if (!no_n1 && c.N > 1 && nc && ((uintptr_t)g.a & need) == 0 && (c.M + 31) / 32 <= 65535) {
      const dim3 grid((unsigned)((c.N + nc - 1) / nc), (unsigned)((c.M + 31) / 32)), block(1024);  // 32 rows
      const size_t lds = nc * col_lds;
      switch (a->type) {
        case LK_TYPE_Q2_K: launch_kq_nc<LK_TYPE_Q2_K>(nc, grid, block, lds, st, g); break;
        case LK_TYPE_Q4_K: launch_kq_nc<LK_TYPE_Q4_K>(nc, grid, block, lds, st, g); break;
        default: launch_kq_nc<LK_TYPE_Q8_K>(nc, grid, block, lds, st, g); break;
      }
      HIP_TRY(hipGetLastError());
      return LK_OK;
    }
    switch (a->type) {
      case LK_TYPE_Q2_K: launch_kq_gemv<LK_TYPE_Q2_K>(g, vx, al, st); break;
      case LK_TYPE_Q4_K: launch_kq_gemv<LK_TYPE_Q4_K>(g, vx, al, st); break;
      case LK_TYPE_Q8_K: launch_kq_gemv<LK_TYPE_Q8_K>(g, vx, al, st); break;
      default: return fail(LK_ERR_NOT_IMPLEMENTED, "K-quant: type %d", a->type);
    }
    HIP_TRY(hipGetLastError());
    return LK_OK;
  }
  const int64_t blocks = (c.M * c.N + 3) / 4;
  if (blocks > (int64_t)INT32_MAX) return fail(LK_ERR_NOT_IMPLEMENTED, "output too large for the K-quant kernel");
  dim3 grid((unsigned)blocks), block(256);
  switch (a->type) {
    case LK_TYPE_Q2_K: hipLaunchKernelGGL(kquant_mul_mat_kernel<LK_TYPE_Q2_K>, grid, block, 0, st, g); break;
    case LK_TYPE_Q4_K: hipLaunchKernelGGL(kquant_mul_mat_kernel<LK_TYPE_Q4_K>, grid, block, 0, st, g); break;
    case LK_TYPE_Q8_K: hipLaunchKernelGGL(kquant_mul_mat_kernel<LK_TYPE_Q8_K>, grid, block, 0, st, g); break;
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "K-quant: type %d", a->type);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

// Single eligible GEMV: the descriptor travels in the kernel arguments (no
// allocation, no host sync: stream-ordered and graph-capturable).
int run_single_gemv(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  const GemvDesc d = make_desc(a, b, dst, c);
  if (const int cls = stream_class(a, c))
    return launch_stream(a->type, cls, stream_grid(c.M), d, nullptr, 0, st);
  return launch_gemv_v1(a->type, d, st);
}

// True when mul_mat_device_checked would run these operands on gemm_skinny_pair_kernel with the slab-sum
// launch after it (Q4_0 / Q4_1, 17 <= N <= 32, not w32 / kpart): the nodes a plan may group (lk_plan_launch).
bool pair_routed(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const Checked &c) {
  static const bool kpart_all = getenv_flag("LK_KPART_ALL");
  if (c.empty || c.K == 0 || c.path == Path::kKQuantF32 || c.path == Path::kF32) return false;
  if (a->type != LK_TYPE_Q4_0 && a->type != LK_TYPE_Q4_1) return false;
  if (c.N <= 16 || c.N > 32 || kpart_all) return false;
  if (gemv_eligible(a, b, dst, c) || !gemm_eligible(c) || w32_eligible(a, c) || !skinny_eligible(a, c)) return false;
  return true;
}

int mul_mat_device_checked(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c, hipStream_t st) {
  if (c.empty) return LK_OK;
  if (c.K == 0) { // every dot product is the empty sum: dst := 0 (F32 or F16 +0.0)
    if (dst->nb[0] == (c.path == Path::kF16 ? 2u : 4u) && dst->nb[1] == dst->nb[0] * (uint64_t)c.N) {
      HIP_TRY(hipMemsetAsync((uint8_t *)dst->data + dst->data_offset, 0, (size_t)(c.d_hi - c.d_lo), st));
      return LK_OK;
    }
    return launch_generic(a, b, dst, c, st);
  }
  if (c.path == Path::kKQuantF32) return launch_kquant(a, b, dst, c, st);
  static const bool no_f32_mfma = getenv_flag("LK_NO_F32_MFMA");
  if (c.path == Path::kF32 && !no_f32_mfma) return launch_f32_mfma(a, b, dst, c, st);
  if (gemv_eligible(a, b, dst, c)) return run_single_gemv(a, b, dst, c, st);
  if (gemm_eligible(c)) {
    if (w32_eligible(a, c)) return launch_w32(a, b, dst, c, st);
    return skinny_eligible(a, c) ? launch_skinny(a, b, dst, c, st) : launch_gemm(a, b, dst, c, st);
  }
  return launch_generic(a, b, dst, c, st);
}

int ensure_scratch(Dev &s, int idx, size_t bytes) {
  if (s.scratch_bytes[idx] >= bytes) return LK_OK;
  if (s.scratch[idx]) HIP_TRY(hipFree(s.scratch[idx]));
  s.scratch[idx] = nullptr;
  s.scratch_bytes[idx] = 0;
  size_t want = std::max<size_t>(bytes, 1 << 20);
  HIP_TRY(hipMalloc(&s.scratch[idx], want));
  s.scratch_bytes[idx] = want;
  return LK_OK;
}

// Lazily create the library stream on the caller's CURRENT device (a rank that
// selected device r keeps device r) and report that device. The host entry points work on the
// device this returns — the calling thread's own HIP device — never on a process-wide field
// another thread may change meanwhile (lk_mul_mat_sharded_at's P = 1 path used to
// set S().device without the lock and leave it changed).
int ensure_init(int *dev_out = nullptr) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev < 0 || dev >= kMaxDevices || !S().devs[dev].stream || !S().devs[dev].fail_flag) {
    int rc = lk_init(dev);
    if (rc) return rc;
  }
  if (dev_out) *dev_out = dev;
  return LK_OK;
}

// The library stream of device d (created on first use); leaves d current.
int init_dev(int d) {
  HIP_TRY(hipSetDevice(d));
  Dev &v = S().devs[d];
  if (!v.stream) HIP_TRY(hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking));
  if (!v.fail_flag) {  // the word a device-side wait raises when it gives up (lk_note_timeout)
    unsigned *f = nullptr;
    HIP_TRY(hipHostMalloc((void **)&f, 64, hipHostMallocCoherent));
    *(volatile unsigned *)f = 0;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(lk_sync_fail_flag), &f, sizeof(f)));
    v.fail_flag = f;
  }
  return LK_OK;
}

// The failure word of device d before a synchronous entry point's launches (lk_note_timeout
// stores the device's running count of waits that gave up into it).
unsigned fail_mark(int d) {
  Dev &v = S().devs[d];
  return v.fail_flag ? __atomic_load_n(v.fail_flag, __ATOMIC_ACQUIRE) : 0u;
}

// After a host synchronisation of device d: LK_ERR_DEVICE when the word moved since `before`,
// i.e. a device-side wait gave up while this call's launches ran — their results are undefined.
// Each call compares against its own mark, so a failure is never consumed by another thread's
// call (a concurrent failure on the same device may be reported by both).
int sync_failures(int d, unsigned before) {
  if (fail_mark(d) == before) return LK_OK;
  return fail(LK_ERR_DEVICE,
              "device %d: a split-K or chain wait gave up at its bound (workgroups not co-resident: another launch "
              "shares the GPU); the results of that launch are undefined", d);
}

// The current mirror covering host bytes [lo, hi) of base on this device, or null.
MirrorRef find_pinned(Dev &v, const void *base, uint64_t lo, uint64_t hi) {
  std::lock_guard<std::mutex> lk(S().cache_mu);
  for (auto &m : v.weights)
    if (m->covers((uintptr_t)base, lo, hi)) return m;
  return nullptr;
}

// Drop (and mark stale) every current mirror of `base` on v overlapping [lo, hi) whose
// generation is not `keep_gen` (all of them when keep_all is false). Caller holds cache_mu.
int drop_overlapping(Dev &v, uintptr_t base, uint64_t lo, uint64_t hi, bool keep_same_gen, uint64_t keep_gen) {
  int n = 0;
  for (size_t i = 0; i < v.weights.size();) {
    Mirror &m = *v.weights[i];
    if (m.overlaps(base, lo, hi) && !(keep_same_gen && m.gen == keep_gen)) {
      m.stale = true;
      v.weight_bytes -= m.bytes;
      v.weights.erase(v.weights.begin() + i);
      n++;
    } else {
      i++;
    }
  }
  return n;
}

// Make host bytes [lo, lo + bytes) of a->data current on device d (the caller made d
// current) as of `generation`: a current mirror of the same generation covering them is
// kept; mirrors of other generations overlapping them are superseded (host bytes rewritten).
int pin_on(int d, const lk_tensor *a, uint64_t lo, uint64_t bytes, uint64_t generation, MirrorRef *out = nullptr) {
  Dev &v = S().devs[d];
  const uintptr_t base = (uintptr_t)a->data;
  std::lock_guard<std::mutex> lk(S().cache_mu);
  for (auto &m : v.weights)
    if (m->gen == generation && m->covers(base, lo, lo + bytes)) {
      if (out) *out = m;
      return LK_OK;
    }
  drop_overlapping(v, base, lo, lo + bytes, true, generation);
  auto m = std::make_shared<Mirror>();
  m->dev = d; m->base = base; m->lo = lo; m->bytes = bytes; m->gen = generation;
  HIP_TRY(hipMalloc(&m->ptr, bytes + kASlack));
  HIP_TRY(hipMemcpy(m->ptr, (const uint8_t *)a->data + lo, bytes, hipMemcpyHostToDevice));
  v.weights.push_back(m);
  v.weight_bytes += bytes;
  if (out) *out = m;
  return LK_OK;
}

// Bytes a pin of `a` covers (its whole tensor), as lk_weights_pin computes them.
uint64_t pin_bytes(const lk_tensor *a) {
  if (is_q(a->type)) return (uint64_t)(t_num_elements(a) / 32) * block_bytes(a->type);
  if (is_kq(a->type)) return (uint64_t)(t_num_elements(a) / 256) * kblock_bytes(a->type);
  return (uint64_t)t_num_elements(a) * (a->type == LK_TYPE_F16 ? 2 : 4);
}

int evict_range(uintptr_t base, uint64_t lo, uint64_t hi) {
  std::lock_guard<std::mutex> lk(S().cache_mu);
  int n = 0;
  for (auto &v : S().devs) n += drop_overlapping(v, base, lo, hi, false, 0);
  return n;
}

}  // namespace

// ============================================================================
// C-ABI
// ============================================================================

extern "C" {

const char *lk_version(void) { return "lk_hip 0.1 (gfx950)"; }

const char *lk_last_error(void) { return g_err.c_str(); }

const char *lk_debug_route(void) { return g_route.c_str(); }

void lk_debug_route_clear(void) { g_route.clear(); }

// Test hook: store `value` into gemm_q_*'s split-K tile counter `index` of the
// (current device, stream) scratch, allocating the counters if needed; stream-ordered on `stream`.
int lk_debug_poke_gemm_counter(void *stream, int64_t index, int32_t value) {
  int rc = ensure_init();
  if (rc) return rc;
  if (index < 0 || index >= (1 << 20)) return fail(LK_ERR_INVALID_ARG, "counter index %lld", (long long)index);
  hipStream_t st = pick_stream(stream);
  int32_t *ctr = nullptr;
  if ((rc = gemm_counters((size_t)index + 1, st, &ctr))) return rc;
  HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(ctr + index), value, 1, st));
  HIP_TRY(hipStreamSynchronize(st));
  return LK_OK;
}

// Frees the batched-kernel scratch (activation fragments, split-K slabs, counters, retired buffers)
// of (current device, stream) after synchronising that stream (the per-stream map never
// shrank). The caller guarantees that no HIP graph it will replay captured a launch on that stream.
int lk_scratch_release(void *stream) {
  int rc = ensure_init();
  if (rc) return rc;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(LK_ERR_DEVICE, "scratch release: no device");
  hipStream_t st = pick_stream(stream);
  HIP_TRY(hipStreamSynchronize(st));
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  auto it = scratch_map().find(ScratchKey{dev, st});
  if (it == scratch_map().end()) return LK_OK;
  GemmScratch &G = it->second;
  for (void *p : G.retired) HIP_TRY(hipFree(p));
  for (void *p : {G.frag, G.partial, (void *)G.counter, (void *)G.tcnt})
    if (p) HIP_TRY(hipFree(p));
  scratch_map().erase(it);
  return LK_OK;
}

// Device bytes held by the batched-kernel scratch of the current device, all streams (live + retired).
uint64_t lk_scratch_bytes(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  uint64_t t = 0;
  for (auto &kv : scratch_map())
    if (kv.first.dev == dev) {
      const GemmScratch &G = kv.second;
      t += G.frag_bytes + G.partial_bytes + G.counter_n * sizeof(int32_t) + G.tcnt_n * sizeof(unsigned) + G.retired_bytes;
    }
  return t;
}

uint64_t lk_debug_scratch_epoch(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  uint64_t e = 0;
  for (auto &kv : scratch_map())
    if (kv.first.dev == dev) e += kv.second.epoch;
  return e;
}

int lk_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int lk_init(int device) {
  State &s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(LK_ERR_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n || device >= kMaxDevices)
    return fail(LK_ERR_INVALID_ARG, "device %d out of range (%d devices)", device, n);
  int rc = init_dev(device);
  if (rc) return rc;
  s.device = device;
  return LK_OK;
}

void lk_weights_evict_all(void) {
  std::vector<MirrorRef> gone;  // freed after the lock is released (hipFree synchronizes)
  {
    std::lock_guard<std::mutex> lk(S().cache_mu);
    for (auto &v : S().devs) {
      for (auto &m : v.weights) { m->stale = true; gone.push_back(m); }
      v.weights.clear();
      v.weight_bytes = 0;
    }
  }
}

int lk_weights_evict(const lk_tensor *a) {
  if (!a) return fail(LK_ERR_INVALID_ARG, "evict: null tensor");
  if (!a->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  const uint64_t bytes = pin_bytes(a);
  evict_range((uintptr_t)a->data, a->data_offset, a->data_offset + std::max<uint64_t>(bytes, 1));
  return LK_OK;
}

int lk_weights_evict_buffer(const void *data, uint64_t buf_bytes) {
  if (!data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  evict_range((uintptr_t)data, 0, std::max<uint64_t>(buf_bytes, 1));
  return LK_OK;
}

uint64_t lk_weights_cached_bytes(void) {
  std::lock_guard<std::mutex> lk(S().cache_mu);
  uint64_t t = 0;
  for (auto &v : S().devs) t += v.weight_bytes;
  return t;
}

uint64_t lk_weights_cached_count(void) {
  std::lock_guard<std::mutex> lk(S().cache_mu);
  uint64_t t = 0;
  for (auto &v : S().devs) t += v.weights.size();
  return t;
}

void lk_shutdown(void) {
  State &s = S();
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int d = 0; d < kMaxDevices; d++) {
    Dev &v = s.devs[d];
    if (!v.stream) continue;
    (void)hipSetDevice(d);
    (void)hipStreamSynchronize(v.stream);
    for (int i = 0; i < 3; i++) {
      if (v.scratch[i]) (void)hipFree(v.scratch[i]);
      v.scratch[i] = nullptr;
      v.scratch_bytes[i] = 0;
    }
    (void)hipStreamDestroy(v.stream);
    v.stream = nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto &kv : scratch_map()) {
      (void)hipSetDevice(kv.first.dev);
      (void)hipDeviceSynchronize();
      GemmScratch &G = kv.second;
      for (void *p : G.retired) (void)hipFree(p);
      for (void *p : {G.frag, G.partial, (void *)G.counter, (void *)G.tcnt})
        if (p) (void)hipFree(p);
    }
    scratch_map().clear();
  }
  lk_weights_evict_all();
  (void)hipSetDevice(prev);
  s.device = -1;
}

int lk_mul_mat_validate(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst) {
  Checked c;
  return check(a, b, dst, &c);
}

int lk_mul_mat_device(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, void *stream) {
  Checked c;
  int rc = check(a, b, dst, &c);
  if (rc) return rc;
  return mul_mat_device_checked(a, b, dst, c, pick_stream(stream));
}

int lk_weights_pin(const lk_tensor *a, uint64_t generation) {
  int dev = 0;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (!a || !a->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  const uint64_t bytes = pin_bytes(a);
  if (a->data_offset + bytes > a->buf_bytes) return fail(LK_ERR_OUT_OF_BOUNDS, "pin: tensor exceeds its buffer");
  return pin_on(dev, a, a->data_offset, bytes, generation);
}

// Host-buffer operator: the Kotlin drop-in. ByteArrays stay authoritative; A comes
// from the residency cache when a current mirror covers its bytes (the latest generation
// pinned over them: older ones were superseded), otherwise it is staged per call.
namespace {
// The host operator on device `dev` (current on this thread; its state initialised by the caller).
int mul_mat_host_on(int dev, const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, const Checked &c) {
  int rc = LK_OK;
  Dev &s = S().devs[dev];
  hipStream_t st = s.stream;
  const unsigned mark = fail_mark(dev);
  const uint64_t a_bytes = c.a_hi - c.a_lo, b_bytes = c.b_hi - c.b_lo, d_bytes = c.d_hi - c.d_lo;
  // A: cached mirror or staged copy
  const MirrorRef pinned = find_pinned(s, a->data, c.a_lo, c.a_hi);  // held for the call
  const void *a_dev = pinned ? (const uint8_t *)pinned->ptr + (c.a_lo - pinned->lo) : nullptr;
  if (pinned) note_route("A=mirror[%llu,+%llu)g%llu", (unsigned long long)pinned->lo, (unsigned long long)pinned->bytes,
                         (unsigned long long)pinned->gen);
  else note_route("A=staged");
  if (!a_dev && a_bytes) {
    if ((rc = ensure_scratch(s, 0, a_bytes + kASlack))) return rc;
    HIP_TRY(hipMemcpyAsync(s.scratch[0], (const uint8_t *)a->data + c.a_lo, a_bytes, hipMemcpyHostToDevice, st));
    a_dev = s.scratch[0];
  }
  if ((rc = ensure_scratch(s, 1, std::max<uint64_t>(b_bytes, 16)))) return rc;
  if ((rc = ensure_scratch(s, 2, d_bytes))) return rc;
  if (b_bytes) HIP_TRY(hipMemcpyAsync(s.scratch[1], (const uint8_t *)b->data + c.b_lo, b_bytes, hipMemcpyHostToDevice, st));
  // strided dst: preserve the bytes between written elements
  HIP_TRY(hipMemcpyAsync(s.scratch[2], (const uint8_t *)dst->data + c.d_lo, d_bytes, hipMemcpyHostToDevice, st));
  lk_tensor da = *a, db = *b, dd = *dst;
  // A's device copy (mirror or staging) has kASlack readable bytes past the matrix
  da.data = const_cast<void *>(a_dev); da.data_offset = 0;
  da.buf_bytes = pinned ? pinned->lo + pinned->bytes + kASlack - c.a_lo : a_bytes + kASlack;
  db.data = s.scratch[1]; db.data_offset = 0; db.buf_bytes = b_bytes;
  dd.data = s.scratch[2]; dd.data_offset = 0; dd.buf_bytes = d_bytes;
  Checked cd = c;
  cd.a_lo = 0; cd.a_hi = a_bytes; cd.b_lo = 0; cd.b_hi = b_bytes; cd.d_lo = 0; cd.d_hi = d_bytes;
  rc = mul_mat_device_checked(&da, &db, &dd, cd, st);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync((uint8_t *)dst->data + c.d_lo, s.scratch[2], d_bytes, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return sync_failures(dev, mark);
}
}  // namespace

int lk_mul_mat(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst) {
  Checked c;
  int rc = check(a, b, dst, &c);
  if (rc) return rc;
  if (c.empty) return LK_OK;
  int dev = 0;
  if ((rc = ensure_init(&dev))) return rc;
  return mul_mat_host_on(dev, a, b, dst, c);
}

// ---- row-sharded host operator: one process, several GPUs (SURVEY §8b lk_mul_mat_sharded) -----
//
// Shard r owns rows [r·⌈M/P⌉, …) of A (whole blocks: contiguous bytes) and the same rows
// of dst (ggml_hip/sharded.py shard_rows). Shard r runs on device r mod (visible devices),
// so P may exceed the device count (shards on one device run back to back on its stream).
// No collective: each shard writes its own disjoint rows of the host dst (D2H), which is
// the all-gather of the in-process case. Work is issued on every device before any result
// is read back, so the kernels of different devices overlap.

namespace {

void shard_span(int64_t M, int P, int r, int64_t *r0, int64_t *r1) {
  const int64_t per = (M + P - 1) / P;
  *r0 = std::min<int64_t>((int64_t)r * per, M);
  *r1 = std::min<int64_t>(*r0 + per, M);
}

// Row pitch of A in bytes when rows can be cut as byte ranges, else 0.
uint64_t a_row_pitch(const lk_tensor *a) {
  if (is_q(a->type)) return a->ne[0] % 32 ? 0 : (uint64_t)(a->ne[0] / 32) * block_bytes(a->type);
  return a->nb[1];
}

struct Shard {
  int dev;
  lk_tensor a, d;
  Checked c;
  MirrorRef pin;  // held for the call
  const void *a_dev;
  uint64_t a_stage_off, d_off;
};

}  // namespace

int lk_weights_pin_sharded(const lk_tensor *a, uint64_t generation, int n_shards) {
  return lk_weights_pin_sharded_at(a, generation, n_shards, 0);
}

int lk_weights_pin_sharded_at(const lk_tensor *a, uint64_t generation, int n_shards, int first_device) {
  if (!a || !a->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(LK_ERR_DEVICE, "no HIP device visible");
  if (n_shards < 1) return fail(LK_ERR_INVALID_ARG, "n_shards %d", n_shards);
  const uint64_t pitch = a_row_pitch(a);
  if (!pitch || !is_q(a->type)) return fail(LK_ERR_NOT_IMPLEMENTED, "pin_sharded: quantized A with K %% 32 == 0 only");
  if (a->data_offset + (uint64_t)a->ne[1] * pitch > a->buf_bytes)
    return fail(LK_ERR_OUT_OF_BOUNDS, "pin: tensor exceeds its buffer");
  int prev = 0;
  (void)hipGetDevice(&prev);
  int rc = LK_OK;
  for (int r = 0; r < n_shards && rc == LK_OK; r++) {
    int64_t r0, r1;
    shard_span(a->ne[1], n_shards, r, &r0, &r1);
    if (r1 <= r0) continue;
    const int d = (first_device + r) % std::min(ndev, kMaxDevices);
    if ((rc = init_dev(d))) break;
    rc = pin_on(d, a, a->data_offset + (uint64_t)r0 * pitch, (uint64_t)(r1 - r0) * pitch, generation);
  }
  (void)hipSetDevice(prev);
  return rc;
}

int lk_mul_mat_sharded(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int n_shards) {
  return lk_mul_mat_sharded_at(a, b, dst, n_shards, 0);
}

int lk_mul_mat_sharded_at(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int n_shards, int first_device) {
  Checked c;
  int rc = check(a, b, dst, &c);
  if (rc) return rc;
  if (n_shards < 1) return fail(LK_ERR_INVALID_ARG, "n_shards %d", n_shards);
  if (first_device < 0) return fail(LK_ERR_INVALID_ARG, "first_device %d", first_device);
  if (c.empty) return LK_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(LK_ERR_DEVICE, "no HIP device visible");
  ndev = std::min(ndev, kMaxDevices);
  // Rows must be byte ranges of A, and dst rows must not interleave (each shard copies
  // its dst span back whole): otherwise one device computes everything.
  const uint64_t pitch = a_row_pitch(a);
  const uint64_t ew = dst->type == LK_TYPE_F16 ? 2 : 4;
  const bool rows_ok = pitch && (uint64_t)(c.N - 1) * dst->nb[0] + ew <= dst->nb[1];
  const int P = rows_ok ? (int)std::min<int64_t>(n_shards, c.M) : 1;
  if (P == 1) {  // one device: first_device's (explicitly: no process-wide device field is touched)
    int prev = 0;
    (void)hipGetDevice(&prev);
    const int d = first_device % ndev;
    int rc1;
    {
      std::lock_guard<std::mutex> lk(S().mu);  // init_dev creates the stream / flag once
      rc1 = init_dev(d);
    }
    if (rc1 == LK_OK) rc1 = mul_mat_host_on(d, a, b, dst, c);
    (void)hipSetDevice(prev);
    return rc1;
  }

  int prev = 0;
  (void)hipGetDevice(&prev);
  std::vector<Shard> sh;
  for (int r = 0; r < P; r++) {
    int64_t r0, r1;
    shard_span(c.M, P, r, &r0, &r1);
    if (r1 <= r0) continue;
    Shard x{};
    x.dev = (first_device + r) % ndev;
    x.a = *a; x.a.ne[1] = r1 - r0; x.a.data_offset = a->data_offset + (uint64_t)r0 * pitch;
    x.d = *dst; x.d.ne[1] = r1 - r0; x.d.data_offset = dst->data_offset + (uint64_t)r0 * dst->nb[1];
    if ((rc = check(&x.a, b, &x.d, &x.c))) return rc;
    sh.push_back(x);
  }
  // per device: B once, A from the pin cache or staged, one dst span per shard
  const uint64_t b_bytes = c.b_hi - c.b_lo;
  std::vector<uint64_t> a_need(ndev, 0), d_need(ndev, 0);
  std::vector<char> used(ndev, 0);
  std::vector<unsigned> mark(ndev, 0);
  for (auto &x : sh) {
    if ((rc = init_dev(x.dev))) goto out;
    Dev &v = S().devs[x.dev];
    if (!used[x.dev]) mark[x.dev] = fail_mark(x.dev);
    used[x.dev] = 1;
    x.pin = find_pinned(v, a->data, x.c.a_lo, x.c.a_hi);
    x.a_dev = x.pin ? (const uint8_t *)x.pin->ptr + (x.c.a_lo - x.pin->lo) : nullptr;
    x.a_stage_off = a_need[x.dev];
    if (!x.a_dev) a_need[x.dev] += (x.c.a_hi - x.c.a_lo + kASlack + 255) & ~255ull;
    x.d_off = d_need[x.dev];
    d_need[x.dev] += (x.c.d_hi - x.c.d_lo + 255) & ~255ull;
  }
  for (int d = 0; d < ndev; d++) {
    if (!used[d]) continue;
    Dev &v = S().devs[d];
    if ((rc = init_dev(d))) goto out;
    if ((rc = ensure_scratch(v, 0, std::max<uint64_t>(a_need[d], 16)))) goto out;
    if ((rc = ensure_scratch(v, 1, std::max<uint64_t>(b_bytes, 16)))) goto out;
    if ((rc = ensure_scratch(v, 2, std::max<uint64_t>(d_need[d], 16)))) goto out;
    if (b_bytes && hipMemcpyAsync(v.scratch[1], (const uint8_t *)b->data + c.b_lo, b_bytes, hipMemcpyHostToDevice,
                                  v.stream) != hipSuccess) { rc = fail(LK_ERR_DEVICE, "sharded: B upload"); goto out; }
  }
  for (auto &x : sh) {
    Dev &v = S().devs[x.dev];
    if ((rc = init_dev(x.dev))) goto out;
    const uint64_t ab = x.c.a_hi - x.c.a_lo, db = x.c.d_hi - x.c.d_lo;
    const void *a_dev = x.a_dev;
    if (!a_dev) {
      a_dev = (uint8_t *)v.scratch[0] + x.a_stage_off;
      if (hipMemcpyAsync((void *)a_dev, (const uint8_t *)a->data + x.c.a_lo, ab, hipMemcpyHostToDevice, v.stream) !=
          hipSuccess) { rc = fail(LK_ERR_DEVICE, "sharded: A upload"); goto out; }
    }
    void *d_dev = (uint8_t *)v.scratch[2] + x.d_off;
    if (hipMemcpyAsync(d_dev, (const uint8_t *)dst->data + x.c.d_lo, db, hipMemcpyHostToDevice, v.stream) !=
        hipSuccess) { rc = fail(LK_ERR_DEVICE, "sharded: dst upload"); goto out; }
    lk_tensor da = x.a, dbt = *b, dd = x.d;
    da.data = const_cast<void *>(a_dev); da.data_offset = 0;
    da.buf_bytes = x.pin ? x.pin->lo + x.pin->bytes + kASlack - x.c.a_lo : ab + kASlack;
    dbt.data = v.scratch[1]; dbt.data_offset = 0; dbt.buf_bytes = b_bytes;
    dd.data = d_dev; dd.data_offset = 0; dd.buf_bytes = db;
    Checked cd = x.c;
    cd.a_lo = 0; cd.a_hi = ab; cd.b_lo = 0; cd.b_hi = b_bytes; cd.d_lo = 0; cd.d_hi = db;
    if ((rc = mul_mat_device_checked(&da, &dbt, &dd, cd, v.stream))) goto out;
  }
  for (auto &x : sh) {  // read back in issue order: every device's kernels are in flight
    Dev &v = S().devs[x.dev];
    if ((rc = init_dev(x.dev))) goto out;
    if (hipMemcpyAsync((uint8_t *)dst->data + x.c.d_lo, (uint8_t *)v.scratch[2] + x.d_off, x.c.d_hi - x.c.d_lo,
                       hipMemcpyDeviceToHost, v.stream) != hipSuccess) { rc = fail(LK_ERR_DEVICE, "sharded: dst read"); goto out; }
  }
  for (int d = 0; d < ndev; d++)
    if (used[d] && hipStreamSynchronize(S().devs[d].stream) != hipSuccess && rc == LK_OK)
      rc = fail(LK_ERR_DEVICE, "sharded: device %d failed", d);
  for (int d = 0; d < ndev; d++)
    if (used[d] && rc == LK_OK) rc = sync_failures(d, mark[d]);
out:
  (void)hipSetDevice(prev);
  return rc;
}

// ---- plans: independent MUL_MAT nodes, one launch per quant type ---------------------------
//
// Stream-eligible nodes of one class share a launch: the concatenated rows are split
// into one contiguous, byte-balanced range per workgroup (one workgroup per CU), cut at
// node boundaries into segments.

struct lk_plan {
  struct Group { int32_t qt; int cls; int grid; int spw; StreamWork *work; };
  std::vector<Group> groups;
  // independent 17 <= N <= 32 Q4 nodes of one type in one gemm_skinny_pair_group_kernel launch plus one
  // splitk_reduce_group_kernel launch (round 6); slabs owned by the plan, so one plan must not run on two
  // streams at once (as a chain plan's barrier words)
  std::vector<PairGroupLaunch> pairs;
  struct Single { lk_tensor a, b, d; Checked c; };
  std::vector<Single> singles;
  unsigned *sync = nullptr;  // chain plans: barrier counters, exit counter, timeout flag
  int nbar = 0;
  const PeerDesc *peer = nullptr;  // one rank of a multi-GPU chain (lk_p2p_chain): device PeerDesc
#ifdef LK_PF
  const StreamWork *pf_work = nullptr;  // lab: the successor plan's first group (same grid)
  int pf_spw = 0;
#endif
};

namespace {

// A plan's singles that run on the pair kernel, two or more of one quant type, become one grouped launch
// (PairGroupLaunch, built before the extern "C" section; LK_PLAN_NO_PAIR_GROUP=1: one launch pair per node,
// as before; A/B only).
int group_pair_singles(lk_plan *plan) {
  static const bool off = getenv_flag("LK_PLAN_NO_PAIR_GROUP");
  // only nodes small enough that their per-launch fixed cost matters (LK_PLAN_PAIR_GROUP_MB overrides; A/B)
  static const double max_mb = [] { const char *e = getenv("LK_PLAN_PAIR_GROUP_MB"); return e ? atof(e) : 1e9; }();
  if (off) return LK_OK;
  for (int32_t qt : {LK_TYPE_Q4_0, LK_TYPE_Q4_1}) {
    std::vector<lk_plan::Single> mine, rest;
    for (auto &sg : plan->singles) {
      const double mb = (double)sg.c.M * (double)(sg.c.K / 32) * (qt == LK_TYPE_Q4_0 ? 18 : 20) / 1e6;
      (sg.a.type == qt && mb <= max_mb && pair_routed(&sg.a, &sg.b, &sg.d, sg.c) ? mine : rest).push_back(sg);
    }
    if (mine.size() < 2) continue;
    std::vector<PairNodeOps> ops;
    for (auto &sg : mine) ops.push_back({&sg.a, &sg.b, &sg.d, &sg.c});
    plan->pairs.emplace_back();
    const int rc = build_pair_group(qt, ops, plan->pairs.back());  // freed by lk_plan_destroy on failure too
    if (rc) return rc;
    plan->singles.swap(rest);
  }
  return LK_OK;
}

// Workgroup g gets global rows [bound[g], bound[g+1]) of the concatenation of descs,
// balanced by weight bytes, cut at node boundaries into segments.
void split_rows(const std::vector<GemvDesc> &descs, int32_t qt, int grid, std::vector<std::vector<StreamWork>> &per);

// Adjacent nodes that read the same activations and whose weight rows and output rows continue each
// other in memory (a model's q, k and v projections allocated back to back; gate and up) become one
// node, so the launch's rows split evenly over its waves: per-node workgroup shares gave the q, k, v
// stage 48 or 49 rows per workgroup (85.3 workgroups per node), and the 49-row workgroups' waves ran a
// seventh row and ended the launch ~0.8 µs late (lab stamps). Same bits either way:
// every row is one wave's dot. LK_NO_MERGE=1 keeps the nodes apart (A/B).
void merge_adjacent(std::vector<GemvDesc> &descs, int32_t qt) {
  static const bool off = [] {
    const char *e = std::getenv("LK_NO_MERGE");
    return e && *e == '1';
  }();
  if (off || descs.size() < 2) return;
  const int64_t pb = stream_pair_bytes(qt);
  std::vector<GemvDesc> out;
  for (const GemvDesc &d : descs) {
    if (!out.empty()) {
      GemvDesc &p = out.back();
      const int64_t row_bytes = (int64_t)(p.K / 64) * pb;
      if (p.x == d.x && p.K == d.K && p.dst_row_stride == d.dst_row_stride && d.a == p.a + (int64_t)p.M * row_bytes &&
          d.dst == p.dst + (int64_t)p.M * p.dst_row_stride && (int64_t)p.M + d.M <= INT32_MAX) {
        p.M += d.M;
        continue;
      }
    }
    out.push_back(d);
  }
  descs.swap(out);
}

void build_work(const std::vector<GemvDesc> &descs, int32_t qt, int grid, std::vector<StreamWork> &work, int *spw) {
  std::vector<std::vector<StreamWork>> per;
  split_rows(descs, qt, grid, per);
  size_t most = 1;
  for (auto &v : per) most = std::max(most, v.size());
  *spw = (int)most;
  work.assign((size_t)grid * most, StreamWork{});
  for (int g = 0; g < grid; g++) {
    for (size_t k = 0; k < per[g].size(); k++) work[(size_t)g * most + k] = per[g][k];
    work[(size_t)g * most].count = (int32_t)per[g].size();
  }
}

// LK_STRADDLE=1 (lab A/B): the old byte-balanced cut, where a workgroup may straddle two nodes
const bool g_straddle = [] {
  const char *e = std::getenv("LK_STRADDLE");
  return e && *e == '1';
}();

// Whole nodes per workgroup when there are workgroups enough: node i gets a share wg[i] of the
// grid proportional to its bytes (largest remainder, at least one), its rows split evenly over
// them (workgroup k of the node: rows [M·k/wg, M·(k+1)/wg)). A workgroup then runs ONE segment:
// no second prologue (activation image, ring refill) behind a workgroup barrier halfway through,
// which left the straddling workgroups ~3 µs behind the rest of a Llama-7B layer launch. The byte
// imbalance the rounding leaves is under 1 % on the Llama shapes. One node: the whole grid.
// False when the grid is too small for whole nodes (or LK_STRADDLE=1): split_rows then cuts
// the concatenated rows by bytes.
bool whole_node_shares(const std::vector<GemvDesc> &descs, int32_t qt, int grid, std::vector<int> &wg) {
  const int64_t pb = stream_pair_bytes(qt);
  const size_t n = descs.size();
  if (n == 1) {
    wg.assign(1, (int)std::min<int64_t>(grid, std::max<int64_t>(1, descs[0].M)));
    return !g_straddle;
  }
  int64_t all_bytes = 0;
  std::vector<int64_t> nbytes(n);
  for (size_t i = 0; i < n; i++) all_bytes += nbytes[i] = (int64_t)descs[i].M * (descs[i].K / 64) * pb;
  if (g_straddle || (int)n > grid / 2 || all_bytes <= 0) return false;
  {
    wg.assign(n, 0);
    std::vector<std::pair<double, size_t>> rem;
    int used = 0;
    for (size_t i = 0; i < n; i++) {
      const double share = (double)grid * nbytes[i] / all_bytes;
      wg[i] = std::max(1, (int)share);
      wg[i] = (int)std::min<int64_t>(wg[i], std::max<int64_t>(1, descs[i].M));
      used += wg[i];
      rem.push_back({share - (int)share, i});
    }
    std::sort(rem.begin(), rem.end(), [](const std::pair<double, size_t> &x, const std::pair<double, size_t> &y) {
      return x.first > y.first;
    });
    for (size_t k = 0; used < grid && k < rem.size(); k++) {
      const size_t i = rem[k].second;
      if (wg[i] < descs[i].M) { wg[i]++; used++; }
    }
    while (used > grid) {  // the at-least-one floor overshot: take from the widest nodes
      size_t w = 0;
      for (size_t i = 1; i < n; i++) if (wg[i] > wg[w]) w = i;
      wg[w]--; used--;
    }
  }
  return true;
}

void split_rows(const std::vector<GemvDesc> &descs, int32_t qt, int grid, std::vector<std::vector<StreamWork>> &per) {
  const int64_t pb = stream_pair_bytes(qt);
  const size_t n = descs.size();
  std::vector<int> wg;
  if (whole_node_shares(descs, qt, grid, wg)) {
    per.assign(grid, {});
    int g = 0;
    for (size_t i = 0; i < n; i++) {
      for (int k = 0; k < wg[i]; k++, g++) {
        const int64_t lo = descs[i].M * k / wg[i], hi = descs[i].M * (k + 1) / wg[i];
        if (lo >= hi) continue;
        StreamWork w{};
        w.a = descs[i].a; w.x = descs[i].x; w.dst = descs[i].dst; w.dst_row_stride = descs[i].dst_row_stride;
        w.K = descs[i].K; w.row_begin = (int32_t)lo; w.row_end = (int32_t)hi;
        per[g].push_back(w);
      }
    }
    return;
  }
  std::vector<int64_t> row0(n + 1, 0), byte0(n + 1, 0);
  for (size_t i = 0; i < n; i++) {
    row0[i + 1] = row0[i] + descs[i].M;
    byte0[i + 1] = byte0[i] + (int64_t)descs[i].M * (descs[i].K / 64) * pb;
  }
  const int64_t total = byte0[n];
  std::vector<int64_t> bound(grid + 1);
  for (int g = 0; g <= grid; g++) {
    const int64_t target = (int64_t)((__int128)total * g / grid);
    size_t i = 0;
    while (i + 1 < n && byte0[i + 1] <= target) i++;
    const int64_t rb = (descs[i].K / 64) * pb;
    int64_t r = rb ? (target - byte0[i] + rb - 1) / rb : 0;
    r = std::min<int64_t>(std::max<int64_t>(r, 0), descs[i].M);
    bound[g] = (g == grid) ? row0[n] : row0[i] + r;
  }
  per.assign(grid, {});
  for (int g = 0; g < grid; g++) {
    for (size_t i = 0; i < n; i++) {
      const int64_t lo = std::max(bound[g], row0[i]), hi = std::min(bound[g + 1], row0[i + 1]);
      if (lo >= hi) continue;
      StreamWork w{};
      w.a = descs[i].a; w.x = descs[i].x; w.dst = descs[i].dst; w.dst_row_stride = descs[i].dst_row_stride;
      w.K = descs[i].K; w.row_begin = (int32_t)(lo - row0[i]); w.row_end = (int32_t)(hi - row0[i]);
      per[g].push_back(w);
    }
  }
}

}  // namespace

int lk_plan_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n, lk_plan **out) {
  if (!out || n < 0) return fail(LK_ERR_INVALID_ARG, "bad plan arguments");
  int rc = ensure_init();
  if (rc) return rc;
  auto plan = new lk_plan();
  // one launch per quant type: the kernel instance for the largest units-per-row class
  // also runs the nodes with fewer units (same occupancy: 8 waves per CU either way)
  std::map<int32_t, std::vector<GemvDesc>> by_type;
  std::map<int32_t, int> type_cls;
  for (int i = 0; i < n; i++) {
    Checked c;
    rc = check(&a[i], &b[i], &dst[i], &c);
    if (rc) { lk_plan_destroy(plan); return rc; }
    if (c.empty) continue;
    const int cls = gemv_eligible(&a[i], &b[i], &dst[i], c) ? stream_class(&a[i], c) : 0;
    if (cls) {
      by_type[a[i].type].push_back(make_desc(&a[i], &b[i], &dst[i], c));
      type_cls[a[i].type] = std::max(type_cls[a[i].type], cls);
    }
    else plan->singles.push_back({a[i], b[i], dst[i], c});
  }
  if ((rc = group_pair_singles(plan))) { lk_plan_destroy(plan); return rc; }
  for (auto &kv : by_type) {
    const int32_t qt = kv.first;
    const int cls = type_cls[qt];
    auto &descs = kv.second;
    merge_adjacent(descs, qt);
    int64_t rows = 0;
    for (auto &d : descs) rows += d.M;
    const int grid = stream_grid(rows);
    std::vector<StreamWork> work;
    int spw = 1;
    build_work(descs, qt, grid, work, &spw);
    void *dev = nullptr;
    const size_t wb = work.size() * sizeof(StreamWork);
    if (hipMalloc(&dev, wb) != hipSuccess) { lk_plan_destroy(plan); return fail(LK_ERR_DEVICE, "plan alloc"); }
    plan->groups.push_back({qt, cls, grid, spw, (StreamWork *)dev});
    if (hipMemcpy(dev, work.data(), wb, hipMemcpyHostToDevice) != hipSuccess) {
      lk_plan_destroy(plan);
      return fail(LK_ERR_DEVICE, "plan upload");
    }
  }
  *out = plan;
  return LK_OK;
}

// Chain plans: dependent stages in one launch of the streaming GEMV, one grid barrier per stage
// boundary (gemv_stream_kernel's chain mode). One workgroup per CU, all co-resident (the
// kernel's LDS admits one per CU).
// Chain plan on `grid` workgroups of the current device; peer: a device PeerDesc (a rank of a
// multi-GPU chain, lk_p2p.hip) or null.
int lk_detail_chain_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage, int n,
                           int grid, const void *peer, lk_plan **out);

int lk_plan_create_chain(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage, int n,
                         lk_plan **out) {
  if (!out || n <= 0 || !stage) return fail(LK_ERR_INVALID_ARG, "bad chain arguments");
  int rc = ensure_init();
  if (rc) return rc;
  return lk_detail_chain_create(a, b, dst, stage, n, cu_count(), nullptr, out);
}

int lk_detail_chain_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage, int n,
                           int grid, const void *peer, lk_plan **out) {
  if (!out || n <= 0 || !stage || grid < 1) return fail(LK_ERR_INVALID_ARG, "bad chain arguments");
  int rc = LK_OK;
  std::vector<std::vector<GemvDesc>> stages;
  int32_t qt = -1;
  int cls = 0;
  for (int i = 0; i < n; i++) {
    if (stage[i] < 0 || (i > 0 && stage[i] < stage[i - 1]) || stage[i] > (i ? stage[i - 1] + 1 : 0))
      return fail(LK_ERR_INVALID_ARG, "chain: stage ids must start at 0 and grow by at most 1 (node %d)", i);
    Checked c;
    if ((rc = check(&a[i], &b[i], &dst[i], &c))) return rc;
    if (c.empty || !gemv_eligible(&a[i], &b[i], &dst[i], c) || !stream_class(&a[i], c))
      return fail(LK_ERR_NOT_IMPLEMENTED, "chain: node %d is not a streaming GEMV node", i);
    if (qt >= 0 && a[i].type != qt) return fail(LK_ERR_NOT_IMPLEMENTED, "chain: one quant type per chain");
    qt = a[i].type;
    cls = std::max(cls, stream_class(&a[i], c));
    if ((int)stages.size() <= stage[i]) stages.emplace_back();
    stages[stage[i]].push_back(make_desc(&a[i], &b[i], &dst[i], c));
  }
  const int nbar = (int)stages.size() - 1;
  auto plan = new lk_plan();
  plan->nbar = nbar;
  plan->peer = (const PeerDesc *)peer;
  const size_t sync_bytes = (size_t)(nbar * 9 + 2) * kChainLine * sizeof(unsigned);
  if (hipMalloc(&plan->sync, sync_bytes) != hipSuccess || hipMemset(plan->sync, 0, sync_bytes) != hipSuccess) {
    lk_plan_destroy(plan);
    return fail(LK_ERR_DEVICE, "chain: sync alloc");
  }
  std::vector<std::vector<StreamWork>> per(grid);
  for (size_t s = 0; s < stages.size(); s++) {
    std::vector<std::vector<StreamWork>> ps;
    merge_adjacent(stages[s], qt);
    split_rows(stages[s], qt, grid, ps);
    for (int g = 0; g < grid; g++) {
      if (ps[g].empty()) {  // no rows here: the workgroup still takes part in the barrier
        StreamWork w{};
        w.a = stages[s][0].a; w.x = stages[s][0].x; w.dst = stages[s][0].dst; w.dst_row_stride = stages[s][0].dst_row_stride;
        w.K = stages[s][0].K;
        ps[g].push_back(w);
      }
      ps[g][0].barrier = (int32_t)s;  // barrier #s−1 before stage s (none before stage 0)
      for (auto &w : ps[g]) per[g].push_back(w);
    }
  }
  size_t most = 1;
  for (auto &v : per) most = std::max(most, v.size());
  std::vector<StreamWork> work((size_t)grid * most, StreamWork{});
  for (int g = 0; g < grid; g++) {
    for (size_t k = 0; k < per[g].size(); k++) {
      per[g][k].nbar = nbar;
      per[g][k].sync = plan->sync;
      work[(size_t)g * most + k] = per[g][k];
    }
    work[(size_t)g * most].count = (int32_t)per[g].size();
  }
  void *dev = nullptr;
  const size_t wb = work.size() * sizeof(StreamWork);
  if (hipMalloc(&dev, wb) != hipSuccess) { lk_plan_destroy(plan); return fail(LK_ERR_DEVICE, "plan alloc"); }
  plan->groups.push_back({qt, cls, grid, (int)most, (StreamWork *)dev});
  if (hipMemcpy(dev, work.data(), wb, hipMemcpyHostToDevice) != hipSuccess) {
    lk_plan_destroy(plan);
    return fail(LK_ERR_DEVICE, "plan upload");
  }
  *out = plan;
  return LK_OK;
}

int lk_plan_chain_timed_out(lk_plan *plan) {
  if (!plan || !plan->sync) return 0;
  unsigned flag = 0;
  if (hipDeviceSynchronize() != hipSuccess) return fail(LK_ERR_DEVICE, "chain: sync");
  const int words = (plan->nbar * 9 + 2) * kChainLine;
  if (hipMemcpy(&flag, plan->sync + words - kChainLine, sizeof(flag), hipMemcpyDeviceToHost) != hipSuccess) return fail(LK_ERR_DEVICE, "chain: flag");
  if (flag) {
    (void)hipMemset(plan->sync, 0, (size_t)words * sizeof(unsigned));
    return 1;
  }
  return 0;
}

int lk_sync_timeouts(uint32_t *count) {
  if (!count) return fail(LK_ERR_INVALID_ARG, "null count");
  int dev = 0;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  unsigned v = 0;
  if (hipDeviceSynchronize() != hipSuccess) return fail(LK_ERR_DEVICE, "sync");
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(lk_sync_timeout_count), sizeof(v)) != hipSuccess)
    return fail(LK_ERR_DEVICE, "timeout count");
  Dev &d = S().devs[dev];  // the device count is monotonic: report the increase since the last call
  *count = v - d.timeouts_seen;
  d.timeouts_seen = v;
  return LK_OK;
}

int lk_set_sync_wait_bound(uint64_t ticks) {
  int rc = ensure_init();
  if (rc) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(lk_sync_wait_bound), &ticks, sizeof(ticks)));
  return LK_OK;
}

int lk_sync_counters_sum(uint64_t *sum) {
  if (!sum) return fail(LK_ERR_INVALID_ARG, "null sum");
  int rc = ensure_init();
  if (rc) return rc;
  *sum = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  HIP_TRY(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (auto &kv : scratch_map()) {  // every stream's scratch on this device
    if (kv.first.dev != dev) continue;
    const GemmScratch &G = kv.second;
    if (G.tcnt) {
      std::vector<unsigned> w(G.tcnt_n);
      HIP_TRY(hipMemcpy(w.data(), G.tcnt, w.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
      for (unsigned x : w) *sum += x;
    }
    if (G.counter) {  // gemm_q_mfma_kernel / gemm_q_lds_kernel tile counters
      std::vector<int32_t> w(G.counter_n);
      HIP_TRY(hipMemcpy(w.data(), G.counter, w.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
      for (int32_t x : w) *sum += (uint32_t)x;
    }
  }
  return LK_OK;
}

int lk_plan_launch(lk_plan *plan, void *stream) {
  if (!plan) return fail(LK_ERR_INVALID_ARG, "null plan");
  hipStream_t st = pick_stream(stream);
  for (size_t k = 0; k < plan->groups.size(); k++) {
    auto &g = plan->groups[k];
    GemvDesc pf{};
#ifdef LK_PF
    if (k + 1 == plan->groups.size() && plan->pf_work) {  // lab: the last group prefetches for the successor
      pf.a = (const uint8_t *)plan->pf_work;
      pf.M = plan->pf_spw;
    }
#endif
    int rc = launch_stream(g.qt, g.cls, g.grid, pf, g.work, g.spw, st, plan->peer);
    if (rc) return rc;
  }
  for (auto &pg : plan->pairs) {
    int rc = launch_pair_group(pg, st);
    if (rc) return rc;
  }
  for (auto &s : plan->singles) {
    int rc = mul_mat_device_checked(&s.a, &s.b, &s.d, s.c, st);
    if (rc) return rc;
  }
  return LK_OK;
}

#ifdef LK_PF
// lab only (not in include/lk_hip.h): plan's last launch prefetches `next`'s first units per wave;
// `next` must outlive every launch of `plan`. NULL unlinks.
extern "C" int lk_plan_prefetch_next(lk_plan *plan, const lk_plan *next) {
  if (!plan) return fail(LK_ERR_INVALID_ARG, "null plan");
  plan->pf_work = nullptr;
  plan->pf_spw = 0;
  if (!next || plan->sync || next->sync || plan->groups.empty() || next->groups.empty()) return LK_OK;
  const auto &a = plan->groups.back(), &b = next->groups.front();
  if (a.grid != b.grid || a.qt != b.qt) return LK_OK;  // same grid and block type only
  plan->pf_work = b.work;
  plan->pf_spw = b.spw;
  return LK_OK;
}
#endif

int lk_plan_num_launches(const lk_plan *plan) {
  return plan ? (int)(plan->groups.size() + plan->pairs.size() + plan->singles.size()) : 0;
}

void lk_plan_destroy(lk_plan *plan) {
  if (!plan) return;
  for (auto &g : plan->groups) (void)hipFree(g.work);
  for (auto &pg : plan->pairs) free_pair_group(pg);
  if (plan->sync) (void)hipFree(plan->sync);
  delete plan;
}

// ---- format kernels ----------------------------------------------------------------

int lk_dequantize_device(const lk_tensor *src, float *out, void *stream) {
  if (!src) return fail(LK_ERR_INVALID_ARG, "null tensor");
  if (!is_q(src->type)) return fail(LK_ERR_NOT_IMPLEMENTED, "dequantize: type %d not offloaded", src->type);
  if (!src->data || !out) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  const int64_t nblk = t_num_elements(src) / 32;
  if (src->data_offset + (uint64_t)nblk * block_bytes(src->type) > src->buf_bytes)
    return fail(LK_ERR_OUT_OF_BOUNDS, "dequantize: blocks exceed buffer");
  if (nblk == 0) return LK_OK;
  hipStream_t st = pick_stream(stream);
  const uint8_t *p = (const uint8_t *)src->data + src->data_offset;
  static const bool legacy = getenv("LK_FORMAT_LEGACY") != nullptr;  // A/B only
  if (!legacy && ((uintptr_t)p & 1) == 0 && ((uintptr_t)out & 15) == 0 && (nblk + 31) / 32 <= (int64_t)UINT32_MAX) {
    dim3 g8((unsigned)((nblk + 31) / 32)), b8(256);  // eight lanes per block
    switch (src->type) {
      case LK_TYPE_Q4_0: hipLaunchKernelGGL(dequantize_coop_kernel<LK_TYPE_Q4_0>, g8, b8, 0, st, p, out, nblk); break;
      case LK_TYPE_Q4_1: hipLaunchKernelGGL(dequantize_coop_kernel<LK_TYPE_Q4_1>, g8, b8, 0, st, p, out, nblk); break;
      default: hipLaunchKernelGGL(dequantize_coop_kernel<LK_TYPE_Q8_0>, g8, b8, 0, st, p, out, nblk); break;
    }
    HIP_TRY(hipGetLastError());
    return LK_OK;
  }
  dim3 grid((unsigned)((nblk + 255) / 256)), block(256);
  switch (src->type) {
    case LK_TYPE_Q4_0: hipLaunchKernelGGL(dequantize_kernel<LK_TYPE_Q4_0>, grid, block, 0, st, p, out, nblk); break;
    case LK_TYPE_Q4_1: hipLaunchKernelGGL(dequantize_kernel<LK_TYPE_Q4_1>, grid, block, 0, st, p, out, nblk); break;
    default: hipLaunchKernelGGL(dequantize_kernel<LK_TYPE_Q8_0>, grid, block, 0, st, p, out, nblk); break;
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

int lk_quantize_device(const float *src, int64_t n, int32_t type, void *out, void *stream) {
  if (!is_q(type)) return fail(LK_ERR_NOT_IMPLEMENTED, "quantize: type %d not offloaded", type);
  if (n % 32 != 0) return fail(LK_ERR_INVALID_ARG, "numElements %lld not div by 32", (long long)n); /* :1062, :1074, :1089 */
  if (n == 0) return LK_OK;
  if (!src || !out) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  hipStream_t st = pick_stream(stream);
  const int64_t nblk = n / 32;
  static const bool legacy = getenv("LK_FORMAT_LEGACY") != nullptr;  // A/B only
  if (!legacy && ((uintptr_t)src & 15) == 0 && ((uintptr_t)out & 1) == 0 && (nblk + 31) / 32 <= (int64_t)UINT32_MAX) {
    dim3 g8((unsigned)((nblk + 31) / 32)), b8(256);  // eight lanes per block
    switch (type) {
      case LK_TYPE_Q4_0: hipLaunchKernelGGL(quantize_coop_kernel<LK_TYPE_Q4_0>, g8, b8, 0, st, src, (uint8_t *)out, nblk); break;
      case LK_TYPE_Q4_1: hipLaunchKernelGGL(quantize_coop_kernel<LK_TYPE_Q4_1>, g8, b8, 0, st, src, (uint8_t *)out, nblk); break;
      default: hipLaunchKernelGGL(quantize_coop_kernel<LK_TYPE_Q8_0>, g8, b8, 0, st, src, (uint8_t *)out, nblk); break;
    }
    HIP_TRY(hipGetLastError());
    return LK_OK;
  }
  dim3 grid((unsigned)((nblk + 255) / 256)), block(256);
  switch (type) {
    case LK_TYPE_Q4_0: hipLaunchKernelGGL(quantize_kernel<LK_TYPE_Q4_0>, grid, block, 0, st, src, (uint8_t *)out, nblk); break;
    case LK_TYPE_Q4_1: hipLaunchKernelGGL(quantize_kernel<LK_TYPE_Q4_1>, grid, block, 0, st, src, (uint8_t *)out, nblk); break;
    default: hipLaunchKernelGGL(quantize_kernel<LK_TYPE_Q8_0>, grid, block, 0, st, src, (uint8_t *)out, nblk); break;
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

int lk_repack_q4_device(void *blocks, int64_t n_blocks, int32_t type, int32_t direction, void *stream) {
  if (type != LK_TYPE_Q4_0 && type != LK_TYPE_Q4_1)
    return fail(LK_ERR_NOT_IMPLEMENTED, "repack: type %d has no nibble-order variant", type);
  if (direction != LK_REPACK_UPSTREAM_TO_KOTLIN && direction != LK_REPACK_KOTLIN_TO_UPSTREAM)
    return fail(LK_ERR_INVALID_ARG, "repack: direction %d", direction);
  if (n_blocks < 0) return fail(LK_ERR_INVALID_ARG, "repack: n_blocks %lld", (long long)n_blocks);
  if (n_blocks == 0) return LK_OK;
  if (!blocks) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  if ((uintptr_t)blocks & 1) return fail(LK_ERR_INVALID_ARG, "repack: blocks not 2-byte aligned");
  hipStream_t st = pick_stream(stream);
  uint8_t *p = (uint8_t *)blocks;
  dim3 grid((unsigned)((n_blocks + 255) / 256)), block(256);
  if (type == LK_TYPE_Q4_0) {
    if (direction == 0) hipLaunchKernelGGL((repack_q4_kernel<LK_TYPE_Q4_0, 0>), grid, block, 0, st, p, n_blocks);
    else hipLaunchKernelGGL((repack_q4_kernel<LK_TYPE_Q4_0, 1>), grid, block, 0, st, p, n_blocks);
  } else {
    if (direction == 0) hipLaunchKernelGGL((repack_q4_kernel<LK_TYPE_Q4_1, 0>), grid, block, 0, st, p, n_blocks);
    else hipLaunchKernelGGL((repack_q4_kernel<LK_TYPE_Q4_1, 1>), grid, block, 0, st, p, n_blocks);
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

}  // extern "C"

// ---- graph residency over host buffers ----------------------------------
//
// A sequence of MUL_MAT nodes over host ByteArrays, analysed once: quantized weights are
// pinned on the device, every activation byte range (B operands, F32/F16 A operands, dst)
// gets one device mirror, nodes are levelled by their read/write overlaps, and each level
// becomes one lk_plan. A compute uploads only the graph's inputs (ranges no earlier node
// produces, plus strided dst ranges whose gap bytes must survive), runs the levels
// back to back on the device, and writes back the dst ranges of the output nodes.
// Intermediate activations never cross PCIe.

struct lk_graph {
  struct Region { uintptr_t host; uint64_t lo, hi; uint8_t *dev; void *alloc; bool direct; };
  // direct: the mirror is page-locked host memory the kernels store into (see lk_graph_create);
  // the copy is then a host memcpy after the sync, no DMA
  struct Copy { uint8_t *host; uint8_t *dev; uint64_t bytes; uint64_t stage; bool direct; };
  int device = 0;
  uint64_t generation = 0;
  int nlev = 0;
  std::vector<Region> regions;
  // per non-empty dependency level: one plan of the nodes every device computes whole and, on a
  // sharded graph, one sharded plan of the row-sharded nodes (their in-place all-gathers after it)
  struct Level { lk_plan *plan = nullptr; lk_sharded_plan *sp = nullptr; };
  std::vector<Level> levels;
  // per node: host A descriptor, checks, weight flag, device descriptors, bound weight mirror
  std::vector<lk_tensor> ha, da, db, dd;
  // row sharding over an RCCL communicator (lk_graph_create_sharded): a node with shard[i] runs
  // this rank's rows of its weight (device descriptor sa[i], rows [rank·M/P, (rank+1)·M/P)) into
  // the full dst mirror, which the in-place all-gather then completes on every rank
  lk_comm *comm = nullptr;
  int nranks = 1, rank = 0;
  std::vector<char> shard;
  std::vector<lk_tensor> sa;
  // one host thread driving several devices (lk_comm_init_all): a sub-graph per device; this
  // graph only orchestrates (uploads to every part, levels in RCCL groups, outputs from part 0)
  std::vector<lk_graph *> parts;
  bool broken = false;  // a compute failed inside an RCCL group: communicators aborted
  std::vector<Checked> c;
  std::vector<char> a_weight;
  std::vector<MirrorRef> pins;
  int rebinds = 0;
  std::vector<Copy> h2d, d2h;
  std::vector<int> node_level;
  uint8_t *staging = nullptr;  // page-locked bounce buffer for the per-compute copies
  int computes = 0;             // the second compute captures the device part in a HIP graph
  bool no_capture = false;
  hipGraphExec_t exec = nullptr;
  uint64_t h2d_bytes = 0, d2h_bytes = 0;
};

namespace {

struct Span {
  uintptr_t host;
  uint64_t lo, hi;
};
bool overlaps(const Span &x, const Span &y) { return x.host == y.host && x.lo < y.hi && y.lo < x.hi; }

// Union of spans per host buffer, as sorted disjoint intervals.
std::vector<Span> merge_spans(std::vector<Span> v) {
  std::sort(v.begin(), v.end(), [](const Span &x, const Span &y) {
    return x.host != y.host ? x.host < y.host : x.lo < y.lo;
  });
  std::vector<Span> out;
  for (auto &s : v) {
    if (s.hi <= s.lo) continue;
    if (!out.empty() && out.back().host == s.host && s.lo <= out.back().hi) out.back().hi = std::max(out.back().hi, s.hi);
    else out.push_back(s);
  }
  return out;
}

// (Re)bind a graph's weights to the current residency cache and build one plan per level.
// A weight reuses the current mirror covering its bytes (whatever generation a caller
// pinned last), else it is pinned from the host bytes with the graph's generation. Called at
// create and again by lk_graph_compute when one of the bound mirrors went stale (superseded
// or evicted): plans and the captured HIP graph hold raw device pointers, so both are rebuilt.
void destroy_levels(lk_graph *g) {
  for (auto &L : g->levels) {
    if (L.plan) lk_plan_destroy(L.plan);
    if (L.sp) lk_sharded_plan_destroy(L.sp);
  }
  g->levels.clear();
}

int graph_bind(lk_graph *g, bool at_create) {
  destroy_levels(g);
  if (g->exec) (void)hipGraphExecDestroy(g->exec);
  g->exec = nullptr;
  g->computes = 0;  // first compute after a bind runs eager (sizes scratch), then capture
  const int n = (int)g->ha.size();
  int rc = LK_OK;
  for (int i = 0; i < n; i++) {
    if (!g->a_weight[i] || g->c[i].empty) continue;
    const Checked &c = g->c[i];
    // the bytes this device holds: the whole weight, or this rank's row shard of it
    lk_tensor src = g->ha[i];
    uint64_t lo = c.a_lo, hi = c.a_hi;
    if (g->shard[i]) {
      const int64_t rows = c.M / g->nranks;
      const uint64_t pitch = (uint64_t)(c.K / 32) * block_bytes(src.type);
      src.ne[1] = rows;
      src.data_offset += (uint64_t)g->rank * rows * pitch;
      lo = src.data_offset;
      hi = lo + (uint64_t)rows * pitch;
    }
    // at create the graph's generation rules (it supersedes other generations over these
    // bytes); at a rebind whatever a caller pinned since is current
    MirrorRef m = at_create ? nullptr : find_pinned(S().devs[g->device], src.data, lo, hi);
    if (!m && (rc = pin_on(g->device, &src, lo, hi - lo, g->generation, &m))) return rc;
    g->pins[i] = m;
    lk_tensor &d = g->shard[i] ? g->sa[i] : g->da[i];
    d = src;
    d.data = (uint8_t *)m->ptr + (lo - m->lo) - lo;  // base shifted: base + offset = mirror
    d.buf_bytes = m->lo + m->bytes + kASlack;          // the mirror's end, its slack included
  }
  for (int l = 0; l < g->nlev; l++) {
    std::vector<lk_tensor> la, lb, ld, sa, sb, sd;
    for (int i = 0; i < n; i++) {
      if (g->node_level[i] != l || g->c[i].empty) continue;
      if (g->shard[i]) { sa.push_back(g->sa[i]); sb.push_back(g->db[i]); sd.push_back(g->dd[i]); }
      else { la.push_back(g->da[i]); lb.push_back(g->db[i]); ld.push_back(g->dd[i]); }
    }
    if (la.empty() && sa.empty()) continue;
    lk_graph::Level L;
    if (!la.empty() && (rc = lk_plan_create(la.data(), lb.data(), ld.data(), (int)la.size(), &L.plan))) return rc;
    if (!sa.empty() && (rc = lk_sharded_plan_create(g->comm, sa.data(), sb.data(), sd.data(), (int)sa.size(), &L.sp))) {
      if (L.plan) lk_plan_destroy(L.plan);
      return rc;
    }
    g->levels.push_back(L);
  }
  return LK_OK;
}

// Enqueue level `l` of g on its device's stream (the caller made g->device current).
int launch_level(lk_graph *g, size_t l, hipStream_t st) {
  const lk_graph::Level &L = g->levels[l];
  if (L.plan)
    if (int r = lk_plan_launch(L.plan, st)) return r;
  if (L.sp)
    if (int r = lk_sharded_plan_launch(L.sp, st)) return r;
  return LK_OK;
}

bool graph_stale(const lk_graph *g) {
  for (auto &m : g->pins)
    if (m && m->stale) return true;
  return false;
}

// LK_GRAPH_NO_DIRECT=1 (lab A/B): every region in device memory, outputs copied back by DMA
const bool g_no_direct = [] {
  const char *e = std::getenv("LK_GRAPH_NO_DIRECT");
  return e && *e == '1';
}();

bool direct_at(lk_graph *g, const Span &s) {
  for (auto &r : g->regions)
    if (r.host == s.host && r.lo <= s.lo && s.lo < r.hi) return r.direct;
  return false;
}

uint8_t *mirror_of(lk_graph *g, uintptr_t host, uint64_t lo) {
  for (auto &r : g->regions)
    if (r.host == host && r.lo <= lo && lo < r.hi) return r.dev + (lo - r.lo);
  for (auto &r : g->regions)  // empty span at a region end
    if (r.host == host && r.lo <= lo && lo <= r.hi) return r.dev + (lo - r.lo);
  return nullptr;
}

}  // namespace

extern "C" {

void lk_graph_destroy(lk_graph *g) {
  if (!g) return;
  for (auto *p : g->parts) lk_graph_destroy(p);
  destroy_levels(g);
  g->pins.clear();
  for (auto &r : g->regions) (void)(r.direct ? hipHostFree(r.alloc) : hipFree(r.alloc));
  if (g->staging) (void)hipHostFree(g->staging);
  if (g->exec) (void)hipGraphExecDestroy(g->exec);
  delete g;
}

}  // extern "C"

namespace {

// Builds a graph on the current device (lk_graph_create), or rank comm's part of a sharded one.
int graph_build(lk_comm *comm, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n, const uint8_t *outputs,
                uint64_t weight_generation, lk_graph **out) {
  int rc = LK_OK;
  std::vector<Checked> c(n);
  std::vector<char> a_weight(n, 0);
  std::vector<Span> dsp(n), asp(n), bsp(n);
  for (int i = 0; i < n; i++) {
    if ((rc = check(&a[i], &b[i], &dst[i], &c[i]))) return rc;
    asp[i] = {(uintptr_t)a[i].data, c[i].a_lo, c[i].a_hi};
    bsp[i] = {(uintptr_t)b[i].data, c[i].b_lo, c[i].b_hi};
    dsp[i] = {(uintptr_t)dst[i].data, c[i].d_lo, c[i].d_hi};
  }
  // quantized A that no node writes: a weight (pinned); anything else is an activation
  for (int i = 0; i < n; i++) {
    bool produced = false;
    for (int j = 0; j < n && !produced; j++) produced = overlaps(asp[i], dsp[j]);
    a_weight[i] = is_q(a[i].type) && !produced && !c[i].empty;
  }
  auto g = new lk_graph();
  if (hipGetDevice(&g->device) != hipSuccess) g->device = S().device;
  g->comm = comm;
  g->nranks = comm ? lk_comm_nranks(comm) : 1;
  g->rank = comm ? lk_comm_rank(comm) : 0;
  g->node_level.assign(n, 0);
  int nlev = 0;
  for (int j = 0; j < n; j++) {  // level = 1 + deepest earlier node it conflicts with
    int lev = 0;
    for (int i = 0; i < j; i++) {
      const bool raw = overlaps(dsp[i], bsp[j]) || overlaps(dsp[i], asp[j]);
      const bool war = overlaps(bsp[i], dsp[j]) || overlaps(asp[i], dsp[j]);
      const bool waw = overlaps(dsp[i], dsp[j]);
      if (raw || war || waw) lev = std::max(lev, g->node_level[i] + 1);
    }
    g->node_level[j] = lev;
    nlev = std::max(nlev, lev + 1);
  }
  // device mirrors of every activation range
  std::vector<Span> act;
  for (int i = 0; i < n; i++) {
    if (c[i].empty) continue;
    act.push_back(bsp[i]);
    act.push_back(dsp[i]);
    if (!a_weight[i]) act.push_back(asp[i]);
  }
  // inputs: read ranges not produced by an earlier node, and non-dense dst ranges (their gap
  // bytes are copied back whole); uploading all of them up front is safe because levels
  // order every in-graph write after the reads that precede it
  std::vector<Span> up, down;
  for (int j = 0; j < n; j++) {
    if (c[j].empty) continue;
    auto produced_before = [&](const Span &s) {
      for (int i = 0; i < j; i++) if (overlaps(dsp[i], s)) return true;
      return false;
    };
    if (!produced_before(bsp[j])) up.push_back(bsp[j]);
    if (!a_weight[j] && !produced_before(asp[j])) up.push_back(asp[j]);
    const uint64_t ew = dst[j].type == LK_TYPE_F16 ? 2 : 4;
    if (dsp[j].hi - dsp[j].lo != (uint64_t)c[j].M * c[j].N * ew) up.push_back(dsp[j]);
    if (!outputs || outputs[j]) down.push_back(dsp[j]);
  }
  // A region no node reads, that is not uploaded, holding results the caller wants back (a
  // graph's pure outputs) is mirrored in page-locked host memory: the kernels store the
  // results straight over PCIe (a few KB per node) and no DMA copy is queued after them.
  std::vector<Span> reads;
  for (int i = 0; i < n; i++) {
    if (c[i].empty) continue;
    reads.push_back(bsp[i]);
    if (!a_weight[i]) reads.push_back(asp[i]);
  }
  const std::vector<Span> up_m = merge_spans(up), down_m = merge_spans(down);
  auto hits = [](const std::vector<Span> &v, const Span &s) {
    for (auto &x : v) if (overlaps(x, s)) return true;
    return false;
  };
  for (auto &s : merge_spans(act)) {
    // the mirror keeps the host address modulo 256, so operands keep their alignment class
    lk_graph::Region r{s.host, s.lo, s.hi, nullptr, nullptr, false};
    // (never on a sharded graph: its all-gathers write the dst mirrors)
    r.direct = !g_no_direct && !comm && hits(down_m, s) && !hits(reads, s) && !hits(up_m, s);
    const uint64_t skew = (s.host + s.lo) & 255;
    const hipError_t e = r.direct ? hipHostMalloc(&r.alloc, s.hi - s.lo + skew, hipHostMallocDefault)
                                  : hipMalloc(&r.alloc, s.hi - s.lo + skew);
    if (e != hipSuccess) {
      lk_graph_destroy(g);
      return fail(LK_ERR_DEVICE, "graph: mirror allocation of %llu B", (unsigned long long)(s.hi - s.lo));
    }
    r.dev = (uint8_t *)r.alloc + skew;
    g->regions.push_back(r);
  }
  // a read range produced by an earlier node is not uploaded even in part: the producer writes it
  for (auto &s : up_m) {
    g->h2d.push_back({(uint8_t *)s.host + s.lo, mirror_of(g, s.host, s.lo), s.hi - s.lo, 0, false});
    g->h2d_bytes += s.hi - s.lo;
  }
  for (auto &s : down_m) {
    g->d2h.push_back({(uint8_t *)s.host + s.lo, mirror_of(g, s.host, s.lo), s.hi - s.lo, 0, direct_at(g, s)});
    g->d2h_bytes += s.hi - s.lo;
  }
  // pinned staging for everything that crosses PCIe each compute: the host side of a copy
  // is a CPU memcpy, the PCIe side a DMA from page-locked memory (pageable copies are staged
  // by the runtime in small synchronous chunks). User memory is never page-locked: a
  // registration covering part of a ByteArray breaks other copies that straddle its edge.
  {
    uint64_t off = 0;
    for (auto &x : g->h2d) { x.stage = off; off += (x.bytes + 255) & ~255ull; }
    for (auto &x : g->d2h) if (!x.direct) { x.stage = off; off += (x.bytes + 255) & ~255ull; }
    if (off && hipHostMalloc((void **)&g->staging, off, hipHostMallocDefault) != hipSuccess) {
      lk_graph_destroy(g);
      return fail(LK_ERR_DEVICE, "graph: pinned staging of %llu B", (unsigned long long)off);
    }
  }
  // device descriptors of the activations; weights and plans are bound by graph_bind
  g->generation = weight_generation;
  g->nlev = nlev;
  g->ha.assign(a, a + n);
  g->c = c;
  g->a_weight = a_weight;
  g->pins.assign(n, nullptr);
  g->da.resize(n); g->db.resize(n); g->dd.resize(n); g->sa.resize(n);
  g->shard.assign(n, 0);
  for (int i = 0; i < n && comm; i++)  // row-shardable: a quantized weight, whole blocks per row, M % P, dense F32 dst
    g->shard[i] = a_weight[i] && c[i].K % 32 == 0 && c[i].M % g->nranks == 0 && dst[i].type == LK_TYPE_F32 &&
                  dst[i].nb[0] == 4 && dst[i].nb[1] == 4 * (uint64_t)c[i].N;
  for (int i = 0; i < n; i++) {
    g->da[i] = a[i]; g->db[i] = b[i]; g->dd[i] = dst[i];
    if (c[i].empty) continue;
    if (!a_weight[i]) {
      g->da[i].data = mirror_of(g, asp[i].host, c[i].a_lo) - c[i].a_lo;
      g->da[i].buf_bytes = c[i].a_hi;
    }
    g->db[i].data = mirror_of(g, bsp[i].host, c[i].b_lo) - c[i].b_lo;
    g->db[i].buf_bytes = c[i].b_hi;
    g->dd[i].data = mirror_of(g, dsp[i].host, c[i].d_lo) - c[i].d_lo;
    g->dd[i].buf_bytes = c[i].d_hi;
  }
  if ((rc = graph_bind(g, true))) { lk_graph_destroy(g); return rc; }
  *out = g;
  return LK_OK;
}

// One compute of a single-device graph: staged uploads, every level, staged write-backs on the
// device's library stream; from the second compute on replayed as one HIP graph.
int graph_compute_one(lk_graph *g) {
  int rc = lk_init(g->device);
  if (rc) return rc;
  if (graph_stale(g)) {  // a bound weight mirror was superseded or evicted since the last bind
    if ((rc = graph_bind(g, false))) return rc;
    g->rebinds++;
  }
  hipStream_t st = S().devs[g->device].stream;
  auto enqueue = [&]() -> int {
    for (auto &x : g->h2d) HIP_TRY(hipMemcpyAsync(x.dev, g->staging + x.stage, x.bytes, hipMemcpyHostToDevice, st));
    for (size_t l = 0; l < g->levels.size(); l++)
      if (int r = launch_level(g, l, st)) return r;
    for (auto &x : g->d2h)
      if (!x.direct) HIP_TRY(hipMemcpyAsync(g->staging + x.stage, x.dev, x.bytes, hipMemcpyDeviceToHost, st));
    return LK_OK;
  };
  for (auto &x : g->h2d) std::memcpy(g->staging + x.stage, x.host, x.bytes);
  if (!g->exec && !g->no_capture && g->computes >= 1) {
    hipGraph_t graph = nullptr;
    bool ok = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess;
    const int r = ok ? enqueue() : LK_ERR_DEVICE;
    ok = (hipStreamEndCapture(st, &graph) == hipSuccess) && ok && r == LK_OK;
    if (ok) ok = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0) == hipSuccess;
    if (graph) (void)hipGraphDestroy(graph);
    if (!ok) {
      g->exec = nullptr;
      g->no_capture = true;  // stay eager
      (void)hipGetLastError();
    }
  }
  const unsigned mark = fail_mark(g->device);
  if (g->exec) HIP_TRY(hipGraphLaunch(g->exec, st));
  else if ((rc = enqueue())) return rc;
  HIP_TRY(hipStreamSynchronize(st));
  if ((rc = sync_failures(g->device, mark))) return rc;  // nothing is written back from a failed launch
  for (auto &x : g->d2h) std::memcpy(x.host, x.direct ? x.dev : g->staging + x.stage, x.bytes);
  g->computes++;
  return LK_OK;
}

// One compute of a graph whose parts run on several devices of this thread (eager: uploads to
// every part, each level of every part inside one RCCL group so the parts' all-gathers meet,
// outputs read back from part 0, which like every part holds every gathered result).
int graph_compute_parts(lk_graph *top) {
  if (top->broken)
    return fail(LK_ERR_DEVICE, "graph: unusable since a compute failed inside an RCCL group (communicators aborted)");
  int prev = 0;
  (void)hipGetDevice(&prev);
  int rc = LK_OK;
  std::vector<unsigned> mark;
  for (auto *g : top->parts) {
    if ((rc = init_dev(g->device))) goto out;
    mark.push_back(fail_mark(g->device));
    if (graph_stale(g)) {
      if ((rc = graph_bind(g, false))) goto out;
      g->rebinds++;
    }
    hipStream_t st = S().devs[g->device].stream;
    for (auto &x : g->h2d) {
      std::memcpy(g->staging + x.stage, x.host, x.bytes);
      if (hipMemcpyAsync(x.dev, g->staging + x.stage, x.bytes, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = fail(LK_ERR_DEVICE, "graph: upload to device %d", g->device);
        goto out;
      }
    }
  }
  for (size_t l = 0; l < top->parts[0]->levels.size(); l++) {
    if ((rc = lk_comm_group_start())) goto out;
    for (auto *g : top->parts) {
      if ((rc = init_dev(g->device)) || (rc = launch_level(g, l, S().devs[g->device].stream))) break;
    }
    const int re = lk_comm_group_end();
    if (rc || (rc = re)) {
      // some parts enqueued their all-gathers and others did not: those collectives would wait for
      // peers that never arrive. Abort every communicator (its enqueued work is torn down) and
      // refuse further computes of this graph.
      for (auto *g : top->parts) (void)lk_comm_abort(g->comm);
      top->broken = true;
      goto out;
    }
  }
  {
    lk_graph *g0 = top->parts[0];
    if ((rc = init_dev(g0->device))) goto out;
    for (auto &x : g0->d2h)
      if (hipMemcpyAsync(g0->staging + x.stage, x.dev, x.bytes, hipMemcpyDeviceToHost, S().devs[g0->device].stream) != hipSuccess) {
        rc = fail(LK_ERR_DEVICE, "graph: read back from device %d", g0->device);
        goto out;
      }
  }
  for (auto *g : top->parts)
    if (hipSetDevice(g->device) != hipSuccess || hipStreamSynchronize(S().devs[g->device].stream) != hipSuccess) {
      rc = fail(LK_ERR_DEVICE, "graph: device %d failed", g->device);
      goto out;
    }
  for (size_t k = 0; k < top->parts.size(); k++)
    if ((rc = sync_failures(top->parts[k]->device, mark[k]))) goto out;
  for (auto &x : top->parts[0]->d2h) std::memcpy(x.host, top->parts[0]->staging + x.stage, x.bytes);
  for (auto *g : top->parts) g->computes++;
out:
  (void)hipSetDevice(prev);
  return rc;
}

}  // namespace

extern "C" {

int lk_graph_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n, const uint8_t *outputs,
                    uint64_t weight_generation, lk_graph **out) {
  if (!out || n < 0 || (n && (!a || !b || !dst))) return fail(LK_ERR_INVALID_ARG, "bad graph arguments");
  *out = nullptr;
  int rc = ensure_init();
  if (rc) return rc;
  return graph_build(nullptr, a, b, dst, n, outputs, weight_generation, out);
}

int lk_graph_create_sharded(lk_comm *const *comms, int ncomms, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst,
                            int n, const uint8_t *outputs, uint64_t weight_generation, lk_graph **out) {
  if (!out || !comms || ncomms < 1 || n < 0 || (n && (!a || !b || !dst)))
    return fail(LK_ERR_INVALID_ARG, "bad sharded graph arguments");
  *out = nullptr;
  for (int r = 0; r < ncomms; r++)
    if (!comms[r] || (ncomms > 1 && (lk_comm_nranks(comms[r]) != ncomms || lk_comm_rank(comms[r]) != r)))
      return fail(LK_ERR_INVALID_ARG, "sharded graph: comms[r] must be rank r of one %d-rank communicator", ncomms);
  int prev = 0;
  (void)hipGetDevice(&prev);
  int rc = LK_OK;
  std::vector<lk_graph *> parts;
  for (int r = 0; r < ncomms && rc == LK_OK; r++) {
    lk_graph *p = nullptr;
    if ((rc = init_dev(lk_comm_device(comms[r]))) == LK_OK &&
        (rc = graph_build(comms[r], a, b, dst, n, outputs, weight_generation, &p)) == LK_OK)
      parts.push_back(p);
  }
  (void)hipSetDevice(prev);
  if (rc) {
    for (auto *p : parts) lk_graph_destroy(p);
    return rc;
  }
  if (ncomms == 1) {
    *out = parts[0];
    return LK_OK;
  }
  auto top = new lk_graph();
  top->device = parts[0]->device;
  top->parts = parts;
  *out = top;
  return LK_OK;
}

int lk_graph_compute(lk_graph *g) {
  if (!g) return fail(LK_ERR_INVALID_ARG, "null graph");
  return g->parts.empty() ? graph_compute_one(g) : graph_compute_parts(g);
}

int lk_graph_num_levels(const lk_graph *g) {
  if (g && !g->parts.empty()) g = g->parts[0];
  return g ? (int)g->levels.size() : 0;
}

int lk_graph_num_rebinds(const lk_graph *g) {
  if (g && !g->parts.empty()) g = g->parts[0];
  return g ? g->rebinds : 0;
}

// Kernel launches of one compute on one device (a sharded plan's local launch counts; its
// all-gathers do not).
int lk_graph_num_launches(const lk_graph *g) {
  if (g && !g->parts.empty()) g = g->parts[0];
  int t = 0;
  if (g)
    for (auto &L : g->levels) t += (L.plan ? lk_plan_num_launches(L.plan) : 0) + (L.sp ? 1 : 0);
  return t;
}

int lk_graph_num_sharded(const lk_graph *g) {
  if (g && !g->parts.empty()) g = g->parts[0];
  int t = 0;
  if (g)
    for (char x : g->shard) t += x != 0;
  return t;
}

uint64_t lk_graph_transfer_bytes(const lk_graph *g, int to_device) {
  if (!g) return 0;
  if (!g->parts.empty()) return to_device ? g->parts.size() * g->parts[0]->h2d_bytes : g->parts[0]->d2h_bytes;
  return to_device ? g->h2d_bytes : g->d2h_bytes;
}

}  // extern "C"

// ---- direct dot products (core/GGMLComputeOps.kt:349-629) --------------------------------

namespace {

struct DotCheck {
  int64_t M, N;
  uint64_t a_lo, a_hi, b_lo, b_hi;  // byte extents read (buffer-relative)
};

// The Kotlin functions' require()s in order, then the accessors' checks: block index past
// numBlocks (IllegalArgumentException), missing buffer, bytes past the buffer.
int dot_check(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, DotCheck *c) {
  int32_t ta, tb;
  switch (kind) {
    case LK_DOT_F32_Q4_1: ta = LK_TYPE_F32; tb = LK_TYPE_Q4_1; break;
    case LK_DOT_F32_Q8_0: ta = LK_TYPE_F32; tb = LK_TYPE_Q8_0; break;
    case LK_DOT_Q8_0_Q8_0: ta = LK_TYPE_Q8_0; tb = LK_TYPE_Q8_0; break;
    case LK_DOT_Q4_0_Q4_0: ta = LK_TYPE_Q4_0; tb = LK_TYPE_Q4_0; break;
    case LK_DOT_Q4_1_Q4_1: ta = LK_TYPE_Q4_1; tb = LK_TYPE_Q4_1; break;
    case LK_DOT_Q8_0_Q4_0: ta = LK_TYPE_Q8_0; tb = LK_TYPE_Q4_0; break;
    default: return fail(LK_ERR_NOT_IMPLEMENTED, "direct dot kind %d", kind);
  }
  if (!a || !b) return fail(LK_ERR_INVALID_ARG, "null tensor");
  if (a->type != ta) return fail(LK_ERR_INVALID_ARG, "tensorA must be type %d. Got %d", ta, a->type);
  if (b->type != tb) return fail(LK_ERR_INVALID_ARG, "tensorB must be type %d. Got %d", tb, b->type);
  if (a->ne[0] != K) return fail(LK_ERR_INVALID_ARG, "tensorA K dim (%lld) must match commonDimK (%lld)", (long long)a->ne[0], (long long)K);
  if (b->ne[1] != K) return fail(LK_ERR_INVALID_ARG, "tensorB K dim (%lld) must match commonDimK (%lld)", (long long)b->ne[1], (long long)K);
  c->M = a->ne[1];
  c->N = b->ne[0];
  c->a_lo = c->a_hi = a->data_offset;
  c->b_lo = c->b_hi = b->data_offset;
  if (c->M <= 0 || c->N <= 0 || K <= 0) return LK_OK;  // no accessor runs
  if (!a->data || !b->data) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  // flat indices reach M·K − 1 (A, Q types) and K·N − 1 (B)
  auto q_extent = [](const lk_tensor *t, int64_t last_flat, uint64_t *hi) {
    const int64_t blk = last_flat / 32, nblk = t_num_elements(t) / 32;
    if (blk >= nblk) return fail(LK_ERR_INVALID_ARG, "blockIndex %lld out of bounds for %lld blocks", (long long)blk, (long long)nblk);
    *hi = t->data_offset + (uint64_t)(blk + 1) * block_bytes(t->type);
    return (int)LK_OK;
  };
  int rc;
  if (ta == LK_TYPE_F32) {
    if (a->nb[0] < 4 || a->nb[0] % 4 || a->nb[1] % 4)
      return fail(LK_ERR_NOT_IMPLEMENTED, "direct dot: F32 strides %llu/%llu not offloaded", (unsigned long long)a->nb[0],
                  (unsigned long long)a->nb[1]);
    c->a_hi = a->data_offset + (uint64_t)(K - 1) * a->nb[0] + (uint64_t)(c->M - 1) * a->nb[1] + 4;
  } else if ((rc = q_extent(a, c->M * K - 1, &c->a_hi))) {
    return rc;
  }
  if ((rc = q_extent(b, K * c->N - 1, &c->b_hi))) return rc;
  if (c->a_hi > a->buf_bytes) return fail(LK_ERR_OUT_OF_BOUNDS, "tensorA read past its buffer (%llu > %llu)", (unsigned long long)c->a_hi, (unsigned long long)a->buf_bytes);
  if (c->b_hi > b->buf_bytes) return fail(LK_ERR_OUT_OF_BOUNDS, "tensorB read past its buffer (%llu > %llu)", (unsigned long long)c->b_hi, (unsigned long long)b->buf_bytes);
  return LK_OK;
}

int launch_dot_direct(int32_t kind, const uint8_t *a, const uint8_t *b, const lk_tensor *at, int64_t M, int64_t N, int64_t K, float *out,
                      hipStream_t st) {
  if (M * N == 0) return LK_OK;
  if (K == 0) { HIP_TRY(hipMemsetAsync(out, 0, (size_t)(M * N) * sizeof(float), st)); return LK_OK; }
  DotArgs g{a, b, out, M, N, K, (int64_t)at->nb[0], (int64_t)at->nb[1]};
  const int64_t blocks = (M * N + 255) / 256;
  if (blocks > (int64_t)INT32_MAX) return fail(LK_ERR_NOT_IMPLEMENTED, "direct dot: output too large");
  dim3 grid((unsigned)blocks), block(256);
  switch (kind) {
    case LK_DOT_F32_Q4_1: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_F32_Q4_1>, grid, block, 0, st, g); break;
    case LK_DOT_F32_Q8_0: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_F32_Q8_0>, grid, block, 0, st, g); break;
    case LK_DOT_Q8_0_Q8_0: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_Q8_0_Q8_0>, grid, block, 0, st, g); break;
    case LK_DOT_Q4_0_Q4_0: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_Q4_0_Q4_0>, grid, block, 0, st, g); break;
    case LK_DOT_Q4_1_Q4_1: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_Q4_1_Q4_1>, grid, block, 0, st, g); break;
    default: hipLaunchKernelGGL(dot_direct_kernel<LK_DOT_Q8_0_Q4_0>, grid, block, 0, st, g); break;
  }
  HIP_TRY(hipGetLastError());
  return LK_OK;
}

}  // namespace

int lk_dot_direct_device(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out, void *stream) {
  DotCheck c;
  int rc = dot_check(kind, a, b, K, &c);
  if (rc) return rc;
  if (c.M <= 0 || c.N <= 0) return LK_OK;
  if (!out) return fail(LK_ERR_NO_BUFFER, "output buffer not found");
  if ((rc = ensure_init())) return rc;
  return launch_dot_direct(kind, (const uint8_t *)a->data + a->data_offset, (const uint8_t *)b->data + b->data_offset, a, c.M, c.N, K,
                           out, pick_stream(stream));
}

int lk_dot_direct(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out) {
  DotCheck c;
  int rc = dot_check(kind, a, b, K, &c);
  if (rc) return rc;
  if (c.M <= 0 || c.N <= 0) return LK_OK;
  if (!out) return fail(LK_ERR_NO_BUFFER, "output buffer not found");
  int dev = 0;
  if ((rc = ensure_init(&dev))) return rc;
  Dev &s = S().devs[dev];
  hipStream_t st = s.stream;
  const uint64_t a_bytes = c.a_hi - c.a_lo, b_bytes = c.b_hi - c.b_lo, o_bytes = (uint64_t)(c.M * c.N) * sizeof(float);
  if ((rc = ensure_scratch(s, 0, std::max<uint64_t>(a_bytes, 16)))) return rc;
  if ((rc = ensure_scratch(s, 1, std::max<uint64_t>(b_bytes, 16)))) return rc;
  if ((rc = ensure_scratch(s, 2, o_bytes))) return rc;
  if (a_bytes) HIP_TRY(hipMemcpyAsync(s.scratch[0], (const uint8_t *)a->data + c.a_lo, a_bytes, hipMemcpyHostToDevice, st));
  if (b_bytes) HIP_TRY(hipMemcpyAsync(s.scratch[1], (const uint8_t *)b->data + c.b_lo, b_bytes, hipMemcpyHostToDevice, st));
  rc = launch_dot_direct(kind, (const uint8_t *)s.scratch[0], (const uint8_t *)s.scratch[1], a, c.M, c.N, K, (float *)s.scratch[2], st);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, s.scratch[2], o_bytes, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return LK_OK;
}

#ifdef LK_LAB_STAMPS
// lab builds only (tools/stamp_kpart.py): the gemm_kpart_kernel timeline stamps
extern "C" int lk_lab_stamps(uint64_t *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lk::lk_kp_stamps), sizeof(uint64_t) * (size_t)std::min(n, 1024 * 8 * 10)) == hipSuccess ? 0 : 5;
}
extern "C" int lk_lab_stamps_clear(void) {
  static uint64_t zero[1024 * 8 * 10];
  return hipMemcpyToSymbol(HIP_SYMBOL(lk::lk_kp_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : 5;
}
#endif
#ifdef LK_LAB_CHAIN_STAMPS
extern "C" int lk_lab_chain_stamps(uint64_t *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lk::lk_chain_stamps), sizeof(uint64_t) * (size_t)std::min(n, 256 * 256 * 8)) == hipSuccess ? 0 : 5;
}
extern "C" int lk_lab_chain_stamps_clear(void) {
  static uint64_t zero[256 * 256 * 8];
  return hipMemcpyToSymbol(HIP_SYMBOL(lk::lk_chain_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : 5;
}
#endif
