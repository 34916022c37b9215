// lk_kernels.hpp — gfx950 (CDNA4) device code for llama.kotlin's quantized MUL_MAT.
//
// Semantics follow computeMatMul (core/GGMLComputeOps.kt:1435-1565): A is the
// quantized weight tensor ne=[K,M] (blocks of 32 weights, llama.kotlin layout),
// B is F32 ne=[N,K] (N fastest), dst is F32 ne=[N,M]; dst(j,i) = Σ_k w(i,k)·B(j,k).
//
// Block layouts (core/GGMLTypes.kt:543-732), interleaved nibbles: weight 2j is the
// low nibble of quant byte j, weight 2j+1 the high nibble, so within one dword of
// quant bytes the 8 nibbles, low to high, are 8 consecutive weights.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lk_hip.h"

namespace lk {

constexpr int kWave = 64;

// Pointers the kernels stream through are global memory; saying so lets hipcc emit
// global_load (vmcnt only) instead of flat_load (vmcnt + lgkmcnt).
#define LK_GLOBAL __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- per-type traits -------------------------------------------------------
template <int QT> struct QTraits;
template <> struct QTraits<LK_TYPE_Q4_0> { static constexpr int BB = 18; static constexpr int PAIR_DW = 9; };
template <> struct QTraits<LK_TYPE_Q4_1> { static constexpr int BB = 20; static constexpr int PAIR_DW = 10; };
template <> struct QTraits<LK_TYPE_Q8_0> { static constexpr int BB = 34; static constexpr int PAIR_DW = 17; };

// ---- numeric helpers --------------------------------------------------------

// halfToFloat (core/NumericConversions.kt:9-54) is exact IEEE f16 -> f32 for every
// non-NaN input; v_cvt_f32_f16 is the same map (NaN payload quieting differs only
// in NaN bits, which no comparison observes).
__device__ __forceinline__ float h2f(uint32_t bits16) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(bits16 & 0xFFFFu));
}

// Kotlin Int shift semantics (count masked to 5 bits).
__device__ __forceinline__ int32_t kshl(int32_t x, int32_t s) { return (int32_t)((uint32_t)x << (s & 31)); }
__device__ __forceinline__ int32_t kushr(int32_t x, int32_t s) { return (int32_t)((uint32_t)x >> (s & 31)); }

// floatToHalf (core/NumericConversions.kt:61-124), bit for bit, including the
// denormal branch's off-by-one exponent and masked shift counts.
__device__ __forceinline__ uint16_t kotlin_float_to_half(float f) {
  int32_t bits = __builtin_bit_cast(int32_t, f);
  int32_t fSign = kushr(bits, 16) & 0x8000;
  int32_t absF = bits & 0x7FFFFFFF;
  if (absF > 0x47FFEFFF) return (uint16_t)(fSign | 0x7C00 | (((absF & 0x007FFFFF) != 0) ? 0x0200 : 0));
  if (absF < 0x38800000) {
    int32_t fMant = (absF & 0x007FFFFF) | 0x00800000;
    int32_t shift = 127 - kushr(absF, 23);
    int32_t hMant = (shift < 24) ? kushr(fMant, shift) : 0;
    int32_t roundBits = fMant & (int32_t)((uint32_t)kshl(1, shift) - 1u);
    int32_t half = kshl(1, shift - 1);
    if (roundBits > half || (roundBits == half && (hMant & 1) != 0)) {
      int32_t h = hMant + 1;
      if (h == 0x0400) return (uint16_t)(fSign | 0x0400);
      return (uint16_t)(fSign | h);
    }
    return (uint16_t)(fSign | hMant);
  }
  int32_t hExp = kshl(kushr(absF, 23) - 112, 10);
  int32_t hMant = kushr(absF & 0x007FFFFF, 13);
  if ((absF & 0x1000) != 0 && ((absF & 0xFFF) != 0 || (hMant & 1) != 0)) {
    hMant++;
    if (hMant == 0x0400) return (uint16_t)(fSign | (int32_t)((uint32_t)hExp + 0x400u));
  }
  return (uint16_t)(fSign | hExp | hMant);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ---- block dot products (the fused dequant inner loop) -----------------------
//
// Each returns the block's contribution Σ_{k<32} w_k·x_k for one row, where x
// points at the 32 activations of that block. The per-block f32 scale is applied
// once per block (d·Σq·x), with the constant offsets folded through Σx:
//   Q4_0: w = d·(q−8)      → d·(Σ q·x − 8·Σx)          (GGMLComputeOps.kt:133-144)
//   Q4_1: w = d·q + m      → d·Σ q·x + m·Σx             (GGMLComputeOps.kt:92-114)
//   Q8_0: w = d·q          → d·(Σ (q+128)·x − 128·Σx)   (GGMLComputeOps.kt:56-67)
// Accumulation order differs from the Kotlin loop; the parity bar for these F32
// results is ≤1e-3 relative (tests/test_gpu_parity.py).

// Σ nibble_n(u)·x[n] for the 8 nibbles of quant dword u (8 consecutive weights).
__device__ __forceinline__ float dot_nib8(uint32_t u, const float *x, float s) {
  uint32_t lo = u & 0x0F0F0F0Fu;        // nibbles 0,2,4,6 in bytes 0..3
  uint32_t hi = (u >> 4) & 0x0F0F0F0Fu; // nibbles 1,3,5,7
  s = fmaf((float)(lo & 0xFF), x[0], s);
  s = fmaf((float)(hi & 0xFF), x[1], s);
  s = fmaf((float)((lo >> 8) & 0xFF), x[2], s);
  s = fmaf((float)((hi >> 8) & 0xFF), x[3], s);
  s = fmaf((float)((lo >> 16) & 0xFF), x[4], s);
  s = fmaf((float)((hi >> 16) & 0xFF), x[5], s);
  s = fmaf((float)(lo >> 24), x[6], s);
  s = fmaf((float)(hi >> 24), x[7], s);
  return s;
}

// Σ (q_n+128)·x[n] for the 4 signed bytes of dword u.
__device__ __forceinline__ float dot_i8x4_biased(uint32_t u, const float *x, float s) {
  uint32_t b = u ^ 0x80808080u;
  s = fmaf((float)(b & 0xFF), x[0], s);
  s = fmaf((float)((b >> 8) & 0xFF), x[1], s);
  s = fmaf((float)((b >> 16) & 0xFF), x[2], s);
  s = fmaf((float)(b >> 24), x[3], s);
  return s;
}

__device__ __forceinline__ uint32_t align2(uint32_t hi, uint32_t lo) {
  return __builtin_amdgcn_alignbyte(hi, lo, 2);
}

// One pair of consecutive blocks (2·BB bytes, 4-byte aligned, loaded as PAIR_DW
// dwords w[]) against 64 activations x[0..63]; xs0/xs1 are Σx of each block.
template <int QT>
__device__ __forceinline__ float pair_dot(const uint32_t *w, const float *x, float xs0, float xs1, float acc);

template <>
__device__ __forceinline__ float pair_dot<LK_TYPE_Q4_0>(const uint32_t *w, const float *x, float xs0, float xs1, float acc) {
  // block 0: d = bytes 0..1, quants = bytes 2..17; block 1: d = bytes 18..19, quants = 20..35
  float d0 = h2f(w[0]);
  float s = 0.f;
  s = dot_nib8(align2(w[1], w[0]), x + 0, s);
  s = dot_nib8(align2(w[2], w[1]), x + 8, s);
  s = dot_nib8(align2(w[3], w[2]), x + 16, s);
  s = dot_nib8(align2(w[4], w[3]), x + 24, s);
  acc = fmaf(d0, fmaf(-8.f, xs0, s), acc);
  float d1 = h2f(w[4] >> 16);
  float t = 0.f;
  t = dot_nib8(w[5], x + 32, t);
  t = dot_nib8(w[6], x + 40, t);
  t = dot_nib8(w[7], x + 48, t);
  t = dot_nib8(w[8], x + 56, t);
  return fmaf(d1, fmaf(-8.f, xs1, t), acc);
}

template <>
__device__ __forceinline__ float pair_dot<LK_TYPE_Q4_1>(const uint32_t *w, const float *x, float xs0, float xs1, float acc) {
  // block 0: d,m = bytes 0..3, quants 4..19; block 1: d,m = 20..23, quants 24..39 (all aligned)
  float d0 = h2f(w[0]), m0 = h2f(w[0] >> 16);
  float s = 0.f;
  s = dot_nib8(w[1], x + 0, s);
  s = dot_nib8(w[2], x + 8, s);
  s = dot_nib8(w[3], x + 16, s);
  s = dot_nib8(w[4], x + 24, s);
  acc = fmaf(d0, s, fmaf(m0, xs0, acc));
  float d1 = h2f(w[5]), m1 = h2f(w[5] >> 16);
  float t = 0.f;
  t = dot_nib8(w[6], x + 32, t);
  t = dot_nib8(w[7], x + 40, t);
  t = dot_nib8(w[8], x + 48, t);
  t = dot_nib8(w[9], x + 56, t);
  return fmaf(d1, t, fmaf(m1, xs1, acc));
}

template <>
__device__ __forceinline__ float pair_dot<LK_TYPE_Q8_0>(const uint32_t *w, const float *x, float xs0, float xs1, float acc) {
  // block 0: d = bytes 0..1, q = bytes 2..33; block 1: d = bytes 34..35, q = 36..67 (aligned)
  float d0 = h2f(w[0]);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) s = dot_i8x4_biased(align2(w[t + 1], w[t]), x + 4 * t, s);
  acc = fmaf(d0, fmaf(-128.f, xs0, s), acc);
  float d1 = h2f(w[8] >> 16);
  float u = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) u = dot_i8x4_biased(w[9 + t], x + 32 + 4 * t, u);
  return fmaf(d1, fmaf(-128.f, xs1, u), acc);
}

// ---- grouped batch-1 GEMV (the hot kernel) ------------------------------------

// One MUL_MAT node of a grouped launch (device-resident operands).
struct GemvDesc {
  const uint8_t *a;   // first byte of A's blocks (buffer base + dataOffset)
  const float *x;     // B column 0 (contiguous K floats)
  float *dst;         // dst(0, 0)
  int64_t dst_row_stride; // elements between dst(0,i) and dst(0,i+1) (= nb[1]/4)
  int32_t M, K;
  int32_t tile_begin; // first workgroup tile of this node
  int32_t pad;
};

constexpr int kGemvWaves = 4;  // waves per workgroup

// Grid: one workgroup per tile of kGemvWaves*ROWS rows of one node; tile_map[blockIdx.x]
// names the node. Each wave owns ROWS consecutive rows; each lane owns block pairs
// p = lane, lane+64, ... of those rows. Per pair the lane loads its 64 activations
// once (float4, L1/L2-resident) and reuses them for all ROWS rows, whose 2·BB-byte
// pairs it loads with dword-aligned vector loads (coalesced at wave level: 64 lanes
// cover 64·2·BB contiguous bytes of a row).
template <int QT, int ROWS>
__global__ __launch_bounds__(256) void gemv_q_n1_kernel(const GemvDesc single, const GemvDesc *__restrict__ descs,
                                                        const uint16_t *__restrict__ tile_map) {
  constexpr int BB = QTraits<QT>::BB;
  constexpr int PDW = QTraits<QT>::PAIR_DW;
  const int tile = blockIdx.x;
  // single node: descriptor in kernel arguments; grouped: tile_map names the node
  GemvDesc d = single;
  if (tile_map) {
    const int di = __builtin_amdgcn_readfirstlane(((const LK_GLOBAL uint16_t *)tile_map)[tile]);
    const LK_GLOBAL uint64_t *src = (const LK_GLOBAL uint64_t *)(descs + di);
    uint64_t words[sizeof(GemvDesc) / 8];
#pragma unroll
    for (int i = 0; i < (int)(sizeof(GemvDesc) / 8); i++) words[i] = src[i];
    __builtin_memcpy(&d, words, sizeof(GemvDesc));
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = ((tile - d.tile_begin) * kGemvWaves + wave) * ROWS;
  if (row0 >= d.M) return;
  const int nrows = min(ROWS, d.M - row0);
  const int npairs = d.K >> 6;
  const int64_t row_bytes = (int64_t)(d.K >> 5) * BB;
  const LK_GLOBAL uint8_t *arow = (const LK_GLOBAL uint8_t *)d.a + (int64_t)row0 * row_bytes;

  float acc[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; r++) acc[r] = 0.f;

  for (int p = lane; p < npairs; p += kWave) {
    uint32_t w[ROWS][PDW];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      if (r < nrows) {
        const LK_GLOBAL uint32_t *src = (const LK_GLOBAL uint32_t *)(arow + r * row_bytes + (int64_t)p * (2 * BB));
#pragma unroll
        for (int t = 0; t < PDW; t++) w[r][t] = __builtin_nontemporal_load(src + t);
      }
    }
    float x[64];
    const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)((const LK_GLOBAL float *)d.x + (int64_t)p * 64);
#pragma unroll
    for (int t = 0; t < 16; t++) {
      f32x4 v = xv[t];
      x[4 * t + 0] = v.x; x[4 * t + 1] = v.y; x[4 * t + 2] = v.z; x[4 * t + 3] = v.w;
    }
    float xs0 = 0.f, xs1 = 0.f;
#pragma unroll
    for (int t = 0; t < 32; t++) { xs0 += x[t]; xs1 += x[32 + t]; }
#pragma unroll
    for (int r = 0; r < ROWS; r++)
      if (r < nrows) acc[r] = pair_dot<QT>(w[r], x, xs0, xs1, acc[r]);
  }
#pragma unroll
  for (int r = 0; r < ROWS; r++) {
    float v = wave_sum(acc[r]);
    if (lane == 0 && r < nrows) ((LK_GLOBAL float *)d.dst)[(int64_t)(row0 + r) * d.dst_row_stride] = v;
  }
}

// ---- generic path (any K, any byte strides, ragged blocks) ----------------------

struct GenericArgs {
  const uint8_t *a; const uint8_t *b; uint8_t *dst; // buffer base + dataOffset
  int64_t M, N, K;
  int64_t a_nb0, a_nb1, b_nb0, b_nb1, d_nb0, d_nb1; // byte strides (A's used for F32/F16 only)
};

__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }
__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

// w(i,k) exactly as the reference accessors compute it: flat index i*K+k, block
// flat/32, item flat%32 (blocks may straddle rows when K % 32 != 0).
template <int TA>
__device__ __forceinline__ float load_a(const GenericArgs &g, int64_t i, int64_t k) {
  if constexpr (TA == LK_TYPE_F32) {
    return *(const float *)(g.a + k * g.a_nb0 + i * g.a_nb1);
  } else if constexpr (TA == LK_TYPE_F16) {
    return h2f(*(const uint16_t *)(g.a + k * g.a_nb0 + i * g.a_nb1));
  } else {
    const int64_t flat = i * g.K + k;
    const int64_t blk = flat >> 5;
    const int item = (int)(flat & 31);
    const uint8_t *p = g.a + blk * QTraits<TA>::BB;
    const float d = h2f(ld_u16(p));
    if constexpr (TA == LK_TYPE_Q4_0) {
      uint32_t byte = ld_u8(p + 2 + (item >> 1));
      uint32_t q = (item & 1) ? (byte >> 4) : (byte & 0xF);
      return __fmul_rn(d, (float)q - 8.0f);
    } else if constexpr (TA == LK_TYPE_Q4_1) {
      const float m = h2f(ld_u16(p + 2));
      uint32_t byte = ld_u8(p + 4 + (item >> 1));
      uint32_t q = (item & 1) ? (byte >> 4) : (byte & 0xF);
      return __fadd_rn(__fmul_rn(d, (float)q), m);
    } else {
      int32_t q = (int32_t)(int8_t)ld_u8(p + 2 + item);
      return __fmul_rn(d, (float)q);
    }
  }
}

// One wave per output element (i,j); lanes stride over k.
template <int TA>
__global__ __launch_bounds__(256) void mul_mat_generic_kernel(GenericArgs g) {
  const int64_t out = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (out >= g.M * g.N) return;
  const int lane = threadIdx.x & 63;
  const int64_t i = out / g.N, j = out % g.N;
  float s = 0.f;
  for (int64_t k = lane; k < g.K; k += kWave) {
    float w = load_a<TA>(g, i, k);
    float x;
    if constexpr (TA == LK_TYPE_F16) x = h2f(*(const uint16_t *)(g.b + j * g.b_nb0 + k * g.b_nb1));
    else x = *(const float *)(g.b + j * g.b_nb0 + k * g.b_nb1);
    s = fmaf(w, x, s);
  }
  s = wave_sum(s);
  if (lane == 0) {
    uint8_t *o = g.dst + j * g.d_nb0 + i * g.d_nb1;
    if constexpr (TA == LK_TYPE_F16) *(uint16_t *)o = kotlin_float_to_half(s);
    else *(float *)o = s;
  }
}

// ---- format kernels (dequantizeTensor / quantizeTensor) -------------------------

// dequantizeTensor (GGMLComputeOps.kt:918-964): one thread per block, bit-exact
// (explicit non-contracted roundings).
template <int QT>
__global__ __launch_bounds__(256) void dequantize_kernel(const uint8_t *__restrict__ src, float *__restrict__ out, int64_t nblk) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const uint8_t *p = src + b * QTraits<QT>::BB;
  float *o = out + b * 32;
  const float d = h2f(ld_u16(p));
  if constexpr (QT == LK_TYPE_Q8_0) {
#pragma unroll
    for (int k = 0; k < 32; k++) o[k] = __fmul_rn(d, (float)(int32_t)(int8_t)p[2 + k]);
  } else if constexpr (QT == LK_TYPE_Q4_0) {
#pragma unroll
    for (int k = 0; k < 32; k++) {
      uint32_t byte = p[2 + (k >> 1)];
      uint32_t q = (k & 1) ? (byte >> 4) : (byte & 0xF);
      o[k] = __fmul_rn(d, (float)q - 8.0f);
    }
  } else {
    const float m = h2f(ld_u16(p + 2));
#pragma unroll
    for (int k = 0; k < 32; k++) {
      uint32_t byte = p[4 + (k >> 1)];
      uint32_t q = (k & 1) ? (byte >> 4) : (byte & 0xF);
      o[k] = __fadd_rn(__fmul_rn(d, (float)q), m);
    }
  }
}

// kotlin maxOf / minOf on Float: NaN-propagating, -0.0 < +0.0.
__device__ __forceinline__ float kmax(float a, float b) {
  if (__builtin_isnan(a) || __builtin_isnan(b)) return __builtin_nanf("");
  if (a == 0.f && b == 0.f) return __builtin_signbit(a) ? b : a;
  return a > b ? a : b;
}
__device__ __forceinline__ float kmin(float a, float b) {
  if (__builtin_isnan(a) || __builtin_isnan(b)) return __builtin_nanf("");
  if (a == 0.f && b == 0.f) return __builtin_signbit(a) ? a : b;
  return a < b ? a : b;
}
// round(x).toInt(): half-even, NaN -> 0, saturating; then coerceIn(lo, hi).
__device__ __forceinline__ int32_t kround_coerce(float x, int32_t lo, int32_t hi) {
  float r = __builtin_rintf(x);
  if (__builtin_isnan(r)) return lo <= 0 && hi >= 0 ? 0 : (0 < lo ? lo : hi);
  if (r < (float)lo) return lo;
  if (r > (float)hi) return hi;
  return (int32_t)r;
}

// quantizeTensor (GGMLComputeOps.kt:1040-1204): one thread per 32-element block.
template <int QT>
__global__ __launch_bounds__(256) void quantize_kernel(const float *__restrict__ src, uint8_t *__restrict__ out, int64_t nblk) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const float *x = src + b * 32;
  uint8_t *o = out + b * QTraits<QT>::BB;
  if constexpr (QT == LK_TYPE_Q8_0) {
    float amax = 0.f;
    for (int k = 0; k < 32; k++) amax = kmax(amax, __builtin_fabsf(x[k]));
    float scale = (amax == 0.f) ? 1.f : __fdiv_rn(amax, 127.f);
    float invS = __fdiv_rn(1.f, scale);
    uint16_t h = kotlin_float_to_half(scale);
    o[0] = h & 0xFF; o[1] = h >> 8;
    for (int k = 0; k < 32; k++) o[2 + k] = (uint8_t)(int8_t)kround_coerce(__fmul_rn(x[k], invS), -128, 127);
  } else if constexpr (QT == LK_TYPE_Q4_0) {
    float amax = 0.f;
    for (int k = 0; k < 32; k++) amax = kmax(amax, __builtin_fabsf(x[k]));
    float scale = (amax == 0.f) ? 1.f : __fdiv_rn(amax, 8.f);
    float invS = (scale == 0.f) ? 0.f : __fdiv_rn(1.f, scale);
    uint16_t h = kotlin_float_to_half(scale);
    o[0] = h & 0xFF; o[1] = h >> 8;
    for (int j = 0; j < 16; j++) {
      int32_t q1 = kround_coerce(__fadd_rn(__fmul_rn(x[2 * j], invS), 8.f), 0, 15);
      int32_t q2 = kround_coerce(__fadd_rn(__fmul_rn(x[2 * j + 1], invS), 8.f), 0, 15);
      o[2 + j] = (uint8_t)((q1 & 0xF) | ((q2 & 0xF) << 4));
    }
  } else {
    float fmin = x[0], fmax = x[0];
    for (int k = 1; k < 32; k++) { fmin = kmin(fmin, x[k]); fmax = kmax(fmax, x[k]); }
    float dsc = __fdiv_rn(__fsub_rn(fmax, fmin), 15.f);
    if (dsc == 0.f) dsc = 1.f;
    float invD = __fdiv_rn(1.f, dsc);
    uint16_t hd = kotlin_float_to_half(dsc), hm = kotlin_float_to_half(fmin);
    o[0] = hd & 0xFF; o[1] = hd >> 8; o[2] = hm & 0xFF; o[3] = hm >> 8;
    for (int j = 0; j < 16; j++) {
      int32_t q1 = kround_coerce(__fmul_rn(__fsub_rn(x[2 * j], fmin), invD), 0, 15);
      int32_t q2 = kround_coerce(__fmul_rn(__fsub_rn(x[2 * j + 1], fmin), invD), 0, 15);
      o[4 + j] = (uint8_t)((q1 & 0xF) | ((q2 & 0xF) << 4));
    }
  }
}

}  // namespace lk
