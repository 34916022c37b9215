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

// ---- batch-1 GEMV ----------------------------------------------------------------

// One MUL_MAT node with N == 1 (device-resident operands).
struct GemvDesc {
  const uint8_t *a;   // first byte of A's blocks (buffer base + dataOffset)
  const float *x;     // B column 0 (contiguous K floats)
  float *dst;         // dst(0, 0)
  int64_t dst_row_stride; // elements between dst(0,i) and dst(0,i+1) (= nb[1]/4)
  int32_t M, K;
};

constexpr int kGemvWaves = 4;  // waves per workgroup of the register-streaming kernel

// Register-streaming GEMV: the path for batch-1 shapes the LDS-DMA kernel below does not
// take (K > 12288, rows not 16-byte multiples). One workgroup per kGemvWaves*ROWS rows.
// Each wave owns ROWS consecutive rows; each lane owns block pairs p = lane, lane+64, ...
// of those rows. Per pair the lane loads its 64 activations once (float4, L1/L2-resident)
// and reuses them for all ROWS rows, whose 2·BB-byte pairs it loads with dword-aligned
// vector loads (coalesced at wave level: 64 lanes cover 64·2·BB contiguous bytes of a row).
template <int QT, int ROWS>
__global__ __launch_bounds__(256) void gemv_q_n1_kernel(const GemvDesc d) {
  constexpr int BB = QTraits<QT>::BB;
  constexpr int PDW = QTraits<QT>::PAIR_DW;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = ((int)blockIdx.x * kGemvWaves + wave) * ROWS;
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

// ---- LDS-DMA streaming GEMV (the hot kernel) -------------------------------------
//
// A batch-1 quantized GEMV moves ~0.56 (Q4_0) to ~1.06 (Q8_0) bytes of weights per
// multiply-add, so it is bound by HBM. Keeping HBM busy takes ~40 KB of loads in flight
// per CU; VGPR-destination loads cannot hold that much at useful occupancy. This kernel
// puts the weight bytes in flight with global_load_lds (LDS-DMA: 1 KB per wave
// instruction, no VGPRs) into a per-wave ring of D slots, and decodes from LDS.
//
// Work: a "unit" is 64 consecutive block pairs of one row (one pair per lane). A row of
// K weights is nch = ceil(K/4096) units. A workgroup (kStreamWaves waves, one per CU)
// processes a list of segments (node, row range); each wave takes a contiguous share of
// a segment's rows and streams its units through its ring, D-1 units ahead, waiting
// with a counted vmcnt. The activations of the segment's node are staged once into LDS
// in the decode order and then held in VGPRs (16 float4 per unit of the row).
//
// Q4 decode: v_cvt_pk_f32_fp8 of a nibble n (exponent field 0/1) is exactly n·2^-9, so
// one conversion turns two nibbles into two floats; the sums are rescaled by 512.
// Q8 decode: bytes biased to unsigned (xor 0x80) go through v_cvt_f32_ubyteN.

typedef float f2v __attribute__((ext_vector_type(2)));
#define LK_LDS __attribute__((address_space(3)))

// Cache policy (aux) of the weight stream's LDS-DMA: 2 = nt (bytes read once per launch).
#ifndef LK_WEIGHT_AUX
#define LK_WEIGHT_AUX 2
#endif
// Prologue order: 0 = activations then D weight units; 1 = weight unit 0, activations, units 1..D-1.
#ifndef LK_PROLOGUE_ORDER
#define LK_PROLOGUE_ORDER 0
#endif

constexpr int kStreamWaves = 8;
constexpr int kLdsBytes = 160 * 1024;
constexpr int kStreamMaxUnits = 3;   // units per row held in VGPRs: K <= 12288

// A workgroup's piece of one node: rows [row_begin, row_end) of the node, with the node's
// operands inlined so a workgroup reaches its first weight load after one scalar load.
// Workgroup g owns slots work[g*spw .. g*spw + work[g*spw].count).
struct StreamWork {
  const uint8_t *a;
  const float *x;
  float *dst;
  int64_t dst_row_stride;
  int32_t K, row_begin, row_end, count;
  int64_t pad[2];
};
static_assert(sizeof(StreamWork) == 64, "one s_load_dwordx16");

template <int QT, int CPL> struct StreamGeom {
  static constexpr int PB = 2 * QTraits<QT>::BB;         // bytes per block pair
  static constexpr int PDW = PB / 4;
  static constexpr int UB = 64 * PB;                      // bytes per unit
  static constexpr int L = (UB + 1023) / 1024;            // DMA instructions per unit
  static constexpr int SLOT = L * 1024;
  static constexpr int IMG = 64 * CPL * 256;              // activation image: 256 B per pair
  static constexpr int DFIT = (kLdsBytes - IMG) / (kStreamWaves * SLOT);
  static constexpr int D = DFIT < 3 ? DFIT : 3;            // ring depth (units)
  static constexpr int LDS = IMG + kStreamWaves * D * SLOT;
  static constexpr int VMCNT = (D - 1) * L;               // DMA ops allowed in flight past the unit in use
  static_assert(D >= 2, "ring must double-buffer");
  static_assert(VMCNT < 64, "vmcnt field is 6 bits");
};

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding).
template <int N> __device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | 0x0F70);
}
__device__ __forceinline__ void wait_lgkmcnt0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

template <bool HI> __device__ __forceinline__ f2v fp8x2(uint32_t v) { return __builtin_amdgcn_cvt_pk_f32_fp8(v, HI); }

// Σ (n_k/512)·x_k over the 8 nibbles of dword u; xa = (x0,x2,x4,x6), xb = (x1,x3,x5,x7).
__device__ __forceinline__ f2v nib8(uint32_t u, f32x4 xa, f32x4 xb, f2v s) {
  const uint32_t lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
  s = __builtin_elementwise_fma(fp8x2<false>(lo), f2v{xa.x, xa.y}, s);
  s = __builtin_elementwise_fma(fp8x2<true>(lo), f2v{xa.z, xa.w}, s);
  s = __builtin_elementwise_fma(fp8x2<false>(hi), f2v{xb.x, xb.y}, s);
  s = __builtin_elementwise_fma(fp8x2<true>(hi), f2v{xb.z, xb.w}, s);
  return s;
}

// Σ (q_k+128)·x_k over the 4 signed bytes of dword u; xv = (x0,x1,x2,x3).
__device__ __forceinline__ f2v i8x4(uint32_t u, f32x4 xv, f2v s) {
  const uint32_t b = u ^ 0x80808080u;
  s = __builtin_elementwise_fma(f2v{(float)(b & 0xFF), (float)((b >> 8) & 0xFF)}, f2v{xv.x, xv.y}, s);
  s = __builtin_elementwise_fma(f2v{(float)((b >> 16) & 0xFF), (float)(b >> 24)}, f2v{xv.z, xv.w}, s);
  return s;
}

// One block pair (w = PDW dwords, LDS) against its 64 activations in decode order.
template <int QT>
__device__ __forceinline__ float pair_dot_s(const uint32_t *w, const f32x4 *xr, float xs0, float xs1);

template <>
__device__ __forceinline__ float pair_dot_s<LK_TYPE_Q4_0>(const uint32_t *w, const f32x4 *xr, float xs0, float xs1) {
  // d0 = bytes 0..1, quants 2..17 (realigned by 2); d1 = bytes 18..19, quants 20..35
  f2v s = {0.f, 0.f}, t = {0.f, 0.f};
  s = nib8(align2(w[1], w[0]), xr[0], xr[1], s);
  s = nib8(align2(w[2], w[1]), xr[2], xr[3], s);
  s = nib8(align2(w[3], w[2]), xr[4], xr[5], s);
  s = nib8(align2(w[4], w[3]), xr[6], xr[7], s);
  t = nib8(w[5], xr[8], xr[9], t);
  t = nib8(w[6], xr[10], xr[11], t);
  t = nib8(w[7], xr[12], xr[13], t);
  t = nib8(w[8], xr[14], xr[15], t);
  const float acc = h2f(w[0]) * fmaf(512.f, s.x + s.y, -8.f * xs0);
  return fmaf(h2f(w[4] >> 16), fmaf(512.f, t.x + t.y, -8.f * xs1), acc);
}

template <>
__device__ __forceinline__ float pair_dot_s<LK_TYPE_Q4_1>(const uint32_t *w, const f32x4 *xr, float xs0, float xs1) {
  // (d0,m0) = bytes 0..3, quants 4..19; (d1,m1) = 20..23, quants 24..39
  f2v s = {0.f, 0.f}, t = {0.f, 0.f};
  s = nib8(w[1], xr[0], xr[1], s);
  s = nib8(w[2], xr[2], xr[3], s);
  s = nib8(w[3], xr[4], xr[5], s);
  s = nib8(w[4], xr[6], xr[7], s);
  t = nib8(w[6], xr[8], xr[9], t);
  t = nib8(w[7], xr[10], xr[11], t);
  t = nib8(w[8], xr[12], xr[13], t);
  t = nib8(w[9], xr[14], xr[15], t);
  float acc = fmaf(h2f(w[0]), 512.f * (s.x + s.y), h2f(w[0] >> 16) * xs0);
  acc = fmaf(h2f(w[5] >> 16), xs1, acc);
  return fmaf(h2f(w[5]), 512.f * (t.x + t.y), acc);
}

template <>
__device__ __forceinline__ float pair_dot_s<LK_TYPE_Q8_0>(const uint32_t *w, const f32x4 *xr, float xs0, float xs1) {
  // d0 = bytes 0..1, q = 2..33 (realigned by 2); d1 = bytes 34..35, q = 36..67
  f2v s = {0.f, 0.f}, t = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; k++) s = i8x4(align2(w[k + 1], w[k]), xr[k], s);
#pragma unroll
  for (int k = 0; k < 8; k++) t = i8x4(w[9 + k], xr[8 + k], t);
  const float acc = h2f(w[0]) * fmaf(-128.f, xs0, s.x + s.y);
  return fmaf(h2f(w[8] >> 16), fmaf(-128.f, xs1, t.x + t.y), acc);
}

// DPP reduction over the wave (VALU only); lane 63 ends with the total.
__device__ __forceinline__ float dpp_sum(float v) {
#define LK_DPP(ctrl, rmask, bc) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, rmask, 0xF, bc))
  LK_DPP(0xB1, 0xF, true);    // quad_perm [1,0,3,2]
  LK_DPP(0x4E, 0xF, true);    // quad_perm [2,3,0,1]
  LK_DPP(0x141, 0xF, true);   // row_half_mirror
  LK_DPP(0x140, 0xF, true);   // row_mirror
  LK_DPP(0x142, 0xA, false);  // row_bcast:15
  LK_DPP(0x143, 0xC, false);  // row_bcast:31
#undef LK_DPP
  return v;
}

// Optional per-wave timeline (tools/lab/trace.hip defines LK_STREAM_TRACE): s_memrealtime
// (100 MHz) at kernel entry, activations in VGPRs, first unit decoded, and exit.
#ifdef LK_STREAM_TRACE
__device__ uint64_t *lk_trace_buf;
#define LK_TRACE(slot)                                                                                  \
  do {                                                                                                  \
    if (lane == 0 && lk_trace_buf)                                                                      \
      lk_trace_buf[((size_t)blockIdx.x * kStreamWaves + wave) * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LK_TRACE(slot) do {} while (0)
#endif

// Grid: one workgroup per CU. work == nullptr: one node (`single`), rows split evenly
// over the grid; otherwise workgroup g runs its slots of `work`.
// Requirements (checked by the host): K % 64 == 0, ceil(K/4096) <= CPL, row bytes
// (K/64·PB) % 16 == 0, A and x 16-byte aligned, x contiguous.
template <int QT, int CPL>
__global__ __launch_bounds__(kStreamWaves * 64) void gemv_stream_kernel(const GemvDesc single,
                                                                        const StreamWork *__restrict__ work, int spw) {
  using G = StreamGeom<QT, CPL>;
  extern __shared__ f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint8_t *ring = (uint8_t *)lds + G::IMG + wave * (G::D * G::SLOT);
  LK_TRACE(0);
  const StreamWork *wk = work ? work + (int64_t)blockIdx.x * spw : nullptr;
  const int nseg = wk ? ((const __attribute__((address_space(4))) int32_t *)wk)[offsetof(StreamWork, count) / 4] : 1;
  for (int si = 0; si < nseg; si++) {
    const uint8_t *a_node;
    const float *x_node;
    float *dst_node;
    int64_t dst_stride;
    int K, rb, re;
    if (wk) {
      StreamWork w;  // scalar loads (constant address space: the work list is never written)
      {
        const __attribute__((address_space(4))) uint64_t *src = (const __attribute__((address_space(4))) uint64_t *)(wk + si);
        uint64_t words[sizeof(StreamWork) / 8];
#pragma unroll
        for (int i = 0; i < (int)(sizeof(StreamWork) / 8); i++) words[i] = src[i];
        __builtin_memcpy(&w, words, sizeof(StreamWork));
      }
      a_node = w.a; x_node = w.x; dst_node = w.dst; dst_stride = w.dst_row_stride;
      K = w.K; rb = w.row_begin; re = w.row_end;
    } else {
      a_node = single.a; x_node = single.x; dst_node = single.dst; dst_stride = single.dst_row_stride;
      K = single.K;
      const int per = (single.M + (int)gridDim.x - 1) / (int)gridDim.x;
      rb = min((int)blockIdx.x * per, single.M);
      re = min(rb + per, single.M);
    }
    const int per_w = (re - rb + kStreamWaves - 1) / kStreamWaves;
    const int r0 = __builtin_amdgcn_readfirstlane(min(rb + wave * per_w, re));
    const int nrows = __builtin_amdgcn_readfirstlane(min(r0 + per_w, re) - r0);
    const int NP = K >> 6;                         // block pairs per row
    const int nch = (NP + 63) >> 6;                // units per row
    const int64_t RB = (int64_t)NP * G::PB;        // row bytes
    const int nunits = nrows * nch;
    const LK_GLOBAL uint8_t *A = (const LK_GLOBAL uint8_t *)a_node + (int64_t)r0 * RB;

    // 1. prologue, all by LDS-DMA:
    //    - weights: exactly D units in flight; past the wave's last unit (or for a wave
    //      without rows) the slots are filled from the node's first row and never decoded;
    //    - the activation image: float4 t (x[4t..4t+3]) of pair p at lds[16p + (t ^ (p & 15))]
    //      (XOR swizzle: each DMA instruction reads 1 KB of x contiguously, and the per-lane
    //      reads below hit 64 distinct banks); image float4 i = 64·k + lane comes from DMA
    //      instruction k, issued by wave k % 8.
    //    LK_PROLOGUE_ORDER 1 issues weight unit 0 first, then the image, then units 1..D-1:
    //    the HBM stream starts at once and the wait for the image covers unit 0 too.
    int irow = 0, ich = 0, islot = 0, issued = 0;
    auto dma_unit = [&](const LK_GLOBAL uint8_t *base, int ubytes, int sl) {
      LK_LDS uint8_t *slot = (LK_LDS uint8_t *)(ring + sl * G::SLOT);
#pragma unroll
      for (int j = 0; j < G::L; j++) {
        int off = j * 1024 + lane * 16;
        off = off < ubytes ? off : 0;  // lanes past the unit re-read its first 16 B (never decoded)
        __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(base + off), (LK_LDS void *)(slot + j * 1024), 16, 0,
                                         LK_WEIGHT_AUX);
      }
    };
    auto issue = [&]() {
      dma_unit(A + (int64_t)irow * RB + (int64_t)ich * G::UB, (int)min((int64_t)G::UB, RB - (int64_t)ich * G::UB), islot);
      if (++ich == nch) { ich = 0; ++irow; }
      islot = (islot + 1 == G::D) ? 0 : islot + 1;
      ++issued;
    };
    auto dma_x = [&]() {
      const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)x_node;
      const int ninst = (NP + 3) / 4;  // 64 float4 per instruction
      for (int k = wave; k < ninst; k += kStreamWaves) {
        const int i = k * 64 + lane;          // image position
        const int p = min(i >> 4, NP - 1), t = (i & 15) ^ ((i >> 4) & 15);  // past the last pair: never read
        __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(xv + p * 16 + t), (LK_LDS void *)(lds + k * 64), 16, 0, 0);
      }
    };
    __builtin_amdgcn_s_barrier();  // every wave is done with the previous segment's image
    if (LK_PROLOGUE_ORDER == 0) dma_x();
#pragma unroll
    for (int k = 0; k < G::D; k++) {
      if (LK_PROLOGUE_ORDER == 1 && k == 1) dma_x();
      const bool real = k < nunits;
      const LK_GLOBAL uint8_t *base = real ? A + (int64_t)irow * RB + (int64_t)ich * G::UB : (const LK_GLOBAL uint8_t *)a_node;
      const int ubytes = real ? (int)min((int64_t)G::UB, RB - (int64_t)ich * G::UB) : (int)min((int64_t)G::UB, RB);
      dma_unit(base, ubytes, k);
      if (real) {
        if (++ich == nch) { ich = 0; ++irow; }
        ++issued;
      }
    }
    islot = 0;  // the next unit to issue is unit D, slot D % D

    wait_vmcnt<(LK_PROLOGUE_ORDER == 0 ? G::D : G::D - 1) * G::L>();  // this wave's activation DMA has landed
    __builtin_amdgcn_s_barrier();  // ... and every other wave's

    // 2. activations into VGPRs in decode order, and Σx per block
    f32x4 xr[CPL][16];
    float xs0[CPL], xs1[CPL];
    bool valid[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++) {
      const int p = c * 64 + lane;
      valid[c] = p < NP;
      const int pc = valid[c] ? p : 0;
#pragma unroll
      for (int jj = 0; jj < 8; jj++) {
        const f32x4 n0 = lds[16 * pc + ((2 * jj) ^ (pc & 15))], n1 = lds[16 * pc + ((2 * jj + 1) ^ (pc & 15))];
        if constexpr (QT == LK_TYPE_Q8_0) {
          xr[c][2 * jj] = n0;
          xr[c][2 * jj + 1] = n1;
        } else {  // nibble order: (x0,x2,x4,x6), (x1,x3,x5,x7)
          xr[c][2 * jj] = f32x4{n0.x, n0.z, n1.x, n1.z};
          xr[c][2 * jj + 1] = f32x4{n0.y, n0.w, n1.y, n1.w};
        }
      }
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int t = 0; t < 8; t++) {
        a0 += (xr[c][t].x + xr[c][t].y) + (xr[c][t].z + xr[c][t].w);
        a1 += (xr[c][t + 8].x + xr[c][t + 8].y) + (xr[c][t + 8].z + xr[c][t + 8].w);
      }
      xs0[c] = a0;
      xs1[c] = a1;
    }

    if (si == 0) LK_TRACE(1);
    int slot = 0, u = 0;
    LK_GLOBAL float *out = (LK_GLOBAL float *)dst_node + (int64_t)r0 * dst_stride;
    for (int row = 0; row < nrows; row++) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CPL; c++) {
        if (c < nch) {
          if (u + G::D - 1 < nunits) wait_vmcnt<G::VMCNT>();
          else wait_vmcnt<0>();
          const uint32_t *rp = (const uint32_t *)(ring + slot * G::SLOT + lane * G::PB);
          uint32_t w[G::PDW];
#pragma unroll
          for (int k = 0; k < G::PDW; k++) w[k] = rp[k];
          const float v = pair_dot_s<QT>(w, xr[c], xs0[c], xs1[c]);
          acc += valid[c] ? v : 0.f;
          if (issued < nunits) {
            wait_lgkmcnt0();  // this slot's LDS reads have landed: the DMA may overwrite it
            issue();
          }
          slot = (slot + 1 == G::D) ? 0 : slot + 1;
          ++u;
        }
      }
      if (si == 0 && row == 0) LK_TRACE(2);
      const float tot = dpp_sum(acc);
      if (lane == 63) out[(int64_t)row * dst_stride] = tot;
    }
  }
  LK_TRACE(3);
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
