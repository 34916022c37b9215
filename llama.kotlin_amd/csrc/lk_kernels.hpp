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

#include <type_traits>

#include "../../include/lk_hip.h"
#include "lk_peer.hpp"

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
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#define LK_LDS __attribute__((address_space(3)))

// The weight stream's LDS-DMA uses cache policy nt (aux 2: bytes read once per launch). The
// prologue issues the activation image, then the ring's D weight units. Rows are split over the
// workgroup's waves statically (an eighth each): handing rows out at run time evened the waves'
// exits but made the layer launch slower (26.8-31.0 vs 24.6-25.8 us).

constexpr int kStreamWaves = 8;
constexpr int kLdsBytes = 160 * 1024;
constexpr int kStreamMaxUnits = 3;   // units per row held in VGPRs: K <= 12288

// A workgroup's piece of one node: rows [row_begin, row_end) of the node, with the node's
// operands inlined so a workgroup reaches its first weight load after one scalar load.
// Workgroup g owns slots work[g*spw .. g*spw + work[g*spw].count).
// Lab timelines (built only with -DLK_LAB_STAMPS by tools/build_lab.sh, never in the product
// library): per (workgroup, wave) s_memrealtime stamps and per-wave sums, read by lk_lab_stamps
// (lk_hip.hip) into tools/stamp_kpart.py. Slot meanings are the kernel's (see its LK_KP_SET calls).
#ifdef LK_LAB_STAMPS
__device__ uint64_t lk_kp_stamps[1024][8][10];
#define LK_KP_T() __builtin_amdgcn_s_memrealtime()
#define LK_KP_SET(i, v) do { if (lane == 0 && blockIdx.x < 1024) lk_kp_stamps[blockIdx.x][wave][i] = (v); } while (0)
#else
#define LK_KP_T() 0ull
#define LK_KP_SET(i, v) do { } while (0)
#endif
// Lab (-DLK_LAB_CHAIN_STAMPS, never the product): per (workgroup, segment) stamps of the stream
// kernel's wave 0, lane 0 — slot 0 segment start, 1 stores drained (grid barrier), 2 released, 3
// image ready, 4 x in VGPRs, 5 first unit landed, 6 segment done, 7 the segment's barrier number
#ifdef LK_LAB_CHAIN_STAMPS
__device__ uint64_t lk_chain_stamps[256][256][8];
#define LK_CS(i, v) do { if (tid == 0 && blockIdx.x < 256 && si < 256) lk_chain_stamps[blockIdx.x][si][i] = (v); } while (0)
#else
#define LK_CS(i, v) do { } while (0)
#endif

struct StreamWork {
  const uint8_t *a;
  const float *x;
  float *dst;
  int64_t dst_row_stride;
  int32_t K, row_begin, row_end, count;
  // chain plans (lk_plan_create_chain): barrier > 0 puts grid barrier #barrier−1 before this
  // segment; sync = per barrier 9 words (top, 8 shards), then the exit counter and the timeout
  // flag, each word on a 128-B line of its own (kChainLine words apart)
  int32_t barrier, nbar;
  unsigned *sync;
};
static_assert(sizeof(StreamWork) == 64, "one s_load_dwordx16");


// Device-side waits (only the opt-in chain plans' grid barriers since round 4: the split-K
// reductions elect a last arriver and never wait) are bounded: a wait that gives up counts itself
// in lk_sync_timeout_count (monotonic; lk_sync_timeouts reports the increase since its last call)
// and stores the new count into the host-visible word *lk_sync_fail_flag (page-locked host memory
// the library installs per device). Every synchronous entry point reads that word before its
// launches and again after its sync, and a change becomes LK_ERR_DEVICE: a launch whose wait gave
// up never reports success, whichever thread syncs first. The bound is lk_sync_wait_bound
// s_memrealtime ticks (100 MHz; 200 ms), changed only by lk_set_sync_wait_bound.
__device__ unsigned lk_sync_timeout_count;
__device__ unsigned *lk_sync_fail_flag;
__device__ uint64_t lk_sync_wait_bound = 20000000ull;

__device__ __forceinline__ void lk_note_timeout() {
  const unsigned n = __hip_atomic_fetch_add(&lk_sync_timeout_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  unsigned *f = lk_sync_fail_flag;
  if (f) __hip_atomic_store(f, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


template <int QT> constexpr int stream_pb() {
  if constexpr (QT == LK_TYPE_Q4_K) return LK_Q4_K_BLOCK_BYTES / 4;
  else if constexpr (QT == LK_TYPE_Q2_K) return LK_Q2_K_BLOCK_BYTES / 4;
  else return 2 * QTraits<QT>::BB;
}
#ifndef LK_STREAM_D
#define LK_STREAM_D 3  // stream-kernel ring depth cap (lab: deeper rings)
#endif
template <int QT, int CPL> struct StreamGeom {
  // bytes per 64 items (a lane's share of a unit): a block pair, or a quarter Q4_K block
  static constexpr int PB = stream_pb<QT>();
  static constexpr int PDW = PB / 4;
  static constexpr int UB = 64 * PB;                      // bytes per unit
  static constexpr int L = (UB + 1023) / 1024;            // DMA instructions per unit
  static constexpr int SLOT = L * 1024;                   // a ring slot: the unit's DMA instructions
  static constexpr int IMG = 64 * CPL * 256;              // activation image: 256 B per pair
  static constexpr bool KQ = QT == LK_TYPE_Q4_K || QT == LK_TYPE_Q2_K;
  static constexpr int AUX = KQ ? 256 : 0;                // K-quants: the i/63 (Q4_K) or i/15 (Q2_K) table
  static constexpr int DFIT = (kLdsBytes - IMG - AUX) / (kStreamWaves * SLOT);
  static constexpr int D = DFIT < LK_STREAM_D ? DFIT : LK_STREAM_D;  // ring depth (units in flight per wave)
  static constexpr int TOFF = IMG + kStreamWaves * D * SLOT;
  static constexpr int LDS = TOFF + AUX;
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A lane's 64 items of a Q4_K unit (two 32-item sub-blocks of one block; defined with the
// K-quant dots below): header h (d, dmin, the 12 scale bytes), the sub-blocks' codes c0, c1.
__device__ float q4k_stream_dot(const u32x4 &h, const u32x4 &c0, const u32x4 &c1, int lane, const f32x4 *xr, float xs0,
                                float xs1, const float *q63);
// A lane's 64 items of a Q2_K unit: four 16-item sub-blocks of one block (scale bytes sc, code
// dwords c, d | dmin in dd), activations per 16 in bit-pair order, Σx per 16 in xq.
__device__ float q2k_stream_dot(uint32_t sc, const uint32_t *c, uint32_t dd, const f32x4 *xr, const float *xq,
                                const float *q15);

// Grid: one workgroup per CU. args.work == nullptr: the nodes of args.node (workgroups
// [wg0, wg0 + nwg) per node, rows split evenly over them); otherwise workgroup g runs its slots
// of args.work (chain plans).
// Requirements (checked by the host): K % 64 == 0, ceil(K/4096) <= CPL, row bytes
// (K/64·PB) % 16 == 0, A and x 16-byte aligned, x contiguous. Scalar arguments only (no
// aggregate), the work list first, so the compiler can preload them into SGPRs.
// Ranks of a multi-GPU chain (lk_p2p_chain, lk_hip.hip): one launch per rank, each a chain plan over
// its row shards; rank `rank`'s rows are stored into its own full dst and, at dst + delta[r], into
// every other rank's copy (system-scope write-through stores: over xGMI on a node, plain device
// memory when ranks share a GPU). Barrier #s waits until every rank has completed stage s: the rank
// whose top-counter add completes its stage adds 1 to cross[r] + s·kChainLine of every rank r
// (system scope); a rank's pollers wait for its own word to reach P·(epoch + 1), where epoch counts
// the chain's launches (the words are monotonic: a fast rank's next launch may add before a slow
// rank has left this one, so nothing is re-armed; the rank's last workgroup out bumps its epoch).

template <int QT, int CPL, bool PEER>
__device__ __forceinline__ void gemv_stream_body(const StreamWork *__restrict__ work, int spw, const uint8_t *s_a,
                                                 const float *s_x, float *s_dst, int64_t s_dst_stride, int s_M, int s_K,
                                                 const PeerDesc *__restrict__ peer) {
  using G = StreamGeom<QT, CPL>;
  extern __shared__ f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  [[maybe_unused]] const uint64_t t_entry = LK_KP_T();
  [[maybe_unused]] int st_units = 0;
  [[maybe_unused]] uint64_t t_rec = 0, t_iss = 0, t_img = 0, t_x = 0, t_u0 = 0;  // lab stamps (first segment)
  uint8_t *ring = (uint8_t *)lds + G::IMG + wave * (G::D * G::SLOT);
  float *q63 = (float *)((uint8_t *)lds + G::TOFF);  // K-quants only; published by the prologue's barrier
  if constexpr (QT == LK_TYPE_Q4_K)
    if (tid < 64) q63[tid] = __fdiv_rn((float)tid, 63.0f);
  if constexpr (QT == LK_TYPE_Q2_K)
    if (tid < 16) q63[tid] = __fdiv_rn((float)tid, 15.0f);
  const StreamWork *wk = work ? work + (int64_t)blockIdx.x * spw : nullptr;
  const int nseg = wk ? ((const __attribute__((address_space(4))) int32_t *)wk)[offsetof(StreamWork, count) / 4] : 1;
  int nbar = 0;
  unsigned *sync = nullptr;
  [[maybe_unused]] unsigned cross_target = 0;
  if constexpr (PEER) {  // this launch's barriers complete at P·(epoch + 1) arrivals
    const unsigned ep = __hip_atomic_load(peer->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cross_target = (unsigned)peer->P * (ep + 1u);
  }
#ifdef LK_PF
  // lab (decode-chain prefetch): a plan launch may carry its successor plan's work list in s_a (its
  // slots per workgroup in s_M, the same grid): each wave first reads the first LK_PF units of its
  // rows there with default-policy LDS-DMA into a landing slot of its own that nobody reads (past
  // the kernel's LDS), so they are in L2 / the Infinity Cache when the successor starts. Issued
  // before everything else, so the counted vmcnt waits below (youngest-first) still hold.
  if (wk && s_a && !PEER) {
    const StreamWork *nw = (const StreamWork *)s_a + (int64_t)blockIdx.x * s_M;
    const __attribute__((address_space(4))) StreamWork *cw = (const __attribute__((address_space(4))) StreamWork *)nw;
    const uint8_t *na = cw->a;
    const int nK = cw->K, nrb = cw->row_begin, nre = cw->row_end;
    if (cw->sync == nullptr) {
      const int nNP = nK >> 6, nnch = (nNP + 63) >> 6;
      const int64_t nRB = (int64_t)nNP * G::PB;
      const int nper = (nre - nrb + kStreamWaves - 1) / kStreamWaves;
      const int nr0 = min(nrb + wave * nper, nre), nrows = min(nr0 + nper, nre) - nr0;
      const int64_t bytes = min((int64_t)LK_PF * G::UB, (int64_t)nrows * nnch * G::UB);  // rows are contiguous
      const LK_GLOBAL uint8_t *base = (const LK_GLOBAL uint8_t *)na + (int64_t)nr0 * nRB;
      LK_LDS uint8_t *land = (LK_LDS uint8_t *)((uint8_t *)lds + G::LDS + wave * 1024);
      for (int64_t o = 0; o < bytes; o += 1024) {
        const int64_t off = o + lane * 16 < bytes ? o + lane * 16 : 0;
        __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(base + off), (LK_LDS void *)land, 16, 0, 0);
      }
    }
  }
#endif
  for (int si = 0; si < nseg; si++) {
    const uint8_t *a_node;
    const float *x_node;
    float *dst_node;
    int64_t dst_stride;
    int K, rb, re, bar = 0;
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
      bar = w.barrier; nbar = w.nbar; sync = w.sync;
    } else {
      a_node = s_a; x_node = s_x; dst_node = s_dst; dst_stride = s_dst_stride;
      K = s_K;
      const int per = (s_M + (int)gridDim.x - 1) / (int)gridDim.x;
      rb = min((int)blockIdx.x * per, s_M);
      re = min(rb + per, s_M);
    }
    const int NP = K >> 6;                         // block pairs per row
    const int nch = (NP + 63) >> 6;                // units per row
    const int64_t RB = (int64_t)NP * G::PB;        // row bytes
    const int per_w = (re - rb + kStreamWaves - 1) / kStreamWaves;
    const int r0 = __builtin_amdgcn_readfirstlane(min(rb + wave * per_w, re));
    const int nrows = __builtin_amdgcn_readfirstlane(min(r0 + per_w, re) - r0);
    const int nunits = nrows * nch;
    st_units += nunits;
    LK_CS(0, __builtin_amdgcn_s_memrealtime()); LK_CS(7, (uint64_t)bar);
#ifdef LK_LAB_STAMPS
    asm volatile("" ::"s"(nunits));
    if (si == 0) t_rec = LK_KP_T();
#endif
    const LK_GLOBAL uint8_t *A = (const LK_GLOBAL uint8_t *)a_node + (int64_t)r0 * RB;

    // 1. prologue, all by LDS-DMA:
    //    - weights: exactly D units in flight; past the wave's last unit (or for a wave
    //      without rows) the slots are filled from the node's first row and never decoded;
    //    - the activation image: float4 t (x[4t..4t+3]) of pair p at lds[16p + (t ^ (p & 15))]
    //      (XOR swizzle: each DMA instruction reads 1 KB of x contiguously, and the per-lane
    //      reads below hit 64 distinct banks); image float4 i = 64·k + lane comes from DMA
    //      instruction k, issued by wave k % 8.
    //    The image is issued first, then the weight units (other orders measured no faster:
    //    DESIGN.md §3.1).
    int irow = 0, ich = 0, islot = 0, issued = 0;
    auto advance = [&]() __attribute__((always_inline)) {  // past an issued unit
      if (++ich == nch) {
        ich = 0;
        ++irow;
      }
    };
    auto dma_unit = [&](const LK_GLOBAL uint8_t *base, int ubytes, int sl) {
      LK_LDS uint8_t *slot = (LK_LDS uint8_t *)(ring + sl * G::SLOT);
#pragma unroll
      for (int j = 0; j < G::L; j++) {
        int off = j * 1024 + lane * 16;
        off = off < ubytes ? off : 0;  // lanes past the unit re-read its first 16 B (never decoded)
        __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(base + off), (LK_LDS void *)(slot + j * 1024), 16, 0,
                                         2);
      }
    };
    auto issue = [&]() {
      dma_unit(A + (int64_t)irow * RB + (int64_t)ich * G::UB, (int)min((int64_t)G::UB, RB - (int64_t)ich * G::UB), islot);
      advance();
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
    // chain plans: the node's activations by sc1 loads to registers (they may be another
    // workgroup's outputs of this launch, stored write-through), four per wave and round, then
    // into the image as dma_x places them (image float4 64k + lane from instruction k, by wave k % 8)
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)x_node, 0, K * 4, 0x00020000);
    const int xinst = (NP + 3) / 4, xrounds = (xinst + 4 * kStreamWaves - 1) / (4 * kStreamWaves);
    auto x_issue = [&](int r, f32x4 (&xv)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int k = min(wave + kStreamWaves * (4 * r + q), xinst - 1), i = k * 64 + lane;
        const int p = min(i >> 4, NP - 1), t = (i & 15) ^ ((i >> 4) & 15);
        // sc1 (aux 16) loads: another workgroup's write-through outputs; a multi-GPU rank loads at
        // system scope (sc0 sc1, aux 17): some of those rows were stored by peers
        // (device-scope loads after the acquire measured the same: the chain's cost is the fences)
        xv[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, (p * 16 + t) * 16, 0, PEER ? 17 : 16));
      }
    };
    auto x_store = [&](int r, const f32x4 (&xv)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int k = wave + kStreamWaves * (4 * r + q);
        if (k < xinst) lds[k * 64 + lane] = xv[q];
      }
    };
    auto load_x_sc1 = [&]() __attribute__((always_inline)) {  // every round after all older loads
      for (int r = 0; r < xrounds; r++) {
        f32x4 xv[4];
        x_issue(r, xv);
        wait_vmcnt<0>();
        x_store(r, xv);
      }
    };
    auto weight_prologue = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < G::D; k++) {
        const bool real = k < nunits;
        // a filler (past the wave's last unit) has every lane read the node's first 16 bytes: one
        // cache line per instruction for the CU's address path instead of sixteen (never decoded)
        const LK_GLOBAL uint8_t *base = real ? A + (int64_t)irow * RB + (int64_t)ich * G::UB : (const LK_GLOBAL uint8_t *)a_node;
        const int ubytes = real ? (int)min((int64_t)G::UB, RB - (int64_t)ich * G::UB) : 16;
        dma_unit(base, ubytes, k);
        if (real) {
          advance();
          ++issued;
        }
      }
      islot = 0;  // the next unit to issue is unit D, slot D % D
    };
    if (bar) {
      // chain plans: grid barrier #bar−1 between dependent stages, inside the launch. The previous
      // stage's outputs were stored write-through (sc1) and this stage reads them with sc1 loads
      // only, so neither side needs an L2 write-back or invalidate (MI355X_MICROARCH.md, visibility:
      // valid forms, row 1).
      // 1. every wave's stores have completed; one lane arrives on this workgroup's shard (8 shards,
      //    one 128-B line each); the shard's last arriver arrives on the top word
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      LK_CS(1, __builtin_amdgcn_s_memrealtime());
      unsigned *bsync = sync + (bar - 1) * kChainLine * 9;
      if (wave == 0 && lane == 0) {
        const int sh = (int)blockIdx.x % 8;
        const unsigned shn = (gridDim.x - sh + 7) / 8;  // workgroups of shard sh
        const unsigned prev = __hip_atomic_fetch_add(bsync + (1 + sh) * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == shn - 1) {
          const unsigned top = __hip_atomic_fetch_add(bsync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (PEER) {  // this rank's stage is complete: tell every rank (itself included)
            const unsigned nsh = gridDim.x < 8 ? gridDim.x : 8;
            if (top == nsh - 1) {
              // every workgroup of this rank drained its stores (vmcnt(0)) before it arrived, and the
              // rows went to the peers as system-scope stores: a system-scope release (L2 write-back)
              // and an explicit drain before the cross adds, so no add can overtake them (the
              // compiler may drop the fence's own wait: MI355X_MICROARCH.md, compiler hazard)
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              for (int r = 0; r < peer->P; r++)
                __hip_atomic_fetch_add(peer->cross[r] + (bar - 1) * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
        }
      }
      // 2. the weights do not depend on the previous stage: their stream starts now
      weight_prologue();
      // 3. one lane waits until all 8 shards are complete (bounded: a grid that is not
      //    co-resident sets the timeout flag and runs on instead of hanging)
      if (wave == 0 && lane == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), bound = lk_sync_wait_bound;
        const unsigned nsh = gridDim.x < 8 ? gridDim.x : 8;
        // PEER: this rank's cross word counts the ranks whose stage is complete (monotonic)
        unsigned *wword = PEER ? peer->cross[PEER ? peer->rank : 0] + (bar - 1) * kChainLine : bsync;
        const unsigned want = PEER ? cross_target : nsh;
        while ((PEER ? __hip_atomic_load(wword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                     : __hip_atomic_load(wword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < want) {
          if (__builtin_amdgcn_s_memrealtime() - t0 >= bound) {  // not co-resident: flag it, run on
            __hip_atomic_store(sync + (nbar * 9 + 1) * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lk_note_timeout();
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if constexpr (PEER) {
          // peers wrote this stage's activations into this rank's dst over the fabric: a system-scope
          // acquire (L1 / non-coherent L2 lines invalidated), waited for before the barrier releases
          // the other waves, whose loads below are system-scope too
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      LK_CS(2, __builtin_amdgcn_s_memrealtime());
      asm volatile("" ::: "memory");  // the loads below stay after the poll
      __builtin_amdgcn_s_barrier();
      // 4. the stage's activations (sc1 loads: the youngest, so wait for all)
      load_x_sc1();
      wait_lgkmcnt0();
      __builtin_amdgcn_s_barrier();
    } else if (sync) {  // chain plans, a later segment of a stage (or stage 0): no grid barrier
      if (si > 0) __builtin_amdgcn_s_barrier();  // every wave is done with the previous segment's image
      {  // the first round of activation loads ahead of the weight prologue, waited for alone
        f32x4 xv[4];
        x_issue(0, xv);
        weight_prologue();
        wait_vmcnt<G::D * G::L>();
        x_store(0, xv);
      }
      for (int r = 1; r < xrounds; r++) {
        f32x4 xv[4];
        x_issue(r, xv);
        wait_vmcnt<0>();
        x_store(r, xv);
      }
      wait_lgkmcnt0();
      __builtin_amdgcn_s_barrier();
    } else {
    if (si > 0) __builtin_amdgcn_s_barrier();  // every wave is done with the previous segment's image
    dma_x();
    weight_prologue();
#ifdef LK_LAB_STAMPS
    if (si == 0) t_iss = LK_KP_T();
#endif
    wait_vmcnt<G::D * G::L>();     // this wave's activation DMA has landed
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
#ifdef LK_LAB_STAMPS
    if (si == 0) t_img = LK_KP_T();
#endif
    }
    LK_CS(3, __builtin_amdgcn_s_memrealtime());

    // 2. activations into VGPRs in decode order, and Σx per block (only the node's own chunks:
    //    a grouped launch runs every node at its largest node's class; A/B, four rounds: layer
    //    launch 26.6 -> 26.3 us, chains unchanged)
    f32x4 xr[CPL][16];
    float xs0[CPL], xs1[CPL], xq[CPL][4];
    bool valid[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++) {
      const int p = c * 64 + lane;
      valid[c] = p < NP;
      const int pc = valid[c] ? p : 0;
      if (c > 0 && c >= nch) {  // uniform: no lane of the chunk is valid (chunk 0 always is)
#pragma unroll
        for (int t = 0; t < 16; t++) xr[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        xs0[c] = xs1[c] = 0.f;
        if constexpr (QT == LK_TYPE_Q2_K)
#pragma unroll
          for (int g4 = 0; g4 < 4; g4++) xq[c][g4] = 0.f;
        continue;
      }
#pragma unroll
      for (int jj = 0; jj < 8; jj++) {
        const f32x4 n0 = lds[16 * pc + ((2 * jj) ^ (pc & 15))], n1 = lds[16 * pc + ((2 * jj + 1) ^ (pc & 15))];
        if constexpr (QT == LK_TYPE_Q8_0 || QT == LK_TYPE_Q2_K) {
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
      if constexpr (QT == LK_TYPE_Q2_K) {  // per 16 items: bit-pair order (x_j, x_4+j, x_8+j, x_12+j), Σx
#pragma unroll
        for (int g4 = 0; g4 < 4; g4++) {
          const f32x4 A = xr[c][4 * g4], B = xr[c][4 * g4 + 1], C = xr[c][4 * g4 + 2], Dv = xr[c][4 * g4 + 3];
          xq[c][g4] = ((A.x + A.y) + (A.z + A.w)) + ((B.x + B.y) + (B.z + B.w)) + (((C.x + C.y) + (C.z + C.w)) +
                                                                                   ((Dv.x + Dv.y) + (Dv.z + Dv.w)));
          xr[c][4 * g4] = f32x4{A.x, B.x, C.x, Dv.x};
          xr[c][4 * g4 + 1] = f32x4{A.y, B.y, C.y, Dv.y};
          xr[c][4 * g4 + 2] = f32x4{A.z, B.z, C.z, Dv.z};
          xr[c][4 * g4 + 3] = f32x4{A.w, B.w, C.w, Dv.w};
        }
      }
    }

#ifdef LK_LAB_STAMPS
    asm volatile("" ::"v"(xs0[0]), "v"(xs1[0]));
    if (si == 0) t_x = LK_KP_T();
#endif
#ifdef LK_LAB_CHAIN_STAMPS
    asm volatile("" ::"v"(xs0[0]), "v"(xs1[0]));
    LK_CS(4, __builtin_amdgcn_s_memrealtime());
#endif
    int slot = 0, u = 0;
    LK_GLOBAL float *out = (LK_GLOBAL float *)dst_node + (int64_t)r0 * dst_stride;
    [[maybe_unused]] float peer_keep = 0.f;  // PEER: lane j holds row (64·k + j) of the wave's current block of 64
    for (int row = 0; row < nrows; row++) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CPL; c++) {
        if (c < nch) {
          // the two waves of a SIMD (w, w + 4) take turns at issue priority, one unit each, the
          // younger first: at equal priority the older wins arbitration and the younger finishes
          // its rows alone at the end (A/B, three rounds: layer launch 26.0 -> 25.4 us, decode
          // chain 35.2 -> 34.6 us per layer, 11008x4096 8.45 -> 8.18 us)
          if ((u + (wave >> 2)) & 1) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
          if (u + G::D - 1 < nunits) wait_vmcnt<G::VMCNT>();  // a full ring: D − 1 units issued past unit u
          else wait_vmcnt<0>();
#ifdef LK_LAB_STAMPS
          if (si == 0 && u == 0) t_u0 = LK_KP_T();
#endif
          if (u == 0) LK_CS(5, __builtin_amdgcn_s_memrealtime());
          const uint32_t *rp = (const uint32_t *)(ring + slot * G::SLOT + lane * G::PB);
          uint32_t w[G::PDW];
          u32x4 kh, kc0, kc1;  // Q4_K: block lane/4's header and sub-blocks 2(lane%4), +1
          uint32_t q2s = 0, q2d = 0, q2c[4];  // Q2_K: scale bytes 4(lane%4).., d | dmin, code dwords
          if constexpr (QT == LK_TYPE_Q2_K) {
            const uint32_t *bp = (const uint32_t *)(ring + slot * G::SLOT + (lane >> 2) * LK_Q2_K_BLOCK_BYTES);
            q2s = bp[lane & 3];
#pragma unroll
            for (int t = 0; t < 4; t++) q2c[t] = bp[4 + 4 * (lane & 3) + t];
            q2d = bp[20];
          } else if constexpr (QT == LK_TYPE_Q4_K) {
            const uint8_t *bp = ring + slot * G::SLOT + (lane >> 2) * LK_Q4_K_BLOCK_BYTES;
            kh = *(const u32x4 *)bp;
            kc0 = *(const u32x4 *)(bp + 4 + LK_K_SCALE_SIZE + 32 * (lane & 3));
            kc1 = *(const u32x4 *)(bp + 20 + LK_K_SCALE_SIZE + 32 * (lane & 3));
          } else {
#pragma unroll
            for (int k = 0; k < G::PDW; k++) w[k] = rp[k];
          }
          if (issued < nunits) {
            wait_lgkmcnt0();
            issue();
          }
          float v;
          if constexpr (QT == LK_TYPE_Q4_K) v = q4k_stream_dot(kh, kc0, kc1, lane, xr[c], xs0[c], xs1[c], q63);
          else if constexpr (QT == LK_TYPE_Q2_K) v = q2k_stream_dot(q2s, q2c, q2d, xr[c], xq[c], q63);
          else v = pair_dot_s<QT>(w, xr[c], xs0[c], xs1[c]);
          acc += valid[c] ? v : 0.f;
          slot = (slot + 1 == G::D) ? 0 : slot + 1;
          ++u;
        }
      }
      const float tot = dpp_sum(acc);
      if (lane == 63) {
        if (sync) __hip_atomic_store(out + (int64_t)row * dst_stride, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
        else out[(int64_t)row * dst_stride] = tot;
      }
      if constexpr (PEER) {
        // the rows into every other rank's copy of dst, one contiguous store per peer for each block of
        // up to 64 of the wave's rows (dst is a dense [1, M] vector: lk_p2p_chain_create checks it)
        // instead of a scattered 4-B system-scope store per row and peer
        const float tb = __shfl(tot, 63, kWave);
        if (lane == (row & 63)) peer_keep = tb;
        if ((row & 63) == 63 || row == nrows - 1) {
          const int base = row & ~63, cnt = row - base + 1;
          if (lane < cnt)
            for (int r = 0; r < peer->P; r++)
              if (r != peer->rank)
                __hip_atomic_store((LK_GLOBAL float *)((LK_GLOBAL uint8_t *)(out + (int64_t)(base + lane) * dst_stride) + peer->delta[r]),
                                   peer_keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    LK_CS(6, __builtin_amdgcn_s_memrealtime());
  }
  LK_KP_SET(0, t_entry); LK_KP_SET(4, LK_KP_T()); LK_KP_SET(8, (uint64_t)st_units);
  LK_KP_SET(1, t_rec); LK_KP_SET(2, t_iss); LK_KP_SET(3, t_img); LK_KP_SET(5, t_x); LK_KP_SET(6, t_u0);
  if (sync) {
    // chain plans: the workgroup that leaves last (every workgroup has passed every barrier)
    // re-arms the counters for the next launch (stream order makes the stores visible to it)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wave == 0) {
      unsigned prev = 0;
      if (lane == 0) prev = __hip_atomic_fetch_add(sync + nbar * 9 * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prev = __shfl(prev, 0, kWave);
      if (prev == gridDim.x - 1) {
        for (int b = lane; b <= nbar * 9; b += kWave) __hip_atomic_store(sync + b * kChainLine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (PEER)
          if (lane == 0) {
            // closing barrier: every workgroup of this rank has drained its last stage's stores
            // (its own and the peers'); the launch ends only once every rank's have, so a rank's dst is
            // complete when its own stream is (line nbar of every rank's cross words; then the epoch)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int r = 0; r < peer->P; r++)
              __hip_atomic_fetch_add(peer->cross[r] + nbar * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), bound = lk_sync_wait_bound;
            unsigned *xw = peer->cross[peer->rank] + nbar * kChainLine;
            while (__hip_atomic_load(xw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < cross_target) {
              if (__builtin_amdgcn_s_memrealtime() - t0 >= bound) {
                __hip_atomic_store(sync + (nbar * 9 + 1) * kChainLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lk_note_timeout();
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            __hip_atomic_fetch_add(peer->epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
      }
    }
  }
}

template <int QT, int CPL>
__global__ __launch_bounds__(kStreamWaves * 64) void gemv_stream_kernel(const StreamWork *__restrict__ work, int spw,
                                                                        const uint8_t *s_a, const float *s_x, float *s_dst,
                                                                        int64_t s_dst_stride, int s_M, int s_K) {
  gemv_stream_body<QT, CPL, false>(work, spw, s_a, s_x, s_dst, s_dst_stride, s_M, s_K, nullptr);
}

// One rank of a multi-GPU chain (lk_p2p_chain): the chain-plan stream kernel with peer row stores and
// cross-rank barriers (PeerDesc).
template <int QT, int CPL>
__global__ __launch_bounds__(kStreamWaves * 64) void gemv_stream_peer_kernel(const StreamWork *__restrict__ work, int spw,
                                                                             const PeerDesc *__restrict__ peer) {
  gemv_stream_body<QT, CPL, true>(work, spw, nullptr, nullptr, nullptr, 0, 0, 0, peer);
}

struct GenericArgs {
  const uint8_t *a; const uint8_t *b; uint8_t *dst; // buffer base + dataOffset
  int64_t M, N, K;
  int64_t a_nb0, a_nb1, b_nb0, b_nb1, d_nb0, d_nb1; // byte strides (A's used for F32/F16 only)
};

// ---- batched (N > 1) quantized GEMM on MFMA ------------------------------------
//
// dst(n, m) = Σ_blocks d_blk(m) · (Σ_k c_k(m) · x(n, k)) on v_mfma_f32_16x16x32_bf16, computed
// transposed (C'[n][m] = X[n][k] · W[k][m]) so that a lane's weight row m is also its output
// column: the lane that reads row m's codes applies row m's block scale, and 4 consecutive n of
// one row leave as one 16-byte store. One MFMA spans exactly one 32-weight block.
//
// Weight operand (exact in bf16; small magnitudes: the bf16 MFMA's sum is only ~2⁻¹⁷-accurate
// relative to its largest terms, so the codes stay centred or small):
//   Q4_0: n·2⁻⁹ (fp8 conversion of the masked nibble); the −8 offset enters through the MFMA's
//         C input, C = T = −2⁻⁶·Σx per (block, column) from xsplit_kernel, so p = 2⁻⁹·Σ(n−8)·x;
//         scale 512·d.
//   Q4_1: n·2⁻⁹, scale 512·d, plus m·Σx per block (T = Σx, applied in f32 after the MFMA).
//   Q8_0: q (int8 -> f32 -> bf16), scale d.
// Within a lane's 8 codes the k order is (0,2,4,6,1,3,5,7) for the Q4 types (the order the
// fp8 conversions of the masked nibbles yield); xsplit_kernel writes the activations in it.
//
// Activations: x = hi + lo, hi = bf16(x) truncated, lo = bf16(x − hi) rounded to nearest:
// |x − (hi + lo)| ≤ 2⁻¹⁷|x| at any f32 exponent. Products are exact, sums are f32; the outputs
// are within 2⁻¹⁷·Σ|c·x| (+ f32 accumulation) of the exact product (tests/_util.py SPLIT_REL).
//
// xsplit_kernel writes operand fragments: x-tile t (16 columns), block kb, split s: lane l holds
// x(n = 16t + (l&15), k = 32kb + 8(l>>4) + order[j]) at frag[((t·nblk + kb)·2 + s)·64 + l]
// (16 B), so each operand is one contiguous 1-KB piece; T = mult·Σx at xsum[kb·N16 + n].

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kXSplits = 2;

struct XSplitArgs {
  const uint8_t *b;   // B(n, k) at n·nb0 + k·nb1
  int64_t b_nb0, b_nb1;
  int64_t N, K;
  u32x4 *frag;        // [ntx][nblk][kXSplits][64] x 16 B
  float *xsum;        // [nblk][N16]: mult · Σ_block x
  float mult;
  int32_t q4_order;   // 1: k order (0,2,4,6,1,3,5,7) within each 8; 2: (0,4,1,5,2,6,3,7) (lk_skinny.hpp)
  // optional: blocks [xblocks, grid) zero dst(n, m) at n·z_nb0 + m·z_nb1, m < zM, n < zN (the GEMM that
  // follows adds its two K slices into it: gemm_kpart_kernel's atomic_dst)
  int32_t xblocks, zM, zN;
  uint8_t *zero;
  int64_t z_nb0, z_nb1;
};

// One wave per kXsItems consecutive (x-tile, block) items, every item's loads issued before any is
// used. One item per wave is the fastest measured (C5 55.6 vs 57.3 us with four: 16 waves per CU
// in flight beat 4 waves with 32 loads each).
constexpr int kXsItems = 1;
#ifndef LK_W32_KERNELS  // (lk_w32.hip includes this header for its helpers only)
__global__ __launch_bounds__(256) void xsplit_kernel(XSplitArgs g) {
  if (g.zero && (int)blockIdx.x >= g.xblocks) {  // dst zeroing: 4 columns of one row per thread
    const int c4 = (g.zN + 3) / 4;
    const int64_t i = (int64_t)(blockIdx.x - g.xblocks) * 256 + threadIdx.x;
    if (i >= (int64_t)g.zM * c4) return;
    const int64_t m = i / c4;
    const int n0 = (int)(i % c4) * 4;
    uint8_t *o = g.zero + m * g.z_nb1 + n0 * g.z_nb0;
    if (g.z_nb0 == 4 && n0 + 4 <= g.zN && (((uintptr_t)o) & 15) == 0) {
      *(f32x4 *)o = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      for (int e = 0; e < 4 && n0 + e < g.zN; e++) *(float *)(o + e * g.z_nb0) = 0.f;
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t nblk = g.K / 32, ntx = (g.N + 15) / 16, total = ntx * nblk;
  const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kXsItems;
  if (base >= total) return;
  float v[kXsItems][8];
#pragma unroll
  for (int it = 0; it < kXsItems; it++) {
    const int64_t idx = min(base + it, total - 1);
    const int64_t t = idx / nblk, kb = idx % nblk;
    const int64_t n = 16 * t + (lane & 15);
    const int64_t k0 = 32 * kb + 8 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int kk = g.q4_order == 2 ? ((j >> 1) + 4 * (j & 1)) : g.q4_order ? ((j & 3) * 2 + (j >> 2)) : j;
      v[it][j] = (n < g.N) ? *(const float *)(g.b + n * g.b_nb0 + (k0 + kk) * g.b_nb1) : 0.f;
    }
  }
#pragma unroll
  for (int it = 0; it < kXsItems; it++) {
    const int64_t idx = base + it;
    if (idx >= total) break;
    const int64_t t = idx / nblk, kb = idx % nblk;
    const int64_t n = 16 * t + (lane & 15);
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) part += v[it][j];
    uint32_t hi[4], lo[4];
    float hsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t h[2], l[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t bx = __builtin_bit_cast(uint32_t, v[it][j + q]);
        const float r = v[it][j + q] - __builtin_bit_cast(float, bx & 0xFFFF0000u);  // exact
        uint32_t br = __builtin_bit_cast(uint32_t, r);
        br += 0x7FFFu + ((br >> 16) & 1u);  // round to nearest even (r is finite, |r| < 2^-7·|x|)
        h[q] = bx;
        l[q] = br;
        // q4_order 2 (codes 128 + n) cancels a 136-fold offset against this sum: take it over the
        // split itself, hi + lo, so the split's own error is not amplified
        if (g.q4_order == 2) hsum += __builtin_bit_cast(float, bx & 0xFFFF0000u) + __builtin_bit_cast(float, br & 0xFFFF0000u);
      }
      hi[j / 2] = __builtin_amdgcn_perm(h[1], h[0], 0x07060302u);
      lo[j / 2] = __builtin_amdgcn_perm(l[1], l[0], 0x07060302u);
    }
    g.frag[(idx * kXSplits + 0) * 64 + lane] = u32x4{hi[0], hi[1], hi[2], hi[3]};
    g.frag[(idx * kXSplits + 1) * 64 + lane] = u32x4{lo[0], lo[1], lo[2], lo[3]};
    if (g.q4_order == 2) part = hsum;
    part += __shfl_xor(part, 16, kWave);
    part += __shfl_xor(part, 32, kWave);
    if (lane < 16) g.xsum[kb * (ntx * 16) + n] = g.mult * part;
  }
}
#endif

// bf16 codes 128 + n of the 8 nibbles of dword u, slots in k order (0,4,1,5,2,6,3,7).
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t o) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(m), "v"(o));  // one VALU (the compiler splits it)
  return r;
}
__device__ __forceinline__ bf16x8 q4_codes_128(uint32_t u) {
  constexpr uint32_t M = 0x000F000Fu, E = 0x43004300u;
  uint32_t w[4] = {and_or(u, M, E), and_or(u >> 4, M, E), and_or(u >> 8, M, E), and_or(u >> 12, M, E)};
  return __builtin_bit_cast(bf16x8, w);
}

// two f32 whose values fit in 8 significant bits -> their exact bf16 pair (lo, hi)
__device__ __forceinline__ uint32_t pack_bf16_exact(float lo, float hi) {
  return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07060302u);
}

// Weight operand of one block for the lane's row, from the code dword(s) of lane group g.
template <int QT> __device__ __forceinline__ bf16x8 w_frag(uint32_t u0, uint32_t u1);
template <int QT> struct Q4Frag {
  static __device__ __forceinline__ bf16x8 make(uint32_t u) {
    const uint32_t lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;  // n0,n2,n4,n6 / n1,n3,n5,n7
    const f2v e0 = fp8x2<false>(lo), e1 = fp8x2<true>(lo), o0 = fp8x2<false>(hi), o1 = fp8x2<true>(hi);
    uint32_t w[4] = {pack_bf16_exact(e0.x, e0.y), pack_bf16_exact(e1.x, e1.y), pack_bf16_exact(o0.x, o0.y),
                     pack_bf16_exact(o1.x, o1.y)};
    return __builtin_bit_cast(bf16x8, w);  // n·2⁻⁹ for k = 0,2,4,6,1,3,5,7
  }
};
template <> __device__ __forceinline__ bf16x8 w_frag<LK_TYPE_Q4_0>(uint32_t u, uint32_t) { return Q4Frag<0>::make(u); }
template <> __device__ __forceinline__ bf16x8 w_frag<LK_TYPE_Q4_1>(uint32_t u, uint32_t) { return Q4Frag<0>::make(u); }
template <>
__device__ __forceinline__ bf16x8 w_frag<LK_TYPE_Q8_0>(uint32_t u0, uint32_t u1) {
  u0 ^= 0x80808080u;
  u1 ^= 0x80808080u;
  const f2v off = {-128.f, -128.f};
  const f2v a = f2v{(float)(u0 & 0xFF), (float)((u0 >> 8) & 0xFF)} + off, b = f2v{(float)((u0 >> 16) & 0xFF), (float)(u0 >> 24)} + off,
            c = f2v{(float)(u1 & 0xFF), (float)((u1 >> 8) & 0xFF)} + off, d = f2v{(float)((u1 >> 16) & 0xFF), (float)(u1 >> 24)} + off;
  uint32_t w[4] = {pack_bf16_exact(a.x, a.y), pack_bf16_exact(b.x, b.y), pack_bf16_exact(c.x, c.y), pack_bf16_exact(d.x, d.y)};
  return __builtin_bit_cast(bf16x8, w);
}

template <int QT> struct GemmQ {
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr bool USES_T = (QT != LK_TYPE_Q8_0);  // per-(block, column) sums needed
  static constexpr bool C_FROM_T = (QT == LK_TYPE_Q4_0);  // T is the MFMA's C input
  static constexpr bool HAS_MIN = (QT == LK_TYPE_Q4_1);  // acc += s2·T after the MFMA
  static constexpr float MULT = (QT == LK_TYPE_Q4_0) ? -0.015625f : 1.f;  // T = MULT·Σx
  static constexpr int CODE = (QT == LK_TYPE_Q4_1) ? 4 : 2;  // byte offset of the codes in a block
  static constexpr int GSTRIDE = (QT == LK_TYPE_Q8_0) ? 8 : 4;
};

// Code dword(s) of lane group g and the block scale terms: acc += s1·p (+ s2·T for Q4_1).
template <int QT, typename Ptr>
__device__ __forceinline__ void read_block(Ptr blk, int g, uint32_t &u0, uint32_t &u1, float &s1, float &s2) {
  typedef uint16_t u16_ua __attribute__((aligned(1)));
  typedef uint32_t u32_ua __attribute__((aligned(1)));
  const float d = h2f(*(const u16_ua *)blk);
  s1 = (QT == LK_TYPE_Q8_0) ? d : 512.f * d;
  u0 = *(const u32_ua *)(blk + GemmQ<QT>::CODE + GemmQ<QT>::GSTRIDE * g);
  u1 = (QT == LK_TYPE_Q8_0) ? *(const u32_ua *)(blk + 6 + 8 * g) : 0u;
  s2 = GemmQ<QT>::HAS_MIN ? h2f(*(const u16_ua *)(blk + 2)) : 0.f;  // m
}

struct GemmArgs {
  const uint8_t *a;      // weights (buffer base + dataOffset)
  const u32x4 *frag;     // xsplit output
  const float *xsum;
  uint8_t *dst;
  int64_t d_nb0, d_nb1;
  int32_t M, N, K;
  int32_t tiles_m, tiles_n, slices, kslice;  // split-K: slice s covers blocks [s·kslice, (s+1)·kslice)
  float *partial;        // [slices][tiles_m·tiles_n][BM·BN] (slices > 1)
  int32_t *counter;      // [tiles_m·tiles_n], zero between launches
};

// acc += s1·p (+ s2·T for Q4_1), as packed FMAs.
template <bool HAS_MIN>
__device__ __forceinline__ void accumulate(f32x4 &acc, float s1, float s2, f32x4 p, f32x4 t) {
  f2v a0 = {acc.x, acc.y}, a1 = {acc.z, acc.w};
  if constexpr (HAS_MIN) {
    const f2v m2 = {s2, s2};
    a0 = __builtin_elementwise_fma(m2, f2v{t.x, t.y}, a0);
    a1 = __builtin_elementwise_fma(m2, f2v{t.z, t.w}, a1);
  }
  const f2v m1 = {s1, s1};
  a0 = __builtin_elementwise_fma(m1, f2v{p.x, p.y}, a0);
  a1 = __builtin_elementwise_fma(m1, f2v{p.z, p.w}, a1);
  acc = f32x4{a0.x, a0.y, a1.x, a1.y};
}

// acc += s1·p (+ s2·T for Q4_1) as four scalar FMAs: v_pk_fma_f32 beside MFMAs costs more
// issue time than two v_fma_f32 (MI355X_MICROARCH.md, cycle constants), and the library is
// built with -fno-slp-vectorize so the compiler does not pack these back.
// A SIMD issues a wave64 v_pk_fma_f32 as fast as a v_fma_f32 (round-2 lab tool valu_rate.hip, removed, see DESIGN §3: ~4.3-4.7
// cycles each at one or two waves per SIMD). Measured per kernel (round-2 lab A/B pk_ab.sh, two boxes):
// the wide GEMM runs C5 2-3 % faster with the packed form (accumulate), the wave-pair skinny
// kernel 1-3 % slower, so each keeps its own.
template <bool HAS_MIN>
__device__ __forceinline__ void accumulate_s(f32x4 &acc, float s1, float s2, f32x4 p, f32x4 t) {
  if constexpr (HAS_MIN) {
    acc.x = fmaf(s2, t.x, acc.x); acc.y = fmaf(s2, t.y, acc.y);
    acc.z = fmaf(s2, t.z, acc.z); acc.w = fmaf(s2, t.w, acc.w);
  }
  acc.x = fmaf(s1, p.x, acc.x); acc.y = fmaf(s1, p.y, acc.y);
  acc.z = fmaf(s1, p.z, acc.z); acc.w = fmaf(s1, p.w, acc.w);
}

__device__ __forceinline__ bool splitk_arrive(unsigned *cnt, unsigned slices);  // below

// Epilogue shared by the GEMM kernels: lane holds C'(n = 16·xtile + 4(lane>>4) + e, m = row),
// e = 0..3. slices == 1: store. Split-K: publish this slice's tile; the last slice to arrive sums
// all slices in slice order (deterministic) and stores, then re-arms the tile counter.
template <int MT, int NT, int BM, int BN>
__device__ __forceinline__ void gemm_finish(const GemmArgs &g, f32x4 (&acc)[MT][NT], int tile, int tiles, int slice, int tm,
                                            int tn, int wm, int wn, int wave, int lane) {
  const int gq = lane >> 4;
  auto store = [&](int i, int j, f32x4 v) __attribute__((always_inline)) {
    const int64_t m = (int64_t)tm * BM + (wm * MT + i) * 16 + (lane & 15);
    const int64_t n0 = (int64_t)(tn * (BN / 16) + wn * NT + j) * 16 + gq * 4;
    if (m >= g.M) return;
    const float e[4] = {v.x, v.y, v.z, v.w};
    if (g.d_nb0 == 4 && n0 + 4 <= g.N && ((((uintptr_t)g.dst + m * g.d_nb1 + n0 * 4) & 15) == 0)) {
      *(f32x4 *)(g.dst + m * g.d_nb1 + n0 * 4) = v;
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (n0 + q < g.N) *(float *)(g.dst + m * g.d_nb1 + (n0 + q) * g.d_nb0) = e[q];
  };
  if (g.slices == 1) {
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) store(i, j, acc[i][j]);
    return;
  }
  // The tile's slab rows are handed to the last arriver by hand-off row 1 of MI355X_MICROARCH.md
  // (as splitk_arrive for the other kernels): written through (sc1), every wave's stores drained
  // (vmcnt(0)), a workgroup barrier, then one lane's agent-scope add; the last arriver reads the
  // slabs with sc1 loads and re-arms the counter with an atomic store. Round 4 published them with
  // plain stores behind per-thread __threadfence(), read them back with plain loads and re-armed the
  // counter with a plain store — none of the guide's validated forms.
  const int tile_elems = BM * BN;
  const int lin0 = wave * MT * NT * 256;  // wave-local layout: [wave][i][j][lane][4]
  const int64_t pbytes = (int64_t)g.slices * tiles * tile_elems * 4;  // < 2^31 (host-checked)
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, (int)pbytes, 0x00020000);
  auto at = [&](int sl, int i, int j) __attribute__((always_inline)) {  // byte offset of a lane's f32x4
    return (int)(((((int64_t)sl * tiles + tile) * tile_elems) + lin0 + (i * NT + j) * 256 + 4 * lane) * 4);
  };
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), prs, at(slice, i, j), 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) last = splitk_arrive((unsigned *)g.counter + tile, (unsigned)g.slices);
  __syncthreads();
  if (!last) return;
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      f32x4 sum = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, at(0, i, j), 0, 16));  // slab 0 as is
      for (int sl = 1; sl < g.slices; sl++) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, at(sl, i, j), 0, 16));
        sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
      }
      store(i, j, sum);
    }
}

// Direct-load variant (any K % 32 == 0): 4 waves in a WM × WN grid, wave tile MT weight tiles
// (16 rows) × NT x-tiles (16 columns); weights and activation fragments go global -> VGPRs one
// block ahead of the MFMAs.
template <int QT, int WM, int WN, int MT, int NT>
__global__ __launch_bounds__(256) void gemm_q_mfma_kernel(GemmArgs g) {
  using Q = GemmQ<QT>;
  constexpr int BB = Q::BB;
  constexpr int BM = WM * MT * 16, BN = WN * NT * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int tiles = g.tiles_m * g.tiles_n;
  const int tile = (int)blockIdx.x % tiles, slice = (int)blockIdx.x / tiles;
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int nblk = g.K / 32;
  const int kb0 = slice * g.kslice, kb1 = min(kb0 + g.kslice, nblk);
  const int64_t RB = (int64_t)nblk * BB;
  const int gq = lane >> 4;
  const int ntx = (g.N + 15) / 16;

  int64_t wrow[MT];  // this lane's weight row per tile (clamped to M-1)
#pragma unroll
  for (int i = 0; i < MT; i++) wrow[i] = min((int64_t)tm * BM + (wm * MT + i) * 16 + (lane & 15), (int64_t)g.M - 1);
  int xt[NT];        // x-tile index per tile (clamped)
#pragma unroll
  for (int j = 0; j < NT; j++) xt[j] = min(tn * (BN / 16) + wn * NT + j, ntx - 1);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const LK_GLOBAL u32x4 *fr = (const LK_GLOBAL u32x4 *)g.frag;
  const LK_GLOBAL f32x4 *xs = (const LK_GLOBAL f32x4 *)g.xsum;
  struct Blk {
    uint32_t u0[MT], u1[MT];
    float s1[MT], s2[MT];
    u32x4 xf[NT][kXSplits];
    f32x4 t[NT];
  };
  auto load_block = [&](int kb, Blk &o) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MT; i++)
      read_block<QT>((const LK_GLOBAL uint8_t *)g.a + wrow[i] * RB + (int64_t)kb * BB, gq, o.u0[i], o.u1[i], o.s1[i], o.s2[i]);
#pragma unroll
    for (int j = 0; j < NT; j++) {
#pragma unroll
      for (int sp = 0; sp < kXSplits; sp++) o.xf[j][sp] = fr[(((int64_t)xt[j] * nblk + kb) * kXSplits + sp) * 64 + lane];
      if constexpr (Q::USES_T) o.t[j] = xs[((int64_t)kb * (ntx * 16) + xt[j] * 16 + gq * 4) / 4];
      else o.t[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  Blk cur, nxt;
  if (kb0 < kb1) load_block(kb0, cur);
  for (int kb = kb0; kb < kb1; kb++) {
    if (kb + 1 < kb1) load_block(kb + 1, nxt);
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const bf16x8 wf = w_frag<QT>(cur.u0[i], cur.u1[i]);
#pragma unroll
      for (int j = 0; j < NT; j++) {
        f32x4 p = Q::C_FROM_T ? cur.t[j] : f32x4{0.f, 0.f, 0.f, 0.f};
        p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cur.xf[j][1]), wf, p, 0, 0, 0);
        p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cur.xf[j][0]), wf, p, 0, 0, 0);
        accumulate<Q::HAS_MIN>(acc[i][j], cur.s1[i], cur.s2[i], p, cur.t[j]);
      }
    }
    if (kb + 1 < kb1) cur = nxt;
  }
  gemm_finish<MT, NT, BM, BN>(g, acc, tile, tiles, slice, tm, tn, wm, wn, wave, lane);
}

// LDS-DMA issued through inline asm: the compiler's waitcnt pass cannot tell which LDS bytes a
// pending global_load_lds writes and inserts vmcnt(0) before LDS reads it cannot disambiguate,
// which drains the whole ring every stage. Hidden from it, the kernel orders the DMA itself
// (counted vmcnt + s_barrier). SGPR base + 32-bit VGPR offset; M0 = wave-uniform LDS
// destination, lane i lands at M0 + 16i. (Only 16-byte pieces: a 12-byte piece does not land
// at M0 + 12i.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <bool NT>
__device__ __forceinline__ void dma16(const void *sbase, uint32_t vofs, const void *lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LK_LDS const void *)lds_dst);
  // the base must live in SGPRs; say so even where uniformity analysis cannot prove it
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  const uint32_t sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);  // (readfirstlane returns int:
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));  //  no sign extension)
  sbase = (const void *)(((uint64_t)sb_hi << 32) | (uint64_t)sb_lo);
  if constexpr (NT) asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1 nt" ::"v"(vofs), "s"(sbase), "s"(m0) : "memory", "m0");
  else asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(vofs), "s"(sbase), "s"(m0) : "memory", "m0");
}
// The same with the LDS destination as a wave-uniform LDS address (no generic-pointer cast per call).
__device__ __forceinline__ void dma16m(const void *sbase, uint32_t vofs, uint32_t m0) {
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  const uint32_t sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  sbase = (const void *)(((uint64_t)sb_hi << 32) | (uint64_t)sb_lo);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(vofs), "s"(sbase), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop

// LDS-DMA pipelined variant: NW waves stacked along M (wave tile: MT = 2 weight tiles × NT
// x-tiles; BM = 32·NW, BN = 16·NT), K in stages of SB = 4 blocks. Each stage — the workgroup's
// BM rows × 4 blocks of raw weight bytes (rounded up to 16-byte pieces; rows then start
// 8-byte aligned), the 4·NT·2 activation fragments (1 KB each) and the T sums — moves
// global -> LDS by LDS-DMA into a ring of D stages. Every wave issues the same number of DMA
// instructions per stage, so a counted vmcnt plus one barrier publishes a stage, and D-1 stages
// stay in flight while the MFMAs consume the oldest. Per-lane DMA offsets are fixed for the
// launch; only the SGPR bases move with the stage.
constexpr int kLdsSB = 4;

template <int QT, int NT, int NW> struct LdsGemmGeom {
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr int SB = kLdsSB;
  static constexpr int MT = 2, BM = NW * MT * 16, BN = 16 * NT;
  static constexpr int AROWP = (SB * BB + 15) / 16 * 16;   // LDS bytes per row per stage
  static constexpr int A_INST = BM * (AROWP / 16) / 64;     // DMA instructions for A
  static constexpr int X_INST = SB * NT * kXSplits;
  static constexpr int T_INST = GemmQ<QT>::USES_T ? 1 : 0;
  // per wave per stage: each kind padded to a multiple of the NW waves, so that a wave's c-th
  // instruction has a compile-time kind (A: c < CA, X: c < CA + CX, T: the rest)
  static constexpr int CA = (A_INST + NW - 1) / NW, CX = (X_INST + NW - 1) / NW, CT = (T_INST + NW - 1) / NW;
  static constexpr int C = CA + CX + CT;
  static constexpr int A_BYTES = BM * AROWP;
  static constexpr int X_BYTES = X_INST * 1024;
  static constexpr int T_BYTES = T_INST * 1024;
  static constexpr int STAGE = A_BYTES + X_BYTES + T_BYTES;
  static constexpr int DFIT = (150 * 1024) / STAGE;
  static constexpr int D = DFIT > 4 ? 4 : DFIT;
  static constexpr int LDS = D * STAGE;
  static constexpr int OVERREAD = AROWP - SB * BB;          // bytes read past a row's stage bytes
  static_assert((BM * (AROWP / 16)) % 64 == 0, "A pieces");
  static_assert(SB * BN / 4 <= 64, "T sums in one DMA instruction");
  static_assert(D >= 2, "ring");
  static_assert((D - 1) * C < 64, "vmcnt");
};

template <int QT, int NT, int NW>
__global__ __launch_bounds__(NW * 64) void gemm_q_lds_kernel(GemmArgs g) {
  using G = LdsGemmGeom<QT, NT, NW>;
  using Q = GemmQ<QT>;
  constexpr int MT = G::MT, BM = G::BM, BN = G::BN, BB = G::BB, SB = G::SB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles = g.tiles_m * g.tiles_n;
  const int tile = (int)blockIdx.x % tiles, slice = (int)blockIdx.x / tiles;
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int nblk = g.K / 32;
  const int kb0 = slice * g.kslice, kb1 = min(kb0 + g.kslice, nblk);
  const int nst = (kb1 - kb0) / SB;  // stages (kslice is a multiple of SB)
  const int64_t RB = (int64_t)nblk * BB;
  const int gq = lane >> 4;
  const int ntx = (g.N + 15) / 16;
  const int n16 = ntx * 16;

  // This wave's DMA instructions: slot c < CA moves A piece-instruction min(wave·CA + c, A_INST-1),
  // CA <= c < CA+CX the X fragment min(wave·CX + c', X_INST-1), the last CT the T sums (padding
  // repeats an instruction: same bytes to the same place). Per lane: the byte offset from the
  // kind's stage base (fixed for the launch) and the LDS byte offset within a stage (uniform).
  uint32_t vofs[G::C];
  int ldso[G::C];
#pragma unroll
  for (int c = 0; c < G::C; c++) {
    if (c < G::CA) {
      const int q = min(wave * G::CA + c, G::A_INST - 1);
      const int piece = q * 64 + lane;
      const int r = piece / (G::AROWP / 16), pc = piece % (G::AROWP / 16);
      const int64_t row = min((int64_t)tm * BM + r, (int64_t)g.M - 1);
      vofs[c] = (uint32_t)(row * RB + pc * 16);
      ldso[c] = q * 1024;
    } else if (c < G::CA + G::CX) {
      const int x = min(wave * G::CX + (c - G::CA), G::X_INST - 1);  // (block b, tile j, split sp)
      const int b = x / (NT * kXSplits), j = (x / kXSplits) % NT, sp = x % kXSplits;
      const int xt = min(tn * NT + j, ntx - 1);
      vofs[c] = (uint32_t)((((int64_t)xt * nblk + b) * kXSplits + sp) * 1024 + lane * 16);
      ldso[c] = G::A_BYTES + x * 1024;
    } else {
      const int li = min(lane, SB * BN / 4 - 1);  // lane -> (block li / (BN/4), 4 columns)
      const int b = li / (BN / 4), c4 = li % (BN / 4);
      const int n = min(tn * BN + 4 * c4, n16 - 4);
      vofs[c] = (uint32_t)(((int64_t)b * n16 + n) * 4);
      ldso[c] = G::A_BYTES + G::X_BYTES;
    }
  }
  auto issue_stage = [&](int st, int sl) __attribute__((always_inline)) {
    const int kb = kb0 + min(st, nst - 1) * SB;  // past the last stage: reload the last (never read)
    const uint8_t *base_a = g.a + (int64_t)kb * BB;
    const uint8_t *base_x = (const uint8_t *)g.frag + (int64_t)kb * kXSplits * 1024;
    const uint8_t *base_t = (const uint8_t *)(g.xsum + (int64_t)kb * n16);
    uint8_t *slot = smem + sl * G::STAGE;
#pragma unroll
    for (int c = 0; c < G::C; c++) {
      if (c < G::CA) dma16<true>(base_a, vofs[c], slot + ldso[c]);
      else if (c < G::CA + G::CX) dma16<false>(base_x, vofs[c], slot + ldso[c]);
      else dma16<false>(base_t, vofs[c], slot + ldso[c]);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nst > 0) {
    for (int st = 0; st < G::D; st++) issue_stage(st, st);
    int slot = 0;
    for (int st = 0; st < nst; st++) {
      wait_vmcnt<(G::D - 1) * G::C>();
      __builtin_amdgcn_s_barrier();
      const uint8_t *A = smem + slot * G::STAGE;
      const uint8_t *X = A + G::A_BYTES;
      const float *T = (const float *)(X + G::X_BYTES);
#pragma unroll 1
      for (int b = 0; b < SB; b++) {  // not unrolled: keeps the fragment reads of one block live
        bf16x8 wf[MT];
        float s1[MT], s2[MT];
#pragma unroll
        for (int i = 0; i < MT; i++) {
          const uint8_t *blk = A + ((wave * MT + i) * 16 + (lane & 15)) * G::AROWP + b * BB;
          uint32_t u0, u1;
          read_block<QT>(blk, gq, u0, u1, s1[i], s2[i]);
          wf[i] = w_frag<QT>(u0, u1);
        }
#pragma unroll
        for (int j = 0; j < NT; j++) {
          const u32x4 *xf = (const u32x4 *)(X + ((b * NT + j) * kXSplits) * 1024) + lane;
          const bf16x8 xh = __builtin_bit_cast(bf16x8, xf[0]), xl = __builtin_bit_cast(bf16x8, xf[64]);
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
          if constexpr (Q::USES_T) t = *(const f32x4 *)(T + b * BN + j * 16 + gq * 4);
#pragma unroll
          for (int i = 0; i < MT; i++) {
            f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl, wf[i], Q::C_FROM_T ? t : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, wf[i], p, 0, 0, 0);
            accumulate<Q::HAS_MIN>(acc[i][j], s1[i], s2[i], p, t);
          }
        }
      }
      wait_lgkmcnt0();
      __builtin_amdgcn_s_barrier();  // every wave is done with this slot
      issue_stage(st + G::D, slot);
      slot = (slot + 1 == G::D) ? 0 : slot + 1;
    }
    wait_vmcnt<0>();  // drain the padding stages before the workgroup's LDS is released
  }
  gemm_finish<MT, NT, BM, BN>(g, acc, tile, tiles, slice, tm, tn, wave, 0, wave, lane);
}

// ---- skinny batched GEMM (2 <= N <= 32): split-K, activations held in VGPRs ---------------
//
// C3's shape (M 11,008, K 4,096, N 32) is still bound by HBM (114 flop per weight byte). Its
// weight stream only runs near HBM speed when each row's DMA piece is long — pieces that
// straddle 128-B lines are fetched twice under `nt` (16 rows x 144 B stream at 3.8 TB/s,
// 8 x 288 B at 5.6, 1 x 2,304 B at 6.3: round-1 lab tool pieces.hip) — and re-reading the
// activations per 16-row tile from LDS left every block waiting on an LDS round trip. So:
//
//   workgroup (range r, slice s): rows of range r x blocks [s·SB, s·SB + SB) of K, one wave
//     per SIMD (4 waves, up to 512 VGPRs each).
//   prologue: each wave starts its weight stream (LDS-DMA), the workgroup converts the slice's
//     activations x(n, k) once into bf16 hi/lo MFMA fragments (x = hi + lo, |x - hi - lo| <=
//     2^-17|x|) staged in LDS, and every wave then holds ALL of them in VGPRs (SB·NT·2·4 =
//     256 VGPRs at N 32): in the main loop only the weight codes come from LDS.
//   main loop: a wave takes one 16-row tile at a time; its unit (16 rows x SB·BB bytes: 288 B
//     per row for Q4_0) lands in the wave's ring of D slots; per block and 16-column x-tile,
//     two v_mfma_f32_16x16x32_bf16 (lo, hi) on exact weight codes, then acc += scale·p:
//       Q4_0: codes (n - 8)·2^-9 (fp8 conversion of the nibble, minus 2^-6), scale 512·d;
//       Q4_1: codes n·2^-9, scale 512·d, plus m·Σx (Σx per block and column, from LDS);
//       Q8_0: codes q, scale d.
//   output: one slice -> dst directly; otherwise an f32 partial slab P[s][m][n] per slice and
//     splitk_reduce_kernel sums the slabs in slice order (deterministic).
//
// A slot holds the unit row-major at a pitch of one extra 16-B cell per row (lanes of one DMA
// instruction read consecutive 16-B pieces of a row; the pad cell keeps the 16 rows' dwords at
// one block offset 2-way bank-conflicted at worst). At the start of a unit a wave reads every
// dword its blocks need (WPB per block) with one burst of LDS reads and one wait.

// Weight DMA policy of the skinny GEMM: default (0) keeps lines in L2, where the neighbouring
// slice's workgroup (same XCD) reads the 128-B line its piece shares with this one. Measured
// instead, the skinny kernels stream with nt: A/B, three rounds, wave-pair kernel C3 Q4_0
// 20.6 -> 20.2 us, Q4_1 20.6-20.8 -> 20.0-20.4 us; one-wave kernel Q4_0 11008x4096 N = 8
// 16.5-17.0 -> 16.3 us, N = 16 16.7-17.3 -> 16.4-16.7 us (nt on gemm_wide_kernel's weight pieces,
// which every CU of a row band re-reads from L2, was 15 % slower: C5 53.3 -> 61.5 us).

template <int QT, int NT> struct SkinnyGeom {
  static constexpr int NW = 4;                         // waves per workgroup: one per SIMD
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr int SB = 16;                        // blocks per K slice
  static constexpr int RP = SB * BB;                   // row bytes of one unit (a multiple of 16)
  static constexpr int PPR = RP / 16;                  // 16-B pieces per row
  static constexpr int PITCH = RP + 16;                // LDS row pitch: one pad cell per row (banks)
  static constexpr int L = (16 * (PPR + 1) + 63) / 64; // DMA instructions per unit
  static constexpr int WPB = QT == LK_TYPE_Q4_1 ? 2 : QT == LK_TYPE_Q4_0 ? 3 : 4;  // code/scale dwords per block
  static constexpr int SLOT = L * 1024;
  static constexpr int XB = SB * NT * kXSplits * 1024; // activation fragments (staging)
  static constexpr int TB = SB * NT * 16 * 4;          // Σx per (block, column) (Q4_1)
  static constexpr int DFIT = (kLdsBytes - XB - TB) / (NW * SLOT);
  static constexpr int D = DFIT > 4 ? 4 : DFIT;         // ring depth (units per wave)
  static constexpr int LDS = XB + TB + NW * D * SLOT;
  static constexpr int FPW = SB * NT / NW;             // fragments each wave converts
  static_assert(RP % 16 == 0, "row pieces");
  static_assert(D >= 2, "ring must double-buffer");
  static_assert((SB * NT) % NW == 0, "fragments per wave");
  static_assert((D - 1) * L + D * NT < 64, "vmcnt");
};

struct SkinnyArgs {
  const uint8_t *a;        // weights (buffer base + dataOffset), rows RB bytes apart
  const uint8_t *b;        // B(n, k) at n·b_nb0 + k·b_nb1
  int64_t b_nb0, b_nb1;
  uint8_t *dst;            // dst(n, m) at n·d_nb0 + m·d_nb1
  int64_t d_nb0, d_nb1;
  float *partial;          // [slices][M][16·NT] when slices > 1
  int32_t M, N, K;
  int32_t slices, tiles_per_range, tasks;  // tasks = ranges·slices (the grid is padded to 8)
  // gemm_skinny_pair_kernel's fused split-K reduction (null: splitk_reduce_kernel runs after):
  // one arrival counter per range on its own 128-B line (kChainLine words apart), a counter row
  // per `slices` value so every counter stays a multiple of slices between calls; the word after
  // the row's last counter is the timeout flag
  unsigned *rsync;
  // gemm_skinny_pair_kernel, Q4_0: 8 when A's buffer holds 8 bytes past the last row, so rows 8-15 of a
  // unit may be staged 8 bytes later in their LDS rows (bank-conflict-free weight reads); else 0
  int32_t shift8;
};

// s_waitcnt vmcnt(BASE + j·STEP) for a run-time j in [0, J].
template <int BASE, int STEP, int J> __device__ __forceinline__ void wait_vmcnt_prog(int j) {
  if (j >= J) wait_vmcnt<BASE + J * STEP>();
  else if constexpr (J > 0) wait_vmcnt_prog<BASE, STEP, J - 1>(j);
}

// Q4_0 weight fragment with the offset folded in: (n - 8)·2^-9, exact in bf16, k order
// (0,2,4,6,1,3,5,7) as Q4Frag.
__device__ __forceinline__ bf16x8 q4_0_frag_biased(uint32_t u) {
  const uint32_t lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
  const f2v bias = {-0.015625f, -0.015625f};
  const f2v e0 = fp8x2<false>(lo) + bias, e1 = fp8x2<true>(lo) + bias, o0 = fp8x2<false>(hi) + bias,
            o1 = fp8x2<true>(hi) + bias;
  uint32_t w[4] = {pack_bf16_exact(e0.x, e0.y), pack_bf16_exact(e1.x, e1.y), pack_bf16_exact(o0.x, o0.y),
                   pack_bf16_exact(o1.x, o1.y)};
  return __builtin_bit_cast(bf16x8, w);
}

// The WPB dwords of block B for lane (row m = lane & 15, group g = lane >> 4): bm = slot + m·PITCH,
// bg = bm + (4 or 8)·g. The caller issues every block's reads, then a compiler barrier, so they
// go out as one burst (the compiler would otherwise sink each next to its use).
template <int QT, int B, int WPB>
__device__ __forceinline__ void skinny_read(const uint8_t *bm, const uint8_t *bg, uint32_t (&w)[WPB]) {
  constexpr int OB = B * QTraits<QT>::BB;  // block offset within the row piece
#define LK_DSR(i, base, off) w[i] = *(const uint32_t *)((base) + (off))
  if constexpr (QT == LK_TYPE_Q4_1) {        // (d, m) dword; codes at +4 + 4g
    LK_DSR(0, bm, OB);
    LK_DSR(1, bg, OB + 4);
  } else if constexpr (QT == LK_TYPE_Q4_0) {
    if constexpr ((OB & 3) == 0) {           // d lo; codes at +2 + 4g: two dwords, realigned by 2
      LK_DSR(0, bm, OB);
      LK_DSR(1, bg, OB);
      LK_DSR(2, bg, OB + 4);
    } else {                                 // d in the high half of the dword before; codes aligned
      LK_DSR(0, bm, OB - 2);
      LK_DSR(1, bg, OB + 2);
      w[2] = 0;
    }
  } else {                                   // Q8_0: codes bytes [2 + 8g, 10 + 8g)
    if constexpr ((OB & 3) == 0) {
      LK_DSR(0, bm, OB);
      LK_DSR(1, bg, OB);
      LK_DSR(2, bg, OB + 4);
      LK_DSR(3, bg, OB + 8);
    } else {
      LK_DSR(0, bm, OB - 2);
      LK_DSR(1, bg, OB + 2);
      LK_DSR(2, bg, OB + 6);
      w[3] = 0;
    }
  }
#undef LK_DSR
}

template <int QT, int SB, int WPB, int B>
__device__ __forceinline__ void skinny_read_all(const uint8_t *bm, const uint8_t *bg, uint32_t (&w)[SB][WPB]) {
  if constexpr (B < SB) {
    skinny_read<QT, B, WPB>(bm, bg, w[B]);
    skinny_read_all<QT, SB, WPB, B + 1>(bm, bg, w);
  }
}

// Block B: weight fragment from its dwords, MFMAs against the held activation fragments, scaled
// accumulation.
template <int QT, int NT, int B, int WPB>
__device__ __forceinline__ void skinny_block(const uint32_t (&w)[WPB], const float *tlds, int lane, const u32x4 (&xh)[16][NT],
                                             const u32x4 (&xl)[16][NT], f32x4 (&acc)[NT]) {
  constexpr int OB = B * QTraits<QT>::BB;
  bf16x8 wf;
  float s1, s2 = 0.f;
  if constexpr (QT == LK_TYPE_Q4_1) {
    wf = Q4Frag<0>::make(w[1]);
    s1 = 512.f * h2f(w[0]);
    s2 = h2f(w[0] >> 16);
  } else if constexpr (QT == LK_TYPE_Q4_0) {
    if constexpr ((OB & 3) == 0) {
      wf = q4_0_frag_biased(align2(w[2], w[1]));
      s1 = 512.f * h2f(w[0]);
    } else {
      wf = q4_0_frag_biased(w[1]);
      s1 = 512.f * h2f(w[0] >> 16);
    }
  } else {
    if constexpr ((OB & 3) == 0) {
      wf = w_frag<LK_TYPE_Q8_0>(align2(w[2], w[1]), align2(w[3], w[2]));
      s1 = h2f(w[0]);
    } else {
      wf = w_frag<LK_TYPE_Q8_0>(w[1], w[2]);
      s1 = h2f(w[0] >> 16);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; j++) {
    f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xl[B][j]), wf, f32x4{0.f, 0.f, 0.f, 0.f},
                                                      0, 0, 0);
    p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xh[B][j]), wf, p, 0, 0, 0);
    f32x4 t = {0.f, 0.f, 0.f, 0.f};
    if constexpr (QT == LK_TYPE_Q4_1) t = *(const f32x4 *)(tlds + (B * NT + j) * 16 + (lane >> 4) * 4);
    accumulate<QT == LK_TYPE_Q4_1>(acc[j], s1, s2, p, t);
  }
}

// Blocks B..nb-1 of a unit, unrolled at compile time. FULL: nb == SB (no guards).
template <int QT, int NT, int SB, int WPB, bool FULL, int B>
__device__ __forceinline__ void skinny_blocks(const uint32_t (&w)[SB][WPB], const float *tlds, int nb, int lane,
                                              const u32x4 (&xh)[16][NT], const u32x4 (&xl)[16][NT], f32x4 (&acc)[NT]) {
  if constexpr (B < SB) {
    if (!FULL && B >= nb) return;
    skinny_block<QT, NT, B, WPB>(w[B], tlds, lane, xh, xl, acc);
    skinny_blocks<QT, NT, SB, WPB, FULL, B + 1>(w, tlds, nb, lane, xh, xl, acc);
  }
}


// Split-K fix-up by the last arriver (round 4; the skinny kernels, gemm_sk_kernel, gemm_wide_kernel).
// Nobody waits for anybody: grids larger than the CUs that are free, and launches sharing the GPU
// with other streams, are both safe. Per output tile (16 rows of a skinny kernel, one BM x BN tile of
// the wide kernel) a counter word counts the slices whose partial slab rows are stored:
//  * every slab is stored write-through (sc1) and the storing wave drains vmcnt(0) before it arrives;
//  * one lane per tile adds 1 (agent-scope atomic); the add that returns slices − 1 is the last
//    arrival: that lane re-arms the counter (stores 0: every slice has arrived, so no add is pending)
//    and its workgroup sums the tile's slabs in slice order with sc1 loads — the order of
//    splitk_reduce_kernel, so the result is bit-identical to it — into dst;
//  * the other workgroups leave.
// MI355X_MICROARCH.md (inter-workgroup visibility), hand-off row 1: sc1 stores and loads, the
// signaller after its wave's vmcnt(0), "the workgroup whose add came last, told by the value its add
// returned", its other waves loading after a workgroup barrier the adding wave joins.
// Counters are per launch-tile, each on a 128-B line of its own (kChainLine words apart: returning
// atomics on one line serialize at the memory side, ~12 ns each), and zero between launches
// (lk_sync_counters_sum); one batched launch at a time per device owns them.
__device__ __forceinline__ bool splitk_arrive(unsigned *cnt, unsigned slices) {
  const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prev + 1u != slices) return false;
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// dst(m, n) = Σ_s slab_s(m, n) in slice order for item idx of a 4-column group: row m, columns
// [n0, n0 + 4) (slab rows N16 floats apart, sc1 loads; all of a group's loads in flight at once).
__device__ __forceinline__ void splitk_sum4(const __amdgpu_buffer_rsrc_t prs, int slices, int64_t m, int n0, int M, int N,
                                            int N16, uint8_t *dst, int64_t d_nb0, int64_t d_nb1) {
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < slices; b += 8) {
    f32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (b + i < slices)
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, (int)((((int64_t)(b + i) * M + m) * N16 + n0) * 4), 0, 16));
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (b + i < slices) {
        if (b + i == 0) sum = v[i];  // slab 0 as is (0 + x would turn -0.0 into +0.0)
        else { sum.x += v[i].x; sum.y += v[i].y; sum.z += v[i].z; sum.w += v[i].w; }
      }
  }
  const float e4[4] = {sum.x, sum.y, sum.z, sum.w};
  if (d_nb0 == 4 && n0 + 4 <= N && (((uintptr_t)(dst + m * d_nb1 + n0 * 4)) & 15) == 0) {
    *(f32x4 *)(dst + m * d_nb1 + n0 * 4) = sum;
  } else {
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (n0 + q < N) *(float *)(dst + m * d_nb1 + (n0 + q) * d_nb0) = e4[q];
  }
}

// The skinny kernels' fix-up, called by every wave of the workgroup once its own stores have drained
// (vmcnt(0)). Stream wave `sw` (or −1: a wave that stored nothing) stored the slab rows of its
// `nunits` tiles t0 + sw + step·u. It arrives on all of them at once, as soon as its own loop is done
// (one instruction: a lane per tile, 64 per round) — no workgroup barrier first, so for each tile the
// last arrival is the slowest of the slices' streams for THAT tile, and the summing spreads over the
// range's workgroups instead of landing on the slowest one. Its last arrivals go to its own LDS list
// (`lst`: the count at lst[0], the tiles from lst[1]; an area only this wave uses by now), then after
// one workgroup barrier all NW·64 threads sum the listed tiles of every stream (lists at lst_of(s)),
// 16 rows x N16 columns each (rows past M skipped), with the loads of 4 items per thread in flight.
template <int NW, typename ListOf>
__device__ __forceinline__ void splitk_tiles_fixup(unsigned *tcnt, const __amdgpu_buffer_rsrc_t prs, int slices, int sw,
                                                   int nstreams, int t0, int step, int nunits, ListOf lst_of,
                                                   int M, int N, int N16, uint8_t *dst, int64_t d_nb0, int64_t d_nb1,
                                                   int lane) {
  if (sw >= 0) {
    LK_LDS int *lst = lst_of(sw);
    int n = 0;
    for (int u0 = 0; u0 < nunits; u0 += 64) {
      const int u = u0 + lane;
      const int t = t0 + sw + step * u;
      bool last = false;
      if (u < nunits) last = splitk_arrive(tcnt + (int64_t)t * kChainLine, (unsigned)slices);
      const uint64_t mask = __ballot(last);
      if (last) lst[1 + n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] = t;
      n += __builtin_popcountll(mask);
    }
    if (lane == 0) lst[0] = n;
  }
  asm volatile("" ::: "memory");  // the slab loads stay after the arrivals
#ifdef LK_LAB_STAMPS
  const int wave = threadIdx.x >> 6;
  LK_KP_SET(5, LK_KP_T());
#endif
  __syncthreads();
#ifdef LK_LAB_STAMPS
  LK_KP_SET(6, LK_KP_T());
  if (sw >= 0) LK_KP_SET(7, (uint64_t)lst_of(sw)[0]);
#endif
  const int c4 = N16 / 4, per = 16 * c4;
  int tot = 0;
  for (int s = 0; s < nstreams; s++) tot += lst_of(s)[0] * per;
  // item i: stream list by list, tile by tile, row by row, 4 columns
  auto item = [&](int i, int64_t &m, int &n0) __attribute__((always_inline)) {
    int s = 0, k = i;
    while (k >= lst_of(s)[0] * per) { k -= lst_of(s)[0] * per; s++; }
    const int t = lst_of(s)[1 + k / per];
    m = (int64_t)t * 16 + (k % per) / c4;
    n0 = (k % c4) * 4;
  };
  constexpr int IB = 4;  // items per thread with their loads in flight together
  for (int i0 = (int)threadIdx.x * IB; i0 < tot; i0 += NW * 64 * IB) {
    int64_t m[IB];
    int n0[IB];
    bool ok[IB];
#pragma unroll
    for (int q = 0; q < IB; q++) {
      ok[q] = i0 + q < tot;
      m[q] = 0; n0[q] = 0;
      if (ok[q]) item(i0 + q, m[q], n0[q]);
      ok[q] = ok[q] && m[q] < M;
    }
    f32x4 sum[IB];
    for (int b = 0; b < slices; b += 8) {
      f32x4 v[IB][8];
#pragma unroll
      for (int q = 0; q < IB; q++)
#pragma unroll
        for (int i = 0; i < 8; i++)
          if (ok[q] && b + i < slices)
            v[q][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, (int)((((int64_t)(b + i) * M + m[q]) * N16 + n0[q]) * 4), 0, 16));
#pragma unroll
      for (int q = 0; q < IB; q++)
#pragma unroll
        for (int i = 0; i < 8; i++)
          if (ok[q] && b + i < slices) {
            if (b + i == 0) sum[q] = v[q][i];  // slab 0 as is (0 + x would turn -0.0 into +0.0)
            else { sum[q].x += v[q][i].x; sum[q].y += v[q][i].y; sum[q].z += v[q][i].z; sum[q].w += v[q][i].w; }
          }
    }
#pragma unroll
    for (int q = 0; q < IB; q++) {
      if (!ok[q]) continue;
      const float e4[4] = {sum[q].x, sum[q].y, sum[q].z, sum[q].w};
      uint8_t *o = dst + m[q] * d_nb1 + n0[q] * d_nb0;
      if (d_nb0 == 4 && n0[q] + 4 <= N && (((uintptr_t)o) & 15) == 0) {
        *(f32x4 *)o = sum[q];
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++)
          if (n0[q] + e < N) *(float *)(dst + m[q] * d_nb1 + (n0[q] + e) * d_nb0) = e4[e];
      }
    }
  }
}

// a partial slab's f32x4, written through (sc1) whenever the slab fits a buffer resource: another
// workgroup of the launch (the last arriver) or the reduce launch after it reads it, and a plain
// store would leave the line dirty in this XCD's L2 — written back at the kernel boundary, which
// costs that boundary ~1 µs per 6 MB (MI355X_MICROARCH.md, boundary; C3's slabs are 11 MB)
#ifndef LK_SLAB_PLAIN
#define LK_SLAB_PLAIN 0  // lab builds only: plain slab stores when the reduction is a separate launch
#endif
__device__ __forceinline__ bool slab_wt(bool fused, int64_t slab_bytes) {
  return fused || (!LK_SLAB_PLAIN && slab_bytes < (1ll << 31));
}
__device__ __forceinline__ void store_partial(bool wt, const __amdgpu_buffer_rsrc_t prs, float *partial, int64_t idx,
                                              f32x4 v) {
  if (wt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), prs, (int)(idx * 4), 0, 16);
  else *(f32x4 *)(partial + idx) = v;
}


template <int QT, int NT>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(SkinnyArgs g) {
  using G = SkinnyGeom<QT, NT>;
  constexpr int BB = G::BB, SB = G::SB, D = G::D, L = G::L, NW = G::NW;
  static_assert(SB == 16, "held activation arrays are [16][NT]");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t *xlds = smem;
  float *tlds = (float *)(smem + G::XB);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t *ring = smem + G::XB + G::TB + wave * D * G::SLOT;
  // XCD-aware task order (speed only: dispatch is observed round-robin over the 8 XCDs):
  // workgroup b runs task (b % 8)·(grid / 8) + b / 8, so the slices of one row range — which
  // share the 128-B lines at their boundaries — and a range's neighbours land on one L2.
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding (before any barrier: the whole workgroup leaves)
  const int slice = task % g.slices, range = task / g.slices;
  const int nblk = g.K / 32;
  const int kb0 = slice * SB, nb = min(SB, nblk - kb0);
  const int64_t RB = (int64_t)nblk * BB;
  const int ntile = (g.M + 15) / 16;
  const int t0 = range * g.tiles_per_range, t1 = min(t0 + g.tiles_per_range, ntile);
  // this wave's tiles: t0 + wave + i·NW
  const int nunits = t1 - t0 - wave > 0 ? (t1 - t0 - wave + NW - 1) / NW : 0;
  const int ppr = nb * BB / 16;  // 16-B pieces per row in this slice (the last slice may be short)

  // unit u = the wave's u-th tile's slice: lane q of the unit's DMA lands at cell q = r·(PPR+1) + c
  // (row r, piece c); pad cells and pieces past a short slice re-read the row's first piece
  const uint8_t *abase = g.a + (int64_t)kb0 * BB;
  uint32_t rofs[L];  // per-lane byte offset of its piece from the tile's first row (the tile's
  int rrow[L];       // rows past M read row M-1 instead)
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int q = j * 64 + lane, r = q / (G::PPR + 1), c = q % (G::PPR + 1);
    rrow[j] = min(r, 15);
    rofs[j] = (uint32_t)((c < ppr && r < 16) ? c * 16 : 0);
  }
  auto issue = [&](int u, int sl) __attribute__((always_inline)) {
    const int t = t0 + wave + u * NW;
    const uint8_t *tb = abase + (int64_t)t * 16 * RB;
    const int rmax = g.M - 1 - t * 16;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const uint32_t vofs = (uint32_t)(min(rrow[j], rmax) * RB) + rofs[j];
      dma16<1>(tb, vofs, ring + sl * G::SLOT + j * 1024);  // nt: read once per launch
    }
  };
  // 1. the HBM stream starts with one unit per wave
  if (nunits > 0) issue(0, 0);

  // 2. activations of the slice -> LDS fragments (x-tile j, block b, split s): lane l holds
  // x(n = 16j + (l & 15), k = 32(kb0 + b) + 8(l >> 4) + order[0..7]) as bf16 hi / lo. Fragment
  // f = b·NT + j is converted by wave f % NW; all its loads are issued before any is used.
  float v[G::FPW][8];
#pragma unroll
  for (int i = 0; i < G::FPW; i++) {
    const int f = wave + i * NW, b = f / NT, j = f % NT;
    const int n = 16 * j + (lane & 15);
    const int64_t k0 = 32 * (int64_t)(kb0 + b) + 8 * (lane >> 4);
    const bool ok = b < nb && n < g.N;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int kk = (QT != LK_TYPE_Q8_0) ? ((e & 3) * 2 + (e >> 2)) : e;
      v[i][e] = ok ? *(const float *)(g.b + n * g.b_nb0 + (k0 + kk) * g.b_nb1) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < G::FPW; i++) {
    const int f = wave + i * NW;
    float part = 0.f;
#pragma unroll
    for (int e = 0; e < 8; e++) part += v[i][e];
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      uint32_t h[2], l[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t bx = __builtin_bit_cast(uint32_t, v[i][e + q]);
        const float r = v[i][e + q] - __builtin_bit_cast(float, bx & 0xFFFF0000u);  // exact
        uint32_t br = __builtin_bit_cast(uint32_t, r);
        br += 0x7FFFu + ((br >> 16) & 1u);  // round to nearest even
        h[q] = bx;
        l[q] = br;
      }
      hi[e / 2] = __builtin_amdgcn_perm(h[1], h[0], 0x07060302u);
      lo[e / 2] = __builtin_amdgcn_perm(l[1], l[0], 0x07060302u);
    }
    u32x4 *xf = (u32x4 *)(xlds + (f * kXSplits) * 1024) + lane;
    xf[0] = u32x4{hi[0], hi[1], hi[2], hi[3]};
    xf[64] = u32x4{lo[0], lo[1], lo[2], lo[3]};
    if constexpr (QT == LK_TYPE_Q4_1) {
      part += __shfl_xor(part, 16, kWave);
      part += __shfl_xor(part, 32, kWave);
      if (lane < 16) tlds[f * 16 + lane] = part;
    }
  }
  // 3. the rest of the ring
  for (int u = 1; u < min(D, nunits); u++) issue(u, u);
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();
  // 4. every wave holds all of the slice's activation fragments
  u32x4 xh[16][NT], xl[16][NT];
#pragma unroll
  for (int b = 0; b < SB; b++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const u32x4 *xf = (const u32x4 *)(xlds + ((b * NT + j) * kXSplits) * 1024) + lane;
      xh[b][j] = xf[0];
      xl[b][j] = xf[64];
    }

  const int N16 = 16 * NT;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4) ? g.slices * g.M * N16 * 4 : 0, 0x00020000);
  int slot = 0;
  for (int u = 0; u < nunits; u++) {
    // ops younger than unit u's DMA (issue order: units 0..D-1 in the prologue, then per tile
    // i: unit i+D, the stores of tile i): units u+1..u+D-1 (L each) and the stores of the
    // min(u, D) previous tiles (>= NT each); short of that steady state (the last units) drain
    if (u + D - 1 < nunits) wait_vmcnt_prog<(D - 1) * L, NT, D>(u);
    else wait_vmcnt<0>();
    asm volatile("" ::: "memory");  // the slot's LDS reads stay behind the wait
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t wd[SB][G::WPB];
    {
      const uint8_t *bm = ring + slot * G::SLOT + (lane & 15) * G::PITCH;
      const uint8_t *bg = bm + (QT == LK_TYPE_Q8_0 ? 8 : 4) * (lane >> 4);
      skinny_read_all<QT, SB, G::WPB, 0>(bm, bg, wd);
      asm volatile("" ::: "memory");  // keep the burst together: no read sinks below this line
    }
    if (nb == SB) skinny_blocks<QT, NT, SB, G::WPB, true, 0>(wd, tlds, nb, lane, xh, xl, acc);
    else skinny_blocks<QT, NT, SB, G::WPB, false, 0>(wd, tlds, nb, lane, xh, xl, acc);
    wait_lgkmcnt0();  // this slot's LDS reads have landed: the DMA may overwrite it
    if (u + D < nunits) issue(u + D, slot);
    slot = (slot + 1 == D) ? 0 : slot + 1;
    // outputs: lane holds C'(n = 16j + 4(lane>>4) + e, m = 16t + (lane&15))
    const int t = t0 + wave + u * NW;
    const int64_t m = (int64_t)t * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const int n0 = 16 * j + 4 * (lane >> 4);
      if (g.slices > 1) {
        if (m < g.M) store_partial(slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4), prs, g.partial, ((int64_t)slice * g.M + m) * N16 + n0, acc[j]);
      } else if (m < g.M) {
        const float e4[4] = {acc[j].x, acc[j].y, acc[j].z, acc[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (n0 + q < g.N) *(float *)(g.dst + m * g.d_nb1 + (n0 + q) * g.d_nb0) = e4[q];
      }
    }
  }
  wait_vmcnt<0>();
  if (g.rsync) {  // the last slice to store a tile sums it; wave w lists in its own ring, drained by now
    auto lst_of = [&](int w) __attribute__((always_inline)) {
      return (LK_LDS int *)(LK_LDS void *)(smem + G::XB + G::TB + w * D * G::SLOT);
    };
    splitk_tiles_fixup<NW>(g.rsync, prs, g.slices, wave, NW, t0, NW, nunits, lst_of, g.M, g.N, N16, g.dst, g.d_nb0,
                           g.d_nb1, lane);
  }
}

// ---- skinny GEMM on wave pairs (Q4_0 / Q4_1, 17 <= N <= 32) -------------------------------
//
// gemm_skinny_kernel runs one wave per SIMD (all of the slice's x-fragments, 256 VGPRs at
// N 32): a lone wave issues VALU every 4 cycles and nothing overlaps its MFMAs. Here the
// slice's 16 blocks are split over a wave pair on one SIMD: wave (stream p = w % 4, half
// h = w / 4) holds x for blocks [8h, 8h + 8) (128 VGPRs), streams its half of each row piece
// through its own LDS-DMA ring and computes that half's partial dot. The h = 1 wave hands its
// accumulators to its partner through LDS (two parities), behind a ready flag; the partner adds
// them in a fixed order (deterministic) and stores, then acknowledges. No workgroup barrier
// after the prologue: each pair runs at its own pace.
template <int QT, int NT> struct SkinnyPairGeom {
  static constexpr int NW = 8;                          // 4 streams x 2 halves
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr int SB = 16, SBH = 8;                // blocks per slice / per half
  static constexpr int RPH = SBH * BB;                  // bytes of a half row piece (multiple of 16)
  static constexpr int PPH = RPH / 16;                  // 16-B cells per half row
  // cells per LDS row: odd, so rows m and m + 8 of a unit do not start on the same 4-bank group (Q4_1's
  // 10 cells put them on the same banks: 2-way conflicts on every weight read). A 16-B cell pitch still
  // maps rows m and m + 8 to one bank group of a 32-lane half (4·CPR·8 ≡ 0 mod 32), so Q4_0 (round 6)
  // stages rows 8-15 8 bytes later (their DMA starts 8 bytes early, one more cell): the two rows' reads
  // land on dwords {0, 1} and {2, 3} of a group — conflict-free — at the same 3 DMA instructions
  static constexpr int XC = QT == LK_TYPE_Q4_0 ? 1 : 0;
  static constexpr int CPR = (PPH + XC) | 1;
  static constexpr int PITCH = CPR * 16;                // LDS row pitch
  static constexpr int L = (16 * CPR + 63) / 64;        // DMA instructions per half unit
  static constexpr int WPB = QT == LK_TYPE_Q4_1 ? 2 : QT == LK_TYPE_Q4_0 ? 3 : 4;
  static constexpr int SLOT = L * 1024;
  static constexpr int XB = SB * NT * kXSplits * 1024;  // activation fragments (staging)
  static constexpr int TB = QT == LK_TYPE_Q8_0 ? 0 : SB * NT * 16 * 4;  // Q4_1 Σx / Q4_0 −136·Σ(hi+lo) per (block, column)
  static constexpr int EB = 2 * 4 * NT * 64 * 16;       // accumulator hand-off, 2 parities x 4 pairs
  static constexpr int FB = 64;                         // ready[4][2], ack[4] (ints)
  static constexpr int DFIT = (kLdsBytes - XB - TB - EB - FB) / (NW * SLOT);
  static constexpr int D = DFIT > 3 ? 3 : DFIT;         // ring depth (half units per wave)
  static constexpr int LDS = XB + TB + EB + FB + NW * D * SLOT;
  static constexpr int FPW = SB * NT / NW;              // fragments each wave converts
  static constexpr int MAXW = L * (D - 1) + D * NT;     // largest vmcnt a wait needs
  static_assert(RPH % 16 == 0, "half row pieces");
  static_assert(D >= 2, "ring must double-buffer");
  static_assert(LDS <= kLdsBytes, "LDS");
  static_assert((SB * NT) % NW == 0, "fragments per wave");
  static_assert(MAXW < 64, "vmcnt");
};

// s_waitcnt vmcnt(x) for a wave-uniform run-time x in [0, J] (x > J waits for J).
template <int J> __device__ __forceinline__ void wait_vmcnt_rt(int x) {
  if constexpr (J == 0) wait_vmcnt<0>();
  else if (x >= J) wait_vmcnt<J>();
  else wait_vmcnt_rt<J - 1>(x);
}

// Block B (0..7) of this wave's half: x held as [8][NT]; T (Q4_0 / Q4_1) indexed by the slice block.
template <int QT, int NT, int B, int WPB>
__device__ __forceinline__ void skinny_pair_block(const uint32_t (&w)[WPB], const float *tl, int lane, const u32x4 (&xh)[8][NT],
                                                  const u32x4 (&xl)[8][NT], f32x4 (&acc)[NT]) {
  constexpr int OB = B * QTraits<QT>::BB;
  bf16x8 wf;
  float s1, s2 = 0.f;
  if constexpr (QT == LK_TYPE_Q4_1) {
    wf = Q4Frag<0>::make(w[1]);
    s1 = 512.f * h2f(w[0]);
    s2 = h2f(w[0] >> 16);
  } else if constexpr (QT == LK_TYPE_Q4_0) {  // codes 128 + n; −136·Σx enters as the MFMA's C (T)
    if constexpr ((OB & 3) == 0) {
      wf = q4_codes_128(align2(w[2], w[1]));
      s1 = h2f(w[0]);
    } else {
      wf = q4_codes_128(w[1]);
      s1 = h2f(w[0] >> 16);
    }
  } else {
    if constexpr ((OB & 3) == 0) {
      wf = w_frag<LK_TYPE_Q8_0>(align2(w[2], w[1]), align2(w[3], w[2]));
      s1 = h2f(w[0]);
    } else {
      wf = w_frag<LK_TYPE_Q8_0>(w[1], w[2]);
      s1 = h2f(w[0] >> 16);
    }
  }
  (void)s2;
#pragma unroll
  for (int j = 0; j < NT; j++) {
    // the offset term (Q4_0 −136·Σx, Q4_1 m·Σx) is added once per unit (skinny_pair_offsets)
    f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xl[B][j]), wf,
                                                      f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xh[B][j]), wf, p, 0, 0, 0);
    accumulate_s<false>(acc[j], s1, 0.f, p, p);
  }
}

template <int QT, int NT, int WPB, bool FULL, int B>
__device__ __forceinline__ void skinny_pair_blocks(const uint32_t (&w)[8][WPB], const float *tl, int nb, int lane,
                                                   const u32x4 (&xh)[8][NT], const u32x4 (&xl)[8][NT], f32x4 (&acc)[NT]) {
  if constexpr (B < 8) {
    if (!FULL && B >= nb) return;
    skinny_pair_block<QT, NT, B, WPB>(w[B], tl, lane, xh, xl, acc);
    skinny_pair_blocks<QT, NT, WPB, FULL, B + 1>(w, tl, nb, lane, xh, xl, acc);
  }
}

// LDS flags between the two waves of a pair. LDS serves one wave's requests in order, so a
// flag written after the data is seen after it; the compiler barriers keep the source order
// (a workgroup-scope atomic would also order the wave's in-flight DMA, which is not needed).
__device__ __forceinline__ int lds_ld(const int *p) {
  asm volatile("" ::: "memory");
  const int v = *(volatile const LK_LDS int *)(LK_LDS const int *)p;
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void lds_st(int *p, int v) {
  asm volatile("" ::: "memory");
  *(volatile LK_LDS int *)(LK_LDS int *)p = v;
  asm volatile("" ::: "memory");
}

template <int QT, int NT>
__device__ __forceinline__ void skinny_pair_body(const SkinnyArgs &g, int task) {
  using G = SkinnyPairGeom<QT, NT>;
  constexpr int BB = G::BB, D = G::D, L = G::L, NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t *xlds = smem;
  float *tlds = (float *)(smem + G::XB);
  f32x4 *xch = (f32x4 *)(smem + G::XB + G::TB);
  int *flags = (int *)(smem + G::XB + G::TB + G::EB);  // ready[p][parity] at 2p + parity, ack[p] at 8 + p
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = wave & 3, h = wave >> 2;
  uint8_t *ring = smem + G::XB + G::TB + G::EB + G::FB + wave * D * G::SLOT;
  [[maybe_unused]] const uint64_t t_entry = LK_KP_T();
  if (threadIdx.x < 16) flags[threadIdx.x] = 0;  // published by the prologue's barrier
  const int slice = task % g.slices, range = task / g.slices;
  const int nblk = g.K / 32;
  const int kb0 = slice * G::SB, nb = min(G::SB, nblk - kb0);
  const int nbh = max(0, min(G::SBH, nb - G::SBH * h));  // this wave's blocks (a short slice may leave h = 1 none)
  const int64_t RB = (int64_t)nblk * BB;
  const int ntile = (g.M + 15) / 16;
  const int t0 = range * g.tiles_per_range, t1 = min(t0 + g.tiles_per_range, ntile);
  const int nunits = t1 - t0 - p > 0 ? (t1 - t0 - p + 3) / 4 : 0;  // stream p: tiles t0 + p + 4i
  const int pph = nbh * BB / 16;
  const int myL = nbh > 0 ? L : 0;
  // Q4_0: rows 8-15 of a unit 8 bytes later in their LDS rows (SkinnyPairGeom::XC); reads follow
  const int sh8 = QT == LK_TYPE_Q4_0 ? g.shift8 : 0;
  const int rsh = (lane & 15) >= 8 ? sh8 : 0;

  // half unit u = rows of tile t0 + p + 4u, bytes [kb0·BB + h·RPH, + nbh·BB) of each; cell
  // q = r·CPR + c lands at slot + 16q (row pitch PITCH); pad cells and cells past the unit re-read cell 0
  const uint8_t *abase = g.a + (int64_t)kb0 * BB + (int64_t)h * G::RPH;
  uint32_t rofs[L], dsh[L];
  int rrow[L];
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int q = j * 64 + lane, r = q / G::CPR, c = q % G::CPR;
    const int shifted = r >= 8 && r < 16 && sh8;
    rrow[j] = min(r, 15);
    rofs[j] = (uint32_t)((c < pph + shifted && r < 16) ? c * 16 : 0);
    dsh[j] = shifted ? 8u : 0u;
  }
  auto issue = [&](int u, int sl) __attribute__((always_inline)) {
    const int t = t0 + p + u * 4;
    const uint8_t *tb = abase + (int64_t)t * 16 * RB;
    const int rmax = g.M - 1 - t * 16;
#pragma unroll
    for (int j = 0; j < L; j++) {
      // a shifted row starts 8 bytes early; a row clamped onto the matrix's first piece (its outputs
      // are never stored) reads unshifted rather than before the tile's base
      const uint32_t at = (uint32_t)(min(rrow[j], rmax) * RB) + rofs[j];
      const uint32_t vofs = at >= dsh[j] ? at - dsh[j] : at;
      dma16<1>(tb, vofs, ring + sl * G::SLOT + j * 1024);  // nt: read once per launch
    }
  };

  // (the weight ring issued before the activation loads measured slower on C3, 24.0 vs 23.1 us
  // per call: the activation loads queue behind the burst)
  // 1. activations of the slice -> LDS fragments, as gemm_skinny_kernel (compiler-visible loads:
  //    issued before the weight ring, so waiting for them never waits for it)
  float v[G::FPW][8];
#pragma unroll
  for (int i = 0; i < G::FPW; i++) {
    const int f = wave + i * NW, b = f / NT, j = f % NT;
    const int n = 16 * j + (lane & 15);
    const int64_t k0 = 32 * (int64_t)(kb0 + b) + 8 * (lane >> 4);
    const bool ok = b < nb && n < g.N;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      // k order within 8: Q4_0 (0,4,1,5,2,6,3,7) for q4_codes_128, Q4_1 (0,2,4,6,1,3,5,7) for Q4Frag
      const int kk = QT == LK_TYPE_Q4_0 ? ((e >> 1) + 4 * (e & 1)) : QT == LK_TYPE_Q4_1 ? ((e & 3) * 2 + (e >> 2)) : e;
      v[i][e] = ok ? *(const float *)(g.b + n * g.b_nb0 + (k0 + kk) * g.b_nb1) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < G::FPW; i++) {
    const int f = wave + i * NW;
    float part = 0.f, hsum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; e++) part += v[i][e];
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      // hi = x truncated to bf16, lo = x − hi (exact in f32) rounded to nearest even by one
      // v_cvt_pk_bf16_f32 for the pair (round 5: the same bits as the former per-element integer
      // rounding, about half the VALU of the split)
      const uint32_t b0 = __builtin_bit_cast(uint32_t, v[i][e]), b1 = __builtin_bit_cast(uint32_t, v[i][e + 1]);
      const float h0 = __builtin_bit_cast(float, b0 & 0xFFFF0000u), h1 = __builtin_bit_cast(float, b1 & 0xFFFF0000u);
      const f2v r = {v[i][e] - h0, v[i][e + 1] - h1};  // exact
      const uint32_t lp = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
      hi[e / 2] = __builtin_amdgcn_perm(b1, b0, 0x07060302u);
      lo[e / 2] = lp;
      // Q4_0's −136·Σx cancels against Σ (128 + n)·(hi + lo): sum the split itself, so the
      // split's own error is not amplified
      hsum += h0 + __builtin_bit_cast(float, lp << 16);
      hsum += h1 + __builtin_bit_cast(float, lp & 0xFFFF0000u);
    }
    u32x4 *xf = (u32x4 *)(xlds + (f * kXSplits) * 1024) + lane;
    xf[0] = u32x4{hi[0], hi[1], hi[2], hi[3]};
    xf[64] = u32x4{lo[0], lo[1], lo[2], lo[3]};
    if constexpr (QT != LK_TYPE_Q8_0) {
      if constexpr (QT == LK_TYPE_Q4_0) part = hsum;
      part += __shfl_xor(part, 16, kWave);
      part += __shfl_xor(part, 32, kWave);
      if (lane < 16) tlds[f * 16 + lane] = QT == LK_TYPE_Q4_0 ? -136.f * part : part;
    }
  }
  [[maybe_unused]] const uint64_t t_split = LK_KP_T();  // (lab stamps) activations in, split, in LDS
  // 2. the weight ring, after the split
  if (myL)
    for (int u = 0; u < min(D, nunits); u++) issue(u, u);
  wait_lgkmcnt0();
  [[maybe_unused]] const uint64_t t_issued = LK_KP_T();
  __builtin_amdgcn_s_barrier();  // fragments and flags visible (bare: the ring stays in flight)
  [[maybe_unused]] const uint64_t t_bar = LK_KP_T();
  // 3. this wave holds the fragments of its 8 blocks
  u32x4 xh[8][NT], xl[8][NT];
#pragma unroll
  for (int b = 0; b < 8; b++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const int bb = min(8 * h + b, G::SB - 1);
      const u32x4 *xf = (const u32x4 *)(xlds + ((bb * NT + j) * kXSplits) * 1024) + lane;
      xh[b][j] = xf[0];
      xl[b][j] = xf[64];
    }
  const float *tl = tlds + 8 * h * NT * 16;
  // offset operands of v_mfma_f32_16x16x4_f32: lane (n = lane & 15, b' = lane >> 4) holds T of
  // block 4c + b' of this wave's half and column 16j + n (zero past the wave's blocks)
  float tf[2][NT];
#pragma unroll
  for (int c = 0; c < 2; c++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const int bl = 4 * c + (lane >> 4);
      tf[c][j] = (QT != LK_TYPE_Q8_0 && bl < nbh) ? tl[(bl * NT + j) * 16 + (lane & 15)] : 0.f;
    }

  const int N16 = 16 * NT;
  // the partial slabs as a buffer (fused reduction: sc1 stores and loads; the host checks the size)
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4) ? g.slices * g.M * N16 * 4 : 0, 0x00020000);
  const int SH = h == 0 ? NT : 0;  // stores per unit (at least; slices == 1 may store more)
  [[maybe_unused]] const uint64_t t_loop = LK_KP_T();
  for (int u = 0; u < nunits; u++) {
    // the pair's two waves take turns at issue priority, one unit each, h = 1 (the younger) first
    // (A/B, three rounds: C3 Q4_0 21.2 -> 20.7 us, Q4_1 21.1 -> 20.7 us)
    if ((u + h) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    const int slot = u % D;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (myL) {
      // ops younger than this unit's DMA: its successors already issued, and the stores since
      wait_vmcnt_rt<G::MAXW>(myL * min(D - 1, nunits - 1 - u) + min(u, D) * SH);
      asm volatile("" ::: "memory");
#ifdef LK_LAB_STAMPS
      if (u == 0) LK_KP_SET(9, LK_KP_T());  // the first unit has landed
#endif
      uint32_t wd[8][G::WPB];
      const uint8_t *slot_ptr = ring + slot * G::SLOT;
      {
        const uint8_t *bm = ring + slot * G::SLOT + (lane & 15) * G::PITCH + rsh;
        const uint8_t *bg = bm + (QT == LK_TYPE_Q8_0 ? 8 : 4) * (lane >> 4);
        skinny_read_all<QT, 8, G::WPB, 0>(bm, bg, wd);
        asm volatile("" ::: "memory");
      }
      if (nbh == 8) skinny_pair_blocks<QT, NT, G::WPB, true, 0>(wd, tl, nbh, lane, xh, xl, acc);
      else skinny_pair_blocks<QT, NT, G::WPB, false, 0>(wd, tl, nbh, lane, xh, xl, acc);
      if constexpr (QT != LK_TYPE_Q8_0) {
        // acc += Σ_b e_b(row)·T_b(column) over the half's 8 blocks, two f32 MFMAs (K = 4 blocks)
        // per 16-column tile: e = d (Q4_0, T = −136·Σ(hi + lo)) or m (Q4_1, T = Σx); lane
        // (m = lane & 15, b' = lane >> 4) reads its row's header of block 4c + b'
        const uint8_t *hrow = slot_ptr + (lane & 15) * G::PITCH + rsh;
#pragma unroll
        for (int c = 0; c < 2; c++) {
          const int bl = 4 * c + (lane >> 4);
          const uint16_t hv = *(const uint16_t *)(hrow + min(bl, 7) * BB + (QT == LK_TYPE_Q4_1 ? 2 : 0));
          const float e = bl < nbh ? h2f(hv) : 0.f;
#pragma unroll
          for (int j = 0; j < NT; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(tf[c][j], e, acc[j], 0, 0, 0);
        }
      }
      wait_lgkmcnt0();  // this slot's LDS reads have landed: the DMA may overwrite it
      if (u + D < nunits) issue(u + D, slot);
    }
    f32x4 *xb = xch + ((u & 1) * 4 + p) * NT * 64 + lane;
    if (h == 1) {
      // the partner has consumed unit u − 2 (this parity's previous contents)
      while (lds_ld(flags + 8 + p) < u - 1) __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < NT; j++) xb[j * 64] = acc[j];
      lds_st(flags + 2 * p + (u & 1), u + 1);
    } else {
      while (lds_ld(flags + 2 * p + (u & 1)) != u + 1) __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < NT; j++) acc[j] += xb[j * 64];
      lds_st(flags + 8 + p, u + 1);
      // outputs: lane holds C'(n = 16j + 4(lane>>4) + e, m = 16t + (lane&15))
      const int t = t0 + p + u * 4;
      const int64_t m = (int64_t)t * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const int n0 = 16 * j + 4 * (lane >> 4);
        if (g.slices > 1) {
          if (m < g.M) store_partial(slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4), prs, g.partial, ((int64_t)slice * g.M + m) * N16 + n0, acc[j]);
        } else if (m < g.M) {
          const float e4[4] = {acc[j].x, acc[j].y, acc[j].z, acc[j].w};
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (n0 + q < g.N) *(float *)(g.dst + m * g.d_nb1 + (n0 + q) * g.d_nb0) = e4[q];
        }
      }
    }
  }
  wait_vmcnt<0>();
  [[maybe_unused]] const uint64_t t_end = LK_KP_T();
  if (g.rsync) {  // the last slice to store a tile sums it; stream p lists in its pair's hand-off area
    // (parity 0 of pair p: both of the pair's waves are past their last hand-off by now)
    auto lst_of = [&](int s) __attribute__((always_inline)) {
      return (LK_LDS int *)(LK_LDS void *)(smem + G::XB + G::TB + s * NT * 64 * 16);
    };
    splitk_tiles_fixup<NW>(g.rsync, prs, g.slices, h == 0 ? p : -1, 4, t0, 4, nunits, lst_of, g.M, g.N, N16, g.dst,
                           g.d_nb0, g.d_nb1, lane);
  }
  LK_KP_SET(0, t_entry); LK_KP_SET(2, t_loop); LK_KP_SET(3, t_end); LK_KP_SET(4, LK_KP_T());
  LK_KP_SET(8, (uint64_t)nunits); LK_KP_SET(1, t_split); LK_KP_SET(5, t_issued); LK_KP_SET(6, t_bar);
}

template <int QT, int NT>
__global__ __launch_bounds__(512) void gemm_skinny_pair_kernel(SkinnyArgs g) {
  // XCD-aware task order, as gemm_skinny_kernel (a single node: the grouped kernel's interleaved order
  // measured the same on C3, 20.2-20.9 vs 20.2-21.0 us, A/B three rounds)
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding (before any barrier: the whole workgroup leaves)
  skinny_pair_body<QT, NT>(g, task);
}

// Several independent nodes of one plan in ONE launch (round 6, lk_plan_launch's grouped singles): node
// k's tasks follow node k − 1's in the grid, each with the SkinnyArgs the single-node launch would use
// (same ranges, slices, slabs: the same bits). The per-node launch gaps and tails of a plan's 2 <= N <= 32
// nodes overlap instead of adding up.
template <int QT, int NT>
__global__ __launch_bounds__(512) void gemm_skinny_pair_group_kernel(const SkinnyArgs *__restrict__ nodes, int nnodes) {
  // task = workgroup index (no XCD-contiguous runs): dispatch deals consecutive workgroups to the 8 XCDs
  // in turn, so every node's tasks spread over all XCDs and the dispatcher balances nodes of different
  // per-task cost (XCD-contiguous runs gave some XCDs only the heavy nodes: the layer set 4 % slower than
  // separate launches); a node's slice s (= task % 8 at 8 slices) then stays on one XCD, whose L2 serves
  // its activation slice to all of that XCD's ranges
  int task = (int)blockIdx.x;
  for (int k = 0; k < nnodes; k++) {
    const int tk = nodes[k].tasks;
    if (task < tk) {
      skinny_pair_body<QT, NT>(nodes[k], task);
      return;
    }
    task -= tk;
  }
}

// splitk_reduce_kernel over a plan's grouped nodes: node k's threads follow node k − 1's.
struct ReduceNode {
  const float *partial;
  uint8_t *dst;
  int64_t d_nb0, d_nb1;
  int32_t slices, M, N, N16;
  int64_t threads;  // M·N16/4
};

// ---- wide batched GEMM (N > 32, e.g. C5's prefill N = 512): 256-row tiles, 8 waves ----------
//
// MFMA-bound once N is large, but the activation operand costs 4 B per element (bf16 hi + lo),
// seven times a Q4_0 weight: a workgroup tile of BM = 256 rows x BN = 64 columns balances the
// two streams (per CU ~0.8 MB at N 512, K split in two). Eight waves, two per SIMD: four along M
// x two K-groups (blocks 0-1 / 2-3 of each stage; the groups' sums meet in LDS at the end). A
// wave owns 64 rows x 64 columns (4 x 4 tiles of v_mfma_f32_16x16x32_bf16): one decoded weight
// fragment feeds four x-tiles and one activation fragment four row tiles, which keeps both the
// decode VALU and the LDS reads per MFMA low (all eight waves read the same activations).
// K runs in stages of 4 blocks through an LDS ring of D stages:
//   weights: 256 rows x an 80-byte window (the stage's 72 bytes of blocks, rounded up to 16-B
//            DMA pieces, rows 8-byte aligned), row-major at an 80-B pitch;
//   activations: the xsplit_kernel fragments of the 4 blocks x 4 x-tiles x (hi, lo), 1 KB each;
//   Q4_1 only: the 4 blocks' column sums (m·Σx term).
// Every wave issues the same DMA count per stage (CW), so a counted vmcnt plus one barrier
// publishes a stage. Q4_0 codes carry their -8 offset ((n - 8)·2^-9, exact), so no T input.
// Split K: each slice stores an f32 partial slab; splitk_reduce_kernel sums them in order.
// LK_WIDE_SCHED bit 1 (the product since round 5): the scale FMAs interleaved with the MFMAs by
// sched_group_barrier (C5 57.8-58.6 -> 56.6-57.4 us per call, A/B three rounds on one box); bit 0
// (lab): scalar instead of packed scale FMAs (58.6-59.4 -> 60.0-61.0 us: slower)
#ifndef LK_WIDE_SCHED
#define LK_WIDE_SCHED 2
#endif
template <int QT> struct WideGeom {
  static constexpr int NW = 8, KG = 2, MW = NW / KG;             // waves: MW along M x KG K-groups
  static constexpr int MT = 4, NT = 4;                           // wave tile: 64 rows x 64 columns
  static constexpr int BM = MW * MT * 16, BN = NT * 16;
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr int SB = 4;                                  // blocks per stage
  static constexpr int WIN = (SB * BB + 15) / 16 * 16;          // weight window bytes per row
  static constexpr int WPIECES = BM * WIN / 16;                 // 16-B DMA pieces of weights
  static constexpr int W_INST = (WPIECES + 63) / 64;
  static constexpr int X_INST = SB * NT * kXSplits;             // 1-KB activation fragments
  static constexpr int T_INST = (QT == LK_TYPE_Q8_0) ? 0 : 1;  // Σx per (block, column): Q4_1 m·Σx, Q4_0 −136·Σx
  // Weight pieces per wave: the first WX waves issue CWW, the rest CWW − 1. Every wave issues the
  // same count per stage (a counted vmcnt + one barrier publish a stage), so the spare slot of the
  // short waves carries T (1 KB = T_PARTS parts of TL lanes, no duplicates) — or, without T
  // (Q8_0) or when no part shape fits, a padding piece into DUMMY.
  static constexpr int CWW = (W_INST + NW - 1) / NW, CWX = (X_INST + NW - 1) / NW;
  static constexpr int WX = W_INST % NW;
  static constexpr int T_PARTS = WX ? NW - WX : 0;
  static constexpr bool T_SPARE = T_INST && WX && 64 % (NW - WX) == 0;
  static constexpr int TL = T_SPARE ? 64 / T_PARTS : 64;
  static constexpr int CWT = T_INST && !T_SPARE ? 1 : 0;         // else: T by every wave (same 1 KB)
  static constexpr int CW = CWW + CWX + CWT;                    // DMA instructions per wave per stage
  static constexpr int W_BYTES = W_INST * 1024;
  static constexpr int X_BYTES = X_INST * 1024;
  static constexpr int T_OFF = W_BYTES + X_BYTES, DUMMY = T_OFF + (T_INST ? 1024 : 0);
  static constexpr bool NEED_DUMMY = WX && !T_SPARE;
  static constexpr int STAGE = DUMMY + (NEED_DUMMY ? 1024 : 0);
  static constexpr int D = (kLdsBytes / STAGE) > 3 ? 3 : (kLdsBytes / STAGE);
  static constexpr int LDS = D * STAGE;
  static constexpr int OVERREAD = WIN - SB * BB;                // bytes read past a row's last block
  static_assert(D >= 2, "ring");
  static_assert((D - 1) * CW < 64, "vmcnt");
  static_assert(X_INST % NW == 0, "activation pieces per wave");
  static_assert(SB % KG == 0, "blocks per K-group");
  static_assert(MW * MT * NT * 256 * 4 <= D * STAGE, "K-group reduction buffer");
  static_assert(!T_INST || T_SPARE || CWT, "T");
};

struct WideArgs {
  const uint8_t *a;      // weights (buffer base + dataOffset)
  const u32x4 *frag;     // xsplit_kernel output (16-column tiles)
  const float *xsum;     // xsplit_kernel Σx per (block, column) (mult 1 for Q4_1)
  uint8_t *dst;
  int64_t d_nb0, d_nb1;
  float *partial;        // [slices][M][tiles_n·BN] when slices > 1
  int32_t M, N, K;
  int32_t tiles_m, tiles_n, slices, kslice;  // kslice: blocks per slice (a multiple of SB)
  int32_t tasks;                             // task space: super-tiles x sm·sn·slices (grid padded to 8)
  int32_t sm, sn;                            // super-tile: sm row bands x sn column tiles
  unsigned *rsync;                           // fused split-K reduction per output tile, or null
};

template <int QT>
__global__ __launch_bounds__(512) void gemm_wide_kernel(WideArgs g) {
  using G = WideGeom<QT>;
  constexpr int MT = G::MT, NT = G::NT, BM = G::BM, BN = G::BN, BB = G::BB, SB = G::SB, D = G::D;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the second-dispatched half of the workgroup loses issue arbitration on its SIMD to the first:
  // static priority for it (MI355X_MICROARCH.md, two waves per SIMD, item 4): C5 ~2 % faster
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  // Task order (speed only: dispatch is observed round-robin over the 8 XCDs): workgroup b runs
  // task (b % 8)·(grid / 8) + b / 8, so each XCD gets a contiguous run of tasks; tasks walk
  // super-tiles of sm row bands x sn column tiles (all slices), so an XCD's L2 holds the
  // activation fragments of only sn column tiles and the weights of only sm row bands.
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding
  const int slice = task % g.slices, u = task / g.slices;
  const int per_st = g.sm * g.sn, nsn = (g.tiles_n + g.sn - 1) / g.sn;
  const int st_idx = u / per_st, within = u % per_st;
  const int tm = (st_idx / nsn) * g.sm + within / g.sn, tn = (st_idx % nsn) * g.sn + within % g.sn;
  if (tm >= g.tiles_m || tn >= g.tiles_n) return;  // a super-tile past the edge
  const int nblk = g.K / 32;
  const int kb0 = slice * g.kslice, kb1 = min(kb0 + g.kslice, nblk);
  const int nst = (kb1 - kb0) / SB;
  const int64_t RB = (int64_t)nblk * BB;
  const int ntx = (g.N + 15) / 16, n16 = ntx * 16;

  // per-lane DMA offsets (fixed for the launch) from each kind's stage base
  uint32_t wofs[G::CWW], xofs[G::CWX], tofs = 0;
  // this wave's weight instructions: q = wq0 .. wq0 + nwq − 1 (see WideGeom)
  const int nwq = (G::WX == 0 || wave < G::WX) ? G::CWW : G::CWW - 1;
  const int wq0 = (G::WX == 0 || wave < G::WX) ? wave * G::CWW : G::WX * G::CWW + (wave - G::WX) * (G::CWW - 1);
#pragma unroll
  for (int c = 0; c < G::CWW; c++) {
    const int piece = min((wq0 + min(c, nwq - 1)) * 64 + lane, G::WPIECES - 1);
    const int r = piece / (G::WIN / 16), pc = piece % (G::WIN / 16);
    const int64_t row = min((int64_t)tm * BM + r, (int64_t)g.M - 1);
    wofs[c] = (uint32_t)(row * RB + pc * 16);
  }
#pragma unroll
  for (int c = 0; c < G::CWX; c++) {
    const int x = wave * G::CWX + c;  // (block b, x-tile j, split s)
    const int b = x / (NT * kXSplits), j = (x / kXSplits) % NT, sp = x % kXSplits;
    const int xt = min(tn * NT + j, ntx - 1);
    xofs[c] = (uint32_t)((((int64_t)xt * nblk + b) * kXSplits + sp) * 1024 + lane * 16);
  }
  if constexpr (G::T_INST) {
    // lane -> T index li = (block li / (BN/4), 4 columns); a spare-slot part covers TL of them
    const int li = min((G::T_SPARE ? (wave - G::WX) * G::TL : 0) + lane, SB * BN / 4 - 1);
    const int b = li / (BN / 4), c4 = li % (BN / 4);
    const int n = min(tn * BN + 4 * c4, n16 - 4);
    tofs = (uint32_t)(((int64_t)b * n16 + n) * 4);
  }
  auto issue_stage = [&](int st, int sl) __attribute__((always_inline)) {
    const int kb = kb0 + min(st, nst - 1) * SB;  // past the last stage: reload the last (never read)
    const uint8_t *base_a = g.a + (int64_t)kb * BB;
    const uint8_t *base_x = (const uint8_t *)g.frag + (int64_t)kb * kXSplits * 1024;
    uint8_t *slot = smem + sl * G::STAGE;
#pragma unroll
    for (int c = 0; c < G::CWW; c++) {
      if (c < nwq) {
        dma16<false>(base_a, wofs[c], slot + (wq0 + c) * 1024);
      } else if constexpr (G::T_SPARE) {  // T part (wave − WX): TL lanes, TL·16 bytes
        if (lane < G::TL)
          dma16<false>((const uint8_t *)(g.xsum + (int64_t)kb * n16), tofs, slot + G::T_OFF + (wave - G::WX) * G::TL * 16);
      } else {
        dma16<false>(base_a, wofs[c], slot + G::DUMMY);  // padding (never read)
      }
    }
#pragma unroll
    for (int c = 0; c < G::CWX; c++) dma16<false>(base_x, xofs[c], slot + G::W_BYTES + (wave * G::CWX + c) * 1024);
    if constexpr (G::CWT)
      dma16<false>((const uint8_t *)(g.xsum + (int64_t)kb * n16), tofs, slot + G::T_OFF);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int mw = wave % G::MW, kg = wave / G::MW;
  constexpr int BPG = SB / G::KG;  // blocks per K-group per stage

  if (nst > 0) {
    for (int st = 0; st < D; st++) issue_stage(st, st);
    int slot = 0;
    const int m = lane & 15, gq = lane >> 4;
    for (int st = 0; st < nst; st++) {
      wait_vmcnt<(D - 1) * G::CW>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const uint8_t *W = smem + slot * G::STAGE;
      const uint8_t *X = W + G::W_BYTES;
      const float *T = (const float *)(W + G::T_OFF);
      // this K-group's blocks of the stage into registers with one burst of LDS reads, so the
      // slot can be refilled at once and the MFMAs never wait on LDS
      constexpr int WD = QT == LK_TYPE_Q4_1 ? 2 : QT == LK_TYPE_Q4_0 ? 3 : 4;
      // Q4_0 / Q4_1 read their Σx during the compute (an early refill with T in a ring of its own, or
      // one barrier per stage refilling the previous stage's slot, measured no faster on C5)
      constexpr bool EARLY = !G::T_INST;
      uint32_t wd[BPG][MT][WD];
      u32x4 xh[BPG][NT], xl[BPG][NT];
#pragma unroll
      for (int bb = 0; bb < BPG; bb++) {
        const int b = kg * BPG + bb;
        const int ob = b * BB;  // kg is wave-uniform: its two parities give two code paths
#pragma unroll
        for (int i = 0; i < MT; i++) {
          const uint8_t *rowp = W + ((mw * MT + i) * 16 + m) * G::WIN;  // window row
          auto rd = [&](int o) __attribute__((always_inline)) { return *(const uint32_t *)(rowp + o); };
          if constexpr (QT == LK_TYPE_Q4_1) {
            wd[bb][i][0] = rd(ob);
            wd[bb][i][1] = rd(ob + 4 + 4 * gq);
          } else if constexpr (QT == LK_TYPE_Q4_0) {  // 18-B blocks: ob % 4 == 0 iff b even
            if ((bb & 1) == 0) {
              wd[bb][i][0] = rd(ob);
              wd[bb][i][1] = rd(ob + 4 * gq);
              wd[bb][i][2] = rd(ob + 4 * gq + 4);
            } else {
              wd[bb][i][0] = rd(ob - 2);
              wd[bb][i][1] = rd(ob + 2 + 4 * gq);
              wd[bb][i][2] = 0;
            }
          } else {  // 34-B blocks: the same parity rule
            if ((bb & 1) == 0) {
              wd[bb][i][0] = rd(ob);
              wd[bb][i][1] = rd(ob + 8 * gq);
              wd[bb][i][2] = rd(ob + 8 * gq + 4);
              wd[bb][i][3] = rd(ob + 8 * gq + 8);
            } else {
              wd[bb][i][0] = rd(ob - 2);
              wd[bb][i][1] = rd(ob + 2 + 8 * gq);
              wd[bb][i][2] = rd(ob + 6 + 8 * gq);
              wd[bb][i][3] = 0;
            }
          }
        }
#pragma unroll
        for (int j = 0; j < NT; j++) {
          const u32x4 *xf = (const u32x4 *)(X + ((b * NT + j) * kXSplits) * 1024) + lane;
          xh[bb][j] = xf[0];
          xl[bb][j] = xf[64];
        }
      }
      asm volatile("" ::: "memory");  // the burst stays ahead of the refill
      if constexpr (EARLY) {
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();  // every wave has its copy of this slot: refill it now
        issue_stage(st + D, slot);
      }
#pragma unroll
      for (int bb = 0; bb < BPG; bb++) {
        const int b = kg * BPG + bb;
        bf16x8 wf[MT];
        float s1[MT], s2[MT];
#pragma unroll
        for (int i = 0; i < MT; i++) {
          s2[i] = 0.f;
          if constexpr (QT == LK_TYPE_Q4_1) {
            wf[i] = Q4Frag<0>::make(wd[bb][i][1]);
            s1[i] = 512.f * h2f(wd[bb][i][0]);
            s2[i] = h2f(wd[bb][i][0] >> 16);
          } else if constexpr (QT == LK_TYPE_Q4_0) {  // codes 128 + n; −136·Σx enters as the MFMA's C
            if ((bb & 1) == 0) {
              wf[i] = q4_codes_128(align2(wd[bb][i][2], wd[bb][i][1]));
              s1[i] = h2f(wd[bb][i][0]);
            } else {
              wf[i] = q4_codes_128(wd[bb][i][1]);
              s1[i] = h2f(wd[bb][i][0] >> 16);
            }
          } else {
            if ((bb & 1) == 0) {
              wf[i] = w_frag<LK_TYPE_Q8_0>(align2(wd[bb][i][2], wd[bb][i][1]), align2(wd[bb][i][3], wd[bb][i][2]));
              s1[i] = h2f(wd[bb][i][0]);
            } else {
              wf[i] = w_frag<LK_TYPE_Q8_0>(wd[bb][i][1], wd[bb][i][2]);
              s1[i] = h2f(wd[bb][i][0] >> 16);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < NT; j++) {
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
          if constexpr (QT != LK_TYPE_Q8_0) t = *(const f32x4 *)(T + b * BN + j * 16 + gq * 4);
#pragma unroll
          for (int i = 0; i < MT; i++) {
            // Q4_0: p = Σ (128 + n)·x − 136·Σx = Σ (n − 8)·x (T is −136·Σ(hi + lo), the split's own sum)
            f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xl[bb][j]), wf[i],
                                                              QT == LK_TYPE_Q4_0 ? t : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xh[bb][j]), wf[i], p, 0, 0, 0);
#if LK_WIDE_SCHED & 1
            accumulate_s<QT == LK_TYPE_Q4_1>(acc[i][j], s1[i], s2[i], p, t);
#else
            accumulate<QT == LK_TYPE_Q4_1>(acc[i][j], s1[i], s2[i], p, t);
#endif
          }
        }
#if LK_WIDE_SCHED & 2
        // the scale FMAs between the MFMAs (the compiler otherwise issues all MFMAs of the block, then
        // all the accumulates: two waves of a SIMD in step then contend for the matrix pipe and the
        // VALU in turn instead of overlapping them)
#pragma unroll
        for (int q = 0; q < MT * NT; q++) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                      // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, (LK_WIDE_SCHED & 1) ? 4 : 2, 0);  // the scale FMAs
        }
#endif
      }
      if constexpr (!EARLY) {
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();  // every wave is done with this slot
        issue_stage(st + D, slot);
      }
      slot = (slot + 1 == D) ? 0 : slot + 1;
    }
    wait_vmcnt<0>();  // drain the padding stages before the ring is reused below
  }
  // K-group 1 hands its sums to K-group 0 through LDS (the ring is free now), in a fixed order
  __syncthreads();
  f32x4 *red = (f32x4 *)smem + (size_t)mw * (MT * NT * 64) + lane;
  if (kg == 1) {
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) red[(i * NT + j) * 64] = acc[i][j];
  }
  __syncthreads();
  const int npad = g.tiles_n * BN;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * npad * 4) ? g.slices * g.M * npad * 4 : 0, 0x00020000);
  auto store_dst = [&](int64_t m, int n0, const f32x4 &v) __attribute__((always_inline)) {
    const float e4[4] = {v.x, v.y, v.z, v.w};
    if (g.d_nb0 == 4 && n0 + 4 <= g.N && ((((uintptr_t)g.dst + m * g.d_nb1 + n0 * 4) & 15) == 0)) {
      *(f32x4 *)(g.dst + m * g.d_nb1 + n0 * 4) = v;
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (n0 + q < g.N) *(float *)(g.dst + m * g.d_nb1 + (n0 + q) * g.d_nb0) = e4[q];
    }
  };
  if (kg == 0) {
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const f32x4 o = red[(i * NT + j) * 64];
        acc[i][j].x += o.x; acc[i][j].y += o.y; acc[i][j].z += o.z; acc[i][j].w += o.w;
      }
    // outputs: lane holds C'(n = 16·(tn·NT + j) + 4(lane>>4) + e, m = tm·BM + (mw·MT + i)·16 + (lane&15))
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const int64_t m = (int64_t)tm * BM + (mw * MT + i) * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const int n0 = tn * BN + j * 16 + 4 * (lane >> 4);
        if (g.slices > 1) store_partial(slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * npad * 4), prs, g.partial, ((int64_t)slice * g.M + m) * npad + n0, acc[i][j]);
        else store_dst(m, n0, acc[i][j]);
      }
    }
  }
  if (g.rsync) {
    // split-K fix-up by the last arriver (splitk_arrive): the workgroup whose slice completes the
    // tile sums it — its own slice from registers, the others' slabs by sc1 loads, in slice order
    // (bit-identical to splitk_reduce_kernel); nobody waits for another workgroup
    wait_vmcnt<0>();
    __syncthreads();
    int *flag = (int *)smem;  // the ring is free (K-group 1's sums were read before this barrier)
    if (threadIdx.x == 0) *flag = splitk_arrive(g.rsync + (int64_t)(tm * g.tiles_n + tn) * kChainLine, (unsigned)g.slices) ? 1 : 0;
    __syncthreads();
    asm volatile("" ::: "memory");
    if (*flag && kg == 0) {
      // per slab all MT·NT loads of the lane in flight at once (rows past M re-read row M − 1)
      f32x4 sum[MT][NT];
      for (int b = 0; b < g.slices; b++) {
        f32x4 v[MT][NT];
#pragma unroll
        for (int i = 0; i < MT; i++) {
          const int64_t m = min((int64_t)tm * BM + (mw * MT + i) * 16 + (lane & 15), (int64_t)g.M - 1);
#pragma unroll
          for (int j = 0; j < NT; j++) {
            const int n0 = tn * BN + j * 16 + 4 * (lane >> 4);
            v[i][j] = b == slice ? acc[i][j]
                                 : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, (int)((((int64_t)b * g.M + m) * npad + n0) * 4), 0, 16));
          }
        }
#pragma unroll
        for (int i = 0; i < MT; i++)
#pragma unroll
          for (int j = 0; j < NT; j++) {
            if (b == 0) sum[i][j] = v[i][j];  // slab 0 as is (0 + x would turn -0.0 into +0.0)
            else { sum[i][j].x += v[i][j].x; sum[i][j].y += v[i][j].y; sum[i][j].z += v[i][j].z; sum[i][j].w += v[i][j].w; }
          }
      }
#pragma unroll
      for (int i = 0; i < MT; i++) {
        const int64_t m = (int64_t)tm * BM + (mw * MT + i) * 16 + (lane & 15);
        if (m >= g.M) continue;
#pragma unroll
        for (int j = 0; j < NT; j++) store_dst(m, tn * BN + j * 16 + 4 * (lane >> 4), sum[i][j]);
      }
    }
  }
}

// dst(n, m) = Σ_s P[s][m][n], slices in order (deterministic); one thread per 4 columns.
#ifndef LK_W32_KERNELS  // (lk_w32.hip includes this header for its helpers only)
__device__ __forceinline__ void splitk_reduce_body(const float *__restrict__ P, int slices, int M, int N, int N16,
                                                   uint8_t *__restrict__ dst, int64_t d_nb0, int64_t d_nb1, int64_t idx);

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float *__restrict__ P, int slices, int M, int N, int N16,
                                                            uint8_t *__restrict__ dst, int64_t d_nb0, int64_t d_nb1) {
  splitk_reduce_body(P, slices, M, N, N16, dst, d_nb0, d_nb1, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

__global__ __launch_bounds__(256) void splitk_reduce_group_kernel(const ReduceNode *__restrict__ nodes, int nnodes) {
  int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int k = 0; k < nnodes; k++) {
    const int64_t blocks = (nodes[k].threads + 255) / 256 * 256;  // each node starts on a block boundary
    if (idx < blocks) {
      const ReduceNode &r = nodes[k];
      splitk_reduce_body(r.partial, r.slices, r.M, r.N, r.N16, r.dst, r.d_nb0, r.d_nb1, idx);
      return;
    }
    idx -= blocks;
  }
}

__device__ __forceinline__ void splitk_reduce_body(const float *__restrict__ P, int slices, int M, int N, int N16,
                                                   uint8_t *__restrict__ dst, int64_t d_nb0, int64_t d_nb1, int64_t idx) {
  const int c4 = N16 / 4;
  if (idx >= (int64_t)M * c4) return;
  const int64_t m = idx / c4;
  const int n0 = (int)(idx % c4) * 4;
  // slabs in slice order (deterministic); all of a group's loads (up to 16) in flight at once,
  // the first slab's included, instead of one dependent round trip per slice
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < slices; b += 16) {
    f32x4 v[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
      if (b + i < slices) v[i] = __builtin_nontemporal_load((const f32x4 *)(P + ((int64_t)(b + i) * M + m) * N16 + n0));
#pragma unroll
    for (int i = 0; i < 16; i++)
      if (b + i < slices) {
        if (b + i == 0) s = v[i];  // slab 0 as is (0 + x would turn -0.0 into +0.0)
        else { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
      }
  }
  const float e4[4] = {s.x, s.y, s.z, s.w};
  if (d_nb0 == 4 && n0 + 4 <= N && (((uintptr_t)(dst + m * d_nb1 + n0 * 4)) & 15) == 0) {
    *(f32x4 *)(dst + m * d_nb1 + n0 * 4) = s;
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; q++)
    if (n0 + q < N) *(float *)(dst + m * d_nb1 + (n0 + q) * d_nb0) = e4[q];
}
#endif

// ---- F32 x F32 -> F32 general path on the f32 MFMA (computeMatMul :1530-1543, config C1) ----
//
// v_mfma_f32_32x32x2_f32: f32 operands, products exact, each accumulation one f32 rounding (a
// k-ordered fmaf chain), so the only difference from the reference's sequential sum is the
// summation order (within the F32 bar). One workgroup per 32x32 output tile, four waves; wave w
// takes K chunks w, w + 4, ... of 128: MFMA step s contracts k = {c + s, c + 64 + s} (lane half
// h supplies k = c + 64h + s), so a lane's A operand is 64 consecutive floats of its row (16
// float4 loads when rows are 16-byte aligned). The four waves' tiles are added in wave order
// through LDS (deterministic).
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <bool V4>
__global__ __launch_bounds__(256) void f32_mfma_kernel(GenericArgs g) {
  __shared__ float red[4][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t i0 = (int64_t)blockIdx.y * 32, j0 = (int64_t)blockIdx.x * 32;
  const int64_t i = i0 + r, j = j0 + r;
  const bool iok = i < g.M, jok = j < g.N;
  f32x16_t acc = {};
  for (int64_t c = (int64_t)wave * 128; c < g.K; c += 4 * 128) {
    const int64_t kb = c + 64 * h;
    float av[64], bv[64];
    if (V4 && iok && c + 128 <= g.K) {
      const f32x4 *ap = (const f32x4 *)(g.a + i * g.a_nb1 + kb * 4);
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const f32x4 t = ap[q];
        av[4 * q] = t.x; av[4 * q + 1] = t.y; av[4 * q + 2] = t.z; av[4 * q + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 64; s++)
        av[s] = (iok && kb + s < g.K) ? *(const float *)(g.a + i * g.a_nb1 + (kb + s) * g.a_nb0) : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 64; s++)
      bv[s] = (jok && kb + s < g.K) ? *(const float *)(g.b + j * g.b_nb0 + (kb + s) * g.b_nb1) : 0.f;
#pragma unroll
    for (int s = 0; s < 64; s++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 16; q++) red[wave][q][lane] = acc[q];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
      float v = red[0][q][lane];
      v += red[1][q][lane];
      v += red[2][q][lane];
      v += red[3][q][lane];
      const int64_t ii = i0 + (q & 3) + 8 * (q >> 2) + 4 * h;  // C row (A row), column = lane r (B column)
      if (ii < g.M && jok) *(float *)(g.dst + j * g.d_nb0 + ii * g.d_nb1) = v;
    }
  }
}

// Dense variant (C1): the same tiles and K split, operands staged in LDS by LDS-DMA in whole
// 16-B pieces (A: row pieces XOR-swizzled by row, so the 16 rows of a ds_read_b128 lane group hit
// distinct bank slots; B: k rows of the tile's 32 columns), then read per MFMA step from LDS —
// instead of per-lane strided global loads (each A load instruction touched 64 lines). Needs
// K % 128 == 0, A rows and B k rows 16-B aligned, N % 4 == 0; rows / columns past M / N re-read
// the last valid ones and are never stored.
constexpr int kF32Chunk = 128;  // k per wave and chunk
#ifndef LK_W32_KERNELS  // (lk_w32.hip includes this header for its helpers only)
__global__ __launch_bounds__(256) void f32_lds_kernel(GenericArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t i0 = (int64_t)blockIdx.y * 32, j0 = (int64_t)blockIdx.x * 32;
  uint8_t *abuf = smem + wave * 32768, *bbuf = abuf + 16384;  // this wave's A (2 x 32 x 64) and B (128 x 32)
  f32x16_t acc = {};
  for (int64_t kc = (int64_t)wave * kF32Chunk; kc < g.K; kc += 4 * kF32Chunk) {
    // two halves of 64 k, each A [32 rows][16 pieces] then B [64 k][32 columns]: the first half's
    // MFMAs run while the second half lands
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
#pragma unroll
      for (int t = 0; t < 8; t++) {
        const int q = t * 64 + lane, ar = q >> 4, cp = (q & 15) ^ (ar & 15);  // A: row ar, piece cp
        const int64_t ai = min(i0 + ar, g.M - 1);
        dma16<false>(g.a, (uint32_t)(ai * g.a_nb1 + (kc + 64 * hf + 4 * cp) * 4), abuf + hf * 8192 + t * 1024);
      }
#pragma unroll
      for (int t = 0; t < 8; t++) {
        const int q = t * 64 + lane, bk = q >> 3, c = q & 7;  // B: k row bk, columns j0 + 4c ..
        const int64_t bj = min(j0 + 4 * c, g.N - 4);
        dma16<false>(g.b, (uint32_t)((kc + 64 * hf + bk) * g.b_nb1 + bj * 4), bbuf + hf * 8192 + t * 1024);
      }
    }
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
      if (hf == 0) wait_vmcnt<16>();
      else wait_vmcnt<0>();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int s4 = 0; s4 < 8; s4++) {  // MFMA steps 4·s4 .. +3: lane half h supplies k = 64·hf + 32h + s
        const int piece = 8 * h + s4;
        const f32x4 av = *(const f32x4 *)(abuf + hf * 8192 + r * 256 + ((piece ^ (r & 15)) * 16));
        const float *bp = (const float *)(bbuf + hf * 8192 + (32 * h + 4 * s4) * 128) + r;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bp[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bp[32], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bp[64], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bp[96], acc, 0, 0, 0);
      }
    }
    wait_lgkmcnt0();  // this chunk's LDS reads are done before the next chunk's DMA overwrites it
  }
  __syncthreads();
  float *red = (float *)smem;  // [4][16][64], over the (now idle) staging area
#pragma unroll
  for (int q = 0; q < 16; q++) red[(wave * 16 + q) * 64 + lane] = acc[q];
  __syncthreads();
  for (int e = (int)threadIdx.x; e < 16 * 64; e += 256) {  // waves summed in order (deterministic)
    const int q = e >> 6, l = e & 63;
    const float v = ((red[q * 64 + l] + red[(16 + q) * 64 + l]) + red[(32 + q) * 64 + l]) + red[(48 + q) * 64 + l];
    const int64_t ii = i0 + (q & 3) + 8 * (q >> 2) + 4 * (l >> 5), jj = j0 + (l & 31);
    if (ii < g.M && jj < g.N) *(float *)(g.dst + jj * g.d_nb0 + ii * g.d_nb1) = v;
  }
}
#endif

// ---- generic path (any K, any byte strides, ragged blocks) ----------------------


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

// ---- K-quant dots: Q2_K / Q4_K / Q8_K x F32 (core/GGMLComputeOps.kt:152-432) -------------------
//
// llama.kotlin's own K-quant formulas (not upstream ggml's), element for element: every weight
// is the value the Kotlin loop computes for (row, k) — f32 roundings in the same order, no
// contraction — including its "full block" reading of block (row·K + blockStart)/256 from item 0
// when K % 256 != 0 and the flat-index partial path with its own formula (Q4_K adds dmin there).
// Only the order of the f32 sum differs. One wave per output (i, j): lane l takes the 4
// consecutive k = 256·s + 4l .. +3 of every 256-span s (one sub-block, so one scale/min).

struct KQuantArgs {
  const uint8_t *a;            // blocks (buffer base + dataOffset)
  const uint8_t *b;            // B(n, k) at n·b_nb0 + k·b_nb1
  uint8_t *dst;                // dst(n, m) at n·d_nb0 + m·d_nb1
  int64_t b_nb0, b_nb1, d_nb0, d_nb1;
  int64_t M, N, K;
};

template <int QT> struct KQTraits;
template <> struct KQTraits<LK_TYPE_Q2_K> { static constexpr int BB = LK_Q2_K_BLOCK_BYTES; };
template <> struct KQTraits<LK_TYPE_Q4_K> { static constexpr int BB = LK_Q4_K_BLOCK_BYTES; };
template <> struct KQTraits<LK_TYPE_Q8_K> { static constexpr int BB = LK_Q8_K_BLOCK_BYTES; };

__device__ __forceinline__ int sbyte(const uint8_t *p) { return (int)(int8_t)*p; }  // Kotlin Byte.toInt()
__device__ __forceinline__ float kq_h(const uint8_t *p) { return h2f((uint32_t)p[0] | ((uint32_t)p[1] << 8)); }

// The weight of item `item` of block `blk`; FULL selects the full-block formulas.
template <int QT, bool FULL>
__device__ __forceinline__ float kq_weight(const uint8_t *blk, int item) {
  if constexpr (QT == LK_TYPE_Q2_K) {  // :182-196 (full), :216-227 (partial): the same formulas
    const float d = kq_h(blk + 80), dmin = kq_h(blk + 82);
    const int sb = item / 16;
    const int sm = sbyte(blk + sb);
    const float scale = __fmul_rn(__fdiv_rn((float)(sm & 0x0F), 15.0f), d);
    const float mn = __fadd_rn(__fmul_rn((float)((sm >> 4) & 0x0F), d), dmin);
    const int qb = sbyte(blk + 16 + sb * 4 + (item % 16) / 4);
    const int q = (qb >> (((item % 16) % 4) * 2)) & 0x03;
    return __fadd_rn(__fmul_rn(__fdiv_rn((float)q, 3.0f), scale), mn);
  } else if constexpr (QT == LK_TYPE_Q4_K) {
    const float d = kq_h(blk), dmin = kq_h(blk + 2);
    const int sb = item / 32;
    const int sc = sbyte(blk + 4 + sb);
    const float scale = __fmul_rn(__fdiv_rn((float)(sc & 0x3F), 63.0f), d);
    const int qb = sbyte(blk + 4 + LK_K_SCALE_SIZE + sb * 16 + (item % 32) / 2);
    const int q = (item % 2 == 0) ? (qb & 0x0F) : ((qb >> 4) & 0x0F);
    float off;
    if constexpr (FULL) {  // :274-287: 6-bit min from the scale byte's top bits + a nibble of byte 4 + 2sb + 1
      const int qmh = (sb * 2 + 1 < LK_K_SCALE_SIZE) ? (sbyte(blk + 4 + sb * 2 + 1) & 0x0F) : 0;
      const int qm = ((sc >> 6) & 0x03) | (qmh << 2);
      off = __fadd_rn(__fmul_rn(__fdiv_rn((float)qm, 63.0f), d), dmin);
    } else {               // :331: the partial path adds dmin itself
      off = dmin;
    }
    return __fadd_rn(__fmul_rn(__fdiv_rn((float)q, 15.0f), scale), off);
  } else {  // Q8_K :404-407, :418-420
    const float d = __builtin_bit_cast(float, (uint32_t)blk[0] | ((uint32_t)blk[1] << 8) | ((uint32_t)blk[2] << 16) |
                                                  ((uint32_t)blk[3] << 24));
    return __fmul_rn((float)sbyte(blk + 4 + item), d);
  }
}

template <int QT>
__global__ __launch_bounds__(256) void kquant_mul_mat_kernel(KQuantArgs g) {
  constexpr int BB = KQTraits<QT>::BB;
  const int64_t out = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (out >= g.M * g.N) return;
  const int lane = threadIdx.x & 63;
  const int64_t i = out / g.N, j = out % g.N;
  const uint8_t *xb = g.b + j * g.b_nb0;
  float s = 0.f;
  for (int64_t bs = 0; bs < g.K; bs += LK_QK_K) {
    const int64_t be = min(bs + (int64_t)LK_QK_K, g.K);
    if (be - bs == LK_QK_K) {
      const uint8_t *blk = g.a + ((i * g.K + bs) / LK_QK_K) * BB;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int item = 4 * lane + e;
        const float w = kq_weight<QT, true>(blk, item);
        s = fmaf(w, *(const float *)(xb + (bs + item) * g.b_nb1), s);
      }
    } else {
      for (int64_t k = bs + lane; k < be; k += 64) {
        const int64_t flat = i * g.K + k;
        const float w = kq_weight<QT, false>(g.a + (flat / LK_QK_K) * BB, (int)(flat % LK_QK_K));
        s = fmaf(w, *(const float *)(xb + k * g.b_nb1), s);
      }
    }
  }
  s = wave_sum(s);
  if (lane == 0) *(float *)(g.dst + j * g.d_nb0 + i * g.d_nb1) = s;
}

// K % 256 == 0 (every super-block full, row i's blocks are i·K/256 .. +K/256-1): one wave per
// (row, group of NC columns), the weights of a block decoded once for the NC columns. Lane l
// owns items 4l .. 4l+3 of every block, which lie in one sub-block, so the scale / min terms are
// decoded once per block per lane; the quotients q/3, q/15, q/63 come from LDS tables filled
// with the same correctly rounded division, so every weight is bit-identical to kq_weight
// (no contraction in this function). U blocks are loaded before any is used. ALIGNED: the
// block base is 4-byte aligned (BB is a multiple of 4), so header / code bytes load as words.
template <bool ALIGNED> __device__ __forceinline__ uint32_t kq_ld32(const uint8_t *p) {
  if constexpr (ALIGNED) return *(const uint32_t *)p;
  else return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
template <bool ALIGNED> __device__ __forceinline__ uint32_t kq_ld16(const uint8_t *p) {
  if constexpr (ALIGNED) return *(const uint16_t *)p;
  else return (uint32_t)p[0] | ((uint32_t)p[1] << 8);
}
__device__ __forceinline__ int sext8(uint32_t b) { return (int)(int8_t)(uint8_t)b; }

struct KqTables { float q3[4], q15[16], q63[64]; };

// A lane's raw bytes of one block (loads only; kq_decode turns them into its 4 weights).
struct KqRaw { uint32_t h, b0, b1, q; };

template <int QT, bool ALIGNED>
__device__ __forceinline__ KqRaw kq_load(const uint8_t *blk, int lane) {
  KqRaw r{};
  if constexpr (QT == LK_TYPE_Q2_K) {  // d | dmin at 80, scale byte l/4, codes byte 16 + l
    r.h = kq_ld32<ALIGNED>(blk + 80);
    r.b0 = blk[lane >> 2];
    r.q = blk[16 + lane];
  } else if constexpr (QT == LK_TYPE_Q4_K) {  // d | dmin at 0, scale byte 4 + l/8, min-high byte, codes 16 + 2l
    const int sb = lane >> 3;
    r.h = kq_ld32<ALIGNED>(blk);
    r.b0 = blk[4 + sb];
    r.b1 = blk[4 + min(sb * 2 + 1, LK_K_SCALE_SIZE - 1)];  // masked off in kq_decode past the scales
    r.q = kq_ld16<ALIGNED>(blk + 4 + LK_K_SCALE_SIZE + 2 * lane);
  } else {  // Q8_K: f32 d at 0, codes 4 + 4l
    r.h = kq_ld32<ALIGNED>(blk);
    r.q = kq_ld32<ALIGNED>(blk + 4 + 4 * lane);
  }
  return r;
}

template <int QT>
__device__ __forceinline__ void kq_decode(const KqRaw &r, int lane, const KqTables &t, float w[4]) {
#pragma clang fp contract(off)
  if constexpr (QT == LK_TYPE_Q2_K) {  // :182-196
    const float d = h2f(r.h & 0xFFFF), dmin = h2f(r.h >> 16);
    const int sm = sext8(r.b0);
    const float scale = t.q15[sm & 0x0F] * d;
    const float mn = (float)((sm >> 4) & 0x0F) * d + dmin;
    const int qb = sext8(r.q);
#pragma unroll
    for (int e = 0; e < 4; e++) w[e] = t.q3[(qb >> (2 * e)) & 0x03] * scale + mn;
  } else if constexpr (QT == LK_TYPE_Q4_K) {  // :274-287
    const float d = h2f(r.h & 0xFFFF), dmin = h2f(r.h >> 16);
    const int sb = lane >> 3;
    const int sc = sext8(r.b0);
    const int qmh = (sb * 2 + 1 < LK_K_SCALE_SIZE) ? (sext8(r.b1) & 0x0F) : 0;
    const int qm = ((sc >> 6) & 0x03) | (qmh << 2);
    const float scale = t.q63[sc & 0x3F] * d;
    const float off = t.q63[qm] * d + dmin;
#pragma unroll
    for (int e = 0; e < 4; e++) w[e] = t.q15[(r.q >> (4 * e)) & 0x0F] * scale + off;
  } else {  // Q8_K :404-407
    const float d = __builtin_bit_cast(float, r.h);
#pragma unroll
    for (int e = 0; e < 4; e++) w[e] = (float)sext8(r.q >> (8 * e)) * d;
  }
}

template <int QT, int NC, bool VX, bool ALIGNED>
__global__ __launch_bounds__(256) void kquant_gemv_kernel(KQuantArgs g) {
  constexpr int BB = KQTraits<QT>::BB, U = NC == 1 ? 8 : 4;
  __shared__ KqTables t;
  {
    const int x = threadIdx.x;
    if (x < 64) t.q63[x] = __fdiv_rn((float)x, 63.0f);
    else if (x < 80) t.q15[x - 64] = __fdiv_rn((float)(x - 64), 15.0f);
    else if (x < 84) t.q3[x - 80] = __fdiv_rn((float)(x - 80), 3.0f);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (i >= g.M) return;
  const int64_t j0 = (int64_t)blockIdx.y * NC;
  const int64_t nb = g.K / LK_QK_K;
  const uint8_t *row = g.a + i * nb * BB;
  int64_t jc[NC];  // column of slot c, clamped (loads only; stores are guarded)
#pragma unroll
  for (int c = 0; c < NC; c++) jc[c] = min(j0 + c, g.N - 1);
  float acc[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) acc[c] = 0.f;
  for (int64_t s0 = 0; s0 < nb; s0 += U) {
    // every load of the U blocks first (block index clamped to the row: no guarded loads)
    KqRaw r[U];
    float x[U][NC][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t sblk = min(s0 + u, nb - 1);
      r[u] = kq_load<QT, ALIGNED>(row + sblk * BB, lane);
      const int64_t k = sblk * LK_QK_K + 4 * lane;
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const uint8_t *xb = g.b + jc[c] * g.b_nb0 + k * g.b_nb1;
        if constexpr (VX) {
          const f32x4 xv = *(const f32x4 *)xb;
          x[u][c][0] = xv.x; x[u][c][1] = xv.y; x[u][c][2] = xv.z; x[u][c][3] = xv.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++) x[u][c][e] = *(const float *)(xb + e * g.b_nb1);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      float w[4];
      kq_decode<QT>(r[u], lane, t, w);
      const bool live = s0 + u < nb;  // wave-uniform
#pragma unroll
      for (int c = 0; c < NC; c++) {
        float a = acc[c];
#pragma unroll
        for (int e = 0; e < 4; e++) a = fmaf(w[e], x[u][c][e], a);
        acc[c] = live ? a : acc[c];
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; c++) {
    const float s = wave_sum(acc[c]);
    if (lane == 0 && (NC == 1 || j0 + c < g.N)) *(float *)(g.dst + (j0 + c) * g.d_nb0 + i * g.d_nb1) = s;
  }
}

// K-quant x F32 at batch 1 (K % 256 == 0): a lane per 32 consecutive items of a block (lane
// l of a wave: block l/8 of the chunk, items 32·(l%8) ..), so a wave covers 8 blocks of its row
// per chunk and a lane's weights are a few wide loads (Q4_K: the 16-byte d / dmin / scales head
// and the 16 code bytes of its sub-block; Q2_K: d | dmin, its two scale bytes, 8 code bytes;
// Q8_K: d and 32 code bytes). The activation vector is staged once per workgroup (ROWS rows) in
// LDS, padded to 36 floats per 32 so a lane's 8 ds_read_b128 spread over the banks. Weights are
// the Kotlin values bit for bit (kq_weight's formulas, LDS quotient tables, no contraction);
// only the f32 sum order differs. Chunks go in pairs, loads first. Block bases must be 16-byte
// (Q4_K) / 4-byte (Q2_K, Q8_K) aligned: the launcher checks.
__device__ __forceinline__ uint32_t byte_of(const u32x4 &h, int idx) {  // byte idx (0..15), idx wave-varying
  const uint32_t w = idx < 4 ? h.x : idx < 8 ? h.y : idx < 12 ? h.z : h.w;
  return (w >> (8 * (idx & 3))) & 0xFF;
}

template <int QT> struct Kq32Raw;
template <> struct Kq32Raw<LK_TYPE_Q4_K> { u32x4 h, c; };
template <> struct Kq32Raw<LK_TYPE_Q2_K> { uint32_t h, sc, c0, c1; };
template <> struct Kq32Raw<LK_TYPE_Q8_K> { uint32_t d; uint32_t c[8]; };

template <int QT>
__device__ __forceinline__ Kq32Raw<QT> kq32_load(const uint8_t *blk, int s) {  // s = lane % 8
  Kq32Raw<QT> r;
  if constexpr (QT == LK_TYPE_Q4_K) {
    r.h = *(const u32x4 *)blk;
    r.c = *(const u32x4 *)(blk + 4 + LK_K_SCALE_SIZE + 16 * s);
  } else if constexpr (QT == LK_TYPE_Q2_K) {  // sub-blocks 2s, 2s+1: scale bytes 2s, 2s+1; codes 16 + 8s
    r.h = *(const uint32_t *)(blk + 80);
    r.sc = *(const uint32_t *)(blk + 4 * (s >> 1)) >> (16 * (s & 1));
    r.c0 = *(const uint32_t *)(blk + 16 + 8 * s);
    r.c1 = *(const uint32_t *)(blk + 20 + 8 * s);
  } else {
    r.d = *(const uint32_t *)blk;
#pragma unroll
    for (int j = 0; j < 8; j++) r.c[j] = *(const uint32_t *)(blk + 4 + 32 * s + 4 * j);
  }
  return r;
}

// a += Σ_e w(item 32s + e) · x[e], e = 0..31 in order
template <int QT>
__device__ __forceinline__ float kq32_dot(const Kq32Raw<QT> &r, int s, const KqTables &t, const f32x4 *xv, float a) {
#pragma clang fp contract(off)
  float xe[32];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const f32x4 v = xv[j];
    xe[4 * j] = v.x; xe[4 * j + 1] = v.y; xe[4 * j + 2] = v.z; xe[4 * j + 3] = v.w;
  }
  if constexpr (QT == LK_TYPE_Q4_K) {  // :274-287, sub-block s
    const float d = h2f(r.h.x & 0xFFFF), dmin = h2f(r.h.x >> 16);
    const int sc = sext8(byte_of(r.h, 4 + s));
    const int qmh = (s * 2 + 1 < LK_K_SCALE_SIZE) ? (sext8(byte_of(r.h, 5 + 2 * s)) & 0x0F) : 0;
    const int qm = ((sc >> 6) & 0x03) | (qmh << 2);
    const float scale = t.q63[sc & 0x3F] * d;
    const float off = t.q63[qm] * d + dmin;
    const uint32_t cw[4] = {r.c.x, r.c.y, r.c.z, r.c.w};
#pragma unroll
    for (int e = 0; e < 32; e++) a = fmaf(t.q15[(cw[e >> 3] >> (4 * (e & 7))) & 0x0F] * scale + off, xe[e], a);
  } else if constexpr (QT == LK_TYPE_Q2_K) {  // :182-196, sub-blocks 2s (items 0..15), 2s+1
    const float d = h2f(r.h & 0xFFFF), dmin = h2f(r.h >> 16);
#pragma unroll
    for (int hsb = 0; hsb < 2; hsb++) {
      const int sm = sext8((r.sc >> (8 * hsb)) & 0xFF);
      const float scale = t.q15[sm & 0x0F] * d;
      const float mn = (float)((sm >> 4) & 0x0F) * d + dmin;
      const uint32_t cw = hsb ? r.c1 : r.c0;  // item 16·hsb + 4m + e: byte m, bits 2e
#pragma unroll
      for (int e = 0; e < 16; e++) a = fmaf(t.q3[(cw >> (8 * (e >> 2) + 2 * (e & 3))) & 0x03] * scale + mn, xe[16 * hsb + e], a);
    }
  } else {  // Q8_K :404-407
    const float d = __builtin_bit_cast(float, r.d);
#pragma unroll
    for (int e = 0; e < 32; e++) a = fmaf((float)sext8(r.c[e >> 2] >> (8 * (e & 3))) * d, xe[e], a);
  }
  return a;
}

// Q4_K at batch 1, factored: Σ_e w_e·x_e with w_e = (q_e/15)·scale + off (:297-306) computed as
// (Σ q_e·x_e)/15·scale + off·Σ x_e: the codes enter as exact fp8 conversions (n·2⁻⁹, two per
// v_cvt_pk_f32_fp8) against the activations in nibble order (x0,x2,x4,x6 | x1,x3,x5,x7 per 8,
// as the stream kernel holds them), Σx comes from the pad slot 32 of the sub-block's LDS row. The
// quotient is correctly rounded (__fdiv_rn) and nothing is contracted, so a one-hot activation
// still yields the Kotlin weight bit for bit (S_q = q, Σx = 1, the other lanes exact zeros); in
// general only the f32 summation order differs from the reference, as everywhere else.
__device__ __forceinline__ float kq32_dot_q4k_factored(const Kq32Raw<LK_TYPE_Q4_K> &r, int s, const KqTables &t,
                                                       const f32x4 *xv, float a) {
#pragma clang fp contract(off)
  const float d = h2f(r.h.x & 0xFFFF), dmin = h2f(r.h.x >> 16);
  const int sc = sext8(byte_of(r.h, 4 + s));
  const int qmh = (s * 2 + 1 < LK_K_SCALE_SIZE) ? (sext8(byte_of(r.h, 5 + 2 * s)) & 0x0F) : 0;
  const int qm = ((sc >> 6) & 0x03) | (qmh << 2);
  const float scale = t.q63[sc & 0x3F] * d;
  const float off = t.q63[qm] * d + dmin;
  const uint32_t cw[4] = {r.c.x, r.c.y, r.c.z, r.c.w};
  f2v s2 = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t lo = cw[j] & 0x0F0F0F0Fu, hi = (cw[j] >> 4) & 0x0F0F0F0Fu;
    const f32x4 xa = xv[2 * j], xb = xv[2 * j + 1];
    s2 = __builtin_elementwise_fma(fp8x2<false>(lo), f2v{xa.x, xa.y}, s2);
    s2 = __builtin_elementwise_fma(fp8x2<true>(lo), f2v{xa.z, xa.w}, s2);
    s2 = __builtin_elementwise_fma(fp8x2<false>(hi), f2v{xb.x, xb.y}, s2);
    s2 = __builtin_elementwise_fma(fp8x2<true>(hi), f2v{xb.z, xb.w}, s2);
  }
  const float sq = (s2.x + s2.y) * 512.f;             // Σ q·x (the 2⁻⁹ scaling is exact)
  const float sx = ((const float *)xv)[32];            // Σ x of the sub-block
  const float part = __fdiv_rn(sq, 15.0f) * scale;
  return a + (part + off * sx);
}

// Q4_K in the stream kernel (gemv_stream_kernel<Q4_K>): the lane's two sub-blocks s = 2(lane%4)
// and s + 1, each as kq32_dot_q4k_factored computes it (the same scale/min decoding of the
// Kotlin layout, :274-306; (Σ q·x)/15·scale + off·Σx, correctly rounded quotient, nothing
// contracted), with the activations and Σx the stream kernel holds in VGPRs and i/63 from LDS.
__device__ float q4k_stream_dot(const u32x4 &h, const u32x4 &c0, const u32x4 &c1, int lane, const f32x4 *xr, float xs0,
                                float xs1, const float *q63) {
#pragma clang fp contract(off)
  const float d = h2f(h.x & 0xFFFF), dmin = h2f(h.x >> 16);
  // sub-blocks s = 2j + q (j = lane % 4): scale bytes 4 + s = the 16-bit field at byte 4 + 2j;
  // the min's high bits from byte 5 + 2s = byte 1 + 2q of header dword j + 1 (none for j = 3,
  // s >= 6: byte 4 + 2s + 1 would lie past the 12 scale bytes)
  const int j = lane & 3;
  const uint32_t scw = ((j & 2) ? h.z : h.y) >> (16 * (j & 1));
  const uint32_t mw = (j & 2) ? ((j & 1) ? 0u : h.w) : ((j & 1) ? h.z : h.y);  // selects, not a switch
  constexpr float r15 = 1.0f / 15.0f;
  float a = 0.f;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t sc = (scw >> (8 * q)) & 0xFF;          // (sext8(sc) >> 6) & 3 == sc >> 6
    const uint32_t qm = (sc >> 6) | (((mw >> (8 + 16 * q)) & 0x0F) << 2);
    const float scale = q63[sc & 0x3F] * d;
    const float off = q63[qm] * d + dmin;
    const u32x4 c = q ? c1 : c0;
    const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
    f2v s2 = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const uint32_t lo = cw[t] & 0x0F0F0F0Fu, hi = (cw[t] >> 4) & 0x0F0F0F0Fu;
      const f32x4 xa = xr[8 * q + 2 * t], xb = xr[8 * q + 2 * t + 1];
      s2 = __builtin_elementwise_fma(fp8x2<false>(lo), f2v{xa.x, xa.y}, s2);
      s2 = __builtin_elementwise_fma(fp8x2<true>(lo), f2v{xa.z, xa.w}, s2);
      s2 = __builtin_elementwise_fma(fp8x2<false>(hi), f2v{xb.x, xb.y}, s2);
      s2 = __builtin_elementwise_fma(fp8x2<true>(hi), f2v{xb.z, xb.w}, s2);
    }
    const float sq = (s2.x + s2.y) * 512.f;
    // sq / 15 correctly rounded without the division sequence: q0 = RN(sq·RN(1/15)) is faithful,
    // the remainder sq − 15·q0 is exact by FMA, and one corrected step RN(q0 + r·RN(1/15)) is the
    // correctly rounded quotient (Markstein); one-hot inputs check it bit for bit
    const float q0 = sq * r15;
    const float rem = __builtin_fmaf(-q0, 15.0f, sq);
    const float quo = __builtin_fmaf(rem, r15, q0);
    a = a + (quo * scale + off * (q ? xs1 : xs0));
  }
  return a;
}

// Q2_K in the stream kernel (gemv_stream_kernel<Q2_K>): the lane's four 16-item sub-blocks
// 4(lane%4) + t of block lane/4, each as kq32_dot_q2k_factored computes it ((Σ q·x)/3·scale +
// min·Σx, :182-196), i/15 from LDS, the quotient by 3 FMA-corrected as for Q4_K.
__device__ float q2k_stream_dot(uint32_t sc, const uint32_t *c, uint32_t dd, const f32x4 *xr, const float *xq,
                                const float *q15) {
#pragma clang fp contract(off)
  const float d = h2f(dd & 0xFFFF), dmin = h2f(dd >> 16);
  constexpr float r3 = 1.0f / 3.0f;
  float a = 0.f;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const uint32_t sm = (sc >> (8 * t)) & 0xFF;  // (sext8(sm) >> 4) & 0x0F == sm >> 4
    const float scale = q15[sm & 0x0F] * d;
    const float mn = (float)(sm >> 4) * d + dmin;
    f2v s2 = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; j++) {  // bit pair j of each byte: items j, 4 + j, 8 + j, 12 + j
      const uint32_t b = (c[t] >> (2 * j)) & 0x03030303u;
      const f32x4 xa = xr[4 * t + j];
      s2 = __builtin_elementwise_fma(fp8x2<false>(b), f2v{xa.x, xa.y}, s2);
      s2 = __builtin_elementwise_fma(fp8x2<true>(b), f2v{xa.z, xa.w}, s2);
    }
    const float sq = (s2.x + s2.y) * 512.f;
    const float q0 = sq * r3;
    const float quo = __builtin_fmaf(__builtin_fmaf(-q0, 3.0f, sq), r3, q0);
    a = a + (quo * scale + mn * xq[t]);
  }
  return a;
}

// Q2_K at batch 1, factored the same way per 16-item sub-block (:182-196): (Σ q·x)/3·scale +
// min·Σx, the 2-bit codes as fp8 conversions against activations ordered (x0,x4,x8,x12 | x1,x5,..)
// per 16; Σx of the two halves in pad slots 32 and 33.
__device__ __forceinline__ float kq32_dot_q2k_factored(const Kq32Raw<LK_TYPE_Q2_K> &r, const KqTables &t, const f32x4 *xv,
                                                       float a) {
#pragma clang fp contract(off)
  const float d = h2f(r.h & 0xFFFF), dmin = h2f(r.h >> 16);
#pragma unroll
  for (int hsb = 0; hsb < 2; hsb++) {
    const int sm = sext8((r.sc >> (8 * hsb)) & 0xFF);
    const float scale = t.q15[sm & 0x0F] * d;
    const float mn = (float)((sm >> 4) & 0x0F) * d + dmin;
    const uint32_t cw = hsb ? r.c1 : r.c0;
    f2v s2 = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; j++) {  // bit pair j of each byte: items j, 4 + j, 8 + j, 12 + j
      const uint32_t b = (cw >> (2 * j)) & 0x03030303u;
      const f32x4 xa = xv[4 * hsb + j];
      s2 = __builtin_elementwise_fma(fp8x2<false>(b), f2v{xa.x, xa.y}, s2);
      s2 = __builtin_elementwise_fma(fp8x2<true>(b), f2v{xa.z, xa.w}, s2);
    }
    const float sq = (s2.x + s2.y) * 512.f;
    const float sx = ((const float *)xv)[32 + hsb];
    a = a + (__fdiv_rn(sq, 3.0f) * scale + mn * sx);
  }
  return a;
}

// Q8_K at batch 1, factored (:404-407): (Σ (q + 128)·x − 128·Σx)·d, the biased bytes converted
// exactly by v_cvt_f32_ubyteN; Σx in pad slot 32. One-hot: (q + 128) − 128 = q, times d: the
// Kotlin weight q·d bit for bit.
__device__ __forceinline__ float kq32_dot_q8k_factored(const Kq32Raw<LK_TYPE_Q8_K> &r, const f32x4 *xv, float a) {
#pragma clang fp contract(off)
  const float d = __builtin_bit_cast(float, r.d);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t u = r.c[j] ^ 0x80808080u;
    const f32x4 x = xv[j];
    s1 = fmaf((float)(u & 0xFF), x.x, s1);  // v_cvt_f32_ubyteN
    s2 = fmaf((float)((u >> 8) & 0xFF), x.y, s2);
    s1 = fmaf((float)((u >> 16) & 0xFF), x.z, s1);
    s2 = fmaf((float)(u >> 24), x.w, s2);
  }
  const float sx = ((const float *)xv)[32];
  const float sq = (s1 + s2) - 128.f * sx;
  return a + sq * d;
}

template <int QT, int ROWS>  // rows (waves) per workgroup
__global__ __launch_bounds__(ROWS * 64) void kquant_n1_kernel(KQuantArgs g) {
  constexpr int BB = KQTraits<QT>::BB, U = 2;
  __shared__ KqTables t;
  extern __shared__ __attribute__((aligned(16))) float xs[];  // (K / 32) x 36 floats
  const int tid = threadIdx.x;
  if (tid < 64) t.q63[tid] = __fdiv_rn((float)tid, 63.0f);
  else if (tid < 80) t.q15[tid - 64] = __fdiv_rn((float)(tid - 64), 15.0f);
  else if (tid < 84) t.q3[tid - 80] = __fdiv_rn((float)(tid - 80), 3.0f);
  // the factored dots' activation order within each 32 (Q4_K: nibble order per 8; Q2_K: bit-pair
  // order per 16; Q8_K: natural), then Σx in the pad: per 32 (Q4_K, Q8_K) or per 16 (Q2_K)
  for (int64_t k = tid; k < g.K; k += ROWS * 64) {
    const int e = (int)(k & 31);
    const int pos = QT == LK_TYPE_Q4_K ? (e & 24) + ((e & 1) ? 4 : 0) + ((e & 7) >> 1)
                    : QT == LK_TYPE_Q2_K ? (e & 16) + (e & 3) * 4 + ((e & 15) >> 2)
                                         : e;
    xs[(k >> 5) * 36 + pos] = *(const float *)(g.b + k * g.b_nb1);
  }
  __syncthreads();
  for (int64_t sbk = tid; sbk < g.K / 32; sbk += ROWS * 64) {
    const f32x4 *v = (const f32x4 *)(xs + sbk * 36);
    const f32x4 h0 = (v[0] + v[1]) + (v[2] + v[3]), h1 = (v[4] + v[5]) + (v[6] + v[7]);
    const float s0 = (h0.x + h0.y) + (h0.z + h0.w), s1 = (h1.x + h1.y) + (h1.z + h1.w);
    if constexpr (QT == LK_TYPE_Q2_K) {
      xs[sbk * 36 + 32] = s0;
      xs[sbk * 36 + 33] = s1;
    } else {
      xs[sbk * 36 + 32] = s0 + s1;
    }
  }
  __syncthreads();
  const int lane = tid & 63;
  const int64_t i = (int64_t)blockIdx.x * ROWS + __builtin_amdgcn_readfirstlane(tid >> 6);
  if (i >= g.M) return;
  const int64_t nb = g.K / LK_QK_K, nch = (nb + 7) / 8;
  const int s = lane & 7;
  const uint8_t *row = g.a + i * nb * BB;
  float acc = 0.f;
  for (int64_t c0 = 0; c0 < nch; c0 += U) {
    Kq32Raw<QT> r[U];
#pragma unroll
    for (int u = 0; u < U; u++)  // block clamped to the row: never summed when past its end
      r[u] = kq32_load<QT>(row + min((c0 + u) * 8 + (lane >> 3), nb - 1) * BB, s);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t blk = (c0 + u) * 8 + (lane >> 3);
      const f32x4 *xv = (const f32x4 *)(xs + (min(blk, nb - 1) * 8 + s) * 36);
      float a;
      if constexpr (QT == LK_TYPE_Q4_K) a = kq32_dot_q4k_factored(r[u], s, t, xv, acc);
      else if constexpr (QT == LK_TYPE_Q2_K) a = kq32_dot_q2k_factored(r[u], t, xv, acc);
      else a = kq32_dot_q8k_factored(r[u], xv, acc);
      acc = blk < nb ? a : acc;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) *(float *)(g.dst + i * g.d_nb1) = acc;
}

// The weights of a lane's 32 items (kq32_dot's formulas and roundings).
template <int QT>
__device__ __forceinline__ void kq32_weights(const Kq32Raw<QT> &r, int s, const KqTables &t, float w[32]) {
#pragma clang fp contract(off)
  if constexpr (QT == LK_TYPE_Q4_K) {
    const float d = h2f(r.h.x & 0xFFFF), dmin = h2f(r.h.x >> 16);
    const int sc = sext8(byte_of(r.h, 4 + s));
    const int qmh = (s * 2 + 1 < LK_K_SCALE_SIZE) ? (sext8(byte_of(r.h, 5 + 2 * s)) & 0x0F) : 0;
    const int qm = ((sc >> 6) & 0x03) | (qmh << 2);
    const float scale = t.q63[sc & 0x3F] * d;
    const float off = t.q63[qm] * d + dmin;
    const uint32_t cw[4] = {r.c.x, r.c.y, r.c.z, r.c.w};
#pragma unroll
    for (int e = 0; e < 32; e++) w[e] = t.q15[(cw[e >> 3] >> (4 * (e & 7))) & 0x0F] * scale + off;
  } else if constexpr (QT == LK_TYPE_Q2_K) {
    const float d = h2f(r.h & 0xFFFF), dmin = h2f(r.h >> 16);
#pragma unroll
    for (int hsb = 0; hsb < 2; hsb++) {
      const int sm = sext8((r.sc >> (8 * hsb)) & 0xFF);
      const float scale = t.q15[sm & 0x0F] * d;
      const float mn = (float)((sm >> 4) & 0x0F) * d + dmin;
      const uint32_t cw = hsb ? r.c1 : r.c0;
#pragma unroll
      for (int e = 0; e < 16; e++) w[16 * hsb + e] = t.q3[(cw >> (8 * (e >> 2) + 2 * (e & 3))) & 0x03] * scale + mn;
    }
  } else {
    const float d = __builtin_bit_cast(float, r.d);
#pragma unroll
    for (int e = 0; e < 32; e++) w[e] = (float)sext8(r.c[e >> 2] >> (8 * (e & 3))) * d;
  }
}

// K-quant x F32 for batch > 1 (K % 256 == 0): kquant_n1_kernel's lane-per-32-items layout with
// NC activation columns staged in LDS per workgroup (column-major, the same 36-per-32 padding),
// each lane's 32 weights decoded once and used for the NC columns. blockIdx.x walks the column
// groups (so the workgroups sharing a row range run together and its weights hit in L2),
// blockIdx.y the groups of 32 rows (two rows per wave: each activation read feeds both). The
// staging reads B(n, k) with n fastest (coalesced for the contiguous [N, K] layout).
template <int QT, int NC, int ROWS>
__global__ __launch_bounds__(ROWS * 64) void kquant_nc_kernel(KQuantArgs g) {
  constexpr int BB = KQTraits<QT>::BB, RPW = 2;  // rows per wave: each x read from LDS feeds both
  __shared__ KqTables t;
  extern __shared__ __attribute__((aligned(16))) float xs[];  // NC x (K / 32) x 36 floats
  const int tid = threadIdx.x;
  if (tid < 64) t.q63[tid] = __fdiv_rn((float)tid, 63.0f);
  else if (tid < 80) t.q15[tid - 64] = __fdiv_rn((float)(tid - 64), 15.0f);
  else if (tid < 84) t.q3[tid - 80] = __fdiv_rn((float)(tid - 80), 3.0f);
  const int64_t j0 = (int64_t)blockIdx.x * NC;
  const int64_t XS = (g.K / 32) * 36;
  for (int64_t idx = tid; idx < g.K * NC; idx += ROWS * 64) {
    const int c = (int)(idx % NC);
    const int64_t k = idx / NC;
    xs[c * XS + (k >> 5) * 36 + (k & 31)] = *(const float *)(g.b + min(j0 + c, g.N - 1) * g.b_nb0 + k * g.b_nb1);
  }
  __syncthreads();
  const int lane = tid & 63;
  const int64_t i0 = ((int64_t)blockIdx.y * ROWS + __builtin_amdgcn_readfirstlane(tid >> 6)) * RPW;
  if (i0 >= g.M) return;
  const int64_t nb = g.K / LK_QK_K, nch = (nb + 7) / 8;
  const int s = lane & 7;
  const uint8_t *rows[RPW];
#pragma unroll
  for (int r = 0; r < RPW; r++) rows[r] = g.a + min(i0 + r, g.M - 1) * nb * BB;  // past M: row M-1, not stored
  float acc[RPW][NC];
#pragma unroll
  for (int r = 0; r < RPW; r++)
#pragma unroll
    for (int c = 0; c < NC; c++) acc[r][c] = 0.f;
  for (int64_t ch = 0; ch < nch; ch++) {
    const int64_t blk = ch * 8 + (lane >> 3);
    const int64_t bc = min(blk, nb - 1);  // clamped: never summed when past the row's end
    Kq32Raw<QT> raw[RPW];
#pragma unroll
    for (int r = 0; r < RPW; r++) raw[r] = kq32_load<QT>(rows[r] + bc * BB, s);
    float w[RPW][32];
#pragma unroll
    for (int r = 0; r < RPW; r++) kq32_weights<QT>(raw[r], s, t, w[r]);
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const f32x4 *xv = (const f32x4 *)(xs + c * XS + (bc * 8 + s) * 36);
      float a[RPW];
#pragma unroll
      for (int r = 0; r < RPW; r++) a[r] = acc[r][c];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const f32x4 v = xv[q];
#pragma unroll
        for (int r = 0; r < RPW; r++) {
          a[r] = fmaf(w[r][4 * q], v.x, a[r]);
          a[r] = fmaf(w[r][4 * q + 1], v.y, a[r]);
          a[r] = fmaf(w[r][4 * q + 2], v.z, a[r]);
          a[r] = fmaf(w[r][4 * q + 3], v.w, a[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < RPW; r++) acc[r][c] = blk < nb ? a[r] : acc[r][c];
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; r++)
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const float sum = wave_sum(acc[r][c]);
      if (lane == 0 && i0 + r < g.M && j0 + c < g.N) *(float *)(g.dst + (j0 + c) * g.d_nb0 + (i0 + r) * g.d_nb1) = sum;
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

// GGUF nibble-order conversion (include/lk_gguf.h), in place, one thread per block.
// Upstream byte j = w[j] | w[j+16] << 4 (ggml-quants.c:1515-1553); llama.kotlin byte
// j = w[2j] | w[2j+1] << 4 (GGMLTypes.kt:647-651). Scale/min bytes are untouched.
// A wave covers 64 consecutive blocks (1152/1280 contiguous bytes): HBM-bound, 2x the
// nibble bytes of traffic per block.
template <int QT, int DIR>
__global__ __launch_bounds__(256) void repack_q4_kernel(uint8_t *__restrict__ blocks, int64_t nblk) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  uint16_t *q = (uint16_t *)(blocks + b * QTraits<QT>::BB + (QT == LK_TYPE_Q4_1 ? 4 : 2));
  uint8_t in[16], o[16];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t v = q[j];
    in[2 * j] = (uint8_t)v;
    in[2 * j + 1] = (uint8_t)(v >> 8);
  }
  if constexpr (DIR == 0) {  // upstream -> kotlin
#pragma unroll
    for (int j = 0; j < 8; j++) {
      o[j] = (uint8_t)((in[2 * j] & 0x0F) | (in[2 * j + 1] << 4));
      o[j + 8] = (uint8_t)((in[2 * j] >> 4) | (in[2 * j + 1] & 0xF0));
    }
  } else {  // kotlin -> upstream: w[j] = nibble (j&1) of byte j>>1
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t lo = (in[j >> 1] >> ((j & 1) * 4)) & 0xF;
      const uint32_t hi = (in[8 + (j >> 1)] >> ((j & 1) * 4)) & 0xF;
      o[j] = (uint8_t)(lo | (hi << 4));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j++) q[j] = (uint16_t)(o[2 * j] | (o[2 * j + 1] << 8));
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

// quantizeTensor again, eight lanes per block: lane l loads elements 4l..4l+3 (a wave reads 8
// consecutive blocks = 1 KB contiguous) and writes its code bytes as 16-bit stores (a wave writes
// its 8 blocks' bytes contiguously); lane 0 of the group writes the f16 header. The block's
// max / min is a butterfly over the 8 lanes: Kotlin's maxOf / minOf fold (NaN-propagating,
// -0.0 < +0.0) is associative and commutative, so the tree gives the fold's value. Every other
// operation is the Kotlin expression with its own rounding (no contraction): bit-identical to
// quantize_kernel. Needs src 16-byte and out 2-byte aligned (the launcher checks).
template <int QT>
__global__ __launch_bounds__(256) void quantize_coop_kernel(const float *__restrict__ src, uint8_t *__restrict__ out, int64_t nblk) {
#pragma clang fp contract(off)
  const int64_t gi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = min(gi >> 3, nblk - 1);  // tail lanes redo the last block (stores guarded)
  const bool live = (gi >> 3) < nblk;
  const int l = threadIdx.x & 7;
  const f32x4 v = *(const f32x4 *)(src + b * 32 + 4 * l);
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint8_t *o = out + b * QTraits<QT>::BB;
  auto bfly = [&](float a, bool is_max) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      const float t = __shfl_xor(a, m, 8);
      a = is_max ? kmax(a, t) : kmin(a, t);
    }
    return a;
  };
  if constexpr (QT == LK_TYPE_Q8_0 || QT == LK_TYPE_Q4_0) {
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 4; e++) amax = kmax(amax, __builtin_fabsf(x[e]));
    amax = bfly(amax, true);
    const float scale = (amax == 0.f) ? 1.f : __fdiv_rn(amax, QT == LK_TYPE_Q8_0 ? 127.f : 8.f);
    const float invS = (QT == LK_TYPE_Q4_0 && scale == 0.f) ? 0.f : __fdiv_rn(1.f, scale);
    if (!live) return;
    if (l == 0) *(uint16_t *)o = kotlin_float_to_half(scale);
    if constexpr (QT == LK_TYPE_Q8_0) {
      uint32_t q[4];
#pragma unroll
      for (int e = 0; e < 4; e++) q[e] = (uint8_t)(int8_t)kround_coerce(x[e] * invS, -128, 127);
      *(uint16_t *)(o + 2 + 4 * l) = (uint16_t)(q[0] | (q[1] << 8));
      *(uint16_t *)(o + 4 + 4 * l) = (uint16_t)(q[2] | (q[3] << 8));
    } else {
      uint32_t q[4];
#pragma unroll
      for (int e = 0; e < 4; e++) q[e] = (uint32_t)kround_coerce(x[e] * invS + 8.f, 0, 15) & 0xF;
      *(uint16_t *)(o + 2 + 2 * l) = (uint16_t)(q[0] | (q[1] << 4) | (q[2] << 8) | (q[3] << 12));
    }
  } else {
    float fmin = x[0], fmax = x[0];
#pragma unroll
    for (int e = 1; e < 4; e++) { fmin = kmin(fmin, x[e]); fmax = kmax(fmax, x[e]); }
    fmin = bfly(fmin, false);
    fmax = bfly(fmax, true);
    float dsc = __fdiv_rn(fmax - fmin, 15.f);
    if (dsc == 0.f) dsc = 1.f;
    const float invD = __fdiv_rn(1.f, dsc);
    if (!live) return;
    if (l == 0) {
      *(uint16_t *)o = kotlin_float_to_half(dsc);
      *(uint16_t *)(o + 2) = kotlin_float_to_half(fmin);
    }
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; e++) q[e] = (uint32_t)kround_coerce((x[e] - fmin) * invD, 0, 15) & 0xF;
    *(uint16_t *)(o + 4 + 2 * l) = (uint16_t)(q[0] | (q[1] << 4) | (q[2] << 8) | (q[3] << 12));
  }
}

// dequantizeTensor, eight lanes per block: lane l reads its 16-bit code words and writes the 4
// values 4l..4l+3 as one 16-byte store (a wave writes 1 KB contiguous). Same roundings as
// dequantize_kernel. Needs blocks 2-byte and out 16-byte aligned (the launcher checks).
template <int QT>
__global__ __launch_bounds__(256) void dequantize_coop_kernel(const uint8_t *__restrict__ src, float *__restrict__ out, int64_t nblk) {
#pragma clang fp contract(off)
  const int64_t gi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = gi >> 3;
  if (b >= nblk) return;
  const int l = threadIdx.x & 7;
  const uint8_t *p = src + b * QTraits<QT>::BB;
  const float d = h2f(*(const uint16_t *)p);
  f32x4 r;
  if constexpr (QT == LK_TYPE_Q8_0) {
    const uint32_t w = (uint32_t) * (const uint16_t *)(p + 2 + 4 * l) | ((uint32_t) * (const uint16_t *)(p + 4 + 4 * l) << 16);
    r.x = d * (float)(int8_t)(w & 0xFF);
    r.y = d * (float)(int8_t)((w >> 8) & 0xFF);
    r.z = d * (float)(int8_t)((w >> 16) & 0xFF);
    r.w = d * (float)(int8_t)(w >> 24);
  } else if constexpr (QT == LK_TYPE_Q4_0) {
    const uint32_t w = *(const uint16_t *)(p + 2 + 2 * l);
    r.x = d * ((float)(w & 0xF) - 8.0f);
    r.y = d * ((float)((w >> 4) & 0xF) - 8.0f);
    r.z = d * ((float)((w >> 8) & 0xF) - 8.0f);
    r.w = d * ((float)(w >> 12) - 8.0f);
  } else {
    const float m = h2f(*(const uint16_t *)(p + 2));
    const uint32_t w = *(const uint16_t *)(p + 4 + 2 * l);
    r.x = d * (float)(w & 0xF) + m;
    r.y = d * (float)((w >> 4) & 0xF) + m;
    r.z = d * (float)((w >> 8) & 0xF) + m;
    r.w = d * (float)(w >> 12) + m;
  }
  *(f32x4 *)(out + b * 32 + 4 * l) = r;
}

// ---- direct dot products (computeDotProduct{F32Q41, F32Q80, Q80Q80, Q40Q40, Q41Q41, Q80Q40},
// GGMLComputeOps.kt:349-629) ----------------------------------------------------------------
// One thread per (row, col), k in order, every element / product / sum the Kotlin expression
// with explicit roundings: bit-identical to the reference arithmetic. Dead code in the
// reference (not reachable from computeMatMul): correctness, not speed, is the point; lanes
// of a wave share the row (A reads broadcast) and take consecutive columns (B reads coalesce).
struct DotArgs {
  const uint8_t *a, *b;  // buffer base + dataOffset
  float *out;            // [M][N]
  int64_t M, N, K;
  int64_t a_nb0, a_nb1;  // F32 A (getFloat(k, row) honours nb)
};

// Q element at a flat index: Q8_0 d·q, Q4_0 d·(n − 8), Q4_1 d·n + m (accessor order). Plain
// operators under contract(off): __fmul_rn / __fadd_rn carry the header's own contraction
// flags and were seen fused into an FMA once inlined next to an add.
template <int QT> __device__ __forceinline__ float q_elem(const uint8_t *base, int64_t flat) {
#pragma clang fp contract(off)
  const uint8_t *p = base + (flat >> 5) * QTraits<QT>::BB;
  const int item = (int)(flat & 31);
  const float d = h2f(ld_u16(p));
  if constexpr (QT == LK_TYPE_Q8_0) {
    return d * (float)(int32_t)(int8_t)ld_u8(p + 2 + item);
  } else if constexpr (QT == LK_TYPE_Q4_1) {
    const float m = h2f(ld_u16(p + 2));
    const uint32_t byte = ld_u8(p + 4 + (item >> 1));
    const float dq = d * (float)((item & 1) ? (byte >> 4) : (byte & 0xF));
    return dq + m;
  } else {
    const uint32_t byte = ld_u8(p + 2 + (item >> 1));
    const float qm = (float)((item & 1) ? (byte >> 4) : (byte & 0xF)) - 8.0f;
    return d * qm;
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void dot_direct_kernel(DotArgs g) {
#pragma clang fp contract(off)
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= g.M * g.N) return;
  const int64_t i = idx / g.N, j = idx % g.N;
  float sum = 0.f;
  for (int64_t k = 0; k < g.K; k++) {
    const int64_t fb = k * g.N + j;
    float p;
    if constexpr (KIND == LK_DOT_F32_Q4_1 || KIND == LK_DOT_F32_Q8_0) {
      const float f = *(const float *)(g.a + k * g.a_nb0 + i * g.a_nb1);
      const float w = q_elem<KIND == LK_DOT_F32_Q4_1 ? LK_TYPE_Q4_1 : LK_TYPE_Q8_0>(g.b, fb);
      p = f * w;
    } else if constexpr (KIND == LK_DOT_Q8_0_Q8_0) {  // (dA·dB)·(qA·qB)
      const int64_t fa = i * g.K + k;
      const uint8_t *pa = g.a + (fa >> 5) * 34, *pb = g.b + (fb >> 5) * 34;
      const float s2 = h2f(ld_u16(pa)) * h2f(ld_u16(pb));
      const float q2 = (float)(int32_t)(int8_t)ld_u8(pa + 2 + (int)(fa & 31)) * (float)(int32_t)(int8_t)ld_u8(pb + 2 + (int)(fb & 31));
      p = s2 * q2;
    } else {
      constexpr int TA = KIND == LK_DOT_Q4_1_Q4_1 ? LK_TYPE_Q4_1 : KIND == LK_DOT_Q8_0_Q4_0 ? LK_TYPE_Q8_0 : LK_TYPE_Q4_0;
      constexpr int TB = KIND == LK_DOT_Q4_1_Q4_1 ? LK_TYPE_Q4_1 : LK_TYPE_Q4_0;
      const float wa = q_elem<TA>(g.a, i * g.K + k);
      const float wb = q_elem<TB>(g.b, fb);
      p = wa * wb;
    }
    sum = sum + p;
  }
  g.out[idx] = sum;
}

}  // namespace lk
