// lk_mfma32.hpp — Q4_0 / Q4_1 x F32 at batch 17..32 on v_mfma_f32_32x32x16_bf16 (gfx950).
//
// computeMatMul (core/GGMLComputeOps.kt:1448-1480) for C3's batch-32 shapes. HBM-bound: a Q4_0
// weight byte feeds 114 flops at N = 32, so the design goal is the weight stream, with the
// per-block dequantization kept off the critical path.
//
// Operands of one MFMA: A = activations (32 x-columns n x 16 k), B = decoded weights (16 k x 32
// weight rows m), C[n][m]. Each lane's 16 accumulators then belong to ONE weight row
// (m = lane & 31), so a block's scale d is one scalar per lane: 16 FMAs per block and 32 rows.
//
// Exact operands:
//  - a weight nibble n (0..15) becomes the bf16 integer n with one v_cvt_scalef32_pk_bf16_fp8
//    per two weights: the masked byte 0000nnnn read as OCP e4m3 is n·2^-9, scaled by 2^9;
//  - x = hi + lo (bf16 each, |x - hi - lo| <= 2^-17 |x|): two MFMAs per product;
//  - the offset of each block (Q4_0: -8·d, Q4_1: m) multiplies S_b[n] = Σ_{k in b} x̃[n][k]
//    (x̃ = hi + lo): Σ_b c_b[m] · S_b[n] is one more 32x32x16 contraction over the slice's
//    blocks, with S split in three bf16 parts and c (an f16 value) in two — 5 MFMAs per 8
//    blocks, products exact, f32 sums.
// So dst = Σ_b d_b·Σ_k n_k x̃_k + Σ_b c_b S_b = Σ_k w_k x̃_k up to f32 summation order.
//
// Lanes and k: lane (r = lane & 31, h = lane >> 5) holds k = 8h + j (j = 0..7) of each 16-k
// MFMA step. Step s of block b takes the block's code bytes 8s..8s+7; lane half h takes nibble
// h of each of them, so element j is weight 16s + 2j + h. Both lane halves read the SAME code
// dwords (only the shift differs), and the activation fragments use the same k order.
//
// Work: split K in slices of 16 blocks (x of a slice, 32 columns x 512 k, is held by every wave
// in 256 VGPRs as bf16 hi / lo fragments), rows in tiles of 32; a workgroup = one slice x a
// range of tiles, 4 waves (one per SIMD), wave w takes tiles w, w + 4, ... A unit = one tile's
// 8 blocks (32 rows x 144 / 160 B), streamed by LDS-DMA through a ring of D units per wave. The
// activation staging area of the prologue (raw x by LDS-DMA, then the bf16 fragments and the
// Σx partials) becomes DB more ring slots once every wave holds its fragments. Each slice
// stores an f32 partial [slice][M][32]; splitk_reduce_kernel adds them in slice order.
#pragma once

#include "lk_kernels.hpp"

// lab knobs (A/B builds only; the defaults are the product)
#ifndef LK_Q32_NT
#define LK_Q32_NT 0         // weight DMA cache policy: 0 default (the 128-B lines a unit shares with the
#endif                      // tile's other unit and the neighbouring slice stay in L2), 1 nt
#ifndef LK_Q32_SKELETON
#define LK_Q32_SKELETON 0   // 1: the DMA / LDS skeleton without the decode and MFMAs (wrong results)
#endif

namespace lk {

struct Q32Args {
  const uint8_t *a;          // weights (buffer base + dataOffset), rows RB bytes apart
  const uint8_t *b;          // activations: B(n, k) at 4n + 4N·k (dense, 16-B aligned)
  float *partial;            // [slices][M][32] when slices > 1
  uint8_t *dst;              // slices == 1: dst(n, m) at n·d_nb0 + m·d_nb1
  int64_t d_nb0, d_nb1;
  int32_t M, N, K;
  int32_t slices, tiles_per_range, tasks;
};

template <int QT> struct Q32Geom {
  static constexpr int BB = QTraits<QT>::BB;
  static constexpr int NW = 4;                             // waves: one per SIMD
  static constexpr int SB = 16, HB = 8;                    // blocks per slice / per unit
  static constexpr int UCELLS = HB * BB / 16;              // 16-B cells of one unit row: 9 / 10
  static constexpr int P = (UCELLS & 1) ? UCELLS : UCELLS + 1;  // row pitch in cells: odd, so the
                                                           // 16 rows of a ds_read_b128 group hit 16 bank quads
  static constexpr int SLOT = 32 * P * 16;                 // 4,608 / 5,632 B
  static constexpr int L = (32 * P + 63) / 64;             // DMA instructions per unit: 5 / 6
  static constexpr int XF = SB * 2 * 2 * 1024;             // fragments: block x step x (hi, lo), 1 KB each
  static constexpr int SPB = SB * 2 * 2 * 32 * 4;          // Σx partials [block][step][h][n]
  static constexpr int STAGE = XF + SPB;                   // 72 KB (raw x, 64 KB, first; then fragments)
  static constexpr int DA = (kLdsBytes - STAGE) / (NW * SLOT);  // ring slots beside the staging area
  static constexpr int DB = STAGE / (NW * SLOT);                // ring slots inside it (after the prologue)
  static constexpr int D = DA + DB;
  static constexpr int LDS = STAGE + NW * DA * SLOT;
  static_assert(UCELLS * 16 == HB * BB, "unit rows are whole 16-B cells");
  static_assert(DA >= 2 && LDS <= kLdsBytes, "LDS");
};

// lab: per-wave timeline (tools/lab/q32_trace.hip defines LK_Q32_TRACE): s_memrealtime at kernel
// entry, activations landed, fragments held, first unit landed, loop done, exit
#ifdef LK_Q32_TRACE
__device__ uint64_t *lk_qtrace_buf;
#define LK_QTRACE(slot)                                                                                  \
  do {                                                                                                   \
    uint64_t *tb_ = (uint64_t *)((const __attribute__((address_space(4))) uint64_t *)&lk_qtrace_buf)[0]; \
    if (lane == 0 && tb_) tb_[((size_t)blockIdx.x * 4 + wave) * 6 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LK_QTRACE(slot) do {} while (0)
#endif

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t bf16pair_trunc(float lo, float hi) {  // high halves of two floats
  return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07060302u);
}
__device__ __forceinline__ float trunc_bf16(float x) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFF0000u);
}
// bf16 integer pair fragment dwords of code dword cw for lane half h (shift sh = 4h)
__device__ __forceinline__ void nib_frag(uint32_t cw, uint32_t sh, uint32_t &f0, uint32_t &f1) {
  const uint32_t v = (cw >> sh) & 0x0F0F0F0Fu;
  f0 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 512.f, false));
  f1 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 512.f, true));
}

__device__ __forceinline__ f32x16 mfma32(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// One unit (8 blocks of the held slice, H2 = which half) against the row piece dw (lane's
// weight row): acc += Σ_b d_b · P_b, then the offset term of the 8 blocks.
template <int QT, int H2, int NDW>
__device__ __forceinline__ void q32_unit(const uint32_t (&dw)[NDW], uint32_t sh, const u32x4 (&xh)[16][2],
                                         const u32x4 (&xl)[16][2], const u32x4 (&sf)[2][3], f32x16 &acc) {
  float c[8];
#pragma unroll
  for (int b = 0; b < 8; b++) {
    float d;
    uint32_t cw[4];
    if constexpr (QT == LK_TYPE_Q4_0) {
      const int o = 18 * b;  // compile time after unrolling
      const uint32_t dword = (o & 3) ? dw[o / 4] >> 16 : dw[o / 4];
      d = h2f(dword & 0xFFFFu);
      c[b] = -8.f * d;
      // code bytes at o + 2 .. o + 17
      if ((o & 3) == 0) {  // codes start 2 bytes into a dword
#pragma unroll
        for (int q = 0; q < 4; q++) cw[q] = __builtin_amdgcn_alignbyte(dw[o / 4 + q + 1], dw[o / 4 + q], 2);
      } else {             // o % 4 == 2: codes dword-aligned
#pragma unroll
        for (int q = 0; q < 4; q++) cw[q] = dw[(o + 2) / 4 + q];
      }
    } else {  // Q4_1: (d, m) dword, codes dword-aligned
      const uint32_t dm = dw[5 * b];
      d = h2f(dm & 0xFFFFu);
      c[b] = h2f(dm >> 16);
#pragma unroll
      for (int q = 0; q < 4; q++) cw[q] = dw[5 * b + 1 + q];
    }
    uint32_t f[8];
    nib_frag(cw[0], sh, f[0], f[1]);
    nib_frag(cw[1], sh, f[2], f[3]);
    nib_frag(cw[2], sh, f[4], f[5]);
    nib_frag(cw[3], sh, f[6], f[7]);
    const u32x4 w0 = {f[0], f[1], f[2], f[3]}, w1 = {f[4], f[5], f[6], f[7]};
    f32x16 p = {};
    p = mfma32(xh[8 * H2 + b][0], w0, p);
    p = mfma32(xl[8 * H2 + b][0], w0, p);
    p = mfma32(xh[8 * H2 + b][1], w1, p);
    p = mfma32(xl[8 * H2 + b][1], w1, p);
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = __builtin_fmaf(d, p[i], acc[i]);
  }
  // offset term: B[k = 8h + j][m] = c_j (both lane halves; A is zero in the h = 1 half)
  u32x4 c0, c1;
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = c[j] - trunc_bf16(c[j]);  // exact: c is an f16 value
  c0.x = bf16pair_trunc(c[0], c[1]); c0.y = bf16pair_trunc(c[2], c[3]);
  c0.z = bf16pair_trunc(c[4], c[5]); c0.w = bf16pair_trunc(c[6], c[7]);
  c1.x = bf16pair_trunc(r[0], r[1]); c1.y = bf16pair_trunc(r[2], r[3]);
  c1.z = bf16pair_trunc(r[4], r[5]); c1.w = bf16pair_trunc(r[6], r[7]);
  acc = mfma32(sf[H2][0], c0, acc);
  acc = mfma32(sf[H2][0], c1, acc);
  acc = mfma32(sf[H2][1], c0, acc);
  acc = mfma32(sf[H2][1], c1, acc);
  acc = mfma32(sf[H2][2], c0, acc);
}

template <int QT>
__global__ __launch_bounds__(256) void gemm_q32_kernel(Q32Args g) {
  using G = Q32Geom<QT>;
  constexpr int D = G::D, DA = G::DA, L = G::L, P = G::P, NW = G::NW;
  constexpr int NDW = 4 * G::UCELLS;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;  // XCD-aware
  if (task >= g.tasks) return;  // grid padding: the whole workgroup leaves before any barrier
  LK_QTRACE(0);
  const int slice = task % g.slices, range = task / g.slices;
  const int nblk = g.K / 32, kb0 = slice * G::SB, nb = min(G::SB, nblk - kb0);  // nb = 8 or 16
  const int upt = nb / G::HB;                                                   // units per tile
  const int64_t RB = (int64_t)nblk * G::BB;
  const int ntile = (g.M + 31) / 32;
  const int t0 = range * g.tiles_per_range, t1 = min(t0 + g.tiles_per_range, ntile);
  const int ntw = t1 - t0 - wave > 0 ? (t1 - t0 - wave + NW - 1) / NW : 0;  // this wave's tiles
  const int nunits = ntw * upt;
  auto slot_ptr = [&](int s) -> uint8_t * {
    return s < DA ? smem + G::STAGE + (wave * DA + s) * G::SLOT : smem + (wave * G::DB + (s - DA)) * G::SLOT;
  };
  // unit u: tile t0 + wave + NW·(u / upt), blocks kb0 + 8·(u % upt) .. + 8 of each of its 32 rows;
  // LDS position p = r·P + c holds cell c of row r (c >= UCELLS: padding, re-reads cell 0)
  uint32_t cofs[L];
  int crow[L];
  bool cok[L];
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int p = j * 64 + lane, r = p / P, c = p % P;
    crow[j] = r;
    cofs[j] = (uint32_t)((c < G::UCELLS ? c : 0) * 16);
    cok[j] = p < 32 * P;
  }
  auto issue = [&](int u, int s) __attribute__((always_inline)) {
    const int t = t0 + wave + NW * (u / upt);
    const uint8_t *base = g.a + (int64_t)t * 32 * RB + (int64_t)(kb0 + G::HB * (u % upt)) * G::BB;
    const int rmax = g.M - 1 - t * 32;
    uint8_t *sp = slot_ptr(s);
#pragma unroll
    for (int j = 0; j < L; j++)
      if (cok[j]) dma16<LK_Q32_NT != 0>(base, (uint32_t)(min(crow[j], rmax) * RB) + cofs[j], sp + j * 1024);
  };

  // 1. raw activations of the slice by LDS-DMA: rows k of B are 4N contiguous bytes
  const int xbytes = nb * 32 * 4 * g.N;
  const int xinst = (xbytes + 1023) / 1024;
  int myx = 0;
  for (int j = wave; j < xinst; j += NW, myx++) {
    const int off = j * 1024 + lane * 16;
    if (off < xbytes) dma16<false>(g.b + (int64_t)kb0 * 32 * 4 * g.N, (uint32_t)off, smem + j * 1024);
  }
  // 2. the first DA units of the weight ring (beside the staging area)
  const int na = min(DA, nunits);
  for (int u = 0; u < na; u++) issue(u, u);
  wait_vmcnt_rt<DA * L>(na * L);  // this wave's activation pieces have landed
  __builtin_amdgcn_s_barrier();
  LK_QTRACE(1);
  // 3. convert: slot q = (block bb, step s, half h, column n) -> 8 values k = 32bb + 16s + 2j + h
  float v[8][8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int q = tid + 256 * i, n = q & 31, h = (q >> 5) & 1, s = (q >> 6) & 1, bb = q >> 7;
    const bool ok = n < g.N && bb < nb;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int k = 32 * bb + 16 * s + 2 * j + h;
      v[i][j] = ok ? *(const float *)(smem + ((int64_t)k * g.N + n) * 4) : 0.f;
    }
  }
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();  // every raw value is in registers: the area becomes fragments
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int q = tid + 256 * i, n = q & 31, h = (q >> 5) & 1, s = (q >> 6) & 1, bb = q >> 7;
    float hi[8], lo[8], ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      hi[j] = trunc_bf16(v[i][j]);
      lo[j] = (float)(__bf16)(v[i][j] - hi[j]);
      ps += hi[j] + lo[j];
    }
    u32x4 fh, fl;
    fh.x = bf16pair_trunc(hi[0], hi[1]); fh.y = bf16pair_trunc(hi[2], hi[3]);
    fh.z = bf16pair_trunc(hi[4], hi[5]); fh.w = bf16pair_trunc(hi[6], hi[7]);
    fl.x = bf16pair_trunc(lo[0], lo[1]); fl.y = bf16pair_trunc(lo[2], lo[3]);
    fl.z = bf16pair_trunc(lo[4], lo[5]); fl.w = bf16pair_trunc(lo[6], lo[7]);
    u32x4 *fr = (u32x4 *)(smem + ((bb * 2 + s) * 2) * 1024) + (n + 32 * h);
    fr[0] = fh;
    fr[64] = fl;
    ((float *)(smem + G::XF))[((bb * 2 + s) * 2 + h) * 32 + n] = ps;
  }
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();
  // 4. every wave holds the slice: x fragments, and S_b[n] split in three bf16 parts as the A
  //    operand of the offset term (unit half H2: lanes h = 0 hold blocks 8·H2 + j, h = 1 zeros)
  u32x4 xh[16][2], xl[16][2];
#pragma unroll
  for (int bb = 0; bb < 16; bb++)
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const u32x4 *fr = (const u32x4 *)(smem + ((bb * 2 + s) * 2) * 1024) + lane;
      xh[bb][s] = fr[0];
      xl[bb][s] = fr[64];
    }
  u32x4 sf[2][3];
  {
    const int n = lane & 31;
    const bool h0 = lane < 32;
    const float *sp = (const float *)(smem + G::XF);
#pragma unroll
    for (int H2 = 0; H2 < 2; H2++) {
      float s0[8], s1[8], s2[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int bb = 8 * H2 + j;
        float S = 0.f;
#pragma unroll
        for (int e = 0; e < 4; e++) S += sp[(bb * 4 + e) * 32 + n];
        S = h0 ? S : 0.f;
        s0[j] = trunc_bf16(S);
        const float r1 = S - s0[j];
        s1[j] = trunc_bf16(r1);
        s2[j] = (float)(__bf16)(r1 - s1[j]);
      }
      sf[H2][0] = u32x4{bf16pair_trunc(s0[0], s0[1]), bf16pair_trunc(s0[2], s0[3]), bf16pair_trunc(s0[4], s0[5]),
                        bf16pair_trunc(s0[6], s0[7])};
      sf[H2][1] = u32x4{bf16pair_trunc(s1[0], s1[1]), bf16pair_trunc(s1[2], s1[3]), bf16pair_trunc(s1[4], s1[5]),
                        bf16pair_trunc(s1[6], s1[7])};
      sf[H2][2] = u32x4{bf16pair_trunc(s2[0], s2[1]), bf16pair_trunc(s2[2], s2[3]), bf16pair_trunc(s2[4], s2[5]),
                        bf16pair_trunc(s2[6], s2[7])};
    }
  }
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();  // the staging area is free: the rest of the ring
  for (int u = na; u < min(D, nunits); u++) issue(u, u);
  LK_QTRACE(2);

  // 5. main loop
  const uint32_t sh = (uint32_t)(lane >> 5) * 4;
  const int m_lane = lane & 31;
  f32x16 acc = {};
  for (int u = 0; u < nunits; u++) {
    const int s = u % D, h2 = u % upt;
    // DMA instructions younger than this unit's: the units issued after it. Stores issued since
    // are younger too; not counting them only makes the wait stricter (a masked-off wave may
    // skip its stores, so counting them could make it too loose).
    wait_vmcnt_rt<L * (D - 1)>(L * (min(u + D - 1, nunits - 1) - u));
    asm volatile("" ::: "memory");
    if (u == 0) LK_QTRACE(3);
    uint32_t dw[NDW];
    {
      const u32x4 *rp = (const u32x4 *)(slot_ptr(s) + m_lane * P * 16);
#pragma unroll
      for (int c = 0; c < G::UCELLS; c++) {
        const u32x4 t4 = rp[c];
        dw[4 * c] = t4.x; dw[4 * c + 1] = t4.y; dw[4 * c + 2] = t4.z; dw[4 * c + 3] = t4.w;
      }
    }
    wait_lgkmcnt0();  // the slot's reads have landed: the DMA may refill it
    if (u + D < nunits) issue(u + D, s);
    if (h2 == 0) acc = f32x16{};
#if LK_Q32_SKELETON
    acc[0] += __builtin_bit_cast(float, dw[0] ^ dw[NDW - 1]);
#else
    if (h2 == 0) q32_unit<QT, 0>(dw, sh, xh, xl, sf, acc);
    else q32_unit<QT, 1>(dw, sh, xh, xl, sf, acc);
#endif
    if (h2 == upt - 1) {
      const int t = t0 + wave + NW * (u / upt);
      const int64_t m = (int64_t)t * 32 + m_lane;
      const int hh = lane >> 5;
      if (g.slices > 1) {
        float *pr = g.partial + ((int64_t)slice * g.M + m) * 32 + 4 * hh;
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (m < g.M) *(f32x4 *)(pr + 8 * q) = f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
      } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
          const int n = (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (m < g.M && n < g.N) *(float *)(g.dst + m * g.d_nb1 + n * g.d_nb0) = acc[i];
        }
      }
    }
  }
  LK_QTRACE(4);
  wait_vmcnt<0>();
  LK_QTRACE(5);
}

}  // namespace lk
