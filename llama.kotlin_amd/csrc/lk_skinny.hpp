// lk_skinny.hpp — gemm_sk_kernel: Q4_K x F32 at 16 <= N <= 32 on gfx950 (wave-pair MFMA).
//
// computeMatMul's Q4_K branch (core/GGMLComputeOps.kt:1483-1514, dot :241-310) for a few
// activation columns, on v_mfma_f32_16x16x32_bf16. Since round 3 the kernel is instantiated for
// Q4_K only (Q4_0 / Q4_1 run on gemm_skinny_pair_kernel, lk_kernels.hpp, which was faster for
// them). Arithmetic:
//
//  * Activations as bf16 hi + lo (|x − hi − lo| ≤ 2⁻¹⁷|x|), in MFMA operand fragments, plus
//    S = Σ(hi + lo) per (sub-block, column). Dense 16-byte-aligned activations (fx) are split by
//    the kernel itself: the slice's raw rows land in LDS by LDS-DMA and each wave splits its items
//    in place; other layouts come from xsplit_kernel (one extra launch).
//  * Codes as the exact bf16 128 + n, two per v_and_or_b32: (u & 0x000F000F) | 0x43004300, k order
//    0,4,1,5,2,6,3,7 (the order the split writes the activations in). The MFMA gives
//    p = Σ (128 + n)·x per 32-weight sub-block.
//  * Per sub-block: acc += s1·p (packed f32 FMAs), s1 = qs·d/945 — the affine form q·s1 + min of
//    the Kotlin (q/15)·scale + min. The offsets fold into one f32 term per sub-block,
//    e·S with e = min − 128·s1, summed over a wave's 8 sub-blocks by two v_mfma_f32_16x16x4_f32
//    per 16-column tile (exact f32 products) straight into the accumulators.
//
// Schedule: workgroup = (row range, K slice of 16 sub-blocks = two Q4_K blocks), 8 waves; wave
// (stream p = w % 4, half h = w / 4) streams 16-row tiles t0 + p + 4i, its half's Q4_K block of
// each row through its own LDS-DMA ring. The h = 1 wave (issue priority 1) hands its accumulators
// to its partner through LDS (ready / ack flags, 2 parities); the h = 0 wave adds them one unit
// later, in a fixed order, and stores a partial slab per slice; the last slice to store a tile sums
// its slabs in slice order (splitk_tiles_fixup, lk_kernels.hpp: deterministic, nobody waits).
#pragma once

#include "lk_kernels.hpp"

namespace lk {


// Bytes per 32 weights: Q4_0 18, Q4_1 20, and Q4_K 18 (a 144-byte block of 256 weights: d, dmin,
// 12 scale bytes, 128 code bytes; core/GGMLComputeOps.kt:241-310). For Q4_K a "block" here is
// one 32-weight sub-block (one MFMA step), and a wave's 8 blocks are exactly one Q4_K block.
template <int QT> struct SkBB { static constexpr int v = QT == LK_TYPE_Q4_1 ? 20 : 18; };

template <int QT, int NT> struct SkGeom {
  static constexpr int NW = 8;                          // 4 streams x 2 halves
  static constexpr int BB = SkBB<QT>::v;
  static constexpr int SB = 16, SBH = 8;                // blocks per slice / per half
  static constexpr int RPH = SBH * BB;                  // bytes of a half row piece (144 / 160)
  static constexpr int PPH = RPH / 16;                  // 16-B cells per half row
  static constexpr int L = (16 * PPH + 63) / 64;        // DMA instructions per half unit
  static constexpr int WPB = QT == LK_TYPE_Q4_K ? 1 : QT == LK_TYPE_Q4_1 ? 2 : 3;
  static constexpr int SLOT = L * 1024;
  static constexpr int XI = SB * NT * kXSplits;         // 1-KB activation fragments of the slice
  static constexpr int XF = XI * 1024;
  static constexpr int TB = SB * 16 * NT * 4;           // S = Σx per (block, column)
  static constexpr int TI = TB / 1024;                  // its DMA instructions
  static constexpr int EB = 2 * 4 * NT * 64 * 16;       // accumulator hand-off, 2 parities x 4 pairs
  static constexpr int FB = 64;                         // ready[4][2], ack[4] (ints)
  static constexpr int DFIT = (kLdsBytes - XF - TB - EB - FB) / (NW * SLOT);
  static constexpr int D = DFIT > 4 ? 4 : DFIT;         // ring depth (half units per wave)
  static constexpr int LDS = XF + TB + EB + FB + NW * D * SLOT;
  static constexpr int MAXW = L * (D - 1) + D * NT;     // largest vmcnt a wait needs
  static_assert(RPH % 16 == 0, "half row pieces");
  static_assert(TB % 1024 == 0, "T DMA");
  static_assert(D >= 2, "ring must double-buffer");
  static_assert(LDS <= kLdsBytes, "LDS");
  static_assert(MAXW < 64, "vmcnt");
};

struct SkArgs {
  const uint8_t *a;        // weights (buffer base + dataOffset), rows RB bytes apart
  const u32x4 *frag;       // xsplit_kernel fragments [ntx][nblk][2][64] (fx == 0)
  const float *xsum;       // [nblk][16·ntx]: Σ(hi + lo) per (block, column) (fx == 0)
  const uint8_t *b;        // fx == 1: dense B (k-major rows of N floats, 16-B aligned), split in-kernel
  int32_t fx;
  uint8_t *dst;            // dst(n, m) at n·d_nb0 + m·d_nb1
  int64_t d_nb0, d_nb1;
  float *partial;          // [slices][M][16·NT] when slices > 1
  int32_t M, N, K;
  int32_t slices, tiles_per_range, tasks;  // tasks = ranges·slices (the grid is padded to 8)
  unsigned *rsync;         // gemm_sk_kernel: fused split-K reduction (SkinnyArgs::rsync), or null
};

// LDS-typed pointers throughout (no generic -> LDS conversions, no null checks on them).
typedef LK_LDS uint8_t lu8;

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// dma16 (lk_kernels.hpp) with the LDS destination as an LDS pointer: M0 is its 32-bit offset.
template <bool NT>
__device__ __forceinline__ void dma16l(const void *sbase, uint32_t vofs, const lu8 *lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst);
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  const uint32_t sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  sbase = (const void *)(((uint64_t)sb_hi << 32) | (uint64_t)sb_lo);
  if constexpr (NT) asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1 nt" ::"v"(vofs), "s"(sbase), "s"(m0) : "memory", "m0");
  else asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(vofs), "s"(sbase), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop
__device__ __forceinline__ int ldsl_ld(const LK_LDS int *p) {
  asm volatile("" ::: "memory");
  const int v = *(volatile const LK_LDS int *)p;
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void ldsl_st(LK_LDS int *p, int v) {
  asm volatile("" ::: "memory");
  *(volatile LK_LDS int *)p = v;
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ uint32_t lds32(const lu8 *p) { return *(const LK_LDS uint32_t *)p; }

// The WPB dwords of block B for lane (row m = lane & 15, group g = lane >> 4): bm = slot + m·RPH,
// bg = bm + 4g (as skinny_read in lk_kernels.hpp).
template <int QT, int B, int WPB>
__device__ __forceinline__ void sk_read(const lu8 *bm, const lu8 *bg, uint32_t (&w)[WPB]) {
  constexpr int OB = B * SkBB<QT>::v;
  if constexpr (QT == LK_TYPE_Q4_K) {  // sub-block B's 16 code bytes at 16 + 16B; lane group g: 4 of them
    w[0] = lds32(bg + 16 + 16 * B);
  } else if constexpr (QT == LK_TYPE_Q4_1) {  // (d, m) dword; codes at +4 + 4g
    w[0] = lds32(bm + OB);
    w[1] = lds32(bg + OB + 4);
  } else if constexpr ((OB & 3) == 0) {  // d lo; codes at +2 + 4g: two dwords, realigned by 2
    w[0] = lds32(bm + OB);
    w[1] = lds32(bg + OB);
    w[2] = lds32(bg + OB + 4);
  } else {  // d in the high half of the dword before; codes aligned
    w[0] = lds32(bm + OB - 2);
    w[1] = lds32(bg + OB + 2);
    w[2] = 0;
  }
}
template <int QT, int WPB, int B, int NBW>
__device__ __forceinline__ void sk_read_all(const lu8 *bm, const lu8 *bg, uint32_t (&w)[NBW][WPB]) {
  if constexpr (B < NBW) {
    sk_read<QT, B, WPB>(bm, bg, w[B]);
    sk_read_all<QT, WPB, B + 1, NBW>(bm, bg, w);
  }
}

// Q4_K block header of the lane's row (per unit): h = its first 16 bytes (d, dmin, 12 scale
// bytes), dk = d/945 (= d/63/15). Sub-block sb's weights are w = (q/15)·scale + min with
// scale = (qs/63)·d, min = (qm/63)·d + dmin (:285-286, :298): here as the affine q·s1 + min with
// s1 = qs·dk — the same values up to the f32 rounding of the Kotlin expression order (the
// batch-1 kernel keeps the Kotlin order bit for bit; this MFMA path is within the F32 bar).
struct SkHdr {
  uint32_t h[4];
  float dk, d63, dmin;
};

// Block B of a unit: codes + scale d from its dwords, 2·NT MFMAs into p.
template <int QT, int NT, int B, int WPB, int NBW>
__device__ __forceinline__ void sk_mfma(const uint32_t (&w)[WPB], const u32x4 (&xh)[NBW][NT], const u32x4 (&xl)[NBW][NT],
                                        f32x4 (&p)[NT], float &s1, const SkHdr &hd) {
  constexpr int OB = B * SkBB<QT>::v;
  bf16x8 wf;
  if constexpr (QT == LK_TYPE_Q4_K) {
    wf = q4_codes_128(w[0]);
    s1 = (float)((hd.h[1 + B / 4] >> (8 * (B % 4))) & 0x3Fu) * hd.dk;
  } else if constexpr (QT == LK_TYPE_Q4_1) {
    wf = q4_codes_128(w[1]);
    s1 = h2f(w[0]);
  } else if constexpr ((OB & 3) == 0) {
    wf = q4_codes_128(align2(w[2], w[1]));
    s1 = h2f(w[0]);
  } else {
    wf = q4_codes_128(w[1]);
    s1 = h2f(w[0] >> 16);
  }
#pragma unroll
  for (int j = 0; j < NT; j++)
    p[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xl[B][j]), wf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < NT; j++)
    p[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xh[B][j]), wf, p[j], 0, 0, 0);
}

// acc += d·p as packed FMAs (two per tile: a wave64 v_pk_fma_f32 issues as fast as a v_fma_f32).
// Masked blocks (past a short slice) have zero activation fragments, so p == 0; d is zeroed
// too, since the slot bytes there are stale (d may be inf / NaN).
template <int NT, int B, bool MASK>
__device__ __forceinline__ void sk_scale(const f32x4 (&p)[NT], float s1, int nb, f32x4 (&acc)[NT]) {
  if (MASK && B >= nb) s1 = 0.f;
  const f2v m1 = {s1, s1};
#pragma unroll
  for (int j = 0; j < NT; j++) {
    const f2v a0 = __builtin_elementwise_fma(m1, f2v{p[j].x, p[j].y}, f2v{acc[j].x, acc[j].y});
    const f2v a1 = __builtin_elementwise_fma(m1, f2v{p[j].z, p[j].w}, f2v{acc[j].z, acc[j].w});
    acc[j] = f32x4{a0.x, a0.y, a1.x, a1.y};
  }
}

// Scheduling hint for a unit's block section (one basic block): alternate each MFMA with a few
// VALU instructions, so the decode of the next block and the scaling of the previous one issue in
// the MFMA gaps instead of as one VALU run ahead of a dependent MFMA chain. 3 = VALU per
// MFMA (0: leave it to the compiler).
template <int NMFMA>
__device__ __forceinline__ void sk_interleave() {
#pragma unroll
  for (int i = 0; i < NMFMA; i++) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // one MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // then VALU
  }
}

// All NBW blocks of a unit, pipelined: block B's MFMAs go out before block B − 1 is scaled in.
template <int QT, int NT, int WPB, bool MASK, int B, int NBW>
__device__ __forceinline__ void sk_blocks(const uint32_t (&w)[NBW][WPB], const u32x4 (&xh)[NBW][NT], const u32x4 (&xl)[NBW][NT],
                                          int nb, f32x4 (&pp)[NT], float ps1, f32x4 (&acc)[NT], const SkHdr &hd) {
  if constexpr (B < NBW) {
    f32x4 p[NT];
    float s1;
    sk_mfma<QT, NT, B, WPB, NBW>(w[B], xh, xl, p, s1, hd);
    if constexpr (B > 0) sk_scale<NT, B - 1, MASK>(pp, ps1, nb, acc);
    if constexpr (B == NBW - 1) sk_scale<NT, NBW - 1, MASK>(p, s1, nb, acc);
    else sk_blocks<QT, NT, WPB, MASK, B + 1, NBW>(w, xh, xl, nb, p, s1, acc, hd);
  }
}

template <int QT, int NT>
__global__ __launch_bounds__(512) void gemm_sk_kernel(SkArgs g) {
  using G = SkGeom<QT, NT>;
  constexpr int BB = G::BB, D = G::D, L = G::L;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = wave & 3, h = wave >> 2;
  lu8 *const sbase = (lu8 *)smem;
  lu8 *xlds = sbase;                                              // the slice's fragments (tile j, block b, split s)
  LK_LDS float *tlds = (LK_LDS float *)(sbase + G::XF);           // S: Σx of the slice's blocks
  LK_LDS f32x4 *xch = (LK_LDS f32x4 *)(sbase + G::XF + G::TB);
  LK_LDS int *flags = (LK_LDS int *)(sbase + G::XF + G::TB + G::EB);  // ready[p][parity] at 2p + parity, ack[p] at 8 + p
  lu8 *ring = sbase + G::XF + G::TB + G::EB + G::FB + wave * D * G::SLOT;
  // XCD-aware task order (speed only): the slices of one row range land on one XCD's L2
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding (before the barrier: the whole workgroup leaves)
  [[maybe_unused]] const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
  [[maybe_unused]] uint64_t c_wait = 0, c_comp = 0, c_hand = 0, c_issue = 0;
  const int slice = task % g.slices, range = task / g.slices;
  const int nblk = g.K / 32;
  const int kb0 = slice * G::SB, nb = min(G::SB, nblk - kb0);
  const int nbh = max(0, min(G::SBH, nb - G::SBH * h));  // this wave's blocks
  const int64_t RB = (int64_t)nblk * BB;
  const int ntile = (g.M + 15) / 16;
  const int t0 = range * g.tiles_per_range, t1 = min(t0 + g.tiles_per_range, ntile);
  const int nunits = t1 - t0 - p > 0 ? (t1 - t0 - p + 3) / 4 : 0;  // stream p: tiles t0 + p + 4i
  const int pph = nbh * BB / 16;
  const int myL = nbh > 0 ? L : 0;

  if (threadIdx.x < 16) flags[threadIdx.x] = 0;  // published by the barrier below

  // half unit u = rows of tile t0 + p + 4u, bytes [kb0·BB + h·RPH, + nbh·BB) of each; cell
  // q = r·PPH + c lands at slot + 16q (row pitch RPH); cells past the unit re-read cell 0
  const uint8_t *abase = g.a + (int64_t)kb0 * BB + (int64_t)h * G::RPH;
  uint32_t rofs[L];
  int rrow[L];
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int q = j * 64 + lane, r = q / G::PPH, c = q % G::PPH;
    rrow[j] = min(r, 15);
    rofs[j] = (uint32_t)((c < pph && r < 16) ? c * 16 : 0);
  }
  auto issue = [&](int u, int sl) __attribute__((always_inline)) {
    const int t = t0 + p + u * 4;
    const uint8_t *tb = abase + (int64_t)t * 16 * RB;
    const int rmax = g.M - 1 - t * 16;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const uint32_t vofs = (uint32_t)(min(rrow[j], rmax) * RB) + rofs[j];
      dma16l<0>(tb, vofs, ring + sl * G::SLOT + j * 1024);
    }
  };

  // 1. the first weight unit; the slice's activation fragments (and Q4_1 block sums) into LDS,
  //    spread over the workgroup's waves; the rest of the ring
  if (myL && nunits > 0) issue(0, 0);
  const int rbytes = 128 * nb * g.N;  // fx: the slice's raw activations, k-major rows of N floats
  if (g.fx) {
    const uint8_t *src = g.b + (int64_t)kb0 * 128 * g.N;
    for (int q = wave; q * 1024 < rbytes; q += G::NW) {
      int off = q * 1024 + lane * 16;
      off = off < rbytes ? off : rbytes - 16;   // lanes past the slice re-read its last piece (unused)
      dma16l<false>(src, (uint32_t)off, xlds + q * 1024);
    }
  } else {
    for (int i = wave; i < G::XI; i += G::NW) {  // fragment i: tile i / 32, block (i % 32) / 2, split i % 2
      const int j = i / (2 * G::SB), b = (i % (2 * G::SB)) / 2, sp = i % 2;
      const int kb = b < nb ? kb0 + b : kb0;      // past a short slice: any valid fragment (masked)
      dma16l<false>(g.frag, (uint32_t)((((int64_t)j * nblk + kb) * kXSplits + sp) * 1024 + lane * 16), xlds + i * 1024);
    }
    const int n16 = 16 * NT;
    const int64_t tot = (int64_t)nblk * n16;   // floats in xsum
    if (wave < G::TI) {
      int64_t f = (int64_t)kb0 * n16 + 256 * wave + 4 * lane;
      if (f + 4 > tot) f = 0;                   // past the last block: masked
      dma16l<false>(g.xsum, (uint32_t)(f * 4), (lu8 *)tlds + wave * 1024);
    }
  }
  if (myL)
    for (int u = 1; u < min(D, nunits); u++) issue(u, u);
  // x landed (and this wave's unit 0: the DMA before it), flags written; the ring's later units
  // stay in flight across the bare barriers
  wait_vmcnt_rt<G::MAXW>(myL * max(0, min(D - 1, nunits - 1)));
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();
  if (g.fx) {
    // split the raw slice in place into the MFMA fragments (as xsplit_kernel, q4_order 2):
    // item (tile j, block b) -> lane (i, gq) holds x(n = 16j + i, k = 32b + 8gq + kk(e)),
    // kk(e) = (e >> 1) + 4(e & 1); every wave reads its items, then all write
    constexpr int NI = (16 * NT + G::NW - 1) / G::NW;  // items per wave
    float v[NI][8];
    const int i16 = lane & 15, gq = lane >> 4;
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int item = wave + it * G::NW, j = item / 16, b = item % 16;
      const int n = 16 * j + i16;
      const bool ok = item < 16 * NT && b < nb && n < g.N;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int kl = 32 * b + 8 * gq + (e >> 1) + 4 * (e & 1);
        v[it][e] = ok ? *(const LK_LDS float *)(xlds + (kl * g.N + n) * 4) : 0.f;
      }
    }
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();  // every raw value is in registers: the image may be overwritten
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int item = wave + it * G::NW, j = item / 16, b = item % 16;
      if (item >= 16 * NT) continue;
      uint32_t hi[4], lo[4];
      float hsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        uint32_t hh[2], ll[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t bx = __builtin_bit_cast(uint32_t, v[it][e + q]);
          const float r = v[it][e + q] - __builtin_bit_cast(float, bx & 0xFFFF0000u);  // exact
          uint32_t br = __builtin_bit_cast(uint32_t, r);
          br += 0x7FFFu + ((br >> 16) & 1u);  // round to nearest even
          hh[q] = bx;
          ll[q] = br;
          hsum += __builtin_bit_cast(float, bx & 0xFFFF0000u) + __builtin_bit_cast(float, br & 0xFFFF0000u);
        }
        hi[e / 2] = __builtin_amdgcn_perm(hh[1], hh[0], 0x07060302u);
        lo[e / 2] = __builtin_amdgcn_perm(ll[1], ll[0], 0x07060302u);
      }
      LK_LDS u32x4 *xf = (LK_LDS u32x4 *)(xlds + ((j * G::SB + b) * kXSplits) * 1024) + lane;
      xf[0] = u32x4{hi[0], hi[1], hi[2], hi[3]};
      xf[64] = u32x4{lo[0], lo[1], lo[2], lo[3]};
      hsum += __shfl_xor(hsum, 16, kWave);
      hsum += __shfl_xor(hsum, 32, kWave);
      if (gq == 0) tlds[b * 16 * NT + 16 * j + i16] = hsum;
    }
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();
  }
  u32x4 xh[8][NT], xl[8][NT];
#pragma unroll
  for (int b = 0; b < 8; b++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const LK_LDS u32x4 *xf = (const LK_LDS u32x4 *)(xlds + ((j * G::SB + G::SBH * h + b) * kXSplits) * 1024) + lane;
      xh[b][j] = xf[0];
      xl[b][j] = xf[64];
      if (b >= nbh) {  // zero, so p == 0 exactly for masked blocks
        xh[b][j] = u32x4{0u, 0u, 0u, 0u};
        xl[b][j] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  // bias operands: lane (i = lane & 15, k' = lane >> 4) of v_mfma_f32_16x16x4_f32 c holds
  // S(block 8h + 4c + k', column 16j + i); zero past the wave's blocks
  float sf[2][NT];
#pragma unroll
  for (int c = 0; c < 2; c++)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const int bl = 4 * c + (lane >> 4);
      sf[c][j] = bl < nbh ? tlds[(G::SBH * h + bl) * 16 * NT + 16 * j + (lane & 15)] : 0.f;
    }
  if (h) __builtin_amdgcn_s_setprio(1);

  const int N16 = 16 * NT;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4) ? g.slices * g.M * N16 * 4 : 0, 0x00020000);
  // h = 0 collects unit u − 1's partner sums after computing unit u (the partner, at higher issue
  // priority, is ahead), so neither wave idles while the other computes: the two waves of a SIMD
  // overlap their VALU / MFMA streams.
  auto collect = [&](int v, const f32x4 (&mine)[NT]) __attribute__((always_inline)) {
    const LK_LDS f32x4 *xb = xch + ((v & 1) * 4 + p) * NT * 64 + lane;
    while (ldsl_ld(flags + 2 * p + (v & 1)) != v + 1) __builtin_amdgcn_s_sleep(1);
    f32x4 sum[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) sum[j] = mine[j] + xb[j * 64];
    ldsl_st(flags + 8 + p, v + 1);
    // outputs: lane holds C'(n = 16j + 4(lane>>4) + e, m = 16t + (lane&15))
    const int t = t0 + p + v * 4;
    const int64_t m = (int64_t)t * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const int n0 = 16 * j + 4 * (lane >> 4);
      if (g.slices > 1) {
        if (m < g.M) store_partial(slab_wt(g.rsync != nullptr, (int64_t)g.slices * g.M * N16 * 4), prs, g.partial, ((int64_t)slice * g.M + m) * N16 + n0, sum[j]);
      } else if (m < g.M) {
        const float e4[4] = {sum[j].x, sum[j].y, sum[j].z, sum[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (n0 + q < g.N) *(float *)(g.dst + m * g.d_nb1 + (n0 + q) * g.d_nb0) = e4[q];
      }
    }
  };
  f32x4 prev[NT];
  for (int u = 0; u < nunits; u++) {
    const int slot = u % D;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (myL) {
      // ops younger than this unit's DMA: its successors already issued, and the stores of the
      // collections since (h = 0: NT or more per iteration from iteration 1 on)
      wait_vmcnt_rt<G::MAXW>(myL * min(D - 1, nunits - 1 - u) + (h == 0 ? NT * min(D, max(u - 1, 0)) : 0));
      asm volatile("" ::: "memory");
      uint32_t wd[8][G::WPB];
      uint32_t eb[2];  // the header (d, and m for Q4_1) of block 4c + (lane >> 4) of the lane's row
      uint32_t ek[2];  // Q4_K: sub-block 4c + (lane >> 4)'s min-high byte
      SkHdr hd{};
      {
        const lu8 *bm = ring + slot * G::SLOT + (lane & 15) * G::RPH;
        const lu8 *bg = bm + 4 * (lane >> 4);
        sk_read_all<QT, G::WPB, 0, 8>(bm, bg, wd);
        if constexpr (QT == LK_TYPE_Q4_K) {
#pragma unroll
          for (int i = 0; i < 4; i++) hd.h[i] = lds32(bm + 4 * i);
#pragma unroll
          for (int c = 0; c < 2; c++) {
            const int sbl = 4 * c + (lane >> 4);
            eb[c] = *(const LK_LDS uint8_t *)(bm + 4 + sbl);                       // scale byte (:274)
            ek[c] = sbl * 2 + 1 < LK_K_SCALE_SIZE ? *(const LK_LDS uint8_t *)(bm + 5 + 2 * sbl) : 0u;  // (:279-282)
          }
        } else {
#pragma unroll
          for (int c = 0; c < 2; c++) {
            const lu8 *hp = bm + (4 * c + (lane >> 4)) * BB;
            if constexpr (QT == LK_TYPE_Q4_1) eb[c] = lds32(hp);
            else eb[c] = *(const LK_LDS uint16_t *)hp;
          }
        }
        asm volatile("" ::: "memory");
      }
      if constexpr (QT == LK_TYPE_Q4_K) {
        const float d = h2f(hd.h[0]);
        hd.dk = d * (1.0f / 945.0f);
        hd.d63 = d * (1.0f / 63.0f);
        hd.dmin = h2f(hd.h[0] >> 16);
      }
      f32x4 pp[NT];
      if (nbh == 8) {
        sk_blocks<QT, NT, G::WPB, false, 0, 8>(wd, xh, xl, nbh, pp, 0.f, acc, hd);
        sk_interleave<8 * 2 * NT>();
      } else {
        sk_blocks<QT, NT, G::WPB, true, 0, 8>(wd, xh, xl, nbh, pp, 0.f, acc, hd);
      }
      // the offsets: acc += Σ_b e_b·S_b over the 8 blocks (f32 MFMA, K = 4 blocks each)
#pragma unroll
      for (int c = 0; c < 2; c++) {
        float e;
        if constexpr (QT == LK_TYPE_Q4_K) {  // min − 128·s1 of sub-block 4c + (lane >> 4)
          const float s1 = (float)(eb[c] & 0x3Fu) * hd.dk;
          const float mn = fmaf((float)(((eb[c] >> 6) & 3u) | ((ek[c] & 0x0Fu) << 2)), hd.d63, hd.dmin);
          e = fmaf(-128.f, s1, mn);
        } else if constexpr (QT == LK_TYPE_Q4_1) {
          e = fmaf(-128.f, h2f(eb[c]), h2f(eb[c] >> 16));
        } else {
          e = -136.f * h2f(eb[c]);
        }
        if (4 * c + (lane >> 4) >= nbh) e = 0.f;  // stale header bytes past the wave's blocks
#pragma unroll
        for (int j = 0; j < NT; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(sf[c][j], e, acc[j], 0, 0, 0);
      }
      wait_lgkmcnt0();  // this slot's LDS reads have landed: the DMA may overwrite it
      if (u + D < nunits) issue(u + D, slot);
    }
    if (h == 1) {
      // the partner has consumed unit u − 2 (this parity's previous contents)
      LK_LDS f32x4 *xb = xch + ((u & 1) * 4 + p) * NT * 64 + lane;
      while (ldsl_ld(flags + 8 + p) < u - 1) __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < NT; j++) xb[j * 64] = acc[j];
      ldsl_st(flags + 2 * p + (u & 1), u + 1);
    } else {
      if (u > 0) collect(u - 1, prev);
#pragma unroll
      for (int j = 0; j < NT; j++) prev[j] = acc[j];
    }
  }
  if (h == 0 && nunits > 0) collect(nunits - 1, prev);
  wait_vmcnt<0>();
  if (g.rsync) {  // the last slice to store a tile sums it; stream p lists in parity 0 of its pair's hand-off
    auto lst_of = [&](int s) __attribute__((always_inline)) { return (LK_LDS int *)(xch + s * NT * 64); };
    splitk_tiles_fixup<G::NW>(g.rsync, prs, g.slices, h == 0 ? p : -1, 4, t0, 4, nunits, lst_of, g.M, g.N, N16, g.dst,
                              g.d_nb0, g.d_nb1, lane);
  }
}


}  // namespace lk
