// lk_wide2.hpp — batched quantized GEMM for N > 32 (config C5's prefill) with dedicated loader waves.
//
// Same tiles, operands and arithmetic as gemm_wide_kernel (lk_kernels.hpp: 256-row x 64-column
// workgroup tile, K in stages of 4 blocks through an LDS ring of D stages, bf16 hi/lo activation
// fragments from xsplit_kernel, two v_mfma_f32_16x16x32_bf16 per block and 16x16 tile, the block
// scale applied in f32 after the MFMA). What changes is who waits for whom. gemm_wide_kernel has
// every wave issue its share of a stage's DMA and meets the others at two workgroup barriers per
// stage, so the DMA, the LDS reads and the MFMAs of the workgroup run one after the other (its
// lab skeleton: DMA + barriers alone 21 µs, + LDS reads 35, + compute 51-55 µs per C5 call).
// Here the waves split by role:
//   * NC = 4 or 8 consumers (one or two per SIMD): consumer c owns rows [64(c % 4), +64) of the
//     tile and 64·4/NC of its columns over the whole K slice (4 x 4 or 4 x 2 MFMA tiles, no
//     K-group reduction); per stage it waits until the stage's slot is FULL, reads each block's
//     operands from LDS and computes, and marks the slot FREE once its last LDS read of the stage
//     has landed;
//   * 4 loaders (one per SIMD): each issues a fixed quarter of every stage's LDS-DMA instructions,
//     marks the stage FULL once its own pieces have landed (vmcnt), and refills a slot once all
//     consumers have freed it — up to D - 1 stages ahead of the slowest consumer.
// FULL / FREE are monotonic per-slot LDS counters (4 arrivals per use), so no wave waits at a
// workgroup barrier after the prologue and the DMA stream overlaps the MFMAs.
#pragma once

#include "lk_kernels.hpp"
#include "lk_skinny.hpp"

namespace lk {

// Operands (gemm_wide2_kernel): Q4_0 / Q4_1 codes as the exact bf16 128 + n, two per v_and_or_b32
// (lk_skinny.hpp q4_codes_128; activations in the matching k order, xsplit_kernel q4_order 2), the
// offset entering through the first MFMA's C input: C = T = −136·S (Q4_0, xsplit mult −136) or
// C = −128·T with T = S (Q4_1, plus m·T after the MFMA), S = Σ(hi + lo) per (block, column). The
// stage carries T for both types; Q8_0 keeps gemm_wide_kernel's decode and has no T.
// LK_W2_MODE (lab skeletons, wrong results): 1 LDS reads only, 2 compute only, 3 reads only and no
// refills after the first D stages, 4 compute + reads and no refills, 5 the FULL / FREE protocol only
#ifndef LK_W2_MODE
#define LK_W2_MODE 0
#endif
#ifndef LK_W2_RW  // lab: which operand reads the consumers issue (weights / activations / T)
#define LK_W2_RW 1
#endif
#ifndef LK_W2_RX
#define LK_W2_RX 1
#endif
#ifndef LK_W2_RT
#define LK_W2_RT 1
#endif
#ifndef LK_W2_SCHED
#define LK_W2_SCHED 1
#endif

template <int QT, int NC_ = 4> struct Wide2Geom {
  using W = WideGeom<QT>;
  static constexpr int NC = NC_, NL = 4, NW = NC + NL;         // consumer / loader waves
  // consumer c: rows [64(c % 4), +64), 16-column tiles [NTC(c / 4), +NTC) of the 64-column tile
  static constexpr int MT = 4, NT = 4, NTC = NT * 4 / NC, BM = 4 * MT * 16, BN = NT * 16;
  static_assert(NC == 4 || NC == 8, "consumers");
  static constexpr bool HAS_T = QT != LK_TYPE_Q8_0;
  static constexpr int W_BYTES = W::W_BYTES, X_BYTES = W::X_BYTES;
  static constexpr int T_OFF = W_BYTES + X_BYTES;
  static constexpr int STAGE = T_OFF + (HAS_T ? 1024 : 0);      // padding DMA re-issues a real piece
  static constexpr int TOT = W::W_INST + W::X_INST + (HAS_T ? 1 : 0);  // DMA instructions per stage
  static constexpr int CWL = (TOT + NL - 1) / NL;               // per loader
  static constexpr int CNT = 64;                                // FULL[8], FREE[8] (ints)
  static constexpr int D = ((kLdsBytes - CNT) / STAGE) > 4 ? 4 : ((kLdsBytes - CNT) / STAGE);
  static constexpr int LDS = D * STAGE + CNT;
  static constexpr float MULT = QT == LK_TYPE_Q4_0 ? -136.f : 1.f;  // xsplit's T = MULT·S
  static_assert(BM == W::BM && BN == W::BN, "same tile as gemm_wide_kernel");
  static_assert(D >= 2 && D <= 8, "ring");
  static_assert(D * CWL < 64, "vmcnt");
  static_assert(W::SB * BN * 4 <= 1024, "T");
};

// Lab (tools/lab/w2_trace.hip defines LK_W2_TRACE): per wave, s_memtime cycles spent waiting on
// the FULL / FREE counters and in total.
#ifdef LK_W2_TRACE
__device__ uint64_t *lk_w2trace_buf;
#endif

template <int QT, int NC>
__global__ __launch_bounds__((NC + 4) * 64) void gemm_wide2_kernel(WideArgs g) {
  using G = Wide2Geom<QT, NC>;
  static_assert(G::NW == NC + 4, "launch bounds");
  using WG = WideGeom<QT>;
  constexpr int MT = G::MT, NT = G::NT, NTC = G::NTC, BM = G::BM, BN = G::BN, BB = WG::BB, SB = WG::SB, D = G::D;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  lu8 *const sbase = (lu8 *)smem;
  LK_LDS int *full = (LK_LDS int *)(sbase + D * G::STAGE);  // (D <= 8)
  LK_LDS int *freec = full + 8;
  // task order as gemm_wide_kernel (XCD super-tiles; speed only)
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;
  const int slice = task % g.slices, u = task / g.slices;
  const int per_st = g.sm * g.sn, nsn = (g.tiles_n + g.sn - 1) / g.sn;
  const int st_idx = u / per_st, within = u % per_st;
  const int tm = (st_idx / nsn) * g.sm + within / g.sn, tn = (st_idx % nsn) * g.sn + within % g.sn;
  if (tm >= g.tiles_m || tn >= g.tiles_n) return;  // the whole workgroup leaves (before the barrier)
  const int nblk = g.K / 32;
  const int kb0 = slice * g.kslice, kb1 = min(kb0 + g.kslice, nblk);
  const int nst = (kb1 - kb0) / SB;
  const int64_t RB = (int64_t)nblk * BB;
  const int ntx = (g.N + 15) / 16, n16 = ntx * 16;
  if (threadIdx.x < 16) full[threadIdx.x] = 0;
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();
  if (nst <= 0) return;

#ifdef LK_W2_TRACE
  uint64_t c_wait = 0;
  const uint64_t c_start = __builtin_amdgcn_s_memtime();
  auto trace_out = [&]() {
    uint64_t *tb = (uint64_t *)((const __attribute__((address_space(4))) uint64_t *)&lk_w2trace_buf)[0];
    if (lane == 0 && tb) {
      tb[((size_t)blockIdx.x * G::NW + wave) * 2 + 0] = c_wait;
      tb[((size_t)blockIdx.x * G::NW + wave) * 2 + 1] = __builtin_amdgcn_s_memtime() - c_start;
    }
  };
#endif
  if (wave >= G::NC) {
    // ---- loader ----
    const int lw = wave - G::NC;
    uint32_t ofs[G::CWL];
    int kind[G::CWL];  // 0 weights, 1 activations, 2 T
    uint32_t dsto[G::CWL];
#pragma unroll
    for (int c = 0; c < G::CWL; c++) {
      const int q = lw + G::NL * c;
      if (q < WG::W_INST) {
        const int piece = min(q * 64 + lane, WG::WPIECES - 1);
        const int r = piece / (WG::WIN / 16), pc = piece % (WG::WIN / 16);
        const int64_t row = min((int64_t)tm * BM + r, (int64_t)g.M - 1);
        ofs[c] = (uint32_t)(row * RB + pc * 16);
        kind[c] = 0;
        dsto[c] = q * 1024;
      } else if (q < WG::W_INST + WG::X_INST) {
        const int x = q - WG::W_INST;  // (block b, x-tile j, split s)
        const int b = x / (NT * kXSplits), j = (x / kXSplits) % NT, sp = x % kXSplits;
        const int xt = min(tn * NT + j, ntx - 1);
        ofs[c] = (uint32_t)((((int64_t)xt * nblk + b) * kXSplits + sp) * 1024 + lane * 16);
        kind[c] = 1;
        dsto[c] = WG::W_BYTES + x * 1024;
      } else if (G::HAS_T && q < G::TOT) {  // the stage's T, lane -> (block, 4 columns)
        const int li = min(lane, SB * BN / 4 - 1);
        const int b = li / (BN / 4), c4 = li % (BN / 4);
        const int n = min(tn * BN + 4 * c4, n16 - 4);
        ofs[c] = (uint32_t)(((int64_t)b * n16 + n) * 4);
        kind[c] = 2;
        dsto[c] = G::T_OFF;
      } else {  // padding: the loader's first piece again (same bytes to the same place)
        ofs[c] = ofs[0];
        kind[c] = kind[0];
        dsto[c] = dsto[0];
      }
    }
    auto issue = [&](int st) __attribute__((always_inline)) {
      const int kb = kb0 + st * SB;
      lu8 *slot = sbase + (st % D) * G::STAGE;
#pragma unroll
      for (int c = 0; c < G::CWL; c++) {
        const uint8_t *base = kind[c] == 1 ? (const uint8_t *)g.frag + (int64_t)kb * kXSplits * 1024
                              : kind[c] == 2 ? (const uint8_t *)(g.xsum + (int64_t)kb * n16)
                                             : g.a + (int64_t)kb * BB;
        dma16l<false>(base, ofs[c], slot + dsto[c]);
      }
    };
    const int pro = min(D, nst);
    for (int s = 0; s < pro; s++) issue(s);
    for (int s = 0; s < nst; s++) {
      // stage s landed: the younger ones in flight are stages s+1 .. s+D-1 (prologue) / s+D-2
      const int hi = min(nst - 1, s == 0 ? pro - 1 : s + D - 2);
      wait_vmcnt_rt<(D - 1) * G::CWL>(G::CWL * (hi - s));
      if (lane == 0) __hip_atomic_fetch_add(full + s % D, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // refill the slot of stage s - 1 once the consumers are done with it
      if (s >= 1 && s - 1 + D < nst) {
        const int need = G::NC * ((s - 1) / D + 1);  // every consumer freed it
#ifdef LK_W2_TRACE
        const uint64_t w0 = __builtin_amdgcn_s_memtime();
#endif
        while (ldsl_ld(freec + (s - 1) % D) < need) __builtin_amdgcn_s_sleep(1);
#ifdef LK_W2_TRACE
        c_wait += __builtin_amdgcn_s_memtime() - w0;
#endif
#if LK_W2_MODE < 3 || LK_W2_MODE == 5
        issue(s - 1 + D);
#endif
      }
    }
#ifdef LK_W2_TRACE
    trace_out();
#endif
    return;
  }

  // ---- consumer ----
  // One block of lookahead: block gb + 1's operands are read from LDS while block gb's MFMAs run
  // (a stage's slot is freed once its last block's reads have landed).
  const int mw = wave % 4, j0 = (wave / 4) * NTC;
  f32x4 acc[MT][NTC];
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NTC; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int m = lane & 15, gq = lane >> 4;
  constexpr int WD = QT == LK_TYPE_Q4_1 ? 2 : QT == LK_TYPE_Q4_0 ? 3 : 4;
  struct Ops {
    uint32_t wd[MT][WD];
    u32x4 xh[NTC], xl[NTC];
    f32x4 tq[NTC];
  };
  auto load = [&](int gb, Ops &o) __attribute__((always_inline)) {
    const int s = gb / SB, b = gb % SB, sl = s % D;
    const lu8 *W = sbase + sl * G::STAGE;
    const lu8 *X = W + WG::W_BYTES;
    const int ob = b * BB;
#if LK_W2_RW
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const lu8 *rowp = W + ((mw * MT + i) * 16 + m) * WG::WIN;
      if constexpr (QT == LK_TYPE_Q4_1) {
        o.wd[i][0] = lds32(rowp + ob);
        o.wd[i][1] = lds32(rowp + ob + 4 + 4 * gq);
      } else if constexpr (QT == LK_TYPE_Q4_0) {  // 18-B blocks: even b 4-aligned
        const int e = (b & 1) ? -2 : 0;             // odd b: d in the high half of the dword before
        o.wd[i][0] = lds32(rowp + ob + e);
        o.wd[i][1] = lds32(rowp + ob + 4 * gq - e);
        o.wd[i][2] = lds32(rowp + ob + 4 * gq + 4);
      } else {
        const int e = (b & 1) ? -2 : 0;
        o.wd[i][0] = lds32(rowp + ob + e);
        o.wd[i][1] = lds32(rowp + ob + 8 * gq - e);
        o.wd[i][2] = lds32(rowp + ob + 8 * gq + 4 - e);
        o.wd[i][3] = lds32(rowp + ob + 8 * gq + 8);
      }
    }
#endif
#if LK_W2_RX
#pragma unroll
    for (int j = 0; j < NTC; j++) {
      const LK_LDS u32x4 *xf = (const LK_LDS u32x4 *)(X + ((b * NT + j0 + j) * kXSplits) * 1024) + lane;
      o.xh[j] = xf[0];
      o.xl[j] = xf[64];
    }
#endif
    if constexpr (G::HAS_T && LK_W2_RT) {
      const LK_LDS float *T = (const LK_LDS float *)(W + G::T_OFF);
#pragma unroll
      for (int j = 0; j < NTC; j++) o.tq[j] = *(const LK_LDS f32x4 *)(T + b * BN + (j0 + j) * 16 + gq * 4);
    }
  };
  auto compute = [&](int gb, const Ops &o) __attribute__((always_inline)) {
    const bool odd = (gb % SB) & 1;
    bf16x8 wf[MT];
    float s1[MT], s2[MT];
#pragma unroll
    for (int i = 0; i < MT; i++) {
      s2[i] = 0.f;
      if constexpr (QT == LK_TYPE_Q4_1) {
        wf[i] = q4_codes_128(o.wd[i][1]);
        s1[i] = h2f(o.wd[i][0]);
        s2[i] = h2f(o.wd[i][0] >> 16);
      } else if constexpr (QT == LK_TYPE_Q4_0) {  // even: codes straddle (realign); odd: aligned
        wf[i] = q4_codes_128(odd ? o.wd[i][1] : align2(o.wd[i][2], o.wd[i][1]));
        s1[i] = h2f(odd ? o.wd[i][0] >> 16 : o.wd[i][0]);
      } else {
        wf[i] = odd ? w_frag<LK_TYPE_Q8_0>(o.wd[i][1], o.wd[i][2])
                    : w_frag<LK_TYPE_Q8_0>(align2(o.wd[i][2], o.wd[i][1]), align2(o.wd[i][3], o.wd[i][2]));
        s1[i] = h2f(odd ? o.wd[i][0] >> 16 : o.wd[i][0]);
      }
    }
    f32x4 c0[NTC], t[NTC];
#pragma unroll
    for (int j = 0; j < NTC; j++) {
      c0[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      t[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (QT == LK_TYPE_Q4_0) c0[j] = o.tq[j];  // −136·S
      if constexpr (QT == LK_TYPE_Q4_1) {
        t[j] = o.tq[j];  // S
        const f2v k = {-128.f, -128.f};
        const f2v a = k * f2v{t[j].x, t[j].y}, bq = k * f2v{t[j].z, t[j].w};
        c0[j] = f32x4{a.x, a.y, bq.x, bq.y};
      }
    }
    // 16 tiles, each an MFMA pair; a tile's result is scaled into acc LAG tiles later, so the
    // VALU never waits on the MFMA it follows (one in-order wave per SIMD)
    constexpr int NTL = MT * NTC, LAG = 3;
    f32x4 pr[LAG + 1];
#pragma unroll
    for (int k = 0; k < NTL + LAG; k++) {
      if (k < NTL) {
        const int i = k % MT, j = k / MT;
        f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, o.xl[j]), wf[i], c0[j], 0, 0, 0);
        pr[k % (LAG + 1)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, o.xh[j]), wf[i], p, 0, 0, 0);
      }
      if (k >= LAG) {
        const int kk = k - LAG, i = kk % MT, j = kk / MT;
        accumulate<QT == LK_TYPE_Q4_1>(acc[i][j], s1[i], s2[i], pr[kk % (LAG + 1)], t[j]);
      }
    }
  };
  const int nbt = nst * SB;  // blocks of the K slice (even: SB = 4)
  // step gb: block gb's operands (in `use`) have landed; free its stage if it was the stage's last
  // block, start reading block gb + 1 into `into`, then compute gb. Two buffers in ping-pong (no
  // register copies); the MFMAs are interleaved with the decode / scale VALU.
  auto step = [&](int gb, const Ops &use, Ops &into) __attribute__((always_inline)) {
    wait_lgkmcnt0();
    if (gb % SB == SB - 1 && lane == 0)  // the stage's last reads: the loaders may refill the slot
      __hip_atomic_fetch_add(freec + (gb / SB) % D, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (gb + 1 < nbt) {
      if ((gb + 1) % SB == 0) {  // the next block opens a stage: wait until it is FULL
        const int s = (gb + 1) / SB;
#ifdef LK_W2_TRACE
        const uint64_t w0 = __builtin_amdgcn_s_memtime();
#endif
        while (ldsl_ld(full + s % D) < G::NL * (s / D + 1)) __builtin_amdgcn_s_sleep(1);
#ifdef LK_W2_TRACE
        c_wait += __builtin_amdgcn_s_memtime() - w0;
#endif
      }
#if LK_W2_MODE == 2 || LK_W2_MODE == 5  // lab skeleton: no LDS reads after the first block
      if (gb < 0) load(gb + 1, into);
      else into = use;
#else
      load(gb + 1, into);
#endif
    }
#if LK_W2_MODE == 5  // lab skeleton: the FULL / FREE protocol alone
    acc[0][0].x += __builtin_bit_cast(float, use.wd[0][0] & 0x3FFFFFFFu);
#elif LK_W2_MODE == 1 || LK_W2_MODE == 3  // lab skeleton: LDS reads only, folded into one accumulator
    {
      uint32_t f = 0;
#pragma unroll
      for (int i = 0; i < MT; i++)
#pragma unroll
        for (int q = 0; q < WD; q++) f ^= use.wd[i][q];
#pragma unroll
      for (int j = 0; j < NTC; j++) f ^= use.xh[j][0] ^ use.xl[j][1] ^ __builtin_bit_cast(uint32_t, use.tq[j].x);
      acc[0][0].x += __builtin_bit_cast(float, f & 0x3FFFFFFFu);
    }
#else
    compute(gb, use);
#endif
#if LK_W2_SCHED
#pragma unroll
    for (int i = 0; i < MT * NTC; i++) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // one tile's MFMA pair
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // then VALU (a lagged tile's scale, decode)
    }
#endif
  };
  Ops o0{}, o1{};
  while (ldsl_ld(full) < G::NL) __builtin_amdgcn_s_sleep(1);
  load(0, o0);
  for (int gb = 0; gb < nbt; gb += 2) {
    step(gb, o0, o1);
    step(gb + 1, o1, o0);
  }
#ifdef LK_W2_TRACE
  trace_out();
#endif
  // outputs: lane holds C'(n = 16·(tn·NT + j) + 4(lane>>4) + e, m = tm·BM + (mw·MT + i)·16 + (lane&15))
  const int npad = g.tiles_n * BN;
#pragma unroll
  for (int i = 0; i < MT; i++) {
    const int64_t mr = (int64_t)tm * BM + (mw * MT + i) * 16 + (lane & 15);
    if (mr >= g.M) continue;
#pragma unroll
    for (int j = 0; j < NTC; j++) {
      const int n0 = tn * BN + (j0 + j) * 16 + 4 * (lane >> 4);
      if (g.slices > 1) {
        *(f32x4 *)(g.partial + (((int64_t)slice * g.M + mr) * npad + n0)) = acc[i][j];
      } else {
        const float e4[4] = {acc[i][j].x, acc[i][j].y, acc[i][j].z, acc[i][j].w};
        if (g.d_nb0 == 4 && n0 + 4 <= g.N && ((((uintptr_t)g.dst + mr * g.d_nb1 + n0 * 4) & 15) == 0)) {
          *(f32x4 *)(g.dst + mr * g.d_nb1 + n0 * 4) = acc[i][j];
        } else {
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (n0 + q < g.N) *(float *)(g.dst + mr * g.d_nb1 + (n0 + q) * g.d_nb0) = e4[q];
        }
      }
    }
  }
}

}  // namespace lk
