// lk_kpart.hpp — gemm_kpart_kernel: Q4_0 / Q4_1 x F32 at 2 <= N <= 16, K <= 4096 (round 4).
//
// computeMatMul's quantized dots (core/GGMLComputeOps.kt:70-145, dispatched at :1448-1480) for a few
// activation columns, on v_mfma_f32_16x16x32_bf16, with the K dimension split INSIDE the workgroup.
//
// Why: the round-2/3 skinny kernels give every workgroup one 16-block K slice (all of its waves hold
// the same activations), so K = 4096 takes 8 workgroups per row range and 8 partial slabs per output
// tile, which round 3 summed by making the slices wait for each other inside the launch. Here the 8
// waves of a workgroup hold DIFFERENT K parts — wave w the activation fragments of KB = 8 blocks
// (64·NT VGPRs: bf16 hi + lo, |x − hi − lo| ≤ 2⁻¹⁷|x|, split once per call by xsplit_kernel and
// loaded as coalesced 16-B pieces) — so a workgroup covers 64 blocks (K = 2048) and K = 4096 is two
// slices, which add their tile sums into dst (zeroed by the xsplit launch): two addends per element,
// so the order cannot change a bit, and no workgroup waits for another. More slices (K > 4096, only
// with LK_KPART_ALL) store slabs summed by the last arriver per tile or by splitk_reduce_kernel.
// The product routes N <= 16 here (measured round 4: N = 8 / 16 16.0 / 16.3 µs against 17.5 / 17.7
// on the skinny kernel with the reduce launch); at N = 32 the pair kernel with the reduce launch is
// as fast (C3 23.0 vs 23.3 µs) and the down projection (K = 11008, six slices) much faster.
//
// Schedule: workgroup = (row range, K slice); each wave streams every 16-row tile of the range
// through its own LDS-DMA ring (its row pieces: KB blocks of 16 rows, nt policy), computes its
// partial 16 x 16·NT tile (codes as bf16 — Q4_0 the exact 128 + n, Q4_1 n·2⁻⁹ — against its held
// fragments, the block scale after each block's MFMA pair, the per-block offset term on the f32
// MFMA once per unit), writes it to an LDS slot of the tile (row-major rows) and counts itself in;
// the tile's owner (the wave of part tile % active parts) sums the partials in part order two units
// later. Inside the workgroup a wave may run at most NB tiles ahead of the slowest (LDS slots).
#pragma once

#include "lk_kernels.hpp"

namespace lk {

// Lab timeline (built only with -DLK_LAB_STAMPS, never in the product library; lk_kernels.hpp):
// per (workgroup, wave) s_memrealtime stamps — 0 entry, 1 activations in registers, 2 loop start,
// 3 loop end, 4 exit — and sums over the wave's units: 5 ring wait, 6 compute, 7 tile sum (slot wait,
// partial, count, the completing wave's sum and stores), 8 units. Read by tools/stamp_kpart.py.

#ifndef LK_KP_ACC_MIX
#define LK_KP_ACC_MIX 0  // lab builds only: the per-block scale as four v_fma_mix_f32
#endif
#ifndef LK_KP_KB
#define LK_KP_KB 0  // lab builds only: 16 = the first round-4 version (16 / NT blocks per wave)
#endif
#ifndef LK_KP_PRIO
#define LK_KP_PRIO 0  // lab builds only (tools/build_lab.sh): issue-priority policies of the SIMD's two waves
#endif

// The waits of gemm_kpart_kernel are on waves of the SAME workgroup (LDS words), which are always
// co-resident: they end by construction. A fixed 200 ms bound (not lk_sync_wait_bound, the test
// hook of the cross-workgroup waits) still turns a logic error into a counted timeout, not a hang.
constexpr uint64_t kIntraWgBound = 20000000ull;
constexpr int kSumLag = 2;  // a tile's owner sums it at its own boundary this many units later

template <int QT, int NT> struct KpartGeom {
  static constexpr int NW = 8;
  static constexpr int BB = QTraits<QT>::BB;
  // blocks per wave: 8 (activations in 64·NT VGPRs). At N <= 16 a wave could hold 16 (one slice
  // spanning K = 4096), but the workgroup then loads 256 KB of fragments before its first unit and
  // each unit is twice as long; 8 halves both and makes K = 4096 two slices added into dst
  static constexpr int KB = LK_KP_KB ? LK_KP_KB / NT : 8;
  static constexpr int SPAN = NW * KB;                // blocks per workgroup (one K slice)
  static constexpr int PIECE = KB * BB;               // bytes of a wave's row piece
  static constexpr int PP = PIECE / 16;               // its 16-B cells
  // cells per LDS row: odd, so the 16 rows of a unit start on 16 distinct 4-bank groups (Q4_1's
  // 10 cells would put rows m and m + 8 on the same banks: 2-way conflicts on every weight read)
  static constexpr int CP = PP | 1;
  static constexpr int PITCH = CP * 16;               // LDS row pitch
  static constexpr int L = (16 * CP + 63) / 64;       // DMA instructions per unit (16 rows)
  static constexpr int SLOT = L * 1024;
  static constexpr int WPB = QT == LK_TYPE_Q4_1 ? 2 : 3;
  static constexpr int NB = 4;                        // tile slots (tiles in flight in the workgroup)
  static constexpr int PT = 16 * NT + 4;              // partial tile row pitch (floats): conflict-free 16-B writes
  static constexpr int PART = 16 * PT * 4;            // bytes of one part's partial tile
  static constexpr int RED = NB * NW * PART;          // partial tiles, [slot][part][row][PT]
  static constexpr int FL = 64;                       // cnt[NB], done[NB]
  static constexpr int DFIT = (kLdsBytes - RED - FL) / (NW * SLOT);
  static constexpr int D = DFIT > 3 ? 3 : DFIT;       // ring depth (units in flight per wave)
  static constexpr int LDS = RED + FL + NW * D * SLOT;
  static constexpr int MAXW = L * (D - 1) + D * NT;   // largest vmcnt a wait needs
  static_assert(PIECE % 16 == 0, "row pieces are whole DMA cells");
  static_assert(D >= 2, "ring must double-buffer");
  static_assert(LDS <= kLdsBytes, "LDS");
  static_assert(MAXW < 64, "vmcnt");
  static_assert(KB % 4 == 0, "offset MFMA takes 4 blocks");
};

struct KpartArgs {
  const uint8_t *a;        // weights (buffer base + dataOffset), rows RB bytes apart
  const u32x4 *frag;       // xsplit_kernel fragments [ntx][nblk][hi, lo][64 lanes] (k order of QT's decode)
  const float *xsum;       // xsplit_kernel T per (block, column): [nblk][16·ntx]
  uint8_t *dst;            // dst(n, m) at n·d_nb0 + m·d_nb1
  int64_t d_nb0, d_nb1;
  float *partial;          // [slices][M][16·NT] when slices > 1
  int32_t M, N, K;
  int32_t slices, tiles_per_range, tasks;  // tasks = ranges·slices (the grid is padded to 8)
  unsigned *tcnt;          // per-tile arrival counters (slices > 1), zero between launches
  int32_t atomic_dst;      // slices == 2: tile sums added into dst (zeroed by the xsplit launch)
};

// LDS atomic add returning the old value (inline asm: the compiler would drain every LDS-DMA in
// flight before a compiler-visible LDS atomic); waited for here.
__device__ __forceinline__ unsigned lds_add_rtn(LK_LDS unsigned *p, unsigned v) {
  unsigned old;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  return old;
}
__device__ __forceinline__ int ldsk_ld(const LK_LDS int *p) {
  asm volatile("" ::: "memory");
  const int v = *(volatile const LK_LDS int *)p;
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void ldsk_st(LK_LDS int *p, int v) {
  asm volatile("" ::: "memory");
  *(volatile LK_LDS int *)p = v;
  asm volatile("" ::: "memory");
}

// acc += s·p as two packed FMAs (v_pk_fma_f32, the scale converted once per block) instead of four
// mixed-precision FMAs
__device__ __forceinline__ void accumulate_pk(f32x4 &acc, float s, f32x4 p) {
  const f2v s2 = {s, s};
  f2v lo = {acc.x, acc.y}, hi = {acc.z, acc.w};
  lo = __builtin_elementwise_fma(s2, f2v{p.x, p.y}, lo);
  hi = __builtin_elementwise_fma(s2, f2v{p.z, p.w}, hi);
  acc = f32x4{lo.x, lo.y, hi.x, hi.y};
}

// Block B of a wave's KB: weight fragment from its dwords, the MFMA pair against the held fragments,
// acc += s·p (the offset term comes once per unit, kpart_offsets).
template <int QT, int NT, int KB, int B, int WPB>
__device__ __forceinline__ void kpart_block(const uint32_t (&w)[WPB], const u32x4 (&xh)[KB][NT], const u32x4 (&xl)[KB][NT],
                                            f32x4 (&acc)[NT]) {
  constexpr int OB = B * QTraits<QT>::BB;
  bf16x8 wf;
  float s1;
  if constexpr (QT == LK_TYPE_Q4_1) {  // n·2⁻⁹ (k order 0,2,4,6,1,3,5,7), d·512; + m·Σx per unit
    wf = Q4Frag<0>::make(w[1]);
    s1 = 512.f * h2f(w[0]);
  } else {                             // 128 + n (k order 0,4,1,5,2,6,3,7), d; −136·d·Σx per unit
    if constexpr ((OB & 3) == 0) {
      wf = q4_codes_128(align2(w[2], w[1]));
      s1 = h2f(w[0]);
    } else {
      wf = q4_codes_128(w[1]);
      s1 = h2f(w[0] >> 16);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; j++) {
    f32x4 p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xl[B][j]), wf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xh[B][j]), wf, p, 0, 0, 0);
    if constexpr (LK_KP_ACC_MIX) accumulate_s<false>(acc[j], s1, 0.f, p, p);
    else accumulate_pk(acc[j], s1, p);
  }
}

template <int QT, int NT, int KB, int WPB, bool FULL, int B>
__device__ __forceinline__ void kpart_blocks(const uint32_t (&w)[KB][WPB], int nb, const u32x4 (&xh)[KB][NT],
                                             const u32x4 (&xl)[KB][NT], f32x4 (&acc)[NT]) {
  if constexpr (B < KB) {
    if (!FULL && B >= nb) return;
    kpart_block<QT, NT, KB, B, WPB>(w[B], xh, xl, acc);
    kpart_blocks<QT, NT, KB, WPB, FULL, B + 1>(w, nb, xh, xl, acc);
  }
}

template <int QT, int NT>
__global__ __launch_bounds__(512) void gemm_kpart_kernel(KpartArgs g) {
  using G = KpartGeom<QT, NT>;
  constexpr int BB = G::BB, KB = G::KB, D = G::D, L = G::L, NW = G::NW, NB = G::NB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  LK_LDS uint8_t *const sbase = (LK_LDS uint8_t *)(LK_LDS void *)smem;
  LK_LDS float *red = (LK_LDS float *)sbase;                         // [NB][NW][16][PT]
  LK_LDS unsigned *cnt = (LK_LDS unsigned *)(sbase + G::RED);        // per slot: partials counted in
  LK_LDS int *done = (LK_LDS int *)(sbase + G::RED) + NB;            // per slot: last unit summed
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t *ring = smem + G::RED + G::FL + wave * D * G::SLOT;
  // XCD-aware task order (speed only: dispatch is observed round-robin over the 8 XCDs): the slices
  // of one row range — which read the same 128-B lines at their edges — land on one L2
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding (before any barrier: the whole workgroup leaves)
  [[maybe_unused]] const uint64_t t_entry = LK_KP_T();
  [[maybe_unused]] uint64_t c_wait = 0, c_comp = 0, c_red = 0;
  const int slice = task % g.slices, range = task / g.slices;
  const int nblk = g.K / 32;
  // K part of this wave, rotated by the range: the 32 CUs of an XCD load their fragments in
  // different orders (the same lines requested by every CU at once serialize on one L2 channel);
  // partials are summed in part order, so the rotation changes no bit of the result
  const int part = (wave + range) % NW;
  const int kbw = slice * G::SPAN + part * KB;                 // this wave's first block
  const int nbw = max(0, min(KB, nblk - kbw));                 // its blocks (a short last slice)
  const int nact = min(NW, (min(G::SPAN, nblk - slice * G::SPAN) + KB - 1) / KB);  // waves with blocks
  const int64_t RB = (int64_t)nblk * BB;
  const int ntile = (g.M + 15) / 16;
  const int t0 = range * g.tiles_per_range, t1 = min(t0 + g.tiles_per_range, ntile);
  const int nunits = nbw > 0 ? t1 - t0 : 0;                    // every tile of the range, in order
  const int pp = nbw * BB / 16;                                // cells of this wave's row piece
  // counts 0; done[s] = s − NB: slot s first holds unit s, with no predecessor to wait for
  if (threadIdx.x < 2 * NB) ldsk_st((LK_LDS int *)cnt + threadIdx.x, threadIdx.x < NB ? 0 : (int)threadIdx.x - 2 * NB);

  // unit u = rows of tile t0 + u, bytes [kbw·BB, + nbw·BB) of each; cell q = r·CP + c lands at
  // slot + 16q (row pitch PITCH); pad cells and cells past the unit re-read cell 0
  const uint8_t *abase = g.a + (int64_t)kbw * BB;
  uint32_t rofs[L];
  int rrow[L];
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int q = j * 64 + lane, r = q / G::CP, c = q % G::CP;
    rrow[j] = min(r, 15);
    rofs[j] = (uint32_t)((c < pp && r < 16) ? c * 16 : 0);
  }
  auto issue = [&](int u, int sl) __attribute__((always_inline)) {
    const int t = t0 + u;
    const uint8_t *tb = abase + (int64_t)t * 16 * RB;
    const int rmax = g.M - 1 - t * 16;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const uint32_t vofs = (uint32_t)(min(rrow[j], rmax) * RB) + rofs[j];
      dma16<true>(tb, vofs, ring + sl * G::SLOT + j * 1024);  // nt: read once per launch
    }
  };

  // 1. this wave's activation fragments (xsplit_kernel, one launch before: bf16 hi / lo of
  //    x(n = 16j + (lane & 15), k = 32(kbw + b) + 8(lane >> 4) + kk), kk in the code order of QT):
  //    2·KB·NT coalesced 16-B loads per lane, all in flight at once; T per (block, column) for the
  //    offset operands of v_mfma_f32_16x16x4_f32 (lane (n, b' = lane >> 4) holds T of block 4c + b')
  u32x4 xh[KB][NT], xl[KB][NT];
  float tf[KB / 4][NT];
  // the weight ring first: the compiler counts only its own loads when it waits for a fragment, so
  // DMAs issued after the fragments would be waited for too (they are younger); issued before, they
  // are older than every fragment and the compiler's waits are exact
  for (int u = 0; u < min(D, nunits); u++) issue(u, u);
  {
    const int ntx = (g.N + 15) / 16;
#pragma unroll
    for (int b = 0; b < KB; b++)
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const int jj = min(j, ntx - 1), kb = min(kbw + b, nblk - 1);
        const u32x4 *f = g.frag + ((int64_t)(jj * nblk + kb) * kXSplits) * 64 + lane;
        xh[b][j] = f[0];
        xl[b][j] = f[64];
      }
#pragma unroll
    for (int c = 0; c < KB / 4; c++)
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const int jj = min(j, ntx - 1), kb = min(kbw + 4 * c + (lane >> 4), nblk - 1);
        tf[c][j] = g.xsum[(int64_t)kb * (16 * ntx) + 16 * jj + (lane & 15)];
      }
#pragma unroll
    for (int b = 0; b < KB; b++)
#pragma unroll
      for (int j = 0; j < NT; j++)
        if (b >= nbw || j >= ntx) {  // past this wave's blocks or the columns: zero, so p == 0 exactly
          xh[b][j] = u32x4{0u, 0u, 0u, 0u};
          xl[b][j] = u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
    for (int c = 0; c < KB / 4; c++)
#pragma unroll
      for (int j = 0; j < NT; j++)
        if (4 * c + (lane >> 4) >= nbw || j >= ntx) tf[c][j] = 0.f;
  }
  [[maybe_unused]] const uint64_t t_split = LK_KP_T();
  wait_lgkmcnt0();
  __builtin_amdgcn_s_barrier();  // slot counters initialised (bare: the ring stays in flight)

  const int N16 = 16 * NT;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, g.tcnt ? g.slices * g.M * N16 * 4 : 0, 0x00020000);
  // stores this wave issued after each of its last D DMA issues (its tile sums), for the ring waits
  int st_hist = 0;  // 8 bits per unit, newest in the low byte
  uint64_t red_mask = 0;  // units whose tile this wave summed and stored (nunits <= 64, host-checked)
  // The sum of a complete tile (all nact partials counted in), by the wave whose count completed it:
  // every part's partial read at once (LDS round trips, not adds, are what a tile sum costs under
  // the ring's DMA traffic), added in part order (so the K rotation changes no bit), then stored
  // (slices == 1), written as this slice's slab, or added into dst (two slices). Returns the store
  // / atomic instructions issued (for the ring waits).
  auto sum_tile = [&](int s, int ut) __attribute__((always_inline)) -> int {
    // lane (row ml0 + i·RPI, column n) for i < NT·4: 64 / N16 whole rows per instruction
    constexpr int RPI = 64 / (16 * NT);
    const int ml0 = lane / (16 * NT), n = lane % (16 * NT);
    const LK_LDS float *pr = red + (s * NW) * (16 * G::PT) + ml0 * G::PT + n;
    float v[NT * 4];
    {
      float q[NW][NT * 4];  // every part at once (one LDS round trip); an idle part's stale slot is not added
#pragma unroll
      for (int p = 0; p < NW; p++)
#pragma unroll
        for (int i = 0; i < NT * 4; i++) q[p][i] = pr[p * 16 * G::PT + i * RPI * G::PT];
      if (nact == NW) {  // every part active (uniform): plain adds, no selects
#pragma unroll
        for (int i = 0; i < NT * 4; i++) {
          v[i] = q[0][i];  // part 0 as is (−0.0 stays)
#pragma unroll
          for (int p = 1; p < NW; p++) v[i] += q[p][i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < NT * 4; i++) {
          v[i] = q[0][i];
#pragma unroll
          for (int p = 1; p < NW; p++)
            if (p < nact) v[i] += q[p][i];
        }
      }
    }
    const int64_t mt = (int64_t)(t0 + ut) * 16 + ml0;
    int ns;
    if (g.atomic_dst) {
      // two K slices: add into dst (zeroed by the xsplit launch); each wave-instruction adds 64 / N16
      // whole dst rows (256 contiguous bytes at N16 = N = 32: the full-rate shape). Lanes past M or N
      // issue nothing (a shared dummy address would serialize every workgroup's idle lanes on one word)
      uint8_t *const lane_dst = g.dst + mt * g.d_nb1 + (int64_t)n * g.d_nb0;
#pragma unroll
      for (int i = 0; i < NT * 4; i++)
        if (mt + i * RPI < g.M && n < g.N)
          __hip_atomic_fetch_add((float *)(lane_dst + (int64_t)(i * RPI) * g.d_nb1), v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (g.slices > 1) {
      // this slice's slab rows [slice][M][N16] (write-through when the fix-up sums them in the launch)
#pragma unroll
      for (int i = 0; i < NT * 4; i++) {
        const int64_t m = mt + i * RPI;
        if (m < g.M) {
          const int64_t idx = ((int64_t)slice * g.M + m) * N16 + n;
          if (g.tcnt) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[i]), prs, (int)(idx * 4), 0, 16);
          else g.partial[idx] = v[i];
        }
      }
      red_mask |= 1ull << ut;
    } else {
#pragma unroll
      for (int i = 0; i < NT * 4; i++) {
        const int64_t m = mt + i * RPI;
        if (m < g.M && n < g.N) *(float *)(g.dst + m * g.d_nb1 + (int64_t)n * g.d_nb0) = v[i];
      }
    }
    {
      // store / atomic instructions certainly issued: those with lane 0's row inside M (lane 0 holds
      // the instruction's smallest row and column 0); a lower bound keeps the ring waits safe
      const int64_t left = (int64_t)g.M - (int64_t)(t0 + ut) * 16;
      ns = (int)min((int64_t)(NT * 4), (left + RPI - 1) / RPI);
    }
    ldsk_st((LK_LDS int *)cnt + s, 0);
    ldsk_st(done + s, ut);
    return ns;
  };
  // tile u complete: the slot's previous tile (u − NB) summed and all nact partials of u counted in
  // (the summer resets the count before it publishes done)
  auto wait_complete = [&](int u) __attribute__((always_inline)) {
    const int s = u % NB;
    for (uint64_t tw = 0; !(ldsk_ld(done + s) == u - NB && ldsk_ld((const LK_LDS int *)cnt + s) == nact);) {
      __builtin_amdgcn_s_sleep(1);
      if (!tw) tw = __builtin_amdgcn_s_memrealtime();
      else if (__builtin_amdgcn_s_memrealtime() - tw >= kIntraWgBound) {
        if (lane == 0) lk_note_timeout();
        break;
      }
    }
  };
  int own = part;  // the next tile this wave sums (tiles u with u % nact == part)
  [[maybe_unused]] const uint64_t t_loop = LK_KP_T();
#if LK_KP_PRIO == 1
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // lab: the younger wave of each SIMD first
#endif
  for (int u = 0; u < nunits; u++) {
    [[maybe_unused]] const uint64_t ta = LK_KP_T();
#if LK_KP_PRIO == 2
    if ((u + (wave >> 2)) & 1) __builtin_amdgcn_s_setprio(1);  // lab: the SIMD's two waves take turns
    else __builtin_amdgcn_s_setprio(0);
#endif
    const int slot = u % D;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      // ops younger than this unit's DMA: its successors already issued, and the tile stores since
      // (issued after DMA u, in the units u − D .. u − 1)
      int younger = 0;
#pragma unroll
      for (int i = 0; i < D; i++) younger += (st_hist >> (8 * i)) & 0xFF;
      wait_vmcnt_rt<G::MAXW>(L * min(D - 1, nunits - 1 - u) + younger);
      asm volatile("" ::: "memory");
#ifdef LK_LAB_STAMPS
      const uint64_t tb = LK_KP_T();
      c_wait += tb - ta;
#endif
      uint32_t wd[KB][G::WPB];
      const uint8_t *slot_ptr = ring + slot * G::SLOT;
      {
        const uint8_t *bm = slot_ptr + (lane & 15) * G::PITCH;
        const uint8_t *bg = bm + 4 * (lane >> 4);
        skinny_read_all<QT, KB, G::WPB, 0>(bm, bg, wd);
        asm volatile("" ::: "memory");
      }
      if (nbw == KB) kpart_blocks<QT, NT, KB, G::WPB, true, 0>(wd, nbw, xh, xl, acc);
      else kpart_blocks<QT, NT, KB, G::WPB, false, 0>(wd, nbw, xh, xl, acc);
      // acc += Σ_b e_b(row)·T_b(column), K = 4 blocks per f32 MFMA: e = d (Q4_0, T = −136·Σ(hi + lo))
      // or m (Q4_1, T = Σx); lane (m = lane & 15, b' = lane >> 4) reads its row's header of 4c + b'
      const uint8_t *hrow = slot_ptr + (lane & 15) * G::PITCH;
#pragma unroll
      for (int c = 0; c < KB / 4; c++) {
        const int bl = 4 * c + (lane >> 4);
        const uint16_t hv = *(const uint16_t *)(hrow + min(bl, KB - 1) * BB + (QT == LK_TYPE_Q4_1 ? 2 : 0));
        const float e = bl < nbw ? h2f(hv) : 0.f;
#pragma unroll
        for (int j = 0; j < NT; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(tf[c][j], e, acc[j], 0, 0, 0);
      }
      wait_lgkmcnt0();  // this slot's LDS reads have landed: the DMA may overwrite it
      if (u + D < nunits) issue(u + D, slot);
#ifdef LK_LAB_STAMPS
      c_comp += LK_KP_T() - tb;
#endif
    }
    [[maybe_unused]] const uint64_t tr = LK_KP_T();
    // the workgroup's sum of tile t0 + u: this wave's partial into slot u % NB (free once the slot's
    // previous tile, u − NB, was summed), counted in; tile u is summed by its owner, the wave of part
    // u % nact, at the owner's boundary u + kSumLag (or after its loop) — every wave sums ~1/nact of
    // the tiles, none sums on the critical path of the slowest (round 4: the wave that completed a
    // tile summed it, and since that wave is the slowest, all sums landed on the critical path)
    const int rs = u % NB;
    for (uint64_t tw = 0; ldsk_ld(done + rs) < u - NB;) {  // waits on waves of this workgroup only
      __builtin_amdgcn_s_sleep(1);
      if (!tw) tw = __builtin_amdgcn_s_memrealtime();
      else if (__builtin_amdgcn_s_memrealtime() - tw >= kIntraWgBound) {
        if (lane == 0) lk_note_timeout();
        break;
      }
    }
    // this wave's partial: lane holds C'(n = 16j + 4(lane>>4) + e, m = lane & 15), as row-major rows
    LK_LDS float *mine = red + (rs * NW + part) * (16 * G::PT) + (lane & 15) * G::PT + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < NT; j++) *(LK_LDS f32x4 *)(mine + 16 * j) = acc[j];
    if (lane == 0) (void)lds_add_rtn(cnt + rs, 1u);
    int nst = 0;
    while (own <= u - kSumLag) {
      wait_complete(own);
      nst += sum_tile(own % NB, own);
      own += nact;
    }
    st_hist = (st_hist << 8) | min(nst, 255);
#ifdef LK_LAB_STAMPS
    c_red += LK_KP_T() - tr;
#endif
  }
  // the owned tiles left (the last ones: completed by the slowest wave)
  for (; own < nunits; own += nact) {
    wait_complete(own);
    (void)sum_tile(own % NB, own);
  }
  [[maybe_unused]] const uint64_t t_end = LK_KP_T();
  wait_vmcnt<0>();  // this wave's tile stores are done
  if (g.tcnt && red_mask) {
    // split-K fix-up, per wave (no barrier): this wave stored the slab rows of the tiles in red_mask;
    // it arrives on each (a lane per tile, one instruction per 64) and sums, in slice order, the
    // tiles for which its arrival was the last (splitk_arrive; bit-identical to splitk_reduce_kernel)
    bool last = false;
    if (lane < nunits && ((red_mask >> lane) & 1ull)) last = splitk_arrive(g.tcnt + (int64_t)(t0 + lane) * kChainLine, (unsigned)g.slices);
    const uint64_t mine = __ballot(last);
    asm volatile("" ::: "memory");  // the slab loads stay after the arrivals
    // the listed tiles' items (16 rows x N16/4 column groups each), IB per lane with their loads in
    // flight together
    const int c4 = N16 / 4, per = 16 * c4, tot = __builtin_popcountll(mine) * per;
    constexpr int IB = 4;
    for (int i0 = lane * IB; i0 < tot; i0 += 64 * IB) {
      int64_t m[IB];
      int n0[IB];
      bool ok[IB];
#pragma unroll
      for (int q = 0; q < IB; q++) {
        const int i = i0 + q;
        ok[q] = i < tot;
        uint64_t mm = mine;
        for (int k = 0; ok[q] && k < i / per; k++) mm &= mm - 1;  // the (i / per)-th listed tile
        const int t = t0 + (ok[q] ? __builtin_ctzll(mm) : 0);
        m[q] = (int64_t)t * 16 + (i % per) / c4;
        n0[q] = (i % c4) * 4;
        ok[q] = ok[q] && m[q] < g.M;
      }
      f32x4 sum[IB];
      for (int b = 0; b < g.slices; b += 8) {
        f32x4 v[IB][8];
#pragma unroll
        for (int q = 0; q < IB; q++)
#pragma unroll
          for (int i = 0; i < 8; i++)
            if (ok[q] && b + i < g.slices)
              v[q][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, (int)((((int64_t)(b + i) * g.M + m[q]) * N16 + n0[q]) * 4), 0, 16));
#pragma unroll
        for (int q = 0; q < IB; q++)
#pragma unroll
          for (int i = 0; i < 8; i++)
            if (ok[q] && b + i < g.slices) {
              if (b + i == 0) sum[q] = v[q][i];  // slab 0 as is (0 + x would turn -0.0 into +0.0)
              else { sum[q].x += v[q][i].x; sum[q].y += v[q][i].y; sum[q].z += v[q][i].z; sum[q].w += v[q][i].w; }
            }
      }
#pragma unroll
      for (int q = 0; q < IB; q++) {
        if (!ok[q]) continue;
        const float e4[4] = {sum[q].x, sum[q].y, sum[q].z, sum[q].w};
        uint8_t *o = g.dst + m[q] * g.d_nb1 + n0[q] * g.d_nb0;
        if (g.d_nb0 == 4 && n0[q] + 4 <= g.N && (((uintptr_t)o) & 15) == 0) {
          *(f32x4 *)o = sum[q];
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++)
            if (n0[q] + e < g.N) *(float *)(g.dst + m[q] * g.d_nb1 + (n0[q] + e) * g.d_nb0) = e4[e];
        }
      }
    }
  }
  LK_KP_SET(0, t_entry); LK_KP_SET(1, t_split); LK_KP_SET(2, t_loop); LK_KP_SET(3, t_end);
  LK_KP_SET(4, LK_KP_T()); LK_KP_SET(5, c_wait); LK_KP_SET(6, c_comp); LK_KP_SET(7, c_red);
  LK_KP_SET(8, (uint64_t)nunits);
}

}  // namespace lk
