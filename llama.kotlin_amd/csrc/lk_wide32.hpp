// lk_wide32.hpp — Q4_0 / Q4_1 x F32 at N > 32 on v_mfma_f32_32x32x16_bf16 (round 6): config C5 (4096 x
// 4096, batch 512) and every N > 32 shape that meets w32_eligible (csrc/lk_hip.hip); N <= 32 stays on the
// pair / kpart kernels (this kernel's <3,1,1> shape measured slower on C3).
//
// Arithmetic (the reference's, K/core/GGMLComputeOps.kt:70-145, within the F32 bar): per 32-weight block
// b of row m and activation column n, with the codes as exact bf16 128 + q and x = hi + lo in bf16 pairs
// (|x − hi − lo| ≤ 2⁻¹⁷|x|), the MFMA chain gives p = Σ_k (128 + q_k)·x_k + T with the C input
// T = −c·Σ_k (hi + lo)_k (c = 136 for Q4_0: p = Σ (q − 8)·x; c = 128 for Q4_1: p = Σ q·x), then
// acc += d·p (Q4_1: + m·Σx = (−m/128)·T) in f32 with the block's f16 scale d, so an Inf / NaN scale gives
// what d·p gives (tests/test_gpu_parity.py::test_w32_route_and_nonfinite_scales).
//
// Shape: gemm_wide_kernel (16x16x32, 256 x 64 tiles, K split in two) was LDS-read bound and
// its two K slices wrote 16 MB of slabs at C5. Here:
//   * a workgroup is MH row halves of 32·MT rows x BN = 32·NT columns; 4·MH waves, wave w takes K group
//     w % 4 of row half w / 4 — the product <2,2,2>: 128 x 64 tiles, 8 waves, two per SIMD (one of each
//     half), issue priority 1 for the second-dispatched half (LK_W32_PRIO);
//   * the 4 K groups split each 4-block stage's K: group g takes block g over its half's MT x NT chains
//     of 32 x 32, so a decoded weight fragment feeds NT column tiles; the chains' MFMAs are interleaved
//     step by step (LK_W32_ILV), each chain's order unchanged;
//   * C layout: one weight row per lane (col = lane & 31), so the block scale is a per-lane scalar; T is
//     16 values per lane, broadcast ds_read_b128 from a 1-KB stage slot;
//   * one LDS-DMA ring of D = 3 stages (the tile's 80-B weight windows, the 64 columns' fragments, T:
//     44 KB), one workgroup barrier per stage, every wave issuing its share of the next stage's DMA;
//     a lane reads the two pieces holding its block and aligns its 8 code bytes in registers;
//   * the 4 K groups are summed through LDS in group order (deterministic); with `slices` > 1 (K split
//     over workgroups when the tiles leave CUs idle) each slice stores its partial write-through and the
//     last to arrive at the tile's counter sums the slabs in slice order (no waits);
//   * blockIdx -> task XCD-aware: each XCD takes a contiguous run of tasks, grouped by `bc` column tiles
//     so a run covers a block of row x column tiles (W32Args::bc).
#ifndef LK_W32_PK
#define LK_W32_PK 1  // packed scale FMAs (lab: 0 = scalar)
#endif
#ifndef LK_W32_SPREAD
#define LK_W32_SPREAD 0  // lab: 1 = half of a stage's DMAs issued before its last column tile's chains
#endif
#ifndef LK_W32_PRIO
#define LK_W32_PRIO 1  // issue priority 1 for the second-dispatched row half (waves 4-7): 52.2-52.5 us vs 54.0 at C5 (lab: 0)
#endif
#ifndef LK_W32_ILV
#define LK_W32_ILV 1  // the chains' MFMAs interleaved step by step (C5 50.6-51.3 vs 51.5-51.9 us; lab: 0 = chain by chain)
#endif
#ifndef LK_W32_PP
#define LK_W32_PP 0  // lab: 1 = the two row halves in ping-pong (w32_main_pp): C5 53.8-54.0 vs 52.3-52.6 us, not kept
#endif
#ifndef LK_W32_ILDMA
#define LK_W32_ILDMA 2  // the stage's refill DMAs one by one between its MFMAs, not as a burst after the barrier:
                        // 2 = DMA c after MFMA c (C5 51.8-52.6 vs 52.7-52.9 us), 1 = spread evenly (~ -0.3 us), 0 = burst
#endif
#ifndef LK_W32_SCHED
#define LK_W32_SCHED 0  // lab: VALU instructions per MFMA enforced by sched_group_barrier (0: the compiler's order)
#endif

namespace lk {

struct W32Args {
  const uint8_t *a;      // weights (buffer base + dataOffset), rows of K/32 blocks
  const u32x4 *frag;     // xsplit32_kernel: [ntx32][nblk][step 2][split 2][64 lanes] x 16 B
  const float *tsum;     // xsplit32_kernel: [nblk][ntx32·32] = −c·Σ_block (hi + lo)
  uint8_t *dst;
  int64_t d_nb0, d_nb1;
  int32_t M, N, K;
  int32_t tiles_m, tiles_n, tasks;
  int32_t slices, sstages;   // split K: slice s covers stages [s·sstages, (s + 1)·sstages)
  int32_t bc;                // column tiles per task group (see gemm_w32_kernel's task order)
  float *partial;            // [slices][tiles][BM·BN] (slices > 1), lane-major per chain
  unsigned *tcnt;            // per-tile arrival counters (kChainLine apart), zero between launches
};

template <int QT, int MT_, int NT_, int MH_> struct W32Geom {
  // MH row halves of MT row tiles each; 4·MH waves: wave w takes K group w % 4 of row half w / 4
  static constexpr int MH = MH_, NW = 4 * MH, MT = MT_, NT = NT_, BM = 32 * MT * MH, BN = 32 * NT, SB = 4;
  static constexpr int BB = QT == LK_TYPE_Q4_1 ? 20 : 18;
  static constexpr int WIN = 80;                            // bytes per row per stage (4 blocks: 72 / 80 B)
  static constexpr int WP = WIN / 16;                       // 16-B pieces per row
  static constexpr int W_INST = (BM * WP + 63) / 64;        // weight DMA instructions
  static constexpr int X_INST = NT * SB * 4;                // 1-KB fragments (2 steps x hi/lo)
  static constexpr int INST = W_INST + X_INST + 1;          // + T (SB x BN floats)
  static constexpr int CW = (INST + NW - 1) / NW;           // per wave (the rest padding)
  static constexpr int X_OFF = W_INST * 1024, T_OFF = X_OFF + X_INST * 1024, PAD_OFF = T_OFF + 1024;
  static constexpr int STAGE = NW * CW * 1024;
  static constexpr int D0 = (160 * 1024) / STAGE;
  static constexpr int D = D0 > 5 ? 5 : D0;                 // ring slots (D − 2 stages in flight ahead)
  static constexpr int LDS = D * STAGE;
  static constexpr int OVERREAD = WIN - SB * BB;            // bytes a row's last window reads past it
  static constexpr int CHAINS = MT * NT;                    // per wave
  static_assert(STAGE >= PAD_OFF + 1024, "stage layout");
  static_assert(D >= 3 && (D - 2) * CW < 64, "ring");
  static_assert(MH * CHAINS * 4 * 4096 <= LDS, "K-group reduction buffer ([half][chain][group] x 4 KB)");
  static_assert(4 * BN <= 1024, "T slot");
};

struct XSplit32Args {
  const uint8_t *b;      // B(n, k) at n·nb0 + k·nb1
  int64_t b_nb0, b_nb1;
  int32_t N, K;
  u32x4 *frag;
  float *tsum;
  float mult;            // −136 (Q4_0) or −128 (Q4_1)
};

#ifdef LK_W32_KERNELS  // the kernels live in their own translation unit (lk_w32.hip: MFMA results in VGPRs)
// One wave per (32-column tile t, block kb); lane (n = lane & 31, h = lane >> 5) writes, for step s,
// x(n, 32kb + 8(2h + s) + ord[j]) (ord = 0,4,1,5,2,6,3,7: q4_codes_128's element order of code dword
// 2h + s) split into bf16 hi (truncated) and lo (x − hi rounded to nearest even), as fragment
// ((t·nblk + kb)·2 + s)·2 + {0: hi, 1: lo}; and T = mult·Σ (hi + lo) over the block's 32 k.
#ifndef LK_XS32_IPW
#define LK_XS32_IPW 2  // (column tile, block) items per wave, both items' loads in flight together: C5 -0.3-0.5 us (1: +0.4, 4: +1.3, A/B)
#endif
__global__ __launch_bounds__(256) void xsplit32_kernel(XSplit32Args g) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t nblk = g.K / 32, ntx = (g.N + 31) / 32, item0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * LK_XS32_IPW;
  if (item0 >= ntx * nblk) return;
  float v[LK_XS32_IPW][2][8];
#pragma unroll
  for (int it = 0; it < LK_XS32_IPW; it++) {
    const int64_t item = min(item0 + it, ntx * nblk - 1);
    const int64_t t = item / nblk, kb = item % nblk;
    const int64_t n = 32 * t + (lane & 31);
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int64_t k = 32 * kb + 8 * (2 * h + s) + ((j >> 1) + 4 * (j & 1));
        v[it][s][j] = n < g.N ? *(const float *)(g.b + n * g.b_nb0 + k * g.b_nb1) : 0.f;
      }
  }
#pragma unroll
  for (int it = 0; it < LK_XS32_IPW; it++) {
    const int64_t item = item0 + it;
    if (item >= ntx * nblk) break;
    const int64_t t = item / nblk, kb = item % nblk;
    const int64_t n = 32 * t + (lane & 31);
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < 2; s++) {
      uint32_t hi[4], lo[4];
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        uint32_t hb[2], lb[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t bx = __builtin_bit_cast(uint32_t, v[it][s][j + q]);
          const float hf = __builtin_bit_cast(float, bx & 0xFFFF0000u);
          const float r = v[it][s][j + q] - hf;  // exact
          uint32_t br = __builtin_bit_cast(uint32_t, r);
          br += 0x7FFFu + ((br >> 16) & 1u);  // round to nearest even (r is finite, |r| < 2^-7·|x|)
          hb[q] = bx;
          lb[q] = br;
          sum += hf + __builtin_bit_cast(float, br & 0xFFFF0000u);
        }
        hi[j / 2] = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
        lo[j / 2] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
      }
      u32x4 *f = g.frag + ((item * 2 + s) * 2) * 64 + lane;
      f[0] = u32x4{hi[0], hi[1], hi[2], hi[3]};
      f[64] = u32x4{lo[0], lo[1], lo[2], lo[3]};
    }
    sum += __shfl_xor(sum, 32, kWave);
    if (h == 0) g.tsum[kb * (ntx * 32) + n] = g.mult * sum;
  }
}

// Block G of a stage window, from its two 16-B pieces G, G + 1 (window bytes [16G, 16G + 32); the block
// starts at BB·G): the code dwords of lane half h for steps 0 and 1 (code bytes [8h, 8h + 8) of the
// block), the scale d and (Q4_1) the min m.
template <int QT, int G>
__device__ __forceinline__ void w32_block(const u32x4 &p0, const u32x4 &p1, int h, uint32_t &c0, uint32_t &c1, float &d,
                                          float &mn) {
  const uint32_t Q[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
  if constexpr (QT == LK_TYPE_Q4_1) {  // 20-B blocks at 4G: d, m, codes all dword-aligned
    c0 = h ? Q[G + 3] : Q[G + 1];
    c1 = h ? Q[G + 4] : Q[G + 2];
    d = h2f(Q[G] & 0xFFFFu);
    mn = h2f(Q[G] >> 16);
  } else {
    constexpr int o = 2 * G + 2;  // first code byte, relative to the pieces
    if constexpr ((o & 3) == 0) {  // G odd: code dwords aligned
      constexpr int a = o / 4;
      c0 = h ? Q[a + 2] : Q[a];
      c1 = h ? Q[a + 3] : Q[a + 1];
    } else {  // G even: two bytes off
      constexpr int a = o / 4;
      const uint32_t l0 = __builtin_amdgcn_alignbit(Q[a + 1], Q[a], 16), l1 = __builtin_amdgcn_alignbit(Q[a + 2], Q[a + 1], 16);
      const uint32_t u0 = __builtin_amdgcn_alignbit(Q[a + 3], Q[a + 2], 16), u1 = __builtin_amdgcn_alignbit(Q[a + 4], Q[a + 3], 16);
      c0 = h ? u0 : l0;
      c1 = h ? u1 : l1;
    }
    constexpr int db = 2 * G;  // scale bytes
    d = h2f((Q[db / 4] >> (8 * (db & 3))) & 0xFFFFu);
    mn = 0.f;
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifdef LK_LAB_W32_STAMPS  // lab builds only (tools/stamp_w32.py): per-wave cycle counts of the main loop
__device__ uint64_t lk_w32_stamps[1024][8][8];  // [workgroup][wave][slot]
#define LK_W32_T() __builtin_amdgcn_s_memtime()
#else
#define LK_W32_T() 0ull
#endif

template <int QT, int MT, int NT, int MH, int G>
__device__ __forceinline__ void w32_main(const W32Args &g, uint8_t *smem, int tm, int tn, int st0, int st1, int wave, int mh,
                                         f32x16 (&acc)[MT][NT]) {
  using W = W32Geom<QT, MT, NT, MH>;
  constexpr int D = W::D, CW = W::CW;
  const int lane = threadIdx.x & 63, h = lane >> 5, m = lane & 31;
  const int nblk = g.K / 32, ntx = (g.N + 31) / 32, n32 = ntx * 32;
  const int64_t RB = (int64_t)nblk * W::BB;
  const int nst = st1 - st0;
  // per-lane DMA offsets from each instruction's stage base (fixed for the launch)
  uint32_t vofs[CW];
  int kind[CW];  // 0 weights, 1 fragments, 2 T, 3 padding (wave-uniform)
#pragma unroll
  for (int c = 0; c < CW; c++) {
    const int q = wave * CW + c;
    if (q < W::W_INST) {
      const int p = min(q * 64 + lane, W::BM * W::WP - 1), r = p / W::WP, pc = p % W::WP;  // past the last piece: re-read it
      const int64_t row = min((int64_t)tm * W::BM + r, (int64_t)g.M - 1);
      vofs[c] = (uint32_t)(row * RB + pc * 16);
      kind[c] = 0;
    } else if (q < W::W_INST + W::X_INST) {
      const int f = q - W::W_INST, j = f / (W::SB * 4), b = (f / 4) % W::SB, s = (f / 2) % 2, sp = f % 2;
      const int64_t xt = min(tn * NT + j, ntx - 1);
      vofs[c] = (uint32_t)(((((xt * nblk + b) * 2 + s) * 2 + sp) * 64 + lane) * 16);
      kind[c] = 1;
    } else if (q == W::W_INST + W::X_INST) {
      const int b = min(lane / (W::BN / 4), W::SB - 1), c4 = lane % (W::BN / 4);  // lanes past 4 x BN: never read
      const int col = min(tn * W::BN + 4 * c4, n32 - 4);
      vofs[c] = (uint32_t)(((int64_t)b * n32 + col) * 4);
      kind[c] = 2;
    } else {
      vofs[c] = 0;
      kind[c] = 3;
    }
  }
  // the ring's LDS address as a number once (a generic -> LDS pointer cast per DMA costs a null check)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LK_LDS const void *)smem);
  // per-lane LDS read offsets inside a slot: this lane's row window at block G's pieces; fragment lane
  // slot of block G; T of block G, rows 4h.. of a column tile
  const uint32_t wofs_l = (uint32_t)((mh * MT * 32 + m) * W::WIN + G * 16), xofs_l = (uint32_t)(W::X_OFF + G * 4 * 1024 + lane * 16),
                 tofs_l = (uint32_t)(W::T_OFF + (G * W::BN + 4 * h) * 4);
  auto issue = [&](int st, int sl, int c0 = 0, int c1 = W::CW) __attribute__((always_inline)) {
    const int kb = (st0 + min(st, nst - 1)) * W::SB;  // past the last stage: reload it (never read)
    const uint8_t *bw = g.a + (int64_t)kb * W::BB;
    const uint8_t *bx = (const uint8_t *)g.frag + (int64_t)kb * 4 * 1024;
    const uint8_t *bt = (const uint8_t *)(g.tsum + (int64_t)kb * n32);
    const uint32_t slot = lds0 + (uint32_t)(sl * W::STAGE);
#pragma unroll
    for (int c = c0; c < c1; c++) {
      const int q = wave * CW + c;
      const uint8_t *base = kind[c] == 0 ? bw : kind[c] == 1 ? bx : bt;
#ifdef LK_LAB_W32_NO_XDMA  // skeleton (wrong results): the fragments' DMA instructions read one 16-B line
      if (kind[c] == 1) { dma16m(bx, 0u, slot + W::PAD_OFF); continue; }
#endif
      dma16m(base, vofs[c], kind[c] == 3 ? slot + W::PAD_OFF : slot + q * 1024);
    }
  };
  // D − 1 stages in flight at the start; stage st's slot is refilled with stage st + D − 1 one stage later
#pragma unroll
  for (int st = 0; st < D - 1; st++) issue(st, st);
  [[maybe_unused]] uint64_t t_wait = 0, t_bar = 0, t_iss = 0, t_rd = 0, t0 = LK_W32_T();
  for (int st = 0; st < nst; st++) {
    [[maybe_unused]] const uint64_t tw0 = LK_W32_T();
    wait_vmcnt<(D - 2) * CW>();    // this wave's DMAs of stage st have landed (D − 2 younger stages may not)
#ifdef LK_LAB_W32_STAMPS
    asm volatile("" ::: "memory");
    const uint64_t tb = LK_W32_T();
    t_wait += tb - tw0;
#endif
    __builtin_amdgcn_s_barrier();  // ... every wave's; and every wave is done reading stage st − 1's slot
    asm volatile("" ::: "memory");
#ifdef LK_LAB_W32_STAMPS
    t_bar += LK_W32_T() - tb;
#endif
#ifdef LK_LAB_W32_STAMPS
    const uint64_t ti0 = LK_W32_T();
#endif
#if defined(LK_LAB_W32_NO_REFILL)  // skeleton (wrong results): the prologue's stages only
#elif LK_W32_ILV && LK_W32_ILDMA
    // (issued between the MFMAs below)
#elif LK_W32_SPREAD
    issue(st + D - 1, (st + D - 1) % D, 0, (CW + 1) / 2);  // refill the slot stage st − 1 used: half now,
#else
    issue(st + D - 1, (st + D - 1) % D);  // refill the slot stage st − 1 used
#endif
#ifdef LK_LAB_W32_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t ti1 = LK_W32_T();
    t_iss += ti1 - ti0;
#endif
    // LDS addresses: one per-lane base per operand kind for this slot, everything else an immediate offset
    const uint32_t sb = lds0 + (uint32_t)((st % D) * W::STAGE);
    const LK_LDS uint8_t *pw = (const LK_LDS uint8_t *)(uintptr_t)(sb + wofs_l);
    const LK_LDS uint8_t *px = (const LK_LDS uint8_t *)(uintptr_t)(sb + xofs_l);
    const LK_LDS uint8_t *pt = (const LK_LDS uint8_t *)(uintptr_t)(sb + tofs_l);
    // block G's weights of every row tile, decoded first (the raw pieces die here)
    bf16x8 w0[MT], w1[MT];
    float d[MT], mq[MT];
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const u32x4 a0 = *(const LK_LDS u32x4 *)(pw + i * 32 * W::WIN), a1 = *(const LK_LDS u32x4 *)(pw + i * 32 * W::WIN + 16);
      uint32_t c0, c1;
      float mn;
      w32_block<QT, G>(a0, a1, h, c0, c1, d[i], mn);
      w0[i] = q4_codes_128(c0);
      w1[i] = q4_codes_128(c1);
      mq[i] = mn * -0.0078125f;  // Q4_1: m·Σx = (−m/128)·T, exact
    }
    // chains c = j·MT + i, column tile major (one column tile's fragments and T live at a time),
    // software-pipelined by hand: chain c's four MFMAs are issued before chain c − 1's scale FMAs, so the
    // matrix pipe runs while the VALU scales
    bf16x8 xh[2], xl[2];
    f32x16 T;
    auto load_x = [&](int j) __attribute__((always_inline)) {
#pragma unroll
      for (int s2 = 0; s2 < 2; s2++) {
#ifdef LK_LAB_W32_HALF_X  // skeleton (wrong results): every column tile reads tile 0's fragments
        const LK_LDS uint8_t *f = px + (s2 * 2) * 1024;
#else
        const LK_LDS uint8_t *f = px + (j * W::SB * 4 + s2 * 2) * 1024;
#endif
#ifdef LK_LAB_W32_NO_XREAD  // skeleton (wrong results): fragments from registers, no LDS reads
        const uint32_t z = (uint32_t)(lane * 3 + j * 5 + s2 * 7 + st);
        xh[s2] = __builtin_bit_cast(bf16x8, u32x4{z, z ^ 1u, z ^ 2u, z ^ 3u});
        xl[s2] = __builtin_bit_cast(bf16x8, u32x4{z ^ 4u, z ^ 5u, z ^ 6u, z ^ 7u});
        (void)f;
        continue;
#endif
        xh[s2] = __builtin_bit_cast(bf16x8, *(const LK_LDS u32x4 *)f);
        xl[s2] = __builtin_bit_cast(bf16x8, *(const LK_LDS u32x4 *)(f + 1024));
      }
#ifdef LK_LAB_W32_NO_T  // skeleton (wrong results): no T reads
#pragma unroll
      for (int q = 0; q < 16; q++) T[q] = (float)(j + q);
#else
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const f32x4 v = *(const LK_LDS f32x4 *)(pt + (32 * j + 8 * q) * 4);
        T[4 * q] = v.x; T[4 * q + 1] = v.y; T[4 * q + 2] = v.z; T[4 * q + 3] = v.w;
      }
#endif
    };
    [[maybe_unused]] auto chain = [&](int i) __attribute__((always_inline)) -> f32x16 {
#ifdef LK_LAB_W32_NO_MFMA  // skeleton (wrong results): operands consumed by one VALU op, no MFMA
      f32x16 q = T;
      q[0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, xl[0]).x ^ __builtin_bit_cast(u32x4, xh[0]).y ^
                                            __builtin_bit_cast(u32x4, xl[1]).z ^ __builtin_bit_cast(u32x4, xh[1]).w ^
                                            __builtin_bit_cast(u32x4, w0[i]).x ^ __builtin_bit_cast(u32x4, w1[i]).y);
      return q;
#endif
      f32x16 p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[0], w0[i], T, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[0], w0[i], p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[1], w1[i], p, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[1], w1[i], p, 0, 0, 0);
    };
    auto scale = [&](int i, int j, const f32x16 &p, const f32x16 &t) __attribute__((always_inline)) {
#ifdef LK_LAB_W32_NO_SCALE  // skeleton (wrong results): one add per chain instead of the scale FMAs
      acc[i][j][0] += p[0] + p[15] + d[i];
      return;
#endif
#if LK_W32_PK
      // packed: 8 v_pk_fma_f32 per chain instead of 16 v_fma (the kernel is VALU-issue bound)
      const f2v dd = {d[i], d[i]};
      [[maybe_unused]] const f2v mm = {mq[i], mq[i]};
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        f2v a = {acc[i][j][r], acc[i][j][r + 1]};
        if constexpr (QT == LK_TYPE_Q4_1) a = __builtin_elementwise_fma(mm, f2v{t[r], t[r + 1]}, a);
        a = __builtin_elementwise_fma(dd, f2v{p[r], p[r + 1]}, a);
        acc[i][j][r] = a.x;
        acc[i][j][r + 1] = a.y;
      }
#else
#pragma unroll
      for (int r = 0; r < 16; r++) {
        if constexpr (QT == LK_TYPE_Q4_1) acc[i][j][r] = fmaf(mq[i], t[r], acc[i][j][r]);
        acc[i][j][r] = fmaf(d[i], p[r], acc[i][j][r]);
      }
#endif
    };
#if LK_W32_ILV
    // the MT·NT chains' MFMAs interleaved step by step (each chain's own order unchanged: the same bits),
    // so no MFMA waits on the one before it; every column tile's fragments and T live at once
    bf16x8 xhj[NT][2], xlj[NT][2];
    f32x16 Tj[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) {
      load_x(j);
      xhj[j][0] = xh[0]; xhj[j][1] = xh[1]; xlj[j][0] = xl[0]; xlj[j][1] = xl[1];
      Tj[j] = T;
    }
    f32x16 pc[MT][NT];
#if LK_W32_ILDMA && !defined(LK_LAB_W32_NO_REFILL)
    // the MFMAs in the same order, with refill DMA c issued after MFMA c (LK_W32_ILDMA 2; 1: after MFMA
    // ((c + 1)·NM)/(CW + 1) − 1): a piece issued in a burst right after the barrier costs its wave ~100
    // issue cycles, between MFMAs a fraction of that (MI355X_MICROARCH.md, LDS-DMA piece issue cost);
    // the scheduling barriers keep the compiler from regrouping them. (Between the chains' scale FMAs
    // instead: C5 53.3-53.9 us, slower.)
    constexpr int NM = 4 * MT * NT;
#pragma unroll
    for (int k = 0; k < NM; k++) {
      const int s4 = k / (MT * NT), i = (k / NT) % MT, j = k % NT;
      const bf16x8 xa = s4 == 0 ? xlj[j][0] : s4 == 1 ? xhj[j][0] : s4 == 2 ? xlj[j][1] : xhj[j][1];
      const bf16x8 wa = s4 < 2 ? w0[i] : w1[i];
      pc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, wa, s4 == 0 ? Tj[j] : pc[i][j], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < CW; c++)
        if (LK_W32_ILDMA == 1 ? ((c + 1) * NM) / (CW + 1) - 1 == k : LK_W32_ILDMA == 2 ? min(c, NM - 1) == k : false) {
          __builtin_amdgcn_sched_barrier(0);
          issue(st + D - 1, (st + D - 1) % D, c, c + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
#else
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) pc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xlj[j][0], w0[i], Tj[j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) pc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xhj[j][0], w0[i], pc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) pc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xlj[j][1], w1[i], pc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) pc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xhj[j][1], w1[i], pc[i][j], 0, 0, 0);
#endif
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
      for (int j = 0; j < NT; j++) {
        scale(i, j, pc[i][j], Tj[j]);
      }
#else
    f32x16 pa, ta;
    int pi = 0, pj = 0;
#pragma unroll
    for (int j = 0; j < NT; j++) {
#if LK_W32_SPREAD
      if (j == NT - 1) issue(st + D - 1, (st + D - 1) % D, (CW + 1) / 2, CW);  // ... half with the last column tile
#endif
      load_x(j);
#pragma unroll
      for (int i = 0; i < MT; i++) {
        const f32x16 pb = chain(i);
        if (j + i > 0) scale(pi, pj, pa, ta);
        pa = pb;
        ta = T;
        pi = i;
        pj = j;
      }
    }
    scale(MT - 1, NT - 1, pa, ta);
#endif
#if LK_W32_SCHED
    // one MFMA, then its share of the VALU (decode + scale FMAs), so the VALU issues in the MFMAs' shadow
#pragma unroll
    for (int q = 0; q < 4 * MT * NT; q++) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, LK_W32_SCHED, 0);
    }
#endif
  }
  wait_vmcnt<0>();  // the padding stages, before the ring is reused for the reduction
#ifdef LK_LAB_W32_STAMPS
  if (lane == 0 && blockIdx.x < 1024) {
    uint64_t *o = lk_w32_stamps[blockIdx.x][wave];
    o[0] = t0; o[1] = LK_W32_T(); o[2] = t_wait; o[3] = t_bar; o[4] = (uint64_t)nst; o[5] = t_iss;
  }
#endif
}

// Two row halves in ping-pong (MH = 2, round 6): each SIMD holds one wave of each half, and the halves
// alternate between an operand phase (the stage's LDS reads and code decode into registers) and a matrix
// phase (the stage's MFMAs and scale FMAs from those registers), two workgroup barriers per stage. While
// one half's wave reads LDS and decodes, the other half's wave on the same SIMD has the matrix pipe to
// itself, instead of both reading, then both queueing for the MFMAs, then both waiting at one barrier.
//   even barrier (stage st): half 0 reads stage st; half 1 multiplies stage st − 1
//   odd barrier:             half 0 multiplies stage st; half 1 reads stage st
// Stage st's slot is read in the even interval (half 0) and the odd one (half 1), so the refill issued
// after the next even barrier may overwrite it; a half waits for its own LDS reads before that barrier.
template <int QT, int MT, int NT, int MH, int G>
__device__ __forceinline__ void w32_main_pp(const W32Args &g, uint8_t *smem, int tm, int tn, int st0, int st1, int wave, int mh,
                                            f32x16 (&acc)[MT][NT]) {
  using W = W32Geom<QT, MT, NT, MH>;
  constexpr int D = W::D, CW = W::CW;
  const int lane = threadIdx.x & 63, h = lane >> 5, m = lane & 31;
  const int nblk = g.K / 32, ntx = (g.N + 31) / 32, n32 = ntx * 32;
  const int64_t RB = (int64_t)nblk * W::BB;
  const int nst = st1 - st0;
  uint32_t vofs[CW];
  int kind[CW];  // 0 weights, 1 fragments, 2 T, 3 padding (wave-uniform)
#pragma unroll
  for (int c = 0; c < CW; c++) {
    const int q = wave * CW + c;
    if (q < W::W_INST) {
      const int p = min(q * 64 + lane, W::BM * W::WP - 1), r = p / W::WP, pc = p % W::WP;
      const int64_t row = min((int64_t)tm * W::BM + r, (int64_t)g.M - 1);
      vofs[c] = (uint32_t)(row * RB + pc * 16);
      kind[c] = 0;
    } else if (q < W::W_INST + W::X_INST) {
      const int f = q - W::W_INST, j = f / (W::SB * 4), b = (f / 4) % W::SB, s = (f / 2) % 2, sp = f % 2;
      const int64_t xt = min(tn * NT + j, ntx - 1);
      vofs[c] = (uint32_t)(((((xt * nblk + b) * 2 + s) * 2 + sp) * 64 + lane) * 16);
      kind[c] = 1;
    } else if (q == W::W_INST + W::X_INST) {
      const int b = min(lane / (W::BN / 4), W::SB - 1), c4 = lane % (W::BN / 4);
      const int col = min(tn * W::BN + 4 * c4, n32 - 4);
      vofs[c] = (uint32_t)(((int64_t)b * n32 + col) * 4);
      kind[c] = 2;
    } else {
      vofs[c] = 0;
      kind[c] = 3;
    }
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LK_LDS const void *)smem);
  const uint32_t wofs_l = (uint32_t)((mh * MT * 32 + m) * W::WIN + G * 16), xofs_l = (uint32_t)(W::X_OFF + G * 4 * 1024 + lane * 16),
                 tofs_l = (uint32_t)(W::T_OFF + (G * W::BN + 4 * h) * 4);
  auto issue = [&](int st, int sl) __attribute__((always_inline)) {
    const int kb = (st0 + min(st, nst - 1)) * W::SB;  // past the last stage: reload it (never read)
    const uint8_t *bw = g.a + (int64_t)kb * W::BB;
    const uint8_t *bx = (const uint8_t *)g.frag + (int64_t)kb * 4 * 1024;
    const uint8_t *bt = (const uint8_t *)(g.tsum + (int64_t)kb * n32);
    const uint32_t slot = lds0 + (uint32_t)(sl * W::STAGE);
#pragma unroll
    for (int c = 0; c < CW; c++) {
      const int q = wave * CW + c;
      const uint8_t *base = kind[c] == 0 ? bw : kind[c] == 1 ? bx : bt;
      dma16m(base, vofs[c], kind[c] == 3 ? slot + W::PAD_OFF : slot + q * 1024);
    }
  };
  // the operands of one stage, held from the operand phase to the matrix phase
  bf16x8 w0[MT], w1[MT], xh[NT][2], xl[NT][2];
  float d[MT], mq[MT];
  f32x16 T[NT];
  auto operands = [&](int st) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((st % D) * W::STAGE);
    const LK_LDS uint8_t *pw = (const LK_LDS uint8_t *)(uintptr_t)(sb + wofs_l);
    const LK_LDS uint8_t *px = (const LK_LDS uint8_t *)(uintptr_t)(sb + xofs_l);
    const LK_LDS uint8_t *pt = (const LK_LDS uint8_t *)(uintptr_t)(sb + tofs_l);
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const u32x4 a0 = *(const LK_LDS u32x4 *)(pw + i * 32 * W::WIN), a1 = *(const LK_LDS u32x4 *)(pw + i * 32 * W::WIN + 16);
      uint32_t c0, c1;
      float mn;
      w32_block<QT, G>(a0, a1, h, c0, c1, d[i], mn);
      w0[i] = q4_codes_128(c0);
      w1[i] = q4_codes_128(c1);
      mq[i] = mn * -0.0078125f;  // Q4_1: m·Σx = (−m/128)·T, exact
    }
#pragma unroll
    for (int j = 0; j < NT; j++) {
#pragma unroll
      for (int s2 = 0; s2 < 2; s2++) {
        const LK_LDS uint8_t *f = px + (j * W::SB * 4 + s2 * 2) * 1024;
        xh[j][s2] = __builtin_bit_cast(bf16x8, *(const LK_LDS u32x4 *)f);
        xl[j][s2] = __builtin_bit_cast(bf16x8, *(const LK_LDS u32x4 *)(f + 1024));
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const f32x4 v = *(const LK_LDS f32x4 *)(pt + (32 * j + 8 * q) * 4);
        T[j][4 * q] = v.x; T[j][4 * q + 1] = v.y; T[j][4 * q + 2] = v.z; T[j][4 * q + 3] = v.w;
      }
    }
    wait_lgkmcnt0();  // this half's reads of the slot are done before the barrier that may refill it
  };
  auto matrix = [&]() __attribute__((always_inline)) {
    auto chain = [&](int i, int j) __attribute__((always_inline)) -> f32x16 {
      f32x16 p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[j][0], w0[i], T[j], 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[j][0], w0[i], p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[j][1], w1[i], p, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[j][1], w1[i], p, 0, 0, 0);
    };
    auto scale = [&](int i, int j, const f32x16 &p) __attribute__((always_inline)) {
      const f2v dd = {d[i], d[i]};
      [[maybe_unused]] const f2v mm = {mq[i], mq[i]};
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        f2v a = {acc[i][j][r], acc[i][j][r + 1]};
        if constexpr (QT == LK_TYPE_Q4_1) a = __builtin_elementwise_fma(mm, f2v{T[j][r], T[j][r + 1]}, a);
        a = __builtin_elementwise_fma(dd, f2v{p[r], p[r + 1]}, a);
        acc[i][j][r] = a.x;
        acc[i][j][r + 1] = a.y;
      }
    };
    // chain c's MFMAs issued before chain c − 1's scale FMAs (hand pipelining, as w32_main)
    f32x16 pa;
    int pi = 0, pj = 0;
#pragma unroll
    for (int j = 0; j < NT; j++)
#pragma unroll
      for (int i = 0; i < MT; i++) {
        const f32x16 pb = chain(i, j);
        if (j + i > 0) scale(pi, pj, pa);
        pa = pb;
        pi = i;
        pj = j;
      }
    scale(MT - 1, NT - 1, pa);
  };
#pragma unroll
  for (int st = 0; st < D - 1; st++) issue(st, st);
  // one loop per half (the same barrier count), so each keeps its operands in place across iterations
  [[maybe_unused]] uint64_t t_op = 0, t_mx = 0, t_bar = 0, t_iss = 0, t0 = LK_W32_T(), ta;
#ifdef LK_LAB_W32_STAMPS
#define LK_PP_ACC(v) do { asm volatile("" ::: "memory"); const uint64_t tb_ = LK_W32_T(); v += tb_ - ta; ta = tb_; } while (0)
#define LK_PP_MX() do { asm volatile("s_nop 0" ::: "memory"); } while (0)
#else
#define LK_PP_ACC(v) do { } while (0)
#define LK_PP_MX() do { } while (0)
#endif
  ta = t0;
  if (mh == 0) {
    for (int st = 0; st < nst; st++) {
      wait_vmcnt<(D - 2) * CW>();  // this wave's DMAs of stage st have landed
      __builtin_amdgcn_s_barrier();  // ... every wave's; both halves are done with stage st − 1's slot
      asm volatile("" ::: "memory");
      LK_PP_ACC(t_bar);
      issue(st + D - 1, (st + D - 1) % D);
      LK_PP_ACC(t_iss);
      operands(st);
      LK_PP_ACC(t_op);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      LK_PP_ACC(t_bar);
      matrix();  // stage st
#ifdef LK_LAB_W32_STAMPS
      { float z = 0.f; for (int i = 0; i < MT; i++) for (int j = 0; j < NT; j++) z += acc[i][j][0]; asm volatile("" :: "v"(z)); }
#endif
      LK_PP_ACC(t_mx);
    }
  } else {
    for (int st = 0; st < nst; st++) {
      wait_vmcnt<(D - 2) * CW>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      LK_PP_ACC(t_bar);
      issue(st + D - 1, (st + D - 1) % D);
      LK_PP_ACC(t_iss);
      if (st > 0) matrix();  // stage st − 1
#ifdef LK_LAB_W32_STAMPS
      { float z = 0.f; for (int i = 0; i < MT; i++) for (int j = 0; j < NT; j++) z += acc[i][j][0]; asm volatile("" :: "v"(z)); }
#endif
      LK_PP_ACC(t_mx);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      LK_PP_ACC(t_bar);
      operands(st);
      LK_PP_ACC(t_op);
    }
    if (nst > 0) matrix();  // the last stage
  }
#undef LK_PP_ACC
#undef LK_PP_MX
  wait_vmcnt<0>();
#ifdef LK_LAB_W32_STAMPS
  if (lane == 0 && blockIdx.x < 1024) {
    uint64_t *o = lk_w32_stamps[blockIdx.x][wave];
    o[0] = t0; o[1] = LK_W32_T(); o[2] = t_op; o[3] = t_bar; o[4] = (uint64_t)nst; o[5] = t_iss; o[6] = t_mx;
  }
#endif  // the padding stages, before the ring is reused for the reduction
}

template <int QT, int MT, int NT, int MH>
__global__ __launch_bounds__(256 * MH, MH) void gemm_w32_kernel(W32Args g) {
  using W = W32Geom<QT, MT, NT, MH>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), kg = wave & 3, mh = wave >> 2;
#if LK_W32_PRIO
  if (mh) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half loses arbitration (MI355X_MICROARCH.md)
#endif
  // task order (speed only: dispatch is observed round-robin over the 8 XCDs): workgroup b runs task
  // (b % 8)·(grid / 8) + b / 8, so each XCD takes a contiguous run of tasks. Tiles are ordered in groups
  // of bc column tiles: group, then row tile, then column tile within the group, then slice — a run of
  // tasks covers a block of row tiles x bc column tiles, whose weight windows and activation fragments
  // the XCD's L2 serves to its CUs (bc = 1: a run walks the row tiles of one column tile and every XCD
  // re-fetches all the weights; C5 FETCH_SIZE x 2 86.6 MB per dispatch)
  const int task = ((int)blockIdx.x % 8) * ((int)gridDim.x / 8) + (int)blockIdx.x / 8;
  if (task >= g.tasks) return;  // grid padding
  const int slice = task % g.slices, tile = task / g.slices;
  const int grp = tile / (g.tiles_m * g.bc), rem = tile - grp * g.tiles_m * g.bc;
  const int bcg = min(g.bc, g.tiles_n - grp * g.bc);  // the last group may be narrower
  const int tm = rem / bcg, tn = grp * g.bc + rem % bcg;
  const int nst = g.K / 32 / W::SB;
  const int st0 = slice * g.sstages, st1 = min(st0 + g.sstages, nst);
  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; i++)
#pragma unroll
    for (int j = 0; j < NT; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
  if (st1 > st0) {
    switch (kg) {  // K group: its block's offsets are compile-time constants
#define LK_W32_MAIN(GG)                                                                   \
  if constexpr (MH == 2 && LK_W32_PP) w32_main_pp<QT, MT, NT, MH, GG>(g, smem, tm, tn, st0, st1, wave, mh, acc); \
  else w32_main<QT, MT, NT, MH, GG>(g, smem, tm, tn, st0, st1, wave, mh, acc);
      case 0: LK_W32_MAIN(0) break;
      case 1: LK_W32_MAIN(1) break;
      case 2: LK_W32_MAIN(2) break;
      default: LK_W32_MAIN(3) break;
#undef LK_W32_MAIN
    }
  }
  // K groups summed in group order: chain c = i·NT + j of row half mh is finished by wave mh·4 + c % 4;
  // every wave parks its chains in LDS ([half][chain][group] x 4 KB, lane-major float4s)
  constexpr int CH = W::CHAINS;
  __syncthreads();
  f32x4 *red = (f32x4 *)smem;
#pragma unroll
  for (int c = 0; c < CH; c++) {
    f32x4 *o = red + ((mh * CH + c) * 4 + kg) * 256 + lane;
#pragma unroll
    for (int q = 0; q < 4; q++) o[q * 64] = f32x4{acc[c / NT][c % NT][4 * q], acc[c / NT][c % NT][4 * q + 1], acc[c / NT][c % NT][4 * q + 2], acc[c / NT][c % NT][4 * q + 3]};
  }
  __syncthreads();
  constexpr int OWN = (CH + 3) / 4;  // chains finished per wave (at most)
  f32x4 sum[OWN][4];
#pragma unroll
  for (int oc = 0; oc < OWN; oc++) {
    const int c = oc * 4 + kg;
    if (c >= CH) break;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int gk = 0; gk < 4; gk++) {
        const f32x4 p = red[((mh * CH + c) * 4 + gk) * 256 + q * 64 + lane];
        if (gk == 0) v = p;  // group 0 as is (0 + x would turn −0.0 into +0.0)
        else { v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w; }
      }
      sum[oc][q] = v;
    }
  }
  auto store_chain = [&](int c, const f32x4 (&s)[4]) __attribute__((always_inline)) {
    const int i = c / NT, j = c % NT;
    const int64_t mrow = (int64_t)tm * W::BM + 32 * (mh * MT + i) + (lane & 31);
    if (mrow >= g.M) return;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int n0 = tn * W::BN + 32 * j + 8 * q + 4 * h;  // C rows 8q + 4h .. + 3 of the chain
      uint8_t *o = g.dst + mrow * g.d_nb1 + (int64_t)n0 * g.d_nb0;
      if (g.d_nb0 == 4 && n0 + 4 <= g.N && (((uintptr_t)o) & 15) == 0) {
        *(f32x4 *)o = s[q];
      } else {
        const float e[4] = {s[q].x, s[q].y, s[q].z, s[q].w};
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (n0 + u < g.N) *(float *)(o + u * g.d_nb0) = e[u];
      }
    }
  };
  if (g.slices == 1) {
#pragma unroll
    for (int oc = 0; oc < OWN; oc++)
      if (oc * 4 + kg < CH) store_chain(oc * 4 + kg, sum[oc]);
    return;
  }
  // split K: this slice's tile written through (sc1), every wave drained, one agent-scope arrival; the
  // last slice to arrive sums the slabs in slice order (its own from registers) with sc1 loads and stores
  // (splitk_arrive re-arms the counter). Nobody waits for another workgroup.
  const int64_t tiles = (int64_t)g.tiles_m * g.tiles_n;
  const int64_t slab = (int64_t)W::BM * W::BN;  // floats per tile
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)g.partial, 0, (int)((int64_t)g.slices * tiles * slab * 4), 0x00020000);
  auto at = [&](int sl, int c, int q) __attribute__((always_inline)) {  // a lane's float4 of chain c of half mh
    return (int)((((int64_t)sl * tiles + tile) * slab + ((int64_t)(mh * CH + c) * 4 + q) * 256 + 4 * lane) * 4);
  };
#pragma unroll
  for (int oc = 0; oc < OWN; oc++)
    if (oc * 4 + kg < CH)
#pragma unroll
      for (int q = 0; q < 4; q++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sum[oc][q]), prs, at(slice, oc * 4 + kg, q), 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int *flag = (int *)smem + 64 * 1024 / 4;  // inside the reduction buffer, every read of which is done
  if (threadIdx.x == 0) *flag = splitk_arrive(g.tcnt + (int64_t)tile * kChainLine, (unsigned)g.slices) ? 1 : 0;
  __syncthreads();
  asm volatile("" ::: "memory");
  if (!*flag) return;
#pragma unroll
  for (int oc = 0; oc < OWN; oc++) {
    const int c = oc * 4 + kg;
    if (c >= CH) break;
    f32x4 t[4];
    for (int sl = 0; sl < g.slices; sl++) {
      f32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; q++)
        v[q] = sl == slice ? sum[oc][q] : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, at(sl, c, q), 0, 16));
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (sl == 0) t[q] = v[q];
        else { t[q].x += v[q].x; t[q].y += v[q].y; t[q].z += v[q].z; t[q].w += v[q].w; }
      }
    }
    store_chain(c, t);
  }
}

#endif  // LK_W32_KERNELS

// Launchers (lk_w32.hip): enqueue on `st`; hipGetLastError is the caller's.
void w32_launch_xsplit(const XSplit32Args &xa, unsigned items, hipStream_t st);  // items = column tiles x blocks
void w32_launch(int qt, int mt, int nt, int mh, const W32Args &g, unsigned grid, size_t lds, hipStream_t st);

}  // namespace lk
