// lab.hip — micro-benchmark lab for the batch-1 Q4_0 GEMV (not part of the product).
//
// Times, on one stream with hipEvents, launches over COPIES distinct 4096x4096 Q4_0 weight
// matrices (COPIES x 9.4 MB > 256 MiB Infinity Cache), in two regimes:
//   per-launch : one launch per matrix, rotating (launch boundaries included)
//   one launch : a single launch over all copies as one tall matrix (steady-state rate)
// Variants:
//   prod : the production kernel (C-ABI lk_mul_mat_device for per-launch)
//   X0   : pure coalesced float4 read of the same bytes (achievable read BW)
//   A<RG>: lane = one quant dword (8 weights) of a block: unaligned dword + ushort scale
//          loads (16 consecutive blocks per wave instruction), x read coalesced from L1
//          (2 x float4 per lane per 512-k chunk), RG rows per group, optional prefetch.
// Build/run: tools/lab/run_lab.sh (on the GPU box).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../llama.kotlin_amd/csrc/lk_kernels.hpp"

using namespace lk;

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

constexpr int M = 4096, K = 4096, BB = 18;
constexpr int RB = K / 32 * BB;
constexpr size_t MAT_BYTES = (size_t)M * RB;
constexpr size_t ALG_BYTES = MAT_BYTES + 4 * K + 4 * M;
typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint16_t u16_ua __attribute__((aligned(1)));

__global__ void fill_blocks(uint8_t *p, size_t nblk, uint32_t seed) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  uint8_t *q = p + b * BB;
  uint32_t s = (uint32_t)b * 2654435761u ^ seed;
  q[0] = 0x00; q[1] = 0x24;  // f16 0.015625
  for (int i = 0; i < 16; i++) { s = s * 1664525u + 1013904223u; q[2 + i] = (uint8_t)(s >> 24); }
}

__global__ void x0_read(const f32x4 *__restrict__ p, size_t n4, float *out) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    f32x4 v = __builtin_nontemporal_load(p + i);
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 123.456f) out[0] = acc;
}

__device__ __forceinline__ uint32_t opaque(uint32_t v) { asm volatile("" : "+v"(v)); return v; }
__device__ __forceinline__ float ubf(uint32_t v, int n) { return (float)((v >> (8 * n)) & 0xFFu); }

// Σ nibble_n(q)·x[n], n = 0..7 (weights 8t..8t+7 of a block), scalar FMAs in two chains
__device__ __forceinline__ float nib8(uint32_t q, const float *x) {
  const uint32_t lo = opaque(q & 0x0F0F0F0Fu), hi = opaque((q >> 4) & 0x0F0F0F0Fu);
  float s0 = ubf(lo, 0) * x[0], s1 = ubf(hi, 0) * x[1];
  s0 = fmaf(ubf(lo, 1), x[2], s0); s1 = fmaf(ubf(hi, 1), x[3], s1);
  s0 = fmaf(ubf(lo, 2), x[4], s0); s1 = fmaf(ubf(hi, 2), x[5], s1);
  s0 = fmaf(ubf(lo, 3), x[6], s0); s1 = fmaf(ubf(hi, 3), x[7], s1);
  return s0 + s1;
}

template <int RG, bool PREF>
__global__ __launch_bounds__(256) void a_dword(const uint8_t *__restrict__ a, const float *__restrict__ x,
                                               float *__restrict__ dst, int Mrows, int rpw) {
  constexpr int NC = K / 512;  // 512-weight chunks per row (16 blocks each)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * 4 + wave) * rpw;
  const int sub = lane & 3, bl = lane >> 2;
  const LK_GLOBAL uint8_t *A = (const LK_GLOBAL uint8_t *)a;
  uint32_t q[2][RG][NC], sc[2][RG][NC];
  auto load = [&](int buf, int g) {
#pragma unroll
    for (int r = 0; r < RG; r++) {
      const int row = min(row0 + g * RG + r, Mrows - 1);
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const LK_GLOBAL uint8_t *blk = A + (size_t)row * RB + (size_t)(16 * c + bl) * BB;
        q[buf][r][c] = __builtin_nontemporal_load((const LK_GLOBAL u32_ua *)(blk + 2 + 4 * sub));
        sc[buf][r][c] = __builtin_nontemporal_load((const LK_GLOBAL u16_ua *)blk);
      }
    }
  };
  const int ng = rpw / RG;
  load(0, 0);
#pragma unroll 1
  for (int g = 0; g < ng; g++) {
    const int cur = PREF ? (g & 1) : 0;
    if (PREF && g + 1 < ng) load(cur ^ 1, g + 1);
    float acc[RG];
#pragma unroll
    for (int r = 0; r < RG; r++) acc[r] = 0.f;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)((const LK_GLOBAL float *)x + 512 * c + 8 * lane);
      const f32x4 u = xv[0], v = xv[1];
      const float xx[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      const float xs = ((u.x + u.y) + (u.z + u.w)) + ((v.x + v.y) + (v.z + v.w));
#pragma unroll
      for (int r = 0; r < RG; r++) {
        const float s = nib8(q[cur][r][c], xx);
        acc[r] = fmaf(h2f(sc[cur][r][c]), fmaf(-8.f, xs, s), acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < RG; r++) {
      const float v = wave_sum(acc[r]);
      if (lane == 0 && row0 + g * RG + r < Mrows) dst[row0 + g * RG + r] = v;
    }
    if (!PREF && g + 1 < ng) load(0, g + 1);
  }
}


// ---- V4: pair per lane, x staged once per workgroup in LDS (permuted for v_pk_fma), fp8 decode
typedef float f2v __attribute__((ext_vector_type(2)));
template <bool HI> __device__ __forceinline__ f2v fp8x2(uint32_t v) { return __builtin_amdgcn_cvt_pk_f32_fp8(v, HI); }
// Σ (q_n/512)·x_n for the 8 nibbles of u; xa = (x0,x2,x4,x6), xb = (x1,x3,x5,x7)
__device__ __forceinline__ f2v nib8_fp8(uint32_t u, f32x4 xa, f32x4 xb, f2v s) {
  const uint32_t lo = u & 0x0F0F0F0Fu, hi = (u >> 4) & 0x0F0F0F0Fu;
  s = __builtin_elementwise_fma(fp8x2<false>(lo), f2v{xa.x, xa.y}, s);
  s = __builtin_elementwise_fma(fp8x2<true>(lo), f2v{xa.z, xa.w}, s);
  s = __builtin_elementwise_fma(fp8x2<false>(hi), f2v{xb.x, xb.y}, s);
  s = __builtin_elementwise_fma(fp8x2<true>(hi), f2v{xb.z, xb.w}, s);
  return s;
}
template <int RG, bool PREF>
__global__ __launch_bounds__(256) void v4_kernel(const uint8_t *__restrict__ a, const float *__restrict__ x,
                                                 float *__restrict__ dst, int Mrows, int rpw) {
  constexpr int NP = K / 64, PITCH = NP + 1, XS = NP * 16 / 256;
  extern __shared__ f32x4 lds[];
  float *lds_sum = (float *)(lds + 16 * PITCH);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = (blockIdx.x * 4 + wave) * rpw;
  const int ng = rpw / RG;
  const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)x;
  f32x4 xq[XS];
#pragma unroll
  for (int i = 0; i < XS; i++) xq[i] = xv[tid + 256 * i];
  const LK_GLOBAL uint8_t *A = (const LK_GLOBAL uint8_t *)a;
  const uint32_t loff = (uint32_t)lane * 36u;
  uint32_t wa[RG][9], wb[RG][9];
  auto load = [&](uint32_t (&w)[RG][9], int g) {
#pragma unroll
    for (int r = 0; r < RG; r++) {
      const int row = __builtin_amdgcn_readfirstlane(min(row0 + g * RG + r, Mrows - 1));
      const LK_GLOBAL uint8_t *rp = A + (size_t)row * RB;
      const LK_GLOBAL uint32_t *src = (const LK_GLOBAL uint32_t *)(rp + loff);
#pragma unroll
      for (int t = 0; t < 9; t++) w[r][t] = __builtin_nontemporal_load(src + t);
    }
  };
  load(wa, 0);
  // x image: slot (s, p) = 4 floats; per 8-weight dword jj of pair p: s = 2jj holds (x0,x2,x4,x6), 2jj+1 (x1,x3,x5,x7)
#pragma unroll
  for (int i = 0; i < XS; i++) {
    const int q = tid + 256 * i;            // float4 index: elements 4q..4q+3
    const int p = q >> 4, jj = (q & 15) >> 1, h = q & 1;
    const f32x4 v = xq[i];
    f2v *sa = (f2v *)(lds + (2 * jj) * PITCH + p) + h;
    f2v *sb = (f2v *)(lds + (2 * jj + 1) * PITCH + p) + h;
    *sa = f2v{v.x, v.z};
    *sb = f2v{v.y, v.w};
    float s = (v.x + v.y) + (v.z + v.w);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((q & 7) == 0) lds_sum[2 * p + ((q >> 3) & 1)] = s;
  }
  __syncthreads();
  const int p = lane;
  const float xs0 = lds_sum[2 * p], xs1 = lds_sum[2 * p + 1];
  auto compute = [&](const uint32_t (&w)[RG][9], int g) {
    float acc[RG];
    f32x4 xa[8];
#pragma unroll
    for (int t = 0; t < 8; t++) xa[t] = lds[t * PITCH + p];
#pragma unroll
    for (int r = 0; r < RG; r++) {
      f2v s = {0.f, 0.f};
      s = nib8_fp8(align2(w[r][1], w[r][0]), xa[0], xa[1], s);
      s = nib8_fp8(align2(w[r][2], w[r][1]), xa[2], xa[3], s);
      s = nib8_fp8(align2(w[r][3], w[r][2]), xa[4], xa[5], s);
      s = nib8_fp8(align2(w[r][4], w[r][3]), xa[6], xa[7], s);
      acc[r] = h2f(w[r][0]) * fmaf(512.f, s.x + s.y, -8.f * xs0);
    }
#pragma unroll
    for (int t = 0; t < 8; t++) xa[t] = lds[(t + 8) * PITCH + p];
#pragma unroll
    for (int r = 0; r < RG; r++) {
      f2v s = {0.f, 0.f};
      s = nib8_fp8(w[r][5], xa[0], xa[1], s);
      s = nib8_fp8(w[r][6], xa[2], xa[3], s);
      s = nib8_fp8(w[r][7], xa[4], xa[5], s);
      s = nib8_fp8(w[r][8], xa[6], xa[7], s);
      acc[r] = fmaf(h2f(w[r][4] >> 16), fmaf(512.f, s.x + s.y, -8.f * xs1), acc[r]);
      const float v = wave_sum(acc[r]);
      if (lane == 0 && row0 + g * RG + r < Mrows) dst[row0 + g * RG + r] = v;
    }
  };
  if (PREF) {
    int g = 0;
    for (; g + 1 < ng; g += 2) {
      load(wb, g + 1);
      compute(wa, g);
      if (g + 2 < ng) load(wa, g + 2);
      compute(wb, g + 1);
    }
    if (g < ng) compute(wa, g);
  } else {
    for (int g = 0; g < ng; g++) {
      if (g) load(wa, g);
      compute(wa, g);
    }
  }
}


// ---- S: LDS-DMA weight stream. WG = 8 waves, each wave owns a contiguous row range and a ring
// of D row slots (3 KB each: 2304 B of a K=4096 Q4_0 row) filled by global_load_lds (1 KB per
// wave instruction, no VGPRs); x for the lane's pair lives in registers (staged once via LDS).
template <int D>
__global__ __launch_bounds__(512) void s_kernel(const uint8_t *__restrict__ a, const float *__restrict__ x,
                                                float *__restrict__ dst, int Mrows) {
  constexpr int NP = K / 64, PITCH = NP + 1, SLOT = 3072;
  extern __shared__ f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // rows of this workgroup / wave (contiguous ranges)
  const int per_wg = (Mrows + gridDim.x - 1) / gridDim.x;
  const int wg0 = blockIdx.x * per_wg, wg1 = min(wg0 + per_wg, Mrows);
  const int per_w = (max(wg1 - wg0, 0) + 7) / 8;
  const int r0 = __builtin_amdgcn_readfirstlane(wg0 + wave * per_w);
  const int r1 = __builtin_amdgcn_readfirstlane(min(r0 + per_w, wg1));
  const int nrows = max(r1 - r0, 0);
  uint8_t *ring = (uint8_t *)(lds + 16 * PITCH) + wave * D * SLOT;
  const uint8_t *A = a + (size_t)r0 * RB;
  auto issue = [&](int i) {  // DMA row r0+i into slot i % D
    const uint8_t *src = A + (size_t)i * RB + lane * 16;
    uint8_t *s = ring + (i % D) * SLOT;
    __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)src, (__attribute__((address_space(3))) void *)s, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(src + 1024), (__attribute__((address_space(3))) void *)(s + 1024), 16, 0, 0);
    if (lane < 16)
      __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(src + 2048), (__attribute__((address_space(3))) void *)(s + 2048), 16, 0, 0);
  };
  // prologue: weights first, then x
  const int npre = min(D, nrows);
  for (int i = 0; i < npre; i++) issue(i);
  // x image (whole WG), then x for this lane's pair into registers
  {
    const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)x;
    for (int q = tid; q < NP * 16; q += 512) {
      const int p = q >> 4, jj = (q & 15) >> 1, h = q & 1;
      const f32x4 v = xv[q];
      f2v *sa = (f2v *)(lds + (2 * jj) * PITCH + p) + h;
      f2v *sb = (f2v *)(lds + (2 * jj + 1) * PITCH + p) + h;
      *sa = f2v{v.x, v.z};
      *sb = f2v{v.y, v.w};
    }
  }
  __syncthreads();
  f32x4 xr[16];
#pragma unroll
  for (int t = 0; t < 16; t++) xr[t] = lds[t * PITCH + lane];
  float xs0 = 0.f, xs1 = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) { xs0 += (xr[t].x + xr[t].y) + (xr[t].z + xr[t].w); xs1 += (xr[t + 8].x + xr[t + 8].y) + (xr[t + 8].z + xr[t + 8].w); }
  for (int i = 0; i < nrows; i++) {
    const int ahead = min(D - 1, nrows - 1 - i);  // rows issued after row i still in flight
    // wait for row i's 3 pieces: at most 3*ahead younger DMA ops may remain
    if (ahead >= D - 1) __builtin_amdgcn_s_waitcnt((3 * (D - 1)) & 0xF | 0x0F70 | ((((3 * (D - 1)) >> 4) & 3) << 14));
    else __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) in the tail
    const uint32_t *rp = (const uint32_t *)(ring + (i % D) * SLOT + lane * 36);
    uint32_t w[9];
#pragma unroll
    for (int t = 0; t < 9; t++) w[t] = rp[t];
    f2v s = {0.f, 0.f}, u = {0.f, 0.f};
    s = nib8_fp8(align2(w[1], w[0]), xr[0], xr[1], s);
    s = nib8_fp8(align2(w[2], w[1]), xr[2], xr[3], s);
    s = nib8_fp8(align2(w[3], w[2]), xr[4], xr[5], s);
    s = nib8_fp8(align2(w[4], w[3]), xr[6], xr[7], s);
    u = nib8_fp8(w[5], xr[8], xr[9], u);
    u = nib8_fp8(w[6], xr[10], xr[11], u);
    u = nib8_fp8(w[7], xr[12], xr[13], u);
    u = nib8_fp8(w[8], xr[14], xr[15], u);
    float acc = h2f(w[0]) * fmaf(512.f, s.x + s.y, -8.f * xs0);
    acc = fmaf(h2f(w[4] >> 16), fmaf(512.f, u.x + u.y, -8.f * xs1), acc);
    const float v = wave_sum(acc);
    if (lane == 0) dst[r0 + i] = v;
    if (i + D < nrows) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): our LDS reads of this slot are done
      issue(i + D);
    }
  }
}


// DPP reduction over the 64 lanes (VALU only; lane 63 ends with the total)
__device__ __forceinline__ float dpp_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));  // quad_perm [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true)); // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true)); // row_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false)); // row_bcast:15
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false)); // row_bcast:31
  return v;
}

// S2: S + DPP reduction + RPI rows per loop iteration; NW waves per workgroup
template <int D, int NW, int RPI>
__global__ __launch_bounds__(NW * 64) void s2_kernel(const uint8_t *__restrict__ a, const float *__restrict__ x,
                                                     float *__restrict__ dst, int Mrows) {
  constexpr int NP = K / 64, PITCH = NP + 1, SLOT = 3072;
  extern __shared__ f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_wg = (Mrows + gridDim.x - 1) / gridDim.x;
  const int wg0 = blockIdx.x * per_wg, wg1 = min(wg0 + per_wg, Mrows);
  const int per_w = ((max(wg1 - wg0, 0) + NW - 1) / NW + RPI - 1) / RPI * RPI;
  const int r0 = __builtin_amdgcn_readfirstlane(min(wg0 + wave * per_w, wg1));
  const int r1 = __builtin_amdgcn_readfirstlane(min(r0 + per_w, wg1));
  const int nrows = max(r1 - r0, 0);
  uint8_t *ring = (uint8_t *)(lds + 16 * PITCH) + wave * D * RPI * SLOT;
  const uint8_t *A = a + (size_t)r0 * RB;
  const int last = max(nrows - 1, 0);
  auto issue = [&](int u) {  // DMA rows u*RPI .. +RPI-1 (clamped) into unit slot u % D
#pragma unroll
    for (int k = 0; k < RPI; k++) {
      const uint8_t *src = A + (size_t)min(u * RPI + k, last) * RB + lane * 16;
      uint8_t *s = ring + ((u % D) * RPI + k) * SLOT;
      __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)src, (__attribute__((address_space(3))) void *)s, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(src + 1024), (__attribute__((address_space(3))) void *)(s + 1024), 16, 0, 0);
      if (lane < 16)
        __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(src + 2048), (__attribute__((address_space(3))) void *)(s + 2048), 16, 0, 0);
    }
  };
  const int nunits = (nrows + RPI - 1) / RPI;
  const int npre = min(D, nunits);
  for (int u = 0; u < npre; u++) issue(u);
  {
    const LK_GLOBAL f32x4 *xv = (const LK_GLOBAL f32x4 *)x;
    for (int q = tid; q < NP * 16; q += NW * 64) {
      const int p = q >> 4, jj = (q & 15) >> 1, h = q & 1;
      const f32x4 v = xv[q];
      f2v *sa = (f2v *)(lds + (2 * jj) * PITCH + p) + h;
      f2v *sb = (f2v *)(lds + (2 * jj + 1) * PITCH + p) + h;
      *sa = f2v{v.x, v.z};
      *sb = f2v{v.y, v.w};
    }
  }
  __syncthreads();
  f32x4 xr[16];
#pragma unroll
  for (int t = 0; t < 16; t++) xr[t] = lds[t * PITCH + lane];
  float xs0 = 0.f, xs1 = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) { xs0 += (xr[t].x + xr[t].y) + (xr[t].z + xr[t].w); xs1 += (xr[t + 8].x + xr[t + 8].y) + (xr[t + 8].z + xr[t + 8].w); }
  constexpr int PER_UNIT = 3 * RPI;  // DMA instructions per unit
  for (int u = 0; u < nunits; u++) {
    const int ahead = min(D - 1, nunits - 1 - u);
    if (ahead >= D - 1) __builtin_amdgcn_s_waitcnt(((PER_UNIT * (D - 1)) & 0xF) | 0x0F70 | ((((PER_UNIT * (D - 1)) >> 4) & 3) << 14));
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    float acc[RPI];
#pragma unroll
    for (int k = 0; k < RPI; k++) {
      const uint32_t *rp = (const uint32_t *)(ring + ((u % D) * RPI + k) * SLOT + lane * 36);
      uint32_t w[9];
#pragma unroll
      for (int t = 0; t < 9; t++) w[t] = rp[t];
      f2v s = {0.f, 0.f}, v = {0.f, 0.f};
      s = nib8_fp8(align2(w[1], w[0]), xr[0], xr[1], s);
      s = nib8_fp8(align2(w[2], w[1]), xr[2], xr[3], s);
      s = nib8_fp8(align2(w[3], w[2]), xr[4], xr[5], s);
      s = nib8_fp8(align2(w[4], w[3]), xr[6], xr[7], s);
      v = nib8_fp8(w[5], xr[8], xr[9], v);
      v = nib8_fp8(w[6], xr[10], xr[11], v);
      v = nib8_fp8(w[7], xr[12], xr[13], v);
      v = nib8_fp8(w[8], xr[14], xr[15], v);
      acc[k] = h2f(w[0]) * fmaf(512.f, s.x + s.y, -8.f * xs0);
      acc[k] = fmaf(h2f(w[4] >> 16), fmaf(512.f, v.x + v.y, -8.f * xs1), acc[k]);
    }
    if (u + D < nunits) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this unit's LDS reads are done
      issue(u + D);
    }
#pragma unroll
    for (int k = 0; k < RPI; k++) {
      const float tot = dpp_sum(acc[k]);
      const int row = u * RPI + k;
      if (lane == 63 && row < nrows) dst[r0 + row] = tot;
    }
  }
}

extern "C" int lk_mul_mat_device(const lk_tensor *, const lk_tensor *, lk_tensor *, void *);

template <class F>
double time_launches(hipStream_t st, int copies, int reps, F launch) {
  for (int c = 0; c < copies; c++) launch(c);
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++)
    for (int c = 0; c < copies; c++) launch(c);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / (reps * copies);
}

int main(int argc, char **argv) {
  const int copies = argc > 1 ? atoi(argv[1]) : 48;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const bool prof = argc > 3 && !strcmp(argv[3], "prof");
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint8_t *w;
  float *x, *d, *junk;
  CK(hipMalloc(&w, MAT_BYTES * copies));
  CK(hipMalloc(&x, 4 * K));
  CK(hipMalloc(&d, 4 * (size_t)M * copies));
  CK(hipMalloc(&junk, 64));
  const size_t nblk = (size_t)M * K / 32 * copies;
  hipLaunchKernelGGL(fill_blocks, dim3((nblk + 255) / 256), dim3(256), 0, st, w, nblk, 1234u);
  std::vector<float> hx(K);
  for (int i = 0; i < K; i++) hx[i] = (float)((i * 37) % 101 - 50) / 25.f;
  CK(hipMemcpy(x, hx.data(), 4 * K, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());

  // reference result for checking variants (production path, first matrix)
  lk_tensor ta{}, tb{}, td{};
  ta.type = LK_TYPE_Q4_0; ta.ne[0] = K; ta.ne[1] = M; ta.ne[2] = ta.ne[3] = 1; ta.nb[0] = 18; ta.buf_bytes = MAT_BYTES * copies;
  tb.type = LK_TYPE_F32; tb.ne[0] = 1; tb.ne[1] = K; tb.ne[2] = tb.ne[3] = 1; tb.nb[0] = 4; tb.nb[1] = 4; tb.data = x; tb.buf_bytes = 4 * K;
  td.type = LK_TYPE_F32; td.ne[0] = 1; td.ne[1] = M; td.ne[2] = td.ne[3] = 1; td.nb[0] = 4; td.nb[1] = 4; td.buf_bytes = 4 * (size_t)M * copies;
  ta.data = w; td.data = d;
  std::vector<float> ref(M), got(M);
  if (lk_mul_mat_device(&ta, &tb, &td, st)) { fprintf(stderr, "lk error\n"); return 1; }
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), d, 4 * M, hipMemcpyDeviceToHost));
  auto check = [&](const char *name) {
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(got.data(), d, 4 * M, hipMemcpyDeviceToHost));
    double md = 0, mr = 0;
    for (int i = 0; i < M; i++) { md = fmax(md, fabs(got[i] - ref[i])); mr = fmax(mr, fabs(ref[i])); }
    if (md > 1e-4 * mr) printf("  !! %s mismatch: max|diff| %.3g vs max|ref| %.3g\n", name, md, mr);
  };

  auto report = [&](const char *name, double us) {
    printf("%-34s %9.3f us/launch %8.1f GB/s  (%.1f%% of 8 TB/s)\n", name, us, ALG_BYTES / us / 1e3,
           100.0 * ALG_BYTES / us / 1e3 / 8000.0);
    fflush(stdout);
  };
  auto report_big = [&](const char *name, double us) {
    printf("%-34s %9.3f us / %d mats   %8.1f GB/s  (%.1f%% of 8 TB/s)\n", name, us, copies, ALG_BYTES * copies / us / 1e3,
           100.0 * ALG_BYTES * copies / us / 1e3 / 8000.0);
    fflush(stdout);
  };
  auto prod_big = [&]() {  // production kernel, one launch over all copies
    GemvDesc g{};
    g.a = w; g.x = x; g.dst = d; g.dst_row_stride = 1; g.M = M * copies; g.K = K; g.tile_begin = 0;
    hipLaunchKernelGGL((gemv_q_n1_kernel<LK_TYPE_Q4_0, 4>), dim3(M * copies / 16), dim3(256), 0, st, g,
                       (const GemvDesc *)nullptr, (const uint16_t *)nullptr);
  };
  auto a_launch = [&](int variant, const uint8_t *A, int Mrows, float *D, int rpw) {
    const int grid = (Mrows + 4 * rpw - 1) / (4 * rpw);
    switch (variant) {
      case 0: hipLaunchKernelGGL((a_dword<4, false>), dim3(grid), dim3(256), 0, st, A, x, D, Mrows, rpw); break;
      case 1: hipLaunchKernelGGL((a_dword<4, true>), dim3(grid), dim3(256), 0, st, A, x, D, Mrows, rpw); break;
      case 2: hipLaunchKernelGGL((a_dword<2, true>), dim3(grid), dim3(256), 0, st, A, x, D, Mrows, rpw); break;
      case 3: hipLaunchKernelGGL((a_dword<8, false>), dim3(grid), dim3(256), 0, st, A, x, D, Mrows, rpw); break;
    }
  };
  auto v4p = [&](int rgv, int rpw) {
    const size_t lds = 16 * (K / 64 + 1) * 16 + (K / 64) * 8;
    const int grid = (M * copies + 4 * rpw - 1) / (4 * rpw);
    if (rgv == 2) hipLaunchKernelGGL((v4_kernel<2, false>), dim3(grid), dim3(256), lds, st, w, x, d, M * copies, rpw);
    else hipLaunchKernelGGL((v4_kernel<4, false>), dim3(grid), dim3(256), lds, st, w, x, d, M * copies, rpw);
  };
  if (prof) {
    for (int r = 0; r < 3; r++) {
      hipLaunchKernelGGL(x0_read, dim3(4096), dim3(256), 0, st, (const f32x4 *)w, MAT_BYTES * copies / 16, junk);
      v4p(2, 16);
      v4p(4, 4);
    }
    CK(hipStreamSynchronize(st));
    return 0;
  }
  report("prod lk_mul_mat_device", time_launches(st, copies, reps, [&](int c) {
           ta.data_offset = MAT_BYTES * c; td.data_offset = 4 * (size_t)M * c;
           if (lk_mul_mat_device(&ta, &tb, &td, st)) { fprintf(stderr, "lk error\n"); exit(1); }
         }));
  report("X0 coalesced read", time_launches(st, copies, reps, [&](int c) {
           hipLaunchKernelGGL(x0_read, dim3(2048), dim3(256), 0, st, (const f32x4 *)(w + MAT_BYTES * c), MAT_BYTES / 16, junk);
         }));
  report_big("X0 one launch", time_launches(st, 1, 5, [&](int) {
               hipLaunchKernelGGL(x0_read, dim3(4096), dim3(256), 0, st, (const f32x4 *)w, MAT_BYTES * copies / 16, junk);
             }));
  report_big("prod one launch", time_launches(st, 1, 5, [&](int) { prod_big(); }));
  auto v4_launch = [&](int variant, const uint8_t *A, int Mrows, float *D, int rpw) {
    const int grid = (Mrows + 4 * rpw - 1) / (4 * rpw);
    const size_t lds = 16 * (K / 64 + 1) * 16 + (K / 64) * 8;
    switch (variant) {
      case 0: hipLaunchKernelGGL((v4_kernel<2, false>), dim3(grid), dim3(256), lds, st, A, x, D, Mrows, rpw); break;
      case 1: hipLaunchKernelGGL((v4_kernel<2, true>), dim3(grid), dim3(256), lds, st, A, x, D, Mrows, rpw); break;
      case 2: hipLaunchKernelGGL((v4_kernel<4, false>), dim3(grid), dim3(256), lds, st, A, x, D, Mrows, rpw); break;
      case 3: hipLaunchKernelGGL((v4_kernel<4, true>), dim3(grid), dim3(256), lds, st, A, x, D, Mrows, rpw); break;
      case 4: hipLaunchKernelGGL((v4_kernel<1, false>), dim3(grid), dim3(256), lds, st, A, x, D, Mrows, rpw); break;
    }
  };
  auto s_launch = [&](int D, int grid, const uint8_t *A, int Mrows, float *Dd) {
    const size_t lds = 16 * (K / 64 + 1) * 16 + 8 * D * 3072;
    switch (D) {
      case 2: hipLaunchKernelGGL((s_kernel<2>), dim3(grid), dim3(512), lds, st, A, x, Dd, Mrows); break;
      case 3: hipLaunchKernelGGL((s_kernel<3>), dim3(grid), dim3(512), lds, st, A, x, Dd, Mrows); break;
      case 4: hipLaunchKernelGGL((s_kernel<4>), dim3(grid), dim3(512), lds, st, A, x, Dd, Mrows); break;
      case 5: hipLaunchKernelGGL((s_kernel<5>), dim3(grid), dim3(512), lds, st, A, x, Dd, Mrows); break;
    }
  };
  struct Cfg { int D, NW, RPI, grid; };
  auto s2_launch = [&](const Cfg &c, const uint8_t *A, int Mrows, float *Dd) {
    const size_t lds = 16 * (K / 64 + 1) * 16 + (size_t)c.NW * c.D * c.RPI * 3072;
#define S2(d, nw, rpi) if (c.D == d && c.NW == nw && c.RPI == rpi) hipLaunchKernelGGL((s2_kernel<d, nw, rpi>), dim3(c.grid), dim3(nw * 64), lds, st, A, x, Dd, Mrows)
    S2(3, 8, 1); S2(2, 8, 2); S2(3, 8, 2); S2(2, 12, 1); S2(3, 12, 1); S2(2, 12, 2); S2(4, 8, 1); S2(2, 16, 1); S2(1, 16, 2);
#undef S2
  };
  const Cfg cfgs[] = {{3, 8, 1, 256}, {4, 8, 1, 256}, {2, 8, 2, 256}, {3, 8, 2, 256}, {2, 12, 1, 256}, {3, 12, 1, 256},
                      {2, 12, 2, 256}, {2, 16, 1, 256}, {1, 16, 2, 256}, {2, 8, 2, 512}};
  for (const Cfg &c : cfgs) {
    if (16 * (K / 64 + 1) * 16 + (size_t)c.NW * c.D * c.RPI * 3072 > 160 * 1024) continue;
    char name[64];
    s2_launch(c, w, M, d);
    snprintf(name, sizeof name, "S2 D=%d NW=%d RPI=%d g=%d", c.D, c.NW, c.RPI, c.grid);
    check(name);
    char n1[96], n2[96];
    snprintf(n1, sizeof n1, "%s per-launch", name);
    snprintf(n2, sizeof n2, "%s one", name);
    report(n1, time_launches(st, copies, reps, [&](int cc) { s2_launch(c, w + MAT_BYTES * cc, M, d + (size_t)M * cc); }));
    report_big(n2, time_launches(st, 1, 5, [&](int) { s2_launch(c, w, M * copies, d); }));
  }
  return 0;
}
