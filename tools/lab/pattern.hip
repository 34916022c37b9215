// pattern.hip — lab: does the HBM access pattern (who reads which rows when) limit the
// LDS-DMA streaming GEMV? Q4_0, K=4096, one launch over COPIES x 4096 rows (454 MB at 48).
//   X0       : grid-stride float4 nontemporal read of the same bytes (reference rate)
//   XW<mode> : pure LDS-DMA streaming, no decode, rows assigned by <mode>
//   S<mode>  : the production decode loop (lk:: helpers), rows assigned by <mode>
// modes: 0 = contiguous rows per wave (production), 1 = rows cyclic over all waves,
//        2 = contiguous per workgroup, cyclic over its 8 waves
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../llama.kotlin_amd/csrc/lk_kernels.hpp"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

constexpr int K = 4096, RB = K / 32 * 18, NP = K / 64, SLOT = 3072, L = 3;
using lk::f32x4;
using lk::f2v;

__global__ void fill_q4(uint8_t *p, size_t nblk, uint32_t seed) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  uint8_t *q = p + b * 18;
  uint32_t s = (uint32_t)b * 2654435761u ^ seed;
  q[0] = 0x00; q[1] = 0x24;
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

// row of the i-th unit of (workgroup g, wave w); returns -1 past the end
template <int MODE, int NW = 8>
__device__ __forceinline__ int row_of(int i, int g, int w, int G, int M) {
  if (MODE == 0) {
    const int per_wg = (M + G - 1) / G, r0 = g * per_wg, r1 = min(r0 + per_wg, M);
    const int per_w = (max(r1 - r0, 0) + NW - 1) / NW;
    const int r = r0 + w * per_w + i;
    return (i < per_w && r < r1) ? r : -1;
  } else if (MODE == 1) {
    const int r = (g * NW + w) + i * G * NW;
    return r < M ? r : -1;
  } else {
    const int per_wg = (M + G - 1) / G, r0 = g * per_wg, r1 = min(r0 + per_wg, M);
    const int r = r0 + w + 8 * i;
    return r < r1 ? r : -1;
  }
}

template <int MODE, bool DECODE, int D, bool BATCH = false, int AUX = 0, int NW = 8, bool NOX = false>
__global__ __launch_bounds__(NW * 64) void s_kernel(const uint8_t *__restrict__ a, const float *__restrict__ x, float *__restrict__ dst,
                                                int M) {
  extern __shared__ f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, g = blockIdx.x;
  uint8_t *ring = (uint8_t *)lds + NP * 256 + wave * D * SLOT;
  auto dma = [&](int r, int sl) {
    const uint8_t *src = a + (size_t)(r < 0 ? 0 : r) * RB;
#pragma unroll
    for (int j = 0; j < L; j++) {
      int off = j * 1024 + lane * 16;
      off = off < RB ? off : 0;
      __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(src + off),
                                       (__attribute__((address_space(3))) void *)(ring + sl * SLOT + j * 1024), 16, 0, AUX);
    }
  };
  // activations (natural, swizzled) by DMA
  for (int k = wave; k < (NOX ? 0 : NP / 4); k += NW) {
    const int i = k * 64 + lane, p = i >> 4, t = (i & 15) ^ (p & 15);
    __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)((const f32x4 *)x + p * 16 + t),
                                     (__attribute__((address_space(3))) void *)(lds + k * 64), 16, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < D; k++) dma(row_of<MODE, NW>(k, g, wave, G, M), k);
  lk::wait_vmcnt<D * L>();
  __builtin_amdgcn_s_barrier();
  f32x4 xr[16];
  for (int jj = 0; jj < 8; jj++) {
    const f32x4 n0 = lds[16 * lane + ((2 * jj) ^ (lane & 15))], n1 = lds[16 * lane + ((2 * jj + 1) ^ (lane & 15))];
    xr[2 * jj] = f32x4{n0.x, n0.z, n1.x, n1.z};
    xr[2 * jj + 1] = f32x4{n0.y, n0.w, n1.y, n1.w};
  }
  float xs0 = 0.f, xs1 = 0.f;
  for (int t = 0; t < 8; t++) {
    xs0 += (xr[t].x + xr[t].y) + (xr[t].z + xr[t].w);
    xs1 += (xr[t + 8].x + xr[t + 8].y) + (xr[t + 8].z + xr[t + 8].w);
  }
  int slot = 0;
  float outv = 0.f;
  int rows_seen[1] = {0};
  for (int i = 0;; i++) {
    const int r = row_of<MODE, NW>(i, g, wave, G, M);
    if (r < 0) break;
    const bool more = row_of<MODE, NW>(i + D - 1, g, wave, G, M) >= 0;
    if (more) lk::wait_vmcnt<(D - 1) * L>();
    else lk::wait_vmcnt<0>();
    const uint32_t *rp = (const uint32_t *)(ring + slot * SLOT + lane * 36);
    uint32_t w[9];
    for (int k = 0; k < 9; k++) w[k] = rp[k];
    float v = 0.f;
    if (DECODE) v = lk::pair_dot_s<LK_TYPE_Q4_0>(w, xr, xs0, xs1);
    else v = __builtin_bit_cast(float, w[0] ^ w[4] ^ w[8]);
    const int rn = row_of<MODE, NW>(i + D, g, wave, G, M);
    if (rn >= 0) {
      lk::wait_lgkmcnt0();
      dma(rn, slot);
    }
    slot = slot + 1 == D ? 0 : slot + 1;
    const float tot = lk::dpp_sum(v);
    if (!BATCH) {
      if (lane == 63) dst[r] = tot;
    } else {
      // hold row i's total in lane i % 64; one store per 64 rows (row index of lane l kept in rsl)
      const float tv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tot), 63));
      if (lane == (i & 63)) { outv = tv; rows_seen[0] = r; }
      const bool last = row_of<MODE, NW>(i + 1, g, wave, G, M) < 0;
      if ((i & 63) == 63 || last) {
        if (lane <= (i & 63)) dst[rows_seen[0]] = outv;
      }
    }
  }
}

int main(int argc, char **argv) {
  // usage: pattern <copies per launch> [rotation buffers]
  const int copies = argc > 1 ? atoi(argv[1]) : 48;
  const int rot = argc > 2 ? atoi(argv[2]) : 1;
  const int M = 4096 * copies;
  const size_t bytes = (size_t)M * RB;
  std::vector<uint8_t *> bufs(rot);
  float *x, *d;
  for (auto &b : bufs) {
    CK(hipMalloc(&b, bytes));
    hipLaunchKernelGGL(fill_q4, dim3((bytes / 18 + 255) / 256), dim3(256), 0, 0, b, bytes / 18, 7);
  }
  CK(hipMalloc(&x, 4 * K));
  CK(hipMalloc(&d, 4 * (size_t)M));
  CK(hipMemset(x, 0x3c, 4 * K));
  CK(hipDeviceSynchronize());
  printf("launch = %.1f MB, rotating over %d buffers (%.0f MB)\n", bytes / 1e6, rot, rot * bytes / 1e6);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cur = 0;
  uint8_t *a = bufs[0];
  auto timeit = [&](const char *name, auto fn) {
    for (int i = 0; i < rot + 2; i++) { a = bufs[cur++ % rot]; fn(); }
    CK(hipEventRecord(e0));
    const int reps = std::max(10, 2 * rot);
    for (int i = 0; i < reps; i++) { a = bufs[cur++ % rot]; fn(); }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-36s %9.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
  };
  timeit("X0 grid-stride read", [&] { hipLaunchKernelGGL(x0_read, dim3(4096), dim3(256), 0, 0, (const f32x4 *)a, bytes / 16, d); });
#define RUN(MODE, DEC, D, B, AUX)                                                                                   \
  timeit(#DEC " m=" #MODE " D=" #D " batch=" #B " aux=" #AUX, [&] {                                                  \
    hipLaunchKernelGGL((s_kernel<MODE, DEC, D, B, AUX>), dim3(256), dim3(512), NP * 256 + 8 * D * SLOT, 0, a, x, d, M); \
  })
  auto prod = [&](const char *name) {
    timeit(name, [&] {
      lk::GemvDesc gd{};
      gd.a = a; gd.x = x; gd.dst = d; gd.dst_row_stride = 1; gd.M = M; gd.K = K;
      constexpr size_t plds = lk::StreamGeom<LK_TYPE_Q4_0, 1>::LDS;
      hipLaunchKernelGGL((lk::gemv_stream_kernel<LK_TYPE_Q4_0, 1>), dim3(256), dim3(512), plds, 0, gd,
                         (const lk::StreamWork *)nullptr, 0);
    });
  };
#define RUNW(NW, D, G)                                                                                          \
  timeit("decode NW=" #NW " D=" #D " grid=" #G, [&] {                                                          \
    hipLaunchKernelGGL((s_kernel<0, true, D, false, 2, NW>), dim3(G), dim3(NW * 64), NP * 256 + NW * D * SLOT, 0, a, x, d, M); \
  })
  for (int rep = 0; rep < 2; rep++) {
    RUNW(8, 3, 256);
    timeit("decode NW=8 D=3 no-x (timing only)", [&] {
      hipLaunchKernelGGL((s_kernel<0, true, 3, false, 2, 8, true>), dim3(256), dim3(512), NP * 256 + 8 * 3 * SLOT, 0, a, x, d, M);
    });
    timeit("dma-only NW=8 D=3 no-x", [&] {
      hipLaunchKernelGGL((s_kernel<0, false, 3, false, 2, 8, true>), dim3(256), dim3(512), NP * 256 + 8 * 3 * SLOT, 0, a, x, d, M);
    });
    prod("production gemv_stream<Q4_0,1>");
  }
  return 0;
}
