// wide_lab.hip — lab: gemm_wide_kernel<Q4_0> at C5 (M = K = 4096, N = 512, K split in two) on
// synthetic operands, timed alone (no xsplit / reduce). Build variants with -DLK_WIDE_NOCOMPUTE
// (data movement only). usage: wide_lab [M K N]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../llama.kotlin_amd/csrc/lk_kernels.hpp"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = ((uint32_t)i * 2654435761u ^ seed) & 0x3BFF3BFFu;
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 4096, N = argc > 3 ? atoi(argv[3]) : 512;
  using WG = lk::WideGeom<LK_TYPE_Q4_0>;
  const int nblk = K / 32, ntx = (N + 15) / 16;
  lk::WideArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.tiles_m = (M + WG::BM - 1) / WG::BM;
  g.tiles_n = (N + WG::BN - 1) / WG::BN;
  const int tiles = g.tiles_m * g.tiles_n, nst = nblk / WG::SB;
  int slices = std::max(1, std::min({(256 + tiles - 1) / tiles, 16, nst}));
  g.kslice = ((nst + slices - 1) / slices) * WG::SB;
  slices = (nblk + g.kslice - 1) / g.kslice;
  g.slices = slices;
  const int per_xcd = (tiles + 7) / 8;
  int best = 1;
  double cost = 1e30;
  for (int sn = 1; sn <= g.tiles_n; sn++) {
    const int sm = std::min(g.tiles_m, (per_xcd + sn - 1) / sn);
    const double c = sn * WG::BN * 4.0 + sm * WG::BM * (18 / 32.0);
    if (sm * sn >= per_xcd && c < cost) { cost = c; best = sn; }
  }
  g.sn = argc > 4 ? atoi(argv[4]) : best;
  g.sm = std::min(g.tiles_m, (per_xcd + g.sn - 1) / g.sn);
  const int nsuper = ((g.tiles_m + g.sm - 1) / g.sm) * ((g.tiles_n + g.sn - 1) / g.sn);
  g.tasks = nsuper * g.sm * g.sn * slices;
  const int grid = (g.tasks + 7) / 8 * 8;
  printf("super-tile %d x %d\n", g.sm, g.sn);
  const size_t abytes = (size_t)M * nblk * 18 + 256, fbytes = (size_t)ntx * nblk * 2 * 1024, npad = g.tiles_n * WG::BN;
  const int rot = 8;
  std::vector<uint8_t *> as(rot);
  for (auto &a : as) {
    CK(hipMalloc(&a, abytes));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)a, abytes / 4, 7);
  }
  uint8_t *frag;
  float *xsum, *part, *dst;
  CK(hipMalloc(&frag, fbytes));
  CK(hipMalloc(&xsum, (size_t)nblk * ntx * 16 * 4));
  CK(hipMalloc(&part, (size_t)slices * M * npad * 4));
  CK(hipMalloc(&dst, (size_t)M * N * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)frag, fbytes / 4, 3);
  g.frag = (const lk::u32x4 *)frag; g.xsum = xsum; g.partial = part; g.dst = (uint8_t *)dst;
  g.d_nb0 = 4; g.d_nb1 = 4 * N;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int pass = 0; pass < 2; pass++) {
    CK(hipEventRecord(e0));
    const int reps = 40;
    for (int i = 0; i < reps; i++) {
      g.a = as[i % rot];
      hipLaunchKernelGGL((lk::gemm_wide_kernel<LK_TYPE_Q4_0>), dim3(grid), dim3(512), WG::LDS, 0, g);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("M=%d K=%d N=%d grid=%d slices=%d D=%d STAGE=%d: %.2f us  %.1f useful TFLOP/s\n", M, K, N, grid, slices, WG::D,
           WG::STAGE, us, 2.0 * M * N * K / us / 1e6);
  }
  return 0;
}
