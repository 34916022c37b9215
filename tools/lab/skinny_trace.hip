// skinny_trace.hip — lab: per-wave timeline of gemm_skinny_kernel (s_memrealtime, 100 MHz):
// 0 entry, 1 activation loads converted, 2 after the barrier, 3 first unit landed,
// 4 first unit done, 5 loop done, 6 drained. usage: skinny_trace M K N [waves]
// PAIR=1: gemm_skinny_pair_kernel (Q4_0, N > 16) instead; LK_SKP_SKEL builds its skeletons.
#define LK_SKINNY_TRACE 1
#ifndef LK_SKINNY_NT
#define LK_SKINNY_NT 0
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
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
    p[i] = ((uint32_t)i * 2654435761u ^ seed) & 0x3BFF3BFFu;  // finite halves
}

template <int NT, bool PAIR>
void run(int M, int K, int N) {
  using SG = std::conditional_t<PAIR, lk::SkinnyPairGeom<LK_TYPE_Q4_0, NT>, lk::SkinnyGeom<LK_TYPE_Q4_0, NT>>;
  constexpr int NW = SG::NW;
  const int nblk = K / 32, slices = (nblk + SG::SB - 1) / SG::SB, ntile = (M + 15) / 16;
  int ranges = std::max(1, std::min(ntile, (256 + slices - 1) / slices));
  const int tpr = (ntile + ranges - 1) / ranges;
  ranges = (ntile + tpr - 1) / tpr;
  const int tasks = ranges * slices, grid = (tasks + 7) / 8 * 8;
  const size_t abytes = (size_t)M * nblk * 18;
  const int rot = 16;
  std::vector<uint8_t *> as(rot);
  for (auto &a : as) {
    CK(hipMalloc(&a, abytes));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)a, abytes / 4, 7);
  }
  float *b, *dst, *part;
  CK(hipMalloc(&b, 4 * (size_t)K * N));
  CK(hipMalloc(&dst, 4 * (size_t)M * N));
  CK(hipMalloc(&part, 4 * (size_t)slices * M * 32));
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, (uint32_t *)b, (size_t)K * N, 3);
  uint64_t *tb;
  constexpr int SL = PAIR ? 16 : 8;  // stamp slots per wave (the pair kernel adds phase cycles)
  const size_t nst = (size_t)grid * NW * SL;
  CK(hipMalloc(&tb, nst * 8));
  CK(hipMemset(tb, 0, nst * 8));
  lk::SkinnyArgs g{};
  g.b = (const uint8_t *)b; g.b_nb0 = 4; g.b_nb1 = 4 * N;
  g.dst = (uint8_t *)dst; g.d_nb0 = 4; g.d_nb1 = 4 * N;
  g.partial = part; g.M = M; g.N = N; g.K = K; g.slices = slices; g.tiles_per_range = tpr; g.tasks = tasks;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint64_t *null = nullptr;
  for (int pass = 0; pass < 2; pass++) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(lk::lk_strace_buf), pass ? &tb : &null, sizeof(tb)));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = pass ? 1 : 3 * rot;
    for (int i = 0; i < reps; i++) {
      g.a = as[i % rot];
      if constexpr (PAIR) hipLaunchKernelGGL((lk::gemm_skinny_pair_kernel<LK_TYPE_Q4_0, NT>), dim3(grid), dim3(NW * 64), SG::LDS, 0, g);
      else hipLaunchKernelGGL((lk::gemm_skinny_kernel<LK_TYPE_Q4_0, NT>), dim3(grid), dim3(NW * 64), SG::LDS, 0, g);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("NW=%d M=%d K=%d N=%d grid=%d slices=%d tiles/range=%d D=%d: %s %.2f us/launch\n", NW, M, K, N, grid, slices, tpr, SG::D,
           pass ? "traced" : "untraced", ms * 1e3 / reps);
  }
  std::vector<uint64_t> h(nst);
  CK(hipMemcpy(h.data(), tb, nst * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull;
  for (size_t w = 0; w < (size_t)grid * NW; w++) t0 = std::min(t0, h[w * SL]);
  const char *names[8] = {"entry", "x converted", "barrier", "unit0 landed", "unit0 done", "loop done", "drained",
                          "unit0 computed"};
  for (int k : {0, 1, 2, 3, 7, 4, 5, 6}) {
    std::vector<double> v;
    for (size_t w = 0; w < (size_t)grid * NW; w++)
      if (h[w * SL + k]) v.push_back((h[w * SL + k] - t0) / 100.0);  // us
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    printf("  %-14s n=%5zu  min %7.2f  p10 %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", names[k], v.size(), v.front(),
           v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  }
  if (PAIR) {  // per-phase shader cycles, per wave, by half (h = 0 collects and stores)
    const char *ph[5] = {"ring wait (vmcnt)", "LDS reads + blocks", "ring refill issue", "hand-off waits", "stores"};
    for (int hh = 0; hh < 2; hh++)
      for (int k = 0; k < 5; k++) {
        std::vector<double> v;
        for (size_t w = 0; w < (size_t)grid * NW; w++)
          if ((int)((w % NW) >> 2) == hh && h[w * SL + 1]) v.push_back((double)h[w * SL + 8 + k]);
        std::sort(v.begin(), v.end());
        if (!v.empty()) printf("  h=%d %-20s med %9.0f  p90 %9.0f cycles\n", hh, ph[k], v[v.size() / 2], v[v.size() * 9 / 10]);
      }
  }
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 11008, K = argc > 2 ? atoi(argv[2]) : 4096, N = argc > 3 ? atoi(argv[3]) : 32;
  const bool pair = getenv("PAIR") && atoi(getenv("PAIR"));
  if (pair) run<2, true>(M, K, N);
  else if (N > 16) run<2, false>(M, K, N);
  else run<1, false>(M, K, N);
  return 0;
}
