// sk_trace.hip — lab: per-wave timeline of gemm_sk_kernel (lk_skinny.hpp, LK_SK_TRACE):
// s_memrealtime (100 MHz) at entry, after the barrier, unit 0 landed, unit 0 computed, loop done;
// s_memtime cycles summed over the units waiting for the DMA, computing, and in the hand-off.
// usage: sk_trace M K N [q4_1]
#define LK_SK_TRACE 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../llama.kotlin_amd/csrc/lk_skinny.hpp"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = ((uint32_t)i * 2654435761u ^ seed) & 0x3BFF3BFFu;  // finite halves / bf16
}

template <int QT, int NT>
void run(int M, int K, int N) {
  using SG = lk::SkGeom<QT, NT>;
  const int nblk = K / 32, slices = (nblk + SG::SB - 1) / SG::SB, ntile = (M + 15) / 16;
  int ranges = std::max(1, std::min(ntile, (256 + slices - 1) / slices));
  const int tpr = (ntile + ranges - 1) / ranges;
  ranges = (ntile + tpr - 1) / tpr;
  const int tasks = ranges * slices, grid = (tasks + 7) / 8 * 8;
  const size_t abytes = (size_t)M * nblk * SG::BB;
  const int rot = 16;
  std::vector<uint8_t *> as(rot);
  for (auto &a : as) {
    CK(hipMalloc(&a, abytes));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)a, abytes / 4, 7);
  }
  const int ntx = (N + 15) / 16;
  const size_t fbytes = (size_t)ntx * nblk * 2 * 1024, sbytes = (size_t)nblk * ntx * 16 * 4;
  uint8_t *frag;
  float *dst, *part;
  CK(hipMalloc(&frag, fbytes + sbytes));
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, (uint32_t *)frag, (fbytes + sbytes) / 4, 3);
  CK(hipMalloc(&dst, 4 * (size_t)M * N));
  CK(hipMalloc(&part, 4 * (size_t)slices * M * 16 * NT));
  uint64_t *tb;
  const size_t nst = (size_t)grid * 8 * 8;
  CK(hipMalloc(&tb, nst * 8));
  CK(hipMemset(tb, 0, nst * 8));
  lk::SkArgs g{};
  g.frag = (const lk::u32x4 *)frag;
  g.xsum = (const float *)(frag + fbytes);
  g.dst = (uint8_t *)dst; g.d_nb0 = 4; g.d_nb1 = 4 * N;
  g.partial = part; g.M = M; g.N = N; g.K = K; g.slices = slices; g.tiles_per_range = tpr; g.tasks = tasks;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint64_t *null = nullptr;
  for (int pass = 0; pass < 2; pass++) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(lk::lk_sktrace_buf), pass ? &tb : &null, sizeof(tb)));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = pass ? 1 : 3 * rot;
    for (int i = 0; i < reps; i++) {
      g.a = as[(i + pass) % rot];
      hipLaunchKernelGGL((lk::gemm_sk_kernel<QT, NT>), dim3(grid), dim3(512), SG::LDS, 0, g);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("QT=%d M=%d K=%d N=%d grid=%d slices=%d tiles/range=%d D=%d L=%d: %s %.2f us/launch\n", QT, M, K, N, grid, slices, tpr,
           SG::D, SG::L, pass ? "traced" : "untraced", ms * 1e3 / reps);
  }
  std::vector<uint64_t> h(nst);
  CK(hipMemcpy(h.data(), tb, nst * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull;  // the earliest barrier stamp (slot 0 holds DMA-issue cycles)
  for (size_t w = 0; w < (size_t)grid * 8; w++)
    if (h[w * 8 + 1]) t0 = std::min(t0, h[w * 8 + 1]);
  const char *names[8] = {"cyc issue DMA", "barrier", "unit0 landed", "unit0 computed", "loop done", "cyc wait DMA", "cyc compute",
                          "cyc hand-off"};
  for (int k = 0; k < 8; k++) {
    for (int half = 0; half < 2; half++) {
      std::vector<double> v;
      for (size_t w = 0; w < (size_t)grid * 8; w++) {
        if ((int)(w % 8) / 4 != half || !h[(w / 8) * 64 + (w % 8) * 8 + 1]) continue;
        const uint64_t x = h[w * 8 + k];
        v.push_back(k >= 1 && k < 5 ? (x - t0) / 100.0 : (double)x);
      }
      std::sort(v.begin(), v.end());
      if (v.empty()) continue;
      printf("  %-15s h=%d n=%5zu  min %9.2f  p10 %9.2f  med %9.2f  p90 %9.2f  max %9.2f %s\n", names[k], half, v.size(), v.front(),
             v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back(), k >= 1 && k < 5 ? "us" : "cyc");
    }
  }
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 11008, K = argc > 2 ? atoi(argv[2]) : 4096, N = argc > 3 ? atoi(argv[3]) : 32;
  const bool q41 = argc > 4 && atoi(argv[4]);
  if (q41) { if (N > 16) run<LK_TYPE_Q4_1, 2>(M, K, N); else run<LK_TYPE_Q4_1, 1>(M, K, N); }
  else { if (N > 16) run<LK_TYPE_Q4_0, 2>(M, K, N); else run<LK_TYPE_Q4_0, 1>(M, K, N); }
  return 0;
}
