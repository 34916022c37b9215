// dma_rate.hip — lab: LDS-DMA (global_load_lds_dwordx4, 1 KB per wave instruction) intake per CU
// from an L2-resident buffer, by waves per workgroup (one workgroup per CU) and instructions in
// flight per wave. No compute, no LDS reads. usage: dma_rate [buffer KB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../llama.kotlin_amd/csrc/lk_kernels.hpp"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

// each wave: ITERS instructions, at most F in flight; source walks a buf_kb buffer
template <int F>
__global__ void dma_kernel(const uint8_t *buf, uint32_t mask, int iters, float *out) {
  extern __shared__ uint8_t smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t *ring = smem + wave * F * 1024;
  uint32_t off = ((blockIdx.x * 64 + wave) * 1024) & mask;
  for (int i = 0; i < iters; i++) {
    lk::dma16<false>(buf, off + lane * 16, ring + (i % F) * 1024);
    off = (off + 1024 * 7) & mask;
    if (i >= F - 1) lk::wait_vmcnt<F - 1>();
  }
  lk::wait_vmcnt<0>();
  if (((const uint32_t *)ring)[lane] == 0x12345u) out[0] = 1.f;
}

int main(int argc, char **argv) {
  const int kb = argc > 1 ? atoi(argv[1]) : 1024;
  uint8_t *buf;
  float *out;
  CK(hipMalloc(&buf, (size_t)kb * 1024 + 4096));
  CK(hipMemset(buf, 1, (size_t)kb * 1024 + 4096));
  CK(hipMalloc(&out, 64));
  const uint32_t mask = (uint32_t)(kb * 1024 - 1) & ~1023u;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 2048;
  auto run = [&](const char *name, auto kern, int nw, int f) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipEventRecord(e0));
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(256), dim3(nw * 64), nw * f * 1024, 0, buf, mask, iters, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 5, bytes = 256.0 * nw * iters * 1024;
      if (rep) printf("%-10s waves=%d inflight/wave=%2d: %8.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n", name, nw, f, us,
                      bytes / 256 / us / 1e3, bytes / us / 1e6);
    }
  };
  printf("buffer %d KB\n", kb);
  for (int nw : {1, 2, 4, 8}) {
    run("F=4", dma_kernel<4>, nw, 4);
    run("F=8", dma_kernel<8>, nw, 8);
    run("F=16", dma_kernel<16>, nw, 16);
  }
  return 0;
}
