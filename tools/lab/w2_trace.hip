// w2_trace.hip — lab: gemm_wide2_kernel's waits on C5 (Q4_0 4096 x 4096, N = 512): per wave,
// cycles spent waiting on FULL (consumers) / FREE (loaders) against its total cycles. LK_WIDE2=2
// for 8 consumers; -DLK_W2_MODE=1 (LDS reads only) / 2 (compute only) for the skeletons.
#define LK_W2_TRACE 1
#include "../../llama.kotlin_amd/csrc/lk_hip.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = ((uint32_t)i * 2654435761u ^ seed) & 0x3BFF3BFFu;
}

static lk_tensor mk(int32_t type, int64_t ne0, int64_t ne1, void *data, uint64_t bytes, uint64_t nb1) {
  lk_tensor t{};
  t.type = type; t.ne[0] = ne0; t.ne[1] = ne1; t.ne[2] = t.ne[3] = 1;
  t.nb[0] = type == LK_TYPE_Q4_0 ? 18 : 4; t.nb[1] = nb1; t.nb[2] = t.nb[3] = nb1 * ne1;
  t.data = data; t.buf_bytes = bytes; t.data_offset = 0;
  return t;
}

int main() {
  if (!getenv("LK_WIDE2")) setenv("LK_WIDE2", "1", 1);
  const int NW = atoi(getenv("LK_WIDE2")) == 2 ? 12 : 8, NC = NW - 4;
  const int M = 4096, K = 4096, N = 512;
  const size_t ab = (size_t)M * K / 32 * 18 + 256;
  void *a, *b, *d;
  CK(hipMalloc(&a, ab)); CK(hipMalloc(&b, 4 * (size_t)K * N)); CK(hipMalloc(&d, 4 * (size_t)M * N));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)a, ab / 4, 7);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)b, (size_t)K * N, 3);
  lk_tensor A = mk(LK_TYPE_Q4_0, K, M, a, ab, K / 32 * 18), B = mk(LK_TYPE_F32, N, K, b, 4 * (size_t)K * N, 4 * N),
            Dd = mk(LK_TYPE_F32, N, M, d, 4 * (size_t)M * N, 4 * N);
  for (int i = 0; i < 5; i++) lk_mul_mat_device(&A, &B, &Dd, 0);
  CK(hipDeviceSynchronize());
  const int grid = 256;
  uint64_t *tb;
  CK(hipMalloc(&tb, (size_t)grid * NW * 2 * 8));
  CK(hipMemset(tb, 0, (size_t)grid * NW * 2 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lk_w2trace_buf), &tb, sizeof(tb)));
  lk_mul_mat_device(&A, &B, &Dd, 0);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h((size_t)grid * NW * 2);
  CK(hipMemcpy(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost));
  for (int role = 0; role < 2; role++) {
    std::vector<double> wf, tot;
    for (int g = 0; g < grid; g++)
      for (int w = role ? NC : 0; w < (role ? NW : NC); w++) {
        const uint64_t *q = &h[((size_t)g * NW + w) * 2];
        if (q[1]) { wf.push_back((double)q[0] / q[1]); tot.push_back((double)q[1]); }
      }
    std::sort(wf.begin(), wf.end());
    std::sort(tot.begin(), tot.end());
    if (wf.empty()) continue;
    printf("%s: n=%zu  wait share p10 %.3f p50 %.3f p90 %.3f | total cycles p50 %.0f max %.0f\n", role ? "loaders (FREE)" : "consumers (FULL)",
           wf.size(), wf[wf.size() / 10], wf[wf.size() / 2], wf[wf.size() * 9 / 10], tot[tot.size() / 2], tot.back());
  }
  return 0;
}
