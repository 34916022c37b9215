// q32_trace.hip — lab: per-wave timeline of gemm_q32_kernel on C3 (Q4_0 11008x4096, N = 32).
// Compiles the library source with LK_Q32_TRACE; rotates 16 weight copies (> Infinity Cache),
// times the launches, then records one launch's stamps (s_memrealtime, 100 MHz) per wave:
// entry, activations landed, fragments held, first unit landed, loop done, exit.
// usage: q32_trace [M K N]
#define LK_Q32_TRACE 1
#include "../../llama.kotlin_amd/csrc/lk_hip.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__global__ void fill_q4(uint8_t *p, size_t nblk, uint32_t seed) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  uint8_t *q = p + b * 18;
  uint32_t s = (uint32_t)b * 2654435761u ^ seed;
  q[0] = 0x00; q[1] = 0x24;
  for (int i = 0; i < 16; i++) { s = s * 1664525u + 1013904223u; q[2 + i] = (uint8_t)(s >> 24); }
}

static lk_tensor mk(int32_t type, int64_t ne0, int64_t ne1, void *data, uint64_t bytes) {
  lk_tensor t{};
  t.type = type; t.ne[0] = ne0; t.ne[1] = ne1; t.ne[2] = t.ne[3] = 1;
  if (type == LK_TYPE_Q4_0) { t.nb[0] = 18; t.nb[1] = ne0 / 32 * 18; }
  else { t.nb[0] = 4; t.nb[1] = 4 * ne0; }
  t.nb[2] = t.nb[3] = t.nb[1] * ne1;
  t.data = data; t.buf_bytes = bytes; t.data_offset = 0;
  return t;
}

int main(int argc, char **argv) {
  const int M = argc > 3 ? atoi(argv[1]) : 11008, K = argc > 3 ? atoi(argv[2]) : 4096, N = argc > 3 ? atoi(argv[3]) : 32;
  CK(hipSetDevice(0));
  const int ROT = 16;
  const size_t wb = (size_t)M * K / 32 * 18;
  std::vector<lk_tensor> A(ROT);
  void *x, *d;
  CK(hipMalloc(&x, 4 * (size_t)K * N)); CK(hipMalloc(&d, 4 * (size_t)M * N));
  CK(hipMemset(x, 0x3c, 4 * (size_t)K * N));
  for (int r = 0; r < ROT; r++) {
    void *w;
    CK(hipMalloc(&w, wb));
    hipLaunchKernelGGL(fill_q4, dim3((wb / 18 + 255) / 256), dim3(256), 0, 0, (uint8_t *)w, wb / 18, 77 + r);
    A[r] = mk(LK_TYPE_Q4_0, K, M, w, wb);
  }
  lk_tensor B = mk(LK_TYPE_F32, N, K, x, 4 * (size_t)K * N), D = mk(LK_TYPE_F32, N, M, d, 4 * (size_t)M * N);
  CK(hipDeviceSynchronize());
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int r = 0; r < 3 * ROT; r++) if (lk_mul_mat_device(&A[r % ROT], &B, &D, st)) { fprintf(stderr, "%s\n", lk_last_error()); return 1; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < 5 * ROT; r++) lk_mul_mat_device(&A[r % ROT], &B, &D, st);
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("computeMatMul %dx%dx%d: %.2f us per call (kernel + reduce)\n", M, K, N, ms * 1e3 / (5 * ROT));
  const int grid = 512;
  uint64_t *tb;
  CK(hipMalloc(&tb, (size_t)grid * 4 * 6 * 8));
  CK(hipMemset(tb, 0, (size_t)grid * 4 * 6 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lk_qtrace_buf), &tb, sizeof(tb)));
  lk_mul_mat_device(&A[0], &B, &D, st);
  lk_mul_mat_device(&A[1], &B, &D, st);
  CK(hipStreamSynchronize(st));
  uint64_t *null = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lk_qtrace_buf), &null, sizeof(null)));
  std::vector<uint64_t> h((size_t)grid * 4 * 6);
  CK(hipMemcpy(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull;
  for (size_t w = 0; w < h.size() / 6; w++) if (h[w * 6]) t0 = std::min(t0, h[w * 6]);
  const char *nm[6] = {"entry", "x landed", "frags held", "1st unit", "loop done", "exit"};
  for (int k = 0; k < 6; k++) {
    std::vector<double> v;
    for (size_t w = 0; w < h.size() / 6; w++) if (h[w * 6 + k]) v.push_back((h[w * 6 + k] - t0) * 0.01);
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    auto pc = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))]; };
    printf("%-10s n=%5zu  min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", nm[k], v.size(), v.front(), pc(0.1), pc(0.5), pc(0.9), v.back());
  }
  return 0;
}
