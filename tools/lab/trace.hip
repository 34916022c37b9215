// trace.hip — per-wave timeline of gemv_stream_kernel on a Llama-7B layer (lab, not product).
// Compiles the library source into this TU with LK_STREAM_TRACE, builds one MulMat plan per
// layer over NL layers of distinct Q4_0 weights (NL x 114 MB > Infinity Cache), replays them,
// and for one launch records s_memrealtime (100 MHz) per wave at: entry, activations ready,
// first unit decoded, exit. Prints percentiles relative to the earliest entry.
#ifndef NO_TRACE
#define LK_STREAM_TRACE 1
#endif
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
  const int NL = argc > 1 ? atoi(argv[1]) : 8;
  // argv[2]: the layer's matrices as digits into the Llama-7B shapes (default "0123456")
  struct Mat { int M, K; };
  const std::vector<Mat> shapes = {{4096, 4096}, {4096, 4096}, {4096, 4096}, {4096, 4096}, {11008, 4096}, {11008, 4096},
                                   {4096, 11008}, {0, 0}, {0, 0}, {49152, 4096}};  // '9': one tall node of 12 x 4096 rows
  std::vector<Mat> mats;
  for (const char *c = argc > 2 ? argv[2] : "0123456"; *c; c++) mats.push_back(shapes[*c - '0']);
  CK(hipSetDevice(0));
  std::vector<lk_plan *> plans;
  std::vector<lk_tensor> singleA, singleB, singleD;
  size_t layer_bytes = 0;
  for (auto &m : mats) layer_bytes += (size_t)m.M * m.K / 32 * 18;
  for (int l = 0; l < NL; l++) {
    std::vector<lk_tensor> A, B, D;
    for (auto &m : mats) {
      size_t wb = (size_t)m.M * m.K / 32 * 18;
      void *w, *x, *d;
      CK(hipMalloc(&w, wb)); CK(hipMalloc(&x, 4 * m.K)); CK(hipMalloc(&d, 4 * m.M));
      hipLaunchKernelGGL(fill_q4, dim3((wb / 18 + 255) / 256), dim3(256), 0, 0, (uint8_t *)w, wb / 18, 77 + l);
      CK(hipMemset(x, 0x3c, 4 * m.K));
      A.push_back(mk(LK_TYPE_Q4_0, m.K, m.M, w, wb));
      B.push_back(mk(LK_TYPE_F32, 1, m.K, x, 4 * m.K));
      B.back().nb[1] = 4;
      D.push_back(mk(LK_TYPE_F32, 1, m.M, d, 4 * m.M));
    }
    singleA.push_back(A[0]); singleB.push_back(B[0]); singleD.push_back(D[0]);
    lk_plan *p = nullptr;
    if (lk_plan_create(A.data(), B.data(), D.data(), (int)mats.size(), &p)) { fprintf(stderr, "plan: %s\n", lk_last_error()); return 1; }
    plans.push_back(p);
  }
  CK(hipDeviceSynchronize());
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; r++) for (auto *p : plans) lk_plan_launch(p, st);
  CK(hipStreamSynchronize(st));
  if (mats.size() == 1) {  // the same node through the single-launch path (no work list)
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 10; r++)
      for (size_t l = 0; l < plans.size(); l++) lk_mul_mat_device(&singleA[l], &singleB[l], &singleD[l], st);
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms1 = 0;
    CK(hipEventElapsedTime(&ms1, e0, e1));
    printf("single launch: %.3f us\n", ms1 * 1e3 / (10 * plans.size()));
  }
  CK(hipEventRecord(e0, st));
  const int reps = 10;
  for (int r = 0; r < reps; r++) for (auto *p : plans) lk_plan_launch(p, st);
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / (reps * NL);
  printf("layer launch: %.3f us  %.1f GB/s (weights only)  grid=%d spw=%d class=%d\n", us, layer_bytes / us / 1e3,
         plans[0]->groups[0].grid, plans[0]->groups[0].spw, plans[0]->groups[0].cls);
#ifndef NO_TRACE
  // traced launch (the middle layer, after its predecessor)
  const int grid = plans[0]->groups[0].grid;
  uint64_t *tb;
  CK(hipMalloc(&tb, (size_t)grid * kStreamWaves * 4 * 8));
  CK(hipMemset(tb, 0, (size_t)grid * kStreamWaves * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lk_trace_buf), &tb, sizeof(tb)));
  lk_plan_launch(plans[NL / 2 - 1], st);
  lk_plan_launch(plans[NL / 2], st);
  uint64_t *null = nullptr;
  CK(hipStreamSynchronize(st));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lk_trace_buf), &null, sizeof(null)));
  std::vector<uint64_t> h((size_t)grid * kStreamWaves * 4);
  CK(hipMemcpy(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost));
  // the buffer holds the LAST of the two traced launches (each wave overwrites)
  uint64_t t0min = ~0ull;
  for (size_t w = 0; w < h.size() / 4; w++) if (h[w * 4]) t0min = std::min(t0min, h[w * 4]);
  const char *nm[4] = {"entry", "x ready", "1st unit", "exit"};
  for (int k = 0; k < 4; k++) {
    std::vector<double> v;
    for (size_t w = 0; w < h.size() / 4; w++) if (h[w * 4 + k]) v.push_back((h[w * 4 + k] - t0min) * 0.01);
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    auto pc = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))]; };
    printf("%-9s n=%5zu  min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", nm[k], v.size(), v.front(), pc(0.1), pc(0.5),
           pc(0.9), v.back());
  }
  // late finishers: mean exit per XCD (blockIdx % 8) and per contiguous eighth of the grid
  double xcd[8] = {0}, oct[8] = {0};
  int nx[8] = {0}, no[8] = {0};
  for (int g = 0; g < grid; g++) {
    for (int w = 0; w < kStreamWaves; w++) {
      uint64_t t = h[((size_t)g * kStreamWaves + w) * 4 + 3];
      if (!t) continue;
      double v = (t - t0min) * 0.01;
      xcd[g % 8] += v; nx[g % 8]++;
      oct[g * 8 / grid] += v; no[g * 8 / grid]++;
    }
  }
  printf("exit by xcd:   ");
  for (int i = 0; i < 8; i++) printf(" %6.2f", nx[i] ? xcd[i] / nx[i] : 0);
  printf("\nexit by octile:");
  for (int i = 0; i < 8; i++) printf(" %6.2f", no[i] ? oct[i] / no[i] : 0);
  printf("\n");
  // where the spread lives: inside a workgroup (its waves) or between workgroups (CUs)
  std::vector<double> wg_max, wg_min, wg_span, wave_mean;
  double tot = 0;
  int cnt = 0;
  for (int g = 0; g < grid; g++) {
    double mx = 0, mn = 1e30;
    for (int w = 0; w < kStreamWaves; w++) {
      uint64_t t = h[((size_t)g * kStreamWaves + w) * 4 + 3];
      if (!t) continue;
      const double v = (t - t0min) * 0.01;
      mx = std::max(mx, v); mn = std::min(mn, v);
      tot += v; cnt++;
    }
    if (mx > 0) { wg_max.push_back(mx); wg_min.push_back(mn); wg_span.push_back(mx - mn); }
  }
  auto stats = [](const char *name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    auto pc = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))]; };
    printf("%-22s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", name, v.front(), pc(0.1), pc(0.5), pc(0.9), v.back());
  };
  stats("workgroup last exit", wg_max);
  stats("workgroup first exit", wg_min);
  stats("span inside workgroup", wg_span);
  printf("mean wave exit %.2f us (a perfectly balanced launch ends about here)\n", cnt ? tot / cnt : 0.0);
  {  // the latest workgroups: index, last exit, its waves' first-unit and exit times
    std::vector<std::pair<double, int>> late;
    for (int g = 0; g < grid; g++) {
      double mx = 0;
      for (int w = 0; w < kStreamWaves; w++) {
        uint64_t t = h[((size_t)g * kStreamWaves + w) * 4 + 3];
        if (t) mx = std::max(mx, (t - t0min) * 0.01);
      }
      late.push_back({mx, g});
    }
    std::sort(late.rbegin(), late.rend());
    for (int i = 0; i < 10 && i < (int)late.size(); i++) {
      const int g = late[i].second;
      printf("late wg %3d (xcd %d) last exit %6.2f | 1st unit/exit per wave:", g, g % 8, late[i].first);
      for (int w = 0; w < kStreamWaves; w++) {
        const uint64_t *q = &h[((size_t)g * kStreamWaves + w) * 4];
        printf(" %.1f/%.1f", q[2] ? (q[2] - t0min) * 0.01 : -1.0, q[3] ? (q[3] - t0min) * 0.01 : -1.0);
      }
      printf("\n");
    }
  }
  // by wave index inside the workgroup: VALU arbitration favours the older wave of a SIMD pair
  printf("mean exit by wave index:");
  for (int w = 0; w < kStreamWaves; w++) {
    double sw = 0; int nw = 0;
    for (int g = 0; g < grid; g++) {
      uint64_t t = h[((size_t)g * kStreamWaves + w) * 4 + 3];
      if (t) { sw += (t - t0min) * 0.01; nw++; }
    }
    printf(" %6.2f", nw ? sw / nw : 0.0);
  }
  printf("\n");
#endif
  return 0;
}
