// valu_rate.hip — lab: cycles per wave-instruction of VALU streams at one and two waves per
// SIMD (256- vs 512-thread workgroups, one workgroup per CU), with and without an MFMA stream in
// the same wave. Each lane runs ITER x 16 independent ops; s_memtime around the loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int ITER = 256;

template <int OP>
__global__ void k(float *out, uint64_t *cyc, float seed) {
  float a[16];
  uint32_t u[16];
  f2v v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) { a[i] = seed * (i + threadIdx.x); u[i] = __float_as_uint(a[i]); v[i] = f2v{a[i], a[i] + 1}; }
  f32x4 acc[4] = {};
  bf16x8 bx = __builtin_bit_cast(bf16x8, f32x4{seed, seed, seed, seed});
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if constexpr (OP == 0) a[i] = fmaf(a[i], 1.0001f, 0.5f);                                   // v_fma_f32
      if constexpr (OP == 1) v[i] = __builtin_elementwise_fma(v[i], f2v{1.0001f, 1.0001f}, f2v{0.5f, 0.5f});  // v_pk_fma_f32
      if constexpr (OP == 2) v[i] = __builtin_amdgcn_cvt_pk_f32_fp8(u[i] + it, false);           // cvt_pk_f32_fp8 (+ add)
      if constexpr (OP == 3) u[i] = __builtin_amdgcn_perm(u[i], u[(i + 1) & 15], 0x07060302u);  // v_perm_b32
      if constexpr (OP == 4) u[i] = (u[i] & 0x000F000Fu) | 0x43004300u;                         // v_and_or_b32
      if constexpr (OP == 5) {                                                                   // fma + MFMA 1:4
        a[i] = fmaf(a[i], 1.0001f, 0.5f);
        if ((i & 3) == 0) acc[i >> 2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, bx, acc[i >> 2], 0, 0, 0);
      }
      if constexpr (OP == 6) {                                                                   // MFMA only
        if ((i & 3) == 0) acc[i >> 2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, bx, acc[i >> 2], 0, 0, 0);
      }
    }
    asm volatile("" ::: "memory");
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += a[i] + v[i].x + v[i].y + __uint_as_float(u[i]);
  for (int i = 0; i < 4; i++) s += acc[i].x + acc[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char *name, int threads) {
  const int grid = 256;
  float *out;
  uint64_t *cyc;
  CK(hipMalloc(&out, 4 * grid * threads));
  CK(hipMalloc(&cyc, 8 * grid * threads / 64));
  for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(threads), 0, 0, out, cyc, 1.0f);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h(grid * threads / 64);
  CK(hipMemcpy(h.data(), cyc, 8 * h.size(), hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double per = (double)h[h.size() / 2] / (ITER * 16.0);
  printf("%-26s waves/SIMD=%d  cycles per loop-op per wave: %.2f\n", name, threads / 256, per);
  CK(hipFree(out));
  CK(hipFree(cyc));
}

int main() {
  for (int t : {256, 512}) {
    run<0>("v_fma_f32", t);
    run<1>("v_pk_fma_f32", t);
    run<2>("cvt_pk_f32_fp8 (+v_add)", t);
    run<3>("v_perm_b32", t);
    run<4>("v_and_or_b32", t);
    run<5>("v_fma + mfma16x16x32/4", t);
    run<6>("mfma16x16x32 per 4 ops", t);
  }
  return 0;
}
