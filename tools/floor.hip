// Launch floors of the batch-1 stream shape (lab tool, not part of the product): an empty
// kernel and a bare LDS-DMA read of a matrix's bytes, both at the stream kernel's grid (one
// 512-thread workgroup per CU) and LDS size, for tools/floor.py to time in HIP-graph replay.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libfloor.so tools/floor.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LK_GLOBAL __attribute__((address_space(1)))
#define LK_LDS __attribute__((address_space(3)))

// per (workgroup, wave): entry, first weight piece landed, exit (s_memrealtime, 100 MHz)
__device__ uint64_t floor_st[1024 * 8 * 4];

__global__ __launch_bounds__(512) void empty_kernel(float *out) {
  if (out && threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1.f;
}

// Each workgroup reads its contiguous share of `bytes` as 1-KB LDS-DMA pieces, DEPTH pieces in
// flight per wave, and stores one word per workgroup (the last piece's first dword).
template <int DEPTH>
__global__ __launch_bounds__(512) void read_kernel(const uint8_t *src, int64_t bytes, const float *x, int xbytes,
                                                   float *out) {
  extern __shared__ uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
  uint64_t t_first = 0;
  const int64_t per = (bytes / gridDim.x) & ~(int64_t)1023;
  const LK_GLOBAL uint8_t *base = (const LK_GLOBAL uint8_t *)src + per * blockIdx.x;
  const int64_t npieces = per / 1024;
  if (x)  // the activation image first, as the stream kernel does
    for (int k = wave; k < xbytes / 1024; k += 8)
      __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)((const LK_GLOBAL uint8_t *)x + k * 1024 + lane * 16),
                                       (LK_LDS void *)(lds + 140 * 1024 + (k % 16) * 1024), 16, 0, 0);
  int slot = 0;
  for (int64_t p = wave; p < npieces; p += 8) {
    __builtin_amdgcn_global_load_lds((const LK_GLOBAL void *)(base + p * 1024 + lane * 16),
                                     (LK_LDS void *)(lds + (wave * DEPTH + slot) * 1024), 16, 0, 2);
    slot = slot + 1 == DEPTH ? 0 : slot + 1;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
    if (!t_first && p >= wave + 8 * (DEPTH - 1)) t_first = __builtin_amdgcn_s_memrealtime();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!t_first) t_first = __builtin_amdgcn_s_memrealtime();
  const uint64_t t_exit = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < 1024) {
    uint64_t *st = floor_st + ((size_t)blockIdx.x * 8 + wave) * 4;
    st[0] = t_entry; st[1] = t_first; st[2] = t_exit;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = *(const float *)(lds);
}

extern "C" {
int floor_stamps(uint64_t *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(floor_st), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
int floor_empty(int grid, int lds, float *out, void *stream) {
  hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(512), lds, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}
int floor_read(const void *src, int64_t bytes, const float *x, int xbytes, int grid, int depth, float *out,
               void *stream) {
  const size_t lds = 160 * 1024;
  if (depth == 6)
    hipLaunchKernelGGL(read_kernel<6>, dim3(grid), dim3(512), lds, (hipStream_t)stream, (const uint8_t *)src, bytes, x,
                       xbytes, out);
  else
    hipLaunchKernelGGL(read_kernel<12>, dim3(grid), dim3(512), lds, (hipStream_t)stream, (const uint8_t *)src, bytes,
                       x, xbytes, out);
  return (int)hipGetLastError();
}
}
