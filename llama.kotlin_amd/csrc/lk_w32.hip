// lk_w32.hip — the gemm_w32 / xsplit32 kernels (lk_wide32.hpp) in a translation unit of their own, built
// with -mllvm -amdgpu-mfma-vgpr-form: MFMA results land in VGPRs, where the scale FMAs read them (by
// default the compiler put each chain's result in AGPRs and copied it out with 16 v_accvgpr_read per
// chain and block).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/lk_hip.h"
#define LK_W32_KERNELS 1
#include "lk_kernels.hpp"
#include "lk_wide32.hpp"

namespace lk {

void w32_launch_xsplit(const XSplit32Args &xa, unsigned items, hipStream_t st) {
  const unsigned grid = (items + 4 * LK_XS32_IPW - 1) / (4 * LK_XS32_IPW);  // 4 waves per workgroup
  hipLaunchKernelGGL(xsplit32_kernel, dim3(grid), dim3(256), 0, st, xa);
}

void w32_launch(int qt, int mt, int nt, int mh, const W32Args &g, unsigned grid, size_t lds, hipStream_t st) {
  const dim3 b(256 * mh);
#define LK_W32_CASE(Q, A, B, C)                                                        \
  if (qt == Q && mt == A && nt == B && mh == C) {                                      \
    hipLaunchKernelGGL((gemm_w32_kernel<Q, A, B, C>), dim3(grid), b, lds, st, g);      \
    return;                                                                            \
  }
  LK_W32_CASE(LK_TYPE_Q4_0, 2, 2, 2)
  LK_W32_CASE(LK_TYPE_Q4_1, 2, 2, 2)
  LK_W32_CASE(LK_TYPE_Q4_0, 3, 1, 1)
  LK_W32_CASE(LK_TYPE_Q4_1, 3, 1, 1)
  LK_W32_CASE(LK_TYPE_Q4_0, 4, 2, 1)
  LK_W32_CASE(LK_TYPE_Q4_1, 4, 2, 1)
#undef LK_W32_CASE
}

}  // namespace lk

#ifdef LK_LAB_W32_STAMPS
extern "C" int lk_lab_w32_stamps(uint64_t *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lk::lk_w32_stamps), sizeof(uint64_t) * (size_t)n) == hipSuccess ? 0 : 5;
}
#endif
