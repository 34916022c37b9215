/*
 * lk_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of llama.kotlin's CPU computeMatMul path and the
 * numeric helpers it depends on. It is the parity checker for the HIP backend:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and never as the thing measured or shipped. The product library
 * (llama.kotlin_amd/csrc) does not link it and has no CPU fallback.
 *
 * The Kotlin/Native reference cannot be built or run in this image (no JDK,
 * kotlinc, konan or Gradle, no network: SURVEY.md §0.5 / §8c), so this
 * restatement is pinned by the reference's own known-answer tests (see
 * tests/test_oracle_kats.py) and IEEE f16 conversion (exhaustive), not by
 * bit-level outputs of the reference itself.
 *
 * Every function names the reference file:line it follows (paths relative to
 * src/nativeMain/kotlin/ai/solace/llamakotlin/). Compiled with
 * -ffp-contract=off -fno-fast-math: Kotlin/Native emits separate fmul/fadd.
 */
#ifndef LK_ORACLE_H
#define LK_ORACLE_H

#include <stdint.h>
#include "../include/lk_hip.h" /* lk_tensor / lk_type / lk_status (layout only) */

#ifdef __cplusplus
extern "C" {
#endif

/* core/NumericConversions.kt:9-54 */
float lko_half_to_float(uint16_t h);
/* core/NumericConversions.kt:61-124, including Kotlin's masked shift counts */
uint16_t lko_float_to_half(float f);
/* kotlin.math.round(Float): ties to even */
float lko_kotlin_round(float x);
/* Float.toInt(): NaN -> 0, saturating */
int32_t lko_float_to_int(float x);

/* Block byte size for a type (core/GGMLTypes.kt:99-133); 0 for non-block types. */
int lko_block_bytes(int32_t type);

/* quantizeTensor (core/GGMLComputeOps.kt:1040-1204) for a flat F32 array of n
 * elements (n % 32 == 0) into Q8_0/Q4_0/Q4_1 bytes. Returns lk_status. */
int lko_quantize(int32_t type, const float *src, int64_t n, uint8_t *out);
/* dequantizeTensor (core/GGMLComputeOps.kt:918-964) for n elements. */
int lko_dequantize(int32_t type, const uint8_t *src, int64_t n, float *out);

/* computeMatMul (core/GGMLComputeOps.kt:1435-1565), structural restatement:
 * per-element accessor work (f16 scale decode per weight, block index
 * recompute, bounds checks) exactly as the Kotlin path does it. */
int lko_compute_mat_mul(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst);
/* Same arithmetic order without the per-element accessor overhead ("tight"
 * CPU variant for the baseline); only Q4_0/Q4_1/Q8_0 x F32, contiguous B/dst. */
int lko_compute_mat_mul_tight(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst);
/* The tight variant with rows split over `threads` OpenMP threads (bit-identical: every
 * dot keeps its own order). The CPU baseline's all-cores line. */
int lko_compute_mat_mul_tight_mt(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int threads);

/* The direct dot products computeDotProduct{F32Q41, F32Q80, Q80Q80, Q40Q40, Q41Q41,
 * Q80Q40} (core/GGMLComputeOps.kt:349-629), kind = lk_dot_kind: one dot, and every
 * (row, col) of a.ne[1] x b.ne[0] into out (row-major). */
int lko_dot_direct(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, float *out);
int lko_dot_direct_matrix(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out);

/* Batch forms of the conversions (for exhaustive tests). */
void lko_half_to_float_n(const uint16_t *in, float *out, int64_t n);
void lko_float_to_half_n(const float *in, uint16_t *out, int64_t n);

/* Message for the last non-OK status. */
const char *lko_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
