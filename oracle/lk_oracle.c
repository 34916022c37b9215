/*
 * lk_oracle.c — TEST INFRASTRUCTURE ONLY (see lk_oracle.h).
 *
 * Plain-C restatement of llama.kotlin's CPU MUL_MAT path. Paths below are
 * relative to src/nativeMain/kotlin/ai/solace/llamakotlin/ of the reference.
 * Kotlin `Int` arithmetic is 32-bit two's complement with shift counts masked
 * to 5 bits; the helpers kshl/kushr reproduce that, because floatToHalf's
 * denormal branch depends on it.
 *
 * Build: oracle/Makefile (-O2 -ffp-contract=off -fno-fast-math).
 */
#include "lk_oracle.h"

#include <fenv.h>
#include <math.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

static __thread char g_err[512];

static int fail(int status, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return status;
}

const char *lko_last_error(void) { return g_err; }

/* ---- Kotlin Int helpers ------------------------------------------------ */

static inline int32_t kshl(int32_t x, int32_t s) { return (int32_t)((uint32_t)x << (s & 31)); }
static inline int32_t kushr(int32_t x, int32_t s) { return (int32_t)((uint32_t)x >> (s & 31)); }
static inline int32_t kadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t ksub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

static inline float bits_to_float(int32_t b) {
  float f;
  memcpy(&f, &b, 4);
  return f;
}
static inline int32_t float_to_bits(float f) {
  int32_t b;
  memcpy(&b, &f, 4);
  return b;
}

/* ---- NumericConversions.kt ---------------------------------------------- */

/* halfToFloat — core/NumericConversions.kt:9-54 */
float lko_half_to_float(uint16_t h_bits) {
  int32_t h = (int32_t)h_bits & 0xFFFF;
  const int32_t f32Infinity = 0x7F800000;
  int32_t hSign = kushr(h, 15);
  int32_t hExp = kushr(h, 10) & 0x1F;
  int32_t hMant = h & 0x03FF;
  if (hExp == 0) {
    if (hMant == 0) return bits_to_float(kshl(hSign, 31)); /* :20-21 */
    int32_t mant = hMant, exp = hExp;                      /* :23-36 */
    while ((mant & 0x0400) == 0) {
      mant = kshl(mant, 1);
      exp--;
    }
    mant &= 0x03FF;
    int32_t f32Exp = (exp + 1) + (127 - 15);
    int32_t f32Mant = kshl(mant, 13);
    return bits_to_float(kshl(hSign, 31) | kshl(f32Exp, 23) | f32Mant);
  } else if (hExp == 0x1F) {
    if (hMant == 0) return bits_to_float(kshl(hSign, 31) | f32Infinity); /* :40 */
    /* :44 quiet NaN, payload << 13 */
    return bits_to_float(kshl(hSign, 31) | f32Infinity | kshl(hMant, 13) | kshl(1, 22));
  }
  int32_t f32Sign = kshl(hSign, 31); /* :47-52 */
  int32_t f32Exp = kshl(hExp - 15 + 127, 23);
  int32_t f32Mant = kshl(hMant, 13);
  return bits_to_float(f32Sign | f32Exp | f32Mant);
}

/* floatToHalf — core/NumericConversions.kt:61-124, bit for bit (Kotlin shifts). */
uint16_t lko_float_to_half(float f_val) {
  int32_t f32bits = float_to_bits(f_val);
  int32_t fSign = kushr(f32bits, 16) & 0x8000;
  int32_t absF = f32bits & 0x7FFFFFFF;

  if (absF > 0x47FFEFFF) { /* :67-73 (note: threshold ~131056, not 65520) */
    int mantissaIsNonZero = (absF & 0x007FFFFF) != 0;
    return (uint16_t)(fSign | 0x7C00 | (mantissaIsNonZero ? 0x0200 : 0));
  }
  if (absF < 0x38800000) { /* :75-104 denormal / zero */
    int32_t fMant = (absF & 0x007FFFFF) | 0x00800000;
    int32_t shift = 127 - kushr(absF, 23);
    int32_t hMant = (shift < 24) ? kushr(fMant, shift) : 0;
    int32_t roundBits = fMant & ksub(kshl(1, shift), 1);
    int32_t half = kshl(1, shift - 1);
    if (roundBits > half || (roundBits == half && (hMant & 1) != 0)) {
      int32_t h_temp = hMant + 1;
      if (h_temp == 0x0400) return (uint16_t)(fSign | kshl(1, 10));
      return (uint16_t)(fSign | h_temp);
    }
    return (uint16_t)(fSign | hMant);
  }
  /* :106-123 normal */
  int32_t hExp = kshl(kushr(absF, 23) - 112, 10);
  int32_t hMant = kushr(absF & 0x007FFFFF, 13);
  if ((absF & 0x00001000) != 0) {
    if ((absF & 0x00000FFF) != 0 || (hMant & 1) != 0) {
      hMant++;
      if (hMant == 0x0400) {
        hMant = 0;
        return (uint16_t)(fSign | kadd(hExp, kshl(1, 10)) | hMant);
      }
    }
  }
  return (uint16_t)(fSign | hExp | hMant);
}

void lko_half_to_float_n(const uint16_t *in, float *out, int64_t n) {
  for (int64_t i = 0; i < n; i++) out[i] = lko_half_to_float(in[i]);
}
void lko_float_to_half_n(const float *in, uint16_t *out, int64_t n) {
  for (int64_t i = 0; i < n; i++) out[i] = lko_float_to_half(in[i]);
}

/* kotlin.math.round(Float): round half to even. */
float lko_kotlin_round(float x) {
  int old = fegetround();
  if (old != FE_TONEAREST) fesetround(FE_TONEAREST);
  float r = rintf(x);
  if (old != FE_TONEAREST) fesetround(old);
  return r;
}

/* Float.toInt(): NaN -> 0, saturating. */
int32_t lko_float_to_int(float x) {
  if (isnan(x)) return 0;
  if (x >= 2147483648.0f) return INT32_MAX;
  if (x <= -2147483648.0f) return INT32_MIN;
  return (int32_t)x;
}

static inline int32_t coerce_in(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

/* kotlin maxOf/minOf(Float, Float): NaN-propagating, -0.0 < +0.0 */
static inline float kmax(float a, float b) {
  if (isnan(a) || isnan(b)) return NAN;
  if (a == 0.0f && b == 0.0f) return signbit(a) ? b : a;
  return a > b ? a : b;
}
static inline float kmin(float a, float b) {
  if (isnan(a) || isnan(b)) return NAN;
  if (a == 0.0f && b == 0.0f) return signbit(a) ? a : b;
  return a < b ? a : b;
}

/* ---- GGMLTypes.kt tensor model -------------------------------------------- */

int lko_block_bytes(int32_t type) { /* core/GGMLTypes.kt:99-114 */
  switch (type) {
    case LK_TYPE_Q4_0: return LK_Q4_0_BLOCK_BYTES;
    case LK_TYPE_Q4_1: return LK_Q4_1_BLOCK_BYTES;
    case LK_TYPE_Q8_0: return LK_Q8_0_BLOCK_BYTES;
    case LK_TYPE_Q2_K: return LK_Q2_K_BLOCK_BYTES; /* :117 */
    case LK_TYPE_Q4_K: return LK_Q4_K_BLOCK_BYTES; /* :119 */
    case LK_TYPE_Q8_K: return LK_Q8_K_BLOCK_BYTES; /* :122 */
    default: return 0;
  }
}

/* rank — core/GGMLTypes.kt:275-280 */
static int t_rank(const lk_tensor *t) {
  int all_le1 = 1, any_gt0 = 0, last = -1;
  for (int i = 0; i < 4; i++) {
    if (t->ne[i] > 1) all_le1 = 0;
    if (t->ne[i] > 0) any_gt0 = 1;
    if (t->ne[i] > 1) last = i;
  }
  if (all_le1) return any_gt0 ? 1 : 0;
  return last + 1;
}

/* numElements — core/GGMLTypes.kt:286-300 */
static int64_t t_num_elements(const lk_tensor *t) {
  int64_t count = 1;
  int r = t_rank(t);
  int all_le1 = 1, any_eq0 = 0;
  for (int i = 0; i < 4; i++) {
    if (t->ne[i] > 1) all_le1 = 0;
    if (t->ne[i] == 0) any_eq0 = 1;
  }
  if (r == 0 && all_le1) return 1;
  if (r == 0 && any_eq0) return 0;
  int lim = r < 1 ? 1 : r;
  for (int i = 0; i < lim; i++) {
    if (t->ne[i] == 0 && r > 1) return 0;
    if (t->ne[i] > 0) count *= t->ne[i];
  }
  return count;
}

/* getNumBlocks — core/GGMLTypes.kt:507-535 (Q types of this path) */
static int64_t t_num_blocks(const lk_tensor *t) {
  int64_t total = t_num_elements(t);
  if (total == 0) return 0;
  if (t->type == LK_TYPE_Q4_0 || t->type == LK_TYPE_Q4_1 || t->type == LK_TYPE_Q8_0) return total / 32;
  if (t->type == LK_TYPE_Q2_K || t->type == LK_TYPE_Q4_K || t->type == LK_TYPE_Q8_K) return total / LK_QK_K; /* :518 */
  return 0;
}

static inline uint16_t rd_u16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline float rd_f32(const uint8_t *p) {
  uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  float f;
  memcpy(&f, &v, 4);
  return f;
}
static inline void wr_f32(uint8_t *p, float f) {
  uint32_t v;
  memcpy(&v, &f, 4);
  p[0] = v & 0xFF; p[1] = (v >> 8) & 0xFF; p[2] = (v >> 16) & 0xFF; p[3] = (v >> 24) & 0xFF;
}

/* Accessors return lk_status via *st; on error the value is 0. */

/* getElementByteOffset + buffer lookup + bounds: getFloat/setFloat/getHalf
 * (core/GGMLTypes.kt:328-380, :426-452). Two indices (2-D access as computeMatMul uses). */
static int elem_offset(const lk_tensor *t, int64_t i0, int64_t i1, uint64_t width, uint64_t *off) {
  if (t->data == NULL) return fail(LK_ERR_NO_BUFFER, "Tensor buffer not found");
  if (i0 < 0 || i0 >= t->ne[0]) return fail(LK_ERR_INVALID_ARG, "Index %lld for dimension 0 is out of bounds", (long long)i0);
  if (i1 < 0 || i1 >= t->ne[1]) return fail(LK_ERR_INVALID_ARG, "Index %lld for dimension 1 is out of bounds", (long long)i1);
  uint64_t o = t->data_offset + (uint64_t)i0 * t->nb[0] + (uint64_t)i1 * t->nb[1];
  if (o + width > t->buf_bytes) return fail(LK_ERR_OUT_OF_BOUNDS, "Calculated offset %llu + %llu bytes is out of bounds for buffer size %llu",
                                             (unsigned long long)o, (unsigned long long)width, (unsigned long long)t->buf_bytes);
  *off = o;
  return LK_OK;
}

static float get_float(const lk_tensor *t, int64_t i0, int64_t i1, int *st) {
  uint64_t o;
  *st = elem_offset(t, i0, i1, 4, &o);
  return *st ? 0.0f : rd_f32((const uint8_t *)t->data + o);
}
static void set_float(lk_tensor *t, float v, int64_t i0, int64_t i1, int *st) {
  uint64_t o;
  *st = elem_offset(t, i0, i1, 4, &o);
  if (!*st) wr_f32((uint8_t *)t->data + o, v);
}
static float get_half(const lk_tensor *t, int64_t i0, int64_t i1, int *st) {
  uint64_t o;
  *st = elem_offset(t, i0, i1, 2, &o);
  return *st ? 0.0f : lko_half_to_float(rd_u16((const uint8_t *)t->data + o));
}
static void set_half(lk_tensor *t, float v, int64_t i0, int64_t i1, int *st) {
  uint64_t o;
  *st = elem_offset(t, i0, i1, 2, &o);
  if (!*st) {
    uint16_t h = lko_float_to_half(v);
    uint8_t *p = (uint8_t *)t->data + o;
    p[0] = h & 0xFF;
    p[1] = h >> 8;
  }
}

/* Block-relative byte: common body of getQ*_BlockScale / getQ*_Weight
 * (core/GGMLTypes.kt:543-732): require(type), require(0<=blk<numBlocks),
 * buffer lookup, bounds check, read. `width` bytes at `inner` inside the block. */
static const uint8_t *block_byte(const lk_tensor *t, int32_t want_type, int64_t blk, uint64_t inner, uint64_t width, int *st) {
  if (t->type != want_type) { *st = fail(LK_ERR_INVALID_ARG, "Tensor type mismatch for block accessor"); return NULL; }
  int64_t nblk = t_num_blocks(t);
  if (blk < 0 || blk >= nblk) { *st = fail(LK_ERR_INVALID_ARG, "blockIndex %lld out of bounds for %lld blocks", (long long)blk, (long long)nblk); return NULL; }
  if (t->data == NULL) { *st = fail(LK_ERR_NO_BUFFER, "Tensor buffer not found"); return NULL; }
  uint64_t o = t->data_offset + (uint64_t)blk * (uint64_t)lko_block_bytes(want_type) + inner;
  if (o + width > t->buf_bytes) { *st = fail(LK_ERR_OUT_OF_BOUNDS, "block read at offset %llu out of buffer bounds", (unsigned long long)o); return NULL; }
  *st = LK_OK;
  return (const uint8_t *)t->data + o;
}

/* getQ8_0BlockScale :543-562, getQ4_0BlockScale :598-617, getQ4_1BlockScale :660-677 */
static float q_scale(const lk_tensor *t, int32_t type, int64_t blk, int *st) {
  const uint8_t *p = block_byte(t, type, blk, 0, 2, st);
  return p ? lko_half_to_float(rd_u16(p)) : 0.0f;
}
/* getQ4_1BlockMin :682-700 */
static float q41_min(const lk_tensor *t, int64_t blk, int *st) {
  const uint8_t *p = block_byte(t, LK_TYPE_Q4_1, blk, 2, 2, st);
  return p ? lko_half_to_float(rd_u16(p)) : 0.0f;
}
/* getQ4_0NibbleWeight :627-653 / getQ4_1NibbleWeight :706-732 — interleaved nibbles */
static int32_t q4_nibble(const lk_tensor *t, int32_t type, int64_t blk, int32_t item, int *st) {
  if (item < 0 || item >= 32) { *st = fail(LK_ERR_INVALID_ARG, "itemIndexInBlock out of bounds"); return 0; }
  uint64_t base = (type == LK_TYPE_Q4_0) ? 2 : 4;
  const uint8_t *p = block_byte(t, type, blk, base + (uint64_t)(item / 2), 1, st);
  if (!p) return 0;
  int32_t packed = (int32_t)(int8_t)p[0];
  return (item % 2 == 0) ? (packed & 0x0F) : (kushr(packed, 4) & 0x0F);
}
/* getQ8_0Weight :571-588 */
static int32_t q8_weight(const lk_tensor *t, int64_t blk, int32_t item, int *st) {
  if (item < 0 || item >= 32) { *st = fail(LK_ERR_INVALID_ARG, "itemIndexInBlock out of bounds"); return 0; }
  const uint8_t *p = block_byte(t, LK_TYPE_Q8_0, blk, 2 + (uint64_t)item, 1, st);
  return p ? (int32_t)(int8_t)p[0] : 0;
}

/* ---- quantize / dequantize (core/GGMLComputeOps.kt:918-964, :1040-1204) ----- */

static void put_u16(uint8_t *p, uint16_t v) { p[0] = v & 0xFF; p[1] = v >> 8; }

int lko_quantize(int32_t type, const float *src, int64_t n, uint8_t *out) {
  if (n % 32 != 0) return fail(LK_ERR_INVALID_ARG, "numElements %lld not div by 32", (long long)n);
  int64_t nblk = n / 32;
  for (int64_t b = 0; b < nblk; b++) {
    const float *x = src + b * 32;
    if (type == LK_TYPE_Q8_0) { /* :1063-1071 */
      uint8_t *o = out + b * LK_Q8_0_BLOCK_BYTES;
      float amax = 0.0f;
      for (int k = 0; k < 32; k++) amax = kmax(amax, fabsf(x[k]));
      float scale = (amax == 0.0f) ? 1.0f : amax / 127.0f;
      float invS = 1.0f / scale;
      put_u16(o, lko_float_to_half(scale));
      for (int k = 0; k < 32; k++) {
        float prod = x[k] * invS;
        o[2 + k] = (uint8_t)(int8_t)coerce_in(lko_float_to_int(lko_kotlin_round(prod)), -128, 127);
      }
    } else if (type == LK_TYPE_Q4_0) { /* :1073-1087 */
      uint8_t *o = out + b * LK_Q4_0_BLOCK_BYTES;
      float amax = 0.0f;
      for (int k = 0; k < 32; k++) amax = kmax(amax, fabsf(x[k]));
      float scale = (amax == 0.0f) ? 1.0f : amax / 8.0f;
      float invS = (scale == 0.0f) ? 0.0f : 1.0f / scale;
      put_u16(o, lko_float_to_half(scale));
      for (int j = 0; j < 16; j++) {
        float t1 = x[2 * j] * invS;
        t1 = t1 + 8.0f;
        float t2 = x[2 * j + 1] * invS;
        t2 = t2 + 8.0f;
        int32_t q1 = coerce_in(lko_float_to_int(lko_kotlin_round(t1)), 0, 15);
        int32_t q2 = coerce_in(lko_float_to_int(lko_kotlin_round(t2)), 0, 15);
        o[2 + j] = (uint8_t)((q1 & 0x0F) | ((q2 & 0x0F) << 4));
      }
    } else if (type == LK_TYPE_Q4_1) { /* :1161-1199 */
      uint8_t *o = out + b * LK_Q4_1_BLOCK_BYTES;
      float f_min = x[0], f_max = x[0]; /* FloatArray.minOrNull / maxOrNull */
      for (int k = 1; k < 32; k++) { f_min = kmin(f_min, x[k]); f_max = kmax(f_max, x[k]); }
      float d = (f_max - f_min) / 15.0f;
      if (d == 0.0f) d = 1.0f;
      float m = f_min;
      float invD = 1.0f / d;
      put_u16(o, lko_float_to_half(d));
      put_u16(o + 2, lko_float_to_half(m));
      for (int j = 0; j < 16; j++) {
        float t1 = (x[2 * j] - m) * invD;
        float t2 = (x[2 * j + 1] - m) * invD;
        int32_t q1 = coerce_in(lko_float_to_int(lko_kotlin_round(t1)), 0, 15);
        int32_t q2 = coerce_in(lko_float_to_int(lko_kotlin_round(t2)), 0, 15);
        o[4 + j] = (uint8_t)((q1 & 0x0F) | ((q2 & 0x0F) << 4));
      }
    } else {
      return fail(LK_ERR_NOT_IMPLEMENTED, "quantize: unsupported type %d", type);
    }
  }
  return LK_OK;
}

int lko_dequantize(int32_t type, const uint8_t *src, int64_t n, float *out) {
  if (n % 32 != 0) return fail(LK_ERR_INVALID_ARG, "numElements %lld not div by 32", (long long)n);
  for (int64_t b = 0; b < n / 32; b++) {
    if (type == LK_TYPE_Q8_0) { /* :929-935 */
      const uint8_t *p = src + b * LK_Q8_0_BLOCK_BYTES;
      float d = lko_half_to_float(rd_u16(p));
      for (int k = 0; k < 32; k++) out[b * 32 + k] = d * (float)(int8_t)p[2 + k];
    } else if (type == LK_TYPE_Q4_0) { /* :936-943 */
      const uint8_t *p = src + b * LK_Q4_0_BLOCK_BYTES;
      float d = lko_half_to_float(rd_u16(p));
      for (int k = 0; k < 32; k++) {
        int q = (k & 1) ? (p[2 + k / 2] >> 4) : (p[2 + k / 2] & 0x0F);
        float qm = (float)q - 8.0f;
        out[b * 32 + k] = d * qm;
      }
    } else if (type == LK_TYPE_Q4_1) { /* :944-957 — d*q then + m: two roundings */
      const uint8_t *p = src + b * LK_Q4_1_BLOCK_BYTES;
      float d = lko_half_to_float(rd_u16(p));
      float m = lko_half_to_float(rd_u16(p + 2));
      for (int k = 0; k < 32; k++) {
        int q = (k & 1) ? (p[4 + k / 2] >> 4) : (p[4 + k / 2] & 0x0F);
        float dq = d * (float)q;
        out[b * 32 + k] = dq + m;
      }
    } else {
      return fail(LK_ERR_NOT_IMPLEMENTED, "dequantize: unsupported type %d", type);
    }
  }
  return LK_OK;
}

/* ---- dot products (core/GGMLComputeOps.kt:43-145) ----------------------- */

/* computeDotProductQ40F32 — :120-145 */
static float dot_q40_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  float sum = 0.0f;
  for (int64_t k = 0; k < K; k++) {
    int64_t flat = row * K + k;
    int64_t blk = flat / 32;
    int32_t item = (int32_t)(flat % 32);
    float scale = q_scale(a, LK_TYPE_Q4_0, blk, st); if (*st) return 0;
    int32_t q = q4_nibble(a, LK_TYPE_Q4_0, blk, item, st); if (*st) return 0;
    float qm = (float)q - 8.0f;
    float w = scale * qm;
    float x = get_float(b, col, k, st); if (*st) return 0;
    float p = w * x;
    sum = sum + p;
  }
  return sum;
}

/* computeDotProductQ41F32 — :70-115 (d*q + m: two roundings) */
static float dot_q41_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  int64_t M = a->ne[1], N = b->ne[0];
  if (!(row < M)) { *st = fail(LK_ERR_INVALID_ARG, "rowIndexInQ41 out of bounds"); return 0; } /* :87 */
  if (!(col < N)) { *st = fail(LK_ERR_INVALID_ARG, "colIndexInF32 out of bounds"); return 0; } /* :88 */
  float sum = 0.0f;
  for (int64_t k = 0; k < K; k++) {
    int64_t flat = row * K + k;
    int64_t blk = flat / 32;
    int32_t item = (int32_t)(flat % 32);
    float d = q_scale(a, LK_TYPE_Q4_1, blk, st); if (*st) return 0;
    float m = q41_min(a, blk, st); if (*st) return 0;
    int32_t q = q4_nibble(a, LK_TYPE_Q4_1, blk, item, st); if (*st) return 0;
    float dq = d * (float)q;
    float w = dq + m;
    float x = get_float(b, col, k, st); if (*st) return 0;
    float p = w * x;
    sum = sum + p;
  }
  return sum;
}

/* computeDotProductQ80F32 — :43-68 */
static float dot_q80_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  float sum = 0.0f;
  for (int64_t k = 0; k < K; k++) {
    int64_t flat = row * K + k;
    int64_t blk = flat / 32;
    int32_t item = (int32_t)(flat % 32);
    float scale = q_scale(a, LK_TYPE_Q8_0, blk, st); if (*st) return 0;
    int32_t q = q8_weight(a, blk, item, st); if (*st) return 0;
    float w = scale * (float)q;
    float x = get_float(b, col, k, st); if (*st) return 0;
    float p = w * x;
    sum = sum + p;
  }
  return sum;
}


/* ---- K-quants (core/GGMLComputeOps.kt:152-432, core/GGMLTypes.kt:734-916) ----------------
 * Block layouts (llama.kotlin's, core/GGMLTypes.kt:117-122 and the accessors):
 *   Q2_K (84 B):  scales[16] | qs[64] | d f16 @80 | dmin f16 @82
 *   Q4_K (144 B): d f16 @0 | dmin f16 @2 | scales[12] @4 | qs[128] @16
 *   Q8_K (292 B): d f32 @0 | qs[256] int8 @4 | bsums[16] int16 @260 (not read)
 * The "full block" paths take blockIndex = (row*K + blockStart) / 256 and read its items
 * 0..255 for k = blockStart..blockStart+255, also when K % 256 != 0 (then that block does not
 * start at the row's k = blockStart); the trailing partial block goes element by element
 * through the flat index, with its own formulas (Q4_K's partial path adds dmin, not min). */

/* raw buffer byte (buffer[offset], Kotlin ByteArray index: AIOOBE past the end) */
static int raw_byte(const lk_tensor *t, uint64_t off, int *st) {
  if (t->data == NULL) { *st = fail(LK_ERR_NO_BUFFER, "Tensor buffer not found"); return 0; }
  if (off >= t->buf_bytes) { *st = fail(LK_ERR_OUT_OF_BOUNDS, "buffer index %llu out of bounds", (unsigned long long)off); return 0; }
  *st = LK_OK;
  return (int)(int8_t)((const uint8_t *)t->data)[off]; /* Byte: signed */
}
/* getQ2_KBlockScale :740-752 (d @ 16+64), getQ2_KBlockScaleMin :757-769 (dmin @ 82) */
static float q2k_d(const lk_tensor *t, int64_t blk, uint64_t inner, int *st) {
  const uint8_t *p = block_byte(t, LK_TYPE_Q2_K, blk, inner, 2, st);
  return p ? lko_half_to_float(rd_u16(p)) : 0.0f;
}
/* getQ2_KScale :774-783 / getQ2_KQuant :788-797: index range only, then buffer[...] */
static int q2k_byte(const lk_tensor *t, int64_t blk, uint64_t inner, int *st) {
  return raw_byte(t, t->data_offset + (uint64_t)blk * LK_Q2_K_BLOCK_BYTES + inner, st);
}
/* getQ4_KBlockScale :822-833 (d @ 0), getQ4_KBlockScaleMin :838-849 (dmin @ 2) */
static float q4k_d(const lk_tensor *t, int64_t blk, uint64_t inner, int *st) {
  const uint8_t *p = block_byte(t, LK_TYPE_Q4_K, blk, inner, 2, st);
  return p ? lko_half_to_float(rd_u16(p)) : 0.0f;
}
/* getQ8_KBlockScale :881-894 (getFloatLe @ 0), getQ8_KWeight :903-916 */
static float q8k_d(const lk_tensor *t, int64_t blk, int *st) {
  const uint8_t *p = block_byte(t, LK_TYPE_Q8_K, blk, 0, 4, st);
  return p ? rd_f32(p) : 0.0f;
}
static int32_t q8k_weight(const lk_tensor *t, int64_t blk, int32_t item, int *st) {
  const uint8_t *p = block_byte(t, LK_TYPE_Q8_K, blk, 4 + (uint64_t)item, 1, st);
  return p ? (int32_t)(int8_t)p[0] : 0;
}

/* Q2_K scale/min of sub-block sb: (qs/15)*d, qm*d + dmin — :182-187 */
static void q2k_scale_min(int sm, float d, float dmin, float *scale, float *min) {
  const int32_t qs = sm & 0x0F, qm = kushr(sm, 4) & 0x0F; /* shr on the sign-extended byte, & 0x0F */
  const float r = (float)qs / 15.0f;
  *scale = r * d;
  const float md = (float)qm * d;
  *min = md + dmin;
}
/* (q/3)*scale + min — :196, :227 */
static float q2k_value(int32_t q, float scale, float min) {
  const float r = (float)q / 3.0f;
  const float t = r * scale;
  return t + min;
}

/* computeDotProductQ2_KF32 — :152-234 */
static float dot_q2k_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  float sum = 0.0f;
  for (int64_t bs = 0; bs < K; bs += LK_QK_K) {
    const int64_t be = bs + LK_QK_K < K ? bs + LK_QK_K : K;
    if (be - bs == LK_QK_K) {
      const int64_t blk = (row * K + bs) / LK_QK_K;
      const float d = q2k_d(a, blk, 80, st); if (*st) return 0;
      const float dmin = q2k_d(a, blk, 82, st); if (*st) return 0;
      for (int sb = 0; sb < LK_QK_K / 16; sb++) {
        const int sm = q2k_byte(a, blk, (uint64_t)sb, st); if (*st) return 0;
        float scale, min;
        q2k_scale_min(sm, d, dmin, &scale, &min);
        for (int i = 0; i < 16; i += 4) {
          const int qb = q2k_byte(a, blk, 16 + (uint64_t)(sb * 4 + i / 4), st); if (*st) return 0;
          for (int j = 0; j < 4; j++) {
            const int64_t k = bs + sb * 16 + i + j;
            if (k < be) {
              const int32_t q = kushr(qb, j * 2) & 0x03; /* qb >> 2j on the sign-extended byte */
              const float w = q2k_value(q, scale, min);
              const float x = get_float(b, col, k, st); if (*st) return 0;
              const float p = w * x;
              sum = sum + p;
            }
          }
        }
      }
    } else {
      for (int64_t k = bs; k < be; k++) {
        const int64_t flat = row * K + k, blk = flat / LK_QK_K;
        const int32_t item = (int32_t)(flat % LK_QK_K);
        const float d = q2k_d(a, blk, 80, st); if (*st) return 0;
        const float dmin = q2k_d(a, blk, 82, st); if (*st) return 0;
        const int sb = item / 16;
        const int sm = q2k_byte(a, blk, (uint64_t)sb, st); if (*st) return 0;
        float scale, min;
        q2k_scale_min(sm, d, dmin, &scale, &min);
        const int qb = q2k_byte(a, blk, 16 + (uint64_t)(sb * 4 + (item % 16) / 4), st); if (*st) return 0;
        const int32_t q = kushr(qb, ((item % 16) % 4) * 2) & 0x03;
        const float w = q2k_value(q, scale, min);
        const float x = get_float(b, col, k, st); if (*st) return 0;
        const float p = w * x;
        sum = sum + p;
      }
    }
  }
  return sum;
}

/* (q/15)*scale + off — :297-306, :331 */
static float q4k_value(int32_t q, float scale, float off) {
  const float r = (float)q / 15.0f;
  const float t = r * scale;
  return t + off;
}

/* computeDotProductQ4_KF32 — :241-339 */
static float dot_q4k_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  float sum = 0.0f;
  for (int64_t bs = 0; bs < K; bs += LK_QK_K) {
    const int64_t be = bs + LK_QK_K < K ? bs + LK_QK_K : K;
    if (be - bs == LK_QK_K) {
      const int64_t blk = (row * K + bs) / LK_QK_K;
      const float d = q4k_d(a, blk, 0, st); if (*st) return 0;
      const float dmin = q4k_d(a, blk, 2, st); if (*st) return 0;
      const uint64_t bo = a->data_offset + (uint64_t)blk * LK_Q4_K_BLOCK_BYTES;
      for (int sb = 0; sb < 8; sb++) {
        const int sc = raw_byte(a, bo + 4 + (uint64_t)sb, st); if (*st) return 0;
        const int32_t qs = sc & 0x3F, qml = kushr(sc, 6) & 0x03;
        int32_t qmh = 0;
        if (sb * 2 + 1 < LK_K_SCALE_SIZE) { qmh = raw_byte(a, bo + 4 + (uint64_t)(sb * 2 + 1), st) & 0x0F; if (*st) return 0; }
        const int32_t qm = qml | kshl(qmh, 2);
        const float scale = ((float)qs / 63.0f) * d;
        const float mr = (float)qm / 63.0f;
        const float mt = mr * d;
        const float min = mt + dmin;
        const uint64_t qo = bo + 4 + LK_K_SCALE_SIZE + (uint64_t)sb * 16;
        for (int i = 0; i < 32; i += 2) {
          const int64_t k1 = bs + sb * 32 + i, k2 = k1 + 1;
          if (k1 < be) {
            const int qb = raw_byte(a, qo + (uint64_t)(i / 2), st); if (*st) return 0;
            const float w1 = q4k_value(qb & 0x0F, scale, min);
            const float x1 = get_float(b, col, k1, st); if (*st) return 0;
            const float p1 = w1 * x1;
            sum = sum + p1;
            if (k2 < be) {
              const float w2 = q4k_value(kushr(qb, 4) & 0x0F, scale, min);
              const float x2 = get_float(b, col, k2, st); if (*st) return 0;
              const float p2 = w2 * x2;
              sum = sum + p2;
            }
          }
        }
      }
    } else {
      for (int64_t k = bs; k < be; k++) {
        const int64_t flat = row * K + k, blk = flat / LK_QK_K;
        const int32_t item = (int32_t)(flat % LK_QK_K);
        const float d = q4k_d(a, blk, 0, st); if (*st) return 0;
        const float dmin = q4k_d(a, blk, 2, st); if (*st) return 0;
        const int sb = item / 32;
        const uint64_t bo = a->data_offset + (uint64_t)blk * LK_Q4_K_BLOCK_BYTES;
        const int sc = raw_byte(a, bo + 4 + (uint64_t)sb, st); if (*st) return 0;
        const float scale = ((float)(sc & 0x3F) / 63.0f) * d;
        const int qb = raw_byte(a, bo + 4 + LK_K_SCALE_SIZE + (uint64_t)sb * 16 + (uint64_t)((item % 32) / 2), st); if (*st) return 0;
        const int32_t q = ((item % 32) % 2 == 0) ? (qb & 0x0F) : (kushr(qb, 4) & 0x0F);
        const float w = q4k_value(q, scale, dmin);
        const float x = get_float(b, col, k, st); if (*st) return 0;
        const float p = w * x;
        sum = sum + p;
      }
    }
  }
  return sum;
}

/* computeDotProductQ8_KF32 — :385-432 */
static float dot_q8k_f32(const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, int *st) {
  float sum = 0.0f;
  for (int64_t bs = 0; bs < K; bs += LK_QK_K) {
    const int64_t be = bs + LK_QK_K < K ? bs + LK_QK_K : K;
    if (be - bs == LK_QK_K) {
      const int64_t blk = (row * K + bs) / LK_QK_K;
      const float d = q8k_d(a, blk, st); if (*st) return 0;
      for (int i = 0; i < LK_QK_K; i++) {
        const int32_t q = q8k_weight(a, blk, i, st); if (*st) return 0;
        const float w = (float)q * d;
        const float x = get_float(b, col, bs + i, st); if (*st) return 0;
        const float p = w * x;
        sum = sum + p;
      }
    } else {
      for (int64_t k = bs; k < be; k++) {
        const int64_t flat = row * K + k, blk = flat / LK_QK_K;
        const int32_t item = (int32_t)(flat % LK_QK_K);
        const float d = q8k_d(a, blk, st); if (*st) return 0;
        const int32_t q = q8k_weight(a, blk, item, st); if (*st) return 0;
        const float w = (float)q * d;
        const float x = get_float(b, col, k, st); if (*st) return 0;
        const float p = w * x;
        sum = sum + p;
      }
    }
  }
  return sum;
}

/* Error replay of dequantizeTensor(t) (:918-964) for the dead fallbacks: it
 * reads every element through the accessors, so its errors surface first. */
static int dequant_errors(const lk_tensor *t) {
  int st = LK_OK;
  if (t->type == LK_TYPE_F16) {
    /* applyNDIter over a 2-D view is what computeMatMul's operands are. */
    for (int64_t i1 = 0; i1 < (t->ne[1] > 0 ? t->ne[1] : 1) && !st; i1++)
      for (int64_t i0 = 0; i0 < t->ne[0] && !st; i0++) (void)get_half(t, i0, i1, &st);
    return st;
  }
  if (t->type == LK_TYPE_Q4_0 || t->type == LK_TYPE_Q4_1 || t->type == LK_TYPE_Q8_0) {
    int64_t nb = t_num_blocks(t);
    for (int64_t blk = 0; blk < nb && !st; blk++) (void)q_scale(t, t->type, blk, &st);
    return st;
  }
  return LK_OK; /* other types: warning + zero array, no reads */
}

/* computeMatMul — core/GGMLComputeOps.kt:1435-1565 */
int lko_compute_mat_mul(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst) {
  int st = LK_OK;
  int64_t M = a->ne[1], K_a = a->ne[0], N = b->ne[0], K_b = b->ne[1];
  if (K_a != K_b) return fail(LK_ERR_INVALID_ARG, "Dim mismatch K: a.ne[0](%lld) != b.ne[1](%lld)", (long long)K_a, (long long)K_b); /* :1440 */
  int64_t K = K_a;
  if (dst->ne[0] != N || dst->ne[1] != M) /* :1444-1446 */
    return fail(LK_ERR_INVALID_ARG, "Result tensor dimensions must match expected output size: expected [%lld, %lld], got [%lld, %lld]",
                (long long)N, (long long)M, (long long)dst->ne[0], (long long)dst->ne[1]);

  if (b->type == LK_TYPE_F32 && (a->type == LK_TYPE_Q4_0 || a->type == LK_TYPE_Q4_1 || a->type == LK_TYPE_Q8_0)) {
    /* :1448-1461 (Q4_0), :1462-1480 (Q4_1), :1516-1527 (Q8_0) */
    if (dst->type != LK_TYPE_F32) return fail(LK_ERR_INVALID_ARG, "Result tensor type must be F32 for quantized x F32 matmul");
    for (int64_t i = 0; i < M; i++) {
      for (int64_t j = 0; j < N; j++) {
        float r;
        if (a->type == LK_TYPE_Q4_0) r = dot_q40_f32(a, b, i, j, K, &st);
        else if (a->type == LK_TYPE_Q4_1) r = dot_q41_f32(a, b, i, j, K, &st);
        else r = dot_q80_f32(a, b, i, j, K, &st);
        if (st) return st;
        set_float(dst, r, j, i, &st);
        if (st) return st;
      }
    }
    return LK_OK;
  }
  if (b->type == LK_TYPE_F32 && (a->type == LK_TYPE_Q2_K || a->type == LK_TYPE_Q4_K || a->type == LK_TYPE_Q8_K)) {
    /* :1483-1514 */
    if (dst->type != LK_TYPE_F32) return fail(LK_ERR_INVALID_ARG, "Result tensor type must be F32 for K-quant x F32 matmul");
    for (int64_t i = 0; i < M; i++) {
      for (int64_t j = 0; j < N; j++) {
        float r;
        if (a->type == LK_TYPE_Q2_K) r = dot_q2k_f32(a, b, i, j, K, &st);
        else if (a->type == LK_TYPE_Q4_K) r = dot_q4k_f32(a, b, i, j, K, &st);
        else r = dot_q8k_f32(a, b, i, j, K, &st);
        if (st) return st;
        set_float(dst, r, j, i, &st);
        if (st) return st;
      }
    }
    return LK_OK;
  }
  /* general fallback :1530-1564 */
  if (dst->type != a->type) return fail(LK_ERR_INVALID_ARG, "Result tensor type must match first input type for general matmul");
  switch (a->type) {
    case LK_TYPE_F32: {
      if (b->type != LK_TYPE_F32) {
        /* effB = dequantizeTensor(b): a detached FloatArray with bufferId -1, so the first
         * effB.getFloat throws IndexOutOfBoundsException (buffers[-1]); SURVEY §8a A12. */
        if ((st = dequant_errors(b))) return st;
        for (int64_t i = 0; i < M; i++)
          for (int64_t j = 0; j < N; j++)
            for (int64_t l = 0; l < K; l++) {
              (void)get_float(a, l, i, &st);
              if (st) return st;
              return fail(LK_ERR_OUT_OF_BOUNDS, "Index -1 out of bounds (dequantized operand has no buffer)");
            }
        for (int64_t i = 0; i < M; i++)
          for (int64_t j = 0; j < N; j++) { set_float(dst, 0.0f, j, i, &st); if (st) return st; }
        return LK_OK;
      }
      for (int64_t i = 0; i < M; i++) /* :1536-1542 */
        for (int64_t j = 0; j < N; j++) {
          float sum = 0.0f;
          for (int64_t l = 0; l < K; l++) {
            float x = get_float(a, l, i, &st); if (st) return st;
            float y = get_float(b, j, l, &st); if (st) return st;
            float p = x * y;
            sum = sum + p;
          }
          set_float(dst, sum, j, i, &st);
          if (st) return st;
        }
      return LK_OK;
    }
    case LK_TYPE_F16: { /* :1544-1556 */
      if (b->type != LK_TYPE_F16) {
        if (b->type != LK_TYPE_F32 && (st = dequant_errors(b))) return st;
        if (b->type == LK_TYPE_F32) { /* dequantizeTensor(F32) reads b */
          for (int64_t i1 = 0; i1 < (b->ne[1] > 0 ? b->ne[1] : 1) && !st; i1++)
            for (int64_t i0 = 0; i0 < b->ne[0] && !st; i0++) (void)get_float(b, i0, i1, &st);
          if (st) return st;
        }
        return fail(LK_ERR_NOT_IMPLEMENTED, "F16xnon-F16 matmul to F16 not implemented");
      }
      for (int64_t i = 0; i < M; i++)
        for (int64_t j = 0; j < N; j++) {
          float sum = 0.0f;
          for (int64_t l = 0; l < K; l++) {
            float x = get_half(a, l, i, &st); if (st) return st;
            float y = get_half(b, j, l, &st); if (st) return st;
            float p = x * y;
            sum = sum + p;
          }
          set_half(dst, sum, j, i, &st);
          if (st) return st;
        }
      return LK_OK;
    }
    case LK_TYPE_Q4_0: case LK_TYPE_Q4_1: case LK_TYPE_Q5_0: case LK_TYPE_Q5_1: case LK_TYPE_Q8_0:
    case LK_TYPE_Q8_1: case LK_TYPE_Q2_K: case LK_TYPE_Q3_K: case LK_TYPE_Q4_K: case LK_TYPE_Q5_K:
    case LK_TYPE_Q6_K: case LK_TYPE_Q8_K: case LK_TYPE_BITNET_1_58: {
      /* :1557-1562 dequantize both, recurse on detached F32 copies -> buffers[-1] IOOBE.
       * Restated up to that failure; the empty-shape re-quantize tail is not restated. */
      if ((st = dequant_errors(a))) return st;
      if ((st = dequant_errors(b))) return st;
      if (M > 0 && N > 0 && K > 0) return fail(LK_ERR_OUT_OF_BOUNDS, "Index -1 out of bounds (dequantized operand has no buffer)");
      return LK_OK;
    }
    default:
      return fail(LK_ERR_NOT_IMPLEMENTED, "computeMatMul not implemented for input type %d", a->type);
  }
}

/* "tight" CPU baseline: identical arithmetic order to the structural path for
 * Q4_0/Q4_1/Q8_0 x F32 with contiguous B/dst and K % 32 == 0, without the
 * per-element accessor overhead. Results are bit-identical to lko_compute_mat_mul. */
/* rows [i0, i1) of the tight path: the dot expressions of :43-145 without the accessors */
static void tight_rows(int32_t type, int bb, const uint8_t *A, const float *B, float *D, int64_t K, int64_t N, int64_t i0, int64_t i1) {
  int64_t nbk = K / 32;
  for (int64_t i = i0; i < i1; i++) {
    const uint8_t *row = A + i * nbk * bb;
    for (int64_t j = 0; j < N; j++) {
      float sum = 0.0f;
      for (int64_t blk = 0; blk < nbk; blk++) {
        const uint8_t *p = row + blk * bb;
        float d = lko_half_to_float(rd_u16(p));
        if (type == LK_TYPE_Q4_0) {
          for (int k = 0; k < 32; k++) {
            int q = (k & 1) ? (p[2 + k / 2] >> 4) : (p[2 + k / 2] & 0x0F);
            float qm = (float)q - 8.0f;
            float w = d * qm;
            float p2 = w * B[(blk * 32 + k) * N + j];
            sum = sum + p2;
          }
        } else if (type == LK_TYPE_Q4_1) {
          float m = lko_half_to_float(rd_u16(p + 2));
          for (int k = 0; k < 32; k++) {
            int q = (k & 1) ? (p[4 + k / 2] >> 4) : (p[4 + k / 2] & 0x0F);
            float dq = d * (float)q;
            float w = dq + m;
            float p2 = w * B[(blk * 32 + k) * N + j];
            sum = sum + p2;
          }
        } else {
          for (int k = 0; k < 32; k++) {
            float w = d * (float)(int8_t)p[2 + k];
            float p2 = w * B[(blk * 32 + k) * N + j];
            sum = sum + p2;
          }
        }
      }
      D[i * N + j] = sum;
    }
  }
}

int lko_compute_mat_mul_tight_mt(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int threads) {
  int64_t M = a->ne[1], K = a->ne[0], N = b->ne[0];
  if (K != b->ne[1] || dst->ne[0] != N || dst->ne[1] != M) return fail(LK_ERR_INVALID_ARG, "shape mismatch");
  if (K % 32 || b->type != LK_TYPE_F32 || dst->type != LK_TYPE_F32) return fail(LK_ERR_NOT_IMPLEMENTED, "tight path: unsupported");
  if (b->nb[0] != 4 || b->nb[1] != 4 * (uint64_t)N || dst->nb[0] != 4 || dst->nb[1] != 4 * (uint64_t)N)
    return fail(LK_ERR_NOT_IMPLEMENTED, "tight path: non-contiguous");
  int bb = lko_block_bytes(a->type);
  if (!bb) return fail(LK_ERR_NOT_IMPLEMENTED, "tight path: type");
  const uint8_t *A = (const uint8_t *)a->data + a->data_offset;
  const float *B = (const float *)((const uint8_t *)b->data + b->data_offset);
  float *D = (float *)((uint8_t *)dst->data + dst->data_offset);
  if (threads <= 1) {
    tight_rows(a->type, bb, A, B, D, K, N, 0, M);
    return LK_OK;
  }
  /* rows are independent (each dot keeps its own k order): the parallel split is bit-identical */
  const int64_t chunk = 16;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (int64_t c = 0; c < (M + chunk - 1) / chunk; c++) {
    int64_t i0 = c * chunk, i1 = i0 + chunk < M ? i0 + chunk : M;
    tight_rows(a->type, bb, A, B, D, K, N, i0, i1);
  }
  return LK_OK;
}

int lko_compute_mat_mul_tight(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst) {
  return lko_compute_mat_mul_tight_mt(a, b, dst, 1);
}

/* ---- direct dot products (core/GGMLComputeOps.kt:349-629) --------------------------------
 * Unreachable from computeMatMul in the reference; restated for the lk_dot_direct offload.
 * A: M x K (ne[0] = K), Q elements at the flat index row*K + k, F32 through getFloat(k, row).
 * B: K x N (ne[0] = N, ne[1] = K), flat index k*N + col. Each function first runs its
 * require()s (types, A.ne[0] == K, B.ne[1] == K), then the accessors in the Kotlin order. */

/* one Q element of t at flat index `flat`: Q8_0 -> d*q; Q4_0 -> d*(n - 8); Q4_1 -> d*n + m
 * (the expressions of :366-367, :461-462, :498-505, :539-541, :579-581, :620-621) */
static float q_elem(const lk_tensor *t, int64_t flat, int *st) {
  int64_t blk = flat / 32;
  int32_t item = (int32_t)(flat % 32);
  float d = q_scale(t, t->type, blk, st); if (*st) return 0;
  if (t->type == LK_TYPE_Q8_0) {
    int32_t q = q8_weight(t, blk, item, st); if (*st) return 0;
    return d * (float)q;
  }
  if (t->type == LK_TYPE_Q4_1) {
    float m = q41_min(t, blk, st); if (*st) return 0;
    int32_t q = q4_nibble(t, LK_TYPE_Q4_1, blk, item, st); if (*st) return 0;
    float dq = d * (float)q;
    return dq + m;
  }
  int32_t q = q4_nibble(t, LK_TYPE_Q4_0, blk, item, st); if (*st) return 0;
  float qm = (float)q - 8.0f;
  return d * qm;
}

static int dot_kind_types(int32_t kind, int32_t *ta, int32_t *tb) {
  switch (kind) {
    case LK_DOT_F32_Q4_1: *ta = LK_TYPE_F32; *tb = LK_TYPE_Q4_1; return 1;
    case LK_DOT_F32_Q8_0: *ta = LK_TYPE_F32; *tb = LK_TYPE_Q8_0; return 1;
    case LK_DOT_Q8_0_Q8_0: *ta = LK_TYPE_Q8_0; *tb = LK_TYPE_Q8_0; return 1;
    case LK_DOT_Q4_0_Q4_0: *ta = LK_TYPE_Q4_0; *tb = LK_TYPE_Q4_0; return 1;
    case LK_DOT_Q4_1_Q4_1: *ta = LK_TYPE_Q4_1; *tb = LK_TYPE_Q4_1; return 1;
    case LK_DOT_Q8_0_Q4_0: *ta = LK_TYPE_Q8_0; *tb = LK_TYPE_Q4_0; return 1;
    default: return 0;
  }
}

int lko_dot_direct(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t row, int64_t col, int64_t K, float *out) {
  int32_t ta, tb;
  if (!dot_kind_types(kind, &ta, &tb)) return fail(LK_ERR_NOT_IMPLEMENTED, "direct dot kind %d", kind);
  if (a->type != ta) return fail(LK_ERR_INVALID_ARG, "tensorA must be type %d. Got %d", ta, a->type);
  if (b->type != tb) return fail(LK_ERR_INVALID_ARG, "tensorB must be type %d. Got %d", tb, b->type);
  if (a->ne[0] != K) return fail(LK_ERR_INVALID_ARG, "tensorA K dim (%lld) must match commonDimK (%lld)", (long long)a->ne[0], (long long)K);
  if (b->ne[1] != K) return fail(LK_ERR_INVALID_ARG, "tensorB K dim (%lld) must match commonDimK (%lld)", (long long)b->ne[1], (long long)K);
  const int64_t N = b->ne[0];
  int st = LK_OK;
  float sum = 0.0f;
  for (int64_t k = 0; k < K; k++) {
    const int64_t flat_b = k * N + col;
    float p;
    switch (kind) {
      case LK_DOT_F32_Q4_1:   /* :364-375 */
      case LK_DOT_F32_Q8_0: { /* :457-466 */
        float f = get_float(a, k, row, &st); if (st) return st;
        float w = q_elem(b, flat_b, &st); if (st) return st;
        p = f * w;
        break;
      }
      case LK_DOT_Q8_0_Q8_0: { /* :488-505: scaleA * scaleB * (qA * qB) */
        int64_t fa = row * K + k;
        float sa = q_scale(a, LK_TYPE_Q8_0, fa / 32, &st); if (st) return st;
        int32_t qa = q8_weight(a, fa / 32, (int32_t)(fa % 32), &st); if (st) return st;
        float sb = q_scale(b, LK_TYPE_Q8_0, flat_b / 32, &st); if (st) return st;
        int32_t qb = q8_weight(b, flat_b / 32, (int32_t)(flat_b % 32), &st); if (st) return st;
        float s2 = sa * sb;
        float q2 = (float)qa * (float)qb;
        p = s2 * q2;
        break;
      }
      default: { /* Q40Q40 :526-546, Q41Q41 :566-587, Q80Q40 :608-627: dequantA * dequantB */
        float wa = q_elem(a, row * K + k, &st); if (st) return st;
        float wb = q_elem(b, flat_b, &st); if (st) return st;
        p = wa * wb;
        break;
      }
    }
    sum = sum + p;
  }
  *out = sum;
  return LK_OK;
}

int lko_dot_direct_matrix(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out) {
  const int64_t M = a->ne[1], N = b->ne[0];
  for (int64_t i = 0; i < M; i++)
    for (int64_t j = 0; j < N; j++) {
      int st = lko_dot_direct(kind, a, b, i, j, K, out + i * N + j);
      if (st) return st;
    }
  if (M == 0 || N == 0) {  /* the requires still run once a caller would have called the function */
    int32_t ta, tb;
    if (!dot_kind_types(kind, &ta, &tb)) return fail(LK_ERR_NOT_IMPLEMENTED, "direct dot kind %d", kind);
  }
  return LK_OK;
}
