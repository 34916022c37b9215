/*
 * lk_gguf.h — GGUF quantized-tensor loading into llama.kotlin's block layout
 * (SURVEY.md §8f, row "next" #1). Part of liblk_hip.so; same status codes as
 * lk_hip.h.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * src/nativeMain/kotlin/ai/solace/llamakotlin/):
 *
 *   lk_gguf_open_memory   gguf/GGUFParser.kt:13-56   GGUFParser(data).parse()
 *   lk_gguf_open_file     gguf/ModelLoader.kt:13-15  loadFromFile (a stub in the reference;
 *                         here the file is memory-mapped, never read whole)
 *   lk_gguf_version, _alignment, _data_offset
 *                         gguf/GGUFContext.kt:6-13   GGUFContext fields
 *   lk_gguf_kv_*          gguf/GGUFParser.kt:58-126  readKeyValue / readArray, and the
 *                         GGUFContext.kt:17-73 typed getters built on them
 *   lk_gguf_get_tensor_info, lk_gguf_find_tensor
 *                         gguf/GGUFParser.kt:86-100  readTensorInfo; GGUFContext.kt:78-80
 *   lk_gguf_tensor_data   gguf/GGUFContext.kt:85-103 getTensorData (file bytes, as stored)
 *   lk_gguf_load_tensor   gguf/ModelLoader.kt:78-96  loadTensorData, which in the reference
 *                         loads F32 only; here every block type the MUL_MAT path computes
 *                         lands in llama.kotlin's layout (see "Layout" below)
 *   lk_gguf_load_all_device  graph residency: the whole data section in one HBM buffer,
 *                         every tensor at dev_base + its GGUF offset
 *   lk_repack_q4_device   the nibble-order conversion itself (device kernel)
 *
 * Type ids. GGUF files written by llama.cpp/ggml carry upstream ggml_type ids
 * (Q8_0 = 8). The reference parser feeds them to GGMLType.fromValue
 * (GGUFParser.kt:93-95), whose ids differ (core/GGMLTypes.kt:145-168: 8 is Q2_K),
 * so it misreads every upstream file past Q4_1. LK_GGUF_UPSTREAM_IDS (default)
 * decodes the file's ids as upstream ggml_type and maps them to lk_type;
 * LK_GGUF_KOTLIN_IDS reproduces the reference's fromValue reading, for files
 * written with llama.kotlin ids.
 *
 * Layout. Upstream Q4_0/Q4_1 blocks store weight j in the low nibble and weight
 * j+16 in the high nibble of byte j (ggml/src/ggml-quants.c:1515-1553).
 * llama.kotlin stores weight 2j low and 2j+1 high (core/GGMLTypes.kt:647-651).
 * Loading an upstream-id Q4_0/Q4_1 tensor therefore repacks the nibbles on the
 * GPU (lk_gguf_tensor_info.repack = 1). Scales, mins and Q8_0 blocks are
 * byte-identical in both layouts. Every other type is copied as stored.
 */
#ifndef LK_GGUF_H
#define LK_GGUF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lk_gguf lk_gguf;

/* open flags */
#define LK_GGUF_UPSTREAM_IDS 0 /* tensor type ids are upstream ggml_type (llama.cpp files) */
#define LK_GGUF_KOTLIN_IDS 1   /* tensor type ids are GGMLType.fromValue ids (reference reading) */

/* GGUF value types (gguf/GGUFTypes.kt:6-20) */
enum lk_gguf_type {
  LK_GGUF_UINT8 = 0, LK_GGUF_INT8 = 1, LK_GGUF_UINT16 = 2, LK_GGUF_INT16 = 3,
  LK_GGUF_UINT32 = 4, LK_GGUF_INT32 = 5, LK_GGUF_FLOAT32 = 6, LK_GGUF_BOOL = 7,
  LK_GGUF_STRING = 8, LK_GGUF_ARRAY = 9, LK_GGUF_UINT64 = 10, LK_GGUF_INT64 = 11,
  LK_GGUF_FLOAT64 = 12
};

/* lk_repack_q4_device directions */
#define LK_REPACK_UPSTREAM_TO_KOTLIN 0
#define LK_REPACK_KOTLIN_TO_UPSTREAM 1

/* GGUFTensorInfo (gguf/GGUFTypes.kt:33-54) plus what loading needs. */
typedef struct lk_gguf_tensor_info {
  const char *name;   /* NUL-terminated, owned by the handle */
  int32_t n_dims;     /* 1..4 */
  int32_t file_type;  /* type id as stored in the file */
  int32_t type;       /* lk_type (GGMLType.fromValue id), -1 if llama.kotlin has none */
  int32_t repack;     /* 1: loading converts upstream nibble order to llama.kotlin's */
  int64_t ne[4];      /* dimensions, ne[0] fastest; unused dims are 1 */
  uint64_t offset;    /* GGUFTensorInfo.offset: relative to the data section */
  uint64_t bytes;     /* stored size: nelements / block * block bytes */
} lk_gguf_tensor_info;

/* Parse a GGUF image held by the caller (borrowed: it must outlive the handle).
 * Bad magic, an unknown value or tensor type, nested arrays, n_dims > 4 or
 * version < 2 -> LK_ERR_INVALID_ARG (IllegalArgumentException, GGUFParser.kt:22-23,
 * :94-95, :123); truncated data -> LK_ERR_OUT_OF_BOUNDS (IndexOutOfBoundsException,
 * GGUFParser.kt:129, :191-193). */
int lk_gguf_open_memory(const void *data, uint64_t bytes, int32_t flags, lk_gguf **out);
/* Memory-map a file read-only and parse it; the handle owns the mapping. */
int lk_gguf_open_file(const char *path, int32_t flags, lk_gguf **out);
void lk_gguf_close(lk_gguf *g);

uint32_t lk_gguf_version(const lk_gguf *g);
uint64_t lk_gguf_alignment(const lk_gguf *g);   /* general.alignment, default 32 */
uint64_t lk_gguf_data_offset(const lk_gguf *g); /* aligned start of the data section */
uint64_t lk_gguf_data_bytes(const lk_gguf *g);  /* max(offset + bytes) over tensors */

/* metadata */
int64_t lk_gguf_kv_count(const lk_gguf *g);
int64_t lk_gguf_find_key(const lk_gguf *g, const char *key); /* -1 if absent */
const char *lk_gguf_kv_key(const lk_gguf *g, int64_t i);    /* NULL if out of range */
int32_t lk_gguf_kv_type(const lk_gguf *g, int64_t i);       /* lk_gguf_type, -1 if out of range */
/* ARRAY values: element type and length. */
int lk_gguf_kv_array_info(const lk_gguf *g, int64_t i, int32_t *elem_type, uint64_t *n);
/* A numeric/bool value (elem = -1 for a scalar, else an array element), written
 * to out in its natural little-endian width (1, 2, 4 or 8 bytes). */
int lk_gguf_kv_get(const lk_gguf *g, int64_t i, int64_t elem, void *out, uint64_t out_bytes);
/* Raw little-endian elements of a numeric array, in place in the GGUF image. */
int lk_gguf_kv_array_data(const lk_gguf *g, int64_t i, const void **data, uint64_t *elem_bytes);
/* A STRING value (elem = -1) or a string array element; not NUL-terminated. */
int lk_gguf_kv_get_string(const lk_gguf *g, int64_t i, int64_t elem, const char **s, uint64_t *len);

/* tensors */
int64_t lk_gguf_tensor_count(const lk_gguf *g);
int64_t lk_gguf_find_tensor(const lk_gguf *g, const char *name); /* -1 if absent */
int lk_gguf_get_tensor_info(const lk_gguf *g, int64_t i, lk_gguf_tensor_info *out);
/* The stored bytes (file layout), bounds-checked against the image. */
int lk_gguf_tensor_data(const lk_gguf *g, int64_t i, const void **data, uint64_t *bytes);
/* Tensor i into dst in llama.kotlin's layout. dst_on_device = 1: dst is device
 * memory, the copy and repack are enqueued on stream (NULL = the null stream)
 * and complete before return. dst_on_device = 0: host memory; a tensor that
 * needs a repack is staged through the GPU. dst_bytes < info.bytes ->
 * LK_ERR_INVALID_ARG; a type llama.kotlin has no id for -> LK_ERR_NOT_IMPLEMENTED. */
int lk_gguf_load_tensor(const lk_gguf *g, int64_t i, void *dst, uint64_t dst_bytes,
                        int32_t dst_on_device, void *stream);
/* The whole data section into one device buffer (dev_bytes >= lk_gguf_data_bytes),
 * streamed through pinned staging, then every tensor with repack = 1 repacked in
 * place. Tensor i is at dev_base + info.offset afterwards. */
int lk_gguf_load_all_device(const lk_gguf *g, void *dev_base, uint64_t dev_bytes, void *stream);

/* In-place nibble-order conversion of n_blocks contiguous Q4_0 or Q4_1 blocks
 * (type = LK_TYPE_Q4_0 / LK_TYPE_Q4_1) in device memory. Bit-exact inverse pair. */
int lk_repack_q4_device(void *blocks, int64_t n_blocks, int32_t type, int32_t direction,
                        void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LK_GGUF_H */
