/*
 * lk_hip.h — C-ABI of the MI355X (gfx950) backend for llama.kotlin's quantized
 * MUL_MAT hot path.
 *
 * This is the drop-in boundary. Everything above it (the Kotlin/Native cinterop
 * shim in llama.kotlin_amd/shim/, or the Python host mirror in
 * llama.kotlin_amd/ggml_hip/) passes plain pointers and sizes; nothing below it
 * is visible to the caller. No torch, HIP or C++ types cross this header.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * src/nativeMain/kotlin/ai/solace/llamakotlin/ in SolaceHarmony/llama.kotlin):
 *
 *   lk_mul_mat            core/GGMLComputeOps.kt:1435  fun computeMatMul(graphAllocator,
 *                         context, a, b, dst)  — destination-tensor semantics: dst is
 *                         pre-allocated, results land in graphAllocator.buffers[dst.bufferId]
 *                         at dst.dataOffset, nothing is returned, inputs are not mutated.
 *   lk_mul_mat_validate   core/GGMLComputeOps.kt:1436-1446, :1449, :1463, :1517, :1530,
 *                         :1546, :1563 — the checks computeMatMul performs, in its order,
 *                         without computing anything.
 *   lk_mul_mat_device     the same operator over device-resident buffers, enqueued on a
 *                         HIP stream (what GGMLBackend.graphCompute uses once operands
 *                         are resident; core/GGMLBackend.kt:146).
 *   lk_plan_*             core/GGMLBackend.kt:146 graphCompute(graph) over a graph whose
 *                         MUL_MAT nodes are mutually independent: one launch for the set;
 *                         lk_plan_create_chain: a sequence of dependent stages of such nodes
 *                         (computeGraph's node order, core/GGMLComputeOps.kt:2515) in one launch.
 *   lk_comm_* / lk_sharded_plan_*  the north star's row sharding over the GPUs of a node with
 *                         an RCCL all-gather over xGMI (the reference is single-device).
 *   lk_mul_mat_sharded    SURVEY §8b's sharded entry: computeMatMul with A's rows split
 *                         over the GPUs of one node from one host thread (the reference
 *                         is single-device; this is the north star's row sharding).
 *   lk_graph_*            core/GGMLComputeOps.kt:2515-2652 computeGraph/computeMulMat over
 *                         host buffers with activations kept in HBM between nodes.
 *   lk_weights_pin/evict  residency cache behind GGMLBackendBuffer.setTensor
 *                         (core/GGMLBackend.kt:63-69) for host-authoritative ByteArrays.
 *   lk_dequantize_device  core/GGMLComputeOps.kt:918 dequantizeTensor (Q8_0/Q4_0/Q4_1).
 *   lk_quantize_device    core/GGMLComputeOps.kt:1040 quantizeTensor (Q8_0/Q4_0/Q4_1).
 *   lk_dot_direct*        core/GGMLComputeOps.kt:349-629 the direct dot products
 *                         computeDotProduct{F32Q41, F32Q80, Q80Q80, Q40Q40, Q41Q41, Q80Q40}
 *                         (graphAllocator, tensorA, tensorB, row, col, commonDimK): Float,
 *                         evaluated for every (row, col) of A's rows x B's columns.
 *
 * Status codes map back to the exceptions the Kotlin operator throws
 * (see INTEGRATION.md for the cinterop mapping):
 *   LK_OK                   0  — success
 *   LK_ERR_INVALID_ARG      1  — IllegalArgumentException (shape/type checks, require())
 *   LK_ERR_NOT_IMPLEMENTED  2  — NotImplementedError, or "not offloaded: use the CPU path"
 *   LK_ERR_OUT_OF_BOUNDS    3  — IndexOutOfBoundsException (accessor buffer bounds)
 *   LK_ERR_NO_BUFFER        4  — IllegalStateException ("Tensor buffer not found")
 *   LK_ERR_DEVICE           5  — HIP runtime failure (GGMLStatus.FAILED at backend level)
 */
#ifndef LK_HIP_H
#define LK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Type ids follow GGMLType.fromValue (core/GGMLTypes.kt:145-168). These are NOT
 * upstream ggml/GGUF ids (Q8_0 is 6 here, 8 upstream). */
enum lk_type {
  LK_TYPE_F32 = 0,
  LK_TYPE_F16 = 1,
  LK_TYPE_Q4_0 = 2,
  LK_TYPE_Q4_1 = 3,
  LK_TYPE_Q5_0 = 4,
  LK_TYPE_Q5_1 = 5,
  LK_TYPE_Q8_0 = 6,
  LK_TYPE_Q8_1 = 7,
  LK_TYPE_Q2_K = 8,
  LK_TYPE_Q3_K = 9,
  LK_TYPE_Q4_K = 10,
  LK_TYPE_Q5_K = 11,
  LK_TYPE_Q6_K = 12,
  LK_TYPE_Q8_K = 13,
  LK_TYPE_Q1_5_K = 14,
  LK_TYPE_I8 = 15,
  LK_TYPE_I16 = 16,
  LK_TYPE_I32 = 17,
  LK_TYPE_I64 = 18,
  LK_TYPE_BITNET_1_58 = 19 /* not in fromValue; GGMLType.BITNET_1_58 */
};

enum lk_status {
  LK_OK = 0,
  LK_ERR_INVALID_ARG = 1,
  LK_ERR_NOT_IMPLEMENTED = 2,
  LK_ERR_OUT_OF_BOUNDS = 3,
  LK_ERR_NO_BUFFER = 4,
  LK_ERR_DEVICE = 5
};

/* Block geometry (core/GGMLTypes.kt:84-86, :108-114): 32 weights per block.
 *   Q4_0: f16 d | 16 B nibbles                         = 18 B
 *   Q4_1: f16 d | f16 m | 16 B nibbles                 = 20 B
 *   Q8_0: f16 d | 32 x int8                            = 34 B
 * Nibble order is llama.kotlin's interleaved order: weight 2j is the low nibble
 * of byte j, weight 2j+1 the high nibble (core/GGMLTypes.kt:647-651). */
#define LK_QK 32
#define LK_Q4_0_BLOCK_BYTES 18
#define LK_Q4_1_BLOCK_BYTES 20
#define LK_Q8_0_BLOCK_BYTES 34
/* K-quants: 256-weight super-blocks (core/GGMLTypes.kt:92-93, :117-122, accessors :734-916).
 *   Q2_K: scales[16] | qs[64] (2-bit, 4 per byte, low bits first) | f16 d | f16 dmin = 84 B
 *   Q4_K: f16 d | f16 dmin | scales[12] | qs[128] (low nibble first)       = 144 B
 *   Q8_K: f32 d | 256 x int8 | 16 x int16 bsums                            = 292 B */
#define LK_QK_K 256
#define LK_K_SCALE_SIZE 12
#define LK_Q2_K_BLOCK_BYTES 84
#define LK_Q4_K_BLOCK_BYTES 144
#define LK_Q8_K_BLOCK_BYTES 292

/* A GGMLTensor descriptor (core/GGMLTypes.kt:251-270) as the operator sees it.
 *  - ne/nb: GGMLTensor.ne / GGMLTensor.nb (nb in bytes). Quantized tensors ignore nb,
 *    exactly like the reference block accessors (core/GGMLTypes.kt:598-732).
 *  - data: base address of graphAllocator.buffers[bufferId] (host ByteArray for
 *    lk_mul_mat, device allocation for *_device). NULL = missing buffer.
 *  - buf_bytes: size of that buffer; every access is bounds-checked against it
 *    as the Kotlin accessors do (core/GGMLTypes.kt:360-369).
 *  - data_offset: GGMLTensor.dataOffset. */
typedef struct lk_tensor {
  int32_t type;
  int32_t reserved;
  int64_t ne[4];
  uint64_t nb[4];
  void *data;
  uint64_t buf_bytes;
  uint64_t data_offset;
} lk_tensor;

/* ---- runtime ---------------------------------------------------------- */

/* Select HIP device `device` for this thread and create the library's stream.
 * Idempotent per device. Returns LK_OK or LK_ERR_DEVICE. */
int lk_init(int device);
/* Number of visible HIP devices (0 when none; never initialises a context). */
int lk_device_count(void);
/* Human-readable message for the last non-OK status on this thread. */
const char *lk_last_error(void);
/* Release the weight cache, plans and the stream. */
void lk_shutdown(void);
/* Library version string. */
const char *lk_version(void);

/* ---- operator ----------------------------------------------------------- */

/* computeMatMul's validation only (same order, same exceptions). No device work. */
int lk_mul_mat_validate(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst);

/* computeMatMul over HOST buffers (the Kotlin drop-in): weights are copied to a
 * device mirror (cached when pinned with lk_weights_pin), activations uploaded,
 * the kernel runs, dst bytes are written back into dst->data before return. */
int lk_mul_mat(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst);

/* computeMatMul over DEVICE buffers, enqueued on `stream` (hipStream_t; NULL =
 * the HIP null stream of the current device). Asynchronous: returns after the
 * launch; no allocation, no host synchronisation (graph-capturable). */
int lk_mul_mat_device(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, void *stream);

/* computeMatMul over HOST buffers with A's rows split into n_shards equal row ranges
 * (ceil(M/n_shards) rows each), shard r computed on device r mod lk_device_count().
 * Each shard writes its own rows of dst back into dst->data (the in-process all-gather);
 * results meet lk_mul_mat's parity bar (bit-identical to it at N = 1, where every row is
 * one wave's sequential sum). Falls back to one device when rows are not byte
 * ranges (quantized A with K % 32 != 0) or dst rows interleave. Synchronous. */
int lk_mul_mat_sharded(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int n_shards);
/* The same with shard r on device (first_device + r) mod lk_device_count() (a backend bound to
 * GPU first_device; lk_mul_mat_sharded is first_device = 0). */
int lk_mul_mat_sharded_at(const lk_tensor *a, const lk_tensor *b, lk_tensor *dst, int n_shards, int first_device);

/* ---- grouped execution of independent MUL_MAT nodes ------------------------ */

typedef struct lk_plan lk_plan;
/* Validate n independent nodes (device buffers) and upload their descriptors once.
 * Batch-1 streaming nodes with the same quant type run as one grouped launch each; since round 6
 * so do Q4_0 / Q4_1 nodes at 17 <= N <= 32 (one pair-kernel launch + one slab-sum launch per type,
 * the same bits as single launches; split-K slabs owned by the plan). */
int lk_plan_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                   lk_plan **out);
/* Enqueue every node of the plan on `stream`. A plan's launches are stream-ordered: one plan must not
 * run on two streams at once (its slabs and, for chain plans, its barrier words are its own). */
int lk_plan_launch(lk_plan *plan, void *stream);
/* Number of kernel launches one lk_plan_launch issues. */
int lk_plan_num_launches(const lk_plan *plan);
/* A chain of DEPENDENT stages in one launch (a persistent streaming GEMV): node i belongs to
 * stage stage[i] (0, then non-decreasing by at most 1). Stage s+1 starts only after every
 * node of stage s has stored its outputs — a device-side grid barrier (write-through outputs,
 * sharded arrival counters, activations re-read past the caches) — so a stage may read what the
 * previous one wrote; the next stage's weights are already streaming while the barrier completes. Same results as launching the stages' plans
 * in order. Every node must be an N = 1 streaming-GEMV node of one quant type
 * (LK_ERR_NOT_IMPLEMENTED otherwise). Launch with lk_plan_launch (graph-capturable). */
int lk_plan_create_chain(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage, int n,
                         lk_plan **out);
/* 1 if a chain launch gave up waiting at a barrier (its grid was not co-resident: results are
 * then undefined) and re-arms the plan; 0 otherwise. Synchronizes the device. */
int lk_plan_chain_timed_out(lk_plan *plan);
void lk_plan_destroy(lk_plan *plan);
/* Batched MUL_MATs (2 <= N) split K over workgroups without any workgroup waiting for another
 * (round 4): two slices add into dst, more store slabs summed by a reduce launch after the GEMM (or,
 * in the wide kernel, by the LAST ARRIVER per output tile inside it), so any grid size and kernels of
 * other streams sharing the GPU are safe. Only chain plans still wait (grid barriers,
 * every workgroup resident: one per CU). Such a wait is bounded (200 ms); one that gives up is
 * counted on the device and moves a per-device failure word: every synchronous entry point
 * (lk_mul_mat, lk_mul_mat_sharded, lk_graph_compute) reads the word before its launches and again
 * after its sync and returns LK_ERR_DEVICE when it moved — those results are undefined
 * (GGMLStatus.FAILED at backend level, core/GGMLCpuBackend.kt:167-176). Stream-ordered entry points
 * (lk_mul_mat_device, lk_plan_launch) cannot report it at launch; a caller of chain plans reads
 * lk_plan_chain_timed_out, or here: *count = how many waits on the current device gave up since
 * the last call (the device count is monotonic). Synchronizes the device. Diagnostic; no reference
 * counterpart. */
int lk_sync_timeouts(uint32_t *count);
/* Test hooks of the same mechanism (current device; synchronize it first):
 * lk_set_sync_wait_bound — the wait bound in 100 MHz ticks (default 20000000 = 200 ms); 0 makes a
 *   waiter that does not find its peers already arrived give up at once (tests of the error path);
 * lk_sync_counters_sum — the sum of every split-K per-tile arrival counter word, 0 between
 *   launches (the last arrival of each tile re-arms its word). */
int lk_set_sync_wait_bound(uint64_t ticks);
int lk_sync_counters_sum(uint64_t *sum);
/* Diagnostic (no reference counterpart): the kernels the calls on this thread launched since the
 * last lk_debug_route_clear, and for lk_mul_mat where A came from ("A=mirror" / "A=staged"), as
 * space-separated words, e.g. "A=mirror gemm_q_mfma<2>:t2s12". Lets a parity test name the route
 * that produced a result. */
const char *lk_debug_route(void);
void lk_debug_route_clear(void);
/* Diagnostic: how many times the batched kernels' device scratch (activation fragments, split-K
 * slabs, tile counters) of the current device was reallocated. Outgrown buffers are retired, never
 * freed before lk_shutdown, so HIP graphs captured earlier stay valid. */
uint64_t lk_debug_scratch_epoch(void);
/* Test hook: store `value` into split-K tile counter `index` of the gemm_q_* fallback GEMMs'
 * scratch for (current device, stream), synchronously. Every split-K launch re-arms the counters
 * it uses on its own stream first, so a poked (or otherwise stale) word never leaves a tile
 * unwritten (round 4's failure mechanism). */
int lk_debug_poke_gemm_counter(void *stream, int64_t index, int32_t value);
/* Scratch lifetime: lk_scratch_release frees the batched kernels' scratch of
 * (current device, stream), retired buffers included, after synchronising that stream; the caller
 * guarantees that no HIP graph it will still replay captured a launch on that stream. lk_scratch_bytes
 * = device bytes that scratch holds on the current device, all streams. */
int lk_scratch_release(void *stream);
uint64_t lk_scratch_bytes(void);

/* ---- multi-GPU: row shards + RCCL all-gather over xGMI -----------------
 * The reference is single-device; this is the north star's partition of the same operator.
 * Rank r of P owns rows [r·M/P, (r+1)·M/P) of every weight matrix (contiguous bytes: rows are
 * whole blocks) and computes those rows of dst in place inside the FULL dst; an in-place
 * ncclAllGather per node fills in the other ranks' rows, so on completion every rank holds
 * every dst whole — the activations the next MUL_MAT reads.
 *
 * One process per GPU: rank 0 calls lk_comm_unique_id, the caller broadcasts the
 * LK_COMM_ID_BYTES bytes, every rank calls lk_comm_init_rank on its current device.
 * One process driving several GPUs (the Kotlin host): lk_comm_init_all fills comms[ndev];
 * launches on different devices go between lk_comm_group_start / lk_comm_group_end. */
#define LK_COMM_ID_BYTES 128
typedef struct lk_comm lk_comm;
int lk_comm_unique_id(void *id);
int lk_comm_init_rank(const void *id, int nranks, int rank, lk_comm **out);
int lk_comm_init_all(int ndev, const int *devices, lk_comm **comms);
int lk_comm_nranks(const lk_comm *comm);
int lk_comm_rank(const lk_comm *comm);
/* The HIP device the communicator's rank runs on. */
int lk_comm_device(const lk_comm *comm);
/* How many ncclAllGather calls were enqueued through the communicator (a HIP-graph replay of
 * captured ones does not count again). */
uint64_t lk_comm_num_collectives(const lk_comm *comm);
void lk_comm_destroy(lk_comm *comm);
/* Tears down the communicator's enqueued collectives (ncclCommAbort), e.g. after a failure left
 * some ranks' all-gathers waiting for peers that never arrive; later collectives through it fail
 * with LK_ERR_DEVICE. The handle still needs lk_comm_destroy. A failure inside an RCCL group
 * aborts the communicators involved itself (a sharded graph then refuses further computes). */
int lk_comm_abort(lk_comm *comm);
int lk_comm_group_start(void);
int lk_comm_group_end(void);

/* n independent MUL_MAT nodes, row-sharded over the communicator (device buffers):
 * a[i] is this rank's row shard (ne[1] = M_i / P), b[i] the full activations, dst[i] the full
 * destination (ne = [N, M_i], dense rows: nb[1] == N · element size, M_i % P == 0).
 * lk_sharded_plan_launch enqueues on `stream`: one grouped launch of the local rows, then one
 * RCCL group of in-place all-gathers. Same bytes in dst as lk_plan_create over the unsharded
 * nodes (each row is computed by the same kernel from the same bytes). */
typedef struct lk_sharded_plan lk_sharded_plan;
int lk_sharded_plan_create(lk_comm *comm, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                           lk_sharded_plan **out);
int lk_sharded_plan_launch(lk_sharded_plan *plan, void *stream);
/* Throughput form: the local rows on `compute`, the node set's RCCL group of in-place all-gathers on
 * `gather` behind an event of the local launch, so independent plans issued back to back overlap one
 * plan's exchange with the next plan's rows (both streams on the communicator's device; capturable when
 * the caller joins `gather` back into the capture's origin stream). */
int lk_sharded_plan_launch_split(lk_sharded_plan *plan, void *compute_stream, void *gather_stream);
int lk_sharded_plan_num_gathers(const lk_sharded_plan *plan);
void lk_sharded_plan_destroy(lk_sharded_plan *plan);
/* lk_sharded_plan_launch always issues its RCCL group, at one rank too (in-place copies), so the
 * one-GPU tests run the code a multi-GPU node runs. */

/* ---- multi-GPU: the one-shot peer-write alternative ----------------
 * Same partition as lk_sharded_plan, without a collective: rank r's push kernel writes its rows of
 * every dst straight into every peer's full dst (xGMI stores, peer access enabled by the group)
 * and adds 1 to the plan's arrival signal on every rank; the next plan launched in the group is
 * gated on each rank by hipStreamWaitValue64(signal >= launches · P) — the command processor holds
 * the queue, no kernel spins. One process drives the P ranks (the Kotlin host's shape).
 *   lk_p2p_group_create: ranks 0..P-1 on devices[r] (P <= 8); devices may repeat (several ranks on
 *     one GPU, each with its own buffers: the one-GPU tests); distinct devices must be peers.
 *   lk_p2p_plan_create: a, b, dst hold P·n tensors, rank-major: a[r·n+i] rank r's rows of node i
 *     (ne[1] = M_i / P), b[r·n+i] rank r's full activations, dst[r·n+i] rank r's full dst (dense
 *     rows, M_i % P == 0), all on rank r's device.
 *   lk_p2p_plan_launch: streams[r] on rank r's device; ranks on one device share one stream. Each
 *     launch waits (per rank) for every rank's rows of the plan launched before it in the group —
 *     plans launched in sequence form a chain of dependent stages, like a model's layers. Eager
 *     only: LK_ERR_NOT_IMPLEMENTED while the stream is capturing (the gate values grow with every
 *     launch; lk_sharded_plan is the graph-replayable path). A launch that fails part-way leaves
 *     the group refusing further launches (LK_ERR_DEVICE).
 *   lk_p2p_plan_signal: synchronizes rank's device, reads its arrival signal (launches · P when
 *     every push arrived). Destroy plans only after the streams are synchronized.
 * Same bytes in every rank's dst as lk_plan over the unsharded nodes. No reference counterpart
 * beyond the archived row split's peer copies (archive/cuda/src/ggml-cuda.cu:521, :645-680). */
typedef struct lk_p2p_group lk_p2p_group;
typedef struct lk_p2p_plan lk_p2p_plan;
int lk_p2p_group_create(int nranks, const int *devices, lk_p2p_group **out);
int lk_p2p_group_nranks(const lk_p2p_group *g);
void lk_p2p_group_destroy(lk_p2p_group *g);
int lk_p2p_plan_create(lk_p2p_group *g, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                       lk_p2p_plan **out);
int lk_p2p_plan_launch(lk_p2p_plan *plan, void *const *streams);
uint64_t lk_p2p_plan_num_launches(const lk_p2p_plan *plan);
int lk_p2p_plan_signal(lk_p2p_plan *plan, int rank, uint64_t *value);
void lk_p2p_plan_destroy(lk_p2p_plan *plan);
/* The persistent form of the same partition: a CHAIN of dependent stages of N = 1 nodes
 * (lk_plan_create_chain's semantics: node i in stage stage[i]) as ONE launch per rank. Rank r's
 * launch streams its row shard of every node; each row it computes is stored into its own full dst
 * and into every other rank's (system-scope stores: xGMI on a node); the grid barrier between stages
 * waits until EVERY rank has completed the stage (the rank that completes its stage adds 1 to a
 * monotonic arrival word of every rank), so stage s + 1 reads whole activations. No host gate, no
 * collective, no extra launch per layer. Tensors rank-major as lk_p2p_plan_create, every dst a dense
 * F32 [1, M] (N = 1 streaming nodes of one quant type), and every rank's dst tensors laid out alike
 * (one byte offset per pair of ranks over all nodes). Ranks on one device share its CUs and need
 * streams of their own (they wait for each other inside their launches). Waits are bounded like a
 * chain plan's: lk_p2p_chain_timed_out reports (and re-arms) a rank whose barrier gave up.
 * Memory model (round 6): arrival words in fine-grained device memory; the rank completing a stage
 * issues a system-scope release before its cross adds, the poller a system-scope acquire after its
 * poll, and the next stage loads its activations at system scope; each wave stores its rows to a peer
 * as one contiguous store per block of 64 rows; a closing barrier ends every rank's launch only once
 * every rank's last stage has drained, so a rank's dst is complete when that rank's stream is.
 * Ranks on several GPUs are refused (LK_ERR_NOT_IMPLEMENTED) until a multi-GPU run validates this
 * (LK_P2P_CHAIN_CROSS_DEVICE=1 opts in; the dst buffers must then be fine-grained allocations); the
 * one-GPU tests run P ranks on device 0. */
typedef struct lk_p2p_chain lk_p2p_chain;
int lk_p2p_chain_create(lk_p2p_group *g, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage,
                        int n, lk_p2p_chain **out);
/* streams[r] on rank r's device, or NULL: the group's own stream per rank, where ranks sharing a device
 * get disjoint equal CU masks (hipExtStreamCreateWithCUMask: separate queues, every rank resident). */
int lk_p2p_chain_launch(lk_p2p_chain *chain, void *const *streams);
int lk_p2p_chain_timed_out(lk_p2p_chain *chain);
uint64_t lk_p2p_chain_num_launches(const lk_p2p_chain *chain);
/* The group's own stream of rank r (the one lk_p2p_chain_launch(chain, NULL) uses), or NULL. */
void *lk_p2p_chain_rank_stream(lk_p2p_chain *chain, int r);
void lk_p2p_chain_destroy(lk_p2p_chain *chain);

/* ---- graph residency over host buffers ---------------------------------------
 * GGMLComputeOps.computeGraph / computeMulMat (core/GGMLComputeOps.kt:2515-2652) for a
 * graph of n MUL_MAT nodes on host ByteArrays, kept device-resident between nodes
 * (SURVEY §8f row 2). Nodes are given in graph order; a node that reads bytes an earlier
 * node writes runs after it. Quantized A operands no node writes are weights: pinned at
 * create with weight_generation (lk_weights_pin semantics); when a later pin of another
 * generation or an eviction supersedes one, the next compute re-binds to the current mirror. Every other range gets a device mirror; a compute
 * uploads only ranges no earlier node produces, runs each dependency level as one
 * lk_plan, and writes back the dst of nodes with outputs[i] != 0 (outputs = NULL: all).
 * Same results as n lk_mul_mat calls in order. */
typedef struct lk_graph lk_graph;
int lk_graph_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                    const uint8_t *outputs, uint64_t weight_generation, lk_graph **out);
/* The same graph row-sharded over the GPUs of a node (the north star's partition behind the
 * graph API): every quantized weight node whose rows split evenly (M % P == 0, K % 32 == 0, dense
 * F32 dst) runs rank r's rows [r·M/P, (r+1)·M/P) on rank r's device — only that shard of the
 * weight is pinned there — into the full dst mirror, and one in-place RCCL all-gather per level
 * completes every dst on every device, so the next level reads whole activations on each. Other
 * nodes run whole on every device. Results are the bytes lk_graph_create's graph produces.
 *   ncomms == 1: comms[0] is this process's rank (one process per GPU; lk_comm_init_rank, or a
 *                one-rank communicator); the graph runs on its device, HIP-graph replayed.
 *   ncomms  > 1: comms[r] = rank r of lk_comm_init_all (one thread drives every device); each
 *                level's launches and all-gathers of all devices form one RCCL group; outputs are
 *                read back from rank 0's device.
 * The communicators must outlive the graph. */
int lk_graph_create_sharded(lk_comm *const *comms, int ncomms, const lk_tensor *a, const lk_tensor *b,
                            const lk_tensor *dst, int n, const uint8_t *outputs, uint64_t weight_generation,
                            lk_graph **out);
/* Nodes of the graph that run row-sharded (0 for lk_graph_create's graphs). */
int lk_graph_num_sharded(const lk_graph *g);
/* Upload inputs, run, write outputs back; synchronous. */
int lk_graph_compute(lk_graph *g);
int lk_graph_num_levels(const lk_graph *g);
/* How many times a compute found a bound weight mirror superseded / evicted and re-bound. */
int lk_graph_num_rebinds(const lk_graph *g);
int lk_graph_num_launches(const lk_graph *g);
/* Bytes one lk_graph_compute moves host->device (to_device = 1) or back (0). */
uint64_t lk_graph_transfer_bytes(const lk_graph *g, int to_device);
void lk_graph_destroy(lk_graph *g);

/* ---- weight residency (host path) ------------------------------------------ */

/* Residency contract (the host ByteArrays stay authoritative, core/GGMLAlloc.kt:271): a
 * device mirror is current for (ByteArray base, byte range, generation). The caller bumps the
 * generation whenever it rewrites or re-places bytes a pin covers (GGMLGraphAllocator.
 * allocateGraph re-placing tensors, core/GGMLAlloc.kt:404-480; reserve replacing a buffer,
 * :392, :638), or evicts the range. A mirror that is superseded or evicted is never read
 * again: lk_mul_mat stages the bytes instead, and an lk_graph re-binds its weights at its
 * next compute.
 *
 * lk_weights_pin: make a's bytes current on the device as of `generation`. Same generation
 * and already covered: nothing is copied. Any current mirror of other generation that
 * overlaps those bytes is superseded (dropped from the cache; its memory is freed once no
 * graph holds it). A later lk_mul_mat whose A bytes a current mirror covers skips the upload. */
int lk_weights_pin(const lk_tensor *a, uint64_t generation);
/* Drop every current mirror overlapping a's bytes (all devices). */
int lk_weights_evict(const lk_tensor *a);
/* Drop every current mirror of the ByteArray at data (buffer replaced or freed). */
int lk_weights_evict_buffer(const void *data, uint64_t buf_bytes);
/* Drop every current mirror. Live graphs keep their memory until they re-bind. */
void lk_weights_evict_all(void);
/* Bytes / mirrors currently held by the weight cache (superseded mirrors excluded). */
uint64_t lk_weights_cached_bytes(void);
uint64_t lk_weights_cached_count(void);
/* Pin each row shard of a quantized A on the device lk_mul_mat_sharded(…, n_shards)
 * runs it on (the mirror lk_weights_pin keeps, per shard and device). */
int lk_weights_pin_sharded(const lk_tensor *a, uint64_t generation, int n_shards);
int lk_weights_pin_sharded_at(const lk_tensor *a, uint64_t generation, int n_shards, int first_device);

/* ---- format kernels (the steps either side of the path) --------------------- */

/* dequantizeTensor for Q8_0/Q4_0/Q4_1 (device buffers): writes numElements f32
 * values (flat order) to out. Bit-exact with the reference. */
int lk_dequantize_device(const lk_tensor *src, float *out, void *stream);
/* quantizeTensor for a contiguous F32 source into Q8_0/Q4_0/Q4_1 block bytes
 * (device buffers): out receives numElements/32 blocks. Bit-exact with the
 * reference (round-half-even, Kotlin floatToHalf). */
int lk_quantize_device(const float *src, int64_t n_elements, int32_t type, void *out,
                       void *stream);

/* ---- direct dot products (core/GGMLComputeOps.kt:349-629) -------------------
 * Not reachable from computeMatMul in the reference; offloaded as one
 * matrix of dots: out[row·N + col] = computeDotProduct<kind>(ga, a, b, row, col, K) for
 * row < M = a.ne[1], col < N = b.ne[0]. A is M x K (ne[0] = K): its Q elements are read at
 * the flat index row·K + k, its F32 elements through nb (getFloat(k, row)). B is K x N
 * (ne[0] = N, ne[1] = K), read at the flat index k·N + col. Every element, product and sum
 * is the Kotlin expression in the Kotlin order (sequential k, no fused multiply-add), so
 * results are bit-identical to the reference arithmetic. */
enum lk_dot_kind {
  LK_DOT_F32_Q4_1 = 1, /* :349-377 computeDotProductF32Q41: f · (d·q + m)               */
  LK_DOT_F32_Q8_0 = 2, /* :442-468 computeDotProductF32Q80: f · (d·q)                   */
  LK_DOT_Q8_0_Q8_0 = 3, /* :474-507 computeDotProductQ80Q80: (dA·dB) · (qA·qB)           */
  LK_DOT_Q4_0_Q4_0 = 4, /* :512-548 computeDotProductQ40Q40: dA·(nA−8) · dB·(nB−8)      */
  LK_DOT_Q4_1_Q4_1 = 5, /* :552-589 computeDotProductQ41Q41: (dA·nA + mA)·(dB·nB + mB)  */
  LK_DOT_Q8_0_Q4_0 = 6  /* :594-629 computeDotProductQ80Q40: dA·qA · dB·(nB−8)          */
};
/* Host buffers (a->data / b->data are the ByteArrays), synchronous; out: M·N floats (host).
 * The require() checks of the Kotlin functions come first (types, a.ne[0] == K,
 * b.ne[1] == K: LK_ERR_INVALID_ARG), then the accessors' (block index past numBlocks:
 * LK_ERR_INVALID_ARG; bytes past the buffer: LK_ERR_OUT_OF_BOUNDS; no buffer:
 * LK_ERR_NO_BUFFER). Unknown kind: LK_ERR_NOT_IMPLEMENTED. */
int lk_dot_direct(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out);
/* The same over device buffers, enqueued on `stream` (NULL: the library's stream). */
int lk_dot_direct_device(int32_t kind, const lk_tensor *a, const lk_tensor *b, int64_t K, float *out,
                         void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LK_HIP_H */
