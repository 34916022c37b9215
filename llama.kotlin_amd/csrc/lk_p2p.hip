// lk_p2p.hip — the one-shot peer-write alternative to the RCCL all-gather.
//
// Same partition as lk_comm.cpp: rank r of P owns rows [r·M/P, (r+1)·M/P) of every weight matrix
// and computes them in place inside its FULL dst. Instead of an ncclGroup of all-gathers, rank r's
// push kernel writes those rows straight into every peer's dst over xGMI (plain stores to peer
// memory, peer access enabled) and then adds 1 to a per-plan arrival signal on every rank. The next
// plan's launch on rank q is gated by hipStreamWaitValue64(signal >= launches·P): the command
// processor holds the queue, no kernel spins. One process drives the P devices (the Kotlin host's
// shape, lk_comm_init_all's): one launch call enqueues every rank's work on its stream.
//
// Arrival values are monotonic (launch k leaves k·P on every rank's signal), which is why this path
// is eager-only: a captured hipStreamWaitValue64 would replay one baked value. Capturing returns
// LK_ERR_NOT_IMPLEMENTED; lk_sharded_plan stays the graph-replayable path.
//
// Ranks may share a device (the one-GPU tests run P ranks on device 0, each with its own dst
// buffers); ranks on one device must then share one stream, so a rank's gate can only wait for
// pushes enqueued before it on that stream (different streams of one device may share a hardware
// queue, where a gate ahead of the push it waits for would never open).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/lk_hip.h"
#include "lk_peer.hpp"

int lk_detail_fail(int st, const char *msg);
extern "C" int lk_detail_chain_create(const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage,
                                      int n, int grid, const void *peer, lk_plan **out);

namespace {

constexpr int kMaxRanks = 8;  // one node

struct PushSeg {
  const uint8_t *src;          // this rank's rows inside its own full dst
  uint8_t *dst[kMaxRanks];     // the same rows inside rank q's full dst (q = self: unused)
  uint64_t bytes;
  int vec;                     // 16-byte copies (sizes and addresses aligned) or byte copies
};

struct PushArgs {
  const PushSeg *seg;
  int nseg, P, self;
  unsigned long long *sig[kMaxRanks];  // every rank's arrival signal of this plan
  unsigned *arrive;                    // this launch's block count (last block re-arms it)
};

// One block per (segment, peer): copy, release at system scope, count the block; the last block
// of the launch (no waits: the last arriver) signals every rank. A launch with nothing to copy
// (P = 1) is one block that only signals.
__global__ __launch_bounds__(256) void p2p_push_kernel(PushArgs g) {
  const int peers = g.P - 1;
  if (peers > 0 && g.nseg > 0) {
    const int s = (int)blockIdx.x / peers;
    int q = (int)blockIdx.x % peers;
    q += q >= g.self;  // skip self: its rows are already in place
    const PushSeg &sg = g.seg[s];
    uint8_t *to = sg.dst[q];
    if (sg.vec) {
      const uint4 *src = (const uint4 *)sg.src;
      uint4 *dst = (uint4 *)to;
      for (uint64_t i = threadIdx.x; i < sg.bytes / 16; i += blockDim.x) dst[i] = src[i];
    } else {
      for (uint64_t i = threadIdx.x; i < sg.bytes; i += blockDim.x) to[i] = sg.src[i];
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned before = __hip_atomic_fetch_add(g.arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (before + 1 == gridDim.x) {
      __hip_atomic_store(g.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 0; q < g.P; q++)
        __hip_atomic_fetch_add(g.sig[q], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <typename F>
int on_device(int dev, F f) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = dev;
  if (prev != dev && hipSetDevice(dev) != hipSuccess) return lk_detail_fail(LK_ERR_DEVICE, "p2p: cannot select a device");
  const int rc = f();
  if (prev != dev) (void)hipSetDevice(prev);
  return rc;
}

}  // namespace

struct lk_p2p_plan;

struct lk_p2p_group {
  int P = 0;
  std::vector<int> dev;
  // per rank: the plan launched last in this group and the value its signal on this rank reaches
  // once every rank's rows of that launch are in place here
  std::vector<lk_p2p_plan *> tail;
  std::vector<uint64_t> tail_target;
  // lk_p2p_chain_launch with streams == NULL: per rank a stream of its own; ranks sharing a device
  // get disjoint CU masks (hipExtStreamCreateWithCUMask), so they run at once on separate queues
  std::vector<hipStream_t> rank_stream;
  uint64_t plans_alive = 0;
  bool destroyed = false;  // lk_p2p_group_destroy ran while plans were alive: the last plan deletes the group
  bool broken = false;  // a launch failed after some ranks enqueued theirs: later gates could never open
};

struct lk_p2p_plan {
  lk_p2p_group *g = nullptr;
  int n = 0;
  uint64_t launches = 0;
  std::vector<lk_plan *> local;             // per rank: its rows of every node, one grouped launch
  std::vector<unsigned long long *> sig;    // per rank: arrival signal (hipMallocSignalMemory)
  std::vector<unsigned *> arrive;           // per rank: push-kernel block counter (device memory)
  std::vector<PushSeg *> seg;               // per rank: device copy of its segments
  std::vector<int> blocks;                  // per rank: push grid
};

namespace {

void free_plan(lk_p2p_plan *p) {
  for (int r = 0; r < (int)p->local.size(); r++) {
    (void)on_device(p->g->dev[r], [&] {
      if (p->local[r]) lk_plan_destroy(p->local[r]);
      if (p->sig[r]) (void)hipFree(p->sig[r]);
      if (p->arrive[r]) (void)hipFree(p->arrive[r]);
      if (p->seg[r]) (void)hipFree(p->seg[r]);
      return 0;
    });
  }
  delete p;
}

}  // namespace

extern "C" {

int lk_p2p_group_create(int nranks, const int *devices, lk_p2p_group **out) {
  if (!out || nranks < 1 || nranks > kMaxRanks || !devices)
    return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p group: 1..8 ranks and their devices");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return lk_detail_fail(LK_ERR_DEVICE, "p2p group: no device");
  for (int r = 0; r < nranks; r++)
    if (devices[r] < 0 || devices[r] >= ndev) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p group: no such device");
  for (int r = 0; r < nranks; r++) {  // every rank's stream is gated on a memory value
    int ok = 1;
    if (hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, devices[r]) != hipSuccess || !ok)
      return lk_detail_fail(LK_ERR_DEVICE, "p2p group: a device cannot gate a stream on a memory value");
  }
  for (int r = 0; r < nranks; r++) {
    int rc = lk_init(devices[r]);
    if (rc) return rc;
  }
  // peer access between every pair of distinct devices (both directions: each rank writes to all)
  for (int i = 0; i < nranks; i++)
    for (int j = 0; j < nranks; j++) {
      const int di = devices[i], dj = devices[j];
      if (di == dj) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, di, dj) != hipSuccess || !can)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p group: devices are not peers");
      const int rc = on_device(di, [&] {
        const hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
          return lk_detail_fail(LK_ERR_DEVICE, "p2p group: hipDeviceEnablePeerAccess failed");
        (void)hipGetLastError();
        return (int)LK_OK;
      });
      if (rc) return rc;
    }
  auto g = new lk_p2p_group();
  g->P = nranks;
  g->dev.assign(devices, devices + nranks);
  g->tail.assign(nranks, nullptr);
  g->tail_target.assign(nranks, 0);
  *out = g;
  return LK_OK;
}

int lk_p2p_group_nranks(const lk_p2p_group *g) { return g ? g->P : 0; }

namespace {
void delete_group(lk_p2p_group *g) {
  for (size_t r = 0; r < g->rank_stream.size(); r++)
    if (g->rank_stream[r]) (void)on_device(g->dev[r], [&] { (void)hipStreamDestroy(g->rank_stream[r]); return 0; });
  delete g;
}
}  // namespace

// A group with live plans is only marked: each plan holds a pointer to it, and the last plan's
// destroy deletes it (a caller closing the group before its plans must not leave them dangling).
void lk_p2p_group_destroy(lk_p2p_group *g) {
  if (!g) return;
  if (g->plans_alive) {
    g->destroyed = true;
    return;
  }
  delete_group(g);
}

int lk_p2p_plan_create(lk_p2p_group *g, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                       lk_p2p_plan **out) {
  if (!g || !out || n < 0 || (n && (!a || !b || !dst))) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: bad arguments");
  *out = nullptr;
  const int P = g->P;
  // validate: dst[r*n+i] is rank r's full dst of node i, dense rows, rows split evenly
  for (int i = 0; i < n; i++) {
    const lk_tensor &d0 = dst[i];
    for (int r = 0; r < P; r++) {
      const lk_tensor &d = dst[r * n + i];
      const int64_t M = d.ne[1], N = d.ne[0];
      const uint64_t ew = d.type == LK_TYPE_F16 ? 2 : 4;
      if (d.type != d0.type || d.ne[0] != d0.ne[0] || d.ne[1] != d0.ne[1])
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: every rank's dst of a node must have one shape");
      if (M % P != 0 || a[r * n + i].ne[1] != M / P)
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: A must hold rows [r*M/P, (r+1)*M/P) with M % P == 0");
      if (d.nb[0] != ew || d.nb[1] != (uint64_t)N * ew || !d.data)
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: dst rows must be dense (nb[1] == N * element size)");
      if (d.data_offset + (uint64_t)M * d.nb[1] > d.buf_bytes)
        return lk_detail_fail(LK_ERR_OUT_OF_BOUNDS, "p2p plan: dst exceeds its buffer");
    }
  }
  auto p = new lk_p2p_plan();
  p->g = g;
  p->n = n;
  p->local.assign(P, nullptr);
  p->sig.assign(P, nullptr);
  p->arrive.assign(P, nullptr);
  p->seg.assign(P, nullptr);
  p->blocks.assign(P, 1);
  for (int r = 0; r < P; r++) {
    std::vector<lk_tensor> la(a + r * n, a + (r + 1) * n), lb(b + r * n, b + (r + 1) * n), ld(dst + r * n, dst + (r + 1) * n);
    std::vector<PushSeg> segs(n);
    for (int i = 0; i < n; i++) {
      const uint64_t chunk = (uint64_t)(ld[i].ne[1] / P) * ld[i].nb[1];
      ld[i].ne[1] /= P;
      ld[i].data_offset += (uint64_t)r * chunk;  // this rank's rows land at their place in its full dst
      PushSeg &s = segs[i];
      std::memset(&s, 0, sizeof s);
      s.src = (const uint8_t *)ld[i].data + ld[i].data_offset;
      s.bytes = chunk;
      bool aligned = chunk % 16 == 0 && (uintptr_t)s.src % 16 == 0;
      for (int q = 0; q < P; q++) {
        const lk_tensor &dq = dst[q * n + i];
        s.dst[q] = (uint8_t *)dq.data + dq.data_offset + (uint64_t)r * chunk;
        aligned = aligned && (uintptr_t)s.dst[q] % 16 == 0;
      }
      s.vec = aligned;
    }
    const int rc = on_device(g->dev[r], [&]() -> int {
      int rc2 = lk_plan_create(la.data(), lb.data(), ld.data(), n, &p->local[r]);
      if (rc2) return rc2;
      if (hipExtMallocWithFlags((void **)&p->sig[r], sizeof(unsigned long long), hipMallocSignalMemory) != hipSuccess) {
        p->sig[r] = nullptr;
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: cannot allocate signal memory");
      }
      if (hipMalloc((void **)&p->arrive[r], sizeof(unsigned)) != hipSuccess) {
        p->arrive[r] = nullptr;
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: out of device memory");
      }
      if (n && hipMalloc((void **)&p->seg[r], sizeof(PushSeg) * n) != hipSuccess) {
        p->seg[r] = nullptr;
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: out of device memory");
      }
      const unsigned long long zero = 0;
      const unsigned zero32 = 0;
      if (hipMemcpy(p->sig[r], &zero, sizeof zero, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(p->arrive[r], &zero32, sizeof zero32, hipMemcpyHostToDevice) != hipSuccess ||
          (n && hipMemcpy(p->seg[r], segs.data(), sizeof(PushSeg) * n, hipMemcpyHostToDevice) != hipSuccess))
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: upload failed");
      return (int)LK_OK;
    });
    if (rc) { free_plan(p); return rc; }
    p->blocks[r] = (P > 1 && n > 0) ? n * (P - 1) : 1;
  }
  g->plans_alive++;
  *out = p;
  return LK_OK;
}

int lk_p2p_plan_launch(lk_p2p_plan *p, void *const *streams) {
  if (!p || !streams) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: null plan or streams");
  lk_p2p_group *g = p->g;
  const int P = g->P;
  for (int r = 0; r < P; r++) {
    for (int q = 0; q < r; q++)
      if (g->dev[q] == g->dev[r] && streams[q] != streams[r])
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: ranks on one device must share one stream");
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const int rc = on_device(g->dev[r], [&]() -> int {
      if (hipStreamIsCapturing((hipStream_t)streams[r], &cs) != hipSuccess)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: cannot query the stream");
      return (int)LK_OK;
    });
    if (rc) return rc;
    if (cs != hipStreamCaptureStatusNone)
      return lk_detail_fail(LK_ERR_NOT_IMPLEMENTED, "p2p plan: eager only (its gates wait for monotonic values); "
                                                    "capture lk_sharded_plan instead");
  }
  if (g->broken) return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: an earlier launch in this group failed part-way");
  const uint64_t epoch = p->launches + 1;
  for (int r = 0; r < P; r++) {
    hipStream_t st = (hipStream_t)streams[r];
    const int rc = on_device(g->dev[r], [&]() -> int {
      if (g->tail[r] &&
          hipStreamWaitValue64(st, g->tail[r]->sig[r], g->tail_target[r], hipStreamWaitValueGte, ~0ull) != hipSuccess)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: hipStreamWaitValue64 failed");
      int rc2 = lk_plan_launch(p->local[r], st);
      if (rc2) return rc2;
      PushArgs args;
      std::memset(&args, 0, sizeof args);
      args.seg = p->seg[r];
      args.nseg = p->n;
      args.P = P;
      args.self = r;
      for (int q = 0; q < P; q++) args.sig[q] = p->sig[q];
      args.arrive = p->arrive[r];
      hipLaunchKernelGGL(p2p_push_kernel, dim3(p->blocks[r]), dim3(256), 0, st, args);
      if (hipGetLastError() != hipSuccess) return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: push launch failed");
      return (int)LK_OK;
    });
    if (rc) {  // ranks before r have enqueued this launch: a later gate on it would never open
      g->broken = true;
      return rc;
    }
  }
  p->launches = epoch;
  for (int r = 0; r < P; r++) {
    g->tail[r] = p;
    g->tail_target[r] = epoch * (uint64_t)P;
  }
  return LK_OK;
}

uint64_t lk_p2p_plan_num_launches(const lk_p2p_plan *p) { return p ? p->launches : 0; }

int lk_p2p_plan_signal(lk_p2p_plan *p, int rank, uint64_t *value) {
  if (!p || !value || rank < 0 || rank >= p->g->P) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p plan: bad rank");
  return on_device(p->g->dev[rank], [&]() -> int {
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(value, p->sig[rank], sizeof(uint64_t), hipMemcpyDefault) != hipSuccess)
      return lk_detail_fail(LK_ERR_DEVICE, "p2p plan: cannot read the signal");
    return (int)LK_OK;
  });
}

void lk_p2p_plan_destroy(lk_p2p_plan *p) {
  if (!p) return;
  lk_p2p_group *g = p->g;
  for (int r = 0; r < g->P; r++)
    if (g->tail[r] == p) g->tail[r] = nullptr;  // the caller synchronized: nothing left to gate on
  g->plans_alive--;
  free_plan(p);
  if (g->destroyed && g->plans_alive == 0) delete_group(g);
}

}  // extern "C"

// ---- multi-GPU chains: one persistent stream-kernel launch per rank, cross-rank barriers ------------
//
// lk_p2p_chain (include/lk_hip.h): the chain plan of lk_plan_create_chain (dependent stages of N = 1
// nodes in one launch, a grid barrier between stages), per rank over its row shards, with the rows
// stored into every rank's copy of dst and every barrier waiting for every rank's stage (PeerDesc,
// gemv_stream_peer_kernel in lk_kernels.hpp). No host gate, no collective, no extra launch: a token's
// whole layer stack is P concurrent launches. Ranks sharing one device (the one-GPU tests) each take
// an equal share of its CUs and need streams of their own, since the ranks wait for each other
// inside their launches and must therefore run at the same time.

struct lk_p2p_chain {
  lk_p2p_group *g = nullptr;
  int nbar = 0;
  std::vector<lk_plan *> plan;         // per rank: its chain plan (gemv_stream_peer_kernel)
  std::vector<lk::PeerDesc *> desc;    // per rank: device copy of its PeerDesc
  std::vector<unsigned *> cross;       // per rank: nbar arrival lines (monotonic) + the epoch line
  uint64_t launches = 0;
};

namespace {

void free_chain(lk_p2p_chain *c) {
  for (int r = 0; r < (int)c->plan.size(); r++) {
    (void)on_device(c->g->dev[r], [&] {
      if (c->plan[r]) lk_plan_destroy(c->plan[r]);
      if (c->desc[r]) (void)hipFree(c->desc[r]);
      if (c->cross[r]) (void)hipFree(c->cross[r]);
      return 0;
    });
  }
  delete c;
}

}  // namespace

extern "C" {

int lk_p2p_chain_create(lk_p2p_group *g, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, const int32_t *stage,
                        int n, lk_p2p_chain **out) {
  if (!g || !out || n <= 0 || !a || !b || !dst || !stage) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: bad arguments");
  *out = nullptr;
  const int P = g->P;
  if (P > lk::kMaxPeerRanks) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: at most 8 ranks");
  // every rank's dst of node i: one shape, dense rows, M % P == 0, and one byte offset per rank
  // between rank q's dst and rank r's over all nodes (the kernel stores rank r's rows at dst + delta)
  std::vector<int64_t> delta((size_t)P * P, 0);
  for (int i = 0; i < n; i++) {
    const lk_tensor &d0 = dst[i];
    for (int r = 0; r < P; r++) {
      const lk_tensor &d = dst[r * n + i];
      const int64_t M = d.ne[1];
      if (d.type != LK_TYPE_F32 || d.ne[0] != 1 || d0.ne[1] != M || d.nb[1] != 4 || !d.data)
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: every dst must be a dense F32 [1, M], one shape per node");
      if (M % P != 0 || a[r * n + i].ne[1] != M / P)
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: A must hold rows [r*M/P, (r+1)*M/P) with M % P == 0");
      if (d.data_offset + (uint64_t)M * 4 > d.buf_bytes) return lk_detail_fail(LK_ERR_OUT_OF_BOUNDS, "p2p chain: dst exceeds its buffer");
      for (int q = 0; q < P; q++) {
        const lk_tensor &dq = dst[q * n + i];
        const int64_t dl = (int64_t)((uintptr_t)d.data + d.data_offset) - (int64_t)((uintptr_t)dq.data + dq.data_offset);
        if (i == 0) delta[(size_t)q * P + r] = dl;
        else if (delta[(size_t)q * P + r] != dl)
          return lk_detail_fail(LK_ERR_NOT_IMPLEMENTED, "p2p chain: each rank's dst tensors must share one layout (one offset per rank pair)");
      }
    }
  }
  int nstage = 0;
  for (int i = 0; i < n; i++) nstage = std::max(nstage, stage[i] + 1);
  auto c = new lk_p2p_chain();
  c->g = g;
  c->nbar = nstage - 1;
  c->plan.assign(P, nullptr);
  c->desc.assign(P, nullptr);
  c->cross.assign(P, nullptr);
  // ranks per device: they share its CUs (all of a rank's workgroups and every other rank's must be
  // resident at once: a barrier waits for every rank)
  std::vector<int> share(P, 0);
  for (int r = 0; r < P; r++)
    for (int q = 0; q < P; q++) share[r] += g->dev[q] == g->dev[r];
  // Ranks on different GPUs: the memory model below (fine-grained arrival words, system-scope release
  // before every cross add, system-scope acquire and loads after every poll, a closing barrier) has only
  // run with every rank on one GPU, where one L2 hides any gap in it. Refused until a multi-GPU run
  // validates it; LK_P2P_CHAIN_CROSS_DEVICE=1 opts in (unvalidated).
  {
    bool multi = false;
    for (int r = 1; r < P; r++) multi |= g->dev[r] != g->dev[0];
    static const bool cross_ok = [] { const char *e = std::getenv("LK_P2P_CHAIN_CROSS_DEVICE"); return e && *e == '1'; }();
    if (multi && !cross_ok)
      return lk_detail_fail(LK_ERR_NOT_IMPLEMENTED, "p2p chain: ranks on several GPUs are not validated yet (set "
                                                    "LK_P2P_CHAIN_CROSS_DEVICE=1 to opt in); use lk_sharded_plan");
  }
  // per rank: one line per stage barrier, the closing barrier's line (nbar), the epoch line (nbar + 1);
  // fine-grained device memory, so the peers' system-scope adds and this rank's polls meet coherently
  const size_t lines = (size_t)c->nbar + 2;
  for (int r = 0; r < P; r++) {
    const int rc = on_device(g->dev[r], [&]() -> int {
      if (hipExtMallocWithFlags((void **)&c->cross[r], lines * lk::kChainLine * sizeof(unsigned), hipDeviceMallocFinegrained) !=
          hipSuccess) {
        c->cross[r] = nullptr;
        return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: out of device memory");
      }
      if (hipMemset(c->cross[r], 0, lines * lk::kChainLine * sizeof(unsigned)) != hipSuccess)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: cannot zero the arrival words");
      return (int)LK_OK;
    });
    if (rc) { free_chain(c); return rc; }
  }
  for (int r = 0; r < P; r++) {
    lk::PeerDesc pd;
    std::memset(&pd, 0, sizeof pd);
    pd.P = P;
    pd.rank = r;
    for (int q = 0; q < P; q++) {
      pd.delta[q] = delta[(size_t)r * P + q];
      pd.cross[q] = c->cross[q];
    }
    pd.epoch = c->cross[r] + (lines - 1) * lk::kChainLine;
    // this rank's nodes: its row shard of A, its copy of B, its rows inside its full dst
    std::vector<lk_tensor> la(a + r * n, a + (r + 1) * n), lb(b + r * n, b + (r + 1) * n), ld(dst + r * n, dst + (r + 1) * n);
    for (int i = 0; i < n; i++) {
      const int64_t rows = ld[i].ne[1] / P;
      ld[i].ne[1] = rows;
      ld[i].data_offset += (uint64_t)r * rows * 4;
    }
    const int rc = on_device(g->dev[r], [&]() -> int {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->dev[r]) != hipSuccess || cus <= 0) cus = 256;
      const int grid = std::max(1, cus / share[r]);
      if (hipMalloc((void **)&c->desc[r], sizeof pd) != hipSuccess) {
        c->desc[r] = nullptr;
        return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: out of device memory");
      }
      if (hipMemcpy(c->desc[r], &pd, sizeof pd, hipMemcpyHostToDevice) != hipSuccess)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: upload failed");
      return lk_detail_chain_create(la.data(), lb.data(), ld.data(), stage, n, grid, c->desc[r], &c->plan[r]);
    });
    if (rc) { free_chain(c); return rc; }
  }
  g->plans_alive++;
  *out = c;
  return LK_OK;
}

namespace {
// The group's own per-rank streams (created once): ranks sharing a device get disjoint, equal CU masks.
int rank_streams(lk_p2p_group *g) {
  if (!g->rank_stream.empty()) return LK_OK;
  const int P = g->P;
  std::vector<hipStream_t> st(P, nullptr);
  for (int r = 0; r < P; r++) {
    int share = 0, idx = 0;
    for (int q = 0; q < P; q++) {
      share += g->dev[q] == g->dev[r];
      idx += q < r && g->dev[q] == g->dev[r];
    }
    const int rc = on_device(g->dev[r], [&]() -> int {
      if (share == 1) return hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking) == hipSuccess ? (int)LK_OK
                                                                                                  : lk_detail_fail(LK_ERR_DEVICE, "p2p chain: stream");
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->dev[r]) != hipSuccess || cus <= 0)
        return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: CU count");
      const int per = cus / share;
      std::vector<uint32_t> mask((cus + 31) / 32, 0u);
      for (int cu = idx * per; cu < (idx + 1) * per; cu++) mask[cu / 32] |= 1u << (cu % 32);
      return hipExtStreamCreateWithCUMask(&st[r], (uint32_t)mask.size(), mask.data()) == hipSuccess
                 ? (int)LK_OK : lk_detail_fail(LK_ERR_DEVICE, "p2p chain: CU-masked stream");
    });
    if (rc) {
      for (int q = 0; q < r; q++) (void)on_device(g->dev[q], [&] { (void)hipStreamDestroy(st[q]); return 0; });
      return rc;
    }
  }
  g->rank_stream = st;
  return LK_OK;
}
}  // namespace

int lk_p2p_chain_launch(lk_p2p_chain *c, void *const *streams) {
  if (!c) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: null chain");
  lk_p2p_group *g = c->g;
  const int P = g->P;
  std::vector<void *> own;
  if (!streams) {  // the group's per-rank streams (CU-partitioned where ranks share a device)
    if (int rc = rank_streams(g)) return rc;
    own.assign(g->rank_stream.begin(), g->rank_stream.end());
    streams = own.data();
  }
  for (int r = 0; r < P; r++)
    for (int q = 0; q < r; q++)
      if (g->dev[q] == g->dev[r] && streams[q] == streams[r])
        return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: ranks on one device need streams of their own (they run at once)");
  if (g->broken) return lk_detail_fail(LK_ERR_DEVICE, "p2p chain: an earlier launch in this group failed part-way");
  for (int r = 0; r < P; r++) {
    const int rc = on_device(g->dev[r], [&]() -> int { return lk_plan_launch(c->plan[r], streams[r]); });
    if (rc) {  // ranks before r wait at their first barrier for this one: they give up at the bound
      g->broken = true;
      return rc;
    }
  }
  c->launches++;
  return LK_OK;
}

int lk_p2p_chain_timed_out(lk_p2p_chain *c) {
  if (!c) return lk_detail_fail(LK_ERR_INVALID_ARG, "p2p chain: null chain");
  int any = 0;
  for (int r = 0; r < c->g->P; r++) {
    const int rc = on_device(c->g->dev[r], [&]() -> int { return lk_plan_chain_timed_out(c->plan[r]); });
    if (rc < 0 || rc > 1) return rc;
    any |= rc;
  }
  return any;
}

uint64_t lk_p2p_chain_num_launches(const lk_p2p_chain *c) { return c ? c->launches : 0; }

void *lk_p2p_chain_rank_stream(lk_p2p_chain *c, int r) {
  if (!c || r < 0 || r >= c->g->P) return nullptr;
  if (rank_streams(c->g)) return nullptr;
  return (void *)c->g->rank_stream[r];
}

void lk_p2p_chain_destroy(lk_p2p_chain *c) {
  if (!c) return;
  lk_p2p_group *g = c->g;
  g->plans_alive--;
  free_chain(c);
  if (g->destroyed && g->plans_alive == 0) delete_group(g);
}

}  // extern "C"
