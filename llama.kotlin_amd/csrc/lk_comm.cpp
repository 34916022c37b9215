// lk_comm.cpp — multi-GPU row sharding of the MUL_MAT path with an RCCL all-gather over xGMI
// (BASELINE north_star: "weight rows shard naturally across the 8 GPUs of one node
// with an RCCL all-gather over xGMI to reassemble output activations").
//
// The reference is single-device (no collective code at all); this is the
// north star's partition. Rank r of P owns rows [r·M/P, (r+1)·M/P) of every weight matrix (a
// contiguous byte range: rows are whole blocks) and computes those rows of dst straight into
// their place in the FULL dst buffer. One in-place ncclAllGather per node (sendbuff = recvbuff +
// r·chunk) then fills in the other ranks' rows, so no rank ever copies or permutes: the gathered
// dst is exactly the tensor the next MUL_MAT reads as its activations. Independent nodes share
// one grouped kernel launch and one ncclGroup of gathers, all enqueued on the caller's stream
// (graph-capturable). At batch 1 a Llama-7B layer moves 2–5.5 KB per rank per matrix: the
// collective is latency-bound, so the gathers of a stage are grouped into one RCCL call.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "../../include/lk_hip.h"

int lk_detail_fail(int st, const char *msg);

namespace {

int failf(int st, const char *what, ncclResult_t r) {
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, ncclGetErrorString(r));
  return lk_detail_fail(st, buf);
}

#define NCCL_TRY(expr, what)                                   \
  do {                                                         \
    ncclResult_t r_ = (expr);                                  \
    if (r_ != ncclSuccess) return failf(LK_ERR_DEVICE, what, r_); \
  } while (0)

}  // namespace

struct lk_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0, device = 0;
  uint64_t collectives = 0;  // ncclAllGather calls enqueued through this communicator
};

struct lk_sharded_plan {
  lk_comm *comm = nullptr;
  lk_plan *local = nullptr;                 // this rank's rows of every node: one grouped launch
  struct Gather { void *full; uint64_t chunk; };
  std::vector<Gather> gathers;             // per node: in-place all-gather of chunk bytes per rank
  hipEvent_t rows_done = nullptr;          // lk_sharded_plan_launch_split: the local launch's completion
};

namespace {

// Runs f with the communicator's device current (one host thread may drive several devices:
// lk_comm_init_all), then restores the caller's device.
template <typename F>
int on_device(int dev, F f) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = dev;
  if (prev != dev && hipSetDevice(dev) != hipSuccess) return lk_detail_fail(LK_ERR_DEVICE, "comm: cannot select its device");
  const int rc = f();
  if (prev != dev) (void)hipSetDevice(prev);
  return rc;
}

}  // namespace

extern "C" {

int lk_comm_unique_id(void *id) {
  if (!id) return lk_detail_fail(LK_ERR_INVALID_ARG, "comm: null id");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof u);
  return LK_OK;
}

int lk_comm_init_rank(const void *id, int nranks, int rank, lk_comm **out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return lk_detail_fail(LK_ERR_INVALID_ARG, "comm: bad rank arguments");
  *out = nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return lk_detail_fail(LK_ERR_DEVICE, "comm: no current device");
  int rc = lk_init(dev);
  if (rc) return rc;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  auto c = new lk_comm();
  c->nranks = nranks; c->rank = rank; c->device = dev;
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) { delete c; return failf(LK_ERR_DEVICE, "ncclCommInitRank", r); }
  *out = c;
  return LK_OK;
}

int lk_comm_init_all(int ndev, const int *devices, lk_comm **out) {
  if (ndev < 1 || !out) return lk_detail_fail(LK_ERR_INVALID_ARG, "comm: bad device list");
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; i++) devs[i] = devices ? devices[i] : i;
  std::vector<ncclComm_t> comms(ndev);
  NCCL_TRY(ncclCommInitAll(comms.data(), ndev, devs.data()), "ncclCommInitAll");
  for (int i = 0; i < ndev; i++) {
    auto c = new lk_comm();
    c->comm = comms[i]; c->nranks = ndev; c->rank = i; c->device = devs[i];
    out[i] = c;
  }
  return LK_OK;
}

int lk_comm_nranks(const lk_comm *c) { return c ? c->nranks : 0; }
int lk_comm_rank(const lk_comm *c) { return c ? c->rank : -1; }
int lk_comm_device(const lk_comm *c) { return c ? c->device : -1; }
uint64_t lk_comm_num_collectives(const lk_comm *c) { return c ? c->collectives : 0; }

// Tears down the communicator's enqueued collectives (ncclCommAbort): after a failure left some
// ranks' collectives waiting for peers that never arrive. The handle stays valid for
// lk_comm_destroy; any later collective through it fails.
int lk_comm_abort(lk_comm *c) {
  if (!c) return lk_detail_fail(LK_ERR_INVALID_ARG, "comm: null");
  if (!c->comm) return LK_OK;
  const ncclResult_t r = ncclCommAbort(c->comm);
  c->comm = nullptr;
  if (r != ncclSuccess) return failf(LK_ERR_DEVICE, "ncclCommAbort", r);
  return LK_OK;
}

void lk_comm_destroy(lk_comm *c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int lk_comm_group_start(void) {
  NCCL_TRY(ncclGroupStart(), "ncclGroupStart");
  return LK_OK;
}

int lk_comm_group_end(void) {
  NCCL_TRY(ncclGroupEnd(), "ncclGroupEnd");
  return LK_OK;
}

int lk_sharded_plan_create(lk_comm *comm, const lk_tensor *a, const lk_tensor *b, const lk_tensor *dst, int n,
                           lk_sharded_plan **out) {
  if (!comm || !out || n < 0 || (n && (!a || !b || !dst)))
    return lk_detail_fail(LK_ERR_INVALID_ARG, "sharded plan: bad arguments");
  *out = nullptr;
  const int P = comm->nranks, r = comm->rank;
  std::vector<lk_tensor> la(a, a + n), lb(b, b + n), ld(dst, dst + n);
  auto p = new lk_sharded_plan();
  p->comm = comm;
  for (int i = 0; i < n; i++) {
    const lk_tensor &d = dst[i];
    const int64_t M = d.ne[1], N = d.ne[0];
    const uint64_t ew = d.type == LK_TYPE_F16 ? 2 : 4;
    if (M % P != 0 || a[i].ne[1] != M / P) {
      delete p;
      return lk_detail_fail(LK_ERR_INVALID_ARG, "sharded plan: A must hold rows [r*M/P, (r+1)*M/P) with M % P == 0");
    }
    if (d.nb[0] != ew || d.nb[1] != (uint64_t)N * ew || !d.data) {
      delete p;
      return lk_detail_fail(LK_ERR_INVALID_ARG, "sharded plan: dst rows must be dense (nb[1] == N * element size)");
    }
    const uint64_t chunk = (uint64_t)(M / P) * d.nb[1];
    if (d.data_offset + (uint64_t)M * d.nb[1] > d.buf_bytes) {
      delete p;
      return lk_detail_fail(LK_ERR_OUT_OF_BOUNDS, "sharded plan: dst exceeds its buffer");
    }
    // this rank's rows land at their place in the full dst
    ld[i].ne[1] = M / P;
    ld[i].data_offset = d.data_offset + (uint64_t)r * chunk;
    p->gathers.push_back({(uint8_t *)d.data + d.data_offset, chunk});
  }
  const int rc = on_device(comm->device, [&] { return lk_plan_create(la.data(), lb.data(), ld.data(), n, &p->local); });
  if (rc) { delete p; return rc; }
  *out = p;
  return LK_OK;
}

// The local launch, then one RCCL group of in-place all-gathers — at every world size: at one rank
// the gathers are RCCL's (trivial) in-place copies, so the code path a multi-GPU node runs is the
// one the one-GPU tests exercise. Inside an outer lk_comm_group_start / end (one thread driving
// several devices) the gathers join that group.
namespace {
// One RCCL group of the plan's in-place all-gathers on stream st (the plan's device current).
int issue_gathers(lk_sharded_plan *p, hipStream_t st) {
    if (p->gathers.empty()) return LK_OK;
    NCCL_TRY(ncclGroupStart(), "ncclGroupStart");
    for (auto &g : p->gathers) {
      uint8_t *full = (uint8_t *)g.full;
      const ncclResult_t r = ncclAllGather(full + (uint64_t)p->comm->rank * g.chunk, full, g.chunk, ncclChar,
                                           p->comm->comm, st);
      if (r != ncclSuccess) {
        // part of this rank's gathers may be enqueued, waiting for peers: tear them down
        (void)ncclGroupEnd();
        (void)lk_comm_abort(p->comm);
        return failf(LK_ERR_DEVICE, "ncclAllGather", r);
      }
      p->comm->collectives++;
    }
    NCCL_TRY(ncclGroupEnd(), "ncclGroupEnd");
    return LK_OK;
}
}  // namespace

int lk_sharded_plan_launch(lk_sharded_plan *p, void *stream) {
  if (!p) return lk_detail_fail(LK_ERR_INVALID_ARG, "null sharded plan");
  hipStream_t st = (hipStream_t)stream;
  if (!p->comm->comm) return lk_detail_fail(LK_ERR_DEVICE, "sharded plan: its communicator was aborted");
  return on_device(p->comm->device, [&]() -> int {
    int rc = lk_plan_launch(p->local, stream);
    if (rc) return rc;
    return issue_gathers(p, st);
  });
}

// Throughput form (round 6): the local rows on `compute`, the all-gathers on `gather` behind an event
// of the local launch, so a caller issuing many independent plans overlaps plan i's exchange over xGMI
// with plan i + 1's rows. Both streams on the communicator's device; graph-capturable (the event makes
// `gather` part of a capture begun on `compute`; the caller joins it back before ending the capture).
int lk_sharded_plan_launch_split(lk_sharded_plan *p, void *compute, void *gather) {
  if (!p) return lk_detail_fail(LK_ERR_INVALID_ARG, "null sharded plan");
  if (!p->comm->comm) return lk_detail_fail(LK_ERR_DEVICE, "sharded plan: its communicator was aborted");
  return on_device(p->comm->device, [&]() -> int {
    if (!p->rows_done && hipEventCreateWithFlags(&p->rows_done, hipEventDisableTiming) != hipSuccess) {
      p->rows_done = nullptr;
      return lk_detail_fail(LK_ERR_DEVICE, "sharded plan: event");
    }
    int rc = lk_plan_launch(p->local, compute);
    if (rc) return rc;
    if (hipEventRecord(p->rows_done, (hipStream_t)compute) != hipSuccess ||
        hipStreamWaitEvent((hipStream_t)gather, p->rows_done, 0) != hipSuccess)
      return lk_detail_fail(LK_ERR_DEVICE, "sharded plan: stream hand-off");
    return issue_gathers(p, (hipStream_t)gather);
  });
}

int lk_sharded_plan_num_gathers(const lk_sharded_plan *p) { return p ? (int)p->gathers.size() : 0; }

void lk_sharded_plan_destroy(lk_sharded_plan *p) {
  if (!p) return;
  if (p->rows_done) (void)on_device(p->comm->device, [&] { (void)hipEventDestroy(p->rows_done); return 0; });
  if (p->local) lk_plan_destroy(p->local);
  delete p;
}

}  // extern "C"
