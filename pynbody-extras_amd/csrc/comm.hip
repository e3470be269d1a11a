// comm.hip — RCCL communicator of libpbx.so (one process per GPU, xGMI).
//
// The reference has no distributed backend (rayon threads only,
// SURVEY.md §2); this is the MI355X multi-GPU layer of the north star:
// the direct-sum solve shards TARGETS across ranks and all-gathers the
// 32-byte SOURCE records (pbx_comm_allgatherv: one ncclBroadcast per
// root inside an ncclGroup, so shards may be uneven), and per-bin profile
// partials are summed with pbx_comm_allreduce_*.
// All collectives run on the library stream of the calling thread's device.
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "pbx_common.h"

namespace pbx {

#define PBX_NCCL(call)                                                             \
  do {                                                                             \
    ncclResult_t _r = (call);                                                      \
    if (_r != ncclSuccess)                                                         \
      ::pbx::fail(PBX_ERR_RUNTIME, "%s failed: %s", #call, ncclGetErrorString(_r)); \
  } while (0)

struct Comm {
  ncclComm_t nccl = nullptr;
  // host transport (pbx_comm_init_host) instead of RCCL
  pbx_host_collective_fn host = nullptr;
  void *host_ctx = nullptr;
  int nranks = 0;
  int rank = 0;
  int device = -1;
  // persistent staging of pbx_comm_allreduce_host (HBM + pinned host),
  // grown on demand: no allocation per call
  void *dstage = nullptr, *hstage = nullptr;
  size_t stage_bytes = 0;
};

static size_t dtype_size(int dtype) { return dtype == 3 ? 4 : 8; }

static const ncclDataType_t kTypes[] = {ncclFloat64, ncclInt64, ncclUint64, ncclUint32};
static const ncclRedOp_t kOps[] = {ncclSum, ncclMin, ncclMax};

static Comm *as_comm(void *comm) {
  Comm *c = (Comm *)comm;
  if (!c) fail(PBX_ERR_VALUE, "null communicator");
  return c;
}

static Device &comm_device(Comm *c) {
  Device &d = current_device();
  if (d.id != c->device) fail(PBX_ERR_VALUE, "communicator belongs to device %d", c->device);
  return d;
}

static void check_codes(int dtype, int op) {
  if (dtype < 0 || dtype > 3) fail(PBX_ERR_VALUE, "bad dtype %d", dtype);
  if (op < 0 || op > 2) fail(PBX_ERR_VALUE, "bad reduction op %d", op);
}

// The communicator's pinned host staging, grown on demand (with its HBM twin
// for pbx_comm_allreduce_host).
static void *host_stage(Comm *c, size_t bytes) {
  if (bytes > c->stage_bytes) {
    if (c->dstage) (void)hipFree(c->dstage);
    if (c->hstage) (void)hipHostFree(c->hstage);
    c->dstage = c->hstage = nullptr;
    c->stage_bytes = 0;
    const size_t want = bytes < 65536 ? 65536 : bytes;
    PBX_HIP(hipMalloc(&c->dstage, want));
    PBX_HIP(hipHostMalloc(&c->hstage, want, hipHostMallocDefault));
    c->stage_bytes = want;
  }
  return c->hstage;
}

// Call the host transport.  `lk`: the caller's hold on the device lock d.mu
// (a library pipeline issuing a collective between its kernels), or null;
// it is released while the transport waits for the other ranks, which may be
// threads of this process driving the same device (pbx_common.h states what
// such a pipeline may not keep across the wait).
static void host_call(Comm *c, std::unique_lock<std::mutex> *lk, int kind, void *h, int64_t count,
                      int dtype, int op, const int64_t *counts, const int64_t *displs) {
  if (lk) lk->unlock();
  const int r = c->host(c->host_ctx, kind, h, count, dtype, op, counts, displs);
  if (lk) lk->lock();
  if (r != 0) fail(PBX_ERR_RUNTIME, "host collective (kind %d, rank %d of %d) failed: %d", kind,
                   c->rank, c->nranks, r);
}

// Device all-reduce through the host transport: D2H, transport, H2D, each
// step drained (the staging is reused by the next collective).
static void host_allreduce_dev(Comm *c, Device &d, std::unique_lock<std::mutex> *lk,
                               const void *send, void *recv, int64_t count, int dtype, int op) {
  const size_t bytes = dtype_size(dtype) * (size_t)count;
  void *h = host_stage(c, bytes);
  PBX_HIP(hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, d.stream));
  PBX_HIP(hipStreamSynchronize(d.stream));
  host_call(c, lk, PBX_COLL_ALLREDUCE, h, count, dtype, op, nullptr, nullptr);
  PBX_HIP(hipMemcpyAsync(recv, h, bytes, hipMemcpyHostToDevice, d.stream));
  PBX_HIP(hipStreamSynchronize(d.stream));
}

CommRanks comm_ranks(void *comm) {
  Comm *c = as_comm(comm);
  comm_device(c);
  return CommRanks{c->nranks, c->rank};
}

// (called by library pipelines that hold the device lock: `lk`)
void comm_allreduce(void *comm, const void *send, void *recv, int64_t count, int dtype, int op,
                    hipStream_t st, std::unique_lock<std::mutex> &lk) {
  Comm *c = as_comm(comm);
  check_codes(dtype, op);
  if (count <= 0) return;
  if (c->host) {
    if (!lk.owns_lock() || lk.mutex() != &comm_device(c).mu)
      fail(PBX_ERR_RUNTIME, "comm_allreduce: the caller does not hold the device lock");
    host_allreduce_dev(c, comm_device(c), &lk, send, recv, count, dtype, op);
    return;
  }
  PBX_NCCL(ncclAllReduce(send, recv, (size_t)count, kTypes[dtype], kOps[op], c->nccl, st));
}

}  // namespace pbx

using namespace pbx;

extern "C" {

int pbx_comm_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

int pbx_comm_unique_id(unsigned char *buf, int buflen) {
  return guard([&] {
    if (buflen < (int)sizeof(ncclUniqueId))
      fail(PBX_ERR_VALUE, "unique id buffer needs %d bytes", (int)sizeof(ncclUniqueId));
    ncclUniqueId id;
    PBX_NCCL(ncclGetUniqueId(&id));
    std::memcpy(buf, &id, sizeof(id));
  });
}

int pbx_comm_init(void **comm, int nranks, int rank, const unsigned char *uid) {
  return guard([&] {
    if (nranks < 1 || rank < 0 || rank >= nranks)
      fail(PBX_ERR_VALUE, "bad rank %d / nranks %d", rank, nranks);
    Device &d = current_device();
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    Comm *c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = d.id;
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, id, rank);
    if (r != ncclSuccess) {
      delete c;
      fail(PBX_ERR_RUNTIME, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
    }
    *comm = c;
  });
}

int pbx_comm_init_host(void **comm, int nranks, int rank, pbx_host_collective_fn fn, void *ctx) {
  return guard([&] {
    if (nranks < 1 || rank < 0 || rank >= nranks)
      fail(PBX_ERR_VALUE, "bad rank %d / nranks %d", rank, nranks);
    if (!fn) fail(PBX_ERR_VALUE, "null host collective");
    Device &d = current_device();
    Comm *c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = d.id;
    c->host = fn;
    c->host_ctx = ctx;
    *comm = c;
  });
}

int pbx_comm_destroy(void *comm) {
  return guard([&] {
    Comm *c = (Comm *)comm;
    if (!c) return;
    if (c->nccl) PBX_NCCL(ncclCommDestroy(c->nccl));
    if (c->dstage) (void)hipFree(c->dstage);
    if (c->hstage) (void)hipHostFree(c->hstage);
    delete c;
  });
}

// d_buf holds every rank's segment; segment r occupies
// [displs[r], displs[r] + counts[r]) bytes and this rank's segment is
// already in place.  Afterwards every rank holds all segments.
int pbx_comm_allgatherv(void *comm, void *d_buf, const int64_t *counts, const int64_t *displs) {
  return guard([&] {
    Comm *c = as_comm(comm);
    Device &d = comm_device(c);
    char *base = (char *)d_buf;
    if (c->host) {  // the whole span through host staging
      int64_t lo = INT64_MAX, hi = 0;
      for (int r = 0; r < c->nranks; ++r) {
        if (counts[r] < 0 || displs[r] < 0) fail(PBX_ERR_VALUE, "negative segment");
        if (counts[r] == 0) continue;
        lo = std::min(lo, displs[r]);
        hi = std::max(hi, displs[r] + counts[r]);
      }
      if (hi == 0) return;
      std::vector<int64_t> dl(displs, displs + c->nranks);
      for (auto &v : dl) v -= lo;
      char *h = (char *)host_stage(c, (size_t)(hi - lo));
      PBX_HIP(hipMemcpyAsync(h, base + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, d.stream));
      PBX_HIP(hipStreamSynchronize(d.stream));
      host_call(c, nullptr, PBX_COLL_ALLGATHERV, h, c->nranks, 0, 0, counts, dl.data());
      PBX_HIP(hipMemcpyAsync(base + lo, h, (size_t)(hi - lo), hipMemcpyHostToDevice, d.stream));
      PBX_HIP(hipStreamSynchronize(d.stream));
      return;
    }
    PBX_NCCL(ncclGroupStart());
    for (int r = 0; r < c->nranks; ++r) {
      if (counts[r] <= 0) continue;
      PBX_NCCL(ncclBroadcast(base + displs[r], base + displs[r], (size_t)counts[r], ncclChar, r,
                             c->nccl, d.stream));
    }
    PBX_NCCL(ncclGroupEnd());
  });
}

// Generic all-reduce on the library stream.  dtype: 0 f64, 1 i64, 2 u64,
// 3 u32; op: 0 sum, 1 min, 2 max (e.g. the u32 digit histograms and the u64
// key range of the distributed equaln).
static void allreduce_dev(void *comm, const void *d_send, void *d_recv, int64_t count, int dtype,
                          int op) {
  Comm *c = as_comm(comm);
  check_codes(dtype, op);
  if (count < 0) fail(PBX_ERR_VALUE, "negative count");
  Device &d = comm_device(c);
  if (c->host) {
    if (count) host_allreduce_dev(c, d, nullptr, d_send, d_recv, count, dtype, op);
    return;
  }
  PBX_NCCL(ncclAllReduce(d_send, d_recv, (size_t)count, kTypes[dtype], kOps[op], c->nccl, d.stream));
}

int pbx_comm_allreduce(void *comm, const void *d_send, void *d_recv, int64_t count, int dtype,
                       int op) {
  return guard([&] { allreduce_dev(comm, d_send, d_recv, count, dtype, op); });
}

int pbx_comm_allreduce_f64(void *comm, const double *d_send, double *d_recv, int64_t count) {
  return guard([&] { allreduce_dev(comm, d_send, d_recv, count, 0, 0); });
}

int pbx_comm_allreduce_i64(void *comm, const int64_t *d_send, int64_t *d_recv, int64_t count) {
  return guard([&] { allreduce_dev(comm, d_send, d_recv, count, 1, 0); });
}

// All-reduce of a small host array in place (dtype / op as above): one H2D,
// the collective and one D2H on the library stream through the
// communicator's persistent staging, one stream sync (host transport: the
// transport on the caller's array).
static void allreduce_host(Comm *c, void *h_buf, int64_t count, int dtype, int op) {
  check_codes(dtype, op);
  if (count < 0) fail(PBX_ERR_VALUE, "negative count");
  Device &d = comm_device(c);
  const size_t bytes = dtype_size(dtype) * (size_t)count;
  if (bytes == 0) return;
  if (c->host) {
    host_call(c, nullptr, PBX_COLL_ALLREDUCE, h_buf, count, dtype, op, nullptr, nullptr);
    return;
  }
  host_stage(c, bytes);
  std::memcpy(c->hstage, h_buf, bytes);
  PBX_HIP(hipMemcpyAsync(c->dstage, c->hstage, bytes, hipMemcpyHostToDevice, d.stream));
  PBX_NCCL(ncclAllReduce(c->dstage, c->dstage, (size_t)count, kTypes[dtype], kOps[op], c->nccl,
                         d.stream));
  PBX_HIP(hipMemcpyAsync(c->hstage, c->dstage, bytes, hipMemcpyDeviceToHost, d.stream));
  PBX_HIP(hipStreamSynchronize(d.stream));
  std::memcpy(h_buf, c->hstage, bytes);
}

int pbx_comm_allreduce_host(void *comm, void *h_buf, int64_t count, int dtype, int op) {
  return guard([&] { allreduce_host(as_comm(comm), h_buf, count, dtype, op); });
}

// Control-plane helpers on the data-plane communicator: a device barrier
// (1-element all-reduce + stream sync) and max-over-ranks of a host scalar.
int pbx_comm_barrier(void *comm) {
  return guard([&] {
    Comm *c = as_comm(comm);
    Device &d = comm_device(c);
    if (c->host) {
      PBX_HIP(hipStreamSynchronize(d.stream));
      int64_t one = 1;
      allreduce_host(c, &one, 1, 1, 0);
      return;
    }
    int64_t *buf = (int64_t *)d.slot(kSlotComm).ensure(64);
    PBX_NCCL(ncclAllReduce(buf, buf, 1, ncclInt64, ncclSum, c->nccl, d.stream));
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

int pbx_comm_max_f64(void *comm, double value, double *out) {
  return guard([&] {
    Comm *c = as_comm(comm);
    Device &d = comm_device(c);
    if (c->host) {
      double v = value;
      allreduce_host(c, &v, 1, 0, 2);
      *out = v;
      return;
    }
    double *buf = (double *)d.slot(kSlotComm).ensure(64);
    PBX_HIP(hipMemcpyAsync(buf, &value, sizeof(double), hipMemcpyHostToDevice, d.stream));
    PBX_NCCL(ncclAllReduce(buf, buf, 1, ncclFloat64, ncclMax, c->nccl, d.stream));
    PBX_HIP(hipMemcpyAsync(out, buf, sizeof(double), hipMemcpyDeviceToHost, d.stream));
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

}  // extern "C"
