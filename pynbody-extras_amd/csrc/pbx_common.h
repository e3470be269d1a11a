// pbx_common.h — shared host-side plumbing of libpbx.so: status codes,
// thread-local error text, per-device context (stream, grow-only HBM
// workspace), GRAVITY_TIMING instrumentation.
//
// The timing switch mirrors the reference's GRAVITY_TIMING env variable
// (crates/pynbodyext-rust/src/gravity.rs:12-31): any value other than "",
// "0" or "false" prints "[pynbodyext-timing] <label>: <ms> ms" to stderr.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pbx.h"

namespace pbx {

void set_error(const char *fmt, ...);

// Error carrying a pbx status code; thrown inside the library, converted to
// a status at the extern "C" boundary by guard().
struct Error {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const char *fmt, ...);

#define PBX_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess)                                                    \
      ::pbx::fail(PBX_ERR_RUNTIME, "%s failed: %s (%s:%d)", #call,           \
                  hipGetErrorString(_e), __FILE__, __LINE__);                \
  } while (0)

// Run f() and translate exceptions into a status code + last-error text.
template <class F> int guard(F &&f) {
  try {
    f();
    return PBX_OK;
  } catch (const Error &e) {
    set_error("%s", e.msg.c_str());
    return e.code;
  } catch (const std::bad_alloc &) {
    set_error("host allocation failed");
    return PBX_ERR_RUNTIME;
  } catch (...) {
    set_error("unknown internal error");
    return PBX_ERR_RUNTIME;
  }
}

// A grow-only device buffer.  Host-array entry points reuse these across
// calls so a profile or gravity call does not pay hipMalloc each time.
struct DevBuf {
  void *ptr = nullptr;
  size_t bytes = 0;
  void *ensure(size_t need);
  ~DevBuf();
};

// Caching device allocator (runtime.hip) behind the engines' Buf: a block
// of at least `need` bytes (*got: its size, *dev: the current device), and
// its return to that device's cache (or hipFree when the cache is full).
void *dev_alloc(size_t need, size_t *got, int *dev);
void dev_release(void *p, size_t bytes, int dev);

// Per-device state.  All library kernels of a device run on `stream`.
struct Device {
  int id = -1;
  hipStream_t stream = nullptr;
  std::mutex mu;                      // serialises host-array entry points
  std::vector<DevBuf *> slots;        // workspace slots, indexed by enum
  DevBuf &slot(int k);
  // h2d_staged / d2h_staged: pinned chunks and the events of their last DMA
  std::vector<void *> ring;
  std::vector<hipEvent_t> ring_ev;
  std::vector<bool> ring_used;
};

// Workspace slot ids (one namespace for every module).
enum Slot {
  kSlotSrc = 0,
  kSlotSrcH,
  kSlotTgt,
  kSlotTgtH,
  kSlotPos,
  kSlotMass,
  kSlotPot,
  kSlotAcc,
  kSlotPart,
  kSlotProf0,
  kSlotProf1,
  kSlotProf2,
  kSlotProf3,
  kSlotProf4,
  kSlotProf5,
  kSlotProf6,
  kSlotProf7,
  kSlotComm,
  kSlotSymRec,
  kSlotSymAcc,
  kSlotSymUnits,
  kSlotCount
};

// Device of the calling thread (initialised on first use; fails with
// PBX_ERR_NODEV when there is no GPU).
Device &current_device();

// Copies between PAGEABLE host memory and the device through a ring of
// pinned chunks: a few host threads memcpy chunk i + 1 while the DMA engine
// moves chunk i (a pageable hipMemcpy stages through the runtime's own
// buffers one copy at a time).  Queued on `st`; h2d_staged returns once the
// last chunk's DMA is queued (the source may be reused then), d2h_staged
// once the data is in `dst`.  Small copies take a plain hipMemcpyAsync.
// The caller holds the device's lock (the ring is per device).
void h2d_staged(Device &d, void *dst, const void *src, size_t bytes, hipStream_t st);
void d2h_staged(Device &d, void *dst, const void *src, size_t bytes, hipStream_t st);
// int32 values on the device -> int64 on the host (half the bytes cross PCIe;
// the host threads widen them on the way out of the pinned chunks).  False
// (nothing done) below the staging size: the caller widens on the device.
bool d2h_staged_widen(Device &d, int64_t *dst, const int32_t *src, int64_t n, hipStream_t st);

bool timing_enabled();

struct ScopedTimer {
  const char *label;
  std::chrono::steady_clock::time_point t0;
  bool on;
  explicit ScopedTimer(const char *l)
      : label(l), t0(std::chrono::steady_clock::now()), on(timing_enabled()) {}
  ~ScopedTimer() {
    if (on) {
      double ms = std::chrono::duration<double, std::milli>(
                      std::chrono::steady_clock::now() - t0)
                      .count();
      std::fprintf(stderr, "[pynbodyext-timing] %s: %.3f ms\n", label, ms);
    }
  }
};

// Collectives a device pipeline issues on the library stream between its
// kernels, without a host round trip (comm.hip, RCCL).  `comm` is a
// pbx_comm_init handle; comm_ranks validates it for the calling thread's
// device and returns {nranks, rank}; dtype / op are pbx_comm_allreduce's
// codes (dtype 0 f64, 1 i64, 2 u64, 3 u32; op 0 sum, 1 min, 2 max).
struct CommRanks {
  int nranks, rank;
};
// `lk` is the caller's hold on the device's lock: with a host-transport
// communicator (pbx_comm_init_host) comm_allreduce releases it while the
// transport waits for the other ranks — they may be threads of this process
// driving the same device — and takes it back before returning.  So another
// library call can run on this device and stream in that window: a pipeline
// that issues comm_allreduce must keep its state in its own (per-handle)
// buffers, never in workspace another call may use (Device::slot()), across
// the collective.  (radial_equaln, the one such pipeline, keeps all of it in
// its Profile.)
CommRanks comm_ranks(void *comm);
void comm_allreduce(void *comm, const void *send, void *recv, int64_t count, int dtype, int op,
                    hipStream_t st, std::unique_lock<std::mutex> &lk);

// Direct-sum precision mode (pbx_set_precise): true -> Newton-refined
// 1/sqrt everywhere (~1e-16); false (default, or PBX_PRECISE=0) -> the
// all-particles symmetric kernel uses v_rsq_f64 unrefined (~5e-8).
bool precise_mode();
void set_precise_mode(bool on);

inline unsigned int ceil_div(int64_t a, int64_t b) {
  return (unsigned int)((a + b - 1) / b);
}

// XCD-aware block order (a speed hint only: correctness never depends on
// placement).  The dispatcher is observed to deal workgroups round-robin
// over the 8 XCDs, each with its own L2; this bijection hands every XCD one
// contiguous run of logical blocks, so neighbouring blocks (spatially
// adjacent targets) share an L2 instead of being spread over all eight.
constexpr unsigned kNumXcd = 8;
__device__ __forceinline__ unsigned xcd_swizzle(unsigned b, unsigned nblocks) {
  const unsigned q = nblocks / kNumXcd, r = nblocks % kNumXcd;
  const unsigned x = b % kNumXcd, k = b / kNumXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}
// The same with the grid cut into rounds of kNumXcd chunks of `chunk`
// logical blocks: every XCD works through contiguous chunks, and the XCDs
// still advance over the grid together (uneven per-block cost stays
// balanced).  nblocks must be a multiple of kNumXcd * chunk.
__device__ __forceinline__ unsigned xcd_chunk_swizzle(unsigned b, unsigned chunk) {
  const unsigned x = b % kNumXcd, k = b / kNumXcd;
  return ((k / chunk) * kNumXcd + x) * chunk + k % chunk;
}

}  // namespace pbx
