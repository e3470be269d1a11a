// runtime.hip — device selection, HBM allocation, the library stream and
// HIP events, thread-local error text.  No kernels live here.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <strings.h>

#include "pbx_common.h"

namespace pbx {

static thread_local std::string g_last_error;
static thread_local int g_thread_device = -1;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

void fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw Error{code, std::string(buf)};
}

void *DevBuf::ensure(size_t need) {
  if (need == 0) need = 16;
  if (need <= bytes) return ptr;
  if (ptr) {
    (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  // round up to 2 MiB so slowly growing calls do not re-allocate each time
  size_t want = (need + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
  PBX_HIP(hipMalloc(&ptr, want));
  bytes = want;
  return ptr;
}

// ---- caching allocator for the engines' grow-only buffers (Buf) --------
// A Buf's block goes back to a per-device cache when the buffer grows or its
// handle is destroyed, and the next Buf of about that size takes it instead
// of a hipMalloc (a handle per profile / BinsSet made every call allocate and
// free its ~30 buffers: hipMalloc maps pages, hipFree synchronises the
// device).  Every library kernel of a device runs on its one stream, so a
// block handed to a new owner is only touched by work queued after the old
// owner's.  Cached bytes per device are capped; a failed hipMalloc empties
// the cache and tries again.
namespace {
struct DevPool {
  std::mutex mu;
  std::multimap<size_t, void *> free;  // cached blocks by size
  size_t cached = 0;
  int64_t hits = 0, misses = 0;
};
DevPool g_pools[64];
constexpr size_t kPoolCap = (size_t)8 << 30;        // cached bytes per device
constexpr size_t kPoolMaxBlock = (size_t)2 << 30;   // larger blocks are freed
size_t pool_class(size_t need) {
  if (need <= 256) return 256;
  if (need <= ((size_t)1 << 20)) {
    size_t c = 512;
    while (c < need) c <<= 1;
    return c;
  }
  const size_t g = (size_t)2 << 20;  // 2 MiB granules
  return (need + g - 1) / g * g;
}
void pool_trim(DevPool &P) {
  std::lock_guard<std::mutex> lk(P.mu);
  for (auto &b : P.free) (void)hipFree(b.second);
  P.free.clear();
  P.cached = 0;
}
}  // namespace

void *dev_alloc(size_t need, size_t *got, int *dev_out) {
  int dev = 0;
  PBX_HIP(hipGetDevice(&dev));
  DevPool &P = g_pools[dev & 63];
  const size_t want = pool_class(need);
  *dev_out = dev;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.free.lower_bound(want);
    if (it != P.free.end() && it->first <= 2 * want) {  // (not a much larger block)
      void *p = it->second;
      *got = it->first;
      P.cached -= it->first;
      P.free.erase(it);
      ++P.hits;
#ifdef PBX_POOL_POISON  // test builds: a reused block holds garbage, not zeros
      // (on the device's stream: after the old owner's work, before the new one's)
      PBX_HIP(hipMemsetAsync(p, 0xA5, *got, current_device().stream));
#endif
      return p;
    }
  }
  void *p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) {
    (void)hipGetLastError();
    pool_trim(P);
    PBX_HIP(hipMalloc(&p, want));
  }
  {
    std::lock_guard<std::mutex> lk(P.mu);
    ++P.misses;
  }
  *got = want;
  return p;
}

void dev_release(void *p, size_t bytes, int dev) {
  if (!p) return;
  DevPool &P = g_pools[dev & 63];
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (bytes <= kPoolMaxBlock && P.cached + bytes <= kPoolCap) {
      P.free.emplace(bytes, p);
      P.cached += bytes;
      return;
    }
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  (void)hipFree(p);
  if (cur != dev) (void)hipSetDevice(cur);
}

DevBuf::~DevBuf() {
  // Device buffers of a process-lifetime context are released by the
  // driver at exit; freeing here could run after the HIP runtime is gone.
}

// ---- staged host <-> device copies (pbx_common.h) ---------------------
// A few persistent host threads split each chunk's memcpy; the pool is a
// leaked singleton (its threads block on a condition variable for the life
// of the process: no joinable std::thread is ever destroyed at exit).
namespace {
class CopyPool {
 public:
  static CopyPool &get() {
    static CopyPool *p = new CopyPool();
    return *p;
  }
  // dst[0 .. len) = src[0 .. len), split over the pool and the caller
  void copy(void *dst, const void *src, size_t len) { run(dst, src, len, false); }
  // int64 dst[0 .. n) = int32 src[0 .. n) (a widening copy-out)
  void widen(int64_t *dst, const int32_t *src, size_t n) { run(dst, src, n, true); }

 private:
  CopyPool() {
    unsigned hw = std::thread::hardware_concurrency();
    const int n = (int)std::max(1u, std::min(8u, hw ? hw / 2 : 1u));
    for (int i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  // len bytes (copy) or elements (widen); parts of a multiple of 64 bytes
  void run(void *dst, const void *src, size_t len, bool widen) {
    const int nt = (int)th_.size() + 1;
    if (len < ((size_t)1 << (widen ? 18 : 20)) || nt == 1) {
      widen_ = widen;
      dst_ = (char *)dst;
      src_ = (const char *)src;
      len_ = part_ = len;
      piece(0);
      return;
    }
    const size_t part = ((len + nt - 1) / nt + 63) & ~(size_t)63;
    {
      std::lock_guard<std::mutex> lk(m_);
      widen_ = widen;
      dst_ = (char *)dst;
      src_ = (const char *)src;
      len_ = len;
      part_ = part;
      pending_ = nt - 1;
      ++gen_;
    }
    cv_.notify_all();
    piece(0);  // the caller's share
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
  }
  void piece(int i) {
    const size_t a = (size_t)i * part_;
    if (a >= len_) return;
    const size_t m = std::min(part_, len_ - a);
    if (!widen_) {
      std::memcpy(dst_ + a, src_ + a, m);
      return;
    }
    int64_t *d = (int64_t *)dst_ + a;
    const int32_t *s = (const int32_t *)src_ + a;
    for (size_t j = 0; j < m; ++j) d[j] = s[j];
  }
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      piece(i);
      std::lock_guard<std::mutex> lk(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  char *dst_ = nullptr;
  const char *src_ = nullptr;
  size_t len_ = 0, part_ = 0;
  bool widen_ = false;
  int pending_ = 0;
  uint64_t gen_ = 0;
};

constexpr size_t kStageChunk = (size_t)16 << 20;  // bytes per pinned chunk
constexpr int kStageRing = 4;                     // chunks
constexpr size_t kStageMin = (size_t)8 << 20;     // smaller copies: plain hipMemcpyAsync

void ring_init(Device &d) {
  if (!d.ring.empty()) return;
  d.ring.assign(kStageRing, nullptr);
  d.ring_ev.assign(kStageRing, nullptr);
  d.ring_used.assign(kStageRing, false);
  for (int k = 0; k < kStageRing; ++k) {
    PBX_HIP(hipHostMalloc(&d.ring[k], kStageChunk, hipHostMallocDefault));
    PBX_HIP(hipEventCreateWithFlags(&d.ring_ev[k], hipEventDisableTiming));
  }
}
}  // namespace

void h2d_staged(Device &d, void *dst, const void *src, size_t bytes, hipStream_t st) {
  if (bytes < kStageMin) {
    PBX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    return;
  }
  ring_init(d);
  CopyPool &pool = CopyPool::get();
  size_t off = 0;
  for (int i = 0; off < bytes; ++i, off += kStageChunk) {
    const int k = i % kStageRing;
    const size_t len = std::min(kStageChunk, bytes - off);
    if (d.ring_used[k]) PBX_HIP(hipEventSynchronize(d.ring_ev[k]));  // its last DMA is done
    pool.copy(d.ring[k], (const char *)src + off, len);
    PBX_HIP(hipMemcpyAsync((char *)dst + off, d.ring[k], len, hipMemcpyHostToDevice, st));
    PBX_HIP(hipEventRecord(d.ring_ev[k], st));
    d.ring_used[k] = true;
  }
}

// (widen: src holds bytes / 4 int32 values, dst receives them as int64)
static void d2h_ring(Device &d, void *dst, const void *src, size_t bytes, hipStream_t st,
                     bool widen) {
  ring_init(d);
  CopyPool &pool = CopyPool::get();
  const int nc = (int)((bytes + kStageChunk - 1) / kStageChunk);
  // chunks in flight on the DMA engine while the host copies earlier ones out
  auto issue = [&](int i) {
    const int k = i % kStageRing;
    const size_t off = (size_t)i * kStageChunk, len = std::min(kStageChunk, bytes - off);
    if (d.ring_used[k]) PBX_HIP(hipEventSynchronize(d.ring_ev[k]));
    PBX_HIP(hipMemcpyAsync(d.ring[k], (const char *)src + off, len, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipEventRecord(d.ring_ev[k], st));
    d.ring_used[k] = true;
  };
  for (int i = 0; i < std::min(nc, kStageRing); ++i) issue(i);
  for (int i = 0; i < nc; ++i) {
    const int k = i % kStageRing;
    const size_t off = (size_t)i * kStageChunk, len = std::min(kStageChunk, bytes - off);
    PBX_HIP(hipEventSynchronize(d.ring_ev[k]));
    if (widen) pool.widen((int64_t *)dst + off / 4, (const int32_t *)d.ring[k], len / 4);
    else pool.copy((char *)dst + off, d.ring[k], len);
    d.ring_used[k] = false;  // (copied out: free for the next chunk)
    if (i + kStageRing < nc) issue(i + kStageRing);
  }
}

void d2h_staged(Device &d, void *dst, const void *src, size_t bytes, hipStream_t st) {
  if (bytes < kStageMin) {
    PBX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    return;
  }
  d2h_ring(d, dst, src, bytes, st, false);
}

bool d2h_staged_widen(Device &d, int64_t *dst, const int32_t *src, int64_t n, hipStream_t st) {
  if (sizeof(int32_t) * (size_t)n < kStageMin) return false;
  d2h_ring(d, dst, src, sizeof(int32_t) * (size_t)n, st, true);
  return true;
}

DevBuf &Device::slot(int k) {
  if ((int)slots.size() <= k) slots.resize(kSlotCount > k ? kSlotCount : k + 1, nullptr);
  if (!slots[k]) slots[k] = new DevBuf();
  return *slots[k];
}

static std::mutex g_devices_mu;
static std::vector<Device *> g_devices;

static int device_count_checked() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0)
    fail(PBX_ERR_NODEV,
         "no HIP device available (hipGetDeviceCount: %s); libpbx has no CPU "
         "fallback",
         e == hipSuccess ? "0 devices" : hipGetErrorString(e));
  return n;
}

Device &current_device() {
  int n = device_count_checked();
  int dev = g_thread_device;
  if (dev < 0) dev = 0;
  if (dev >= n) fail(PBX_ERR_VALUE, "device %d out of range (%d devices)", dev, n);
  std::lock_guard<std::mutex> lk(g_devices_mu);
  if ((int)g_devices.size() < n) g_devices.resize(n, nullptr);
  if (!g_devices[dev]) {
    PBX_HIP(hipSetDevice(dev));
    hipDeviceProp_t prop;
    PBX_HIP(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      fail(PBX_ERR_NODEV, "device %d is %s; libpbx is built for gfx950 only",
           dev, prop.gcnArchName);
    Device *d = new Device();
    d->id = dev;
    PBX_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    g_devices[dev] = d;
  }
  PBX_HIP(hipSetDevice(dev));
  return *g_devices[dev];
}

bool timing_enabled() {
  static int cached = -1;
  if (cached < 0) {
    const char *v = std::getenv("GRAVITY_TIMING");
    bool on = false;
    if (v) {
      std::string s(v);
      size_t a = s.find_first_not_of(" \t\n\r");
      size_t b = s.find_last_not_of(" \t\n\r");
      s = (a == std::string::npos) ? std::string() : s.substr(a, b - a + 1);
      on = !(s.empty() || s == "0" || strcasecmp(s.c_str(), "false") == 0);
    }
    cached = on ? 1 : 0;
  }
  return cached == 1;
}

static std::atomic<int> g_precise{-1};

bool precise_mode() {
  int v = g_precise.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = std::getenv("PBX_PRECISE");
    v = (e && e[0] && std::strcmp(e, "0") != 0) ? 1 : 0;
    int expect = -1;
    g_precise.compare_exchange_strong(expect, v);
    v = g_precise.load(std::memory_order_relaxed);
  }
  return v == 1;
}

void set_precise_mode(bool on) { g_precise.store(on ? 1 : 0, std::memory_order_relaxed); }

void set_thread_device(int d) { g_thread_device = d; }
int thread_device() { return g_thread_device < 0 ? 0 : g_thread_device; }

}  // namespace pbx

using namespace pbx;

extern "C" {

const char *pbx_last_error(void) { return g_last_error.c_str(); }

int pbx_version(void) { return 100; }

int pbx_device_count(int *count) {
  return guard([&] { *count = device_count_checked(); });
}

int pbx_set_device(int device) {
  return guard([&] {
    int n = device_count_checked();
    if (device < 0 || device >= n)
      fail(PBX_ERR_VALUE, "device %d out of range (%d devices)", device, n);
    set_thread_device(device);
    current_device();
  });
}

int pbx_get_device(int *device) {
  return guard([&] { *device = thread_device(); });
}

int pbx_set_precise(int on) {
  return guard([&] { set_precise_mode(on != 0); });
}

int pbx_get_precise(int *on) {
  return guard([&] { *on = precise_mode() ? 1 : 0; });
}

int pbx_device_synchronize(void) {
  return guard([&] {
    current_device();
    PBX_HIP(hipDeviceSynchronize());
  });
}

int pbx_device_name(char *buf, int buflen) {
  return guard([&] {
    Device &d = current_device();
    hipDeviceProp_t prop;
    PBX_HIP(hipGetDeviceProperties(&prop, d.id));
    // (the marketing name can be empty on some driver stacks)
    std::snprintf(buf, (size_t)buflen, "%s (%s, %d CUs)", prop.name[0] ? prop.name : "gfx950 device",
                  prop.gcnArchName, prop.multiProcessorCount);
  });
}

int pbx_malloc(void **d_ptr, size_t bytes) {
  return guard([&] {
    current_device();
    PBX_HIP(hipMalloc(d_ptr, bytes ? bytes : 16));
  });
}

int pbx_free(void *d_ptr) {
  return guard([&] {
    current_device();
    if (d_ptr) PBX_HIP(hipFree(d_ptr));
  });
}

int pbx_memcpy_htod(void *d_dst, const void *h_src, size_t bytes) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, d.stream));
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

int pbx_device_pool_stats(int64_t *out) {
  return guard([&] {
    if (!out) fail(PBX_ERR_VALUE, "null output");
    Device &d = current_device();
    DevPool &P = g_pools[d.id & 63];
    std::lock_guard<std::mutex> lk(P.mu);
    out[0] = (int64_t)P.cached;
    out[1] = (int64_t)P.free.size();
    out[2] = P.hits;
    out[3] = P.misses;
  });
}

int pbx_device_pool_trim(void) {
  return guard([&] {
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    PBX_HIP(hipStreamSynchronize(d.stream));
    pool_trim(g_pools[d.id & 63]);
  });
}

int pbx_measure_h2d(int64_t bytes, double *pinned_gbs, double *staged_gbs) {
  return guard([&] {
    if (bytes <= 0) fail(PBX_ERR_VALUE, "bytes must be > 0");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    const size_t nb = (size_t)bytes;
    void *dev = nullptr, *pin = nullptr;
    PBX_HIP(hipMalloc(&dev, nb));
    std::vector<char> pageable(nb, 1);  // (touched: resident pages)
    try {
      PBX_HIP(hipHostMalloc(&pin, nb, hipHostMallocDefault));
      std::memset(pin, 1, nb);
      auto best = [&](auto copy) {
        double t = 1e30;
        for (int r = 0; r < 4; ++r) {  // (the first one warms the path up)
          PBX_HIP(hipStreamSynchronize(d.stream));
          const auto t0 = std::chrono::steady_clock::now();
          copy();
          PBX_HIP(hipStreamSynchronize(d.stream));
          const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          if (r) t = std::min(t, s);
        }
        return (double)nb / t / 1e9;
      };
      if (pinned_gbs)
        *pinned_gbs = best([&] { PBX_HIP(hipMemcpyAsync(dev, pin, nb, hipMemcpyHostToDevice, d.stream)); });
      if (staged_gbs) *staged_gbs = best([&] { h2d_staged(d, dev, pageable.data(), nb, d.stream); });
    } catch (...) {
      if (pin) (void)hipHostFree(pin);
      (void)hipFree(dev);
      throw;
    }
    (void)hipHostFree(pin);
    (void)hipFree(dev);
  });
}

int pbx_memcpy_dtoh(void *h_dst, const void *d_src, size_t bytes) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, d.stream));
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

int pbx_memcpy_dtod(void *d_dst, const void *d_src, size_t bytes) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, d.stream));
  });
}

int pbx_memset(void *d_ptr, int value, size_t bytes) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipMemsetAsync(d_ptr, value, bytes, d.stream));
  });
}

int pbx_stream(void **stream) {
  return guard([&] { *stream = (void *)current_device().stream; });
}

int pbx_event_create(void **event) {
  return guard([&] {
    current_device();
    hipEvent_t e;
    PBX_HIP(hipEventCreate(&e));
    *event = (void *)e;
  });
}

int pbx_event_destroy(void *event) {
  return guard([&] { PBX_HIP(hipEventDestroy((hipEvent_t)event)); });
}

int pbx_event_record(void *event) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipEventRecord((hipEvent_t)event, d.stream));
  });
}

int pbx_event_elapsed_ms(void *start, void *stop, float *ms) {
  return guard([&] {
    PBX_HIP(hipEventSynchronize((hipEvent_t)stop));
    PBX_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  });
}

int pbx_stream_synchronize(void) {
  return guard([&] {
    Device &d = current_device();
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

}  // extern "C"
