// runtime.hip — device selection, HBM allocation, the library stream and
// HIP events, thread-local error text.  No kernels live here.
#include <atomic>
#include <cstdlib>
#include <cstring>
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

DevBuf::~DevBuf() {
  // Device buffers of a process-lifetime context are released by the
  // driver at exit; freeing here could run after the HIP runtime is gone.
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
    std::snprintf(buf, (size_t)buflen, "%s (%s, %d CUs)", prop.name,
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
