// runtime.hip — the C-ABI's runtime entry points (devices, memory, streams,
// events) and the per-device information and occupancy cache the launchers
// share (host.h).

#include "host.h"

#include <atomic>
#include <cstring>
#include <mutex>
#include <vector>

namespace nicgpu_detail {

namespace {
std::mutex g_mu;
DeviceInfo g_dev[64];
struct OccKey {
  int dev;
  const void* kernel;
  int threads;
  uint32_t lds;
  int blocks;
};
std::vector<OccKey> g_occ;
}  // namespace

const DeviceInfo& device_info(int dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceInfo& di = g_dev[dev & 63];
  if (di.init) return di;
  di.init = true;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    di.status = NICGPU_ERR_HIP;
    return di;
  }
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    di.status = NICGPU_ERR_NO_DEVICE;
    return di;
  }
  di.cus = prop.multiProcessorCount;
  return di;
}

int current_device_info(const DeviceInfo** out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return NICGPU_ERR_NO_DEVICE;
  const DeviceInfo& di = device_info(dev);
  if (di.status != NICGPU_OK) return di.status;
  *out = &di;
  return NICGPU_OK;
}

int blocks_per_cu(const void* kernel, int threads, uint32_t lds) {
  int dev = 0;
  (void) hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  for (const auto& o : g_occ)
    if (o.dev == dev && o.kernel == kernel && o.threads == threads && o.lds == lds) return o.blocks;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, threads, lds) != hipSuccess || b < 1) b = 1;
  g_occ.push_back({dev, kernel, threads, lds, b});
  return b;
}

}  // namespace nicgpu_detail

using namespace nicgpu_detail;

extern "C" {

int nicgpu_abi_version(void) { return NICGPU_ABI_VERSION; }

const char* nicgpu_strerror(int status) {
  switch (status) {
    case NICGPU_OK: return "ok";
    case NICGPU_ERR_INVALID: return "invalid argument";
    case NICGPU_ERR_HIP: return "HIP runtime error";
    case NICGPU_ERR_NO_DEVICE: return "no gfx950 device";
    case NICGPU_ERR_NOMEM: return "out of device memory";
    case NICGPU_ERR_RANGE: return "batch too large for 32-bit piece indices";
    case NICGPU_ERR_AGAIN: return "plan outgrew its buffers: redo the batch";
    case NICGPU_ERR_UNSETTLED: return "segmented resolve did not settle: resolve per queue pair";
    default: return "unknown status";
  }
}

int nicgpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return NICGPU_ERR_NO_DEVICE;
  int count = 0;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++count;
  }
  return count;
}

int nicgpu_get_device(int* device) {
  if (!device) return NICGPU_ERR_INVALID;
  return hipGetDevice(device) == hipSuccess ? NICGPU_OK : NICGPU_ERR_NO_DEVICE;
}

int nicgpu_set_device(int device) { return hipSetDevice(device) == hipSuccess ? NICGPU_OK : NICGPU_ERR_NO_DEVICE; }

int nicgpu_malloc(void** dev_ptr, size_t bytes) {
  if (!dev_ptr) return NICGPU_ERR_INVALID;
  *dev_ptr = nullptr;
  if (bytes == 0) return NICGPU_OK;
  return hipMalloc(dev_ptr, bytes) == hipSuccess ? NICGPU_OK : NICGPU_ERR_NOMEM;
}

int nicgpu_free(void* dev_ptr) { return (!dev_ptr || hipFree(dev_ptr) == hipSuccess) ? NICGPU_OK : NICGPU_ERR_HIP; }

int nicgpu_host_alloc(void** host_ptr, size_t bytes) {
  if (!host_ptr) return NICGPU_ERR_INVALID;
  *host_ptr = nullptr;
  if (bytes == 0) return NICGPU_OK;
  return hipHostMalloc(host_ptr, bytes, hipHostMallocDefault) == hipSuccess ? NICGPU_OK : NICGPU_ERR_NOMEM;
}

int nicgpu_host_free(void* host_ptr) {
  return (!host_ptr || hipHostFree(host_ptr) == hipSuccess) ? NICGPU_OK : NICGPU_ERR_HIP;
}

int nicgpu_memset_async(void* dev_ptr, int value, size_t bytes, void* stream) {
  if (bytes == 0) return NICGPU_OK;
  if (!dev_ptr) return NICGPU_ERR_INVALID;
  return hip_status(hipMemsetAsync(dev_ptr, value, bytes, static_cast<hipStream_t>(stream)));
}

}  // extern "C"

// Whole pages around the range: hipHostRegister locks pages, and the staging
// kernels read up to the next 16-B boundary past the last byte.  The page
// ranges this library registered, for nicgpu_memcpy_async.
namespace {
constexpr uintptr_t kPage = 4096;
void page_span(void* p, size_t n, void*& base, size_t& len) {
  const auto a = reinterpret_cast<uintptr_t>(p);
  const uintptr_t lo = a & ~(kPage - 1), hi = (a + n + 16 + kPage - 1) & ~(kPage - 1);
  base = reinterpret_cast<void*>(lo);
  len = hi - lo;
}
std::mutex g_reg_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_reg;  // [base, end)
std::atomic<size_t> g_nreg{0};
// bytes of [p, p + n) before the end of a registered range p starts inside,
// when the range ends first; 0 otherwise
size_t registered_cut1(const void* p, size_t n) {
  const auto a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (const auto& r : g_reg)
    if (a >= r.first && a < r.second && a + n > r.second) return r.second - a;
  return 0;
}
size_t registered_cut(const void* dst, const void* src, size_t n) {
  if (g_nreg.load(std::memory_order_relaxed) == 0) return 0;
  const size_t a = registered_cut1(dst, n), b = registered_cut1(src, n);
  return a && b ? (a < b ? a : b) : (a ? a : b);
}
}  // namespace

extern "C" {

int nicgpu_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return NICGPU_OK;
  if (!dst || !src) return NICGPU_ERR_INVALID;
  // A host range that starts inside pages nicgpu_host_register locked and runs
  // past them (a heap neighbour of a HostMemory buffer that is not page
  // aligned) is not one allocation to the runtime: the copy is cut there.
  for (size_t cut; (cut = registered_cut(dst, src, bytes)) != 0 && cut < bytes;) {
    const int st = hip_status(hipMemcpyAsync(dst, src, cut, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
    if (st != NICGPU_OK) return st;
    dst = static_cast<uint8_t*>(dst) + cut;
    src = static_cast<const uint8_t*>(src) + cut;
    bytes -= cut;
  }
  return hip_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
}

int nicgpu_stream_synchronize(void* stream) {
  return hip_status(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

int nicgpu_stream_create(void** stream) {
  if (!stream) return NICGPU_ERR_INVALID;
  *stream = nullptr;
  hipStream_t s = nullptr;
  const int st = hip_status(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (st == NICGPU_OK) *stream = s;
  return st;
}

int nicgpu_stream_create_priority(void** stream, int low) {
  if (!stream) return NICGPU_ERR_INVALID;
  *stream = nullptr;
  int least = 0, greatest = 0;
  int st = hip_status(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t s = nullptr;
  if (st == NICGPU_OK) st = hip_status(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, low ? least : greatest));
  if (st == NICGPU_OK) *stream = s;
  return st;
}

int nicgpu_stream_destroy(void* stream) {
  if (!stream) return NICGPU_ERR_INVALID;
  return hip_status(hipStreamDestroy(static_cast<hipStream_t>(stream)));
}

int nicgpu_event_create(void** event) {
  if (!event) return NICGPU_ERR_INVALID;
  *event = nullptr;
  hipEvent_t e = nullptr;
  const int st = hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (st == NICGPU_OK) *event = e;
  return st;
}

int nicgpu_event_destroy(void* event) {
  if (!event) return NICGPU_ERR_INVALID;
  return hip_status(hipEventDestroy(static_cast<hipEvent_t>(event)));
}

int nicgpu_event_record(void* event, void* stream) {
  if (!event) return NICGPU_ERR_INVALID;
  return hip_status(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
}

int nicgpu_stream_wait_event(void* stream, void* event) {
  if (!event) return NICGPU_ERR_INVALID;
  return hip_status(hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(event), 0));
}

int nicgpu_event_synchronize(void* event) {
  if (!event) return NICGPU_ERR_INVALID;
  return hip_status(hipEventSynchronize(static_cast<hipEvent_t>(event)));
}



int nicgpu_host_register(void* host_ptr, size_t bytes, void** dev_alias, int* owned) {
  if (!host_ptr || !dev_alias || !owned || bytes == 0) return NICGPU_ERR_INVALID;
  *dev_alias = nullptr;
  *owned = 0;
  void* base = nullptr;
  size_t len = 0;
  page_span(host_ptr, bytes, base, len);
  const hipError_t e = hipHostRegister(base, len, hipHostRegisterMapped);
  if (e == hipSuccess) {
    *owned = 1;
    std::lock_guard<std::mutex> g(g_reg_mu);
    g_reg.emplace_back(reinterpret_cast<uintptr_t>(base), reinterpret_cast<uintptr_t>(base) + len);
    g_nreg.store(g_reg.size());
  }
  else if (e != hipErrorHostMemoryAlreadyRegistered) return NICGPU_ERR_HIP;
  (void) hipGetLastError();  // clear the sticky "already registered"
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
    if (*owned) (void) hipHostUnregister(base);
    *owned = 0;
    return NICGPU_ERR_HIP;
  }
  *dev_alias = static_cast<uint8_t*>(dev) + (reinterpret_cast<uintptr_t>(host_ptr) - reinterpret_cast<uintptr_t>(base));
  return NICGPU_OK;
}

int nicgpu_host_unregister(void* host_ptr) {
  if (!host_ptr) return NICGPU_ERR_INVALID;
  void* base = nullptr;
  size_t len = 0;
  page_span(host_ptr, 1, base, len);
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    for (size_t i = 0; i < g_reg.size(); ++i)
      if (g_reg[i].first == reinterpret_cast<uintptr_t>(base)) {
        g_reg.erase(g_reg.begin() + (long) i);
        break;
      }
    g_nreg.store(g_reg.size());
  }
  return hip_status(hipHostUnregister(base));
}

}  // extern "C"
