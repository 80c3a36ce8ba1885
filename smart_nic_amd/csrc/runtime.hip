// runtime.hip — the C-ABI's runtime entry points (devices, memory, streams,
// events) and the per-device information and occupancy cache the launchers
// share (host.h).

#include "host.h"

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

// Host windows this library registered (nicgpu_host_register): exactly the
// caller's range (no page extension: the runtime then keeps treating heap
// neighbours on the same pages as ordinary pageable memory), with a reference
// count so that several stages binding one HostMemory share one registration
// and only the last release unregisters it.
namespace {
struct Registration {
  uintptr_t lo, hi;  // [lo, hi) as registered
  uint8_t* alias;    // device address of lo
  unsigned refs;
};
std::mutex g_reg_mu;
std::vector<Registration> g_reg;
}  // namespace

extern "C" {

int nicgpu_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return NICGPU_OK;
  if (!dst || !src) return NICGPU_ERR_INVALID;
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
  const auto lo = reinterpret_cast<uintptr_t>(host_ptr), hi = lo + bytes;
  std::lock_guard<std::mutex> g(g_reg_mu);
  // inside a window this library registered: one more reference to it
  for (Registration& r : g_reg)
    if (lo >= r.lo && hi <= r.hi) {
      ++r.refs;
      *dev_alias = r.alias + (lo - r.lo);
      *owned = 1;
      return NICGPU_OK;
    }
  // registered or allocated page-locked by someone else: hipHostRegister would
  // succeed again on an identical range (it does not count registrations), and
  // this library's release would then unregister the owner's
  hipPointerAttribute_t pa{};
  const hipError_t q = hipPointerGetAttributes(&pa, host_ptr);
  (void) hipGetLastError();
  if (q == hipSuccess && pa.type == hipMemoryTypeHost) return NICGPU_ERR_INVALID;
  const hipError_t e = hipHostRegister(host_ptr, bytes, hipHostRegisterMapped);
  if (e != hipSuccess) {
    (void) hipGetLastError();  // not sticky for the caller's next call
    // registered by someone else (or overlapping a window of ours): its
    // lifetime is not ours to hold, so it is refused rather than adopted
    return e == hipErrorHostMemoryAlreadyRegistered ? NICGPU_ERR_INVALID : NICGPU_ERR_HIP;
  }
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, host_ptr, 0) != hipSuccess || dev == nullptr) {
    (void) hipGetLastError();
    (void) hipHostUnregister(host_ptr);
    return NICGPU_ERR_HIP;
  }
  g_reg.push_back({lo, hi, static_cast<uint8_t*>(dev), 1u});
  *dev_alias = dev;
  *owned = 1;
  return NICGPU_OK;
}

int nicgpu_host_unregister(void* host_ptr) {
  if (!host_ptr) return NICGPU_ERR_INVALID;
  const auto a = reinterpret_cast<uintptr_t>(host_ptr);
  std::lock_guard<std::mutex> g(g_reg_mu);
  // the registration starting at host_ptr, else the one holding it
  size_t k = g_reg.size();
  for (size_t i = 0; i < g_reg.size() && k == g_reg.size(); ++i)
    if (g_reg[i].lo == a) k = i;
  for (size_t i = 0; i < g_reg.size() && k == g_reg.size(); ++i)
    if (a >= g_reg[i].lo && a < g_reg[i].hi) k = i;
  if (k == g_reg.size()) return NICGPU_ERR_INVALID;  // not registered by this library
  if (--g_reg[k].refs != 0) return NICGPU_OK;
  void* base = reinterpret_cast<void*>(g_reg[k].lo);
  g_reg.erase(g_reg.begin() + (long) k);
  return hip_status(hipHostUnregister(base));
}

}  // extern "C"
