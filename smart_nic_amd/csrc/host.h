// host.h — host-side pieces shared by the launchers of libnicgpu.so: the
// per-device information (runtime.hip), the occupancy cache, HIP status
// mapping, a device guard, and the RSS context the RX and f1 launchers read.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "nicgpu.h"

namespace nicgpu_detail {

struct DeviceInfo {
  bool init = false;
  int status = 0;
  int cus = 0;
};

// gfx950 check and CU count of device `dev`, computed once.
const DeviceInfo& device_info(int dev);
// device_info of the calling thread's current device (NICGPU_OK or an error).
int current_device_info(const DeviceInfo** out);
// Blocks of `kernel` that fit one CU at `threads` per block and `lds` bytes of
// dynamic LDS on the current device (hipOccupancy..., cached; at least 1).
int blocks_per_cu(const void* kernel, int threads, uint32_t lds);

inline int hip_status(hipError_t e) { return e == hipSuccess ? NICGPU_OK : NICGPU_ERR_HIP; }

// nicgpu_checksum_batch_split over min(n_max, *n_dev) frames, the count read
// on the device (rx.hip; the f1 stage's asynchronous plan)
int checksum_split_count(const uint8_t* frames, const uint64_t* desc, size_t n_max, const uint64_t* n_dev,
                         uint16_t* out_rest, uint16_t* out_head4, void* stream);

// Makes `dev` current for the scope and restores the previous device.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void) hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

#ifdef NICGPU_TUNING
// tools/wave_stamps.py (nicgpu_tune_set_stamps): per-wave {start, end, XCC_ID, HW_ID}
extern unsigned long long* g_tune_stamps;
#endif

}  // namespace nicgpu_detail

// The RSS context of the C-ABI (rss.hip): key, LUT, table on one device.
struct nicgpu_rss_ctx {
  int device = 0;
  unsigned long long* d_rep = nullptr;  // kHistRep x kHistLds hit-histogram replicas (flush_hist), zeroed
  unsigned int* d_done = nullptr;       // their done ticket
  uint8_t* d_key = nullptr;             // NICGPU_MAX_KEY bytes
  uint32_t* d_lut = nullptr;            // kLutWords
  uint16_t* d_table = nullptr;          // capacity table_cap
  size_t table_cap = 0;
  size_t key_len = 0;
  size_t table_n = 0;
};
