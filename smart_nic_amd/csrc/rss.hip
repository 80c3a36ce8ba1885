// rss.hip — the RSS context of the C-ABI (nicgpu_rss_ctx): the Toeplitz key,
// its nibble LUT of 32-bit key windows built on the device, and the
// indirection table (nic::RssEngine's RssConfig, src/rss.cpp:17-41, 96-114).

#include "common.h"
#include "host.h"

#include <vector>

using namespace nicgpu_detail;

namespace {

const uint8_t kDefaultKey[20] = {0x6D, 0x5A, 0x56, 0x6B, 0x65, 0x4E, 0x67, 0x6E, 0x67, 0x55,
                                 0x6A, 0x6B, 0x61, 0x4F, 0x6B, 0x65, 0x6F, 0x49, 0x4D, 0x42};

// -------------------------------------------------------------- LUT build --
// lut[p*16 + v] = XOR over bits of nibble v (MSB first) of the 32-bit key window
// starting at key bit (4p + i) mod key_bits: exactly the windows the reference
// XORs for each set data bit (src/rss.cpp:74-91).
__global__ void build_lut_kernel(const uint8_t* __restrict__ key, uint32_t key_len,
                                 uint32_t* __restrict__ lut) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= kLutWords) return;
  int p = idx >> 4, v = idx & 15;
  uint32_t kb = key_len * 8u;
  uint32_t acc = 0;
  for (int i = 0; i < 4; ++i) {
    if (!((v >> (3 - i)) & 1)) continue;
    uint32_t b0 = (uint32_t) (4 * p + i) % kb;
    uint32_t w = 0;
    for (uint32_t k = 0; k < 32; ++k) {
      uint32_t kbit = (b0 + k) % kb;
      w = (w << 1) | ((key[kbit >> 3] >> (7 - (kbit & 7))) & 1u);
    }
    acc ^= w;
  }
  lut[idx] = acc;
}

int launch_build_lut(nicgpu_rss_ctx* ctx, hipStream_t s) {
  hipLaunchKernelGGL(build_lut_kernel, dim3((kLutWords + 255) / 256), dim3(256), 0, s, ctx->d_key,
                     (uint32_t) ctx->key_len, ctx->d_lut);
  return hip_status(hipGetLastError());
}

int ensure_table(nicgpu_rss_ctx* ctx, size_t n) {
  if (n <= ctx->table_cap) return NICGPU_OK;
  if (ctx->d_table) (void) hipFree(ctx->d_table);
  ctx->d_table = nullptr;
  ctx->table_cap = 0;
  if (hipMalloc(&ctx->d_table, n * sizeof(uint16_t)) != hipSuccess) return NICGPU_ERR_NOMEM;
  ctx->table_cap = n;
  return NICGPU_OK;
}

}  // namespace

extern "C" {

int nicgpu_rss_create(nicgpu_rss_ctx** out, int device) {
  if (!out) return NICGPU_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NICGPU_ERR_NO_DEVICE;
  DeviceGuard g(device);
  const DeviceInfo& di = device_info(device);
  if (di.status != NICGPU_OK) return di.status;
  auto* ctx = new nicgpu_rss_ctx();
  ctx->device = device;
  const size_t rep_bytes = (size_t) kHistRep * kHistLdsMax * sizeof(unsigned long long);
  if (hipMalloc(&ctx->d_key, NICGPU_MAX_KEY) != hipSuccess || hipMalloc(&ctx->d_lut, kLutWords * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&ctx->d_rep, rep_bytes + 256) != hipSuccess) {
    nicgpu_rss_destroy(ctx);
    return NICGPU_ERR_NOMEM;
  }
  ctx->d_done = reinterpret_cast<unsigned int*>(reinterpret_cast<uint8_t*>(ctx->d_rep) + rep_bytes);
  if (hipMemset(ctx->d_rep, 0, rep_bytes + 256) != hipSuccess) {
    nicgpu_rss_destroy(ctx);
    return NICGPU_ERR_HIP;
  }
  // reference defaults (src/rss.cpp:96-108): 20-B key, 128 zeros
  int st = nicgpu_rss_set_key(ctx, nullptr, 0, nullptr);
  if (st == NICGPU_OK) st = nicgpu_rss_set_table(ctx, nullptr, 0, nullptr);
  if (st == NICGPU_OK) st = hip_status(hipDeviceSynchronize());
  if (st != NICGPU_OK) {
    nicgpu_rss_destroy(ctx);
    return st;
  }
  *out = ctx;
  return NICGPU_OK;
}

int nicgpu_rss_destroy(nicgpu_rss_ctx* ctx) {
  if (!ctx) return NICGPU_ERR_INVALID;
  DeviceGuard g(ctx->device);
  if (ctx->d_key) (void) hipFree(ctx->d_key);
  if (ctx->d_lut) (void) hipFree(ctx->d_lut);
  if (ctx->d_table) (void) hipFree(ctx->d_table);
  if (ctx->d_rep) (void) hipFree(ctx->d_rep);
  delete ctx;
  return NICGPU_OK;
}

int nicgpu_rss_set_key(nicgpu_rss_ctx* ctx, const uint8_t* key, size_t len, void* stream) {
  if (!ctx || len > NICGPU_MAX_KEY || (len > 0 && !key)) return NICGPU_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint8_t* src = len ? key : kDefaultKey;
  size_t n = len ? len : sizeof(kDefaultKey);
  // synchronous w.r.t. the host buffer (pageable memcpy), ordered on `stream`
  if (hipMemcpyAsync(ctx->d_key, src, n, hipMemcpyHostToDevice, s) != hipSuccess) return NICGPU_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return NICGPU_ERR_HIP;
  ctx->key_len = n;
  return launch_build_lut(ctx, s);
}

int nicgpu_rss_set_key_device(nicgpu_rss_ctx* ctx, const uint8_t* key_dev, size_t len, void* stream) {
  if (!ctx || len > NICGPU_MAX_KEY || (len > 0 && !key_dev)) return NICGPU_ERR_INVALID;
  if (len == 0) return nicgpu_rss_set_key(ctx, nullptr, 0, stream);
  DeviceGuard g(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(ctx->d_key, key_dev, len, hipMemcpyDeviceToDevice, s) != hipSuccess) return NICGPU_ERR_HIP;
  ctx->key_len = len;
  return launch_build_lut(ctx, s);
}

int nicgpu_rss_set_table(nicgpu_rss_ctx* ctx, const uint16_t* table, size_t n, void* stream) {
  if (!ctx || n > NICGPU_MAX_TABLE || (n > 0 && !table)) return NICGPU_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<uint16_t> def;
  if (n == 0) {
    def.assign(128, 0);
    table = def.data();
    n = def.size();
  }
  int st = ensure_table(ctx, n);
  if (st != NICGPU_OK) return st;
  if (hipMemcpyAsync(ctx->d_table, table, n * sizeof(uint16_t), hipMemcpyHostToDevice, s) != hipSuccess) return NICGPU_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return NICGPU_ERR_HIP;
  ctx->table_n = n;
  return NICGPU_OK;
}

int nicgpu_rss_set_table_device(nicgpu_rss_ctx* ctx, const uint16_t* table_dev, size_t n, void* stream) {
  if (!ctx || n > NICGPU_MAX_TABLE || (n > 0 && !table_dev)) return NICGPU_ERR_INVALID;
  if (n == 0) return nicgpu_rss_set_table(ctx, nullptr, 0, stream);
  DeviceGuard g(ctx->device);
  int st = ensure_table(ctx, n);
  if (st != NICGPU_OK) return st;
  if (hipMemcpyAsync(ctx->d_table, table_dev, n * sizeof(uint16_t), hipMemcpyDeviceToDevice,
                     static_cast<hipStream_t>(stream)) != hipSuccess)
    return NICGPU_ERR_HIP;
  ctx->table_n = n;
  return NICGPU_OK;
}

int nicgpu_rss_info(const nicgpu_rss_ctx* ctx, size_t* key_len, size_t* table_n) {
  if (!ctx) return NICGPU_ERR_INVALID;
  if (key_len) *key_len = ctx->key_len;
  if (table_n) *table_n = ctx->table_n;
  return NICGPU_OK;
}

}  // extern "C"
