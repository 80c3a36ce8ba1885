// image.hip — host-image staging for the batched QueuePair stage (SURVEY §8
// row f1) on the reference's HostMemory (include/nic/host_memory.h:49-73):
// the TX buffers' bytes from the registered host window into the HBM mirror
// before a batch (QueuePair's DMA read, src/queue_pair.cpp:86-92), and the
// bytes the batch's DMA writes delivered from the mirror back into the host
// window after it (:416-426).  Both are byte-exact copies between two images
// of the same memory at the same offsets: 16-B chunks aligned to the image
// offsets, one 16-B load and store per whole chunk, byte stores for the bytes
// of an edge chunk that lie inside the range, so no byte outside the range is
// ever stored to (the host bytes past a frame are the application's).
// One wave per range, a persistent grid walking the ranges; the host side is
// PCIe-bound (≈ 50 GB/s each way), so the kernels only need enough bytes in
// flight: every wave has one 1-KiB chunk step of its range outstanding.

#include <cstdlib>
#include "common.h"
#include "host.h"
#include "qp_logic.h"

using namespace nicgpu_detail;

namespace {

constexpr unsigned kImgWaves = 4;

// dst[a, a + len) <- src[a, a + len), lanes over the 16-B chunks; no byte of
// src at or past `limit` (the window's size) is read: the chunk holding the
// window's end is read byte by byte (a registered host window ends exactly
// there, and the bytes after it are other heap blocks').
__device__ __forceinline__ void copy_range(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t a,
                                           uint64_t len, uint64_t limit, uint32_t lane) {
  const uint64_t e = a + len;
  const uint64_t c1 = (e + 15) & ~15ull;
  for (uint64_t c = (a & ~15ull) + 16ull * lane; c < c1; c += 16ull * kWave) {
    u32x4 v;
    if (c + 16 <= limit) {
      __builtin_memcpy(&v, src + c, 16);
    } else {
      uint8_t t[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) t[k] = c + k < limit ? src[c + k] : (uint8_t) 0;
      __builtin_memcpy(&v, t, 16);
    }
    if (c >= a && c + 16 <= e) {
      __builtin_memcpy(dst + c, &v, 16);
    } else {
      uint8_t b[16];
      __builtin_memcpy(b, &v, 16);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (c + k >= a && c + k < e) dst[c + k] = b[k];
    }
  }
}

__global__ __launch_bounds__(kWave * kImgWaves) void image_stage_kernel(uint8_t* image, const uint8_t* host,
                                                                        uint64_t mem_size,
                                                                        const nicgpu_tx_descriptor* __restrict__ tx,
                                                                        uint64_t n) {
  const uint32_t lane = lane_id();
  // wave-uniform (scalar) index, so the descriptor loads are s_loads
  const uint64_t w0 = (uint32_t) __builtin_amdgcn_readfirstlane(blockIdx.x * kImgWaves + threadIdx.x / kWave);
  const uint64_t stride = (uint64_t) gridDim.x * kImgWaves;
  for (uint64_t i = w0; i < n; i += stride) {
    const uint64_t a = tx[i].buffer_address, len = tx[i].length;
    if (len == 0 || !nicqp::dma_ok(mem_size, a, len)) continue;  // a DMA read fault reads nothing (:86-92)
    copy_range(image, host, a, len, mem_size, lane);
  }
}

__global__ __launch_bounds__(kWave * kImgWaves) void image_writeback_kernel(const uint8_t* image, uint8_t* host,
                                                                            uint64_t mem_size,
                                                                            const nicgpu_segment_write* __restrict__ w,
                                                                            uint64_t n) {
  const uint32_t lane = lane_id();
  const uint64_t w0 = (uint32_t) __builtin_amdgcn_readfirstlane(blockIdx.x * kImgWaves + threadIdx.x / kWave);
  const uint64_t stride = (uint64_t) gridDim.x * kImgWaves;
  for (uint64_t j = w0; j < n; j += stride) {
    const uint64_t d = w[j].dst;
    const uint64_t len = (uint64_t) w[j].prefix_len + w[j].len_a + w[j].len_b;
    if (len == 0 || !nicqp::dma_ok(mem_size, d, len)) continue;
    copy_range(host, image, d, len, mem_size, lane);
  }
}

// Batched device copy (nicgpu_memcpy_batch): the ranges split into tiles of
// kCopyTile units (8 B when the range's pointers and size allow, else 1 B);
// blocks walk the tiles grid-stride, the range found by a scalar binary search
// over the tile prefix held in the kernel arguments.
constexpr unsigned kCopyThreads = 256;
constexpr unsigned kCopyTile = kCopyThreads * 4;

struct CopyBatch {
  uint64_t dst[NICGPU_COPY_BATCH_MAX];
  uint64_t src[NICGPU_COPY_BATCH_MAX];
  uint64_t units[NICGPU_COPY_BATCH_MAX];        // 8-B words (wide) or bytes
  uint64_t tile0[NICGPU_COPY_BATCH_MAX + 1];    // first tile of each range; tile0[n] = all tiles
  uint64_t wide;                                // bit i: range i moves 8-B words
  uint32_t n;
};

__global__ __launch_bounds__(kCopyThreads) void copy_batch_kernel(const CopyBatch B) {
  const uint64_t total = B.tile0[B.n];
  for (uint64_t t = blockIdx.x; t < total; t += gridDim.x) {
    uint32_t lo = 0, hi = B.n;  // the range holding tile t: tile0[lo] <= t < tile0[lo + 1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (B.tile0[mid] <= t) lo = mid;
      else hi = mid;
    }
    const uint64_t u0 = (t - B.tile0[lo]) * kCopyTile;
    const uint64_t u1 = u0 + kCopyTile < B.units[lo] ? u0 + kCopyTile : B.units[lo];
    if ((B.wide >> lo) & 1) {
      uint64_t* d = reinterpret_cast<uint64_t*>(B.dst[lo]);
      const uint64_t* s = reinterpret_cast<const uint64_t*>(B.src[lo]);
      uint64_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t u = u0 + threadIdx.x + (uint64_t) k * kCopyThreads;
        if (u < u1) v[k] = s[u];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t u = u0 + threadIdx.x + (uint64_t) k * kCopyThreads;
        if (u < u1) d[u] = v[k];
      }
    } else {
      uint8_t* d = reinterpret_cast<uint8_t*>(B.dst[lo]);
      const uint8_t* s = reinterpret_cast<const uint8_t*>(B.src[lo]);
      for (uint64_t u = u0 + threadIdx.x; u < u1; u += kCopyThreads) d[u] = s[u];
    }
  }
}

// Workgroups per CU the image kernels may take: 8, or NICGPU_IMG_BLOCKS_PER_CU
// (1..64; tuning A/B — a write-back beside the next batch's kernels shares the CUs)
uint64_t image_blocks_per_cu() {
  static const uint64_t v = [] {
    const char* e = std::getenv("NICGPU_IMG_BLOCKS_PER_CU");
    const long x = e ? std::strtol(e, nullptr, 10) : 0;
    return x >= 1 && x <= 64 ? (uint64_t) x : uint64_t{8};
  }();
  return v;
}

unsigned image_grid(uint64_t n, const DeviceInfo* di) {
  const uint64_t want = (n + kImgWaves - 1) / kImgWaves;
  const uint64_t cap = (uint64_t) di->cus * image_blocks_per_cu();
  return (unsigned) (want < cap ? (want ? want : 1) : cap);
}

}  // namespace

extern "C" {

int nicgpu_image_stage(uint8_t* image, const uint8_t* host, uint64_t mem_size, const nicgpu_tx_descriptor* tx,
                       size_t ntx, void* stream) {
  if (ntx == 0 || mem_size == 0) return NICGPU_OK;
  if (!image || !host || !tx || (reinterpret_cast<uintptr_t>(host) & 15u) || (reinterpret_cast<uintptr_t>(image) & 15u))
    return NICGPU_ERR_INVALID;
  const DeviceInfo* di = nullptr;
  const int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(image_stage_kernel, dim3(image_grid(ntx, di)), dim3(kWave * kImgWaves), 0,
                     static_cast<hipStream_t>(stream), image, host, mem_size, tx, (uint64_t) ntx);
  return hip_status(hipGetLastError());
}

int nicgpu_image_writeback(const uint8_t* image, uint8_t* host, uint64_t mem_size, const nicgpu_segment_write* writes,
                           size_t n, void* stream) {
  if (n == 0 || mem_size == 0) return NICGPU_OK;
  if (!image || !host || !writes || (reinterpret_cast<uintptr_t>(host) & 15u) ||
      (reinterpret_cast<uintptr_t>(image) & 15u))
    return NICGPU_ERR_INVALID;
  const DeviceInfo* di = nullptr;
  const int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(image_writeback_kernel, dim3(image_grid(n, di)), dim3(kWave * kImgWaves), 0,
                     static_cast<hipStream_t>(stream), image, host, mem_size, writes, (uint64_t) n);
  return hip_status(hipGetLastError());
}

int nicgpu_memcpy_batch(const nicgpu_copy_range* r, size_t n, void* stream) {
  if (n == 0) return NICGPU_OK;
  if (!r || n > NICGPU_COPY_BATCH_MAX) return NICGPU_ERR_INVALID;
  CopyBatch B{};
  uint64_t tiles = 0;
  for (size_t i = 0; i < n; ++i) {
    if (r[i].bytes && (!r[i].dst || !r[i].src)) return NICGPU_ERR_INVALID;
    const bool wide = ((reinterpret_cast<uintptr_t>(r[i].dst) | reinterpret_cast<uintptr_t>(r[i].src) | r[i].bytes) & 7u) == 0;
    B.dst[i] = reinterpret_cast<uint64_t>(r[i].dst);
    B.src[i] = reinterpret_cast<uint64_t>(r[i].src);
    B.units[i] = wide ? r[i].bytes / 8 : r[i].bytes;
    B.wide |= (uint64_t) wide << i;
    B.tile0[i] = tiles;
    tiles += (B.units[i] + kCopyTile - 1) / kCopyTile;
  }
  B.tile0[n] = tiles;
  B.n = (uint32_t) n;
  if (tiles == 0) return NICGPU_OK;
  const DeviceInfo* di = nullptr;
  const int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  const uint64_t cap = (uint64_t) di->cus * 8;
  hipLaunchKernelGGL(copy_batch_kernel, dim3((unsigned) (tiles < cap ? tiles : cap)), dim3(kCopyThreads), 0,
                     static_cast<hipStream_t>(stream), B);
  return hip_status(hipGetLastError());
}

}  // extern "C"
