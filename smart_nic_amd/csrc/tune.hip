// tune.hip — tuning-only entry points, built into libnicgpu_tune.so and never
// into the product library: read-only streaming kernels that measure a box's
// HBM read ceiling with the RX kernel's access width, and the FETCH_SIZE
// calibration kernels (tools/calib_fetch.py).

#include "common.h"
#include "host.h"

using namespace nicgpu_detail;

namespace {
template <int U>
__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                          uint32_t* __restrict__ out, unsigned long long* stamps) {
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc = add_halves(v[u].w, add_halves(v[u].z, add_halves(v[u].y, add_halves(v[u].x, acc))));
  }
  for (; i < n16; i += stride) {
    u32x4 v = p[i];
    acc = add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, acc))));
  }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads live
  if (stamps != nullptr && (threadIdx.x & 63) == 0) {  // per wave, as the RX kernel's (tools/wave_stamps.py)
    const uint64_t w = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    stamps[4 * w + 0] = t_start;
    stamps[4 * w + 1] = __builtin_amdgcn_s_memrealtime();
    stamps[4 * w + 2] = (unsigned) __builtin_amdgcn_s_getreg((3 << 11) | 20);
    stamps[4 * w + 3] = (unsigned) __builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
}

// lane l of a wave reads the 32-B pair (2l, 2l+1) of each 2-KiB step
__global__ __launch_bounds__(256) void stream_read_pairs_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                                uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t) gridDim.x * blockDim.x) >> 6;
  for (uint64_t step = wid; step * 128 + 127 < n16; step += nw) {
    const u32x4* q = p + step * 128 + 2 * lane;
    u32x4 a = __builtin_nontemporal_load(q);
    u32x4 b = __builtin_nontemporal_load(q + 1);
    acc = add_halves(a.w, add_halves(a.z, add_halves(a.y, add_halves(a.x, acc))));
    acc = add_halves(b.w, add_halves(b.z, add_halves(b.y, add_halves(b.x, acc))));
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// tile-per-wave streaming (the RX kernel's access pattern without its compute):
// wave w streams region [t*R, (t+1)*R) for tiles t = w, w + nwaves, ...; each
// step every lane loads 16 B (1 KiB per wave), U steps in flight.
template <int U>
__global__ __launch_bounds__(256) void stream_read_tiles_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                                uint64_t tile16, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t) gridDim.x * blockDim.x) >> 6;
  const uint64_t ntiles = n16 / tile16;
  for (uint64_t t = wid; t < ntiles; t += nw) {
    const u32x4* q = p + t * tile16 + lane;
    for (uint64_t st = 0; st + 64 * U <= tile16; st += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(q + st + 64 * u);
#pragma unroll
      for (int u = 0; u < U; ++u) acc = add_halves(v[u].w, add_halves(v[u].z, add_halves(v[u].y, add_halves(v[u].x, acc))));
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// block-cooperative tiles: the block's waves stream ONE tile together, wave w
// reading KiB w of every (waves x 1 KiB) block step.
template <int U>
__global__ __launch_bounds__(256) void stream_read_btiles_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                                 uint64_t tile16, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t ntiles = n16 / tile16;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const u32x4* q = p + t * tile16 + w * 64 + lane;
    for (uint64_t st = 0; st + 256 * U <= tile16; st += 256 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(q + st + 256 * u);
#pragma unroll
      for (int u = 0; u < U; ++u) acc = add_halves(v[u].w, add_halves(v[u].z, add_halves(v[u].y, add_halves(v[u].x, acc))));
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}
}  // namespace

extern "C" {
int nicgpu_tune_stream_btiles(const uint8_t* buf, size_t bytes, size_t tile_bytes, int blocks_per_cu, int unroll,
                              uint32_t* out, void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  const unsigned grid = (unsigned) (di->cus * (blocks_per_cu > 0 ? blocks_per_cu : 4));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p = reinterpret_cast<const u32x4*>(buf);
  const uint64_t t16 = tile_bytes / 16;
  if (unroll == 4) hipLaunchKernelGGL(stream_read_btiles_kernel<4>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  else if (unroll == 2) hipLaunchKernelGGL(stream_read_btiles_kernel<2>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  else hipLaunchKernelGGL(stream_read_btiles_kernel<1>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  return hip_status(hipGetLastError());
}
int nicgpu_tune_stream_tiles(const uint8_t* buf, size_t bytes, size_t tile_bytes, int blocks_per_cu, int unroll,
                             uint32_t* out, void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  const unsigned grid = (unsigned) (di->cus * (blocks_per_cu > 0 ? blocks_per_cu : 4));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p = reinterpret_cast<const u32x4*>(buf);
  const uint64_t t16 = tile_bytes / 16;
  if (unroll == 4) hipLaunchKernelGGL(stream_read_tiles_kernel<4>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  else if (unroll == 2) hipLaunchKernelGGL(stream_read_tiles_kernel<2>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  else hipLaunchKernelGGL(stream_read_tiles_kernel<1>, dim3(grid), dim3(256), 0, s, p, bytes / 16, t16, out);
  return hip_status(hipGetLastError());
}
// blocks_per_cu 0 = occupancy maximum; unroll in {1, 4, 8}
int nicgpu_tune_stream_read(const uint8_t* buf, size_t bytes, int blocks_per_cu, int unroll, uint32_t* out,
                            void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  const uint64_t n16 = bytes / 16;
  const int bpc = blocks_per_cu > 0 ? blocks_per_cu : 8;
  const unsigned grid = (unsigned) (di->cus * bpc);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const u32x4* p = reinterpret_cast<const u32x4*>(buf);
  if (unroll == 2) hipLaunchKernelGGL(stream_read_pairs_kernel, dim3(grid), dim3(256), 0, s, p, n16, out);
  else if (unroll == 8) hipLaunchKernelGGL(stream_read_kernel<8>, dim3(grid), dim3(256), 0, s, p, n16, out, g_tune_stamps);
  else if (unroll == 4) hipLaunchKernelGGL(stream_read_kernel<4>, dim3(grid), dim3(256), 0, s, p, n16, out, g_tune_stamps);
  else hipLaunchKernelGGL(stream_read_kernel<1>, dim3(grid), dim3(256), 0, s, p, n16, out, g_tune_stamps);
  return hip_status(hipGetLastError());
}
// FETCH_SIZE calibration (MI355X_MICROARCH.md: the x2 correction holds for
// 16-B/lane coalesced streaming reads only; "calibrate on a known byte count
// in your own access pattern").  Each kernel reads a known set of whole
// 128-B lines or line prefixes of `buf` in one access shape of this build:
//   shape 0  coalesced 16 B per lane over the whole buffer (the RX stream)
//   shape 1  lane-owned line walk: lane l reads its own 128-B lines, 16 B per
//            load (ICRC: 64 different lines per wave instruction)
//   shape 2  per-packet header gather: 48 B (3 x 16 B) at the start of every
//            1536-B slot (rss_only_kernel's shape on C2 frames)
//   shape 3  the same with 64 B (4 x 16 B) per slot
//   shape 4  the same with 128 B (8 x 16 B, one whole line) per slot
// tools/calib_fetch.py runs them under rocprofv3 --pmc FETCH_SIZE and divides
// the bytes each shape must bring from HBM by what FETCH_SIZE reports.
__global__ __launch_bounds__(256) void calib_kernel(int shape, const u32x4* __restrict__ p, uint64_t n16,
                                                   uint32_t* __restrict__ out) {
  const uint64_t tid = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  const uint64_t nthr = (uint64_t) gridDim.x * 256;
  uint32_t acc = 0;
  if (shape == 0) {
    for (uint64_t i = tid; i < n16; i += nthr) {
      const u32x4 v = __builtin_nontemporal_load(p + i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  } else if (shape == 1) {
    const uint64_t nlines = n16 / 8;
    for (uint64_t l = tid; l < nlines; l += nthr) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const u32x4 v = p[l * 8 + k];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  } else {
    const int nk = shape == 2 ? 3 : (shape == 3 ? 4 : 8);
    const uint64_t nslot = n16 / 96;  // 1536-B slots
    for (uint64_t q = tid; q < nslot; q += nthr) {
      for (int k = 0; k < nk; ++k) {
        const u32x4 v = p[q * 96 + k];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads
}

int nicgpu_tune_calib(int shape, const uint8_t* buf, size_t bytes, uint32_t* out, void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  if (shape < 0 || shape > 4) return NICGPU_ERR_INVALID;
  const unsigned grid = (unsigned) (di->cus * 8);
  hipLaunchKernelGGL(calib_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), shape,
                     reinterpret_cast<const u32x4*>(buf), (uint64_t) (bytes / 16), out);
  return hip_status(hipGetLastError());
}
}  // extern "C"

// Write-pattern ceiling for the f1 delivery (tools/f1_deliver_bench.py
// --patterns): frames of `flen` bytes at `slot`-byte strides (slot = flen
// rounded to 16 = packed), one 16-B store per lane per chunk, consecutive
// lanes on consecutive chunks (a frame's chunks, then the next frame's), no
// loads: what HBM and the caches take for the delivery's store shape.
namespace {
template <bool NT>
__global__ __launch_bounds__(256) void store_pattern_kernel(uint8_t* __restrict__ mem, uint64_t nframes, uint32_t flen,
                                                            uint32_t slot) {
  const uint32_t nch = (flen + 15u) / 16u;
  const uint64_t total = nframes * nch;
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  const u32x4 v = {threadIdx.x, blockIdx.x, 0x5A5A5A5Au, flen};
  for (uint64_t c = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; c < total; c += stride) {
    const uint64_t f = c / nch, k = c - f * nch;
    u32x4* p = reinterpret_cast<u32x4*>(mem + f * slot + k * 16u);
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}
}  // namespace

extern "C" int nicgpu_tune_store_pattern(uint8_t* mem, uint64_t nframes, uint32_t flen, uint32_t slot, int blocks_per_cu,
                                         int nt, void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  if (slot < ((flen + 15u) & ~15u) || (slot & 15u)) return NICGPU_ERR_INVALID;
  const unsigned grid = (unsigned) (di->cus * (blocks_per_cu > 0 ? blocks_per_cu : 8));
  if (nt)
    hipLaunchKernelGGL(store_pattern_kernel<true>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), mem, nframes,
                       flen, slot);
  else
    hipLaunchKernelGGL(store_pattern_kernel<false>, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), mem, nframes,
                       flen, slot);
  return hip_status(hipGetLastError());
}

// ---- unaligned 16-B global accesses (tests/test_gpu_unaligned.py) --------
// deliver_kernel's edge windows load and store 16 B at any byte alignment
// (one dwordx4 each, the HSA unaligned access mode).  Lane i copies the 16 B
// at src + 17 i + soff to dst + 19 i + doff: every byte alignment of both.
__global__ __launch_bounds__(256) void unaligned_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                             uint32_t n, uint32_t soff, uint32_t doff) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  u32x4 v;
  __builtin_memcpy(&v, src + 17u * i + soff, 16);
  __builtin_memcpy(dst + 19u * i + doff, &v, 16);
}

extern "C" int nicgpu_tune_unaligned_copy(const uint8_t* src, uint8_t* dst, uint32_t n, uint32_t soff, uint32_t doff,
                                          void* stream) {
  if (!src || !dst) return NICGPU_ERR_INVALID;
  if (n == 0) return NICGPU_OK;
  hipLaunchKernelGGL(unaligned_copy_kernel, dim3((n + 255u) / 256u), dim3(256), 0, static_cast<hipStream_t>(stream), src,
                     dst, n, soff, doff);
  return hip_status(hipGetLastError());
}

// ---- segmentation copy ceiling ----------------------
// The write pattern of nicgpu_tso_segment on C5 without its work: frame f's
// segment k (k < nseg) is the seg_k = hlen + (k < nseg - 1 ? mss : last)
// bytes at frame offset k * mss (the header's re-read included) copied to slot
// f * nseg + k of `stride` bytes; consecutive lanes on consecutive 16-B chunks
// (16-B loads at the source's alignment, 16-B stores), the segment's last
// chunk stored in part (byte stores: a partial-line write, as segmentation
// must leave the slot's tail alone) unless PAD (the whole chunk written).
namespace {
template <bool NT, bool PAD>
__global__ __launch_bounds__(256) void seg_copy_kernel(const uint8_t* __restrict__ frames, uint32_t nframes,
                                                       uint32_t fstride, uint8_t* __restrict__ out, uint32_t stride,
                                                       uint32_t hlen, uint32_t mss, uint32_t nseg, uint32_t last) {
  const uint32_t segF = hlen + mss, segL = hlen + last;
  const uint32_t nchF = (segF + 15u) / 16u, nchL = (segL + 15u) / 16u;
  const uint32_t per = (nseg - 1u) * nchF + nchL;
  const uint64_t total = (uint64_t) nframes * per;
  const uint64_t step = (uint64_t) gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; c < total; c += step) {
    const uint32_t f = (uint32_t) (c / per), r = (uint32_t) (c - (uint64_t) f * per);
    uint32_t k = r / nchF;
    if (k > nseg - 1u) k = nseg - 1u;
    const uint32_t ch = r - k * nchF;
    const uint32_t seg = k + 1u < nseg ? segF : segL;
    const uint8_t* s = frames + (uint64_t) f * fstride + (uint64_t) k * mss + 16u * ch;
    uint8_t* d = out + ((uint64_t) f * nseg + k) * stride + 16u * ch;
    u32x4 v;
    __builtin_memcpy(&v, s, 16);
    const uint32_t rem = seg - 16u * ch;
    if (PAD || rem >= 16u) {
      if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(d));
      else *reinterpret_cast<u32x4*>(d) = v;
    } else {
      uint8_t b[16];
      __builtin_memcpy(b, &v, 16);
      for (uint32_t i = 0; i < rem; ++i) d[i] = b[i];
    }
  }
}
}  // namespace

extern "C" int nicgpu_tune_seg_copy(const uint8_t* frames, uint32_t nframes, uint32_t fstride, uint8_t* out,
                                    uint32_t stride, uint32_t hlen, uint32_t mss, uint32_t nseg, uint32_t last,
                                    int blocks_per_cu, int flags, void* stream) {
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  if (!frames || !out || nseg == 0 || mss == 0 || (stride & 15u) || stride < ((hlen + mss + 15u) & ~15u) ||
      ((uint64_t) nframes * ((nseg * (hlen + mss)) / 16u + nseg) >= (1ull << 32)))
    return NICGPU_ERR_INVALID;
  const unsigned grid = (unsigned) (di->cus * (blocks_per_cu > 0 ? blocks_per_cu : 8));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool nt = flags & 1, pad = flags & 2;
  if (nt && pad) hipLaunchKernelGGL((seg_copy_kernel<true, true>), dim3(grid), dim3(256), 0, s, frames, nframes, fstride, out, stride, hlen, mss, nseg, last);
  else if (nt) hipLaunchKernelGGL((seg_copy_kernel<true, false>), dim3(grid), dim3(256), 0, s, frames, nframes, fstride, out, stride, hlen, mss, nseg, last);
  else if (pad) hipLaunchKernelGGL((seg_copy_kernel<false, true>), dim3(grid), dim3(256), 0, s, frames, nframes, fstride, out, stride, hlen, mss, nseg, last);
  else hipLaunchKernelGGL((seg_copy_kernel<false, false>), dim3(grid), dim3(256), 0, s, frames, nframes, fstride, out, stride, hlen, mss, nseg, last);
  return hip_status(hipGetLastError());
}
