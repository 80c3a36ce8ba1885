// nicgpu.hip — MI355X (gfx950 / CDNA4) kernels and the C-ABI of include/nicgpu.h.
//
// Hot path: the RX per-packet offload of smart_nic —
//   nic::compute_checksum  (src/checksum.cpp:10-34)  and
//   nic::RssEngine::select_queue (src/rss.cpp:43-94)
// — fused into ONE streaming pass over a packed batch of frames in HBM.
//
// Design:
//  * A wave owns a tile of 64 consecutive packets (one descriptor per lane).
//    The tile's bytes are walked as one flat stream of 16-B chunks: in every
//    step lane l loads chunk (base + l) with a dwordx4 load, so each wave
//    instruction reads up to 1 KiB of contiguous packet bytes whatever the
//    packet sizes (64 B, IMIX, 1518 B, jumbo) — no lanes idle on short packets
//    and no per-size kernels.
//  * chunk -> packet: binary search of the tile's chunk-count prefix in LDS.
//  * checksum: v_dot2_u32_u16(d, {1,1}, acc) adds both little-endian halfwords of a
//    dword in one instruction; a wave-wide DPP inclusive scan turns chunk sums into a
//    running prefix, and each packet's sum is (prefix at its last chunk) -
//    (prefix before its first chunk), recorded by its head/tail lanes in LDS.
//    The ones'-complement fold and the byte swap happen once per packet.
//    Bit-exact with the reference's eager per-add fold.
//  * RSS: the first 64 B of every packet are staged in LDS as they stream past;
//    the tuple is parsed from LDS and hashed with a nibble lookup table of
//    32-bit Toeplitz key windows (built once per key on the device and copied
//    to LDS per block), equivalent to the reference's bit-serial
//    `(bit + k) % key_bits` loop including key wrap.  queue = table[h % n].
//  * No MFMA: this is byte-integer work bounded by HBM read bandwidth.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "nicgpu.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kHdrChunks = 4;      // 64 B of each packet staged in LDS
constexpr int kHdrBytes = kHdrChunks * 16;
constexpr int kLutPos = 2 * NICGPU_MAX_TUPLE;  // nibble positions
constexpr int kLutWords = kLutPos * 16;
constexpr int kHistLds = 1024;     // tables up to this size histogram in LDS
constexpr int kUnroll = 4;         // 16-B chunk loads in flight per lane
constexpr uint64_t kOffMask = (1ull << NICGPU_DESC_OFFSET_BITS) - 1;

const uint8_t kDefaultKey[20] = {0x6D, 0x5A, 0x56, 0x6B, 0x65, 0x4E, 0x67, 0x6E, 0x67, 0x55,
                                 0x6A, 0x6B, 0x61, 0x4F, 0x6B, 0x65, 0x6F, 0x49, 0x4D, 0x42};

// ------------------------------------------------------------ wave helpers --
// Inclusive prefix sum over the 64 lanes (Hillis-Steele inside 16-lane rows by
// row_shr, then row_bcast15 / row_bcast31 across rows — all DPP, no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false); // row_bcast:15
  v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false); // row_bcast:31
  return v;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Keep bytes [lo, hi) of a 16-B chunk (lo in 0..15, hi in 1..16).
__device__ __forceinline__ uint32_t dword_keep(int lo, int hi, int i) {
  int a = lo - 4 * i;
  int b = hi - 4 * i;
  a = a < 0 ? 0 : (a > 4 ? 4 : a);
  b = b < 0 ? 0 : (b > 4 ? 4 : b);
  uint32_t mb = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
  uint32_t ma = a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
  return ma & mb;
}

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

// Sum of the two little-endian 16-bit halves of d, plus acc: one v_dot2_u32_u16.
__device__ __forceinline__ uint32_t add_halves(uint32_t d, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, d), (ushort2_t){1, 1}, acc, false);
}

__device__ __forceinline__ uint32_t chunk_sum(uint4 v) {
  return add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
}

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  uint32_t x = (s & 0xFFFFu) + (s >> 16);
  return (x & 0xFFFFu) + (x >> 16);
}

// Ones'-complement fold of a 64-bit sum: the value in [1, 0xFFFF] congruent to
// s mod 0xFFFF, or 0 only for s == 0 (2^32 == 1 mod 0xFFFF).
__device__ __forceinline__ uint32_t fold64(uint64_t s) {
  if (s == 0) return 0;
  uint32_t r = (uint32_t) (s % 0xFFFFull);
  return r ? r : 0xFFFFu;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }

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

// ------------------------------------------------------------ RX offload --
struct RxParams {
  const uint8_t* frames;
  const uint64_t* desc;
  uint64_t n;
  const uint32_t* lut;
  const uint16_t* table;
  uint32_t table_n;
  uint32_t lut_words;  // LUT words copied to LDS (positions actually hashable)
  int mode;
  uint32_t raw_off, raw_len;
  uint16_t* out_csum;
  uint32_t* out_hash;
  uint16_t* out_queue;
  unsigned long long* out_hits;
};

struct RxShared {
  uint4 hdr[kWavesPerBlock][kWave][kHdrChunks];  // 16 KiB: first 64 B (abs-aligned) per packet
  uint4 pk[kWavesPerBlock][kWave];               // {delta lo, delta hi, end, info} per packet
  uint32_t end[kWavesPerBlock][kWave];           // inclusive chunk-count prefix
  uint32_t S[kWavesPerBlock][kWave];             // running prefix before the packet's first chunk
  uint32_t E[kWavesPerBlock][kWave];             // running prefix after its last chunk
  uint32_t lut[kLutWords];
  uint32_t hist[kHistLds];
};

// One byte of packet `l` at packet offset o: LDS when staged, else global.
__device__ __forceinline__ uint32_t pkt_byte(const RxShared& sh, int w, int l, uint32_t lo,
                                             const uint8_t* __restrict__ pkt, uint32_t o) {
  uint32_t a = lo + o;
  if (a < (uint32_t) kHdrBytes) return reinterpret_cast<const uint8_t*>(&sh.hdr[w][l][0])[a];
  return pkt[o];
}

__device__ __forceinline__ uint32_t hash_bytes(uint32_t h, const RxShared& sh, int w, int l,
                                               uint32_t lo, const uint8_t* __restrict__ pkt,
                                               uint32_t src, uint32_t cnt, uint32_t pos) {
  for (uint32_t i = 0; i < cnt; ++i) {
    uint32_t b = pkt_byte(sh, w, l, lo, pkt, src + i);
    uint32_t p = 2 * (pos + i);
    h ^= sh.lut[p * 16 + (b >> 4)] ^ sh.lut[(p + 1) * 16 + (b & 15)];
  }
  return h;
}

__global__ __launch_bounds__(kBlock) void rx_offload_kernel(RxParams P) {
  __shared__ RxShared sh;
  const int w = threadIdx.x / kWave;
  const uint32_t lane = lane_id();
  const bool want_rss = P.mode != NICGPU_TUPLE_NONE;
  const bool hist_lds = P.out_hits != nullptr && P.table_n <= (uint32_t) kHistLds;

  if (want_rss) {
    for (uint32_t i = threadIdx.x; i < P.lut_words; i += kBlock) sh.lut[i] = P.lut[i];
  }
  if (hist_lds) {
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kBlock) sh.hist[i] = 0;
  }
  __syncthreads();

  const uint64_t ntiles = (P.n + kWave - 1) / kWave;
  const uint64_t wave_gid = (uint64_t) blockIdx.x * kWavesPerBlock + w;
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;

  for (uint64_t tile = wave_gid; tile < ntiles; tile += nwaves) {
    const uint64_t p0 = tile * kWave;
    const uint64_t pid = p0 + lane;
    const bool have = pid < P.n;
    const uint64_t d = have ? P.desc[pid] : 0;
    const uint64_t off = d & kOffMask;
    const uint32_t len = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
    const uint64_t first16 = off >> 4;
    const uint32_t nch = len ? (uint32_t) (((off + len - 1) >> 4) - first16 + 1) : 0u;
    const uint32_t end = wave_incl_scan(nch);
    const uint32_t total = (uint32_t) __builtin_amdgcn_readlane((int) end, 63);
    const uint32_t start = end - nch;
    const int64_t delta = (int64_t) first16 - (int64_t) start;
    const uint32_t lo_first = (uint32_t) (off & 15);
    const uint32_t hi_last = len ? (uint32_t) (((off + len - 1) & 15) + 1) : 16u;
    const uint32_t info = lo_first | (hi_last << 4) | (nch << 9);
    sh.end[w][lane] = end;
    sh.pk[w][lane] = make_uint4((uint32_t) (uint64_t) delta, (uint32_t) ((uint64_t) delta >> 32), end, info);
    __builtin_amdgcn_wave_barrier();

    uint32_t run = 0;  // running chunk-sum prefix of the tile (wave-uniform)
    for (uint32_t base = 0; base < total; base += kWave * kUnroll) {
      uint4 data[kUnroll];
      uint32_t q[kUnroll], c[kUnroll];
      uint4 pk[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        c[u] = base + (uint32_t) u * kWave + lane;
        uint32_t qq = 0;
#pragma unroll
        for (uint32_t s = 32; s >= 1; s >>= 1) {
          if (sh.end[w][qq + s - 1] <= c[u]) qq += s;
        }
        q[u] = qq > 63 ? 63 : qq;
        pk[u] = sh.pk[w][q[u]];
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (c[u] < total) {
          int64_t dl = (int64_t) (((uint64_t) pk[u].y << 32) | pk[u].x);
          uint64_t a16 = (uint64_t) ((int64_t) c[u] + dl);
          data[u] = *reinterpret_cast<const uint4*>(P.frames + a16 * 16);
        } else {
          data[u] = make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const uint32_t endq = pk[u].z, inf = pk[u].w;
        const uint32_t startq = endq - (inf >> 9);
        const bool valid = c[u] < total;
        const bool head = c[u] == startq;
        const bool tail = c[u] + 1 == endq;
        const int lo = head ? (int) (inf & 15u) : 0;
        const int hi = tail ? (int) ((inf >> 4) & 31u) : 16;
        uint4 v = data[u];
        if (lo != 0 || hi != 16) {
          v.x &= dword_keep(lo, hi, 0);
          v.y &= dword_keep(lo, hi, 1);
          v.z &= dword_keep(lo, hi, 2);
          v.w &= dword_keep(lo, hi, 3);
        }
        const uint32_t s = chunk_sum(v);
        const uint32_t incl = wave_incl_scan(s);
        const uint32_t step_total = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
        if (valid) {
          const uint32_t k = c[u] - startq;
          if (head) sh.S[w][q[u]] = run + incl - s;
          if (tail) sh.E[w][q[u]] = run + incl;
          if (want_rss && k < (uint32_t) kHdrChunks) sh.hdr[w][q[u]][k] = v;
        }
        run += step_total;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

    if (have) {
      const uint32_t sum = nch ? (sh.E[w][lane] - sh.S[w][lane]) : 0u;
      const uint32_t x = fold16(sum);
      // LE halfword sums at absolute positions == byte-swapped BE sum when the
      // packet starts at an even address (RFC 1071 byte-order independence).
      const uint32_t be = (off & 1) ? x : bswap16(x);
      if (P.out_csum) P.out_csum[pid] = (uint16_t) (~be & 0xFFFFu);

      if (want_rss) {
        const uint8_t* pkt = P.frames + off;
        uint32_t h = 0;
        if (P.mode == NICGPU_TUPLE_RAW) {
          uint32_t cnt = 0;
          if (P.raw_off < len) {
            uint32_t e = P.raw_off + P.raw_len;
            cnt = (e > len ? len : e) - P.raw_off;
          }
          h = hash_bytes(0u, sh, w, (int) lane, lo_first, pkt, P.raw_off, cnt, 0);
        } else if (len >= 14) {
          uint32_t l3 = 14;
          uint32_t et = (pkt_byte(sh, w, lane, lo_first, pkt, 12) << 8) | pkt_byte(sh, w, lane, lo_first, pkt, 13);
          bool ok = true;
          for (int t = 0; t < 2 && ok && (et == 0x8100u || et == 0x88A8u); ++t) {
            if (len < l3 + 4) {
              ok = false;
            } else {
              et = (pkt_byte(sh, w, lane, lo_first, pkt, l3 + 2) << 8) | pkt_byte(sh, w, lane, lo_first, pkt, l3 + 3);
              l3 += 4;
            }
          }
          if (ok && et == 0x0800u && len >= l3 + 20) {
            uint32_t vihl = pkt_byte(sh, w, lane, lo_first, pkt, l3);
            uint32_t ihl = (vihl & 15u) * 4u;
            if ((vihl >> 4) == 4u && ihl >= 20u) {
              h = hash_bytes(0u, sh, w, (int) lane, lo_first, pkt, l3 + 12, 8, 0);
              uint32_t proto = pkt_byte(sh, w, lane, lo_first, pkt, l3 + 9);
              uint32_t frag = ((pkt_byte(sh, w, lane, lo_first, pkt, l3 + 6) << 8) |
                               pkt_byte(sh, w, lane, lo_first, pkt, l3 + 7)) & 0x3FFFu;
              uint32_t l4 = l3 + ihl;
              if ((proto == 6u || proto == 17u) && frag == 0u && l4 + 4u <= len)
                h = hash_bytes(h, sh, w, (int) lane, lo_first, pkt, l4, 4, 8);
            }
          } else if (ok && et == 0x86DDu && len >= l3 + 40) {
            uint32_t vb = pkt_byte(sh, w, lane, lo_first, pkt, l3);
            if ((vb >> 4) == 6u) {
              h = hash_bytes(0u, sh, w, (int) lane, lo_first, pkt, l3 + 8, 32, 0);
              uint32_t nh = pkt_byte(sh, w, lane, lo_first, pkt, l3 + 6);
              if ((nh == 6u || nh == 17u) && l3 + 44u <= len)
                h = hash_bytes(h, sh, w, (int) lane, lo_first, pkt, l3 + 40, 4, 32);
            }
          }
        }
        const uint32_t idx = h % P.table_n;
        if (P.out_hash) P.out_hash[pid] = h;
        if (P.out_queue) P.out_queue[pid] = P.table[idx];
        if (P.out_hits) {
          if (hist_lds) atomicAdd(&sh.hist[idx], 1u);
          else atomicAdd(&P.out_hits[idx], 1ull);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if (hist_lds) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kBlock) {
      uint32_t v = sh.hist[i];
      if (v) atomicAdd(&P.out_hits[i], (unsigned long long) v);
    }
  }
}

// ------------------------------------------------------------- TSO / GSO --
// One wave per frame.  Each lane streams 16-B chunks of the payload region;
// a chunk overlaps at most two segments (mss >= 16 in the fast path), so the
// chunk's byte sums are split by a mask at the segment boundary and added to
// per-segment accumulators in LDS.  The header's sum is added to every segment
// (byte-swapped when a payload starts at an odd segment offset relative to its
// absolute alignment — ones' complement sums commute with byte swaps).
constexpr int kMaxSeg = 64;  // kMaxTsoSegments, include/nic/offload.h:15

struct TsoParams {
  const uint8_t* frames;
  const uint64_t* desc;
  const uint16_t* hdr_len;
  const uint16_t* mss;
  const uint32_t* seg_base;
  uint64_t n;
  uint16_t* out;
};

__device__ __forceinline__ uint32_t range_sum_chunk(uint4 v, uint64_t cbase, uint64_t lo, uint64_t hi) {
  // sum (LE halfwords) of the bytes of chunk [cbase, cbase+16) that lie in [lo, hi)
  int a = lo > cbase ? (int) (lo - cbase) : 0;
  int b = hi < cbase + 16 ? (int) (hi > cbase ? hi - cbase : 0) : 16;
  if (b <= a) return 0;
  v.x &= dword_keep(a, b, 0);
  v.y &= dword_keep(a, b, 1);
  v.z &= dword_keep(a, b, 2);
  v.w &= dword_keep(a, b, 3);
  return chunk_sum(v);
}

__global__ __launch_bounds__(kBlock) void tso_checksum_kernel(TsoParams P) {
  __shared__ uint32_t seg[kWavesPerBlock][kMaxSeg + 1];
  const int w = threadIdx.x / kWave;
  const uint32_t lane = lane_id();
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;
  for (uint64_t f = (uint64_t) blockIdx.x * kWavesPerBlock + w; f < P.n; f += nwaves) {
    const uint64_t d = P.desc[f];
    const uint64_t off = d & kOffMask;
    const uint64_t L = d >> NICGPU_DESC_OFFSET_BITS;
    const uint32_t mss = P.mss[f];
    uint64_t H = P.hdr_len[f];
    const bool segmented = mss > 0 && L > mss && H < L;
    if (!segmented) H = L;  // one "segment" = the whole frame, all of it header
    const uint32_t nseg = segmented ? (uint32_t) ((L - H + mss - 1) / mss) : 1u;
    if (nseg > (uint32_t) kMaxSeg) continue;  // TooManySegments: the host drops the frame
    for (uint32_t i = lane; i <= (uint32_t) kMaxSeg; i += kWave) seg[w][i] = 0;
    __builtin_amdgcn_wave_barrier();

    const uint64_t a0 = off & ~15ull, a1 = (off + L + 15) & ~15ull;
    uint64_t hsum64 = 0;
    for (uint64_t cb = a0 + 16ull * lane; cb < a1; cb += 16ull * kWave) {
      const uint4 v = *reinterpret_cast<const uint4*>(P.frames + cb);
      hsum64 += range_sum_chunk(v, cb, off, off + H);
      if (segmented && cb + 16 > off + H) {
        // payload bytes of this chunk: segments k0..k1 (k1 <= k0 + 1 when mss >= 16)
        uint64_t plo = cb > off + H ? cb : off + H;
        uint64_t phi = cb + 16 < off + L ? cb + 16 : off + L;
        if (phi > plo) {
          uint32_t k0 = (uint32_t) ((plo - off - H) / mss);
          uint32_t k1 = (uint32_t) ((phi - 1 - off - H) / mss);
          for (uint32_t k = k0; k <= k1; ++k) {
            uint64_t slo = off + H + (uint64_t) k * mss;
            uint64_t shi = slo + mss < off + L ? slo + mss : off + L;
            uint32_t s = range_sum_chunk(v, cb, slo, shi);
            atomicAdd(&seg[w][k], s);
          }
        }
      }
    }
    // wave-reduce the header sum (fold first so the 32-bit adds cannot wrap)
    uint32_t hsum = fold64(hsum64);
    for (int o = 32; o >= 1; o >>= 1) hsum += __shfl_xor(hsum, o);
    hsum = fold16(hsum);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // header BE sum (segment position parity == frame position parity)
    const uint32_t hdr_be = (off & 1) ? hsum : bswap16(hsum);
    for (uint32_t k = lane; k < nseg; k += kWave) {
      uint32_t tot;
      if (segmented) {
        uint32_t px = fold16(seg[w][k]);
        // payload byte at frame offset o sits at segment position o - k*mss
        const bool swap = (((uint64_t) k * mss + off) & 1ull) == 0;
        uint32_t pbe = swap ? bswap16(px) : px;
        tot = fold16(hdr_be + pbe);
      } else {
        tot = hdr_be;
      }
      P.out[P.seg_base[f] + k] = (uint16_t) (~tot & 0xFFFFu);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------ host side --
struct DeviceInfo {
  bool init = false;
  int status = 0;
  int cus = 0;
  int rx_blocks_per_cu = 0;
  int tso_blocks_per_cu = 0;
};

std::mutex g_mu;
DeviceInfo g_dev[64];

int hip_status(hipError_t e) { return e == hipSuccess ? NICGPU_OK : NICGPU_ERR_HIP; }

const DeviceInfo& device_info(int dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceInfo& di = g_dev[dev & 63];
  if (di.init) return di;
  di.init = true;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) { di.status = NICGPU_ERR_HIP; return di; }
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) { di.status = NICGPU_ERR_NO_DEVICE; return di; }
  di.cus = prop.multiProcessorCount;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rx_offload_kernel, kBlock, 0) != hipSuccess || b < 1) b = 1;
  di.rx_blocks_per_cu = b;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tso_checksum_kernel, kBlock, 0) != hipSuccess || b < 1) b = 1;
  di.tso_blocks_per_cu = b;
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

}  // namespace

struct nicgpu_rss_ctx {
  int device = 0;
  uint8_t* d_key = nullptr;      // NICGPU_MAX_KEY bytes
  uint32_t* d_lut = nullptr;     // kLutWords
  uint16_t* d_table = nullptr;   // capacity table_cap
  size_t table_cap = 0;
  size_t key_len = 0;
  size_t table_n = 0;
};

namespace {

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
};

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

int nicgpu_abi_version(void) { return NICGPU_ABI_VERSION; }

const char* nicgpu_strerror(int status) {
  switch (status) {
    case NICGPU_OK: return "ok";
    case NICGPU_ERR_INVALID: return "invalid argument";
    case NICGPU_ERR_HIP: return "HIP runtime error";
    case NICGPU_ERR_NO_DEVICE: return "no gfx950 device";
    case NICGPU_ERR_NOMEM: return "out of device memory";
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
  if (hipMalloc(&ctx->d_key, NICGPU_MAX_KEY) != hipSuccess || hipMalloc(&ctx->d_lut, kLutWords * sizeof(uint32_t)) != hipSuccess) {
    nicgpu_rss_destroy(ctx);
    return NICGPU_ERR_NOMEM;
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

int nicgpu_rx_offload(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                      int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum,
                      uint32_t* out_hash, uint16_t* out_queue, uint64_t* out_hits, void* stream) {
  if (tuple_mode != NICGPU_TUPLE_NONE && tuple_mode != NICGPU_TUPLE_AUTO && tuple_mode != NICGPU_TUPLE_RAW)
    return NICGPU_ERR_INVALID;
  if (tuple_mode == NICGPU_TUPLE_RAW && (raw_off > NICGPU_RAW_MAX_END || raw_len > NICGPU_RAW_MAX_END ||
                                         raw_off + raw_len > NICGPU_RAW_MAX_END))
    return NICGPU_ERR_INVALID;
  if (tuple_mode != NICGPU_TUPLE_NONE && (!ctx || ctx->table_n == 0)) return NICGPU_ERR_INVALID;
  if (tuple_mode == NICGPU_TUPLE_NONE && (out_hash || out_queue || out_hits)) return NICGPU_ERR_INVALID;
  if (n == 0) return NICGPU_OK;
  if (!frames || !desc) return NICGPU_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(frames) & 15u) != 0) return NICGPU_ERR_INVALID;
  if (!out_csum && !out_hash && !out_queue && !out_hits) return NICGPU_OK;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  if (ctx) {
    int dev = 0;
    (void) hipGetDevice(&dev);
    if (dev != ctx->device) return NICGPU_ERR_INVALID;
  }
  RxParams P{};
  P.frames = frames;
  P.desc = desc;
  P.n = n;
  P.mode = tuple_mode;
  P.raw_off = raw_off;
  P.raw_len = raw_len;
  P.out_csum = out_csum;
  P.out_hash = out_hash;
  P.out_queue = out_queue;
  P.out_hits = reinterpret_cast<unsigned long long*>(out_hits);
  if (ctx) {
    P.lut = ctx->d_lut;
    P.table = ctx->d_table;
    P.table_n = (uint32_t) ctx->table_n;
    uint32_t max_tuple = tuple_mode == NICGPU_TUPLE_RAW ? raw_len : 36u;
    P.lut_words = 2u * max_tuple * 16u;
  }
  const uint64_t ntiles = (n + kWave - 1) / kWave;
  const uint64_t want = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) di->rx_blocks_per_cu;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(rx_offload_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

int nicgpu_checksum_batch(const uint8_t* frames, const uint64_t* desc, size_t n, uint16_t* out_csum, void* stream) {
  return nicgpu_rx_offload(nullptr, frames, desc, n, NICGPU_TUPLE_NONE, 0, 0, out_csum, nullptr, nullptr, nullptr,
                           stream);
}

int nicgpu_tso_checksum(const uint8_t* frames, const uint64_t* desc, const uint16_t* hdr_len, const uint16_t* mss,
                        const uint32_t* seg_base, size_t n, uint16_t* out_csum, void* stream) {
  if (n == 0) return NICGPU_OK;
  if (!frames || !desc || !hdr_len || !mss || !seg_base || !out_csum) return NICGPU_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(frames) & 15u) != 0) return NICGPU_ERR_INVALID;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  TsoParams P{frames, desc, hdr_len, mss, seg_base, n, out_csum};
  const uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) di->tso_blocks_per_cu * 2;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(tso_checksum_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

}  // extern "C"
