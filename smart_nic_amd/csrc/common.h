// common.h — device-side helpers shared by the kernels of libnicgpu.so
// (wave scans, checksum arithmetic, the RX parameter block, the per-wave LDS
// header stage, tuple extraction + Toeplitz, L3/L4 verification).  Included by
// every translation unit; everything here is internal (anonymous namespace).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "nicgpu.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kHdrChunks = 3;      // 48 B of each packet staged in LDS (the IPv4 5-tuple fast path's bytes)
constexpr int kHdrBytes = kHdrChunks * 16;
constexpr uint32_t kHdrStride = kHdrChunks;  // LDS uint4 slots per staged packet (see hdr_slot)
constexpr uint32_t kRingTileBytes = kWave * 8;  // held results of one tile: hash u32[64] | csum u16[64] | queue u16[64]
constexpr uint32_t kLdsPerCu = 160u * 1024u;  // gfx950
constexpr int kLutPos = 2 * NICGPU_MAX_TUPLE;  // nibble positions
constexpr int kLutWords = kLutPos * 16;
constexpr int kHistLds = 1024;     // tables up to this size histogram in LDS (kHistLdsMax)
constexpr int kTableLds = 2048;    // tables up to this size are read from LDS
constexpr uint64_t kOffMask = (1ull << NICGPU_DESC_OFFSET_BITS) - 1;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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

// Inclusive prefix max over the 64 lanes (same DPP pattern; 0 is the identity).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true));
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false));
  return v;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// End-of-block flush of a block's LDS hit histogram (RssStats.queue_hits per
// table index, rss.cpp:54-58) into `out`.  Every block adding its bins to the
// same table_n addresses queued 1024-deep same-address atomic chains exactly
// when the blocks finish together (4 M x 64 B: 7.7 of 88 us).  With replicas
// (a context's kHistRep copies of the histogram, each on lines of its own)
// block b adds into replica b % kHistRep; after every flushing wave's
// vmcnt(0) and a barrier, one lane takes a ticket on a done counter (the
// guide's atomic hand-off: no L2 write-back fence), and the block that takes
// the last ticket moves the replicas into `out` with returning exchanges
// (atomics are performed past the XCD L2s, so no stale copy is read) and
// resets the ticket for the next launch.  hist[0] carries the verdict.
// Replicas are built only with -DNICGPU_HIST_REP: the r03 A/B (3 rounds,
// production vs replicas vs direct flush) measured them neutral on C2, C3 and
// 4 M x 64 B, and one context's ticket is shared by every stream using it.
constexpr uint32_t kHistRep = 16;
constexpr int kHistLdsMax = 1024;  // = kHistLds (tables histogrammed in LDS)
static_assert(kHistLdsMax == kHistLds, "replica stride");
__device__ __forceinline__ void flush_hist(uint32_t* hist, uint32_t table_n, unsigned long long* out,
                                           unsigned long long* rep, unsigned int* done, uint32_t nthreads) {
  __syncthreads();
  if (rep == nullptr) {
    for (uint32_t i = threadIdx.x; i < table_n; i += nthreads) {
      const uint32_t v = hist[i];
      if (v) atomicAdd(&out[i], (unsigned long long) v);
    }
    return;
  }
  unsigned long long* mine = rep + (size_t) (blockIdx.x % kHistRep) * kHistLdsMax;
  for (uint32_t i = threadIdx.x; i < table_n; i += nthreads) {
    const uint32_t v = hist[i];
    if (v) atomicAdd(&mine[i], (unsigned long long) v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's adds are performed
  __syncthreads();
  if (threadIdx.x == 0) hist[0] = atomicAdd(done, 1u) == gridDim.x - 1u ? 1u : 0u;
  __syncthreads();
  if (hist[0] == 0u) return;
  for (uint32_t i = threadIdx.x; i < table_n; i += nthreads) {
    unsigned long long sum = 0;
    for (uint32_t r = 0; r < kHistRep; ++r) sum += atomicExch(rep + (size_t) r * kHistLdsMax + i, 0ull);
    if (sum) atomicAdd(&out[i], sum);
  }
  if (threadIdx.x == 0) atomicExch(done, 0u);
}

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


__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  uint32_t x = (s & 0xFFFFu) + (s >> 16);
  return (x & 0xFFFFu) + (x >> 16);
}


__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }

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
  uint8_t* out_l34;  // NICGPU_L34_* flags (L3/L4 checksum verification), may be null
  uint16_t* out_cs4;  // split sums (no RSS): checksum of each packet's first min(4, len) bytes, out_csum then of the rest
  uint32_t hold_r;   // RING kernels: tiles of results each wave holds in LDS before storing them (>= 1)
  uint32_t ring_off; // RING kernels: LDS byte offset of wave 0's result ring (wave w at + w * hold_r * 512)
  uint32_t xpf_chunks;  // XPF kernels: prefetch the next tile's first batch when it has at most this many chunks
  unsigned long long* stamps;  // tuning builds only: per wave {start, end, XCC_ID, HW_ID} (s_memrealtime, 100 MHz)
  const unsigned long long* n_dev;  // batch size read on the device (min(n, *n_dev)); null: n
  uint32_t xcd_w_odd;   // SPLIT kernels: share of an odd blockIdx % 8 group relative to an even one (65536 = 1)
  unsigned long long* hits_rep;  // per-context histogram replicas (flush_hist), or null
  unsigned int* hits_done;       // their done ticket
};

// s_waitcnt immediate for vmcnt(0) alone (gfx9 encoding: expcnt 7, lgkmcnt 15).
constexpr int kVmcnt0 = 0x0F70;

// Dynamic LDS layout (sized per launch by rx_lds_bytes):
//   per wave: S[64] | E[64] | scratch | hdr[64][kHdrStride] uint4 (only when hashing)
//     scratch = general path: pk[64] uint4 {delta lo, delta hi, end, info} + marks[64 U]
//               contiguous path: two slot windows of 64 U words (ping-pong)
//   per block (first): masks | lut[lut_words] | hist[hist_n] | table, then the waves' parts
constexpr uint32_t kScratchOff = kWave * 4 * 2;

__host__ __device__ constexpr uint32_t rx_scratch_bytes(int unroll) {
  return (uint32_t) (kWave * 16 + kWave * unroll * 4) > (uint32_t) (2 * kWave * unroll * 4)
             ? (uint32_t) (kWave * 16 + kWave * unroll * 4)
             : (uint32_t) (2 * kWave * unroll * 4);
}

__host__ __device__ constexpr uint32_t rx_hdr_off(int unroll) { return kScratchOff + rx_scratch_bytes(unroll); }

__host__ __device__ constexpr uint32_t rx_wave_lds(bool rss, int unroll) {
  return rx_hdr_off(unroll) + (rss ? kWave * kHdrStride * 16 : 0);
}

// Byte masks of a 16-B chunk: entries 0..15 keep bytes >= lo, entries 16..32
// keep bytes < hi (hi = entry - 16); a chunk's mask is their AND.  Two small
// tables (528 B) instead of one lo x hi table keep a 4-wave block under 32 KiB
// of LDS, so 5 blocks fit a CU.
constexpr uint32_t kMaskEntries = 16 + 17;
constexpr uint32_t kMaskTableBytes = kMaskEntries * 16;

// The block part (masks | lut | hist | table), 16-B rounded; the waves' parts follow it.
__host__ __device__ inline uint32_t rx_block_bytes(uint32_t lut_words, uint32_t hist_n, uint32_t table_words) {
  return (kMaskTableBytes + lut_words * 4u + hist_n * 4u + table_words * 4u + 15u) & ~15u;
}

__host__ __device__ inline uint32_t rx_lds_bytes(int wpb, int unroll, bool rss, uint32_t lut_words, uint32_t hist_n,
                                                 uint32_t table_words) {
  return rx_block_bytes(lut_words, hist_n, table_words) + (uint32_t) wpb * rx_wave_lds(rss, unroll);
}

// Header stage of one wave: chunk k (0..2) of the packet in lane q lives in
// slot q*3 + k (48-B packet stride).  A wave's ds_read_b128 of one chunk index
// is conflict-free: lanes are served in 16-lane groups ({0-3,12-15,20-27}, ...)
// and 12*q mod 64 takes 16 distinct values on each group, covering all 64
// banks once; dword and byte reads are 4-way.  With a 64-B stride every dword
// read of the epilogue was a 16-way conflict (SQ_LDS_BANK_CONFLICT: ~190
// cycles per 64-packet tile).  A dense stride keeps every chunk at an
// immediate offset from the lane's base, unlike an XOR swizzle, which cost
// hipcc ~100 VGPRs of hoisted addresses.  Bytes past the stage are read from
// global memory (the general parser, L3/L4 verification).
__device__ __forceinline__ uint32_t hdr_slot(uint32_t q, uint32_t k) { return q * kHdrStride + k; }

struct HdrView {
  const uint4* hdr;  // the wave's stage
  uint32_t q;        // this lane's packet
  __device__ __forceinline__ uint32_t byte(uint32_t a) const {
    return reinterpret_cast<const uint8_t*>(hdr + hdr_slot(q, a >> 4))[a & 15u];
  }
  __device__ __forceinline__ uint32_t word(uint32_t k) const {
    return reinterpret_cast<const uint32_t*>(hdr + hdr_slot(q, k >> 2))[k & 3u];
  }
  // chunks 0..2 as three ds_read_b128 (hipcc would otherwise split them into
  // the few dword reads it needs, which are 4-way conflicted even swizzled)
  __device__ __forceinline__ void chunks3(u32x4& c0, u32x4& c1, u32x4& c2) const {
    typedef __attribute__((address_space(3))) const uint4* lds_ptr;
    const uint32_t a0 = (uint32_t) (uintptr_t) (lds_ptr) (hdr + hdr_slot(q, 0));
    const uint32_t a1 = (uint32_t) (uintptr_t) (lds_ptr) (hdr + hdr_slot(q, 1));
    const uint32_t a2 = (uint32_t) (uintptr_t) (lds_ptr) (hdr + hdr_slot(q, 2));
    asm volatile(
        "ds_read_b128 %0, %3\n\t"
        "ds_read_b128 %1, %4\n\t"
        "ds_read_b128 %2, %5\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(c0), "=&v"(c1), "=&v"(c2)
        : "v"(a0), "v"(a1), "v"(a2)
        : "memory");
  }
};

// One byte of packet l at packet offset o: LDS when staged, else pkt[o] —
// a pointer to the packet, or (deliver_kernel) an accessor of the packet's
// source parts.
template <class Pkt>
__device__ __forceinline__ uint32_t pkt_byte(const HdrView& hv, uint32_t lo, const Pkt& pkt, uint32_t o) {
  uint32_t a = lo + o;
  if (a < (uint32_t) kHdrBytes) return hv.byte(a);
  return pkt[o];
}

template <class Pkt>
__device__ __forceinline__ uint32_t hash_bytes(uint32_t h, const uint32_t* lut, const HdrView& hdr_l, uint32_t lo,
                                               const Pkt& pkt, uint32_t src, uint32_t cnt, uint32_t pos) {
  for (uint32_t i = 0; i < cnt; ++i) {
    uint32_t b = pkt_byte(hdr_l, lo, pkt, src + i);
    uint32_t p = 2 * (pos + i);
    h ^= lut[p * 16 + (b >> 4)] ^ lut[(p + 1) * 16 + (b & 15)];
  }
  return h;
}

// Sum of the little-endian halfwords at absolute (even-address-low) positions
// of packet bytes [a, b), from 4-byte words: word k of the packet's 16-B-aligned
// window comes from the LDS header stage (k < 16) or from global memory.  The
// same convention as the streamed chunk sums, so sub-range sums subtract
// exactly from the packet's total.
__device__ __forceinline__ uint32_t range_sum_le(const HdrView& stage_w, const uint32_t* __restrict__ glob_w,
                                                 uint32_t lo, uint32_t a, uint32_t b) {
  uint32_t s = 0;
  if (a >= b) return 0;
  const uint32_t pa = lo + a, pb = lo + b;
  for (uint32_t k = pa >> 2; 4 * k < pb; ++k) {
    uint32_t v = k < (uint32_t) (kHdrBytes / 4) ? stage_w.word(k) : glob_w[k];
    const uint32_t w0 = 4 * k;
    const uint32_t first = pa > w0 ? pa - w0 : 0u;      // bytes of this word before the range
    const uint32_t last = pb < w0 + 4 ? pb - w0 : 4u;   // bytes of this word inside the range end
    const uint32_t keep = (last == 4u ? 0xFFFFFFFFu : ((1u << (8 * last)) - 1u)) & (0xFFFFFFFFu << (8 * first));
    v &= keep;
    s += (v & 0xFFFFu) + (v >> 16);
  }
  return s;
}

// L3/L4 checksum verification of one packet (oracle/oracle.c
// oracle_l34_verify; reference packet_generator.cpp:200-305).  `sum_le` is the
// packet's streamed halfword sum; the L4 segment's sum is that minus the bytes
// before the segment and after the IP datagram, so no byte is read twice
// except the <= 82 header bytes (from the LDS stage) and any trailer.
[[maybe_unused]] __device__ uint32_t l34_flags(const HdrView& stage_w, const uint32_t* __restrict__ glob_w, uint32_t lo, uint32_t len,
                              uint32_t sum_le) {
  const uint8_t* glob_b = reinterpret_cast<const uint8_t*>(glob_w);
  auto B = [&](uint32_t o) -> uint32_t {
    const uint32_t a = lo + o;
    return a < (uint32_t) kHdrBytes ? stage_w.byte(a) : glob_b[a];
  };
  if (len < 14u) return 0;
  if (lo == 0u && len >= 54u) {
    // Fast path: 16-B-aligned frame, Eth (no tag) / IPv4 IHL 5, no trailer
    // after the datagram — every field at a constant offset of the three
    // staged chunks; the same decisions as the general code below.
    u32x4 c0, c1, c2;
    stage_w.chunks3(c0, c1, c2);
    const uint32_t w[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
    auto byte = [&](int i) __attribute__((always_inline)) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
    const uint32_t et0 = (byte(12) << 8) | byte(13);
    const uint32_t total = (byte(16) << 8) | byte(17);
    if (et0 == 0x0800u && byte(14) == 0x45u && 14u + total == len) {
      uint32_t flags = NICGPU_L34_IPV4;
      // bytes 14..33 and 0..33 as little-endian halfwords (even frame start)
      const uint32_t mid = add_halves(w[4], add_halves(w[5], add_halves(w[6], add_halves(w[7], 0u))));  // 16..31
      const uint32_t ip_le = (w[3] >> 16) + mid + (w[8] & 0xFFFFu);
      if (bswap16(fold16(ip_le)) == 0xFFFFu) flags |= NICGPU_L34_IPV4_OK;
      const uint32_t proto = byte(23);
      const uint32_t frag = ((byte(20) << 8) | byte(21)) & 0x3FFFu;
      if ((proto != 6u && proto != 17u) || frag != 0u) return flags;
      const uint32_t seg = total - 20u;
      if (seg < (proto == 6u ? 20u : 8u)) return flags;
      flags |= NICGPU_L34_L4;
      if (proto == 17u && byte(40) == 0u && byte(41) == 0u) return flags | NICGPU_L34_L4_OK | NICGPU_L34_UDP_NOCSUM;
      const uint32_t pre_le =
          add_halves(w[0], add_halves(w[1], add_halves(w[2], add_halves(w[3], 0u)))) + mid + (w[8] & 0xFFFFu);
      const uint32_t seg_be = bswap16(fold16(sum_le - pre_le));  // the segment starts at even offset 34
      uint32_t acc = seg_be + proto + seg;
      acc += (byte(26) << 8) | byte(27);
      acc += (byte(28) << 8) | byte(29);
      acc += (byte(30) << 8) | byte(31);
      acc += (byte(32) << 8) | byte(33);
      if (fold16(acc) == 0xFFFFu) flags |= NICGPU_L34_L4_OK;
      return flags;
    }
  }
  uint32_t l3 = 14;
  uint32_t et = (B(12) << 8) | B(13);
  for (int t = 0; t < 2 && (et == 0x8100u || et == 0x88A8u); ++t) {
    if (len < l3 + 4u) return 0;
    et = (B(l3 + 2) << 8) | B(l3 + 3);
    l3 += 4;
  }
  if (et != 0x0800u || len < l3 + 20u) return 0;
  const uint32_t v0 = B(l3);
  if ((v0 >> 4) != 4u) return 0;
  const uint32_t ihl = (v0 & 15u) * 4u;
  if (ihl < 20u || l3 + ihl > len) return 0;
  const uint32_t odd = lo & 1u;  // absolute parity of the packet start (frames are 16-B aligned)
  uint32_t flags = NICGPU_L34_IPV4;
  // IPv4 header (starts at an even packet offset): big-endian sum = swap of the
  // absolute little-endian sum unless the packet starts at an odd address
  const uint32_t ipx = fold16(range_sum_le(stage_w, glob_w, lo, l3, l3 + ihl));
  if ((odd ? ipx : bswap16(ipx)) == 0xFFFFu) flags |= NICGPU_L34_IPV4_OK;
  const uint32_t proto = B(l3 + 9);
  const uint32_t frag = ((B(l3 + 6) << 8) | B(l3 + 7)) & 0x3FFFu;
  const uint32_t total = (B(l3 + 2) << 8) | B(l3 + 3);
  if ((proto != 6u && proto != 17u) || frag != 0u || total < ihl || l3 + total > len) return flags;
  const uint32_t seg = total - ihl;
  if (seg < (proto == 6u ? 20u : 8u)) return flags;
  flags |= NICGPU_L34_L4;
  const uint32_t l4 = l3 + ihl;
  if (proto == 17u && B(l4 + 6) == 0u && B(l4 + 7) == 0u) return flags | NICGPU_L34_L4_OK | NICGPU_L34_UDP_NOCSUM;
  const uint32_t seg_le = sum_le - range_sum_le(stage_w, glob_w, lo, 0, l4) - range_sum_le(stage_w, glob_w, lo, l3 + total, len);
  const uint32_t sx = fold16(seg_le);
  const uint32_t seg_be = ((l4 + odd) & 1u) ? sx : bswap16(sx);
  uint32_t acc = seg_be + proto + seg;  // pseudo-header: src, dst, zero, protocol, L4 length
  for (uint32_t o = l3 + 12; o < l3 + 20; o += 2) acc += (B(o) << 8) | B(o + 1);
  if (fold16(acc) == 0xFFFFu) flags |= NICGPU_L34_L4_OK;
  return flags;
}

// Tuple extraction + Toeplitz for one packet (oracle/oracle.c oracle_extract_tuple).
template <class Pkt>
__device__ __forceinline__ uint32_t rss_hash_packet(const RxParams& P, const uint32_t* lut, const HdrView& hdr_l,
                                                    uint32_t lo, const Pkt& pkt, uint32_t len) {
  uint32_t h = 0;
  if (P.mode == NICGPU_TUPLE_RAW) {
    uint32_t cnt = 0;
    if (P.raw_off < len) {
      uint32_t e = P.raw_off + P.raw_len;
      cnt = (e > len ? len : e) - P.raw_off;
    }
    return hash_bytes(0u, lut, hdr_l, lo, pkt, P.raw_off, cnt, 0);
  }
  if (len < 14) return 0;
  if (lo == 0u && len >= 38u) {
    // Fast path: 16-B-aligned frame, Eth (no tag) / IPv4 IHL 5 / TCP|UDP, not a
    // fragment — the first 48 bytes come from LDS in three 16-B reads and the
    // fields are extracted at constant shifts.
    u32x4 c0, c1, c2;
    hdr_l.chunks3(c0, c1, c2);
    const uint32_t w3 = c0.w;  // bytes 12..15: ethertype | ver/ihl | tos
    const uint32_t w5 = c1.y;  // bytes 20..23: flags/frag | ttl | proto
    const uint32_t proto = w5 >> 24;
    if ((w3 & 0xFFFFFFu) == 0x450008u && (w5 & 0xFF3Fu) == 0u && (proto == 6u || proto == 17u)) {
      // tuple = bytes 26..37: src ip 26..29, dst ip 30..33, ports 34..37
      const uint32_t t0 = (c1.z >> 16) | (c1.w << 16);   // bytes 26..29
      const uint32_t t1 = (c1.w >> 16) | (c2.x << 16);   // bytes 30..33
      const uint32_t t2 = (c2.x >> 16) | (c2.y << 16);   // bytes 34..37
      // nibbles pre-scaled to byte offsets four at a time: one extract per
      // lookup, the table's offset an immediate of the ds_read
      const uint8_t* lut_b = reinterpret_cast<const uint8_t*>(lut);
      const uint32_t tw[3] = {t0, t1, t2};
      uint32_t hh = 0;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        uint32_t hi4 = (tw[d] >> 2) & 0x3C3C3C3Cu;  // 4 x high nibble of each byte
        uint32_t lo4 = (tw[d] << 2) & 0x3C3C3C3Cu;  // 4 x low nibble
        asm volatile("" : "+v"(hi4), "+v"(lo4));     // keep them: otherwise folded back into 2 ops per lookup
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = 4 * d + k;  // tuple byte
          const uint32_t ah = (hi4 >> (8 * k)) & 0xFFu, al = (lo4 >> (8 * k)) & 0xFFu;
          hh ^= *reinterpret_cast<const uint32_t*>(lut_b + (2 * i) * 64 + ah) ^
                *reinterpret_cast<const uint32_t*>(lut_b + (2 * i + 1) * 64 + al);
        }
      }
      return hh;
    }
  }
  uint32_t l3 = 14;
  uint32_t et = (pkt_byte(hdr_l, lo, pkt, 12) << 8) | pkt_byte(hdr_l, lo, pkt, 13);
  for (int t = 0; t < 2 && (et == 0x8100u || et == 0x88A8u); ++t) {
    if (len < l3 + 4) return 0;
    et = (pkt_byte(hdr_l, lo, pkt, l3 + 2) << 8) | pkt_byte(hdr_l, lo, pkt, l3 + 3);
    l3 += 4;
  }
  if (et == 0x0800u && len >= l3 + 20) {
    uint32_t vihl = pkt_byte(hdr_l, lo, pkt, l3);
    uint32_t ihl = (vihl & 15u) * 4u;
    if ((vihl >> 4) == 4u && ihl >= 20u) {
      h = hash_bytes(0u, lut, hdr_l, lo, pkt, l3 + 12, 8, 0);
      uint32_t proto = pkt_byte(hdr_l, lo, pkt, l3 + 9);
      uint32_t frag = ((pkt_byte(hdr_l, lo, pkt, l3 + 6) << 8) | pkt_byte(hdr_l, lo, pkt, l3 + 7)) & 0x3FFFu;
      uint32_t l4 = l3 + ihl;
      if ((proto == 6u || proto == 17u) && frag == 0u && l4 + 4u <= len)
        h = hash_bytes(h, lut, hdr_l, lo, pkt, l4, 4, 8);
    }
  } else if (et == 0x86DDu && len >= l3 + 40) {
    uint32_t vb = pkt_byte(hdr_l, lo, pkt, l3);
    if ((vb >> 4) == 6u) {
      h = hash_bytes(0u, lut, hdr_l, lo, pkt, l3 + 8, 32, 0);
      uint32_t nh = pkt_byte(hdr_l, lo, pkt, l3 + 6);
      if ((nh == 6u || nh == 17u) && l3 + 44u <= len) h = hash_bytes(h, lut, hdr_l, lo, pkt, l3 + 40, 4, 32);
    }
  }
  return h;
}


// Block part of rss_only_kernel's dynamic LDS (and of deliver_kernel's):
// LUT | histogram | table, 16-B rounded.
__host__ __device__ inline uint32_t rss_only_block_bytes(uint32_t lut_words, uint32_t hist_n, uint32_t table_words) {
  return (lut_words * 4u + hist_n * 4u + table_words * 4u + 15u) & ~15u;
}

// Byte movement shared by the segmentation (tso.hip) and the gather (f1.hip).
__device__ __forceinline__ uint32_t load_dword_clamped(const uint8_t* mem, uint64_t mem_size, uint64_t a) {
  if (a + 4 <= mem_size) return *reinterpret_cast<const uint32_t*>(mem + a);
  uint32_t v = 0;
  for (uint32_t j = 0; j < 4; ++j)
    if (a + j < mem_size) v |= (uint32_t) mem[a + j] << (8 * j);
  return v;
}

// Wave-cooperative copy of smem[src, src+len) to dmem[dst, dst+len), any
// alignment.  CLAMP: source reads stay inside smem[0, smem_size) (a memory
// image whose end need not be 16-B padded); otherwise the source is a frame
// buffer readable in whole 16-B chunks (include/nicgpu.h).  SUM: returns this
// lane's share of the written bytes' little-endian halfword sum at absolute
// destination positions (the convention of the RX chunk sums).
template <bool CLAMP, bool SUM, int DW = 4>  // DW: whole dwords per lane per step
__device__ uint32_t wave_copy(uint8_t* dmem, uint64_t dst, const uint8_t* smem, uint64_t smem_size, uint64_t src,
                              uint64_t len, uint32_t lane) {
  uint32_t sum = 0;
  if (len == 0) return 0;
  auto byte = [&](uint64_t d, uint64_t s_) __attribute__((always_inline)) {
    const uint32_t b = smem[s_];
    dmem[d] = (uint8_t) b;
    if (SUM) sum += b << (8 * (d & 1));
  };
  const uint64_t d1 = dst + len;
  const uint64_t A = (dst + 3) & ~3ull;  // first whole dword
  const uint64_t B = d1 & ~3ull;          // end of the last whole dword
  if (A >= B) {                           // no whole dword: bytes only
    if (lane < len) byte(dst + lane, src + lane);
    return sum;
  }
  const uint64_t head = A - dst, tail = d1 - B;
  if (lane < head) byte(dst + lane, src + lane);
  if (lane >= 8 && lane - 8 < tail) byte(B + (lane - 8), src + (B - dst) + (lane - 8));
  const uint64_t nw = (B - A) >> 2;
  const uint64_t s0 = src + head;  // source of dword A
  const uint32_t sh = (uint32_t) (s0 & 3);
  const uint64_t sa = s0 & ~3ull;
  for (uint64_t i = (uint64_t) lane * DW; i < nw; i += (uint64_t) kWave * DW) {
    uint32_t v[DW + 1];
#pragma unroll
    for (int j = 0; j < DW + 1; ++j) {
      const uint64_t a = sa + 4 * (i + j);
      if (CLAMP) v[j] = (i + j <= nw) ? load_dword_clamped(smem, smem_size, a) : 0u;
      else v[j] = (i + j <= nw && (j < DW || sh)) ? *reinterpret_cast<const uint32_t*>(smem + a) : 0u;
    }
#pragma unroll
    for (int j = 0; j < DW; ++j) {
      if (i + j < nw) {
        const uint32_t o = sh ? __builtin_amdgcn_alignbyte(v[j + 1], v[j], sh) : v[j];
        *reinterpret_cast<uint32_t*>(dmem + A + 4 * (i + j)) = o;
        if (SUM) sum += (o & 0xFFFFu) + (o >> 16);
      }
    }
  }
  return sum;
}

}  // namespace
