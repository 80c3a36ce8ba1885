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
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "nicgpu.h"
#include "qp_logic.h"

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

const uint8_t kDefaultKey[20] = {0x6D, 0x5A, 0x56, 0x6B, 0x65, 0x4E, 0x67, 0x6E, 0x67, 0x55,
                                 0x6A, 0x6B, 0x61, 0x4F, 0x6B, 0x65, 0x6F, 0x49, 0x4D, 0x42};

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
  uint8_t* out_l34;  // NICGPU_L34_* flags (L3/L4 checksum verification), may be null
  uint32_t dbg;      // tuning builds only (kDbg*): switch parts of the RSS work off to attribute its cost
  uint32_t hold_r;   // RING kernels: tiles of results each wave holds in LDS before storing them (>= 1)
  uint32_t ring_off; // RING kernels: LDS byte offset of wave 0's result ring (wave w at + w * hold_r * 512)
  uint32_t xpf_chunks;  // XPF kernels: prefetch the next tile's first batch when it has at most this many chunks
  unsigned long long* stamps;  // tuning builds only: per wave {start, end, XCC_ID, HW_ID} (s_memrealtime, 100 MHz)
  const unsigned long long* n_dev;  // batch size read on the device (min(n, *n_dev)); null: n
  unsigned long long* hits_rep;  // per-context histogram replicas (flush_hist), or null
  unsigned int* hits_done;       // their done ticket
};

// s_waitcnt immediate for vmcnt(0) alone (gfx9 encoding: expcnt 7, lgkmcnt 15).
constexpr int kVmcnt0 = 0x0F70;

// Tuning-only knobs (libnicgpu_tune.so; outputs are wrong with any set).
constexpr uint32_t kDbgNoStage = 1, kDbgNoHash = 2, kDbgNoStore = 4, kDbgNoHist = 8, kDbgNtStore = 16,
                   kDbgNoHashStore = 32, kDbgNoQueueStore = 64, kDbgNoTable = 128, kDbgSmallOut = 256, kDbgBurstOut = 512,
                   kDbgStoreSc = 1024 | 2048 | 4096, kDbgRotate = 8192, kDbgNoFlush = 16384;
__device__ __forceinline__ bool dbg_on(const RxParams& P, uint32_t bit) {
#ifdef NICGPU_TUNING
  return (P.dbg & bit) != 0u;
#else
  (void) P;
  (void) bit;
  return false;
#endif
}

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

// One byte of packet l at packet offset o: LDS when staged, else global.
__device__ __forceinline__ uint32_t pkt_byte(const HdrView& hv, uint32_t lo, const uint8_t* __restrict__ pkt,
                                             uint32_t o) {
  uint32_t a = lo + o;
  if (a < (uint32_t) kHdrBytes) return hv.byte(a);
  return pkt[o];
}

__device__ __forceinline__ uint32_t hash_bytes(uint32_t h, const uint32_t* lut, const HdrView& hdr_l, uint32_t lo,
                                               const uint8_t* __restrict__ pkt, uint32_t src, uint32_t cnt,
                                               uint32_t pos) {
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
__device__ uint32_t l34_flags(const HdrView& stage_w, const uint32_t* __restrict__ glob_w, uint32_t lo, uint32_t len,
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
__device__ __forceinline__ uint32_t rss_hash_packet(const RxParams& P, const uint32_t* lut, const HdrView& hdr_l,
                                                    uint32_t lo, const uint8_t* __restrict__ pkt, uint32_t len) {
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


// A batch of U chunk loads per lane: chunk c = base + 64u + lane.
template <int U>
struct ChunkBatch {
  u32x4 v[U];
  uint32_t q[U];     // packet (lane) index within the tile
  uint32_t meta[U];  // lo | hi<<4 | head<<9 | tail<<10 | valid<<11 | hdr slot (0..7)<<12
};

// chunk -> packet without a search: every non-empty packet whose first chunk
// lies in this batch's window [base, base + 64U) writes its lane index, tagged
// with the batch id, at its position in the wave's mark array; a lane's packet
// is then the prefix-max of the valid marks up to its chunk (DPP), seeded with
// the packet of the previous batch's last chunk (`carry`).  One LDS write and
// one LDS read per batch instead of a chain of dependent reads.  The 16-B load
// is issued unconditionally (lanes past the tile's end re-read its last chunk
// and are zeroed later), so the loads carry no branches.
template <int U, bool NT>
__device__ __forceinline__ void plan_batch(ChunkBatch<U>& B, const uint4* __restrict__ pk, uint32_t* marks,
                                           uint32_t base, uint32_t total, uint32_t lane, uint32_t my_start,
                                           uint32_t my_nch, uint32_t tag, uint32_t& carry,
                                           const uint8_t* __restrict__ frames) {
  const uint32_t rel = my_start - base;
  if (my_nch != 0u && my_start >= base && rel < (uint32_t) (kWave * U)) marks[rel] = (tag << 6) | lane;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t m = marks[u * kWave + lane];
    const uint32_t cand = (m >> 6) == tag ? (m & 63u) : 0u;
    uint32_t q = wave_incl_max(cand);
    q = max(q, carry);
    carry = (uint32_t) __builtin_amdgcn_readlane((int) q, 63);
    const uint32_t c = base + (uint32_t) u * kWave + lane;
    const uint4 e = pk[q];
    const uint32_t endq = e.z, inf = e.w;
    const uint32_t startq = endq - (inf >> 9);
    const bool valid = c < total;
    const bool head = c == startq;
    const bool tail = c + 1 == endq;
    const uint32_t lo = head ? (inf & 15u) : 0u;
    const uint32_t hi = tail ? ((inf >> 4) & 31u) : 16u;
    const uint32_t k = c - startq;
    const uint32_t slot = k < (uint32_t) kHdrChunks ? k : 7u;
    B.q[u] = q;
    B.meta[u] = lo | (hi << 4) | ((uint32_t) head << 9) | ((uint32_t) tail << 10) | ((uint32_t) valid << 11) |
                (slot << 12);
    const uint32_t ce = valid ? c : total - 1u;
    const int64_t dl = (int64_t) (((uint64_t) e.y << 32) | e.x);
    const u32x4* p = reinterpret_cast<const u32x4*>(frames + (uint64_t) ((int64_t) ce + dl) * 16);
    if constexpr (NT) B.v[u] = __builtin_nontemporal_load(p);
    else B.v[u] = *p;
  }
}

// ---- contiguous tiles ----------------------------------------------------
// When every non-empty packet of a tile starts in the 16-B chunk right after
// the previous one's last chunk (a packed batch), chunk c of the tile lives at
// absolute chunk D + c: loads need no chunk -> packet map at all.  The few
// positions that need packet information — the first kHdrChunks chunks of a
// packet (header staging, head mask) and its last chunk (tail mask, prefix
// record) — are scattered by the packet lanes into a per-window slot array
// (0 = nothing); chunk lanes read and clear their slot.
//   slot: bit0 valid | q<<1 (6) | k<<7 (3: header chunk 0..3, 7 = none)
//         | lo<<11 (4) | tail<<15 | hi<<16 (5)
template <int U>
struct ContigBatch {
  u32x4 v[U];
};

// Slot word of a contiguous window position that needs packet information:
//   bit 0 valid | q << 1 (6) | k << 7 (3, 7 = tail beyond the header) |
//   tail << 10 | lo << 11 (4) | hi << 15 (5); lo = 0, hi = 16 is a whole chunk
template <int U>
__device__ __forceinline__ void scatter_slots(uint32_t* slots, uint32_t base, uint32_t lane, uint32_t start,
                                              uint32_t nch, uint32_t info) {
  if (nch == 0u) return;
  constexpr uint32_t W = (uint32_t) kWave * U;
  const uint32_t rs = start - base;          // window-relative start (wraps when before the window)
  const uint32_t re = start + nch - 1u - base;
  const uint32_t lo = info & 15u, hi = (info >> 4) & 31u;
  const uint32_t common = 1u | (lane << 1);
#pragma unroll
  for (uint32_t j = 0; j < (uint32_t) kHdrChunks; ++j) {
    const uint32_t r = rs + j;
    if (j < nch && r < W) {
      const bool tail = j + 1u == nch;
      slots[r] = common | (j << 7) | (tail ? (1u << 10) : 0u) | ((j == 0 ? lo : 0u) << 11) | ((tail ? hi : 16u) << 15);
    }
  }
  if (nch > (uint32_t) kHdrChunks && re < W) slots[re] = common | (7u << 7) | (1u << 10) | (hi << 15);
}

// The tile's chunks through a buffer resource (base = the tile's first chunk,
// num_records = its bytes): lane offset lane * 16 is fixed, the batch offset
// is scalar and the step offset an immediate, so a load costs no VALU, and
// positions past the tile end read zeros (they carry no slot either).
template <int U, int CP>
__device__ __forceinline__ void plan_contig(ContigBatch<U>& B, uint32_t* slots, uint32_t base, uint32_t lane,
                                            uint32_t start, uint32_t nch, uint32_t info,
                                            __amdgpu_buffer_rsrc_t rsrc) {
  scatter_slots<U>(slots, base, lane, start, nch, info);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t vo = lane * 16u + (uint32_t) u * (kWave * 16u);
    B.v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int) vo, (int) (base * 16u),
                                                                            CP));
  }
}

template <int U>
__device__ __forceinline__ uint32_t process_contig(ContigBatch<U>& B, uint32_t* slots, const uint4* masks,
                                                   uint32_t run, uint32_t* E, uint4* hdr, bool stage_hdr,
                                                   uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t sl = slots[u * kWave + lane];
    u32x4 v = B.v[u];
    if (sl != 0u) {
      slots[u * kWave + lane] = 0u;
      const uint32_t mi = sl >> 11;  // lo | hi << 4
      if (mi != (16u << 4)) {
        const uint4 a = masks[mi & 15u], b = masks[16u + (mi >> 4)];
        v.x &= a.x & b.x;
        v.y &= a.y & b.y;
        v.z &= a.z & b.z;
        v.w &= a.w & b.w;
      }
    }
    const uint32_t s = add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
    const uint32_t incl = wave_incl_scan(s);
    const uint32_t step_total = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
    if (sl != 0u) {
      const uint32_t q = (sl >> 1) & 63u, k = (sl >> 7) & 7u;
      if (sl & (1u << 10)) E[q] = run + incl;
      if (stage_hdr && k < (uint32_t) kHdrChunks) hdr[hdr_slot(q, k)] = make_uint4(v.x, v.y, v.z, v.w);
    }
    run += step_total;
  }
  return run;
}

// Mask, sum, scan and record one batch.  `run` is the tile's running prefix.
template <int U>
__device__ __forceinline__ uint32_t process_batch(ChunkBatch<U>& B, uint32_t run, uint32_t* S, uint32_t* E,
                                                  uint4* hdr, bool stage_hdr) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t m = B.meta[u];
    const int lo = (int) (m & 15u), hi = (int) ((m >> 4) & 31u);
    u32x4 v = B.v[u];
    if (!(m & (1u << 11))) v = (u32x4){0u, 0u, 0u, 0u};
    if (lo != 0 || hi != 16) {
      v.x &= dword_keep(lo, hi, 0);
      v.y &= dword_keep(lo, hi, 1);
      v.z &= dword_keep(lo, hi, 2);
      v.w &= dword_keep(lo, hi, 3);
    }
    const uint32_t s = add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
    const uint32_t incl = wave_incl_scan(s);
    const uint32_t step_total = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
    if (m & (1u << 11)) {
      const uint32_t q = B.q[u];
      if (m & (1u << 9)) S[q] = run + incl - s;
      if (m & (1u << 10)) E[q] = run + incl;
      const uint32_t slot = m >> 12;
      if (stage_hdr && slot < (uint32_t) kHdrChunks) hdr[hdr_slot(q, slot)] = make_uint4(v.x, v.y, v.z, v.w);
    }
    run += step_total;
  }
  return run;
}

// Per-lane view of one tile (lane = one packet).  `total` and `contig` are
// wave-uniform.
// (no padding bytes: struct copies with padding leave scratch allocas behind)
struct Tile {
  uint64_t base;  // packet index of lane 0
  uint64_t off;
  int64_t delta;  // first16 - start: chunk c of this packet is absolute chunk c + delta
  int64_t D;      // common delta of a contiguous tile
  uint32_t len, nch, start, end, info;
  uint32_t total;
  uint32_t contig;  // 0/1
  uint32_t nvalid;  // lanes holding a packet of this tile (lanes >= nvalid write nothing)
};
static_assert(sizeof(Tile) == 64, "Tile must stay padding-free");

template <bool CONTIG>
__device__ __forceinline__ Tile make_tile(uint64_t base, uint32_t nvalid, uint64_t d) {
  Tile t;
  t.base = base;
  t.off = d & kOffMask;
  t.len = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
  const uint64_t first16 = t.off >> 4;
  t.nch = t.len ? (uint32_t) (((t.off + t.len - 1) >> 4) - first16 + 1) : 0u;
  t.end = wave_incl_scan(t.nch);
  t.total = (uint32_t) __builtin_amdgcn_readlane((int) t.end, 63);
  t.start = t.end - t.nch;
  t.delta = (int64_t) first16 - (int64_t) t.start;
  const uint32_t lo_first = (uint32_t) (t.off & 15);
  const uint32_t hi_last = t.len ? (uint32_t) (((t.off + t.len - 1) & 15) + 1) : 16u;
  t.info = lo_first | (hi_last << 4) | (t.nch << 9);
  const uint64_t nonempty = __ballot(t.nch != 0u);
  const int first_ne = nonempty ? __builtin_ctzll(nonempty) : 0;
  const uint32_t dl = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (uint64_t) t.delta, first_ne);
  const uint32_t dh = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) ((uint64_t) t.delta >> 32), first_ne);
  t.D = (int64_t) (((uint64_t) dh << 32) | dl);
  t.contig = (CONTIG && __ballot(t.nch != 0u && t.delta != t.D) == 0ull) ? 1u : 0u;
  t.nvalid = nvalid;
  return t;
}

struct RxLdsPtrs {
  uint32_t* S;
  uint32_t* E;
  uint4* pk;
  uint32_t* marks;
  uint32_t* slotsA;
  uint32_t* slotsB;
  uint4* hdr;
  uint32_t* lut;
  uint32_t* hist;
  uint16_t* table_s;
  const uint4* masks;  // kMaskEntries byte masks (per block)
  bool hist_lds, table_lds, want_rss;
  bool stage;  // first 64 B of every packet staged in LDS (hashing or L3/L4 verify)
};

// One lane's results of a tile, held in registers so that (DEFER) they are
// stored only after the next tile's first loads are in flight: on gfx950
// stores count in vmcnt and complete in order with loads, so stores issued
// just before a tile's first loads made the first counted wait of every tile
// also wait for the previous tile's store acknowledgements (tools/tune_rx.py
// --dbg: without the hash/queue stores C2 ran 16 µs faster, IMIX 29 µs).
struct TileOut {
  uint64_t pid;
  uint32_t cs, h, q, l34;
  uint32_t valid;  // lane < nvalid
};

// SST: cache-policy bits of the result stores (0 = plain global stores; 16 =
// sc1 buffer stores, device scope).
template <int SST>
__device__ __forceinline__ void store_out(const RxParams& P, const TileOut& o, bool rss, bool l34 = true) {
  if (SST != 0) {
    if (o.valid) {
      // per-tile resources: base = this tile's first output, offset = lane
      const uint32_t l = (uint32_t) (o.pid & 63u);
      const uint64_t tb = o.pid - l;
      if (P.out_csum)
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.cs,
                                              __builtin_amdgcn_make_buffer_rsrc(P.out_csum + tb, (short) 0, 128, 0x00020000),
                                              (int) (l * 2u), 0, SST);
      if (l34 && P.out_l34) P.out_l34[o.pid] = (uint8_t) o.l34;
      if (rss) {
        if (P.out_hash)
          __builtin_amdgcn_raw_buffer_store_b32(o.h,
                                                __builtin_amdgcn_make_buffer_rsrc(P.out_hash + tb, (short) 0, 256, 0x00020000),
                                                (int) (l * 4u), 0, SST);
        if (P.out_queue)
          __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.q,
                                                __builtin_amdgcn_make_buffer_rsrc(P.out_queue + tb, (short) 0, 128, 0x00020000),
                                                (int) (l * 2u), 0, SST);
      }
    }
    return;
  }
  if (dbg_on(P, kDbgNtStore)) {
    if (o.valid) {
      if (P.out_csum) __builtin_nontemporal_store((uint16_t) o.cs, P.out_csum + o.pid);
      if (rss) {
        if (P.out_hash) __builtin_nontemporal_store(o.h, P.out_hash + o.pid);
        if (P.out_queue) __builtin_nontemporal_store((uint16_t) o.q, P.out_queue + o.pid);
      }
    }
    return;
  }
  if (dbg_on(P, kDbgStoreSc)) {  // cache-policy experiment on the three output stores
    if (o.valid) {
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(P.out_csum, (short) 0, 0x7FFFFFFF, 0x00020000);
      const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(P.out_hash, (short) 0, 0x7FFFFFFF, 0x00020000);
      const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(P.out_queue, (short) 0, 0x7FFFFFFF, 0x00020000);
      const int off2 = (int) (o.pid * 2), off4 = (int) (o.pid * 4);
      if (P.dbg & 1024) {
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.cs, rc, off2, 0, 17);
        __builtin_amdgcn_raw_buffer_store_b32(o.h, rh, off4, 0, 17);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.q, rq, off2, 0, 17);
      } else if (P.dbg & 2048) {
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.cs, rc, off2, 0, 18);
        __builtin_amdgcn_raw_buffer_store_b32(o.h, rh, off4, 0, 18);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.q, rq, off2, 0, 18);
      } else {
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.cs, rc, off2, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(o.h, rh, off4, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.q, rq, off2, 0, 16);
      }
    }
    return;
  }
  if (dbg_on(P, kDbgBurstOut)) {  // same bytes, written as 4-tile (1 KiB hash) bursts by every 4th tile's wave
    if (((o.pid >> 6) & 3u) == 3u) {
      const uint64_t b = (o.pid & ~255ull) + (o.pid & 63u);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (P.out_csum) P.out_csum[b + 64 * j] = (uint16_t) o.cs;
        if (rss) {
          if (P.out_hash) P.out_hash[b + 64 * j] = o.h;
          if (P.out_queue) P.out_queue[b + 64 * j] = (uint16_t) o.q;
        }
      }
    }
    return;
  }
  if (dbg_on(P, kDbgSmallOut)) {  // same stores, into a 64 KiB window (L2-resident): write path vs DRAM
    const uint64_t w = o.pid & 16383u;
    if (o.valid) {
      if (P.out_csum) P.out_csum[w] = (uint16_t) o.cs;
      if (rss) {
        if (P.out_hash) P.out_hash[w] = o.h;
        if (P.out_queue) P.out_queue[w] = (uint16_t) o.q;
      }
    }
    return;
  }
  if (o.valid) {
    if (P.out_csum) P.out_csum[o.pid] = (uint16_t) o.cs;
    if (l34 && P.out_l34) P.out_l34[o.pid] = (uint8_t) o.l34;
    if (rss && !dbg_on(P, kDbgNoStore)) {
      if (P.out_hash && !dbg_on(P, kDbgNoHashStore)) P.out_hash[o.pid] = o.h;
      if (P.out_queue && !dbg_on(P, kDbgNoQueueStore)) P.out_queue[o.pid] = (uint16_t) o.q;
    }
  }
}

// Store the results of the ring's n tiles (bases base0, base0 + step, ...).
// (Holding 6 B per packet and looking the queue up again here fit 9 tiles
// instead of 7 on IMIX for no gain there, and cost 64-B batches 10%.)
template <int SST, typename Lds, typename NValid>
__device__ __forceinline__ void flush_ring(const RxParams& P, const Lds& L, const uint8_t* ring, uint32_t n,
                                           uint64_t base0, uint64_t step, uint32_t lane, const NValid& nvalid_of) {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* slot = ring + i * kRingTileBytes;
    const uint64_t base = base0 + i * step;
    TileOut o;
    o.pid = base + lane;
    o.h = reinterpret_cast<const uint32_t*>(slot)[lane];
    o.cs = reinterpret_cast<const uint16_t*>(slot + kWave * 4)[lane];
    o.q = reinterpret_cast<const uint16_t*>(slot + kWave * 6)[lane];
    o.l34 = 0;
    o.valid = lane < nvalid_of(base) ? 1u : 0u;
    store_out<SST>(P, o, L.want_rss, false);  // out_l34 was stored at the epilogue
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

[[maybe_unused]] __device__ __forceinline__ TileOut held_out(uint64_t base, uint32_t nvalid, uint32_t csq, uint32_t h, uint32_t lane) {
  TileOut o;
  o.pid = base + lane;
  o.cs = csq & 0xFFFFu;
  o.q = csq >> 16;
  o.h = h;
  o.l34 = 0;
  o.valid = lane < nvalid ? 1u : 0u;
  return o;
}

// Checksum finish + tuple hash + queue of the tile's packets (one per lane);
// the hit histogram is updated here (LDS), the outputs are returned.
__device__ __forceinline__ TileOut tile_epilogue(const RxParams& P, const RxLdsPtrs& L, const Tile& t, uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  TileOut o;
  o.pid = t.base + lane;
  o.cs = o.h = o.q = o.l34 = 0;
  o.valid = lane < t.nvalid ? 1u : 0u;
  // contiguous tiles record only tail prefixes: a packet starts where the
  // nearest non-empty packet before it ended (0 at the tile start)
  uint32_t base_prefix = 0;
  if (t.contig) {
    const uint32_t pidx = wave_incl_max(t.nch ? lane + 1u : 0u);
    const uint32_t prev = (uint32_t) __builtin_amdgcn_update_dpp(0, (int) pidx, 0x138, 0xf, 0xf, false);  // wave_shr:1
    base_prefix = (lane != 0u && prev != 0u) ? L.E[prev - 1u] : 0u;
  }
  if (o.valid) {
    const uint32_t sum = t.nch ? (L.E[lane] - (t.contig ? base_prefix : L.S[lane])) : 0u;
    const uint32_t x = fold16(sum);
    // LE halfword sums at absolute positions == byte-swapped BE sum when the
    // packet starts at an even address (RFC 1071 byte-order independence).
    const uint32_t be = (t.off & 1) ? x : bswap16(x);
    o.cs = ~be & 0xFFFFu;
    if (P.out_l34)
      o.l34 = l34_flags(HdrView{L.hdr, lane}, reinterpret_cast<const uint32_t*>(P.frames + (t.off & ~15ull)),
                        (uint32_t) (t.off & 15), t.len, sum);
    if (L.want_rss) {
      const uint32_t h = dbg_on(P, kDbgNoHash)
                             ? (uint32_t) o.pid * 2654435761u
                             : rss_hash_packet(P, L.lut, HdrView{L.hdr, lane}, (uint32_t) (t.off & 15),
                                               P.frames + t.off, t.len);
      const uint32_t idx = h % P.table_n;
      o.h = h;
      if (P.out_queue) {
        if (dbg_on(P, kDbgNoTable)) {
          o.q = idx;
        } else if (L.table_lds) {
          o.q = L.table_s[idx];
        } else {
          o.q = P.table[idx];
          // wait for this load here, on this path only: left to the merged
          // path after the branch, the wait lands at the ring write as a
          // vmcnt(0) on the LDS-table path too, i.e. it drains the next
          // tile's prefetched first batch at every tile end
          __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
      }
      if (P.out_hits && !dbg_on(P, kDbgNoHist)) {
        if (L.hist_lds) atomicAdd(&L.hist[idx], 1u);
        else atomicAdd(&P.out_hits[idx], 1ull);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return o;
}

// General tiles (packets not contiguous in chunk space): chunk -> packet by
// marks + DPP prefix-max, ping-pong over the tile.
template <int U, bool NT, bool DEFER, int SST>
__device__ __forceinline__ void run_general_tile(const RxParams& P, const RxLdsPtrs& L, const Tile& t, uint32_t lane,
                                                 uint32_t& tag, const TileOut& pend) {
  constexpr uint32_t kStep = (uint32_t) kWave * U;
  L.pk[lane] = make_uint4((uint32_t) (uint64_t) t.delta, (uint32_t) ((uint64_t) t.delta >> 32), t.end, t.info);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  uint32_t run = 0, carry = 0;
  ChunkBatch<U> A, B;
  uint32_t b0 = 0;
  // counted pair loop, single exit at the bottom (see the contiguous path)
  const uint32_t nbatch = (t.total + kStep - 1) / kStep;
  plan_batch<U, NT>(A, L.pk, L.marks, b0, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
  if (DEFER) {
    __builtin_amdgcn_sched_barrier(0);  // the previous tile's stores after this tile's first loads
    store_out<SST>(P, pend, L.want_rss);
  }
  uint32_t bi = 0;
  for (; bi + 1 < nbatch; bi += 2, b0 += 2 * kStep) {
    plan_batch<U, NT>(B, L.pk, L.marks, b0 + kStep, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
    __builtin_amdgcn_sched_barrier(0);  // B's loads issue before A's wait
    run = process_batch<U>(A, run, L.S, L.E, L.hdr, L.stage);
    plan_batch<U, NT>(A, L.pk, L.marks, b0 + 2 * kStep, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
    __builtin_amdgcn_sched_barrier(0);
    run = process_batch<U>(B, run, L.S, L.E, L.hdr, L.stage);
  }
  if (bi < nbatch) run = process_batch<U>(A, run, L.S, L.E, L.hdr, L.stage);
}

// CPOL: cache-policy bits of the contiguous path's buffer loads (gfx950: 1 sc0,
// 2 nt, 16 sc1); -1 = nt when NT.
// HOLD > 0: keep up to HOLD tiles' results in registers and store them as one
// burst when the ring is full and at the end (experiment: do output writes
// cost less when they are not interleaved with the read stream?).
// RING: results are held in a per-wave LDS ring of P.hold_r tiles and stored
// when it is full and at the end, so output writes reach DRAM in bursts
// instead of interleaved with the read stream.
// GEN = false (tuning only, names "*_xc"): no general path compiled in, so
// non-contiguous tiles are skipped and their results are wrong; measures what
// the general path's registers cost the contiguous loop.
// XPF: the next contiguous tile's first batch (slots scattered, loads issued)
// goes out before this tile's epilogue, so the epilogue overlaps its latency
// (tiles of at most P.xpf_chunks chunks).
template <int U, bool NT, int WPB, bool CONTIG, bool RANGES, int OCC, bool DEFER, int CPOL = -1, int SST = 0,
          int HOLD = 0, bool RING = false, bool GEN = true, bool XPF = false>
__global__ __launch_bounds__(kWave * WPB) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void rx_offload_kernel(
    RxParams P) {
  extern __shared__ uint4 lds_dyn[];
  const int w = threadIdx.x / kWave;
  const uint32_t lane = lane_id();
  constexpr uint32_t kStep = (uint32_t) kWave * U;

  RxLdsPtrs L;
  L.want_rss = P.mode != NICGPU_TUPLE_NONE;
  L.stage = (L.want_rss || P.out_l34 != nullptr) && !dbg_on(P, kDbgNoStage);
  L.hist_lds = P.out_hits != nullptr && P.table_n <= (uint32_t) kHistLds;
  L.table_lds = L.want_rss && P.table_n <= (uint32_t) kTableLds;
  uint8_t* base_b = reinterpret_cast<uint8_t*>(lds_dyn);
  // block part first — masks | lut | hist | table — so the LUT sits at a
  // constant LDS address and the hash's table offsets fold into ds_read
  // immediates; then the waves' parts
  const uint32_t block_bytes = rx_block_bytes(L.want_rss ? P.lut_words : 0u, L.hist_lds ? P.table_n : 0u,
                                              L.table_lds ? (P.table_n + 1u) / 2u : 0u);
  uint8_t* wave_b = base_b + block_bytes + (uint32_t) w * rx_wave_lds(L.stage, U);
  L.S = reinterpret_cast<uint32_t*>(wave_b);
  L.E = L.S + kWave;
  L.pk = reinterpret_cast<uint4*>(wave_b + kScratchOff);
  L.marks = reinterpret_cast<uint32_t*>(wave_b + kScratchOff + kWave * 16);
  L.slotsA = reinterpret_cast<uint32_t*>(wave_b + kScratchOff);
  L.slotsB = L.slotsA + kWave * U;
  L.hdr = reinterpret_cast<uint4*>(wave_b + rx_hdr_off(U));
  uint4* masks_w = reinterpret_cast<uint4*>(base_b);
  L.masks = masks_w;
  L.lut = reinterpret_cast<uint32_t*>(base_b + kMaskTableBytes);
  L.hist = L.lut + (L.want_rss ? P.lut_words : 0u);
  L.table_s = reinterpret_cast<uint16_t*>(L.hist + (L.hist_lds ? P.table_n : 0u));
  // marks never match a live tag (tags start at 1; cleared slots read as 0)
  for (uint32_t i = lane; i < (uint32_t) (kWave * U); i += kWave) L.marks[i] = 0xFFFFFFFFu;
  uint32_t tag = 0;  // batch id of the general path (never reaches 0x3FFFFFF within a launch)

  for (uint32_t i = threadIdx.x; i < kMaskEntries; i += kWave * WPB) {
    const int lo = i < 16u ? (int) i : 0, hi = i < 16u ? 16 : (int) i - 16;
    masks_w[i] = make_uint4(dword_keep(lo, hi, 0), dword_keep(lo, hi, 1), dword_keep(lo, hi, 2), dword_keep(lo, hi, 3));
  }
  if (L.want_rss) {
    for (uint32_t i = threadIdx.x; i < P.lut_words; i += kWave * WPB) L.lut[i] = P.lut[i];
  }
  if (L.hist_lds) {
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kWave * WPB) L.hist[i] = 0;
  }
  if (L.table_lds) {
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kWave * WPB) L.table_s[i] = P.table[i];
  }
  __syncthreads();
#ifdef NICGPU_TUNING
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif

  // Work split.  RANGES: wave g owns packets [g*n/W, (g+1)*n/W), walked in
  // tiles of 64 (the last one partial), so every wave streams the same number
  // of bytes give or take one packet (whole-tile round robin leaves the last
  // round to a fraction of the waves: 1 M packets = 3.2 tiles per wave).
  // Otherwise tile k*W + g (round robin).
  const uint64_t nwaves = (uint64_t) gridDim.x * WPB;
  const uint64_t gw_hw = (uint64_t) blockIdx.x * WPB + w;
  // packets in this launch: n, or a count another kernel left on the device
  // (the grid is sized for n; waves past the count have no tile)
  const uint64_t n_all = P.n_dev ? (*P.n_dev < P.n ? (uint64_t) *P.n_dev : P.n) : P.n;
  // tuning: kDbgRotate hands block b the tiles of block b + 1 (does a slow
  // XCD follow its hardware or its data?  Its hardware: profiles/r02_wave_stamps_c2.jsonl)
  const uint64_t gw = dbg_on(P, kDbgRotate) ? (gw_hw + WPB) % nwaves : gw_hw;
  uint64_t end, step;
  uint64_t first;
  if (RANGES) {
    first = gw * n_all / nwaves;
    end = (gw + 1) * n_all / nwaves;
    step = kWave;
  } else {
    first = gw * kWave;
    end = n_all;
    step = nwaves * kWave;
  }
  auto nvalid_of = [&](uint64_t b) __attribute__((always_inline)) -> uint32_t {
    return b < end ? (uint32_t) (end - b < (uint64_t) kWave ? end - b : (uint64_t) kWave) : 0u;
  };
  auto desc_of = [&](uint64_t b) __attribute__((always_inline)) -> uint64_t {
    return lane < nvalid_of(b) ? P.desc[b + lane] : 0ull;
  };
  // descriptors are prefetched one tile ahead
  uint64_t d_next = desc_of(first + step);
  Tile cur = make_tile<CONTIG>(first, nvalid_of(first), desc_of(first));
  uint64_t held_b[HOLD > 0 ? HOLD : 1];
  uint32_t held_v[HOLD > 0 ? HOLD : 1], held_c[HOLD > 0 ? HOLD : 1], held_h[HOLD > 0 ? HOLD : 1];
  int hold_n = 0;
  uint8_t* ring = base_b + P.ring_off + (uint32_t) w * P.hold_r * kRingTileBytes;
  uint32_t ring_n = 0;
  uint64_t ring_base0 = 0;
  TileOut pend;
  pend.valid = 0;
  pend.pid = 0;
  pend.cs = pend.h = pend.q = pend.l34 = 0;

  // wave-uniform descriptor inputs of a contiguous tile (readfirstlane: provably scalar)
  auto tile_rsrc = [&](const Tile& t) __attribute__((always_inline)) {
    const uint64_t tb = reinterpret_cast<uint64_t>(P.frames) + (uint64_t) t.D * 16u;
    const uint32_t tb_lo = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) tb);
    const uint32_t tb_hi = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (tb >> 32));
    const uint32_t tbytes = (uint32_t) __builtin_amdgcn_readfirstlane((int) (t.total * 16u));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t) tb_hi << 32) | tb_lo), (short) 0,
                                             (int) tbytes, 0x00020000);
  };
  // a contiguous tile's first batch: clear both slot windows, scatter, load
  ContigBatch<U> A, B;
  auto tile_first = [&](const Tile& t, __amdgpu_buffer_rsrc_t r) __attribute__((always_inline)) {
    for (uint32_t i = lane; i < (uint32_t) (2 * kWave * U); i += kWave) L.slotsA[i] = 0u;
    __builtin_amdgcn_wave_barrier();
    plan_contig<U, (CPOL >= 0 ? CPOL : (NT ? 2 : 0))>(A, L.slotsA, 0, lane, t.start, t.nch, t.info, r);
  };
  bool pre = false;  // (XPF) A already holds cur's first batch
  __amdgpu_buffer_rsrc_t rsrc_pre = tile_rsrc(cur);
  while (cur.nvalid != 0u) {
    if (cur.contig && cur.total != 0u) {
      // Contiguous tile: chunk c is absolute chunk D + c.  Ping-pong: batch
      // i+1's loads are in flight while batch i is reduced; every plan is
      // unconditional (positions past the end read zeros through the buffer
      // bounds check) so the compiler keeps counted vmcnt waits.
      const __amdgpu_buffer_rsrc_t rsrc = pre ? rsrc_pre : tile_rsrc(cur);
      // A counted loop over pairs of batches with its only exit at the bottom
      // (a mid-loop break made the wait-count pass drain vmcnt to 0 at the
      // loop header); an odd last batch is processed after the loop.
      uint32_t run = 0, b0 = 0;
      const uint32_t nbatch = (cur.total + kStep - 1) / kStep;
      if (!pre) tile_first(cur, rsrc);
      if (DEFER) {
        __builtin_amdgcn_sched_barrier(0);  // the previous tile's stores after this tile's first loads
        store_out<SST>(P, pend, L.want_rss);
      }
      uint32_t bi = 0;
      for (; bi + 1 < nbatch; bi += 2, b0 += 2 * kStep) {
        plan_contig<U, (CPOL >= 0 ? CPOL : (NT ? 2 : 0))>(B, L.slotsB, b0 + kStep, lane, cur.start, cur.nch, cur.info, rsrc);
        __builtin_amdgcn_sched_barrier(0);  // B's loads issue before A's wait
        run = process_contig<U>(A, L.slotsA, L.masks, run, L.E, L.hdr, L.stage, lane);
        plan_contig<U, (CPOL >= 0 ? CPOL : (NT ? 2 : 0))>(A, L.slotsA, b0 + 2 * kStep, lane, cur.start, cur.nch, cur.info, rsrc);
        __builtin_amdgcn_sched_barrier(0);
        run = process_contig<U>(B, L.slotsB, L.masks, run, L.E, L.hdr, L.stage, lane);
      }
      if (bi < nbatch) run = process_contig<U>(A, L.slotsA, L.masks, run, L.E, L.hdr, L.stage, lane);
    } else if (GEN && cur.total != 0u) {
      run_general_tile<U, NT, DEFER, SST>(P, L, cur, lane, tag, pend);
    } else if (DEFER) {
      store_out<SST>(P, pend, L.want_rss);
    }
    const uint64_t nb = cur.base + step;
    const Tile nxt = make_tile<CONTIG>(nb, nvalid_of(nb), d_next);
    pre = false;
    if (XPF && nxt.contig && nxt.total != 0u && nxt.total <= P.xpf_chunks) {
      rsrc_pre = tile_rsrc(nxt);
      tile_first(nxt, rsrc_pre);
      __builtin_amdgcn_sched_barrier(0);  // the next tile's loads go out before this tile's epilogue
      pre = true;
    }
    const TileOut o = tile_epilogue(P, L, cur, lane);
    if constexpr (RING) {
      if (P.out_l34 != nullptr) P.out_l34[o.pid] = (uint8_t) o.l34;
      if (ring_n == P.hold_r) {
        flush_ring<SST>(P, L, ring, ring_n, ring_base0, step, lane, nvalid_of);
        ring_n = 0;
      }
      if (ring_n == 0) ring_base0 = cur.base;
      uint8_t* slot = ring + ring_n * kRingTileBytes;
      reinterpret_cast<uint32_t*>(slot)[lane] = o.h;
      reinterpret_cast<uint16_t*>(slot + kWave * 4)[lane] = (uint16_t) o.cs;
      reinterpret_cast<uint16_t*>(slot + kWave * 6)[lane] = (uint16_t) o.q;
      ++ring_n;
    } else if constexpr (HOLD > 0) {
      if (P.out_l34 != nullptr) {
        store_out<SST>(P, o, L.want_rss);
      } else {
        if (hold_n == HOLD) {
#pragma unroll
          for (int i = 0; i < HOLD; ++i) store_out<SST>(P, held_out(held_b[i], held_v[i], held_c[i], held_h[i], lane), L.want_rss);
          hold_n = 0;
        }
#pragma unroll
        for (int i = 0; i < HOLD; ++i)
          if (i == hold_n) {
            held_b[i] = cur.base;
            held_v[i] = cur.nvalid;
            held_c[i] = o.cs | (o.q << 16);
            held_h[i] = o.h;
          }
        ++hold_n;
      }
    } else if (DEFER) {
      pend = o;
    } else {
      store_out<SST>(P, o, L.want_rss);
    }
    cur = nxt;
    d_next = desc_of(nb + step);
  }

  if (DEFER) store_out<SST>(P, pend, L.want_rss);
  if constexpr (RING) flush_ring<SST>(P, L, ring, ring_n, ring_base0, step, lane, nvalid_of);
  if constexpr (HOLD > 0) {
#pragma unroll
    for (int i = 0; i < HOLD; ++i)
      if (i < hold_n) store_out<SST>(P, held_out(held_b[i], held_v[i], held_c[i], held_h[i], lane), L.want_rss);
  }
  if (L.hist_lds && !dbg_on(P, kDbgNoFlush))
    flush_hist(L.hist, P.table_n, P.out_hits, P.hits_rep, P.hits_done, kWave * WPB);
#ifdef NICGPU_TUNING
  if (P.stamps != nullptr && lane == 0) {  // vector stores from lane 0
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    P.stamps[4 * gw_hw + 0] = t_start;
    P.stamps[4 * gw_hw + 1] = t_end;
    P.stamps[4 * gw_hw + 2] = (unsigned) __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID[3:0]
    P.stamps[4 * gw_hw + 3] = (unsigned) __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
  }
#endif
}

// ------------------------------------------------------- RSS, headers only --
// nicgpu_rx_offload with neither checksums nor L3/L4 flags requested (the
// batched stage's dispatch, RssEngine::select_queue_batch): the hash and the
// queue depend on a packet's headers only, so a batch need not stream its
// frames.  One lane per packet loads the packet's first kHdrChunks chunks (the
// ones inside it) into the same per-wave header stage rx_offload_kernel fills
// and runs the same rss_hash_packet — bytes past the stage come from global
// memory there as well — then the table lookup and the LDS histogram.  About
// 48 B read per packet instead of the whole frame.
__host__ __device__ inline uint32_t rss_only_block_bytes(uint32_t lut_words, uint32_t hist_n, uint32_t table_words) {
  return (lut_words * 4u + hist_n * 4u + table_words * 4u + 15u) & ~15u;
}
constexpr uint32_t kRssOnlyWaveBytes = (uint32_t) kWave * kHdrStride * 16u;
constexpr int kRssWpb = 16;  // waves per block: more header gathers in flight per CU, 1/4 of the flushes of 4

template <int WPB>  // waves per block
__global__ __launch_bounds__(kWave * WPB) void rss_only_kernel(RxParams P) {
  constexpr uint32_t kThreads = kWave * WPB;
  extern __shared__ uint4 lds_dyn[];
  const uint32_t w = (uint32_t) __builtin_amdgcn_readfirstlane((int) (threadIdx.x / kWave));
  const uint32_t lane = lane_id();
  const bool hist_lds = P.out_hits != nullptr && P.table_n <= (uint32_t) kHistLds;
  const bool table_lds = P.table_n <= (uint32_t) kTableLds;
  uint8_t* base_b = reinterpret_cast<uint8_t*>(lds_dyn);
  uint32_t* lut = reinterpret_cast<uint32_t*>(base_b);
  uint32_t* hist = lut + P.lut_words;
  uint16_t* table_s = reinterpret_cast<uint16_t*>(hist + (hist_lds ? P.table_n : 0u));
  const uint32_t block_bytes =
      rss_only_block_bytes(P.lut_words, hist_lds ? P.table_n : 0u, table_lds ? (P.table_n + 1u) / 2u : 0u);
  uint4* hdr = reinterpret_cast<uint4*>(base_b + block_bytes + w * kRssOnlyWaveBytes);
  for (uint32_t i = threadIdx.x; i < P.lut_words; i += kThreads) lut[i] = P.lut[i];
  if (hist_lds)
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kThreads) hist[i] = 0;
  if (table_lds)
    for (uint32_t i = threadIdx.x; i < P.table_n; i += kThreads) table_s[i] = P.table[i];
  __syncthreads();
  const uint64_t n_all = P.n_dev ? (*P.n_dev < P.n ? (uint64_t) *P.n_dev : P.n) : P.n;
  const uint64_t stride = (uint64_t) gridDim.x * WPB * kWave;
  auto desc_of = [&](uint64_t b) __attribute__((always_inline)) { return b + lane < n_all ? P.desc[b + lane] : 0ull; };
  // the header chunks inside the packet (none for an empty or absent one)
  auto load_hdr = [&](uint64_t d, u32x4* c) __attribute__((always_inline)) {
    const uint64_t off = d & kOffMask;
    const uint32_t len = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
    const uint32_t nch = len ? (uint32_t) (((off + len - 1) >> 4) - (off >> 4) + 1) : 0u;
    const u32x4* src = reinterpret_cast<const u32x4*>(P.frames + (off & ~15ull));
#pragma unroll
    for (int k = 0; k < kHdrChunks; ++k) c[k] = (uint32_t) k < nch ? src[k] : (u32x4){0u, 0u, 0u, 0u};
  };
  // software pipeline: tile b + stride's descriptors and headers are in flight
  // while tile b hashes, and tile b + 2 stride's descriptors behind them
  uint64_t b = ((uint64_t) blockIdx.x * WPB + w) * kWave;
  uint64_t d = desc_of(b), dn = desc_of(b + stride);
  u32x4 c[kHdrChunks];
  load_hdr(d, c);
  for (; b < n_all; b += stride) {
    __builtin_amdgcn_wave_barrier();  // the previous tile's stage reads are done
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int k = 0; k < kHdrChunks; ++k) hdr[hdr_slot(lane, (uint32_t) k)] = make_uint4(c[k].x, c[k].y, c[k].z, c[k].w);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const uint64_t dc = d;
    d = dn;
    dn = desc_of(b + 2 * stride);
    load_hdr(d, c);
    const uint64_t i = b + lane;
    if (i < n_all) {
      const uint64_t off = dc & kOffMask;
      const uint32_t len = (uint32_t) (dc >> NICGPU_DESC_OFFSET_BITS);
      const uint32_t h = rss_hash_packet(P, lut, HdrView{hdr, lane}, (uint32_t) (off & 15u), P.frames + off, len);
      const uint32_t idx = h % P.table_n;
      if (P.out_hash) P.out_hash[i] = h;
      if (P.out_queue) P.out_queue[i] = table_lds ? table_s[idx] : P.table[idx];
      if (P.out_hits) {
        if (hist_lds) atomicAdd(&hist[idx], 1u);
        else atomicAdd(&P.out_hits[idx], 1ull);
      }
    }
  }
  if (hist_lds) flush_hist(hist, P.table_n, P.out_hits, P.hits_rep, P.hits_done, kThreads);
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

// Per-frame TSO state (wave-uniform).  Byte positions are relative to the
// frame's first 16-B chunk a0; the frame is [fo, fo + L), the header
// [fo, fo + H), segment k's payload [fo + H + k*mss, ... + mss) clipped to L.
struct TsoFrame {
  uint64_t f;      // frame index
  uint64_t a0;     // absolute byte address of the first chunk (16-B aligned)
  uint32_t fo, L, H, mss, nseg, nsteps, valid, segmented, seg_base;
  float inv_mss;
};

// u16 element i of a uniform array through a scalar dword load (a vector
// u16 load would make hipcc drain vmcnt, i.e. the in-flight batch, at every
// frame).  An aligned dword never crosses a page, so the <= 2 bytes read past
// the element cannot fault; they are discarded.
__device__ __forceinline__ uint32_t scalar_u16(const uint16_t* a, uint64_t i) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(a + i);
  const uint32_t w = *reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t) 3);
  return (addr & 2u) ? (w >> 16) : (w & 0xFFFFu);
}

__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) x);
  const uint32_t hi = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (x >> 32));
  return ((uint64_t) hi << 32) | lo;
}

__device__ __forceinline__ TsoFrame tso_frame(const TsoParams& P, uint64_t f) {
  f = uniform64(f);  // wave-uniform by construction; makes the frame's loads scalar
  TsoFrame t{};
  t.f = f;
  t.valid = f < P.n ? 1u : 0u;
  if (!t.valid) return t;
  const uint64_t d = P.desc[f];
  const uint64_t off = d & kOffMask;
  t.L = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
  t.a0 = off & ~15ull;
  t.fo = (uint32_t) (off & 15u);
  t.mss = scalar_u16(P.mss, f);
  t.H = scalar_u16(P.hdr_len, f);
  t.segmented = (t.mss > 0u && t.L > t.mss && t.H < t.L) ? 1u : 0u;
  if (!t.segmented) t.H = t.L;  // one "segment" = the whole frame, all of it header
  t.nseg = t.segmented ? (t.L - t.H + t.mss - 1u) / t.mss : 1u;
  // TooManySegments: the host drops the frame; nothing is read or written
  t.nsteps = t.nseg > (uint32_t) kMaxSeg ? 0u : (t.fo + t.L + 1023u) / 1024u;
  t.inv_mss = t.segmented ? 1.0f / (float) t.mss : 0.0f;
  t.seg_base = P.seg_base[f];
  return t;
}

// One step = 64 chunks (1 KiB) of a frame, chunk c = lane.  Masks the bytes
// outside the frame, scans the chunk sums across the wave and records the
// frame prefix sum at every segment boundary x_k = fo + H + k*mss
// (k = 0..nseg-1; x_0 is the header's end) that falls in this lane's chunk:
// prefix(x) = run + (scan before this chunk) + (this chunk's bytes below x).
__device__ __forceinline__ uint32_t tso_step(const TsoFrame& t, u32x4 v, uint32_t step, uint32_t lane, uint32_t run,
                                             uint32_t* bnd) {
  const uint32_t cb = step * 1024u + lane * 16u;  // chunk start, frame-relative (a0 = 0)
  const uint32_t fe = t.fo + t.L;
  if (cb < t.fo || cb + 16u > fe) {
    const int lo = cb < t.fo ? (int) (t.fo - cb) : 0;
    const int hi = cb >= fe ? 0 : (cb + 16u > fe ? (int) (fe - cb) : 16);
    if (hi <= lo) {
      v = (u32x4){0u, 0u, 0u, 0u};
    } else {
      v.x &= dword_keep(lo, hi, 0);
      v.y &= dword_keep(lo, hi, 1);
      v.z &= dword_keep(lo, hi, 2);
      v.w &= dword_keep(lo, hi, 3);
    }
  }
  const uint32_t s = add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
  const uint32_t incl = wave_incl_scan(s);
  const uint32_t before = run + incl - s;
  if (t.segmented) {
    // first boundary at or after the chunk start: k = ceil((cb - x_0) / mss)
    const uint32_t x0 = t.fo + t.H;
    uint32_t k = 0;
    if (cb > x0) {
      const uint32_t rel = cb - x0;
      k = (uint32_t) ((float) rel * t.inv_mss);
      if (k * t.mss < rel) ++k;                      // float estimate off by at most one
      if (k > 0u && (k - 1u) * t.mss >= rel) --k;
    }
    for (; k < t.nseg; ++k) {
      const uint32_t x = x0 + k * t.mss;
      if (x >= cb + 16u) break;
      // bytes of this chunk below x (and inside the frame: already masked)
      const int hi = (int) (x - cb);
      uint32_t part = 0;
      if (hi > 0) {
        part = add_halves(v.x & dword_keep(0, hi, 0), 0u);
        part = add_halves(v.y & dword_keep(0, hi, 1), part);
        part = add_halves(v.z & dword_keep(0, hi, 2), part);
        part = add_halves(v.w & dword_keep(0, hi, 3), part);
      }
      bnd[k] = before + part;
    }
  }
  return run + (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
}

// Segment checksums of a finished frame from its boundary prefixes.
__device__ __forceinline__ void tso_finish(const TsoParams& P, const TsoFrame& t, uint32_t* bnd, uint32_t total,
                                           uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const uint32_t off_odd = t.fo & 1u;  // frames are 16-B aligned at a0
  const uint32_t hsum = fold16(t.segmented ? bnd[0] : total);
  const uint32_t hdr_be = off_odd ? hsum : bswap16(hsum);
  const uint32_t base = t.seg_base;
  for (uint32_t k = lane; k < t.nseg; k += kWave) {
    uint32_t tot;
    if (t.segmented) {
      const uint32_t hi = k + 1u < t.nseg ? bnd[k + 1u] : total;
      const uint32_t px = fold16(hi - bnd[k]);
      // payload byte at frame offset o sits at segment position o - k*mss
      const bool swap = ((k * t.mss + t.fo) & 1u) == 0u;
      tot = fold16(hdr_be + (swap ? bswap16(px) : px));
    } else {
      tot = hdr_be;
    }
    P.out[base + k] = (uint16_t) (~tot & 0xFFFFu);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// One wave per frame (f = wave, wave + W, ...).  All of a frame's chunks are
// requested at once — kTsoSteps loads of 16 B per lane cover 9 KiB, a whole
// MTU-9000 jumbo frame — and reduced in order with counted vmcnt waits; frames
// beyond that repeat the group.  Straight-line code (unconditional loads
// through a per-frame buffer resource whose reads past the frame return
// zeros) keeps the waits counted.  Frame sums are mod 2^32 prefix differences:
// exact below 64 KiB.
//
// Boundaries (mss >= 16: at most one per chunk): before a group's loads, lane
// k < nseg writes k + 1 into the group's LDS slot of the chunk holding x_k;
// in each step a chunk lane reads its slot and, only if it holds a boundary,
// adds the masked bytes below x_k (one LDS mask read) to its exclusive prefix.
// mss < 16 frames (several boundaries per chunk) take tso_step's search.
constexpr int kTsoSteps = 9;
constexpr uint32_t kTsoWindow = (uint32_t) kTsoSteps * kWave;  // chunks per group

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tso_rsrc(const TsoParams& P, const TsoFrame& t) {
  const uint64_t a = reinterpret_cast<uint64_t>(P.frames) + t.a0;
  const uint32_t lo = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) a);
  const uint32_t hi = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (a >> 32));
  const uint32_t nb = (uint32_t) __builtin_amdgcn_readfirstlane((int) ((t.fo + t.L + 15u) & ~15u));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t) hi << 32) | lo), (short) 0, (int) nb,
                                           0x00020000);
}

// Fast step (mss >= 16 or unsegmented): c = group-relative chunk of this lane.
__device__ __forceinline__ uint32_t tso_step_slots(const TsoFrame& t, u32x4 v, uint32_t gchunk0, uint32_t c,
                                                   uint32_t lane, uint32_t run, uint32_t* bnd, uint32_t* slots,
                                                   const uint4* masks) {
  const uint32_t chunk = gchunk0 + c;  // frame-relative chunk index
  const uint32_t clast = (t.fo + t.L + 15u) / 16u - 1u;  // last chunk holding frame bytes (L > 0 here)
  if (chunk == 0u || chunk == clast) {
    const uint32_t lo = chunk == 0u ? t.fo : 0u;
    const uint32_t hi = chunk == clast ? ((t.fo + t.L - 1u) & 15u) + 1u : 16u;
    const uint4 a = masks[lo], b = masks[16u + hi];
    v.x &= a.x & b.x;
    v.y &= a.y & b.y;
    v.z &= a.z & b.z;
    v.w &= a.w & b.w;
  }
  const uint32_t s = add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
  const uint32_t incl = wave_incl_scan(s);
  const uint32_t sl = slots[c];
  if (sl != 0u) {
    slots[c] = 0u;
    const uint32_t k = sl - 1u;
    const uint32_t hi = (t.fo + t.H + k * t.mss) & 15u;  // bytes of this chunk below x_k
    const uint4 m = masks[16u + hi];
    uint32_t part = add_halves(v.x & m.x, 0u);
    part = add_halves(v.y & m.y, part);
    part = add_halves(v.z & m.z, part);
    part = add_halves(v.w & m.w, part);
    bnd[k] = run + incl - s + part;
  }
  (void) lane;
  return run + (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
}

__global__ __launch_bounds__(kBlock) void tso_checksum_kernel(TsoParams P) {
  __shared__ uint32_t bnd_s[kWavesPerBlock][kMaxSeg + 1];
  __shared__ uint32_t slots_s[kWavesPerBlock][kTsoWindow];
  __shared__ uint4 masks[kMaskEntries];
  for (uint32_t i = threadIdx.x; i < kMaskEntries; i += kBlock) {
    const int lo = i < 16u ? (int) i : 0, hi = i < 16u ? 16 : (int) i - 16;
    masks[i] = make_uint4(dword_keep(lo, hi, 0), dword_keep(lo, hi, 1), dword_keep(lo, hi, 2), dword_keep(lo, hi, 3));
  }
  const int w = __builtin_amdgcn_readfirstlane((int) (threadIdx.x / kWave));  // provably wave-uniform: scalar frame state
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < kTsoWindow; i += kWave) slots_s[w][i] = 0u;
  __syncthreads();
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;
  uint32_t* bnd = bnd_s[w];
  uint32_t* slots = slots_s[w];
  for (uint64_t f = (uint64_t) blockIdx.x * kWavesPerBlock + w; f < P.n; f += nwaves) {
    const TsoFrame t = tso_frame(P, f);
    if (t.nseg > (uint32_t) kMaxSeg) continue;  // TooManySegments: the host drops the frame
    const __amdgpu_buffer_rsrc_t rs = tso_rsrc(P, t);
    const bool fast = !t.segmented || t.mss >= 16u;
    uint32_t run = 0;
    for (uint32_t g = 0; g < t.nsteps; g += kTsoSteps) {
      u32x4 v[kTsoSteps];
#pragma unroll
      for (int i = 0; i < kTsoSteps; ++i)
        v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, (int) (lane * 16u), (int) ((g + (uint32_t) i) * 1024u), 2));
      if (fast) {
        // this group's boundaries into its slot window
        const uint32_t c0 = g * 64u;
        if (t.segmented)
          for (uint32_t k = lane; k < t.nseg; k += kWave) {
            const uint32_t ck = (t.fo + t.H + k * t.mss) >> 4;
            if (ck >= c0 && ck < c0 + kTsoWindow) slots[ck - c0] = k + 1u;
          }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int i = 0; i < kTsoSteps; ++i)
          run = tso_step_slots(t, v[i], c0, (uint32_t) i * 64u + lane, lane, run, bnd, slots, masks);
      } else {
#pragma unroll
        for (int i = 0; i < kTsoSteps; ++i) run = tso_step(t, v[i], g + (uint32_t) i, lane, run, bnd);
      }
    }
    tso_finish(P, t, bnd, run, lane);
  }
}

// ------------------------------------------------------------ host side --
// Kernel variants: (loads in flight per lane U, nontemporal loads, waves per
// block, contiguous-tile path, ranges, occupancy hint, deferred stores, load
// cache policy, store cache policy).  Variant 0 is the production choice (tools/tune_rx.py measures the
// others against it on the GPU; DESIGN.md §4 records the result).
struct RxVariant {
  void (*kernel)(RxParams);
  int unroll;
  int wpb;
  const char* name;
  bool ranges = false;  // balanced per-wave packet ranges (grid sized by packets, not tiles)
  bool ring = false;    // LDS result ring (P.hold_r, P.ring_off sized at launch)
  bool xpf = false;     // cross-tile prefetch (P.xpf_chunks)
};

const RxVariant kRxVariants[] = {
    // 0 and 1: production; for variant 0 launch_rx picks plain stores (1) when
    // the ring holds all of a wave's tiles (every write lands after the reads:
    // C2 -1%) and sc1 stores (0) when the ring is flushed mid-stream (IMIX -3%).
    // Both prefetch the next tile's first batch (XPF: 64 B -1..4%, C2 / IMIX /
    // 9000 B within noise).
    // OCC 4: at most 128 VGPRs, the 4 waves per SIMD the LDS allows anyway
    // (left free, hipcc took variant 1 to 129 VGPRs with the histogram
    // replicas' flush: 3 waves per SIMD)
    {rx_offload_kernel<2, true, 4, true, false, 4, false, -1, 16, 0, true, true, true>, 2, 4, "u2_w4_c_sc1_ring_xpf", false, true, true},
    {rx_offload_kernel<2, true, 4, true, false, 4, false, -1, 0, 0, true, true, true>, 2, 4, "u2_w4_c_ring_xpf", false, true, true},
    // 2: production for batches of at least kRxW8Tiles tiles.  8-wave blocks:
    // half the blocks add their histogram bins into the same counters at the
    // end (1024 -> 512 same-address atomics per bin).  IMIX (4 M packets) -2%,
    // 4 M x 64 B -3%; C2 +0.6% and 9000 B +15% (2500 tiles underfill 512
    // slots of 8 waves) keep 4-wave blocks (profiles/r02y_tune_variants.json).
    {rx_offload_kernel<2, true, 8, true, false, 4, false, -1, 16, 0, true, true, true>, 2, 8, "u2_w8_c_sc1_ring_xpf", false, true, true},
#ifdef NICGPU_TUNING
    // candidates and earlier production kernels, timed by tools/tune_rx.py.
    // 8-wave blocks measure the same on C2/IMIX/64 B and 12% slower on 9000 B,
    // whose 2500 tiles underfill 512 slots of 8 waves.
    {rx_offload_kernel<2, true, 8, true, false, 1, false, -1, 16, 0, true>, 2, 8, "u2_nt1_w8_c_sc1_ring", false, true},
    // deeper per-wave batches for lower occupancies (nicgpu_tune_set_bpc)
    {rx_offload_kernel<4, true, 4, true, false, 1, false, -1, 16, 0, true, true, true>, 4, 4, "u4_w4_c_sc1_ring_xpf", false, true, true},
    {rx_offload_kernel<4, true, 4, true, false, 1, false, -1, 0, 0, true, true, true>, 4, 4, "u4_w4_c_ring_xpf", false, true, true},
    {rx_offload_kernel<2, true, 4, true, false, 1, false, -1, 16, 0, true>, 2, 4, "u2_nt1_w4_c_sc1_ring", false, true},
    {rx_offload_kernel<2, true, 4, true, false, 1, false, -1, 0, 0, true>, 2, 4, "u2_nt1_w4_c_ring", false, true},
    {rx_offload_kernel<2, true, 4, true, false, 1, true, -1, 16>, 2, 4, "u2_nt1_w4_c_sc1_defer"},
    {rx_offload_kernel<2, true, 4, true, false, 1, false>, 2, 4, "u2_nt1_w4_c"},
    {rx_offload_kernel<2, true, 4, false, false, 1, false, -1, 16, 0, true>, 2, 4, "u2_nt1_w4_sc1_ring", false, true},
    // bigger blocks still: 256 same-address atomics per bin
    {rx_offload_kernel<2, true, 16, true, false, 1, false, -1, 16, 0, true, true, true>, 2, 16, "u2_w16_c_sc1_ring_xpf", false, true, true},
#endif
};
constexpr int kNumRxVariants = (int) (sizeof(kRxVariants) / sizeof(kRxVariants[0]));
constexpr int kRxW8 = 2;
constexpr uint64_t kRxW8Tiles = 32768;  // 2 M packets: IMIX and 64-B batches of C3's size, not C2 (16 K tiles)

// ------------------------------------------------------ segment gather --
// The DMA writes of the batched QueuePair stage (QueuePair::handle_rx_segment,
// src/queue_pair.cpp:416-426): dst <- prefix (0/4 B, the inserted VLAN tag)
// || [src_a, +len_a) || [src_b, +len_b), all inside one memory image.  One
// wave per write.  Whole destination dwords are assembled from two aligned
// source dwords with v_alignbyte (16 B per lane per step, lanes contiguous,
// wave_copy16); the partial dwords at the ends of each part are written with
// byte stores, so writes that share a dword never race.  Pure byte movement:
// HBM-bound at 2 x bytes.
struct GatherParams {
  uint8_t* mem;
  const uint8_t* src;  // sources: mem itself, or a copy of it
  uint64_t mem_size;
  const nicgpu_segment_write* w;
  size_t n;
};

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

// wave_copy for the gather: each lane moves 16 B per step with one dwordx4
// load and store (4-B aligned: the sources and destinations of segment writes
// have any byte alignment; whole dwords are assembled as in wave_copy), the
// fifth source dword of the byte shift from the next lane.  Sources are
// clamped to the image, whose end need not be 16-B padded.
__device__ void wave_copy16(uint8_t* dmem, uint64_t dst, const uint8_t* smem, uint64_t smem_size, uint64_t src,
                            uint64_t len, uint32_t lane) {
  if (len == 0) return;
  const uint64_t d1 = dst + len;
  const uint64_t A = (dst + 3) & ~3ull;
  const uint64_t B = d1 & ~3ull;
  if (A >= B) {
    if (lane < len) dmem[dst + lane] = smem[src + lane];
    return;
  }
  const uint64_t head = A - dst, tail = d1 - B;
  if (lane < head) dmem[dst + lane] = smem[src + lane];
  if (lane >= 8 && lane - 8 < tail) dmem[B + (lane - 8)] = smem[src + (B - dst) + (lane - 8)];
  const uint64_t nw = (B - A) >> 2;
  const uint64_t s0 = src + head;
  const uint32_t sh = (uint32_t) (s0 & 3);
  const uint64_t sa = s0 & ~3ull;
  const uint64_t steps = (nw + 255) / 256;  // wave-uniform trip count (the shuffle needs every lane)
  for (uint64_t k = 0; k < steps; ++k) {
    const uint64_t i = k * 256 + (uint64_t) lane * 4;
    const uint64_t a = sa + 4 * i;
    uint32_t v[5] = {0, 0, 0, 0, 0};
    if (i < nw) {
      if (a + 16 <= smem_size) {
        __builtin_memcpy(v, smem + a, 16);  // dword-aligned dwordx4 (gfx950 unaligned access mode)
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = load_dword_clamped(smem, smem_size, a + 4 * j);
      }
    }
    const uint32_t up = (uint32_t) __builtin_amdgcn_ds_bpermute((int) (((lane + 1) & 63) << 2), (int) v[0]);
    if (i < nw && sh) v[4] = (lane < 63 && i + 4 < nw) ? up : (i + 4 <= nw ? load_dword_clamped(smem, smem_size, a + 16) : 0u);
    if (i < nw) {
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = sh ? __builtin_amdgcn_alignbyte(v[j + 1], v[j], sh) : v[j];
      uint8_t* d = dmem + A + 4 * i;
      if (i + 4 <= nw) {
        __builtin_memcpy(d, o, 16);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (i + j < nw) reinterpret_cast<uint32_t*>(d)[j] = o[j];
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void segment_gather_kernel(GatherParams P) {
  const uint32_t lane = lane_id();
  const uint64_t wave = (uint64_t) blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;
  // the next write's entry is loaded while this one copies (one memory
  // latency per write instead of two)
  nicgpu_segment_write next{};
  if (wave < P.n) next = P.w[wave];
  for (uint64_t e = wave; e < P.n; e += nwaves) {
    const nicgpu_segment_write w = next;
    if (e + nwaves < P.n) next = P.w[e + nwaves];
    const uint64_t plen = w.prefix_len == 4 ? 4 : 0;
    const uint64_t total = plen + w.len_a + w.len_b;
    // entries outside the image are skipped (the host validated them)
    if (w.prefix_len > 4 || w.dst > P.mem_size || total > P.mem_size - w.dst || w.src_a > P.mem_size ||
        w.len_a > P.mem_size - w.src_a || w.src_b > P.mem_size || w.len_b > P.mem_size - w.src_b)
      continue;
    if (lane < plen) P.mem[w.dst + lane] = (uint8_t) (w.prefix >> (8 * lane));
    wave_copy16(P.mem, w.dst + plen, P.src, P.mem_size, w.src_a, w.len_a, lane);
    wave_copy16(P.mem, w.dst + plen + w.len_a, P.src, P.mem_size, w.src_b, w.len_b, lane);
  }
}

// --------------------------------------------- fused delivery (row f1) --
// The batched QueuePair stage's DMA writes and the RSS of the frames they
// deliver in one launch (nicgpu_qp_deliver).  A wave takes a tile of 64 RX
// completions and walks their bytes as ONE stream of destination 16-B chunks,
// as the RX kernel walks packets: every write splits into up to three items
// (VLAN prefix, part A, part B — queue_pair.cpp:352-359, 392-395, 416-426
// already resolved into the write), every item into the destination chunks it
// touches, and lane l of a step takes stream entry base + l.  So one wave
// instruction moves up to 1 KiB whatever the frame sizes (the one-wave-per-
// write gather left 60 of 64 lanes idle on 64-B frames and kept one write's
// load latency per wave in flight).  A chunk's source is five dwords from the
// item's source at the chunk's byte shift; whole chunks are one 16-B store,
// item edges dword or byte stores, so no byte outside a segment is written.
//
// RSS: for a completion with status Success, the lanes whose chunk lies in its
// frame's first three destination chunks also OR their bytes into the wave's
// header stage (the RX kernel's 48-B-per-packet layout), and after the tile
// the owning lane hashes the frame from the stage exactly as rss_only_kernel
// (rss_hash_packet; bytes past the stage, rare, from the frame just written).
// The hash and queue land per completion (0 / 0xFFFF for the others), the
// table-index hits in a block histogram, the Success count in *count — what
// qp_flag/qp_rss_fill, the RSS launch and qp_scatter produced in four launches
// with the headers read back from HBM.
struct DeliverParams {
  uint8_t* mem;
  uint64_t mem_size;
  const nicgpu_segment_write* w;
  const nicgpu_completion* rxc;  // statuses (RSS of Success completions)
  uint64_t j0, n;                // completions [j0, n) ...
  const unsigned long long* n_dev;  // ... with n lowered to *n_dev (a speculative resolve's settled prefix)
  RxParams rss;                  // mode NICGPU_TUPLE_NONE: no RSS
  uint32_t* rx_hash;
  uint16_t* rx_queue;
  unsigned long long* hits;
  unsigned long long* count;
};

#ifndef NICGPU_DLV_WPB
#define NICGPU_DLV_WPB 8
#endif
#ifndef NICGPU_DLV_U
#define NICGPU_DLV_U 4
#endif
#ifndef NICGPU_DLV_RESERVE
#define NICGPU_DLV_RESERVE 0
#endif
constexpr int kDlvReserveCus = NICGPU_DLV_RESERVE;  // default of NICGPU_DLV_RESERVE_CUS (tuning)
constexpr int kDlvWpb = NICGPU_DLV_WPB;  // waves per block
constexpr int kDlvU = NICGPU_DLV_U;      // 64-entry sub-steps per step (loads in flight per lane)
constexpr uint32_t kDlvRec = 24;  // item record: dst u64 | src (or prefix word) u64 | len u32 | first entry u32
constexpr uint32_t kDlvMarks = (kWave * kDlvU + 15u) & ~15u;  // bytes: one u8 mark per stream entry (item id + 1 <= 192)
constexpr uint32_t kDlvWaveBytes = kDlvMarks + 64u * 8u + 192u * kDlvRec + 64u * kHdrStride * 16u;  // marks|wdst|items|stage

// block part: RSS LUT | histogram | table (as rss_only_kernel), then 16 B for the Success count
__host__ __device__ inline uint32_t dlv_block_bytes(bool rss, uint32_t lut_words, uint32_t hist_n,
                                                    uint32_t table_words) {
  return (rss ? rss_only_block_bytes(lut_words, hist_n, table_words) : 0u) + 16u;
}

__device__ __forceinline__ uint32_t dlv_chunks(uint64_t d, uint64_t n) {
  return n ? (uint32_t) (((d + n - 1) >> 4) - (d >> 4) + 1) : 0u;
}

// Stores the bytes [lo, hi) (absolute) of the 16-B destination chunk at D
// from o; whole chunk: one 16-B store, else whole dwords and bytes.
__device__ __forceinline__ void dlv_store(uint8_t* mem, uint64_t D, uint64_t lo, uint64_t hi, const uint32_t* o) {
  if (lo == D && hi == D + 16) {
    u32x4 v = {o[0], o[1], o[2], o[3]};
    *reinterpret_cast<u32x4*>(mem + D) = v;
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t a = D + 4u * i;
    if (a >= lo && a + 4 <= hi) {
      *reinterpret_cast<uint32_t*>(mem + a) = o[i];
    } else if (a + 4 > lo && a < hi) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (a + b >= lo && a + b < hi) mem[a + b] = (uint8_t) (o[i] >> (8 * b));
    }
  }
}

template <bool RSS>
__global__ __launch_bounds__(kWave * kDlvWpb) __attribute__((amdgpu_waves_per_eu(4, 8))) void deliver_kernel(DeliverParams P) {
  constexpr uint32_t kThreads = kWave * kDlvWpb;
  extern __shared__ uint4 lds_dyn[];
  const uint32_t w = (uint32_t) __builtin_amdgcn_readfirstlane((int) (threadIdx.x / kWave));
  const uint32_t lane = lane_id();
  const RxParams& R = P.rss;
  const bool hist_lds = RSS && R.table_n <= (uint32_t) kHistLds;
  const bool table_lds = RSS && R.table_n <= (uint32_t) kTableLds;
  uint8_t* base_b = reinterpret_cast<uint8_t*>(lds_dyn);
  uint32_t* lut = reinterpret_cast<uint32_t*>(base_b);
  uint32_t* hist = lut + (RSS ? R.lut_words : 0u);
  uint16_t* table_s = reinterpret_cast<uint16_t*>(hist + (hist_lds ? R.table_n : 0u));
  const uint32_t block_bytes = dlv_block_bytes(RSS, R.lut_words, hist_lds ? R.table_n : 0u,
                                               table_lds ? (R.table_n + 1u) / 2u : 0u);
  uint32_t* cnt_s = reinterpret_cast<uint32_t*>(base_b + block_bytes - 16u);
  uint8_t* wave_b = base_b + block_bytes + w * kDlvWaveBytes;
  uint8_t* marks = wave_b;
  uint64_t* wdst = reinterpret_cast<uint64_t*>(wave_b + kDlvMarks);
  uint8_t* items = wave_b + kDlvMarks + 512u;
  uint4* stage = reinterpret_cast<uint4*>(items + 192u * kDlvRec);
  if (RSS) {
    for (uint32_t i = threadIdx.x; i < R.lut_words; i += kThreads) lut[i] = R.lut[i];
    if (hist_lds)
      for (uint32_t i = threadIdx.x; i < R.table_n; i += kThreads) hist[i] = 0;
    if (table_lds)
      for (uint32_t i = threadIdx.x; i < R.table_n; i += kThreads) table_s[i] = R.table[i];
    if (threadIdx.x == 0) *cnt_s = 0;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t) kHdrChunks; ++k) stage[hdr_slot(lane, k)] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  uint64_t n = P.n;
  if (P.n_dev) {
    const uint64_t m = *P.n_dev;
    n = m < n ? m : n;
  }
  const uint64_t ntiles = n > P.j0 ? (n - P.j0 + kWave - 1) / kWave : 0;
  const uint64_t nwaves = (uint64_t) gridDim.x * kDlvWpb;
  uint32_t my_count = 0;
  for (uint64_t tile = (uint64_t) blockIdx.x * kDlvWpb + w; tile < ntiles; tile += nwaves) {
    // ---- this lane's write: its items and their stream entries
    const uint64_t j = P.j0 + tile * kWave + lane;
    nicgpu_segment_write wr{};
    bool flag = false;
    if (j < n) {
      wr = P.w[j];
      if (RSS) flag = P.rxc[j].status == nicqp::kSuccess;
    }
    const uint64_t plen = wr.prefix_len == 4 ? 4 : 0;
    const uint64_t total = plen + wr.len_a + wr.len_b;
    // entries outside the image are skipped (the host validated them)
    const bool ok = j < n && !(wr.prefix_len > 4 || wr.dst > P.mem_size || total > P.mem_size - wr.dst ||
                                 wr.src_a > P.mem_size || wr.len_a > P.mem_size - wr.src_a ||
                                 wr.src_b > P.mem_size || wr.len_b > P.mem_size - wr.src_b);
    const uint64_t d1 = wr.dst + plen, d2 = d1 + wr.len_a;
    const uint32_t c0 = ok ? dlv_chunks(wr.dst, plen) : 0u;
    const uint32_t c1 = ok ? dlv_chunks(d1, wr.len_a) : 0u;
    const uint32_t c2 = ok ? dlv_chunks(d2, wr.len_b) : 0u;
    const uint32_t cw = c0 + c1 + c2;
    const uint32_t incl = wave_incl_scan(cw);
    const uint32_t F = incl - cw;
    const uint32_t total_e = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
    auto put = [&](uint32_t k, uint64_t d, uint64_t src, uint32_t len, uint32_t first) __attribute__((always_inline)) {
      uint8_t* r = items + (lane * 3u + k) * kDlvRec;
      *reinterpret_cast<uint64_t*>(r) = d;
      *reinterpret_cast<uint64_t*>(r + 8) = src;
      *reinterpret_cast<uint32_t*>(r + 16) = len;
      *reinterpret_cast<uint32_t*>(r + 20) = first;
    };
    put(0, wr.dst, wr.prefix, c0 ? 4u : 0u, F);
    put(1, d1, wr.src_a, c1 ? wr.len_a : 0u, F + c0);
    put(2, d2, wr.src_b, c2 ? wr.len_b : 0u, F + c0 + c1);
    wdst[lane] = (wr.dst >> 4) | (flag && ok ? 1ull << 63 : 0ull);
    // ---- the stream: kDlvU x 64 entries per step, every load of the step
    // issued before its first store (one memory latency per step)
    uint32_t carry = 0;  // item (id + 1) of the entry before this step
    for (uint32_t W = 0; W < total_e; W += kWave * kDlvU) {
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) marks[u * kWave + lane] = 0u;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      constexpr uint32_t kSpan = kWave * kDlvU;
      if (c0 && F >= W && F - W < kSpan) marks[F - W] = (uint8_t) (lane * 3u + 1u);
      if (c1 && F + c0 >= W && F + c0 - W < kSpan) marks[F + c0 - W] = (uint8_t) (lane * 3u + 2u);
      if (c2 && F + c0 + c1 >= W && F + c0 + c1 - W < kSpan) marks[F + c0 + c1 - W] = (uint8_t) (lane * 3u + 3u);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      uint32_t itv[kDlvU];
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) {
        uint32_t it = wave_incl_max(marks[u * kWave + lane]);
        it = it > carry ? it : carry;
        carry = (uint32_t) __builtin_amdgcn_readlane((int) it, 63);
        itv[u] = it;
      }
      // phase A: every entry's chunk, item and source window; loads issued.
      // Per entry: the destination chunk, one packed word (bytes [lo, hi) of
      // the chunk, source shift, owning write) and five source dwords — a
      // prefix item's 4 bytes are placed into them here — so that kDlvU
      // entries' loads fit in flight per lane.
      uint64_t Dc[kDlvU];  // destination chunk index; ~0: no entry
      uint32_t pk[kDlvU];  // lo - D (bits 0-4) | hi - D (8-12) | shift (16-17) | write q (20-25)
      uint32_t vv[kDlvU][5];
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) {
        const uint32_t pos = W + (uint32_t) u * kWave + lane;
        Dc[u] = ~0ull;
        pk[u] = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) vv[u][i] = 0;
        if (pos < total_e) {
          const uint32_t id = itv[u] - 1u, q = id / 3u, k = id - 3u * q;
          const uint8_t* r = items + id * kDlvRec;
          const uint64_t d = *reinterpret_cast<const uint64_t*>(r);
          const uint64_t src = *reinterpret_cast<const uint64_t*>(r + 8);
          const uint32_t len = *reinterpret_cast<const uint32_t*>(r + 16);
          const uint32_t first = *reinterpret_cast<const uint32_t*>(r + 20);
          const uint64_t D = ((d >> 4) + (pos - first)) << 4;
          const uint64_t lo = D > d ? D : d;
          const uint64_t hi = D + 16 < d + len ? D + 16 : d + len;
          Dc[u] = D >> 4;
          pk[u] = (uint32_t) (lo - D) | ((uint32_t) (hi - D) << 8) | (q << 20);
          if (k == 0) {
            // VLAN prefix 81 00 tag (queue_pair.cpp:352-359): its 4 bytes at d
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              uint32_t v = 0;
#pragma unroll
              for (int bb = 0; bb < 4; ++bb) {
                const int64_t rel = (int64_t) (D + 4u * i + bb) - (int64_t) d;
                if (rel >= 0 && rel < 4) v |= (uint32_t) ((src >> (8 * rel)) & 0xFFu) << (8 * bb);
              }
              vv[u][i] = v;
            }
          } else {
            // source of destination byte D: before the item's source by up to
            // 15 bytes on its first chunk, so possibly below address 0 (signed)
            const int64_t a = (int64_t) D + ((int64_t) src - (int64_t) d);
            const int64_t a4 = a & ~(int64_t) 3;
            pk[u] |= (uint32_t) (a & 3) << 16;
            if (a4 >= 0 && (uint64_t) a4 + 20 <= P.mem_size) {
              __builtin_memcpy(vv[u], P.mem + a4, 16);  // dword-aligned dwordx4 (gfx950 unaligned access mode)
              // the fifth dword only for a shifted window (equal alignment of
              // source and destination, the common case, needs four)
              vv[u][4] = (a & 3) ? *reinterpret_cast<const uint32_t*>(P.mem + a4 + 16) : 0u;
            } else {  // bytes outside the image read as 0 (never stored: outside [lo, hi))
#pragma unroll
              for (int i = 0; i < 5; ++i) {
                uint32_t x = 0;
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                  const int64_t e = a4 + 4 * i + bb;
                  if (e >= 0 && (uint64_t) e < P.mem_size) x |= (uint32_t) P.mem[e] << (8 * bb);
                }
                vv[u][i] = x;
              }
            }
          }
        }
      }
      // phase B: align, store, and the header stage of Success frames
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) {
        if (Dc[u] == ~0ull) continue;
        const uint64_t D = Dc[u] << 4, lo = D + (pk[u] & 31u), hi = D + ((pk[u] >> 8) & 31u);
        const uint32_t sh = (pk[u] >> 16) & 3u;
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = sh ? __builtin_amdgcn_alignbyte(vv[u][i + 1], vv[u][i], sh) : vv[u][i];
        dlv_store(P.mem, D, lo, hi, o);
        if (RSS) {
          const uint32_t q = pk[u] >> 20;
          const uint64_t wd = wdst[q];
          const uint64_t kc = Dc[u] - (wd & ~(1ull << 63));
          if ((wd >> 63) && kc < (uint64_t) kHdrChunks) {
            uint32_t* st = reinterpret_cast<uint32_t*>(stage + hdr_slot(q, (uint32_t) kc));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint64_t a = D + 4u * i;
              const int b0 = lo > a ? (int) (lo - a) : 0, b1 = hi < a + 4 ? (int) (hi - a) : 4;
              if (b1 > b0) atomicOr(st + i, o[i] & dword_keep(b0, b1, 0));
            }
          }
        }
      }
    }
    if (RSS) {
      // the frames' bytes are in the stage; bytes past it come from the frame
      // this wave just wrote (its stores retired first)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (j < n) {
        if (flag && ok) {
          uint64_t len = total;
          if (len > NICGPU_MAX_PACKET) len = NICGPU_MAX_PACKET;  // the tuple lies in the first 82 B
          const uint32_t h = rss_hash_packet(R, lut, HdrView{stage, lane}, (uint32_t) (wr.dst & 15u), P.mem + wr.dst,
                                             (uint32_t) len);
          const uint32_t idx = h % R.table_n;
          P.rx_hash[j] = h;
          P.rx_queue[j] = table_lds ? table_s[idx] : R.table[idx];
          if (hist_lds) atomicAdd(&hist[idx], 1u);
          else atomicAdd(&P.hits[idx], 1ull);
          ++my_count;
        } else {
          P.rx_hash[j] = 0u;
          P.rx_queue[j] = 0xFFFFu;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (uint32_t k = 0; k < (uint32_t) kHdrChunks; ++k) stage[hdr_slot(lane, k)] = make_uint4(0u, 0u, 0u, 0u);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  if (RSS) {
    const uint32_t c = (uint32_t) __builtin_amdgcn_readlane((int) wave_incl_scan(my_count), 63);
    if (lane == 0 && c) atomicAdd(cnt_s, c);
    __syncthreads();
    if (threadIdx.x == 0 && *cnt_s) atomicAdd(P.count, (unsigned long long) *cnt_s);
    if (hist_lds) flush_hist(hist, R.table_n, P.hits, R.hits_rep, R.hits_done, kThreads);
  }
}

// ------------------------------------------------- TSO/GSO segmentation --
// QueuePair::build_segments (src/queue_pair.cpp:212-278) plus the
// TX VLAN insert (:324-331) and RX VLAN strip (:389-395) that shape each
// delivered segment, materialised on the GPU.  One wave per frame walks its
// segments; segment g = seg_base[i] + k is written at out + g * stride and its
// length and compute_checksum (what handle_rx_segment verifies, :434-447) are
// reported.  The checksum is summed from the dwords the wave writes, so frame
// bytes are read once (the header once per segment, from L2) and written once.
struct TsoSegParams {
  const uint8_t* frames;
  const uint64_t* desc;
  const uint16_t* hdr_len;
  const uint16_t* mss;
  const uint32_t* seg_base;
  const uint32_t* flags;  // per frame: NICGPU_SEG_* | vlan tag (low 16 bits); may be null
  size_t n;
  uint8_t* out;
  uint64_t out_size;
  uint32_t stride;
  uint32_t* out_len;
  uint16_t* out_csum;
};

// A frame of up to kSegStage bytes (from its first 16-B chunk) is staged in
// LDS once — every chunk requested at once, 9 loads of 16 B per lane — and
// each segment is assembled from the stage: output dwords are written by
// consecutive lanes (256 B per store instruction), a dword that lies inside
// one part is two conflict-free LDS reads and a v_alignbyte, and only the few
// dwords that straddle a part boundary or the segment's ends are built (and,
// at the ends, stored) byte by byte.  Larger frames copy from global memory.
constexpr uint32_t kSegStageChunks = (uint32_t) kTsoSteps * kWave;
constexpr uint32_t kSegStage = kSegStageChunks * 16u;  // 9216 B


// One dword of a segment at absolute address A (4-aligned), any overlap with
// the segment: bytes from the prefix / part A / part B, byte stores at the
// segment's ends.  Returns its halfword sum (absolute positions).
__device__ __forceinline__ uint32_t seg_dword_bytes(uint8_t* out, uint64_t A, uint64_t dst, int sz, int pa, int pb,
                                                    uint32_t tag, const uint8_t* st_b, uint32_t a, uint32_t b) {
  const int r0 = (int) ((int64_t) A - (int64_t) dst);
  uint32_t o = 0, keep = 0;
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + q;
    if (r < 0 || r >= sz) continue;
    uint32_t val;
    if (r < pa) val = r == 0 ? 0x81u : (r == 1 ? 0u : (r == 2 ? (tag >> 8) & 0xFFu : tag & 0xFFu));
    else if (r < pb) val = st_b[a + (uint32_t) (r - pa)];
    else val = st_b[b + (uint32_t) (r - pb)];
    o |= val << (8 * q);
    keep |= 0xFFu << (8 * q);
  }
  uint8_t* p = out + A;
  if (keep == 0xFFFFFFFFu) {
    *reinterpret_cast<uint32_t*>(p) = o;
  } else {
    for (int q = 0; q < 4; ++q)
      if ((keep >> (8 * q)) & 0xFFu) p[q] = (uint8_t) (o >> (8 * q));
  }
  return (o & 0xFFFFu) + (o >> 16);
}

// Segment bytes: pl prefix bytes (81 00 tag), then stage[a, +la), then
// stage[b, ...); written to out[dst, +size) (size = pl + la + lb).  Returns
// this lane's share of their little-endian halfword sum at absolute positions.
//  pass 1: every 16-B-aligned destination block that lies inside part A or
//          part B — five LDS dwords, four v_alignbyte, one 16-B store, and
//          no branch but the inside test (per-dword branching had made the
//          kernel SALU-bound);
//  pass 2: lanes 0..15 take the dwords of the <= 4 blocks pass 1 leaves: the
//          segment's first and last blocks and the ones holding the part
//          boundaries pa and pb, byte by byte where a dword straddles.
__device__ __forceinline__ uint32_t seg_copy_stage(uint8_t* out, uint64_t dst, uint32_t size, uint32_t pl,
                                                   uint32_t tag, const uint8_t* st_b, uint32_t a, uint32_t la,
                                                   uint32_t b, uint32_t lane) {
  const uint32_t* st = reinterpret_cast<const uint32_t*>(st_b);
  const int pa = (int) pl, pb = (int) (pl + la), sz = (int) size;
  const uint64_t E = dst + size;
  const uint64_t D16 = (dst + 15) & ~15ull, E16 = E & ~15ull;
  const uint32_t nblk = E16 > D16 ? (uint32_t) ((E16 - D16) >> 4) : 0u;
  auto inside16 = [&](int r0) __attribute__((always_inline)) {
    return (r0 >= pb && r0 + 16 <= sz) || (r0 >= pa && r0 + 16 <= pb);
  };
  uint32_t sum = 0;
  for (uint32_t j = lane; j < nblk; j += kWave) {
    const int r0 = (int) (D16 - dst) + 16 * (int) j;
    const bool inB = r0 >= pb && r0 + 16 <= sz;
    const bool inA = r0 >= pa && r0 + 16 <= pb;
    if (inA || inB) {
      const uint32_t src = inB ? b + (uint32_t) (r0 - pb) : a + (uint32_t) (r0 - pa);
      const uint32_t k = src >> 2, sh = src & 3u;
      const uint32_t w0 = st[k], w1 = st[k + 1], w2 = st[k + 2], w3 = st[k + 3], w4 = st[k + 4];
      u32x4 o;
      o.x = sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
      o.y = sh ? __builtin_amdgcn_alignbyte(w2, w1, sh) : w1;
      o.z = sh ? __builtin_amdgcn_alignbyte(w3, w2, sh) : w2;
      o.w = sh ? __builtin_amdgcn_alignbyte(w4, w3, sh) : w3;
      *reinterpret_cast<u32x4*>(out + D16 + 16ull * j) = o;
      sum = add_halves(o.w, add_halves(o.z, add_halves(o.y, add_halves(o.x, sum))));
    }
  }
  if (lane < 16u) {
    const uint64_t blk[4] = {dst & ~15ull, (dst + (uint64_t) pa) & ~15ull, (dst + (uint64_t) pb) & ~15ull,
                             (E - 1) & ~15ull};
    const uint32_t g = lane >> 2;
    const uint64_t B = blk[g];
    bool dup = false;
    for (uint32_t q = 0; q < g; ++q) dup |= blk[q] == B;
    const bool pass1 = B >= D16 && B < E16 && inside16((int) ((int64_t) B - (int64_t) dst));
    const uint64_t A = B + 4ull * (lane & 3u);
    if (size != 0 && !dup && !pass1 && A + 4 > dst && A < E)
      sum += seg_dword_bytes(out, A, dst, sz, pa, pb, tag, st_b, a, b);
  }
  return sum;
}

__global__ __launch_bounds__(kBlock) void tso_segment_kernel(TsoSegParams P) {
  __shared__ uint4 stage_s[kWavesPerBlock][kSegStageChunks + 1];  // +1: stage_u32's second dword
  const int w = __builtin_amdgcn_readfirstlane((int) (threadIdx.x / kWave));
  const uint32_t lane = lane_id();
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;
  uint4* stage = stage_s[w];
  // The wave's frames are f0 + t * nwaves.  Their parameters are fetched 64 at
  // a time, one frame per lane, and broadcast with readlane: a per-frame
  // global load would make hipcc wait on vmcnt(0) — i.e. for the previous
  // segments' stores to complete — before every frame and every segment.
  const uint64_t f0 = (uint64_t) blockIdx.x * kWavesPerBlock + w;
  for (uint64_t t0 = 0; f0 + t0 * nwaves < P.n; t0 += kWave) {
    const uint64_t fl_i = f0 + (t0 + lane) * nwaves;
    const bool have = fl_i < P.n;
    const uint64_t d_l = have ? P.desc[fl_i] : 0ull;
    const uint32_t fl_l = have ? (P.flags ? P.flags[fl_i] : (uint32_t) NICGPU_SEG_TSO) : 0u;
    const uint32_t mh_l = have ? ((uint32_t) P.mss[fl_i] | ((uint32_t) P.hdr_len[fl_i] << 16)) : 0u;
    const uint32_t sb_l = have ? P.seg_base[fl_i] : 0u;
    const uint64_t left = (P.n - (f0 + t0 * nwaves) + nwaves - 1) / nwaves;
    const uint32_t cnt = left < (uint64_t) kWave ? (uint32_t) left : (uint32_t) kWave;
    uint32_t d_lo = (uint32_t) d_l, d_hi = (uint32_t) (d_l >> 32);
    uint32_t fl_v = fl_l, mh_v = mh_l, sb_v = sb_l;
    // consume the loads here, once: otherwise the wait-count pass keeps them
    // pending around the frame loop and drains vmcnt at every frame
    asm volatile("" : "+v"(d_lo), "+v"(d_hi), "+v"(fl_v), "+v"(mh_v), "+v"(sb_v));
  for (uint32_t t = 0; t < cnt; ++t) {
    const uint64_t d = ((uint64_t) (uint32_t) __builtin_amdgcn_readlane((int) d_hi, (int) t) << 32) |
                       (uint32_t) __builtin_amdgcn_readlane((int) d_lo, (int) t);
    const uint64_t off = d & kOffMask;
    const uint32_t L = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
    const uint32_t fl = (uint32_t) __builtin_amdgcn_readlane((int) fl_v, (int) t);
    const uint32_t tag = fl & 0xFFFFu;
    const uint32_t mh = (uint32_t) __builtin_amdgcn_readlane((int) mh_v, (int) t);
    const uint32_t mss = mh & 0xFFFFu;
    uint32_t H = mh >> 16;
    const uint32_t seg_base = (uint32_t) __builtin_amdgcn_readlane((int) sb_v, (int) t);
    // build_segments (:212-278)
    uint32_t nseg = 1;
    bool seg = (fl & NICGPU_SEG_TSO) && mss > 0 && L > mss;
    if (seg) {
      if (mss > 9000u || H > L) continue;  // InvalidMss: no segment
      if (H >= L) {
        seg = false;  // degenerate: one unsegmented copy
      } else {
        nseg = (L - H + mss - 1) / mss;
        if (nseg > 64u) continue;  // TooManySegments
      }
    }
    if (!seg) H = L;
    const bool insert = fl & NICGPU_SEG_VLAN_INSERT;
    const bool has_vlan = insert || (fl & NICGPU_SEG_VLAN_PRESENT);
    const uint64_t a0 = off & ~15ull;
    const uint32_t fo = (uint32_t) (off & 15u);
    const bool staged = fo + L <= kSegStage;
    if (staged) {
      const uint64_t ab = reinterpret_cast<uint64_t>(P.frames) + a0;
      const uint32_t nb = (fo + L + 15u) & ~15u;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(uniform64(ab)), (short) 0, __builtin_amdgcn_readfirstlane((int) nb), 0x00020000);
      u32x4 v[kTsoSteps];
#pragma unroll
      for (int c = 0; c < kTsoSteps; ++c)
        v[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int) (lane * 16u),
                                                                                (int) ((uint32_t) c * 1024u), 2));
      __builtin_amdgcn_wave_barrier();  // the previous frame's stage reads are done
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int c = 0; c < kTsoSteps; ++c) stage[c * kWave + (int) lane] = make_uint4(v[c].x, v[c].y, v[c].z, v[c].w);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    for (uint32_t k = 0; k < nseg; ++k) {
      const uint32_t clen = seg ? min(mss, L - H - k * mss) : 0u;
      const uint64_t base_len = (uint64_t) H + clen;
      uint64_t size = base_len + (insert ? 4 : 0);
      const bool strip = (fl & NICGPU_SEG_VLAN_STRIP) && has_vlan && size >= 4;
      if (strip) size -= 4;
      const bool prefix = insert && !strip;
      const bool strip_base = strip && !insert;
      const uint64_t g = (uint64_t) seg_base + k;
      const uint64_t dst = g * P.stride;
      if (dst > P.out_size || size > P.out_size - dst || size > P.stride) continue;  // does not fit its slot
      uint64_t src_a = off, len_a = H, src_b = off + H + (uint64_t) k * mss, len_b = clen;
      if (strip_base) {  // the base segment loses its first 4 bytes
        const uint64_t from_a = len_a < 4 ? len_a : 4;
        src_a += from_a;
        len_a -= from_a;
        src_b += 4 - from_a;
        len_b -= 4 - from_a;
      }
      uint32_t sum = 0;
      const uint64_t pl = prefix ? 4 : 0;
      if (staged) {
        sum = seg_copy_stage(P.out, dst, (uint32_t) size, (uint32_t) pl, tag, reinterpret_cast<const uint8_t*>(stage),
                             (uint32_t) (src_a - a0), (uint32_t) len_a, (uint32_t) (src_b - a0), lane);
      } else {
        if (lane < pl) {
          const uint32_t b = lane == 0 ? 0x81u : (lane == 1 ? 0x00u : (lane == 2 ? (tag >> 8) : (tag & 0xFFu)));
          P.out[dst + lane] = (uint8_t) b;
          sum += b << (8 * ((dst + lane) & 1));
        }
        sum += wave_copy<false, true>(P.out, dst + pl, P.frames, 0, src_a, len_a, lane);
        sum += wave_copy<false, true>(P.out, dst + pl + len_a, P.frames, 0, src_b, len_b, lane);
      }
      const uint32_t tot = (uint32_t) __builtin_amdgcn_readlane((int) wave_incl_scan(sum), 63);
      if (lane == 0) {
        const uint32_t x = fold16(tot);
        const uint32_t be = (dst & 1) ? x : bswap16(x);
        if (P.out_len) P.out_len[g] = (uint32_t) size;
        if (P.out_csum) P.out_csum[g] = (uint16_t) (~be & 0xFFFFu);
      }
    }
  }
  }
}

// ------------------------------------------------------------ RoCEv2 ICRC --
// nic::rocev2::IcrcCalculator::calculate / verify (src/rocev2/packet.cpp:14-75)
// over a batch: CRC-32C (reflected 0x82F63B78, init/xorout 0xFFFFFFFF) of
// every descriptor's span.  One lane owns one packet at a time and walks it
// to the end of a 128-B line per step (up to 8 x 16-B loads); a finished lane
// takes the next packet of its wave's range through a ballot (a wave-level
// work queue), so IMIX lengths do not leave lanes idle.
struct Crc32cTables {
  uint32_t t[16][256];
};
constexpr Crc32cTables make_crc32c_tables() {
  Crc32cTables T{};
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    T.t[0][i] = c;
  }
  for (int k = 1; k < 16; ++k)
    for (uint32_t i = 0; i < 256; ++i) T.t[k][i] = (T.t[k - 1][i] >> 8) ^ T.t[0][T.t[k - 1][i] & 0xFFu];
  return T;
}
__constant__ Crc32cTables kCrc32c = make_crc32c_tables();

// kCrcLead.s[n]: the CRC state that n zero bytes take to 0xFFFFFFFF (the
// zero-byte step is invertible: the top byte of T0[k] is a permutation of k).
// A packet starting n bytes into its first 16-B chunk starts from s[n] at byte
// 0 of that chunk with the n leading bytes masked to zero, so the state is
// always xored in at byte 0 — no per-chunk shift of the state.
struct CrcLead {
  uint32_t s[16];
};
constexpr CrcLead make_crc_lead() {
  const Crc32cTables T = make_crc32c_tables();
  uint32_t top_inv[256] = {};
  for (uint32_t k = 0; k < 256; ++k) top_inv[T.t[0][k] >> 24] = k;
  CrcLead R{};
  uint32_t s = 0xFFFFFFFFu;
  R.s[0] = s;
  for (int n = 1; n < 16; ++n) {
    const uint32_t k = top_inv[s >> 24];
    s = ((s ^ T.t[0][k]) << 8) | k;
    R.s[n] = s;
  }
  return R;
}
constexpr CrcLead kCrcLeadHost = make_crc_lead();
static_assert(kCrcLeadHost.s[0] == 0xFFFFFFFFu, "lead table");
__constant__ CrcLead kCrcLead = make_crc_lead();

struct IcrcParams {
  const uint8_t* frames;
  const uint64_t* desc;
  uint64_t n;
  int verify;
  uint32_t* out_crc;
  uint8_t* out_ok;
};

constexpr int kIcrcRing = 128;  // descriptor ring per wave (LDS)

// waves per block: one block per CU shares the table image.  8 waves, not 16:
// each lane walks its own packet's lines, so a CU's waves keep waves x 64
// lines in flight; same-box sweep (profiles/r03_icrc_wpb_sweep.txt, median us
// C2 / C3): 4 waves 566 / 727, 6: 435 / 545, 8: 379 / 460, 10: 459 / 444,
// 12: 469 / 434, 16: 452 / 491.
constexpr int kIcrcWpb = 8;
constexpr int kIcrcThreads = kWave * kIcrcWpb;
// a ^ b ^ c in one VALU op (hipcc folds table words one v_xor_b32 at a time)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// Byte tables, slice-by-4: one lookup per byte instead of the nibble tables'
// two, still conflict-free.  The four tables T_3..T_0 of a dword step
// (S ^= x; S = T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3]) are stored 32 times, copy c
// in bank c only: row v of the table for byte j sits at (j >> 1) * 64 KiB +
// v * 256 + (j & 1) * 128, copy c at +4c (a 256-B row is 64 banks wide,
// ds_read_b32 banks by (a / 4) mod 32, so the two halves of a row are two
// tables on the same 32 banks).  A lookup address is one v_perm_b32:
// {copy byte, byte j of the state, table pair, 0}.  128 KiB of LDS: one
// block (8 waves) per CU.  Each lane walks its packet dword by dword
// (a serial chain per lane; 8 waves per CU cover its latency); the packet's
// 1..3 leading bytes in its first dword are masked and the state enters
// through kCrcLead, and its 0..3 bytes past the last whole dword take byte
// steps on T0 at the end, so no trailing-zero unshift is needed.
constexpr uint32_t kB4Bytes = 2u * 65536u;

__device__ __forceinline__ uint32_t b4_lookup(const uint8_t* __restrict__ Tb, uint32_t cbr, uint32_t s, uint32_t sel) {
  return *reinterpret_cast<const uint32_t*>(Tb + __builtin_amdgcn_perm(cbr, s, sel));
}

__device__ __forceinline__ uint32_t b4_dword(const uint8_t* __restrict__ Tb, uint32_t cbr, uint32_t s) {
  const uint32_t t0 = b4_lookup(Tb, cbr, s, 0x0C0C0004u);  // T3[s.b0]
  const uint32_t t1 = b4_lookup(Tb, cbr, s, 0x0C0C0105u);  // T2[s.b1]
  const uint32_t t2 = b4_lookup(Tb, cbr, s, 0x0C070204u);  // T1[s.b2]
  const uint32_t t3 = b4_lookup(Tb, cbr, s, 0x0C070305u);  // T0[s.b3]
  return xor3(t0, t1, t2) ^ t3;
}

// MODE 0: production; 1: timing only, the loads and masks without the table
// work (results wrong).  Measured (profiles/r03_icrc_variants.jsonl): the
// timing-only kernel takes 92% of the production time, so the lane-per-packet
// line walk, not the table work, bounds this kernel; 4-chunk windows, a
// prefetch of the packet's next window, and 32-B windows loaded coalesced and
// transposed back with ds_bpermute were all slower.
template <int CH, int MODE>  // CH: chunks per step, to the end of the packet's aligned CH x 16-B window
__global__ __launch_bounds__(kIcrcThreads) void icrc_b4_kernel(IcrcParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t Tb[kB4Bytes];
  __shared__ uint64_t ring_all[kIcrcWpb][kIcrcRing];
  __shared__ uint4 lead_m[16];  // bytes >= p of a chunk kept
  __shared__ uint32_t lead_s[16];
  if (threadIdx.x < 16u) {
    const int p = (int) threadIdx.x;
    lead_s[p] = kCrcLead.s[p];
    lead_m[p] = make_uint4(dword_keep(p, 16, 0), dword_keep(p, 16, 1), dword_keep(p, 16, 2), dword_keep(p, 16, 3));
  }
  for (uint32_t q = threadIdx.x; q < kB4Bytes / 16u; q += kIcrcThreads) {
    const uint32_t o = q * 16u;
    const uint32_t j = 2u * (o >> 16) + ((o >> 7) & 1u), v = (o >> 8) & 255u;
    const uint32_t val = kCrc32c.t[3u - j][v];
    reinterpret_cast<uint4*>(Tb)[q] = make_uint4(val, val, val, val);
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint32_t cb = (lane & 31u) << 2;  // this lane's copy: bank lane % 32
  const uint32_t cbr = cb | ((cb + 128u) << 8) | (1u << 24);
  uint64_t* ring = ring_all[threadIdx.x / kWave];
  const uint64_t nwaves = (uint64_t) gridDim.x * kIcrcWpb;
  const uint64_t wave = (uint64_t) blockIdx.x * kIcrcWpb + threadIdx.x / kWave;
  const uint64_t per = (P.n + nwaves - 1) / nwaves;
  const uint64_t p0 = wave * per < P.n ? wave * per : P.n;
  const uint64_t p1 = p0 + per < P.n ? p0 + per : P.n;
  const u32x4* f16 = reinterpret_cast<const u32x4*>(P.frames);

  uint64_t loaded = p0;
  auto refill = [&]() __attribute__((always_inline)) {
    const uint64_t i = loaded + lane;
    ring[i & (kIcrcRing - 1)] = i < p1 ? P.desc[i] : 0ull;
    loaded += kWave;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  };
  refill();
  refill();
  uint64_t next = p0 + kWave;
  uint64_t my = p0 + lane;
  // per lane, byte positions relative to the packet's first 16-B chunk c16:
  // the chain enters at byte 0 of that chunk from kCrcLead[pos] with the pos
  // leading bytes zeroed (no predicate on leading dwords); whole dwords
  // [cur, end4) still to process, then tail bytes [end4, end) (bytes < pos
  // zero).  An empty span does nothing: state 0xFFFFFFFF.
  uint64_t c16 = 0;
  uint32_t pos = 0, cur = 0, end4 = 0, end = 0, wend = 0, len = 0, lb = 0, S = 0xFFFFFFFFu;
  auto setup = [&]() __attribute__((always_inline)) {
    const uint64_t d = ring[my & (kIcrcRing - 1)];
    const uint64_t off = d & kOffMask;
    len = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
    const uint32_t span = P.verify ? (len >= 4u ? len - 4u : 0u) : len;
    c16 = off >> 4;
    lb = (uint32_t) c16 & (uint32_t) (CH - 1);
    pos = (uint32_t) off & 15u;
    end = pos + span;
    wend = span ? end : 0u;
    end4 = wend & ~3u;
    cur = 0;
    S = span ? lead_s[pos] : 0xFFFFFFFFu;
  };
  if (my < p1) setup();
  for (;;) {
    const bool active = my < p1;
    if (__ballot(active) == 0ull) break;
    if (active && cur < end4) {
      // up to the end of the current CH-chunk window; every chunk of the
      // step is processed (predicated on the dword being below lim), so all
      // CH loads issue before the first is used
      const uint32_t c0 = cur >> 4, clast = (end4 - 1u) >> 4;
      const uint32_t ce = ((lb + c0) | (uint32_t) (CH - 1)) - lb;
      const uint32_t cl = ce < clast ? ce : clast;
      const uint32_t lim = ((cl + 1u) << 4 < end4 ? (cl + 1u) << 4 : end4) - cur;  // dwords [0, lim) of the step
      u32x4 v[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) v[u] = f16[c16 + (c0 + (uint32_t) u <= cl ? c0 + (uint32_t) u : cl)];
      __builtin_amdgcn_sched_barrier(0);  // every load of the step in flight before the chain starts
      const uint4 m0 = lead_m[c0 == 0u ? pos : 0u];
      v[0][0] &= m0.x;
      v[0][1] &= m0.y;
      v[0][2] &= m0.z;
      v[0][3] &= m0.w;
#pragma unroll
      for (int u = 0; u < CH; ++u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t Sn = MODE == 1 ? S + v[u][i] : b4_dword(Tb, cbr, S ^ v[u][i]);
          S = (uint32_t) (16 * u + 4 * i) < lim ? Sn : S;
        }
      }
      cur = (cl + 1u) << 4;
    }
    const bool finished = active && cur >= end4;
    if (finished) {
      if (end4 < wend) {  // 1..3 bytes past the last whole dword: byte steps on T0
        const uint32_t wv = *reinterpret_cast<const uint32_t*>(P.frames + (c16 << 4) + end4);
#pragma unroll
        for (uint32_t b = 0; b < 3u; ++b) {
          const uint32_t idx = end4 + b;
          const uint32_t z = S ^ (idx < pos ? 0u : (wv >> (8u * b)) & 0xFFu);
          const uint32_t Sn = b4_lookup(Tb, cbr, z, 0x0C070005u) ^ (S >> 8);
          S = idx < wend ? Sn : S;
        }
      }
      const uint32_t crc = S ^ 0xFFFFFFFFu;
      if (P.out_crc) P.out_crc[my] = (P.verify && len < 4u) ? 0u : crc;
      if (P.verify) {
        uint32_t ok = 0;
        if (len >= 4u) {
          const uint8_t* t = P.frames + (c16 << 4) + end;
          const uint32_t stored = ((uint32_t) t[0] << 24) | ((uint32_t) t[1] << 16) | ((uint32_t) t[2] << 8) | t[3];
          ok = stored == crc;
        }
        P.out_ok[my] = (uint8_t) ok;
      }
    }
    const uint64_t m = __ballot(finished);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
    if (finished) my = next + rank;
    next += (uint64_t) __builtin_popcountll(m);
    if (finished && my < p1) setup();
    if (next + kWave > loaded && loaded < p1) refill();
  }
}

struct DeviceInfo {
  bool init = false;
  int status = 0;
  int cus = 0;
  int tso_blocks_per_cu = 0;
  int seg_blocks_per_cu = 0;  // tso_segment_kernel (LDS frame stage)
  int icrc_blocks_per_cu = 0;
  // occupancy cache per (variant, dynamic LDS bytes)
  struct Occ { int variant; uint32_t lds; int blocks; };
  std::vector<Occ> occ;
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
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tso_checksum_kernel, kBlock, 0) != hipSuccess || b < 1) b = 1;
  di.tso_blocks_per_cu = b;
  b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, tso_segment_kernel, kBlock, 0) != hipSuccess || b < 1) b = 1;
  di.seg_blocks_per_cu = b;
  b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, icrc_b4_kernel<8, 0>, kIcrcThreads, 0) != hipSuccess || b < 1) b = 1;
  di.icrc_blocks_per_cu = b;
  return di;
}

#ifdef NICGPU_TUNING
// tuning: at most this many RX blocks per CU (0 = occupancy maximum); the LDS
// request is padded so the hardware cannot place more (nicgpu_tune_set_bpc)
uint32_t g_bpc_cap = 0;
#endif

int rx_blocks_per_cu(int dev, int variant, uint32_t lds) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceInfo& di = g_dev[dev & 63];
#ifdef NICGPU_TUNING
  auto capped = [](int b) { return g_bpc_cap && b > (int) g_bpc_cap ? (int) g_bpc_cap : b; };
#else
  auto capped = [](int b) { return b; };
#endif
  for (const auto& o : di.occ)
    if (o.variant == variant && o.lds == lds) return capped(o.blocks);
  int b = 0;
  const RxVariant& v = kRxVariants[variant];
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, v.kernel, kWave * v.wpb, lds) != hipSuccess || b < 1) b = 1;
  di.occ.push_back({variant, lds, b});
  return capped(b);
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
  unsigned long long* d_rep = nullptr;  // kHistRep x kHistLds hit-histogram replicas (flush_hist), zeroed
  unsigned int* d_done = nullptr;       // their done ticket
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

// XPF variants prefetch the next tile's first batch for tiles up to this many
// 16-B chunks (tools/tune_rx.py sets it through nicgpu_tune_set_xpf).
uint32_t g_xpf_chunks = 0xFFFFFFFFu;

// LDS result ring of a RING variant at its occupancy: tiles held per wave
// (as many as the LDS left over allows, at most a wave's share of the batch),
// and whether that is all of a wave's tiles.
struct RingPlan {
  uint32_t hold_r, ring_off, lds;
  bool holds_all;
};

RingPlan plan_ring(int dev, int variant, uint32_t lds, uint64_t ntiles, const DeviceInfo& di) {
  const RxVariant& v = kRxVariants[variant];
  const int bpc = rx_blocks_per_cu(dev, variant, lds);
  const uint64_t waves = (uint64_t) di.cus * (uint64_t) bpc * (uint64_t) v.wpb;
  const uint64_t per_wave = (ntiles + waves - 1) / waves;
  const uint32_t per_block = kLdsPerCu / (uint32_t) bpc;
  const uint32_t spare = per_block > lds ? per_block - lds : 0u;
  uint64_t r = spare / ((uint32_t) v.wpb * kRingTileBytes);
  if (r > per_wave) r = per_wave;
  if (r < 1) r = 1;
  RingPlan rp;
  rp.hold_r = (uint32_t) r;
  rp.ring_off = (lds + 15u) & ~15u;
  rp.lds = rp.ring_off + (uint32_t) v.wpb * rp.hold_r * kRingTileBytes;
  rp.holds_all = per_wave <= r;
  return rp;
}

int rss_only_blocks_per_cu(int dev, uint32_t lds) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceInfo& di = g_dev[dev & 63];
  constexpr int kRssOnlyVariant = -1;  // occupancy cache key
  for (const auto& o : di.occ)
    if (o.variant == kRssOnlyVariant && o.lds == lds) return o.blocks;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rss_only_kernel<kRssWpb>, kWave * kRssWpb, lds) != hipSuccess ||
      b < 1)
    b = 1;
  di.occ.push_back({kRssOnlyVariant, lds, b});
  return b;
}

template <bool RSS>
int dlv_blocks_per_cu(int dev, uint32_t lds) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceInfo& di = g_dev[dev & 63];
  constexpr int kKey = RSS ? -2 : -3;  // occupancy cache key
  for (const auto& o : di.occ)
    if (o.variant == kKey && o.lds == lds) return o.blocks;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, deliver_kernel<RSS>, kWave * kDlvWpb, lds) != hipSuccess || b < 1)
    b = 1;
  di.occ.push_back({kKey, lds, b});
  return b;
}

int launch_rss_only(const RxParams& P, const DeviceInfo& di, hipStream_t stream) {
  const uint32_t hist_n = (P.out_hits && P.table_n <= (uint32_t) kHistLds) ? P.table_n : 0u;
  const uint32_t table_words = P.table_n <= (uint32_t) kTableLds ? (P.table_n + 1u) / 2u : 0u;
  const uint32_t lds = rss_only_block_bytes(P.lut_words, hist_n, table_words) + kRssWpb * kRssOnlyWaveBytes;
  // as many blocks as fit a CU (registers and LDS), one grid-stride pass each
  int dev = 0;
  (void) hipGetDevice(&dev);
  const uint32_t bpc = (uint32_t) rss_only_blocks_per_cu(dev, lds);
  constexpr uint32_t kThreads = kWave * kRssWpb;
  const uint64_t want = (P.n + kThreads - 1) / kThreads;
  const uint64_t cap = (uint64_t) di.cus * bpc;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(rss_only_kernel<kRssWpb>, dim3(grid), dim3(kThreads), lds, stream, P);
  return hip_status(hipGetLastError());
}

int launch_rx(const RxParams& P, const DeviceInfo& di, int variant, hipStream_t stream) {
  if (variant < 0 || variant >= kNumRxVariants) return NICGPU_ERR_INVALID;
  const bool rss = P.mode != NICGPU_TUPLE_NONE;
  const bool stage = rss || P.out_l34 != nullptr;
  const uint32_t hist_n = (P.out_hits && P.table_n <= (uint32_t) kHistLds) ? P.table_n : 0u;
  const uint32_t table_words = (rss && P.table_n <= (uint32_t) kTableLds) ? (P.table_n + 1u) / 2u : 0u;
  const uint64_t ntiles = (P.n + kWave - 1) / kWave;
  int dev = 0;
  (void) hipGetDevice(&dev);
  auto lds_of = [&](int var) {
    const RxVariant& vv = kRxVariants[var];
    return rx_lds_bytes(vv.wpb, vv.unroll, stage, rss ? P.lut_words : 0u, hist_n, table_words);
  };
  if (variant == 0) {
    // many tiles with a hit histogram: 8-wave blocks (what they save is half
    // the end-of-block histogram flushes; the ring flushes mid-stream: sc1)
    if (ntiles >= kRxW8Tiles && hist_n) variant = kRxW8;
    else variant = plan_ring(dev, 0, lds_of(0), ntiles, di).holds_all ? 1 : 0;
  }
  const RxVariant& v = kRxVariants[variant];
  const uint32_t lds = lds_of(variant);
  // ranges: at least 16 packets per wave; round robin: one tile per wave
  const uint64_t want = v.ranges ? (P.n + 16 * (uint64_t) v.wpb - 1) / (16 * (uint64_t) v.wpb)
                                 : (ntiles + v.wpb - 1) / (uint64_t) v.wpb;
  int bpc = rx_blocks_per_cu(dev, variant, lds);
  RxParams Pl = P;
  Pl.xpf_chunks = v.xpf ? g_xpf_chunks : 0u;
  uint32_t lds_launch = lds;
  if (v.ring) {
    const RingPlan rp = plan_ring(dev, variant, lds, ntiles, di);
    Pl.hold_r = rp.hold_r;
    Pl.ring_off = rp.ring_off;
    lds_launch = rp.lds;
    bpc = rx_blocks_per_cu(dev, variant, lds_launch);
  }
#ifdef NICGPU_TUNING
  if (g_bpc_cap) {  // pad the LDS request so no more than the cap fit on a CU
    const uint32_t floor_lds = kLdsPerCu / (g_bpc_cap + 1u) + 16u;
    if (lds_launch < floor_lds) lds_launch = floor_lds;
  }
#endif
  const uint64_t cap = (uint64_t) di.cus * (uint64_t) bpc;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(v.kernel, dim3(grid), dim3(kWave * v.wpb), lds_launch, stream, Pl);
  return hip_status(hipGetLastError());
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
    case NICGPU_ERR_RANGE: return "batch too large for 32-bit piece indices";
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

namespace {
#ifdef NICGPU_TUNING
uint32_t g_tune_dbg = 0;  // tools/tune_rx.py --dbg (nicgpu_tune_set_dbg)
unsigned long long* g_tune_stamps = nullptr;  // tools/wave_stamps.py (nicgpu_tune_set_stamps)
#endif
int rx_offload_impl(int variant, const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                    int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum, uint32_t* out_hash,
                    uint16_t* out_queue, uint64_t* out_hits, uint8_t* out_l34, void* stream,
                    const uint64_t* n_dev = nullptr) {
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
  if (!out_csum && !out_hash && !out_queue && !out_hits && !out_l34) return NICGPU_OK;
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
  P.out_l34 = out_l34;
  P.n_dev = reinterpret_cast<const unsigned long long*>(n_dev);
#ifdef NICGPU_TUNING
  P.dbg = g_tune_dbg;
  P.stamps = g_tune_stamps;
#endif
  if (ctx) {
    P.lut = ctx->d_lut;
    P.table = ctx->d_table;
    P.table_n = (uint32_t) ctx->table_n;
#ifdef NICGPU_HIST_REP  // off: measured neutral (r03 A/B), and a ctx shared by two streams would race on d_done
    if (out_hits && P.table_n <= (uint32_t) kHistLds) {
      P.hits_rep = ctx->d_rep;
      P.hits_done = ctx->d_done;
    }
#endif
    uint32_t max_tuple = tuple_mode == NICGPU_TUPLE_RAW ? raw_len : 36u;
    P.lut_words = 2u * max_tuple * 16u;
  }
  // hash and queue only: the headers suffice (rss_only_kernel)
  if (variant == 0 && !out_csum && !out_l34 && tuple_mode != NICGPU_TUPLE_NONE)
    return launch_rss_only(P, *di, static_cast<hipStream_t>(stream));
  return launch_rx(P, *di, variant, static_cast<hipStream_t>(stream));
}
}  // namespace

extern "C" {

int nicgpu_rx_offload(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                      int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum,
                      uint32_t* out_hash, uint16_t* out_queue, uint64_t* out_hits, void* stream) {
  return rx_offload_impl(0, ctx, frames, desc, n, tuple_mode, raw_off, raw_len, out_csum, out_hash, out_queue,
                         out_hits, nullptr, stream);
}

int nicgpu_rx_offload_ex(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                         int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum, uint32_t* out_hash,
                         uint16_t* out_queue, uint64_t* out_hits, uint8_t* out_l34, void* stream) {
  return rx_offload_impl(0, ctx, frames, desc, n, tuple_mode, raw_off, raw_len, out_csum, out_hash, out_queue,
                         out_hits, out_l34, stream);
}

int nicgpu_rx_offload_count(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n_max,
                            const uint64_t* n_dev, int tuple_mode, uint32_t raw_off, uint32_t raw_len,
                            uint16_t* out_csum, uint32_t* out_hash, uint16_t* out_queue, uint64_t* out_hits,
                            void* stream) {
  if (!n_dev) return NICGPU_ERR_INVALID;
  return rx_offload_impl(0, ctx, frames, desc, n_max, tuple_mode, raw_off, raw_len, out_csum, out_hash, out_queue,
                         out_hits, nullptr, stream, n_dev);
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

int nicgpu_icrc_batch(const uint8_t* frames, const uint64_t* desc, size_t n, int mode, uint32_t* out_crc,
                      uint8_t* out_ok, void* stream) {
  if (mode != NICGPU_ICRC_CALCULATE && mode != NICGPU_ICRC_VERIFY) return NICGPU_ERR_INVALID;
  if (mode == NICGPU_ICRC_CALCULATE && out_ok) return NICGPU_ERR_INVALID;
  if (mode == NICGPU_ICRC_VERIFY && !out_ok) return NICGPU_ERR_INVALID;
  if (n == 0) return NICGPU_OK;
  if (!frames || !desc) return NICGPU_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(frames) & 15u) != 0) return NICGPU_ERR_INVALID;
  if (!out_crc && !out_ok) return NICGPU_OK;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  IcrcParams P{frames, desc, n, mode == NICGPU_ICRC_VERIFY, out_crc, out_ok};
  // every resident wave slot busy (a wave's range is then >= 64 packets, one
  // work-queue refill); ranges of 8 packets per lane left 3/4 of the slots idle
  // NICGPU_ICRC=b4mem: timing only, the loads without the table work (results wrong)
  static const int var = [] {
    const char* e = std::getenv("NICGPU_ICRC");
    return e && std::strcmp(e, "b4mem") == 0 ? 1 : 0;
  }();
  const uint64_t want = (n + kIcrcThreads - 1) / kIcrcThreads;
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) di->icrc_blocks_per_cu;
  const unsigned grid = (unsigned) (want < 1 ? 1 : (want < cap ? want : cap));
  if (var == 1)
    hipLaunchKernelGGL((icrc_b4_kernel<8, 1>), dim3(grid), dim3(kIcrcThreads), 0, static_cast<hipStream_t>(stream), P);
  else
    hipLaunchKernelGGL((icrc_b4_kernel<8, 0>), dim3(grid), dim3(kIcrcThreads), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

int nicgpu_tso_segment(const uint8_t* frames, const uint64_t* desc, const uint16_t* hdr_len, const uint16_t* mss,
                       const uint32_t* seg_base, const uint32_t* flags, size_t n, uint8_t* out, uint64_t out_size,
                       uint32_t stride, uint32_t* out_len, uint16_t* out_csum, void* stream) {
  if (n == 0) return NICGPU_OK;
  if (!frames || !desc || !hdr_len || !mss || !seg_base || !out || stride == 0) return NICGPU_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(frames) & 15u) != 0) return NICGPU_ERR_INVALID;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  TsoSegParams P{frames, desc, hdr_len, mss, seg_base, flags, n, out, out_size, stride, out_len, out_csum};
  const uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) di->seg_blocks_per_cu;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(tso_segment_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

int nicgpu_segment_gather(uint8_t* mem, uint64_t mem_size, const nicgpu_segment_write* writes, size_t n,
                          void* stream) {
  return nicgpu_segment_gather_from(mem, mem, mem_size, writes, n, stream);
}

int nicgpu_segment_gather_from(uint8_t* mem, const uint8_t* src, uint64_t mem_size,
                               const nicgpu_segment_write* writes, size_t n, void* stream) {
  if (n == 0) return NICGPU_OK;
  if (!mem || !src || !writes) return NICGPU_ERR_INVALID;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  GatherParams P{mem, src, mem_size, writes, n};
  const uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
  const uint64_t cap = (uint64_t) di->cus * 8;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(segment_gather_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

}  // extern "C"

// ---------------------------------------------- batched QueuePair (f1) --
// The per-packet decisions of QueuePair::process_once over a whole batch on
// the device: one thread per TX descriptor, decisions from qp_logic.h (the
// source the host resolve uses, fuzzed against the compiled reference).
//   plan     count pieces per descriptor, exclusive scan, fill the piece
//            descriptors; the RX kernel sums every piece (one pass over the
//            TX bytes)
//   resolve  RX descriptors each packet pops if nothing ends it early
//            (rx_need), exclusive scan = every packet's ring position, while
//            the ring lasts; a dry pass finds the first packet whose RX side
//            ends it early (its pops differ); the full pass posts the
//            completions, DMA writes and per-block statistics of every packet
//            before that.  The caller resolves the rest on the host, in order.
//   rss      Success frames compacted into RSS descriptors; the hashes and
//            queues scattered back per completion.
namespace {

struct QpPlan {
  uint32_t kind, nseg, first_piece, npieces, hdr_len, mss;
};
using QpCtx = nicqp::Ctx<nicgpu_tx_descriptor, nicgpu_rx_descriptor, QpPlan>;
constexpr unsigned kQpBlock = 256;
constexpr unsigned kQpStats = 16;
// after the per-block stats: RX used, first mismatch, settled prefix, then the
// batch's 16 stats totals — the one download a resolve needs
constexpr unsigned kQpTail = 3 + 16;
constexpr int kQpRelaxSteps = 8;  // position relaxations before the host takes the rest

struct QpNullSink {
  __device__ void tx(const nicgpu_completion&, bool) {}
  __device__ void rx(const nicgpu_completion&, const nicgpu_segment_write*) {}
};

struct QpDevSink {
  nicgpu_completion* txc;
  nicgpu_completion* rxc;
  nicgpu_segment_write* w;
  uint64_t ti, rj;
  __device__ void tx(const nicgpu_completion& e, bool) { txc[ti] = e; }
  __device__ void rx(const nicgpu_completion& e, const nicgpu_segment_write* sw) {
    rxc[rj] = e;
    if (sw) {
      w[rj] = *sw;
    } else {
      nicgpu_segment_write z{};
      w[rj] = z;
    }
    ++rj;
  }
};

// counts[n] must be 0 on entry: a descriptor that plans more than
// kQpMaxPieces pieces counts 0 and sets it to 1, so the 32-bit scan of the
// counts (n <= 2^32 / kQpMaxPieces) cannot wrap and the caller sees the flag.
constexpr uint32_t kQpMaxPieces = 256;
__global__ __launch_bounds__(kQpBlock) void qp_count_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t n,
                                                            uint64_t mem_size, uint64_t max_mtu, QpPlan* plans,
                                                            uint32_t* counts) {
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i < n; i += (uint64_t) gridDim.x * kQpBlock) {
    QpPlan pp;
    const uint32_t c = nicqp::plan_packet(max_mtu, mem_size, nicqp::desc_load(tx + i), pp, [](uint64_t, uint64_t) {});
    counts[i] = c <= kQpMaxPieces ? c : 0u;
    if (c > kQpMaxPieces) counts[n] = 1u;
    plans[i] = pp;
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_fill_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t n,
                                                           uint64_t mem_size, uint64_t max_mtu, QpPlan* plans,
                                                           const uint32_t* __restrict__ base, uint64_t* desc) {
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i < n; i += (uint64_t) gridDim.x * kQpBlock) {
    uint32_t at = base[i];
    plans[i].first_piece = at;
    QpPlan pp;
    nicqp::plan_packet(max_mtu, mem_size, nicqp::desc_load(tx + i), pp,
                       [&](uint64_t a, uint64_t len) { desc[at++] = NICGPU_DESC(a, len); });
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_need_kernel(QpCtx C, uint64_t n, uint32_t* need,
                                                           unsigned long long* first) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *first = n;  // the speculative final pass's "nothing differed"
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i <= n; i += (uint64_t) gridDim.x * kQpBlock)
    need[i] = i < n ? nicqp::rx_need(C, i) : 0u;
}

// One relaxation step of the ring positions: every packet resolved (without
// outputs) at pos[i] = the exclusive scan of pops; pops[i] becomes what it
// actually popped there (the ring checks of :75-83 and :293-303 included),
// and scal[0] the first packet whose pops changed.  The sequential positions
// are the fixed point, and each step makes at least one more packet exact:
// pos[0] = 0 always is, so after k steps packets [0, k) are.
__global__ __launch_bounds__(kQpBlock) void qp_relax_kernel(QpCtx C, uint32_t* pops, const uint32_t* __restrict__ pos,
                                                            uint64_t n, unsigned long long* scal) {
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i < n; i += (uint64_t) gridDim.x * kQpBlock) {
    nicgpu_qp_stats st{};
    QpNullSink sink;
    // a guess past the ring's end is clamped to it (the sequential positions
    // never pass it; resolve_packet must not index past rx[nrx - 1])
    const uint64_t rc = pos[i] < C.nrx ? (uint64_t) pos[i] : C.nrx;
    const uint32_t popped = (uint32_t) nicqp::resolve_packet<nicgpu_completion, nicgpu_segment_write>(C, i, rc, st, sink);
    if (popped != pops[i]) {
      atomicMin(&scal[0], (unsigned long long) i);
      pops[i] = popped;
    }
  }
}

// packets [0, lim) at their (exact) positions: completions, writes, per-block
// stats.  With `guess` (the pops the positions were scanned from) the pass is
// speculative: first[0] becomes the first packet that popped otherwise, and
// only [0, first] is exact — all of it when nothing differed.
__global__ __launch_bounds__(kQpBlock) void qp_full_kernel(QpCtx C, const uint32_t* __restrict__ pos, uint64_t lim,
                                                           nicgpu_completion* txc, nicgpu_completion* rxc,
                                                           nicgpu_segment_write* writes, uint64_t* partials,
                                                           const uint32_t* __restrict__ guess) {
  __shared__ uint64_t red[kQpStats][kQpBlock / kWave];
  // after the per-block stats: [0] the RX descriptors used (pos[lim]), [1] the
  // first mismatch (seeded with n by qp_need_kernel) — one download for all
  uint64_t* tail = partials + (uint64_t) gridDim.x * kQpStats;
  unsigned long long* first = reinterpret_cast<unsigned long long*>(tail + 1);
  if (blockIdx.x == 0 && threadIdx.x == 0) tail[0] = pos[lim];
  nicgpu_qp_stats st{};
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i < lim; i += (uint64_t) gridDim.x * kQpBlock) {
    if (pos[i] > C.nrx) {  // exact positions never pass the ring's end: a guess past it is wrong
      if (guess) atomicMin(first, (unsigned long long) i);
      continue;
    }
    QpDevSink sink{txc, rxc, writes, i, pos[i]};
    const uint32_t popped = (uint32_t) nicqp::resolve_packet<nicgpu_completion, nicgpu_segment_write>(C, i, pos[i], st, sink);
    if (guess && popped != guess[i]) atomicMin(first, (unsigned long long) i);
  }
  uint64_t v[kQpStats];
  static_assert(sizeof(nicgpu_qp_stats) == kQpStats * 8, "16 counters");
  __builtin_memcpy(v, &st, sizeof(v));
  const uint32_t lane = lane_id(), w = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < (int) kQpStats; ++k) {
    unsigned long long x = v[k];
    for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if (lane == 0) red[k][w] = x;
  }
  __syncthreads();
  if (threadIdx.x < kQpStats) {
    uint64_t x = 0;
    for (unsigned j = 0; j < kQpBlock / kWave; ++j) x += red[threadIdx.x][j];
    partials[(uint64_t) blockIdx.x * kQpStats + threadIdx.x] = x;
  }
}

// After a final pass: the per-block stats summed into tail[3..19), and after
// the speculative one tail[2] = the RX completions it made final — those of
// the packets before the first mismatch, [0, pos[first]), or all `used` when
// nothing differed.  nicgpu_qp_deliver_range(NICGPU_DELIVER_SETTLED) reads it
// on the device, so the DMA writes start before the host has seen the resolve.
constexpr unsigned kQpReduceThreads = 1024;
__global__ __launch_bounds__(kQpReduceThreads) void qp_reduce_kernel(const uint64_t* __restrict__ partials,
                                                                     unsigned nblocks, const uint32_t* __restrict__ pos,
                                                                     uint64_t ntx, bool settle) {
  __shared__ uint64_t red[kQpReduceThreads];
  uint64_t* tail = const_cast<uint64_t*>(partials) + (size_t) nblocks * kQpStats;
  const unsigned k = threadIdx.x % kQpStats, r = threadIdx.x / kQpStats;
  constexpr unsigned kRows = kQpReduceThreads / kQpStats;
  uint64_t x = 0;
  for (unsigned b = r; b < nblocks; b += kRows) x += partials[(size_t) b * kQpStats + k];
  red[threadIdx.x] = x;
  __syncthreads();
  for (unsigned h = kRows / 2; h > 0; h >>= 1) {
    if (r < h) red[threadIdx.x] += red[threadIdx.x + h * kQpStats];
    __syncthreads();
  }
  if (threadIdx.x < kQpStats) tail[3 + threadIdx.x] = red[threadIdx.x];
  if (settle && threadIdx.x == 0) {
    const uint64_t first = tail[1];
    tail[2] = first < ntx ? (uint64_t) pos[first] : tail[0];
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_flag_kernel(const nicgpu_completion* __restrict__ rxc, uint64_t nrx,
                                                           uint32_t* flags, uint32_t* rx_hash, uint16_t* rx_queue) {
  for (uint64_t j = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; j <= nrx; j += (uint64_t) gridDim.x * kQpBlock) {
    flags[j] = j < nrx && rxc[j].status == nicqp::kSuccess ? 1u : 0u;
    if (j < nrx) {
      rx_hash[j] = 0;
      rx_queue[j] = 0xFFFFu;
    }
  }
}

// The tuple lies in a frame's first 82 bytes, so a frame longer than
// NICGPU_MAX_PACKET (max_mtu above 65531) is hashed over its first
// NICGPU_MAX_PACKET bytes: the same tuple, hash and queue.
__global__ __launch_bounds__(kQpBlock) void qp_rss_fill_kernel(const uint32_t* __restrict__ flags,
                                                               const uint32_t* __restrict__ at,
                                                               const nicgpu_segment_write* __restrict__ writes,
                                                               uint64_t nrx, uint64_t* desc, uint32_t* which,
                                                               unsigned long long* count) {
  for (uint64_t j = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; j <= nrx; j += (uint64_t) gridDim.x * kQpBlock) {
    if (j == nrx) {
      *count = at[nrx];  // the later steps read the count here, in stream order
      continue;
    }
    if (!flags[j]) continue;
    const nicgpu_segment_write w = writes[j];
    uint64_t len = (uint64_t) w.prefix_len + w.len_a + w.len_b;
    if (len > NICGPU_MAX_PACKET) len = NICGPU_MAX_PACKET;
    desc[at[j]] = NICGPU_DESC(w.dst, len);
    which[at[j]] = (uint32_t) j;
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_scatter_kernel(const uint32_t* __restrict__ which,
                                                              const uint32_t* __restrict__ h,
                                                              const uint16_t* __restrict__ q,
                                                              const unsigned long long* __restrict__ count,
                                                              uint32_t* rx_hash, uint16_t* rx_queue) {
  const uint64_t m = *count;
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < m; k += (uint64_t) gridDim.x * kQpBlock) {
    rx_hash[which[k]] = h[k];
    rx_queue[which[k]] = q[k];
  }
}

// sort keys of the first nrx RSS entries: the queue of the first *count, a
// key past every queue (nq) for the rest, so the sort leaves them last
__global__ __launch_bounds__(kQpBlock) void qp_keys_kernel(const uint16_t* __restrict__ q,
                                                           const unsigned long long* __restrict__ count, uint64_t nrx,
                                                           uint32_t nq, uint32_t* key) {
  const uint64_t m = count ? *count : nrx;
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < nrx; k += (uint64_t) gridDim.x * kQpBlock)
    key[k] = k < m ? (uint32_t) q[k] : nq;
}

// Dispatch lists for tables of fewer than 64 queues: a stable counting sort
// of the keys (queue of each delivered frame, nq for entries past *count) in
// 64-entry tiles, one wave per tile.  qp_gcount_kernel writes each tile's
// per-key counts in key-major order (cnt[key * T + tile], plus a trailing 0);
// their exclusive scan is every (key, tile)'s first output slot, and
// qp_gscatter_kernel adds each entry's rank among the tile's entries of its
// key (ballot + mbcnt) — the order radix sort keeps, in 4 launches instead of
// rocprim's ~20 merge-sort passes (128 of ~1020 us of kernels per 1 M batch).
__global__ __launch_bounds__(kQpBlock) void qp_gcount_kernel(const uint16_t* __restrict__ q,
                                                             const unsigned long long* __restrict__ count,
                                                             uint64_t nrx, uint32_t nq, uint64_t T, uint32_t* cnt) {
  const uint64_t m = count ? *count : nrx;
  const uint32_t lane = lane_id();
  const uint64_t waves = (uint64_t) gridDim.x * (kQpBlock / kWave);
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(uint64_t) (nq + 1) * T] = 0u;
  for (uint64_t t = (uint64_t) blockIdx.x * (kQpBlock / kWave) + threadIdx.x / kWave; t < T; t += waves) {
    const uint64_t k = t * kWave + lane;
    const uint32_t key = k < nrx ? (k < m && q[k] < nq ? (uint32_t) q[k] : nq) : nq + 1u;
    uint32_t mine = 0;
    for (uint32_t b = 0; b <= nq; ++b) {
      const uint32_t c = (uint32_t) __builtin_popcountll(__ballot(key == b));
      if (lane == b) mine = c;
    }
    if (lane <= nq) cnt[(uint64_t) lane * T + t] = mine;
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_gscatter_kernel(const uint16_t* __restrict__ q,
                                                               const unsigned long long* __restrict__ count,
                                                               uint64_t nrx, uint32_t nq, uint64_t T,
                                                               const uint32_t* __restrict__ off,
                                                               const uint32_t* __restrict__ which, uint32_t* out,
                                                               uint32_t* start, uint32_t* end) {
  const uint64_t m = count ? *count : nrx;
  const uint32_t lane = lane_id();
  const uint64_t waves = (uint64_t) gridDim.x * (kQpBlock / kWave);
  const uint64_t gt = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x;
  if (gt < nq) {  // queue gt's range; an empty queue gets start = end = 0
    const uint32_t a = off[gt * T], b = off[(gt + 1) * T];
    start[gt] = b > a ? a : 0u;
    end[gt] = b > a ? b : 0u;
  }
  for (uint64_t t = (uint64_t) blockIdx.x * (kQpBlock / kWave) + threadIdx.x / kWave; t < T; t += waves) {
    const uint64_t k = t * kWave + lane;
    const uint32_t key = k < nrx ? (k < m && q[k] < nq ? (uint32_t) q[k] : nq) : nq + 1u;
    uint32_t rank = 0;
    for (uint32_t b = 0; b <= nq; ++b) {
      const uint64_t v = __ballot(key == b);
      if (key == b) rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (v >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) v, 0u));
    }
    if (k < nrx) out[off[(uint64_t) key * T + t] + rank] = which ? which[k] : (uint32_t) k;
  }
}

__global__ __launch_bounds__(kQpBlock) void qp_iota_kernel(uint32_t* v, uint64_t n) {
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < n; k += (uint64_t) gridDim.x * kQpBlock)
    v[k] = (uint32_t) k;
}

// queue range boundaries of the first *count (null: nrx) sorted keys, for queues below nq
__global__ __launch_bounds__(kQpBlock) void qp_bounds_kernel(const uint32_t* __restrict__ key,
                                                             const unsigned long long* __restrict__ count, uint64_t nrx,
                                                             uint64_t nq, uint32_t* start, uint32_t* end) {
  const uint64_t m = count ? *count : nrx;
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < m; k += (uint64_t) gridDim.x * kQpBlock) {
    const uint32_t q = key[k];
    if (q >= nq) continue;
    if (k == 0 || key[k - 1] != q) start[q] = (uint32_t) k;
    if (k + 1 == m || key[k + 1] != q) end[q] = (uint32_t) (k + 1);
  }
}

// Overlap check (nicgpu_qp_check), the spans of rx_stage.cpp buffers_disjoint:
// what an RX descriptor can receive (at most buffer_length bytes inside the
// image, queue_pair.cpp:397-426) and what a TX descriptor is read from.
struct QpRxEnd {  // end of RX descriptor j's span; 0 when it receives nothing
  uint64_t mem_size;
  __host__ __device__ uint64_t operator()(const nicgpu_rx_descriptor& x) const {
    if (x.buffer_address >= mem_size || x.buffer_length == 0) return 0;
    const uint64_t room = mem_size - x.buffer_address;
    return x.buffer_address + (x.buffer_length < room ? (uint64_t) x.buffer_length : room);
  }
};

// end_max = inclusive running max of the RX span ends.  RX spans ascend and are
// disjoint iff every span starts at or after the running max before it
// (flag[0] stays 0); a TX span [a, b) then meets an RX span iff the first RX
// descriptor whose running max passes a (its own end, so it has a span) starts
// before b (flag[1]).  TX order does not matter.
__global__ __launch_bounds__(kQpBlock) void qp_check_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t ntx,
                                                            const nicgpu_rx_descriptor* __restrict__ rx, uint64_t nrx,
                                                            uint64_t mem_size, const uint64_t* __restrict__ end_max,
                                                            unsigned long long* flag) {
  const uint64_t n = ntx > nrx ? ntx : nrx;
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < n; k += (uint64_t) gridDim.x * kQpBlock) {
    if (k < nrx && k > 0 && QpRxEnd{mem_size}(rx[k]) != 0 && rx[k].buffer_address < end_max[k - 1]) flag[0] = 1;
    if (k < ntx) {
      const uint64_t a = tx[k].buffer_address, len = tx[k].length;
      if (len == 0 || !nicqp::dma_ok(mem_size, a, len)) continue;
      uint64_t lo = 0, hi = nrx;
      while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (end_max[mid] <= a) lo = mid + 1;
        else hi = mid;
      }
      if (lo < nrx && rx[lo].buffer_address < a + len) flag[1] = 1;
    }
  }
}

template <class T>
int qp_grow(T*& p, size_t& cap, size_t want) {
  if (want <= cap) return NICGPU_OK;
  if (p) (void) hipFree(p);
  p = nullptr;
  cap = 0;
  size_t n = want + want / 4 + 64;
  if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return NICGPU_ERR_NOMEM;
  cap = n;
  return NICGPU_OK;
}

}  // namespace

struct nicgpu_qp {
  int device = 0;
  size_t cap_tx = 0, cap_rx = 0, cap_pieces = 0, cap_tmp = 0, cap_part = 0;
  size_t c_tx = 0, c_rx = 0, c_plans = 0, c_counts = 0, c_base = 0, c_need = 0, c_pos = 0, c_txc = 0;
  size_t c_rxc = 0, c_w = 0, c_flags = 0, c_at = 0, c_desc = 0, c_which = 0, c_h = 0, c_q = 0, c_rh = 0, c_rq = 0;
  size_t c_pdesc = 0, c_pcs = 0, c_part = 0, c_tmp = 0;
  // the descriptors the kernels read: the context's own copies (tx_own /
  // rx_own, sized by nicgpu_qp_reserve) or the caller's (nicgpu_qp_bind)
  nicgpu_tx_descriptor* tx = nullptr;
  nicgpu_rx_descriptor* rx = nullptr;
  nicgpu_tx_descriptor* tx_own = nullptr;
  nicgpu_rx_descriptor* rx_own = nullptr;
  uint8_t* tmp_chk = nullptr;  // nicgpu_qp_check's scan storage (it may run beside a resolve)
  size_t c_tmp_chk = 0;
  QpPlan* plans = nullptr;
  uint32_t *counts = nullptr, *base = nullptr, *need = nullptr, *pos = nullptr;
  uint64_t* piece_desc = nullptr;
  uint16_t* piece_csum = nullptr;
  nicgpu_completion *txc = nullptr, *rxc = nullptr;
  nicgpu_segment_write* writes = nullptr;
  uint32_t *flags = nullptr, *at = nullptr, *which = nullptr, *rss_hash = nullptr, *rx_hash = nullptr;
  uint64_t* rss_desc = nullptr;
  uint16_t *rss_queue = nullptr, *rx_queue = nullptr;
  uint64_t* partials = nullptr;
  uint32_t *sort_key = nullptr, *sorted_key = nullptr;
  uint32_t *queue_which = nullptr, *queue_start = nullptr, *queue_end = nullptr;
  size_t c_sk = 0, c_qw = 0, c_em = 0, c_key = 0;
  uint64_t* end_max = nullptr;  // [nrx] nicgpu_qp_check's running max of RX span ends
  unsigned long long* scal = nullptr;
  uint8_t* tmp = nullptr;
  uint64_t host_scal[4] = {0, 0, 0, 0};
  // page-locked landing space of the small downloads (a pageable one is staged
  // and waited for on the host): [kQpTail] the resolve's RX count, first
  // mismatch, settled prefix and stats totals, then misc(): piece count, check
  // flags, relax verdict
  uint64_t* hp = nullptr;
  uint64_t* misc() const { return hp + kQpTail; }
  unsigned grid = 1;
  hipEvent_t planned = nullptr;   // nicgpu_qp_plan_on: the piece descriptors are written
  hipEvent_t resolved = nullptr;  // nicgpu_qp_resolve_start: its partials are on the host
  // the resolve between nicgpu_qp_resolve_start and _finish
  struct Pending {
    bool on = false;
    uint64_t mem_size = 0, ntx = 0, nrx = 0, max_mtu = 0;
    uint16_t queue_id = 0;
    hipStream_t s = nullptr;
    unsigned grid = 1;
  } res;
  bool delivered = false;  // the RSS results are per completion (nicgpu_qp_deliver), not compacted
};

namespace {

void qp_fill_view(const nicgpu_qp* q, nicgpu_qp_view* v) {
  if (!v) return;
  v->tx = q->tx;
  v->rx = q->rx;
  v->piece_base = q->base;
  v->piece_csum = q->piece_csum;
  v->txc = q->txc;
  v->rxc = q->rxc;
  v->writes = q->writes;
  v->rss_desc = q->rss_desc;
  v->rss_hash = q->rss_hash;
  v->rss_queue = q->rss_queue;
  v->rx_hash = q->rx_hash;
  v->rx_queue = q->rx_queue;
  v->queue_which = q->queue_which;
  v->queue_start = q->queue_start;
  v->queue_end = q->queue_end;
  v->rss_count = reinterpret_cast<uint64_t*>(q->scal + 3);
}

unsigned qp_grid(const nicgpu_qp* q, uint64_t n) {
  const uint64_t want = (n + kQpBlock) / kQpBlock;
  return (unsigned) (want < q->grid ? (want ? want : 1) : q->grid);
}

// hipcub exclusive sum of in[0, n) into out[0, n) (n includes the trailing 0)
int qp_scan(nicgpu_qp* q, const uint32_t* in, uint32_t* out, size_t n, hipStream_t s) {
  size_t tb = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int) n, s) != hipSuccess) return NICGPU_ERR_HIP;
  int st = qp_grow(q->tmp, q->c_tmp, tb);
  if (st != NICGPU_OK) return st;
  return hip_status(hipcub::DeviceScan::ExclusiveSum(q->tmp, tb, in, out, (int) n, s));
}

}  // namespace

extern "C" {

int nicgpu_qp_create(nicgpu_qp** out, int device) {
  if (!out) return NICGPU_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NICGPU_ERR_NO_DEVICE;
  DeviceGuard g(device);
  const DeviceInfo& di = device_info(device);
  if (di.status != NICGPU_OK) return di.status;
  auto* q = new nicgpu_qp();
  q->device = device;
  q->grid = (unsigned) di.cus * 8u;
  if (hipMalloc(&q->scal, 4 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&q->partials, ((size_t) q->grid * kQpStats + kQpTail) * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&q->queue_start, 65536 * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&q->queue_end, 65536 * sizeof(uint32_t)) != hipSuccess) {
    nicgpu_qp_destroy(q);
    return NICGPU_ERR_NOMEM;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&q->hp), (kQpTail + 16) * sizeof(uint64_t)) !=
      hipSuccess) {
    nicgpu_qp_destroy(q);
    return NICGPU_ERR_NOMEM;
  }
  if (hipEventCreateWithFlags(&q->planned, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&q->resolved, hipEventDisableTiming) != hipSuccess) {
    nicgpu_qp_destroy(q);
    return NICGPU_ERR_HIP;
  }
  *out = q;
  return NICGPU_OK;
}

int nicgpu_qp_destroy(nicgpu_qp* q) {
  if (!q) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  void* bufs[] = {q->tx_own, q->rx_own, q->tmp_chk, q->plans, q->counts, q->base, q->need, q->pos, q->piece_desc, q->piece_csum,
                  q->txc, q->rxc, q->writes, q->flags, q->at, q->which, q->rss_hash, q->rx_hash, q->rss_desc,
                  q->rss_queue, q->rx_queue, q->partials, q->scal, q->tmp, q->sort_key, q->sorted_key, q->queue_which,
                  q->queue_start, q->queue_end, q->end_max};
  for (void* b : bufs)
    if (b) (void) hipFree(b);
  if (q->hp) (void) hipHostFree(q->hp);
  if (q->planned) (void) hipEventDestroy(q->planned);
  if (q->resolved) (void) hipEventDestroy(q->resolved);
  delete q;
  return NICGPU_OK;
}

int nicgpu_qp_reserve(nicgpu_qp* q, size_t ntx, size_t nrx, nicgpu_qp_view* view) {
  if (!q) return NICGPU_ERR_INVALID;
  // 32-bit ring positions; hipcub scans and sorts take int counts
  static_assert(NICGPU_QP_MAX_TX == 0xFFFFFFFFull / kQpMaxPieces, "include/nicgpu.h limit");
  if (ntx > NICGPU_QP_MAX_TX || nrx > NICGPU_QP_MAX_RX) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  int st = NICGPU_OK;
  const size_t t1 = ntx + 1, r1 = nrx + 1;
  if (st == NICGPU_OK) st = qp_grow(q->tx_own, q->c_tx, ntx ? ntx : 1);
  if (st == NICGPU_OK) st = qp_grow(q->rx_own, q->c_rx, nrx ? nrx : 1);
  q->tx = q->tx_own;
  q->rx = q->rx_own;
  if (st == NICGPU_OK) st = qp_grow(q->plans, q->c_plans, t1);
  if (st == NICGPU_OK) st = qp_grow(q->counts, q->c_counts, t1);
  if (st == NICGPU_OK) st = qp_grow(q->base, q->c_base, t1);
  if (st == NICGPU_OK) st = qp_grow(q->need, q->c_need, t1);
  if (st == NICGPU_OK) st = qp_grow(q->pos, q->c_pos, t1);
  if (st == NICGPU_OK) st = qp_grow(q->txc, q->c_txc, t1);
  if (st == NICGPU_OK) st = qp_grow(q->rxc, q->c_rxc, r1);
  if (st == NICGPU_OK) st = qp_grow(q->writes, q->c_w, r1);
  if (st == NICGPU_OK) st = qp_grow(q->flags, q->c_flags, r1);
  if (st == NICGPU_OK) st = qp_grow(q->at, q->c_at, r1);
  if (st == NICGPU_OK) st = qp_grow(q->rss_desc, q->c_desc, r1);
  if (st == NICGPU_OK) st = qp_grow(q->which, q->c_which, r1);
  if (st == NICGPU_OK) st = qp_grow(q->rss_hash, q->c_h, r1);
  if (st == NICGPU_OK) st = qp_grow(q->rss_queue, q->c_q, r1);
  if (st == NICGPU_OK) st = qp_grow(q->rx_hash, q->c_rh, r1);
  if (st == NICGPU_OK) st = qp_grow(q->rx_queue, q->c_rq, r1);
  if (st == NICGPU_OK) st = qp_grow(q->sort_key, q->c_key, r1);
  if (st == NICGPU_OK) st = qp_grow(q->sorted_key, q->c_sk, r1);
  if (st == NICGPU_OK) st = qp_grow(q->queue_which, q->c_qw, r1);
  if (st == NICGPU_OK) st = qp_grow(q->end_max, q->c_em, r1);
  q->cap_tx = ntx;
  q->cap_rx = nrx;
  qp_fill_view(q, view);
  return st;
}

int nicgpu_qp_bind(nicgpu_qp* q, const nicgpu_tx_descriptor* tx, size_t ntx, const nicgpu_rx_descriptor* rx,
                   size_t nrx, nicgpu_qp_view* view) {
  if (!q || ntx > q->cap_tx || nrx > q->cap_rx || (ntx && !tx) || (nrx && !rx)) return NICGPU_ERR_INVALID;
  q->tx = ntx ? const_cast<nicgpu_tx_descriptor*>(tx) : q->tx_own;
  q->rx = nrx ? const_cast<nicgpu_rx_descriptor*>(rx) : q->rx_own;
  qp_fill_view(q, view);
  return NICGPU_OK;
}

int nicgpu_qp_plan(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                   uint64_t* npieces, nicgpu_qp_view* view, void* stream) {
  return nicgpu_qp_plan_on(q, mem, mem_size, ntx, max_mtu, npieces, view, stream, stream);
}

int nicgpu_qp_plan_on(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                      uint64_t* npieces, nicgpu_qp_view* view, void* plan_stream, void* sums_stream) {
  if (!q || !npieces || ntx > q->cap_tx) return NICGPU_ERR_INVALID;
  if (mem_size && (!mem || (reinterpret_cast<uintptr_t>(mem) & 15u) != 0)) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(plan_stream);
  *npieces = 0;
  const unsigned grid = qp_grid(q, ntx + 1);
  int st = hip_status(hipMemsetAsync(q->counts + ntx, 0, sizeof(uint32_t), s));
  if (st == NICGPU_OK)
    hipLaunchKernelGGL(qp_count_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                       q->plans, q->counts);
  if (st == NICGPU_OK) st = hip_status(hipGetLastError());
  uint32_t* np_h = reinterpret_cast<uint32_t*>(q->misc());
  // the overflow flag first: the scan below adds it in as the last count
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(np_h + 1, q->counts + ntx, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = qp_scan(q, q->counts, q->base, ntx + 1, s);
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(np_h, q->base + ntx, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  if (st != NICGPU_OK) return st;
  if (np_h[1] != 0u) return NICGPU_ERR_RANGE;
  const uint64_t np = *np_h;
  st = qp_grow(q->piece_desc, q->c_pdesc, np ? np : 1);
  if (st == NICGPU_OK) st = qp_grow(q->piece_csum, q->c_pcs, np ? np : 1);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_fill_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                     q->plans, q->base, q->piece_desc);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && sums_stream != plan_stream) {  // the sums read the pieces the fill wrote
    st = hip_status(hipEventRecord(q->planned, s));
    if (st == NICGPU_OK) st = hip_status(hipStreamWaitEvent(static_cast<hipStream_t>(sums_stream), q->planned, 0));
  }
  if (st == NICGPU_OK && np) st = nicgpu_checksum_batch(mem, q->piece_desc, np, q->piece_csum, sums_stream);
  *npieces = np;
  qp_fill_view(q, view);
  return st;
}

int nicgpu_qp_check(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, int* verdict, void* stream) {
  if (!q || !verdict || ntx > q->cap_tx || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  *verdict = -1;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int st = hip_status(hipMemsetAsync(q->scal, 0, 2 * sizeof(unsigned long long), s));
  if (st == NICGPU_OK && nrx) {
    hipcub::TransformInputIterator<uint64_t, QpRxEnd, const nicgpu_rx_descriptor*> ends(q->rx, QpRxEnd{mem_size});
    size_t tb = 0;
    if (hipcub::DeviceScan::InclusiveScan(nullptr, tb, ends, q->end_max, hipcub::Max(), (int) nrx, s) != hipSuccess)
      return NICGPU_ERR_HIP;
    st = qp_grow(q->tmp_chk, q->c_tmp_chk, tb);
    if (st == NICGPU_OK)
      st = hip_status(hipcub::DeviceScan::InclusiveScan(q->tmp_chk, tb, ends, q->end_max, hipcub::Max(), (int) nrx, s));
  }
  if (st != NICGPU_OK) return st;
  const uint64_t n = ntx > nrx ? ntx : nrx;
  if (n) {
    hipLaunchKernelGGL(qp_check_kernel, dim3(qp_grid(q, n)), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, q->rx,
                       (uint64_t) nrx, mem_size, q->end_max, q->scal);
    st = hip_status(hipGetLastError());
  }
  uint64_t* f = q->misc() + 1;
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(f, q->scal, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  if (st != NICGPU_OK) return st;
  *verdict = f[0] ? -1 : (f[1] ? 0 : 1);
  return NICGPU_OK;
}

int nicgpu_qp_resolve_start(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, uint64_t max_mtu,
                            uint16_t queue_id, void* stream) {
  if (!q || ntx > q->cap_tx || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  q->res = nicgpu_qp::Pending{};
  QpCtx C{queue_id, max_mtu, mem_size, q->plans, q->piece_csum, q->tx, q->rx, (uint64_t) nrx};
  const unsigned grid = qp_grid(q, ntx + 1);
  uint64_t* tail = q->partials + (size_t) grid * kQpStats;
  // first guess: every packet pops what it needs (rx_need).  The final pass
  // runs on it speculatively and reports the first packet that popped
  // otherwise; a batch that settles at once (uniform RX descriptors, no early
  // ends) needs no relaxation step and no host round trip before its DMA writes.
  hipLaunchKernelGGL(qp_need_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, (uint64_t) ntx, q->need,
                     reinterpret_cast<unsigned long long*>(tail + 1));
  int st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->need, q->pos, ntx + 1, s);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_full_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->pos, (uint64_t) ntx, q->txc, q->rxc,
                     q->writes, q->partials, q->need);
  st = hip_status(hipGetLastError());
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_reduce_kernel, dim3(1), dim3(kQpReduceThreads), 0, s, q->partials, grid, q->pos,
                     (uint64_t) ntx, true);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->hp, tail, kQpTail * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipEventRecord(q->resolved, s));
  if (st != NICGPU_OK) return st;
  q->res = nicgpu_qp::Pending{true, mem_size, (uint64_t) ntx, (uint64_t) nrx, max_mtu, queue_id, s, grid};
  return NICGPU_OK;
}

int nicgpu_qp_resolve_finish(nicgpu_qp* q, uint64_t* done, uint64_t* rx_used, uint64_t* rx_settled,
                             nicgpu_qp_stats* stats) {
  if (!q || !done || !rx_used || !stats || !q->res.on) return NICGPU_ERR_INVALID;
  const nicgpu_qp::Pending R = q->res;
  q->res.on = false;
  DeviceGuard g(q->device);
  hipStream_t s = R.s;
  const uint64_t ntx = R.ntx;
  QpCtx C{R.queue_id, R.max_mtu, R.mem_size, q->plans, q->piece_csum, q->tx, q->rx, R.nrx};
  const unsigned grid = R.grid;
  const uint64_t* part = q->hp;  // the tail, kQpTail words (page-locked)
  uint64_t* tail = q->partials + (size_t) grid * kQpStats;
  int st = hip_status(hipEventSynchronize(q->resolved));
  if (st != NICGPU_OK) return st;
  uint64_t used = part[0];
  const unsigned long long first0 = (unsigned long long) part[1];
  const uint64_t settled = part[2];
  unsigned long long first = first0;
  uint64_t lim = ntx;
  if (first < ntx) {  // relax from the same guess (the speculative pass left `need` as it was)
    // everything from here waits on the stream, behind whatever was enqueued
    // after the start (a settled-prefix delivery reads none of what follows)
    for (int it = 0; st == NICGPU_OK; ++it) {
      if (it > 0) st = qp_scan(q, q->need, q->pos, ntx + 1, s);
      q->misc()[4] = ntx;  // page-locked source; the step below waits for the stream
      if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->scal, q->misc() + 4, sizeof(uint64_t), hipMemcpyHostToDevice, s));
      if (st != NICGPU_OK) break;
      hipLaunchKernelGGL(qp_relax_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->need, q->pos, ntx, q->scal);
      st = hip_status(hipGetLastError());
      if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->misc() + 3, q->scal, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
      if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
      if (st != NICGPU_OK) break;
      first = (unsigned long long) q->misc()[3];
      // pos is exact up to and including `first` (pops before it agreed)
      lim = first < ntx ? (uint64_t) first : ntx;
      if (first >= ntx || it + 1 == kQpRelaxSteps) break;
    }
    if (st == NICGPU_OK) {
      hipLaunchKernelGGL(qp_full_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->pos, lim, q->txc, q->rxc, q->writes,
                         q->partials, static_cast<const uint32_t*>(nullptr));
      st = hip_status(hipGetLastError());
    }
    if (st == NICGPU_OK) {
      hipLaunchKernelGGL(qp_reduce_kernel, dim3(1), dim3(kQpReduceThreads), 0, s, q->partials, grid, q->pos, ntx, false);
      st = hip_status(hipGetLastError());
    }
    if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->hp, tail, kQpTail * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
    if (st != NICGPU_OK) return st;
    used = part[0];
  }
  std::memcpy(stats, part + 3, kQpStats * sizeof(uint64_t));
  *done = lim;
  *rx_used = used;
  if (rx_settled) *rx_settled = settled < used ? settled : used;
  return NICGPU_OK;
}

int nicgpu_qp_resolve(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, uint64_t max_mtu, uint16_t queue_id,
                      uint64_t* done, uint64_t* rx_used, nicgpu_qp_stats* stats, void* stream) {
  if (!q || !done || !rx_used || !stats) return NICGPU_ERR_INVALID;
  const int st = nicgpu_qp_resolve_start(q, mem_size, ntx, nrx, max_mtu, queue_id, stream);
  if (st != NICGPU_OK) return st;
  return nicgpu_qp_resolve_finish(q, done, rx_used, nullptr, stats);
}

int nicgpu_qp_rss_list(nicgpu_qp* q, size_t nrx, void* stream) {
  if (!q || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  q->delivered = false;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned grid = qp_grid(q, nrx + 1);
  hipLaunchKernelGGL(qp_flag_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->rxc, (uint64_t) nrx, q->flags, q->rx_hash,
                     q->rx_queue);
  int st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->flags, q->at, nrx + 1, s);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_rss_fill_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->flags, q->at, q->writes, (uint64_t) nrx,
                     q->rss_desc, q->which, q->scal + 3);
  return hip_status(hipGetLastError());
}

int nicgpu_qp_group(nicgpu_qp* q, size_t nrx, size_t nq, void* stream) {
  if (!q || nrx > q->cap_rx || nq > 65536) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int st = NICGPU_OK;
  if (nq && (nq >= kWave || nrx == 0)) {  // the counting sort writes every queue's bounds itself
    st = hip_status(hipMemsetAsync(q->queue_start, 0, nq * sizeof(uint32_t), s));
    if (st == NICGPU_OK) st = hip_status(hipMemsetAsync(q->queue_end, 0, nq * sizeof(uint32_t), s));
  }
  if (st != NICGPU_OK || nrx == 0) return st;
  // after nicgpu_qp_deliver: the queue of every completion (0xFFFF unless
  // Success), in posting order, and the completion's own index as its entry;
  // after nicgpu_qp_rss_list + scatter: the compacted Success frames
  const uint16_t* keyq = q->delivered ? q->rx_queue : q->rss_queue;
  const unsigned long long* cnt = q->delivered ? nullptr : reinterpret_cast<const unsigned long long*>(q->scal + 3);
  const uint32_t* which = q->delivered ? nullptr : q->which;
  if (nq < kWave) {  // counting sort: counts in sort_key, their scan in sorted_key (both hold nrx + 64)
    const uint64_t T = (nrx + kWave - 1) / kWave;
    const uint64_t nc = (uint64_t) (nq + 1) * T + 1;
    st = qp_grow(q->sort_key, q->c_key, nc);
    if (st == NICGPU_OK) st = qp_grow(q->sorted_key, q->c_sk, nc);
    if (st != NICGPU_OK) return st;
    const unsigned grid = qp_grid(q, nrx > nq ? nrx : nq);
    hipLaunchKernelGGL(qp_gcount_kernel, dim3(grid), dim3(kQpBlock), 0, s, keyq, cnt, (uint64_t) nrx,
                       (uint32_t) nq, T, q->sort_key);
    st = hip_status(hipGetLastError());
    if (st == NICGPU_OK) st = qp_scan(q, q->sort_key, q->sorted_key, nc, s);
    if (st != NICGPU_OK) return st;
    hipLaunchKernelGGL(qp_gscatter_kernel, dim3(grid), dim3(kQpBlock), 0, s, keyq, cnt,
                       (uint64_t) nrx, (uint32_t) nq, T, q->sorted_key, which, q->queue_which, q->queue_start,
                       q->queue_end);
    return hip_status(hipGetLastError());
  }
  hipLaunchKernelGGL(qp_keys_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, keyq, cnt,
                     (uint64_t) nrx, (uint32_t) nq, q->sort_key);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && q->delivered)  // the sort's values: each completion's index
    hipLaunchKernelGGL(qp_iota_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, q->which, (uint64_t) nrx);
  if (st == NICGPU_OK) st = hip_status(hipGetLastError());
  if (st != NICGPU_OK) return st;
  // stable: each queue keeps its completions in posting order.  Keys run
  // 0..nq, so only their low bits are sorted (16 queues: 5 bits, one pass).
  int end_bit = 1;
  while ((1ull << end_bit) <= (unsigned long long) nq) ++end_bit;
  size_t tb = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, q->sort_key, q->sorted_key, q->which, q->queue_which, (int) nrx,
                                         0, end_bit, s) != hipSuccess)
    return NICGPU_ERR_HIP;
  st = qp_grow(q->tmp, q->c_tmp, tb);
  if (st == NICGPU_OK)
    st = hip_status(hipcub::DeviceRadixSort::SortPairs(q->tmp, tb, q->sort_key, q->sorted_key, q->which,
                                                       q->queue_which, (int) nrx, 0, end_bit, s));
  if (st != NICGPU_OK || nq == 0) return st;
  hipLaunchKernelGGL(qp_bounds_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, q->sorted_key, cnt,
                     (uint64_t) nrx, (uint64_t) nq, q->queue_start, q->queue_end);
  return hip_status(hipGetLastError());
}

int nicgpu_qp_rss_scatter(nicgpu_qp* q, size_t nrx, void* stream) {
  if (!q || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  if (nrx == 0) return NICGPU_OK;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(qp_scatter_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, q->which, q->rss_hash,
                     q->rss_queue, q->scal + 3, q->rx_hash, q->rx_queue);
  return hip_status(hipGetLastError());
}


int nicgpu_qp_deliver(nicgpu_qp* q, uint8_t* mem, uint64_t mem_size, size_t nrx, const nicgpu_rss_ctx* ctx,
                      int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint64_t* hits_dev, void* stream) {
  return nicgpu_qp_deliver_range(q, mem, mem_size, 0, nrx, 0u, ctx, tuple_mode, raw_off, raw_len, hits_dev, stream);
}

int nicgpu_qp_deliver_range(nicgpu_qp* q, uint8_t* mem, uint64_t mem_size, size_t rx_begin, size_t rx_end,
                            unsigned flags, const nicgpu_rss_ctx* ctx, int tuple_mode, uint32_t raw_off,
                            uint32_t raw_len, uint64_t* hits_dev, void* stream) {
  if (!q || rx_end > q->cap_rx || rx_begin > rx_end) return NICGPU_ERR_INVALID;
  if (flags & ~(unsigned) (NICGPU_DELIVER_SETTLED | NICGPU_DELIVER_APPEND)) return NICGPU_ERR_INVALID;
  // the settled prefix of the resolve started last (its grid places the tail)
  if ((flags & NICGPU_DELIVER_SETTLED) && !q->res.on) return NICGPU_ERR_INVALID;
  if (mem_size && (!mem || (reinterpret_cast<uintptr_t>(mem) & 15u) != 0)) return NICGPU_ERR_INVALID;
  if (tuple_mode != NICGPU_TUPLE_NONE && tuple_mode != NICGPU_TUPLE_AUTO && tuple_mode != NICGPU_TUPLE_RAW)
    return NICGPU_ERR_INVALID;
  if (tuple_mode == NICGPU_TUPLE_RAW && (raw_off > NICGPU_RAW_MAX_END || raw_len > NICGPU_RAW_MAX_END ||
                                         raw_off + raw_len > NICGPU_RAW_MAX_END))
    return NICGPU_ERR_INVALID;
  const bool rss = tuple_mode != NICGPU_TUPLE_NONE;
  if (rss && (!ctx || ctx->table_n == 0 || !hits_dev || ctx->device != q->device)) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  q->delivered = rss;
  int st = NICGPU_OK;
  if (rss && !(flags & NICGPU_DELIVER_APPEND)) st = hip_status(hipMemsetAsync(q->scal + 3, 0, sizeof(uint64_t), s));
  if (st != NICGPU_OK || rx_end == rx_begin) return st;
  const DeviceInfo* di = nullptr;
  st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  DeliverParams P{};
  P.mem = mem;
  P.mem_size = mem_size;
  P.w = q->writes;
  P.rxc = q->rxc;
  P.j0 = rx_begin;
  P.n = rx_end;
  if (flags & NICGPU_DELIVER_SETTLED)
    P.n_dev = reinterpret_cast<const unsigned long long*>(q->partials + (size_t) q->res.grid * kQpStats + 2);
  P.rss.mode = tuple_mode;
  P.rss.raw_off = raw_off;
  P.rss.raw_len = raw_len;
  if (rss) {
    P.rss.lut = ctx->d_lut;
    P.rss.table = ctx->d_table;
    P.rss.table_n = (uint32_t) ctx->table_n;
    P.rss.lut_words = 2u * (tuple_mode == NICGPU_TUPLE_RAW ? raw_len : 36u) * 16u;
    P.rx_hash = q->rx_hash;
    P.rx_queue = q->rx_queue;
    P.hits = reinterpret_cast<unsigned long long*>(hits_dev);
    P.count = reinterpret_cast<unsigned long long*>(q->scal + 3);
#ifdef NICGPU_HIST_REP
    if (P.rss.table_n <= (uint32_t) kHistLds) {
      P.rss.hits_rep = ctx->d_rep;
      P.rss.hits_done = ctx->d_done;
    }
#endif
  }
  const uint32_t hist_n = (rss && P.rss.table_n <= (uint32_t) kHistLds) ? P.rss.table_n : 0u;
  const uint32_t table_words = (rss && P.rss.table_n <= (uint32_t) kTableLds) ? (P.rss.table_n + 1u) / 2u : 0u;
  const uint32_t lds = dlv_block_bytes(rss, P.rss.lut_words, hist_n, table_words) + kDlvWpb * kDlvWaveBytes;
  int dev = 0;
  (void) hipGetDevice(&dev);
  const int bpc = rss ? dlv_blocks_per_cu<true>(dev, lds) : dlv_blocks_per_cu<false>(dev, lds);
  const uint64_t ntiles = (rx_end - rx_begin + kWave - 1) / kWave;
  const uint64_t want = (ntiles + kDlvWpb - 1) / kDlvWpb;
  // CUs left without a delivery block, so the next batch's plan and check
  // (small launches on a side stream) find wave slots while this one runs
  static const int reserve = [] {
    const char* e = std::getenv("NICGPU_DLV_RESERVE_CUS");
    return e ? std::atoi(e) : kDlvReserveCus;
  }();
  const uint64_t cus = (uint64_t) (di->cus > reserve + 8 ? di->cus - reserve : di->cus);
  const uint64_t cap = cus * (uint64_t) bpc;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  if (rss) hipLaunchKernelGGL(deliver_kernel<true>, dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  else hipLaunchKernelGGL(deliver_kernel<false>, dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  return hip_status(hipGetLastError());
}

}  // extern "C"

#ifdef NICGPU_TUNING
// ------------------------------------------------------------------------
// Tuning-only entry points (built into libnicgpu_tune.so, never into the
// product library): run any RX kernel variant, and a read-only streaming
// kernel that measures this box's HBM read ceiling with the same access width.
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
int nicgpu_tune_num_variants(void) { return kNumRxVariants; }
const char* nicgpu_tune_variant_name(int v) { return (v >= 0 && v < kNumRxVariants) ? kRxVariants[v].name : ""; }
void nicgpu_tune_set_dbg(uint32_t bits) { g_tune_dbg = bits; }
// per-wave {start, end, XCC_ID, HW_ID} of every RX launch into buf (4 u64 per
// wave of the grid; NULL switches it off)
void nicgpu_tune_set_stamps(unsigned long long* buf) { g_tune_stamps = buf; }
void nicgpu_tune_set_xpf(uint32_t max_chunks) { g_xpf_chunks = max_chunks; }
void nicgpu_tune_set_bpc(uint32_t cap) { g_bpc_cap = cap; }
int nicgpu_tune_rx_offload(int variant, const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc,
                           size_t n, int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum,
                           uint32_t* out_hash, uint16_t* out_queue, uint64_t* out_hits, void* stream) {
  return rx_offload_impl(variant, ctx, frames, desc, n, tuple_mode, raw_off, raw_len, out_csum, out_hash,
                         out_queue, out_hits, nullptr, stream);
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
#endif  // NICGPU_TUNING
