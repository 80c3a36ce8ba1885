// rx.hip — the hot path: nic::compute_checksum (src/checksum.cpp:10-34) and
// nic::RssEngine::select_queue (src/rss.cpp:43-94) fused into ONE streaming
// pass over a packed batch of frames in HBM (rx_offload_kernel), and the
// header-only RSS pass (rss_only_kernel).  DESIGN.md §4.1, §4.2b.
//
//  * A wave owns a tile of 64 consecutive packets (one descriptor per lane).
//    The tile's bytes are walked as one flat stream of 16-B chunks: in every
//    step lane l loads chunk (base + l) with a dwordx4 load, so each wave
//    instruction reads up to 1 KiB of contiguous packet bytes whatever the
//    packet sizes — no lanes idle on short packets and no per-size kernels.
//  * checksum: v_dot2_u32_u16(d, {1,1}, acc) adds both little-endian halfwords of a
//    dword in one instruction; a wave-wide DPP inclusive scan turns chunk sums into a
//    running prefix, and each packet's sum is (prefix at its last chunk) -
//    (prefix before its first chunk).  The ones'-complement fold and the byte
//    swap happen once per packet.  Bit-exact with the reference's eager
//    per-add fold.
//  * RSS: the first 48 B of every packet are staged in LDS as they stream past;
//    the tuple is parsed from LDS and hashed with a nibble lookup table of
//    32-bit Toeplitz key windows (rss.hip), equivalent to the reference's
//    bit-serial `(bit + k) % key_bits` loop including key wrap.  queue = table[h % n].
//  * No MFMA: this is byte-integer work bounded by HBM read bandwidth.

#include "common.h"
#include "host.h"

#include <cstdlib>

#include <mutex>
#include <vector>

using namespace nicgpu_detail;

#ifdef NICGPU_TUNING
unsigned long long* nicgpu_detail::g_tune_stamps = nullptr;
#endif

namespace {

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
template <int U>
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
    B.v[u] = __builtin_nontemporal_load(p);
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
constexpr int kLoadNt = 2;  // gfx950 cache policy of the frame loads: nt (sc0/sc1 mixes equal or slower)

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
  t.contig = (__ballot(t.nch != 0u && t.delta != t.D) == 0ull) ? 1u : 0u;
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

// One lane's results of a tile (held in the wave's LDS result ring until it
// is flushed: DESIGN.md §4.1 "Result ring").
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
      if (P.out_cs4)  // (split sums: no RSS, the queue slot holds the first-4 sum)
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t) o.q,
                                              __builtin_amdgcn_make_buffer_rsrc(P.out_cs4 + tb, (short) 0, 128, 0x00020000),
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
  if (o.valid) {
    if (P.out_csum) P.out_csum[o.pid] = (uint16_t) o.cs;
    if (P.out_cs4) P.out_cs4[o.pid] = (uint16_t) o.q;
    if (l34 && P.out_l34) P.out_l34[o.pid] = (uint8_t) o.l34;
    if (rss) {
      if (P.out_hash) P.out_hash[o.pid] = o.h;
      if (P.out_queue) P.out_queue[o.pid] = (uint16_t) o.q;
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
    // LE halfword sums at absolute positions == byte-swapped BE sum when the
    // packet starts at an even address (RFC 1071 byte-order independence).
    auto finish = [&](uint32_t s) __attribute__((always_inline)) {
      const uint32_t x = fold16(s);
      return ~((t.off & 1) ? x : bswap16(x)) & 0xFFFFu;
    };
    if (P.out_cs4) {
      // split sums: the first min(4, len) bytes from the stage, at their
      // absolute halfword positions; the rest is the exact difference (sum
      // is the integer sum of the packet's halfwords), so both equal the
      // sums of two separate pieces [0, 4) and [4, len)
      const uint32_t lo = (uint32_t) (t.off & 15);
      const HdrView hv{L.hdr, lane};
      uint32_t head = 0;
#pragma unroll
      for (uint32_t i = 0; i < 4u; ++i)
        if (i < t.len) head += hv.byte(lo + i) << (8u * ((lo + i) & 1u));
      o.cs = finish(sum - head);
      o.q = finish(head);
    } else {
      o.cs = finish(sum);
    }
    if (P.out_l34)
      o.l34 = l34_flags(HdrView{L.hdr, lane}, reinterpret_cast<const uint32_t*>(P.frames + (t.off & ~15ull)),
                        (uint32_t) (t.off & 15), t.len, sum);
    if (L.want_rss) {
      const uint32_t h =
          rss_hash_packet(P, L.lut, HdrView{L.hdr, lane}, (uint32_t) (t.off & 15), P.frames + t.off, t.len);
      const uint32_t idx = h % P.table_n;
      o.h = h;
      if (P.out_queue) {
        if (L.table_lds) {
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
      if (P.out_hits) {
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
template <int U>
__device__ __forceinline__ void run_general_tile(const RxParams& P, const RxLdsPtrs& L, const Tile& t, uint32_t lane,
                                                 uint32_t& tag) {
  constexpr uint32_t kStep = (uint32_t) kWave * U;
  L.pk[lane] = make_uint4((uint32_t) (uint64_t) t.delta, (uint32_t) ((uint64_t) t.delta >> 32), t.end, t.info);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  uint32_t run = 0, carry = 0;
  ChunkBatch<U> A, B;
  uint32_t b0 = 0;
  // counted pair loop, single exit at the bottom (see the contiguous path)
  const uint32_t nbatch = (t.total + kStep - 1) / kStep;
  plan_batch<U>(A, L.pk, L.marks, b0, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
  uint32_t bi = 0;
  for (; bi + 1 < nbatch; bi += 2, b0 += 2 * kStep) {
    plan_batch<U>(B, L.pk, L.marks, b0 + kStep, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
    __builtin_amdgcn_sched_barrier(0);  // B's loads issue before A's wait
    run = process_batch<U>(A, run, L.S, L.E, L.hdr, L.stage);
    plan_batch<U>(A, L.pk, L.marks, b0 + 2 * kStep, t.total, lane, t.start, t.nch, ++tag, carry, P.frames);
    __builtin_amdgcn_sched_barrier(0);
    run = process_batch<U>(B, run, L.S, L.E, L.hdr, L.stage);
  }
  if (bi < nbatch) run = process_batch<U>(A, run, L.S, L.E, L.hdr, L.stage);
}

// U: 64-chunk loads per lane per batch (ping-pong: batch i+1's loads in
// flight while batch i is reduced).  WPB: waves per block.  SST: cache-policy
// bits of the result stores (0 plain, 16 sc1).  OCC: waves_per_eu hint.
// XPF: the next contiguous tile's first batch (slots scattered, loads issued)
// goes out before this tile's epilogue, so the epilogue overlaps its latency
// (tiles of at most P.xpf_chunks chunks).  Results are held in a per-wave LDS
// ring of P.hold_r tiles and stored when it is full and at the end, so output
// writes reach DRAM in bursts instead of interleaved with the read stream
// (DESIGN.md §4.1).  Loads are nontemporal.
// SPLIT 1: each wave takes one contiguous packet range instead of every
// nwaves-th tile, the ranges of the blockIdx % 8 groups (one XCD each under
// round-robin placement) weighted by P.xcd_w_odd so the odd XCDs, which end
// ~4-8% later (profiles/r02_wave_stamps_c2.jsonl), get less.  The split is a
// function of (blockIdx, wave) and the count only: every packet is covered
// exactly once wherever the blocks land; placement only affects its speed.
template <int U, int WPB, int SST, int OCC = 4, bool XPF = true, int SPLIT = 0>
__global__ __launch_bounds__(kWave * WPB) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void rx_offload_kernel(
    RxParams P) {
  extern __shared__ uint4 lds_dyn[];
  const int w = threadIdx.x / kWave;
  const uint32_t lane = lane_id();
  constexpr uint32_t kStep = (uint32_t) kWave * U;

  RxLdsPtrs L;
  L.want_rss = P.mode != NICGPU_TUPLE_NONE;
  L.stage = L.want_rss || P.out_l34 != nullptr || P.out_cs4 != nullptr;
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

  // Work split: tile k*W + g (round robin over the grid's waves).
  const uint64_t nwaves = (uint64_t) gridDim.x * WPB;
  const uint64_t gw = (uint64_t) blockIdx.x * WPB + w;
  // packets in this launch: n, or a count another kernel left on the device
  // (the grid is sized for n; waves past the count have no tile)
  const uint64_t n_all = P.n_dev ? (*P.n_dev < P.n ? (uint64_t) *P.n_dev : P.n) : P.n;
  uint64_t first = gw * kWave, end = n_all, step = nwaves * kWave;
  if constexpr (SPLIT == 1) {
    // group v = blockIdx % 8 gets [g0, g1), its waves equal parts of it in
    // (blockIdx / 8, wave) order; n_all * weight sums < 2^64 (the host keeps
    // n below 2^34); adjacent ranges share their boundary's expression
    const uint32_t G = gridDim.x, v = blockIdx.x & 7u;
    uint64_t cum = 0, tot = 0, mine = 0;
    for (uint32_t u = 0; u < 8u; ++u) {
      const uint64_t c = (uint64_t) ((G + 7u - u) / 8u) * ((u & 1u) ? (uint64_t) P.xcd_w_odd : 65536ull);
      if (u < v) cum += c;
      if (u == v) mine = c;
      tot += c;
    }
    const uint64_t g0 = n_all * cum / tot, g1 = cum + mine == tot ? n_all : n_all * (cum + mine) / tot;
    const uint64_t nw = (uint64_t) ((G + 7u - v) / 8u) * WPB,
                   rank = (uint64_t) (blockIdx.x >> 3) * WPB + (uint64_t) __builtin_amdgcn_readfirstlane(w);
    first = g0 + (g1 - g0) * rank / nw;
    end = rank + 1 == nw ? g1 : g0 + (g1 - g0) * (rank + 1) / nw;
    step = kWave;
  }
  auto nvalid_of = [&](uint64_t b) __attribute__((always_inline)) -> uint32_t {
    return b < end ? (uint32_t) (end - b < (uint64_t) kWave ? end - b : (uint64_t) kWave) : 0u;
  };
  auto desc_of = [&](uint64_t b) __attribute__((always_inline)) -> uint64_t {
    return lane < nvalid_of(b) ? P.desc[b + lane] : 0ull;
  };
  // descriptors are prefetched one tile ahead
  uint64_t d_next = desc_of(first + step);
  Tile cur = make_tile(first, nvalid_of(first), desc_of(first));
  uint8_t* ring = base_b + P.ring_off + (uint32_t) w * P.hold_r * kRingTileBytes;
  uint32_t ring_n = 0;
  uint64_t ring_base0 = 0;

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
    plan_contig<U, kLoadNt>(A, L.slotsA, 0, lane, t.start, t.nch, t.info, r);
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
      uint32_t bi = 0;
      for (; bi + 1 < nbatch; bi += 2, b0 += 2 * kStep) {
        plan_contig<U, kLoadNt>(B, L.slotsB, b0 + kStep, lane, cur.start, cur.nch, cur.info, rsrc);
        __builtin_amdgcn_sched_barrier(0);  // B's loads issue before A's wait
        run = process_contig<U>(A, L.slotsA, L.masks, run, L.E, L.hdr, L.stage, lane);
        plan_contig<U, kLoadNt>(A, L.slotsA, b0 + 2 * kStep, lane, cur.start, cur.nch, cur.info, rsrc);
        __builtin_amdgcn_sched_barrier(0);
        run = process_contig<U>(B, L.slotsB, L.masks, run, L.E, L.hdr, L.stage, lane);
      }
      if (bi < nbatch) run = process_contig<U>(A, L.slotsA, L.masks, run, L.E, L.hdr, L.stage, lane);
    } else if (cur.total != 0u) {
      run_general_tile<U>(P, L, cur, lane, tag);
    }
    const uint64_t nb = cur.base + step;
    const Tile nxt = make_tile(nb, nvalid_of(nb), d_next);
    pre = false;
    if (XPF && nxt.contig && nxt.total != 0u && nxt.total <= P.xpf_chunks) {
      rsrc_pre = tile_rsrc(nxt);
      tile_first(nxt, rsrc_pre);
      __builtin_amdgcn_sched_barrier(0);  // the next tile's loads go out before this tile's epilogue
      pre = true;
    }
    const TileOut o = tile_epilogue(P, L, cur, lane);
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
    cur = nxt;
    d_next = desc_of(nb + step);
  }

  flush_ring<SST>(P, L, ring, ring_n, ring_base0, step, lane, nvalid_of);
  if (L.hist_lds) flush_hist(L.hist, P.table_n, P.out_hits, P.hits_rep, P.hits_done, kWave * WPB);
#ifdef NICGPU_TUNING
  if (P.stamps != nullptr && lane == 0) {  // vector stores from lane 0
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    P.stamps[4 * gw + 0] = t_start;
    P.stamps[4 * gw + 1] = t_end;
    P.stamps[4 * gw + 2] = (unsigned) __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID[3:0]
    P.stamps[4 * gw + 3] = (unsigned) __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
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
  bool xpf = true;  // cross-tile prefetch (P.xpf_chunks)
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
    {rx_offload_kernel<2, 4, 16>, 2, 4, "u2_w4_c_sc1_ring_xpf"},
    {rx_offload_kernel<2, 4, 0>, 2, 4, "u2_w4_c_ring_xpf"},
    // 2: production for batches of at least kRxW8Tiles tiles.  8-wave blocks:
    // half the blocks add their histogram bins into the same counters at the
    // end (1024 -> 512 same-address atomics per bin).  IMIX (4 M packets) -2%,
    // 4 M x 64 B -3%; C2 +0.6% and 9000 B +15% (2500 tiles underfill 512
    // slots of 8 waves) keep 4-wave blocks (profiles/r02y_tune_variants.json).
    {rx_offload_kernel<2, 8, 16>, 2, 8, "u2_w8_c_sc1_ring_xpf"},
#ifdef NICGPU_TUNING
    // contiguous XCD-weighted ranges (SPLIT 1; P.xcd_w_odd from NICGPU_RX_XCD_ODD)
    {rx_offload_kernel<2, 4, 16, 4, true, 1>, 2, 4, "u2_w4_c_sc1_ring_xpf_xcd"},
    {rx_offload_kernel<2, 4, 0, 4, true, 1>, 2, 4, "u2_w4_c_ring_xpf_xcd"},
    {rx_offload_kernel<2, 8, 16, 4, true, 1>, 2, 8, "u2_w8_c_sc1_ring_xpf_xcd"},
    // candidates timed by tools/tune_rx.py (the rejected experiments of
    // DESIGN.md §7 — deferred stores, register-held results, non-contiguous
    // only, other load policies — are in git history before round 4)
    // deeper per-wave batches for lower occupancies (nicgpu_tune_set_bpc)
    {rx_offload_kernel<4, 4, 16, 1>, 4, 4, "u4_w4_c_sc1_ring_xpf"},
    {rx_offload_kernel<4, 4, 0, 1>, 4, 4, "u4_w4_c_ring_xpf"},
    {rx_offload_kernel<2, 4, 16, 1, false>, 2, 4, "u2_nt1_w4_c_sc1_ring", false},
    {rx_offload_kernel<2, 4, 0, 1, false>, 2, 4, "u2_nt1_w4_c_ring", false},
    // bigger blocks still: 256 same-address atomics per bin
    {rx_offload_kernel<2, 16, 16, 1>, 2, 16, "u2_w16_c_sc1_ring_xpf"},
#endif
};
constexpr int kNumRxVariants = (int) (sizeof(kRxVariants) / sizeof(kRxVariants[0]));
constexpr int kRxW8 = 2;
constexpr uint64_t kRxW8Tiles = 32768;  // 2 M packets: IMIX and 64-B batches of C3's size, not C2 (16 K tiles)

}  // namespace

namespace {
#ifdef NICGPU_TUNING
// tuning: at most this many RX blocks per CU (0 = occupancy maximum); the LDS
// request is padded so the hardware cannot place more (nicgpu_tune_set_bpc)
uint32_t g_bpc_cap = 0;
#endif

int rx_blocks_per_cu(int dev, int variant, uint32_t lds) {
  (void) dev;
#ifdef NICGPU_TUNING
  auto capped = [](int b) { return g_bpc_cap && b > (int) g_bpc_cap ? (int) g_bpc_cap : b; };
#else
  auto capped = [](int b) { return b; };
#endif
  const RxVariant& v = kRxVariants[variant];
  return capped(blocks_per_cu(reinterpret_cast<const void*>(v.kernel), kWave * v.wpb, lds));
}

// XPF variants prefetch the next tile's first batch for tiles up to this many
// 16-B chunks (tools/tune_rx.py sets it through nicgpu_tune_set_xpf).
uint32_t g_xpf_chunks = 0xFFFFFFFFu;

// LDS result ring of a variant at its occupancy: tiles held per wave
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

int rss_only_blocks_per_cu(uint32_t lds) {
  return blocks_per_cu(reinterpret_cast<const void*>(rss_only_kernel<kRssWpb>), kWave * kRssWpb, lds);
}

int launch_rss_only(const RxParams& P, const DeviceInfo& di, hipStream_t stream) {
  const uint32_t hist_n = (P.out_hits && P.table_n <= (uint32_t) kHistLds) ? P.table_n : 0u;
  const uint32_t table_words = P.table_n <= (uint32_t) kTableLds ? (P.table_n + 1u) / 2u : 0u;
  const uint32_t lds = rss_only_block_bytes(P.lut_words, hist_n, table_words) + kRssWpb * kRssOnlyWaveBytes;
  // as many blocks as fit a CU (registers and LDS), one grid-stride pass each
  const uint32_t bpc = (uint32_t) rss_only_blocks_per_cu(lds);
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
  const bool stage = rss || P.out_l34 != nullptr || P.out_cs4 != nullptr;
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
  // round robin: one tile per wave
  const uint64_t want = (ntiles + v.wpb - 1) / (uint64_t) v.wpb;
  int bpc = rx_blocks_per_cu(dev, variant, lds);
  RxParams Pl = P;
  Pl.xpf_chunks = v.xpf ? g_xpf_chunks : 0u;
  // the LDS result ring, sized from the LDS the occupancy leaves over
  const RingPlan rp = plan_ring(dev, variant, lds, ntiles, di);
  Pl.hold_r = rp.hold_r;
  Pl.ring_off = rp.ring_off;
  uint32_t lds_launch = rp.lds;
  bpc = rx_blocks_per_cu(dev, variant, lds_launch);
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

#ifdef NICGPU_TUNING
#endif
int rx_offload_impl(int variant, const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                    int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum, uint32_t* out_hash,
                    uint16_t* out_queue, uint64_t* out_hits, uint8_t* out_l34, void* stream,
                    const uint64_t* n_dev = nullptr, uint16_t* out_cs4 = nullptr) {
  if (tuple_mode != NICGPU_TUPLE_NONE && tuple_mode != NICGPU_TUPLE_AUTO && tuple_mode != NICGPU_TUPLE_RAW)
    return NICGPU_ERR_INVALID;
  if (tuple_mode == NICGPU_TUPLE_RAW && (raw_off > NICGPU_RAW_MAX_END || raw_len > NICGPU_RAW_MAX_END ||
                                         raw_off + raw_len > NICGPU_RAW_MAX_END))
    return NICGPU_ERR_INVALID;
  if (tuple_mode != NICGPU_TUPLE_NONE && (!ctx || ctx->table_n == 0)) return NICGPU_ERR_INVALID;
  if (tuple_mode == NICGPU_TUPLE_NONE && (out_hash || out_queue || out_hits)) return NICGPU_ERR_INVALID;
  if (out_cs4 && (!out_csum || tuple_mode != NICGPU_TUPLE_NONE)) return NICGPU_ERR_INVALID;
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
  P.out_cs4 = out_cs4;
  static const uint32_t xcd_odd = [] {
    const char* e = std::getenv("NICGPU_RX_XCD_ODD");  // tuning: odd groups' share x 65536
    return e ? (uint32_t) std::strtoul(e, nullptr, 10) : 61500u;
  }();
  P.xcd_w_odd = xcd_odd ? xcd_odd : 1u;
  P.n_dev = reinterpret_cast<const unsigned long long*>(n_dev);
#ifdef NICGPU_TUNING
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

}  // extern "C"

namespace nicgpu_detail {
int checksum_split_count(const uint8_t* frames, const uint64_t* desc, size_t n_max, const uint64_t* n_dev,
                         uint16_t* out_rest, uint16_t* out_head4, void* stream) {
  if (!n_dev || (n_max && (!out_rest || !out_head4))) return NICGPU_ERR_INVALID;
  return rx_offload_impl(0, nullptr, frames, desc, n_max, NICGPU_TUPLE_NONE, 0, 0, out_rest, nullptr, nullptr, nullptr,
                         nullptr, stream, n_dev, out_head4);
}
}  // namespace nicgpu_detail

extern "C" {

int nicgpu_checksum_batch_split(const uint8_t* frames, const uint64_t* desc, size_t n, uint16_t* out_rest,
                                uint16_t* out_head4, void* stream) {
  if (n && (!out_rest || !out_head4)) return NICGPU_ERR_INVALID;
  return rx_offload_impl(0, nullptr, frames, desc, n, NICGPU_TUPLE_NONE, 0, 0, out_rest, nullptr, nullptr, nullptr,
                         nullptr, stream, nullptr, out_head4);
}

}  // extern "C"

#ifdef NICGPU_TUNING
extern "C" {
int nicgpu_tune_num_variants(void) { return kNumRxVariants; }
const char* nicgpu_tune_variant_name(int v) { return (v >= 0 && v < kNumRxVariants) ? kRxVariants[v].name : ""; }
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
}  // extern "C"
#endif  // NICGPU_TUNING
