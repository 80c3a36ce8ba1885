// f1.hip — row f1: the batched QueuePair RX stage on the device.
// The DMA writes of resolved completions (segment_gather_kernel), the fused
// delivery + RSS of the delivered frames (deliver_kernel), and the per-packet
// decisions of QueuePair::process_once over a whole batch (nicgpu_qp_*;
// src/queue_pair.cpp:67-460 through qp_logic.h).  DESIGN.md §4.6.

#include "common.h"
#include "host.h"
#include "qp_logic.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

using namespace nicgpu_detail;

namespace {

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
  nicgpu_completion* rxc;  // statuses (RSS of Success completions; a deferred verify's failure patched)
  uint64_t j0, n;                // completions [j0, n) ...
  const unsigned long long* n_dev;  // ... with n lowered to *n_dev (a speculative resolve's settled prefix)
  RxParams rss;                  // mode NICGPU_TUPLE_NONE: no RSS
  uint32_t* rx_hash;
  uint16_t* rx_queue;
  unsigned long long* hits;
  unsigned long long* count;
  // the context's accumulator ([0] count, [1 + i] hits of table entry i; zero
  // between launches) and its done ticket: blocks add into it and the last
  // block moves it into count / hits, so neither needs a memset before the
  // launch; null (tuning): blocks add into count / hits directly
  unsigned long long* acc;
  unsigned int* done;
  uint32_t add_count, add_hits;  // the last block adds (1) or stores (0)
  uint64_t alt_dst;  // tuning (kDlvPackedDst): destination = src_a + alt_dst
  // deferred RX verify (nicgpu_qp_set_deferred_verify; the LATE kernels): the
  // batch deferred when *lateflag != late_gen; completion j < late_n with
  // late[j] & kLateDeferred is verified here from the bytes its write
  // delivers; fix: the running corrections (nicgpu_qp_verify_fixups_async)
  const uint8_t* late;
  const unsigned long long* lateflag;
  unsigned long long late_gen;
  uint64_t late_n;
  unsigned long long* fix;  // [segment][NICGPU_QP_FIXUPS]
  const nicgpu_qp_segment* seg;  // a segmented batch's table (its completion's segment), or null
  uint32_t nseg;
  int reserve;  // (host side) CUs left without a delivery block; < 0: NICGPU_DLV_RESERVE_CUS / the build default
};

// Tuning-only modes of deliver_kernel (libnicgpu_tune.so, tools/f1_deliver_bench.py;
// results are wrong with any set): attribute the delivery's time.
constexpr int kDlvNoStore = 1, kDlvNoLoad = 2, kDlvNoHash = 4, kDlvPackedDst = 8, kDlvV1 = 32;
#ifdef NICGPU_TUNING
constexpr int kDlvNoDrain = 16;  // deliver_v1_kernel only
#endif

#ifndef NICGPU_DLV_WPB
#define NICGPU_DLV_WPB 8
#endif
#ifndef NICGPU_DLV_RESERVE
#define NICGPU_DLV_RESERVE 0
#endif
constexpr int kDlvReserveCus = NICGPU_DLV_RESERVE;  // default of NICGPU_DLV_RESERVE_CUS (tuning)
constexpr int kDlvWpb = NICGPU_DLV_WPB;  // waves per block
// round 3's kernel (deliver_v1_kernel, tuning builds only): sub-steps per step, records, per-wave LDS
constexpr int kDlvU1 = 4;
constexpr uint32_t kDlvRec = 24;  // item record: dst u64 | src (or prefix word) u64 | len u32 | first entry u32
constexpr uint32_t kDlvMarks = (uint32_t) kWave * kDlvU1;  // bytes: one u8 mark per stream entry (item id + 1 <= 192)
constexpr uint32_t kDlvWaveBytes = kDlvMarks + 64u * 8u + 192u * kDlvRec + 64u * kHdrStride * 16u;  // marks|wdst|items|stage

// block part: RSS LUT | histogram | table (as rss_only_kernel), then 16 B for the Success count
__host__ __device__ inline uint32_t dlv_block_bytes(bool rss, uint32_t lut_words, uint32_t hist_n,
                                                    uint32_t table_words) {
  return (rss ? rss_only_block_bytes(lut_words, hist_n, table_words) : 0u) + 16u;
}

__device__ __forceinline__ uint32_t dlv_chunks(uint64_t d, uint64_t n) {
  return n ? (uint32_t) (((d + n - 1) >> 4) - (d >> 4) + 1) : 0u;
}

#ifdef NICGPU_TUNING
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

#endif

// The source parts of a delivered frame, as rss_hash_packet reads bytes past
// the LDS header stage: frame byte o is the VLAN prefix word's byte o (o <
// plen), else part A's, else part B's.  Sources are TX buffers, which the
// device path's overlap check keeps apart from every RX buffer of the batch,
// so they hold the frame's bytes while this wave's stores are in flight.
struct FrameParts {
  const uint8_t* mem;
  uint64_t src_a, src_b;
  uint32_t prefix, plen, len_a;
  __device__ __forceinline__ uint32_t operator[](uint32_t o) const {
    if (o < plen) return (prefix >> (8 * o)) & 0xFFu;
    o -= plen;
    return o < len_a ? (uint32_t) mem[src_a + o] : (uint32_t) mem[src_b + (o - len_a)];
  }
};

// Stores bytes [x, y) (0 <= x < y <= 16, not the whole chunk) of the 16-B
// destination chunk at D from o, in at most seven store instructions per
// wave whatever the lanes' ranges (byte, short, three dwords, short, byte at
// per-lane addresses): a partial chunk then costs a wave seven exec-masked
// stores, not the 20 of a per-byte walk (round 3: more than half of the
// delivery's store instructions, SQ_INSTS_VMEM_WR).
__device__ __forceinline__ uint32_t chunk_word_at(const uint32_t* o, uint32_t p) {  // chunk bytes p..p+3 (p < 16)
  const uint32_t i = p >> 2;
  const uint32_t lo = i == 0u ? o[0] : i == 1u ? o[1] : i == 2u ? o[2] : o[3];
  const uint32_t hi = i == 0u ? o[1] : i == 1u ? o[2] : i == 2u ? o[3] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, p & 3u);
}
__device__ __forceinline__ void dlv_store_partial(uint8_t* mem, uint64_t D, uint32_t x, uint32_t y, const uint32_t* o) {
  uint32_t p = x;
  if ((p & 1u) && p < y) {
    mem[D + p] = (uint8_t) chunk_word_at(o, p);
    ++p;
  }
  if ((p & 2u) && p + 2u <= y) {
    *reinterpret_cast<uint16_t*>(mem + D + p) = (uint16_t) chunk_word_at(o, p);
    p += 2u;
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
    if (p + 4u <= y) {
      *reinterpret_cast<uint32_t*>(mem + D + p) = chunk_word_at(o, p);
      p += 4u;
    }
  if (p + 2u <= y) {
    *reinterpret_cast<uint16_t*>(mem + D + p) = (uint16_t) chunk_word_at(o, p);
    p += 2u;
  }
  if (p < y) mem[D + p] = (uint8_t) chunk_word_at(o, p);
}

// ---- the delivery's steps -------------------------------------------------
// Attribution of round 3's kernel (tools/f1_deliver_bench.py, C3 1 M):
// 234 us, of which 87 us with neither loads nor stores (the stream mapping's
// instructions: SQ_INSTS_VALU 60 M), loads alone +22 us, stores alone +80 us,
// and the two never overlapped.  Round 4's counters (profiles/r04b_f1_stall.txt)
// then showed what bounds a lean stream: the texture addresser, 85 % busy at
// 721 K store instructions where a copy of the same bytes needs 364 K — a
// partial chunk (every 1518-B frame ends 14 B into one) cost four exec-masked
// stores, each as dear to the addresser as a whole 16-B one.  So every chunk
// of an item of 16 B or more is ONE 16-B load and ONE 16-B store: the window
// [W, W + 16) with W = the chunk's start clamped into [d, e - 16] — an edge
// chunk's window reaches into its neighbour, whose bytes it rewrites with
// their own values (both lie in the item), so no byte outside the item is
// written and the result is the same in any order.  Edge windows are byte
// aligned: gfx950 global accesses in the HSA unaligned mode (the mode hipcc
// compiles memcpy of byte pointers for; tests/test_gpu_unaligned.py).  Only
// VLAN prefixes and items under 16 B take a slow path, which the wave runs
// only when one of its lanes has one.  Offsets are 32-bit for images below
// 4 GiB (template WIDE otherwise).  Steps are pipelined: step s+1's loads are
// issued before step s's stores.
#ifndef NICGPU_DLV_U
#define NICGPU_DLV_U 2
#endif
#ifndef NICGPU_DLV_BUF
#define NICGPU_DLV_BUF 1
#endif
#ifndef NICGPU_DLV_LCP
#define NICGPU_DLV_LCP 2  // cache policy of the buffer loads (2: nt)
#endif
#ifndef NICGPU_DLV_SCP
#define NICGPU_DLV_SCP 2  // and of the buffer stores (nt: 218 -> 188 us, r04c A/B)
#endif
constexpr int kDlvU = NICGPU_DLV_U;  // 64-entry sub-steps per step
static_assert(kDlvU <= kDlvU1, "marks area");

template <bool WIDE>
struct DlvOff { typedef uint32_t T; };
template <>
struct DlvOff<true> { typedef uint64_t T; };

// An item (a write's VLAN prefix, part A or part B) as the steps read it: the
// window fields in one 16-B (narrow) LDS record, so that a chunk costs a few
// adds — chunk D = (dbase + pos) << 4, window W = min(max(D, lo), hi), source
// W + sdelta — and a meta word beside it.  The item's bytes are [lo, hi + 16).
template <bool WIDE>
struct DlvWin {
  typedef typename DlvOff<WIDE>::T Off;
  Off dbase;   // (d >> 4) - first entry (wrapping)
  Off sdelta;  // src - d (wrapping); the prefix word for a VLAN prefix item
  Off lo, hi;  // d, e - 16 (wrapping)
};
// meta: window item (bit 0: 16 B or more, not a prefix) | item k (1-2) | write q (3-8)
constexpr uint32_t kDlvWinItem = 1u;

// One step held between its loads and its stores.
template <bool WIDE>
struct DlvStep {
  typename DlvOff<WIDE>::T D[kDlvU];  // the window W (window items), else the chunk D
  uint32_t pk[kDlvU];  // item id (0-7) | window (8) | valid (9)
  u32x4 v[kDlvU];      // the source window (window items)
};

// marks | windows | metas (| LATE: the tile's 64 frame sums); the RSS header
// stage takes the windows' place at the tile end, once every lane holds its
// own three (it is no larger)
template <bool WIDE, bool LATE = false>
__host__ __device__ constexpr uint32_t dlv_wave_bytes() {
  static_assert(192u * sizeof(DlvWin<WIDE>) >= 64u * kHdrStride * 16u, "stage fits the windows");
  return kDlvMarks + 192u * (uint32_t) sizeof(DlvWin<WIDE>) + 192u * 4u + (LATE ? 64u * 4u : 0u);
}

// (LATE) The halfword sum, at absolute byte parities, of bytes [x0, x1) of a
// 16-B window at destination address W: bytes kept, each dword rotated by a
// byte when W is odd (so every byte lands in the half its address parity
// gives), halves added — the RX kernel's convention, under which a frame's
// sums compose whatever its alignment.
__device__ __forceinline__ uint32_t dlv_window_sum(u32x4 v, uint32_t x0, uint32_t x1, uint32_t odd) {
  if (x0 != 0u || x1 != 16u) {
    v.x &= dword_keep((int) x0, (int) x1, 0);
    v.y &= dword_keep((int) x0, (int) x1, 1);
    v.z &= dword_keep((int) x0, (int) x1, 2);
    v.w &= dword_keep((int) x0, (int) x1, 3);
  }
  const uint32_t r = odd ? 8u : 0u;
  v.x = __builtin_amdgcn_alignbit(v.x, v.x, r);
  v.y = __builtin_amdgcn_alignbit(v.y, v.y, r);
  v.z = __builtin_amdgcn_alignbit(v.z, v.z, r);
  v.w = __builtin_amdgcn_alignbit(v.w, v.w, r);
  return add_halves(v.w, add_halves(v.z, add_halves(v.y, add_halves(v.x, 0u))));
}

template <bool RSS, int MODE, bool WIDE, bool LATE>
__device__ __forceinline__ void deliver_tiles(const DeliverParams& P) {
  typedef typename DlvOff<WIDE>::T Off;
  typedef DlvWin<WIDE> Win;
  constexpr uint32_t kThreads = kWave * kDlvWpb;
  constexpr uint32_t kSpan = kWave * kDlvU;
  constexpr bool kHash = RSS && (MODE & kDlvNoHash) == 0;
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
  uint8_t* wave_b = base_b + block_bytes + w * dlv_wave_bytes<WIDE, LATE>();
  uint8_t* marks = wave_b;
  Win* wins = reinterpret_cast<Win*>(wave_b + kDlvMarks);
  uint32_t* metas = reinterpret_cast<uint32_t*>(wins + 192);
  uint32_t* sumc = metas + 192;  // (LATE) per frame of the tile: its running sum
  uint4* stage = reinterpret_cast<uint4*>(wins);  // at the tile end
  if (RSS) {
    for (uint32_t i = threadIdx.x; i < R.lut_words; i += kThreads) lut[i] = R.lut[i];
    if (hist_lds)
      for (uint32_t i = threadIdx.x; i < R.table_n; i += kThreads) hist[i] = 0;
    if (table_lds)
      for (uint32_t i = threadIdx.x; i < R.table_n; i += kThreads) table_s[i] = R.table[i];
    if (threadIdx.x == 0) *cnt_s = 0;
  }
  __syncthreads();
  uint64_t n = P.n;
  if (P.n_dev) {
    const uint64_t m = *P.n_dev;
    n = m < n ? m : n;
  }
  const uint64_t ntiles = n > P.j0 ? (n - P.j0 + kWave - 1) / kWave : 0;
  const uint64_t nwaves = (uint64_t) gridDim.x * kDlvWpb;
  const uint64_t msize = P.mem_size;
  // where lanes without a window load from: the image start, or the write
  // records for an image below 16 B (always >= 40 readable bytes)
  const uint8_t* dummy = msize >= 16u ? P.mem : reinterpret_cast<const uint8_t*>(P.w);
  // images below 4 GiB: the hot path's loads and stores are buffer accesses
  // (scalar base, 32-bit offsets) — with 64-bit per-lane addresses the
  // texture addresser took ~5x the cycles per instruction of a buffer copy
  // and bounded the kernel (profiles/r04b_f1_stall.txt); lanes without a
  // window use offset msize, out of range: no memory access, loads read 0,
  // stores are dropped
  constexpr bool kBuf = !WIDE && NICGPU_DLV_BUF != 0;
  const __amdgpu_buffer_rsrc_t mrs =
      __builtin_amdgcn_make_buffer_rsrc(P.mem, (short) 0, (int) (uint32_t) (WIDE ? 0u : msize), 0x00020000);
  uint32_t my_count = 0;
  // the batch deferred its RX verifies (wave-uniform)
  const bool lateb = LATE && *P.lateflag != P.late_gen;
  for (uint64_t tile = (uint64_t) blockIdx.x * kDlvWpb + w; tile < ntiles; tile += nwaves) {
    // ---- this lane's write: its items and their stream entries
    const uint64_t j = P.j0 + tile * kWave + lane;
    uint32_t F, c0, c1, c2, total_e;
    bool flag;
    {
      nicgpu_segment_write wr{};
      flag = false;
      if (j < n) {
        wr = P.w[j];
        if (RSS) flag = P.rxc[j].status == nicqp::kSuccess;
        if constexpr ((MODE & kDlvPackedDst) != 0) wr.dst = wr.src_a + P.alt_dst;
      }
      const uint64_t plen = wr.prefix_len == 4 ? 4 : 0;
      const uint64_t total = plen + wr.len_a + wr.len_b;
      // entries outside the image are skipped (the host validated them)
      const bool ok = j < n && !(wr.prefix_len > 4 || wr.dst > msize || total > msize - wr.dst ||
                                   wr.src_a > msize || wr.len_a > msize - wr.src_a ||
                                   wr.src_b > msize || wr.len_b > msize - wr.src_b);
      flag = flag && ok;
      const uint64_t d1 = wr.dst + plen, d2 = d1 + wr.len_a;
      c0 = ok ? dlv_chunks(wr.dst, plen) : 0u;
      c1 = ok ? dlv_chunks(d1, wr.len_a) : 0u;
      c2 = ok ? dlv_chunks(d2, wr.len_b) : 0u;
      const uint32_t cw = c0 + c1 + c2;
      const uint32_t incl = wave_incl_scan(cw);
      F = incl - cw;
      total_e = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
      // (lengths kept for the hash even for items without chunks: ok frames only)
      auto put = [&](uint32_t k, uint64_t d, uint64_t src_or_word, uint64_t len, uint32_t first)
                     __attribute__((always_inline)) {
        if (!ok) len = 0;
        Win it;
        it.dbase = (Off) ((d >> 4) - first);
        it.sdelta = k == 0u ? (Off) src_or_word : (Off) (src_or_word - d);
        it.lo = (Off) d;
        it.hi = (Off) (d + len - 16u);
        wins[lane * 3u + k] = it;
        metas[lane * 3u + k] = (k != 0u && len >= 16u ? kDlvWinItem : 0u) | (k << 1) | (lane << 3);
      };
      put(0, wr.dst, wr.prefix, plen, F);
      put(1, d1, wr.src_a, wr.len_a, F + c0);
      put(2, d2, wr.src_b, wr.len_b, F + c0 + c1);
      if (LATE && lateb) sumc[lane] = 0u;
    }
    uint32_t carry = 0;  // item (id + 1) of the entry before the step being planned
    // ---- load phase of the step at stream position W
    auto plan = [&](DlvStep<WIDE>& S, uint32_t W) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) marks[u * kWave + lane] = 0u;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (c0 && F >= W && F - W < kSpan) marks[F - W] = (uint8_t) (lane * 3u + 1u);
      if (c1 && F + c0 >= W && F + c0 - W < kSpan) marks[F + c0 - W] = (uint8_t) (lane * 3u + 2u);
      if (c2 && F + c0 + c1 >= W && F + c0 + c1 - W < kSpan) marks[F + c0 + c1 - W] = (uint8_t) (lane * 3u + 3u);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) {
        uint32_t it = wave_incl_max(marks[u * kWave + lane]);
        it = it > carry ? it : carry;
        carry = (uint32_t) __builtin_amdgcn_readlane((int) it, 63);
        const uint32_t pos = W + (uint32_t) u * kWave + lane;
        const bool valid = pos < total_e;
        const uint32_t id = valid ? it - 1u : 0u;
        const Win I = wins[id];
        const bool win = valid && (metas[id] & kDlvWinItem);
        const Off D = (I.dbase + (Off) pos) << 4;
        const Off Wn = D < I.lo ? I.lo : (D > I.hi ? I.hi : D);
        S.D[u] = win ? Wn : D;
        S.pk[u] = id | ((uint32_t) win << 8) | ((uint32_t) valid << 9);
        if constexpr (LATE) {  // the chunk's own bytes within the window: [x0, x1)
          const Off e = I.hi + (Off) 16u;
          const Off a = D < I.lo ? I.lo : D;
          const Off b = D + (Off) 16u > e ? e : D + (Off) 16u;
          S.pk[u] |= ((uint32_t) (a - Wn) << 10) | ((uint32_t) (b - Wn) << 15);
        }
        if constexpr ((MODE & kDlvNoLoad) != 0) {
          S.v[u] = (u32x4){(uint32_t) D, 1u, 2u, 3u};
        } else if constexpr (kBuf) {
          const uint32_t off = win ? (uint32_t) (Wn + I.sdelta) : (uint32_t) msize;
          S.v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(mrs, (int) off, 0, NICGPU_DLV_LCP));
        } else {
          const uint8_t* src = win ? P.mem + (Off) (Wn + I.sdelta) : dummy;
          u32x4 v;
          __builtin_memcpy(&v, src, 16);  // byte-aligned dwordx4 for edge windows
          S.v[u] = v;
        }
      }
    };
    // ---- store phase
    auto store = [&](const DlvStep<WIDE>& S) __attribute__((always_inline)) {
      bool slow = false;
      uint32_t su[kDlvU];  // (LATE) each entry's sum
#pragma unroll
      for (int u = 0; u < kDlvU; ++u) {
        const uint32_t pk = S.pk[u];
        if constexpr (LATE) {
          su[u] = 0u;
          if (lateb && (pk & 256u))
            su[u] = dlv_window_sum(S.v[u], (pk >> 10) & 31u, (pk >> 15) & 31u, (uint32_t) S.D[u] & 1u);
        }
        if constexpr ((MODE & kDlvNoStore) != 0) {
          if ((pk & 256u) && (S.v[u].x ^ S.v[u].w) == 0x12345678u) P.mem[S.D[u]] = 0;  // keeps the loads
        } else if constexpr (kBuf) {
          const uint32_t off = (pk & 256u) ? (uint32_t) S.D[u] : (uint32_t) msize;
          __builtin_amdgcn_raw_buffer_store_b128(S.v[u], mrs, (int) off, 0, NICGPU_DLV_SCP);
        } else if (pk & 256u) {
          __builtin_memcpy(P.mem + S.D[u], &S.v[u], 16);
        }
        slow = slow || (pk & 768u) == 512u;
      }
      if (slow) {
        // VLAN prefixes and items under 16 B: bytes [x, y) of chunk D, read
        // here byte by byte (waited for in this branch only)
#pragma unroll
        for (int u = 0; u < kDlvU; ++u) {
          const uint32_t pk = S.pk[u];
          if ((pk & 768u) != 512u) continue;
          const Off D = S.D[u];
          const Win I = wins[pk & 255u];
          const uint32_t k = (metas[pk & 255u] >> 1) & 3u;
          const Off dend = I.hi + (Off) 16u;
          const uint32_t x = I.lo > D ? (uint32_t) (I.lo - D) : 0u;
          const uint32_t y = dend - D < 16u ? (uint32_t) (dend - D) : 16u;
          uint32_t o[4] = {0u, 0u, 0u, 0u};
          if (k == 0u) {
            // VLAN prefix 81 00 tag (queue_pair.cpp:352-359): its 4 bytes at d
            const uint32_t pw = (uint32_t) I.sdelta;
            const int32_t rel = (int32_t) (I.lo - D);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              uint32_t z = 0;
#pragma unroll
              for (int bb = 0; bb < 4; ++bb) {
                const int32_t pb = 4 * i + bb - rel;
                if (pb >= 0 && pb < 4) z |= ((pw >> (8 * pb)) & 0xFFu) << (8 * bb);
              }
              o[i] = z;
            }
          } else {
            const Off s0 = D + I.sdelta;
#pragma unroll 1
            for (uint32_t b = x; b < y; ++b) {
              const uint32_t z = (uint32_t) P.mem[(Off) (s0 + b)] << (8u * (b & 3u));
              o[0] |= (b >> 2) == 0u ? z : 0u;
              o[1] |= (b >> 2) == 1u ? z : 0u;
              o[2] |= (b >> 2) == 2u ? z : 0u;
              o[3] |= (b >> 2) == 3u ? z : 0u;
            }
          }
          if constexpr (LATE) su[u] = add_halves(o[3], add_halves(o[2], add_halves(o[1], add_halves(o[0], 0u))));
          if constexpr ((MODE & kDlvNoStore) == 0) dlv_store_partial(P.mem, (uint64_t) D, x, y, o);
        }
      }
      if constexpr (LATE) {
        if (lateb) {
          // each frame's entries are consecutive in the stream: a scan of the
          // step's sums, the frame's last entry in the step adding its prefix
          // and its first one taking away the prefix before it (one LDS add
          // per frame and step)
#pragma unroll
          for (int u = 0; u < kDlvU; ++u) {
            const uint32_t pk = S.pk[u];
            const bool valid = (pk & 512u) != 0u;
            const uint32_t q = valid ? (pk & 255u) / 3u : 0xFFu;
            const uint32_t incl = wave_incl_scan(su[u]);
            const uint32_t qp = (uint32_t) __builtin_amdgcn_update_dpp(0, (int) q, 0x138, 0xf, 0xf, false);  // wave_shr:1
            const uint32_t qn = (uint32_t) __builtin_amdgcn_update_dpp(0, (int) q, 0x130, 0xf, 0xf, false);  // wave_shl:1
            const bool first = lane == 0u || qp != q, last = lane == 63u || qn != q;
            if (valid && (first || last)) atomicAdd(&sumc[q], (last ? incl : 0u) - (first ? incl - su[u] : 0u));
          }
        }
      }
    };
    // ---- the stream: three step buffers in rotation, so a buffer is loaded
    // again only after another step's stores have issued (a buffer reloaded
    // right after its stores makes hipcc wait for them: gfx950 counts stores
    // in vmcnt, in order with the loads); a counted loop with its only exit at
    // the bottom keeps counted waits; plans past the last step are empty
    const uint32_t nsteps = (total_e + kSpan - 1) / kSpan;
    if (nsteps) {
      DlvStep<WIDE> A, B, C;
      plan(A, 0);
      plan(B, kSpan);
      uint32_t s = 0;
      for (; s + 3 <= nsteps; s += 3) {
        plan(C, (s + 2) * kSpan);
        __builtin_amdgcn_sched_barrier(0);
        store(A);
        plan(A, (s + 3) * kSpan);
        __builtin_amdgcn_sched_barrier(0);
        store(B);
        plan(B, (s + 4) * kSpan);
        __builtin_amdgcn_sched_barrier(0);
        store(C);
      }
      if (s < nsteps) store(A);
      if (s + 1 < nsteps) store(B);
    }
    if (LATE && lateb) {
      // the deferred verifies (queue_pair.cpp:434-447) of the tile's frames
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint32_t sum = sumc[lane];
      if (j < n && j < P.late_n) {
        const uint32_t lb = P.late[j];
        if (lb & nicqp::kLateDeferred) {
          nicgpu_completion e = P.rxc[j];
          if (e.status == nicqp::kSuccess && fold16(sum) != 0xFFFFu) {
            // the reference's ChecksumError completion (no VLAN strip) and
            // what the resolve counted for it as delivered
            const Win I0 = wins[lane * 3u], I1 = wins[lane * 3u + 1u], I2 = wins[lane * 3u + 2u];
            const uint64_t len_a = (uint32_t) (I1.hi + 16u - I1.lo), len_b = (uint32_t) (I2.hi + 16u - I2.lo);
            const uint64_t size = (uint64_t) (uint32_t) (I0.hi + 16u - I0.lo) + len_a + len_b;
            uint32_t sg = 0;  // the completion's segment: the last whose ring starts at or before j
            if (P.seg) {
              uint32_t hi = P.nseg;
              while (hi - sg > 1u) {
                const uint32_t mid = (sg + hi) / 2u;
                if (P.seg[mid].rx_begin <= j) sg = mid;
                else hi = mid;
              }
            }
            unsigned long long* fx = P.fix + (uint64_t) sg * NICGPU_QP_FIXUPS;
            atomicAdd(&fx[0], 1ull);
            atomicAdd(&fx[1], (unsigned long long) size);
            if (e.vlan_stripped) atomicAdd(&fx[2], 1ull);
            atomicAdd(&fx[3], (unsigned long long) (len_a + len_b + ((lb & nicqp::kLateStripBase) ? 4u : 0u)));
            if (lb & nicqp::kLateVlanInsert) atomicAdd(&fx[4], 1ull);
            e.status = nicqp::kChecksumError;
            e.vlan_stripped = false;
            e.vlan_tag = 0;
            P.rxc[j] = e;
            flag = false;
          }
        }
      }
    }
    if (kHash) {
      // every lane reads its items before the stage overwrites them
      const Win I0 = wins[lane * 3u], I1 = wins[lane * 3u + 1u], I2 = wins[lane * 3u + 2u];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (j < n) {
        if (flag) {
          const uint32_t plen = (uint32_t) (I0.hi + 16u - I0.lo);
          const uint32_t len_a = (uint32_t) (I1.hi + 16u - I1.lo), len_b = (uint32_t) (I2.hi + 16u - I2.lo);
          uint64_t len = (uint64_t) plen + len_a + len_b;
          if (len > NICGPU_MAX_PACKET) len = NICGPU_MAX_PACKET;  // the tuple lies in the first 82 B
          const uint64_t src_a = (uint64_t) (Off) (I1.lo + I1.sdelta);
          const FrameParts fp{P.mem, src_a, (uint64_t) (Off) (I2.lo + I2.sdelta), (uint32_t) I0.sdelta, plen, len_a};
          // a frame whose first 48 bytes are all part A's (no VLAN prefix)
          // stages them from its source, three 16-B loads; the others byte by byte
          const bool hdr_src = plen == 0u && (len_a >= (uint32_t) kHdrBytes || len_b == 0u);
          const uint32_t hlo = (uint32_t) ((hdr_src ? src_a : (uint64_t) I0.lo) & 15u);
          if (hdr_src) {
            const uint64_t hb = src_a & ~15ull;
            const uint64_t hend = src_a + (len_a < (uint32_t) kHdrBytes ? len_a : (uint32_t) kHdrBytes);
#pragma unroll
            for (int k = 0; k < kHdrChunks; ++k)
              if (hb + 16u * k < hend) stage[hdr_slot(lane, (uint32_t) k)] = *reinterpret_cast<const uint4*>(P.mem + hb + 16u * k);
          } else {
            uint8_t* sb = reinterpret_cast<uint8_t*>(stage + hdr_slot(lane, 0));
            const uint32_t nb = len < (uint64_t) kHdrBytes - hlo ? (uint32_t) len : (uint32_t) kHdrBytes - hlo;
            for (uint32_t o = 0; o < nb; ++o) sb[hdr_slot(0, (hlo + o) >> 4) * 16u + ((hlo + o) & 15u)] = (uint8_t) fp[o];
          }
          const uint32_t h = rss_hash_packet(R, lut, HdrView{stage, lane}, hlo, fp, (uint32_t) len);
          const uint32_t idx = h % R.table_n;
          P.rx_hash[j] = h;
          P.rx_queue[j] = table_lds ? table_s[idx] : R.table[idx];
          if (hist_lds) atomicAdd(&hist[idx], 1u);
          else atomicAdd(P.acc ? &P.acc[1 + idx] : &P.hits[idx], 1ull);
          ++my_count;
        } else {
          P.rx_hash[j] = 0u;
          P.rx_queue[j] = 0xFFFFu;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
  if (RSS) {
    const uint32_t c = (uint32_t) __builtin_amdgcn_readlane((int) wave_incl_scan(my_count), 63);
    if (lane == 0 && c) atomicAdd(cnt_s, c);
    __syncthreads();
    if (P.acc == nullptr) {
      if (threadIdx.x == 0 && *cnt_s) atomicAdd(P.count, (unsigned long long) *cnt_s);
      if (hist_lds) flush_hist(hist, R.table_n, P.hits, R.hits_rep, R.hits_done, kThreads);
      return;
    }
    if (threadIdx.x == 0 && *cnt_s) atomicAdd(&P.acc[0], (unsigned long long) *cnt_s);
    if (hist_lds)
      for (uint32_t i = threadIdx.x; i < R.table_n; i += kThreads)
        if (hist[i]) atomicAdd(&P.acc[1 + i], (unsigned long long) hist[i]);
    // the last block to finish (flush_hist's ticket hand-off) moves the
    // accumulator out and leaves it zero for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's adds are performed
    __syncthreads();
    if (threadIdx.x == 0) *cnt_s = atomicAdd(P.done, 1u) == gridDim.x - 1u ? 1u : 0u;
    __syncthreads();
    if (*cnt_s == 0u) return;
    for (uint32_t i = threadIdx.x; i <= R.table_n; i += kThreads) {
      const unsigned long long v = atomicExch(&P.acc[i], 0ull);
      unsigned long long* dst = i == 0u ? P.count : &P.hits[i - 1u];
      if (i == 0u ? P.add_count : P.add_hits) {
        if (v) atomicAdd(dst, v);
      } else {
        *dst = v;
      }
    }
    if (threadIdx.x == 0) atomicExch(P.done, 0u);
  }
}

#ifndef NICGPU_DLV_OCC
#define NICGPU_DLV_OCC 4
#endif
// waves per SIMD the delivery is compiled for (tuning: 6, 80 VGPRs, which
// its LDS allows, spills the RSS variant and measured slower)
template <bool RSS, int MODE = 0, bool WIDE = false, bool LATE = false>
__global__ __launch_bounds__(kWave * kDlvWpb) __attribute__((amdgpu_waves_per_eu(NICGPU_DLV_OCC, 8))) void deliver_kernel(DeliverParams P) {
  deliver_tiles<RSS, MODE, WIDE, LATE>(P);
}

#ifdef NICGPU_TUNING
// round 3's delivery (each step's loads after the previous step's stores,
// a vmcnt(0) drain before the hash), for the A/B of tools/f1_deliver_bench.py
template <bool RSS, int MODE = 0>
__global__ __launch_bounds__(kWave * kDlvWpb) __attribute__((amdgpu_waves_per_eu(4, 8))) void deliver_v1_kernel(DeliverParams P) {
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
      if constexpr ((MODE & kDlvPackedDst) != 0) wr.dst = wr.src_a + P.alt_dst;
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
    // ---- the stream: kDlvU1 x 64 entries per step, every load of the step
    // issued before its first store (one memory latency per step)
    uint32_t carry = 0;  // item (id + 1) of the entry before this step
    for (uint32_t W = 0; W < total_e; W += kWave * kDlvU1) {
#pragma unroll
      for (int u = 0; u < kDlvU1; ++u) marks[u * kWave + lane] = 0u;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      constexpr uint32_t kSpan = kWave * kDlvU1;
      if (c0 && F >= W && F - W < kSpan) marks[F - W] = (uint8_t) (lane * 3u + 1u);
      if (c1 && F + c0 >= W && F + c0 - W < kSpan) marks[F + c0 - W] = (uint8_t) (lane * 3u + 2u);
      if (c2 && F + c0 + c1 >= W && F + c0 + c1 - W < kSpan) marks[F + c0 + c1 - W] = (uint8_t) (lane * 3u + 3u);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      uint32_t itv[kDlvU1];
#pragma unroll
      for (int u = 0; u < kDlvU1; ++u) {
        uint32_t it = wave_incl_max(marks[u * kWave + lane]);
        it = it > carry ? it : carry;
        carry = (uint32_t) __builtin_amdgcn_readlane((int) it, 63);
        itv[u] = it;
      }
      // phase A: every entry's chunk, item and source window; loads issued.
      // Per entry: the destination chunk, one packed word (bytes [lo, hi) of
      // the chunk, source shift, owning write) and five source dwords — a
      // prefix item's 4 bytes are placed into them here — so that kDlvU1
      // entries' loads fit in flight per lane.
      uint64_t Dc[kDlvU1];  // destination chunk index; ~0: no entry
      uint32_t pk[kDlvU1];  // lo - D (bits 0-4) | hi - D (8-12) | shift (16-17) | write q (20-25)
      uint32_t vv[kDlvU1][5];
#pragma unroll
      for (int u = 0; u < kDlvU1; ++u) {
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
            if constexpr ((MODE & kDlvNoLoad) != 0) {
#pragma unroll
              for (int i = 0; i < 5; ++i) vv[u][i] = (uint32_t) a4 * 0x9E3779B1u + i;
            } else if (a4 >= 0 && (uint64_t) a4 + 20 <= P.mem_size) {
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
      for (int u = 0; u < kDlvU1; ++u) {
        if (Dc[u] == ~0ull) continue;
        const uint64_t D = Dc[u] << 4, lo = D + (pk[u] & 31u), hi = D + ((pk[u] >> 8) & 31u);
        const uint32_t sh = (pk[u] >> 16) & 3u;
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = sh ? __builtin_amdgcn_alignbyte(vv[u][i + 1], vv[u][i], sh) : vv[u][i];
        if constexpr ((MODE & kDlvNoStore) != 0) {
          if ((o[0] ^ o[1] ^ o[2] ^ o[3]) == 0x12345678u && lo == D + 3) P.mem[D] = 0;  // keeps the loads
        } else {
          dlv_store(P.mem, D, lo, hi, o);
        }
        if (RSS && (MODE & kDlvNoHash) == 0) {
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
    if (RSS && (MODE & kDlvNoHash) == 0) {
      // the frames' bytes are in the stage; bytes past it come from the frame
      // this wave just wrote (its stores retired first)
      if constexpr ((MODE & kDlvNoDrain) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
#endif  // NICGPU_TUNING

template <bool RSS, bool LATE = false>
int dlv_blocks_per_cu(uint32_t lds) {
  return blocks_per_cu(reinterpret_cast<const void*>(deliver_kernel<RSS, 0, false, LATE>), kWave * kDlvWpb, lds);
}

template <int MODE>
int launch_deliver(const DeliverParams& P, bool rss, int cus_total, hipStream_t s) {
  const uint32_t hist_n = (rss && P.rss.table_n <= (uint32_t) kHistLds) ? P.rss.table_n : 0u;
  const uint32_t table_words = (rss && P.rss.table_n <= (uint32_t) kTableLds) ? (P.rss.table_n + 1u) / 2u : 0u;
  const bool wide = P.mem_size > 0xFFFFFFF0ull;  // 32-bit offsets for images below 4 GiB
  const bool late = MODE == 0 && P.late != nullptr;
  const uint32_t wave_bytes = (MODE & kDlvV1) ? kDlvWaveBytes
                              : late ? (wide ? dlv_wave_bytes<true, true>() : dlv_wave_bytes<false, true>())
                                     : (wide ? dlv_wave_bytes<true>() : dlv_wave_bytes<false>());
  const uint32_t lds = dlv_block_bytes(rss, P.rss.lut_words, hist_n, table_words) + kDlvWpb * wave_bytes;
  const int bpc = late ? (rss ? dlv_blocks_per_cu<true, true>(lds) : dlv_blocks_per_cu<false, true>(lds))
                       : (rss ? dlv_blocks_per_cu<true>(lds) : dlv_blocks_per_cu<false>(lds));
  const uint64_t ntiles = (P.n - P.j0 + kWave - 1) / kWave;
  const uint64_t want = (ntiles + kDlvWpb - 1) / kDlvWpb;
  // CUs left without a delivery block, so the next batch's plan and check
  // (small launches on a side stream) find wave slots while this one runs
  static const int reserve_default = [] {
    const char* e = std::getenv("NICGPU_DLV_RESERVE_CUS");
    return e ? std::atoi(e) : kDlvReserveCus;
  }();
  const int reserve = P.reserve >= 0 ? P.reserve : reserve_default;
  const uint64_t cus = (uint64_t) (cus_total > reserve + 8 ? cus_total - reserve : cus_total);
  const uint64_t cap = cus * (uint64_t) bpc;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
#ifdef NICGPU_TUNING
  if constexpr ((MODE & kDlvV1) != 0) {
    if (rss) hipLaunchKernelGGL((deliver_v1_kernel<true, MODE & ~kDlvV1>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
    else hipLaunchKernelGGL((deliver_v1_kernel<false, MODE & ~kDlvV1>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
    return hip_status(hipGetLastError());
  }
#endif
  if constexpr (MODE == 0) {
    if (late) {
      if (rss && !wide) hipLaunchKernelGGL((deliver_kernel<true, 0, false, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
      else if (rss) hipLaunchKernelGGL((deliver_kernel<true, 0, true, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
      else if (!wide) hipLaunchKernelGGL((deliver_kernel<false, 0, false, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
      else hipLaunchKernelGGL((deliver_kernel<false, 0, true, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
      return hip_status(hipGetLastError());
    }
  }
  if (rss && !wide) hipLaunchKernelGGL((deliver_kernel<true, MODE, false>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  else if (rss) hipLaunchKernelGGL((deliver_kernel<true, MODE, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  else if (!wide) hipLaunchKernelGGL((deliver_kernel<false, MODE, false>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  else hipLaunchKernelGGL((deliver_kernel<false, MODE, true>), dim3(grid), dim3(kWave * kDlvWpb), lds, s, P);
  return hip_status(hipGetLastError());
}

}  // namespace

extern "C" {

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
constexpr unsigned kQpTail = 3 + 16 + 3;  // ... then [19] the plan overflowed (1 buffers, 2 pieces per descriptor), [20] its piece count, [21] RX verify deferred
constexpr int kQpRelaxSteps = 8;  // position relaxations before the host takes the rest
constexpr unsigned kQpBoundsAt = 8;  // misc()[12..15]: the check's bounds' presets

// Segmented batches (several queue pairs, nicgpu_qp_set_segments): each grid
// block serves one segment — blocks in proportion to its TX descriptors — so a
// block's per-block statistics belong to one queue pair, and a packet's queue
// id, MTU and ring come from its block's segment.  seg == null: one queue pair
// (the context's), every block over all of [0, n).
struct QpBlk {
  uint32_t seg, rank, nb, pad;  // the block's segment, its rank among that segment's blocks, their number
};
struct QpSegs {
  const nicgpu_qp_segment* seg;
  const QpBlk* blk;
  uint32_t nseg;
};
struct QpRange {
  uint64_t i, end, step;
  uint32_t s;
};
__device__ __forceinline__ uint64_t qp_seg_end(const QpSegs& S, uint32_t s, uint64_t n) {
  return s + 1 < S.nseg ? S.seg[s + 1].tx_begin : n;
}
// the TX indices this thread visits
__device__ __forceinline__ QpRange qp_range(const QpSegs& S, uint64_t n) {
  if (!S.seg) return QpRange{(uint64_t) blockIdx.x * kQpBlock + threadIdx.x, n, (uint64_t) gridDim.x * kQpBlock, 0u};
  const QpBlk b = S.blk[blockIdx.x];
  const uint64_t hi = qp_seg_end(S, b.seg, n);
  return QpRange{S.seg[b.seg].tx_begin + (uint64_t) b.rank * kQpBlock + threadIdx.x, hi < n ? hi : n,
                 (uint64_t) b.nb * kQpBlock, b.seg};
}
// segment s's context: its queue id and MTU, its ring's end in the
// concatenated ring (positions are absolute)
__device__ __forceinline__ QpCtx qp_ctx_of(QpCtx C, const QpSegs& S, uint32_t s) {
  if (S.seg) {
    const nicgpu_qp_segment g = S.seg[s];
    C.queue_id = g.queue_id;
    C.max_mtu = g.max_mtu;
    C.nrx = g.rx_begin + g.nrx;
  }
  return C;
}
// the absolute ring position of packet i of segment s: the scan restarted at
// the segment's first packet, from its ring's first slot
__device__ __forceinline__ uint64_t qp_abs(const uint32_t* __restrict__ pos, const QpSegs& S, uint32_t s, uint64_t i) {
  if (!S.seg) return pos[i];
  const nicgpu_qp_segment g = S.seg[s];
  return g.rx_begin + (uint64_t) (uint32_t) (pos[i] - pos[g.tx_begin]);
}
__device__ __forceinline__ uint64_t qp_max_mtu(uint64_t max_mtu, const QpSegs& S, uint32_t s) {
  return S.seg ? S.seg[s].max_mtu : max_mtu;
}

struct QpNullSink {
  __device__ void tx(const nicgpu_completion&, bool) {}
  __device__ void rx(const nicgpu_completion&, const nicgpu_segment_write*) {}
};

struct QpDevSink {
  nicgpu_completion* txc;
  nicgpu_completion* rxc;
  nicgpu_segment_write* w;
  uint64_t ti, rj;
  uint8_t* late;  // a deferred-verify batch: every completion's bits (0: final)
  uint64_t keep;  // completions [0, keep) are already delivered: not rewritten (a deferred verify may have patched them)
  __device__ void tx(const nicgpu_completion& e, bool) { txc[ti] = e; }
  __device__ void rx(const nicgpu_completion& e, const nicgpu_segment_write* sw) { rx_late(e, sw, 0u); }
  __device__ void rx_late(const nicgpu_completion& e, const nicgpu_segment_write* sw, uint32_t bits) {
    if (rj < keep) {
      ++rj;
      return;
    }
    rxc[rj] = e;
    if (sw) {
      w[rj] = *sw;
    } else {
      nicgpu_segment_write z{};
      w[rj] = z;
    }
    if (late) late[rj] = (uint8_t) bits;
    ++rj;
  }
};

// A descriptor that plans more than kQpMaxPieces pieces counts 0 and sets
// *ovf to this call's generation (flags compared with the generation need no
// reset before the launch), so the 32-bit scan of the counts (n <= 2^32 /
// kQpMaxPieces) cannot wrap and the caller sees the flag.
constexpr uint32_t kQpMaxPieces = 256;
// Also whether the batch may defer its RX verifies (defer): g[7]
// becomes the generation when it may not — a packet with a TX verify or more
// than one segment, whose pops a sum can change (qp_logic.h Ctx::late).
__global__ __launch_bounds__(kQpBlock) void qp_count_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t n,
                                                            uint64_t mem_size, uint64_t max_mtu, QpPlan* plans,
                                                            uint32_t* counts, unsigned long long* g,
                                                            unsigned long long gen, QpSegs S, uint32_t defer,
                                                            uint32_t* need, unsigned long long* fix, uint32_t nfix) {
  // this batch's deferred-verify corrections start at 0 (its deliveries follow)
  for (uint32_t k = blockIdx.x * kQpBlock + threadIdx.x; k < nfix; k += gridDim.x * kQpBlock) fix[k] = 0ull;
  const QpRange R = qp_range(S, n);
  const uint64_t mtu = qp_max_mtu(max_mtu, S, R.s);
  const bool may = defer != 0u;
  bool needs = false;
  for (uint64_t i = R.i; i < R.end; i += R.step) {
    QpPlan pp;
    const nicgpu_tx_descriptor t = nicqp::desc_load(tx + i);
    const uint32_t c = nicqp::plan_packet(mtu, mem_size, t, pp, [](uint64_t, uint64_t) {}, /*split4=*/true);
    counts[i] = c <= kQpMaxPieces ? c : 0u;
    if (c > kQpMaxPieces) g[0] = gen;
    plans[i] = pp;
    if (may) {
      needs = needs || nicqp::tx_verify_needed(t) || nicqp::decide_segments(t).nseg > 1u;
      // a deferring batch's need, final: no packet of it has a TX verify
      // (qp_need_kernel then writes only the seed; any other batch's need it
      // recomputes)
      need[i] = nicqp::rx_need_unverified(t, mem_size, mtu);
    }
  }
  if (!may) {
    if (blockIdx.x == 0 && threadIdx.x == 0) g[7] = gen;
  } else if (__ballot(needs) != 0ull && lane_id() == 0u) {
    g[7] = gen;
  }
}

// the batch defers its RX verifies (after its count kernel)
__device__ __forceinline__ bool qp_late(const unsigned long long* g, unsigned long long gen) { return g[7] != gen; }

// Piece descriptors below `cap` only; the first thread leaves the piece count
// in g[5], min(count, cap) in g[6], the count the sums run over in g[4] (that,
// or 0 when the batch defers its RX verifies), and the generation in g[3]
// when the plan does not fit (nicgpu_qp_plan_async).
__global__ __launch_bounds__(kQpBlock) void qp_fill_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t n,
                                                           uint64_t mem_size, uint64_t max_mtu, QpPlan* plans,
                                                           const uint32_t* __restrict__ base, uint64_t* desc,
                                                           uint64_t cap, unsigned long long* g, unsigned long long gen,
                                                           QpSegs S) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t np = base[n];
    g[5] = np;
    g[6] = np < cap ? np : cap;
    g[4] = qp_late(g, gen) ? 0u : g[6];  // a deferred-verify batch reads no piece sum
    if (np > cap) g[3] = gen;
  }
  const QpRange R = qp_range(S, n);
  const uint64_t mtu = qp_max_mtu(max_mtu, S, R.s);
  for (uint64_t i = R.i; i < R.end; i += R.step) {
    uint64_t at = base[i];
    plans[i].first_piece = (uint32_t) at;
    QpPlan pp;
    nicqp::plan_packet(
        mtu, mem_size, nicqp::desc_load(tx + i), pp,
        [&](uint64_t a, uint64_t len) {
          if (at < cap) desc[at] = NICGPU_DESC(a, len);
          ++at;
        },
        /*split4=*/true);
  }
}

// The plan this resolve reads did not fit its buffers (or a descriptor planned
// more than 256 pieces): no kernel of the resolve reads a piece sum then.
__device__ __forceinline__ bool qp_plan_bad(const unsigned long long* g, unsigned long long gen) {
  return g[0] == gen || g[3] == gen;
}

// fresh (the position walk): need recomputed for every batch — after the
// relaxation a deferring batch's need[] holds the last step's pops, not the
// count kernel's needs (rx_need of a deferring batch is rx_need_unverified:
// none of its packets has a TX verify).
__global__ __launch_bounds__(kQpBlock) void qp_need_kernel(QpCtx C, uint64_t n, uint32_t* need,
                                                           unsigned long long* first, const unsigned long long* g,
                                                           unsigned long long gen, QpSegs S, uint32_t fresh) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *first = n;  // the speculative final pass's "nothing differed"
  const bool bad = qp_plan_bad(g, gen);
  if (!bad && !fresh && qp_late(g, gen)) {  // the count kernel wrote every need: only the scan's end
    if (blockIdx.x == 0 && threadIdx.x == 0) need[n] = 0u;
    return;
  }
  if (S.seg) {
    if (blockIdx.x == 0 && threadIdx.x == 0) need[n] = 0u;
    const QpRange R = qp_range(S, n);
    const QpCtx Cs = qp_ctx_of(C, S, R.s);
    for (uint64_t i = R.i; i < R.end; i += R.step) need[i] = !bad ? nicqp::rx_need(Cs, i) : 0u;
    return;
  }
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i <= n; i += (uint64_t) gridDim.x * kQpBlock)
    need[i] = i < n && !bad ? nicqp::rx_need(C, i) : 0u;
}

// One relaxation step of the ring positions: every packet resolved (without
// outputs) at pos[i] = the exclusive scan of pops; pops[i] becomes what it
// actually popped there (the ring checks of :75-83 and :293-303 included),
// and scal[0] the first packet whose pops changed.  The sequential positions
// are the fixed point, and each step makes at least one more packet exact:
// pos[0] = 0 always is, so after k steps packets [0, k) are.
__global__ __launch_bounds__(kQpBlock) void qp_relax_kernel(QpCtx C, uint32_t* pops, const uint32_t* __restrict__ pos,
                                                            uint64_t n, unsigned long long* scal, QpSegs S) {
  const QpRange R = qp_range(S, n);
  const QpCtx Cs = qp_ctx_of(C, S, R.s);
  for (uint64_t i = R.i; i < R.end; i += R.step) {
    nicgpu_qp_stats st{};
    QpNullSink sink;
    // a guess past the ring's end is clamped to it (the sequential positions
    // never pass it; resolve_packet must not index past rx[nrx - 1])
    const uint64_t p = qp_abs(pos, S, R.s, i);
    const uint64_t rc = p < Cs.nrx ? p : Cs.nrx;
    const uint32_t popped = (uint32_t) nicqp::resolve_packet<nicgpu_completion, nicgpu_segment_write>(Cs, i, rc, st, sink);
    if (popped != pops[i]) {
      atomicMin(&scal[0], (unsigned long long) i);
      pops[i] = popped;
    }
  }
}

// When the relaxation has not settled within kQpRelaxSteps (a long chain of
// packets each shifting the ring under the next), the positions are made by a
// walk instead.  Only a packet that needs more than one RX descriptor (a
// TSO/GSO packet) can pop a count other than its need while the ring lasts — a
// segment's RX check ends it early — and a packet with need 1 pops 1 until the
// ring's end.  So with u_i = (scan of need)_i + delta_i, where delta_i adds
// (pops - need) over the multi-descriptor packets before i, the exact position
// is min(u_i, ring end): one thread per segment walks those packets in ring
// order, resolving each at its exact position and carrying delta; the packets
// that reach the ring's end are then settled by one relaxation step.
__global__ __launch_bounds__(kQpBlock) void qp_multi_flag_kernel(const uint32_t* __restrict__ need, uint64_t n,
                                                                 uint32_t* flag) {
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i <= n; i += (uint64_t) gridDim.x * kQpBlock)
    flag[i] = i < n && need[i] >= 2u ? 1u : 0u;
}

__global__ __launch_bounds__(kQpBlock) void qp_multi_list_kernel(const uint32_t* __restrict__ flag,
                                                                 const uint32_t* __restrict__ at, uint64_t n,
                                                                 uint32_t* list) {
  for (uint64_t i = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; i < n; i += (uint64_t) gridDim.x * kQpBlock)
    if (flag[i]) list[at[i]] = (uint32_t) i;
}

// one block per segment (one for an unsegmented batch), its first thread walks
__global__ __launch_bounds__(kWave) void qp_walk_kernel(QpCtx C, uint32_t* need, const uint32_t* __restrict__ pos,
                                                        const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ at, uint64_t n, QpSegs S) {
  if (threadIdx.x != 0) return;
  const uint32_t s = blockIdx.x;
  const uint64_t tb = S.seg ? S.seg[s].tx_begin : 0, te = S.seg ? qp_seg_end(S, s, n) : n;
  const QpCtx Cs = qp_ctx_of(C, S, s);
  int64_t delta = 0;
  for (uint32_t k = at[tb], ke = at[te]; k < ke; ++k) {
    const uint64_t m = list[k];
    const int64_t u = (int64_t) qp_abs(pos, S, s, m) + delta;
    const uint64_t p = u < (int64_t) Cs.nrx ? (uint64_t) u : Cs.nrx;
    nicgpu_qp_stats st{};
    QpNullSink sink;
    const uint32_t got = (uint32_t) nicqp::resolve_packet<nicgpu_completion, nicgpu_segment_write>(Cs, m, p, st, sink);
    delta += (int64_t) got - (int64_t) need[m];
    need[m] = got;
  }
}

// packets [0, lim) at their (exact) positions: completions, writes, per-block
// stats.  With `guess` (the pops the positions were scanned from) the pass is
// speculative: first[0] becomes the first packet that popped otherwise, and
// only [0, first] is exact — all of it when nothing differed.
__global__ __launch_bounds__(kQpBlock) void qp_full_kernel(QpCtx C, const uint32_t* __restrict__ pos, uint64_t lim,
                                                           nicgpu_completion* txc, nicgpu_completion* rxc,
                                                           nicgpu_segment_write* writes, uint64_t* partials,
                                                           const uint32_t* __restrict__ guess, const unsigned long long* g,
                                                           unsigned long long gen, QpSegs S, uint8_t* late,
                                                           uint64_t keep) {
  __shared__ uint64_t red[kQpStats][kQpBlock / kWave];
  // after the per-block stats: [0] the RX descriptors used (pos[lim]), [1] the
  // first mismatch (seeded with n by qp_need_kernel) — one download for all
  uint64_t* tail = partials + (uint64_t) gridDim.x * kQpStats;
  unsigned long long* first = reinterpret_cast<unsigned long long*>(tail + 1);
  if (blockIdx.x == 0 && threadIdx.x == 0) tail[0] = pos[lim];
  nicgpu_qp_stats st{};
  if (qp_plan_bad(g, gen)) lim = 0;
  const QpRange R = qp_range(S, lim);
  QpCtx Cs = qp_ctx_of(C, S, R.s);
  Cs.late = qp_late(g, gen);
  for (uint64_t i = R.i; i < R.end; i += R.step) {
    const uint64_t p = qp_abs(pos, S, R.s, i);
    if (p > Cs.nrx) {  // exact positions never pass the ring's end: a guess past it is wrong
      if (guess) atomicMin(first, (unsigned long long) i);
      continue;
    }
    QpDevSink sink{txc, rxc, writes, i, p, Cs.late ? late : nullptr, keep};
    const uint32_t popped = (uint32_t) nicqp::resolve_packet<nicgpu_completion, nicgpu_segment_write>(Cs, i, p, st, sink);
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
                                                                     uint64_t ntx, bool settle, const unsigned long long* g,
                                                                     unsigned long long gen) {
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
  if (threadIdx.x == 0) {
    const bool bad = qp_plan_bad(g, gen);
    if (settle) {
      const uint64_t first = tail[1];
      tail[2] = bad ? 0u : (first < ntx ? (uint64_t) pos[first] : tail[0]);
    }
    tail[19] = g[0] == gen ? 2u : (g[3] == gen ? 1u : 0u);
    tail[20] = g[5];
    tail[21] = qp_late(g, gen) ? 1u : 0u;
  }
}

// Segmented batches, after a final pass and qp_reduce_kernel (one block per
// segment): out[s * kQpSegOut ..] = segment s's 16 statistics summed over its
// blocks' partials, then the RX descriptors its queue pair used (its pops'
// scan across its packets); block 0 sets the settled count the delivery reads,
// tail[2], to the whole concatenated ring when the speculative pass settled
// every packet and to 0 otherwise (a segmented resolve settles all or nothing).
constexpr unsigned kQpSegOut = kQpStats + 1;
__global__ __launch_bounds__(kQpBlock) void qp_seg_reduce_kernel(const uint64_t* __restrict__ partials, QpSegs S,
                                                                 const uint32_t* __restrict__ fb,
                                                                 const uint32_t* __restrict__ pos, uint64_t ntx,
                                                                 uint64_t* out, uint64_t* tail, uint64_t nrx_cat,
                                                                 bool settle, const unsigned long long* g,
                                                                 unsigned long long gen) {
  __shared__ uint64_t red[kQpBlock];
  const uint32_t s = blockIdx.x;
  const uint32_t b0 = fb[s], nb = S.blk[b0].nb;
  const unsigned k = threadIdx.x % kQpStats, r = threadIdx.x / kQpStats;
  constexpr unsigned kRows = kQpBlock / kQpStats;
  uint64_t x = 0;
  for (unsigned b = r; b < nb; b += kRows) x += partials[(size_t) (b0 + b) * kQpStats + k];
  red[threadIdx.x] = x;
  __syncthreads();
  for (unsigned h = kRows / 2; h > 0; h >>= 1) {
    if (r < h) red[threadIdx.x] += red[threadIdx.x + h * kQpStats];
    __syncthreads();
  }
  if (threadIdx.x < kQpStats) out[(size_t) s * kQpSegOut + threadIdx.x] = red[threadIdx.x];
  if (threadIdx.x == 0) {
    const uint64_t a = S.seg[s].tx_begin, e = qp_seg_end(S, s, ntx);
    out[(size_t) s * kQpSegOut + kQpStats] = (uint32_t) (pos[e] - pos[a]);
    if (s == 0 && settle) tail[2] = (!qp_plan_bad(g, gen) && tail[1] >= ntx) ? nrx_cat : 0u;
  }
}

// the segment that RX slot j belongs to (rx_begin ascending)
__device__ __forceinline__ uint32_t qp_seg_of_rx(const QpSegs& S, uint64_t j) {
  uint32_t lo = 0, hi = S.nseg;  // largest s with rx_begin_s <= j
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (S.seg[mid].rx_begin <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Ring slots a segment's queue pair did not use: an empty write and status
// NICGPU_QP_SLOT_UNUSED, so the delivery writes nothing there and RSS skips
// them.  Speculative (`first`): only when the speculative pass settled all.
__global__ __launch_bounds__(kQpBlock) void qp_holes_kernel(QpSegs S, const uint64_t* __restrict__ segout,
                                                            uint64_t nrx_cat, nicgpu_completion* rxc,
                                                            nicgpu_segment_write* w, const unsigned long long* first,
                                                            uint64_t ntx) {
  if (first && *first < ntx) return;
  for (uint64_t j = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; j < nrx_cat; j += (uint64_t) gridDim.x * kQpBlock) {
    const uint32_t s = qp_seg_of_rx(S, j);
    if (j - S.seg[s].rx_begin < segout[(size_t) s * kQpSegOut + kQpStats]) continue;
    nicgpu_segment_write z{};
    w[j] = z;
    rxc[j].status = NICGPU_QP_SLOT_UNUSED;
  }
}

// Dispatch lists of a segmented batch split per segment: split[s * nq + r] =
// the first entry of RSS queue r's list at or past segment s's first slot
// (lists hold absolute slots, ascending), split[nseg * nq + r] = its end.
__global__ __launch_bounds__(kQpBlock) void qp_seg_split_kernel(QpSegs S, uint32_t nq, const uint32_t* __restrict__ which,
                                                                const uint32_t* __restrict__ start,
                                                                const uint32_t* __restrict__ end, uint32_t* split) {
  const uint64_t t = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x;
  if (t >= (uint64_t) (S.nseg + 1) * nq) return;
  const uint32_t s = (uint32_t) (t / nq), r = (uint32_t) (t % nq);
  uint32_t lo = start[r], hi = end[r];
  if (s < S.nseg) {
    const uint64_t v = S.seg[s].rx_begin;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (which[mid] < v) lo = mid + 1;
      else hi = mid;
    }
  }
  split[t] = s < S.nseg ? lo : end[r];
}

// the listed entries relative to their segment's first slot
__global__ __launch_bounds__(kQpBlock) void qp_seg_rel_kernel(QpSegs S, uint32_t* which,
                                                              const unsigned long long* __restrict__ count) {
  const uint64_t m = *count;
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < m; k += (uint64_t) gridDim.x * kQpBlock) {
    const uint32_t e = which[k];
    which[k] = e - (uint32_t) S.seg[qp_seg_of_rx(S, e)].rx_begin;
  }
}

// per-segment RSS hits of the delivered frames.  Each block takes a
// contiguous range of slots, which meets one or two segments: per segment an
// LDS histogram, flushed once (its nonzero bins) with global atomics — one
// atomic per slot on a few thousand addresses took 1.3 ms per 1 M slots.
constexpr uint32_t kQpSegHitsLds = 8192;  // table entries histogrammed in LDS
__global__ __launch_bounds__(kQpBlock) void qp_seg_hits_kernel(QpSegs S, uint64_t nrx, const nicgpu_completion* __restrict__ rxc,
                                                               const uint32_t* __restrict__ rx_hash, uint64_t tn,
                                                               unsigned long long* hits) {
  __shared__ uint32_t h[kQpSegHitsLds];
  const uint64_t per = (nrx + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t) blockIdx.x * per, hi = lo + per < nrx ? lo + per : nrx;
  if (lo >= hi) return;
  for (uint32_t s = qp_seg_of_rx(S, lo); s < S.nseg && S.seg[s].rx_begin < hi; ++s) {
    const uint64_t a = S.seg[s].rx_begin > lo ? S.seg[s].rx_begin : lo;
    const uint64_t e0 = S.seg[s].rx_begin + S.seg[s].nrx, e = e0 < hi ? e0 : hi;
    if (a >= e) continue;
    for (uint32_t k = threadIdx.x; k < tn; k += kQpBlock) h[k] = 0u;
    __syncthreads();
    for (uint64_t j = a + threadIdx.x; j < e; j += kQpBlock)
      if (rxc[j].status == nicqp::kSuccess) atomicAdd(&h[rx_hash[j] % tn], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < tn; k += kQpBlock)
      if (h[k]) atomicAdd(&hits[(uint64_t) s * tn + k], (unsigned long long) h[k]);
    __syncthreads();
  }
}

// (tables above kQpSegHitsLds entries) one global atomic per delivered frame
__global__ __launch_bounds__(kQpBlock) void qp_seg_hits_global_kernel(QpSegs S, uint64_t nrx,
                                                                      const nicgpu_completion* __restrict__ rxc,
                                                                      const uint32_t* __restrict__ rx_hash, uint64_t tn,
                                                                      unsigned long long* hits) {
  for (uint64_t j = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; j < nrx; j += (uint64_t) gridDim.x * kQpBlock) {
    if (rxc[j].status != nicqp::kSuccess) continue;
    atomicAdd(&hits[(uint64_t) qp_seg_of_rx(S, j) * tn + rx_hash[j] % tn], 1ull);
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
// Segmented (several queue pairs): the check is per queue pair — the spans of
// another queue pair are the manager's business (qm_detail::queues_disjoint).
// Each span end is keyed (segment << 48) | end, so the running max restarts at
// every segment's first RX descriptor and a comparison across segments never
// flags; a TX descriptor searches its own segment's ring.
constexpr unsigned kQpSegShift = 48;
__device__ __forceinline__ uint32_t qp_seg_of_tx(const QpSegs& S, uint64_t i) {
  uint32_t lo = 0, hi = S.nseg;  // largest s with tx_begin_s <= i (empty segments share a tx_begin: the last)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (S.seg[mid].tx_begin <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}
struct QpRxEndSeg {  // QpRxEnd keyed by segment, for RX index k
  const nicgpu_rx_descriptor* rx;
  QpSegs S;
  uint64_t mem_size;
  __host__ __device__ uint64_t operator()(uint64_t k) const {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t key = S.seg ? (uint64_t) qp_seg_of_rx(S, k) << kQpSegShift : 0u;
    return key | QpRxEnd{mem_size}(rx[k]);
#else
    (void) k;
    return 0;
#endif
  }
};

// Also the batch's bounds (unsegmented batches; bounds[0..3] preset to
// ~0, 0, ~0, 0): the TX spans' [min start, max end) — per-block reduction, one
// atomic pair per block — and the RX spans' [first start, running max end),
// which bound every byte the batch's DMA writes can touch when the spans
// ascend (the caller's pipelining reads them only then).
// SIMPLE: no running-max scan beforehand — every RX span is taken to be
// nonempty, so the ring ascends iff each span starts at or after the previous
// one's end and the running max is the previous end itself; a span that
// receives nothing sets bounds[4] = gen (the caller then runs the scan form).
template <bool SIMPLE>
__global__ __launch_bounds__(kQpBlock) void qp_check_kernel(const nicgpu_tx_descriptor* __restrict__ tx, uint64_t ntx,
                                                            const nicgpu_rx_descriptor* __restrict__ rx, uint64_t nrx,
                                                            uint64_t mem_size, const uint64_t* __restrict__ end_max,
                                                            unsigned long long* flag, unsigned long long gen, QpSegs S,
                                                            unsigned long long* bounds) {
  __shared__ unsigned long long red_lo[kQpBlock / kWave], red_hi[kQpBlock / kWave];
  const uint64_t n = ntx > nrx ? ntx : nrx;
  uint64_t tlo = ~0ull, thi = 0;
  // key | end of RX span j: the scan's running max, or (SIMPLE) the span's own
  auto end_at = [&](uint64_t j) __attribute__((always_inline)) -> uint64_t {
    if constexpr (SIMPLE) {
      const uint64_t key = S.seg ? (uint64_t) qp_seg_of_rx(S, j) << kQpSegShift : 0u;
      return key | QpRxEnd{mem_size}(rx[j]);
    } else {
      return end_max[j];
    }
  };
  for (uint64_t k = (uint64_t) blockIdx.x * kQpBlock + threadIdx.x; k < n; k += (uint64_t) gridDim.x * kQpBlock) {
    if constexpr (SIMPLE) {
      if (k < nrx && QpRxEnd{mem_size}(rx[k]) == 0) bounds[4] = gen;  // not the simple form
    }
    if (k < nrx && bounds && !S.seg) {
      const uint64_t e = QpRxEnd{mem_size}(rx[k]);
      if (e != 0 && (k == 0 || end_at(k - 1) == 0)) bounds[2] = rx[k].buffer_address;  // the first span's start
      if (k + 1 == nrx) bounds[3] = end_at(k);
    }
    if (k < nrx && k > 0 && QpRxEnd{mem_size}(rx[k]) != 0) {
      const uint64_t key = S.seg ? (uint64_t) qp_seg_of_rx(S, k) << kQpSegShift : 0u;
      if ((key | rx[k].buffer_address) < end_at(k - 1)) flag[0] = gen;
    }
    if (k < ntx) {
      const uint64_t a = tx[k].buffer_address, len = tx[k].length;
      if (len == 0 || !nicqp::dma_ok(mem_size, a, len)) continue;
      tlo = a < tlo ? a : tlo;
      thi = a + len > thi ? a + len : thi;
      uint64_t lo = 0, hi = nrx, key = 0;
      if (S.seg) {
        const uint32_t s = qp_seg_of_tx(S, k);
        lo = S.seg[s].rx_begin;
        hi = lo + S.seg[s].nrx;
        key = (uint64_t) s << kQpSegShift;
      }
      const uint64_t ring_end = hi;
      if constexpr (SIMPLE) {
        // every span nonempty and (when the verdict stands) ascending: a TX
        // span before the range's first RX span or past its last meets none —
        // two reads instead of a search (a TX region apart from the ring)
        if (lo < hi && (a + len <= rx[lo].buffer_address || (key | a) >= end_at(hi - 1))) continue;
      }
      while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (end_at(mid) <= (key | a)) lo = mid + 1;
        else hi = mid;
      }
      if (lo < ring_end && rx[lo].buffer_address < a + len) flag[1] = gen;
    }
  }
  if (!bounds || S.seg) return;
  // the block's TX bounds: wave minimum / maximum, then the block's waves
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const uint64_t l2 = __shfl_xor(tlo, o), h2 = __shfl_xor(thi, o);
    tlo = l2 < tlo ? l2 : tlo;
    thi = h2 > thi ? h2 : thi;
  }
  const unsigned w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    red_lo[w] = tlo;
    red_hi[w] = thi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (unsigned i = 1; i < kQpBlock / kWave; ++i) {
      tlo = red_lo[i] < tlo ? red_lo[i] : tlo;
      thi = red_hi[i] > thi ? red_hi[i] : thi;
    }
    if (thi != 0) {
      atomicMin(&bounds[0], (unsigned long long) tlo);
      atomicMax(&bounds[1], (unsigned long long) thi);
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
  uint32_t *mflag = nullptr, *mscan = nullptr, *mlist = nullptr;  // the position walk's (qp_walk)
  size_t c_mflag = 0, c_mscan = 0, c_mlist = 0;
  uint64_t* piece_desc = nullptr;
  uint16_t* piece_csum = nullptr;  // split sums: each piece past its first 4 bytes ...
  uint16_t* piece_cs4 = nullptr;   // ... and its first min(4, len)
  size_t c_pcs4 = 0;
  uint64_t np = 0;                 // pieces of the last plan (nicgpu_qp_plan_on) or resolved plan
  uint64_t want_pieces = 0;        // piece capacity an overflowing async plan asked for
  unsigned long long plan_gen = 0; // generation of the last plan: its overflow flags in gflags
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
  unsigned long long* bounds = nullptr;  // [8] the check's TX and RX bounds (nicgpu_qp_check_bounds), [4] empty-span flag, [5..6] its two flags
  unsigned long long* scal = nullptr;
  unsigned long long* dlv_acc = nullptr;  // the delivery's accumulator (DeliverParams::acc), zero between launches
  size_t c_dlv_acc = 0;
  unsigned int* dlv_done = nullptr;       // its done ticket
  // zeroed once; flags are set to a call's generation: [0] a descriptor plans
  // > 256 pieces, [1..2] unused, [3] the plan does not fit; then the
  // device piece counts [4] the sums' (below), [5] count, [6] min(count,
  // capacity); [7] the plan's batch may not defer its RX verifies
  unsigned long long* gflags = nullptr;
  // deferred RX verify (nicgpu_qp_set_deferred_verify): per RX completion its
  // bits (qp_logic.h kLate*), the delivery's running corrections [5] (failed
  // verifies, then the rx bytes, rx VLAN strips, tx bytes and tx VLAN
  // insertions they had counted), whether the last resolved batch deferred,
  // and the RX completions its device resolve made (the rest: the host's)
  uint8_t* late = nullptr;
  size_t c_late = 0;
  unsigned long long* fix = nullptr;
  bool defer_verify = false, late_batch = false;
  uint64_t late_used = 0;
  int dlv_reserve = -1;  // nicgpu_qp_set_delivery_reserve (< 0: the default)
  unsigned long long gen = 0;             // generation of the last plan / check call
  uint8_t* tmp = nullptr;
  uint64_t host_scal[4] = {0, 0, 0, 0};
  // page-locked landing space of the small downloads (a pageable one is staged
  // and waited for on the host): [kQpTail] the resolve's RX count, first
  // mismatch, settled prefix and stats totals, then misc(): piece count, check
  // flags, relax verdict
  uint64_t* hp = nullptr;
  uint64_t* misc() const { return hp + kQpTail; }
  // page-locked: the check's download — bounds[0..3], the simple form's
  // "empty span" flag, the unsorted-ring and TX-meets-RX flags (bounds[4..6])
  uint64_t* hp_chk = nullptr;
  unsigned grid = 1;
  // blocks the partials hold: the grid, or one per segment of the largest table
  unsigned part_blocks() const { return grid > NICGPU_QP_MAX_SEGMENTS ? grid : NICGPU_QP_MAX_SEGMENTS; }
  uint64_t walks = 0;  // resolves whose positions the walk made (qp_walk)
  hipEvent_t planned = nullptr;   // nicgpu_qp_plan_on: the piece descriptors are written
  hipEvent_t resolved = nullptr;  // nicgpu_qp_resolve_start: its partials are on the host
  hipEvent_t checked = nullptr;   // nicgpu_qp_check_async: its flags are on the host
  unsigned long long chk_gen = 0; // ... the generation they are compared with
  bool chk_on = false;            // a check is pending (nicgpu_qp_check_wait not yet called)
  struct CheckArgs {              // the pending check's, for its scan form
    uint64_t mem_size = 0, ntx = 0, nrx = 0;
    bool segmented = false;
    hipStream_t s = nullptr;
  } chk_args;
  uint64_t checks_scanned = 0;    // checks that needed the scan form (an RX span receiving nothing)
  // the resolve between nicgpu_qp_resolve_start and _finish
  struct Pending {
    bool on = false;
    uint64_t mem_size = 0, ntx = 0, nrx = 0, max_mtu = 0;
    uint16_t queue_id = 0;
    hipStream_t s = nullptr;
    unsigned grid = 1;
  } res;
  bool delivered = false;  // the RSS results are per completion (nicgpu_qp_deliver), not compacted
  // segmented batches (nicgpu_qp_set_segments): the segment table, the block
  // map of the per-TX launches (seg_grid blocks), each segment's first block,
  // the per-segment results (stats + RX used) on the device and page-locked
  uint32_t nseg = 0;
  unsigned seg_grid = 0;
  uint64_t seg_ntx = 0, seg_nrx = 0;  // the batch the map was made for; the concatenated ring's length
  nicgpu_qp_segment* d_seg = nullptr;
  QpBlk* d_blk = nullptr;
  uint32_t* d_fb = nullptr;
  uint64_t* d_segout = nullptr;
  uint32_t* d_split = nullptr;
  size_t c_seg = 0, c_blk = 0, c_fb = 0, c_segout = 0, c_split = 0;
  uint64_t* seg_hp = nullptr;  // page-locked: nseg * kQpSegOut
  size_t c_seg_hp = 0;
  void* seg_stage = nullptr;   // page-locked staging of the table and the map
  size_t c_seg_stage = 0;
  std::vector<nicgpu_qp_segment> seg_last;  // the table on the device (and its ntx)
  size_t seg_last_ntx = 0;
};

namespace {

void qp_fill_view(const nicgpu_qp* q, nicgpu_qp_view* v) {
  if (!v) return;
  v->tx = q->tx;
  v->rx = q->rx;
  v->piece_base = q->base;
  v->piece_csum = q->piece_csum;
  v->piece_cs4 = q->piece_cs4;
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

QpSegs qp_segs(const nicgpu_qp* q) {
  return q->nseg ? QpSegs{q->d_seg, q->d_blk, q->nseg} : QpSegs{nullptr, nullptr, 0u};
}

// the grid of a per-TX launch over n descriptors: the block map's when segmented
unsigned qp_tx_grid(const nicgpu_qp* q, uint64_t n) { return q->nseg ? q->seg_grid : qp_grid(q, n); }

// hipcub exclusive sum of in[0, n) into out[0, n) (n includes the trailing 0)
int qp_scan(nicgpu_qp* q, const uint32_t* in, uint32_t* out, size_t n, hipStream_t s) {
  size_t tb = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int) n, s) != hipSuccess) return NICGPU_ERR_HIP;
  int st = qp_grow(q->tmp, q->c_tmp, tb);
  if (st != NICGPU_OK) return st;
  return hip_status(hipcub::DeviceScan::ExclusiveSum(q->tmp, tb, in, out, (int) n, s));
}

// After a segmented final pass and its qp_reduce_kernel: per-segment stats and
// RX used (qp_seg_reduce_kernel), the unused ring slots marked (speculative:
// only if everything settled), the results down into seg_hp.
int qp_seg_finish(nicgpu_qp* q, uint64_t ntx, bool speculative, hipStream_t s) {
  const QpSegs S = qp_segs(q);
  uint64_t* tail = q->partials + (size_t) q->seg_grid * kQpStats;
  hipLaunchKernelGGL(qp_seg_reduce_kernel, dim3(q->nseg), dim3(kQpBlock), 0, s, q->partials, S, q->d_fb, q->pos, ntx,
                     q->d_segout, tail, q->seg_nrx, speculative, q->gflags, q->plan_gen);
  int st = hip_status(hipGetLastError());
  if (st != NICGPU_OK) return st;
  if (q->seg_nrx) {
    hipLaunchKernelGGL(qp_holes_kernel, dim3(qp_grid(q, q->seg_nrx)), dim3(kQpBlock), 0, s, S, q->d_segout, q->seg_nrx,
                       q->rxc, q->writes, speculative ? reinterpret_cast<const unsigned long long*>(tail + 1) : nullptr,
                       ntx);
    st = hip_status(hipGetLastError());
  }
  if (st == NICGPU_OK)
    st = hip_status(hipMemcpyAsync(q->seg_hp, q->d_segout, (size_t) q->nseg * kQpSegOut * sizeof(uint64_t),
                                   hipMemcpyDeviceToHost, s));
  return st;
}

// The position walk (qp_walk_kernel): need afresh, its scan, the
// multi-descriptor packets listed, the walk; need then holds every such
// packet's exact pops (the caller scans it and relaxes the ring's end).
int qp_walk(nicgpu_qp* q, const QpCtx& C, const QpSegs& S, uint64_t ntx, unsigned grid, hipStream_t s) {
  int st = qp_grow(q->mflag, q->c_mflag, ntx + 1);
  if (st == NICGPU_OK) st = qp_grow(q->mscan, q->c_mscan, ntx + 1);
  if (st == NICGPU_OK) st = qp_grow(q->mlist, q->c_mlist, ntx + 1);
  if (st != NICGPU_OK) return st;
  uint64_t* tail = q->partials + (size_t) grid * kQpStats;
  hipLaunchKernelGGL(qp_need_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, ntx, q->need,
                     reinterpret_cast<unsigned long long*>(tail + 1), q->gflags, q->plan_gen, S, 1u);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->need, q->pos, ntx + 1, s);
  if (st != NICGPU_OK) return st;
  const unsigned g = qp_grid(q, ntx + 1);
  hipLaunchKernelGGL(qp_multi_flag_kernel, dim3(g), dim3(kQpBlock), 0, s, q->need, ntx, q->mflag);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->mflag, q->mscan, ntx + 1, s);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_multi_list_kernel, dim3(g), dim3(kQpBlock), 0, s, q->mflag, q->mscan, ntx, q->mlist);
  st = hip_status(hipGetLastError());
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_walk_kernel, dim3(S.seg ? S.nseg : 1u), dim3(kWave), 0, s, C, q->need, q->pos, q->mlist,
                     q->mscan, ntx, S);
  return hip_status(hipGetLastError());
}

// The overlap check's launches on s: (simple) the scan-free kernel, or the
// running-max scan then the kernel; bounds and flags (bounds[0..6]) come down
// into hp_chk and q->checked is recorded.
int qp_check_enqueue(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, bool segmented, bool simple,
                     hipStream_t s, unsigned long long gen) {
  // the bounds' presets (page-locked source, constant: no hazard with an
  // earlier copy still reading it)
  uint64_t* preset = q->misc() + kQpBoundsAt + 4;
  preset[0] = ~0ull;
  preset[1] = 0;
  preset[2] = ~0ull;
  preset[3] = 0;
  int st = hip_status(hipMemcpyAsync(q->bounds, preset, 4 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  if (st != NICGPU_OK) return st;
  if (!simple && nrx && segmented) {  // per queue pair: ends keyed by segment
    hipcub::TransformInputIterator<uint64_t, QpRxEndSeg, hipcub::CountingInputIterator<uint64_t>> ends(
        hipcub::CountingInputIterator<uint64_t>(0), QpRxEndSeg{q->rx, qp_segs(q), mem_size});
    size_t tb = 0;
    if (hipcub::DeviceScan::InclusiveScan(nullptr, tb, ends, q->end_max, hipcub::Max(), (int) nrx, s) != hipSuccess)
      return NICGPU_ERR_HIP;
    st = qp_grow(q->tmp_chk, q->c_tmp_chk, tb);
    if (st == NICGPU_OK)
      st = hip_status(hipcub::DeviceScan::InclusiveScan(q->tmp_chk, tb, ends, q->end_max, hipcub::Max(), (int) nrx, s));
  } else if (!simple && nrx) {
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
    const QpSegs S = segmented ? qp_segs(q) : QpSegs{nullptr, nullptr, 0u};
    if (simple)
      hipLaunchKernelGGL(qp_check_kernel<true>, dim3(qp_grid(q, n)), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, q->rx,
                         (uint64_t) nrx, mem_size, q->end_max, q->bounds + 5, gen, S, q->bounds);
    else
      hipLaunchKernelGGL(qp_check_kernel<false>, dim3(qp_grid(q, n)), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx,
                         q->rx, (uint64_t) nrx, mem_size, q->end_max, q->bounds + 5, gen, S, q->bounds);
    st = hip_status(hipGetLastError());
  }
  // one download: bounds, the simple form's empty-span flag, the two flags
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->hp_chk, q->bounds, 7 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipEventRecord(q->checked, s));
  return st;
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
  // blocks per CU of the per-TX kernels (grid-stride loops): 4 measured best
  // on C3 1 M — 8 → 4: one batch at a time 537 → 505 µs, pipelined 480 → 455,
  // qm16 622 → 615; 16 slower, 1–3 no better (profiles/r05_qp_grid_ab.txt).
  // Tuning A/B: NICGPU_QP_BLOCKS_PER_CU.
  static const unsigned grid_per_cu = [] {
    const char* e = std::getenv("NICGPU_QP_BLOCKS_PER_CU");
    const int v = e ? std::atoi(e) : 4;
    return (unsigned) (v >= 1 && v <= 64 ? v : 4);
  }();
  q->grid = (unsigned) di.cus * grid_per_cu;
  if (hipMalloc(&q->scal, 4 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&q->partials, ((size_t) q->part_blocks() * kQpStats + kQpTail) * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&q->queue_start, 65536 * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&q->queue_end, 65536 * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&q->dlv_done, sizeof(unsigned int)) != hipSuccess ||
      hipMemset(q->dlv_done, 0, sizeof(unsigned int)) != hipSuccess ||
      hipMalloc(&q->gflags, 8 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&q->fix, (size_t) NICGPU_QP_MAX_SEGMENTS * NICGPU_QP_FIXUPS * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(q->fix, 0, (size_t) NICGPU_QP_MAX_SEGMENTS * NICGPU_QP_FIXUPS * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&q->bounds, 8 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(q->bounds, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(q->gflags, 0, 8 * sizeof(unsigned long long)) != hipSuccess) {
    nicgpu_qp_destroy(q);
    return NICGPU_ERR_NOMEM;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&q->hp), (kQpTail + 16) * sizeof(uint64_t)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&q->hp_chk), 8 * sizeof(uint64_t)) != hipSuccess) {
    nicgpu_qp_destroy(q);
    return NICGPU_ERR_NOMEM;
  }
  std::memset(q->hp_chk, 0, 8 * sizeof(uint64_t));  // no generation is 0
  if (hipEventCreateWithFlags(&q->planned, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&q->resolved, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&q->checked, hipEventDisableTiming) != hipSuccess) {
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
                  q->queue_start, q->queue_end, q->end_max, q->dlv_acc, q->dlv_done, q->gflags, q->piece_cs4,
                  q->d_seg, q->d_blk, q->d_fb, q->d_segout, q->d_split, q->mflag, q->mscan, q->mlist, q->bounds,
                  q->late, q->fix};
  for (void* b : bufs)
    if (b) (void) hipFree(b);
  if (q->hp) (void) hipHostFree(q->hp);
  if (q->hp_chk) (void) hipHostFree(q->hp_chk);
  if (q->seg_hp) (void) hipHostFree(q->seg_hp);
  if (q->seg_stage) (void) hipHostFree(q->seg_stage);
  if (q->planned) (void) hipEventDestroy(q->planned);
  if (q->resolved) (void) hipEventDestroy(q->resolved);
  if (q->checked) (void) hipEventDestroy(q->checked);
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
  if (st == NICGPU_OK) st = qp_grow(q->late, q->c_late, r1);
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
  if (q->nseg && ntx != q->seg_ntx) return NICGPU_ERR_INVALID;  // the block map is the batch's
  const unsigned grid = qp_tx_grid(q, ntx + 1);
  const unsigned long long gen = ++q->gen;
  q->plan_gen = gen;
  hipLaunchKernelGGL(qp_count_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                     q->plans, q->counts, q->gflags, gen, qp_segs(q), 0u, q->need, q->fix,
                     (q->nseg ? q->nseg : 1u) * NICGPU_QP_FIXUPS);  // (its sums always run)
  int st = hip_status(hipGetLastError());
  uint32_t* np_h = reinterpret_cast<uint32_t*>(q->misc());
  uint64_t* ovf_h = q->misc() + 5;
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(ovf_h, q->gflags, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  // (counts[ntx], the scan's last input, only ends it: base[ntx] = the total)
  if (st == NICGPU_OK) st = qp_scan(q, q->counts, q->base, ntx + 1, s);
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(np_h, q->base + ntx, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  if (st != NICGPU_OK) return st;
  if (*ovf_h == gen) return NICGPU_ERR_RANGE;
  const uint64_t np = *np_h;
  st = qp_grow(q->piece_desc, q->c_pdesc, np ? np : 1);
  if (st == NICGPU_OK) st = qp_grow(q->piece_csum, q->c_pcs, np ? np : 1);
  if (st == NICGPU_OK) st = qp_grow(q->piece_cs4, q->c_pcs4, np ? np : 1);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_fill_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                     q->plans, q->base, q->piece_desc, (uint64_t) q->c_pdesc, q->gflags, gen, qp_segs(q));
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && sums_stream != plan_stream) {  // the sums read the pieces the fill wrote
    st = hip_status(hipEventRecord(q->planned, s));
    if (st == NICGPU_OK) st = hip_status(hipStreamWaitEvent(static_cast<hipStream_t>(sums_stream), q->planned, 0));
  }
  if (st == NICGPU_OK && np)
    st = nicgpu_checksum_batch_split(mem, q->piece_desc, np, q->piece_csum, q->piece_cs4, sums_stream);
  q->np = np;
  *npieces = np;
  qp_fill_view(q, view);
  return st;
}

int nicgpu_qp_plan_async(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                         nicgpu_qp_view* view, void* plan_stream, void* sums_stream) {
  if (!q || ntx > q->cap_tx) return NICGPU_ERR_INVALID;
  if (mem_size && (!mem || (reinterpret_cast<uintptr_t>(mem) & 15u) != 0)) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(plan_stream);
  const uint64_t want = std::max<uint64_t>((uint64_t) ntx + ntx / 4 + 64, q->want_pieces);
  int st = qp_grow(q->piece_desc, q->c_pdesc, want);
  if (st == NICGPU_OK) st = qp_grow(q->piece_csum, q->c_pcs, want);
  if (st == NICGPU_OK) st = qp_grow(q->piece_cs4, q->c_pcs4, want);
  if (st != NICGPU_OK) return st;
  const uint64_t cap = std::min(q->c_pdesc, std::min(q->c_pcs, q->c_pcs4));
  if (q->nseg && ntx != q->seg_ntx) return NICGPU_ERR_INVALID;  // the block map is the batch's
  const unsigned grid = qp_tx_grid(q, ntx + 1);
  const unsigned long long gen = ++q->gen;
  q->plan_gen = gen;
  q->np = 0;  // known once resolved (nicgpu_qp_piece_count)
  hipLaunchKernelGGL(qp_count_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                     q->plans, q->counts, q->gflags, gen, qp_segs(q), q->defer_verify ? 1u : 0u, q->need, q->fix,
                     (q->nseg ? q->nseg : 1u) * NICGPU_QP_FIXUPS);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->counts, q->base, ntx + 1, s);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_fill_kernel, dim3(grid), dim3(kQpBlock), 0, s, q->tx, (uint64_t) ntx, mem_size, max_mtu,
                     q->plans, q->base, q->piece_desc, cap, q->gflags, gen, qp_segs(q));
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && sums_stream != plan_stream) {
    st = hip_status(hipEventRecord(q->planned, s));
    if (st == NICGPU_OK) st = hip_status(hipStreamWaitEvent(static_cast<hipStream_t>(sums_stream), q->planned, 0));
  }
  // the sums over the count the fill left on the device (g[4] <= cap; 0 when
  // the batch defers its RX verifies)
  if (st == NICGPU_OK)
    st = checksum_split_count(mem, q->piece_desc, cap, reinterpret_cast<const uint64_t*>(q->gflags + 4), q->piece_csum,
                              q->piece_cs4, sums_stream);
  qp_fill_view(q, view);
  return st;
}

int nicgpu_qp_piece_count(const nicgpu_qp* q, uint64_t* npieces) {
  if (!q || !npieces) return NICGPU_ERR_INVALID;
  *npieces = q->np;
  return NICGPU_OK;
}

int nicgpu_qp_check(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, int* verdict, void* stream) {
  return nicgpu_qp_check_flags(q, mem_size, ntx, nrx, 0u, verdict, stream);
}

int nicgpu_qp_check_flags(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, unsigned flags, int* verdict,
                          void* stream) {
  if (!verdict) return NICGPU_ERR_INVALID;
  *verdict = -1;
  const int st = nicgpu_qp_check_async(q, mem_size, ntx, nrx, flags, stream);
  return st == NICGPU_OK ? nicgpu_qp_check_wait(q, verdict) : st;
}

int nicgpu_qp_check_bounds(const nicgpu_qp* q, uint64_t* bounds) {
  if (!q || !bounds || q->chk_on || q->nseg) return NICGPU_ERR_INVALID;
  std::memcpy(bounds, q->hp_chk, 4 * sizeof(uint64_t));
  return NICGPU_OK;
}

int nicgpu_qp_resum(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, void* stream) {
  if (!q || (mem_size && (!mem || (reinterpret_cast<uintptr_t>(mem) & 15u) != 0))) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  const uint64_t cap = std::min(q->c_pdesc, std::min(q->c_pcs, q->c_pcs4));
  // (every piece the plan holds, also of a batch that deferred its RX verifies)
  return checksum_split_count(mem, q->piece_desc, cap, reinterpret_cast<const uint64_t*>(q->gflags + 6), q->piece_csum,
                              q->piece_cs4, stream);
}

int nicgpu_qp_check_wait(nicgpu_qp* q, int* verdict) {
  if (!q || !verdict || !q->chk_on) return NICGPU_ERR_INVALID;
  q->chk_on = false;
  DeviceGuard g(q->device);
  int st = hip_status(hipEventSynchronize(q->checked));
  if (st != NICGPU_OK) return st;
  if (q->hp_chk[4] == q->chk_gen) {  // a span that receives nothing: the scan form
    const nicgpu_qp::CheckArgs& A = q->chk_args;
    const unsigned long long gen = ++q->gen;
    st = qp_check_enqueue(q, A.mem_size, A.ntx, A.nrx, A.segmented, false, A.s, gen);
    if (st == NICGPU_OK) st = hip_status(hipEventSynchronize(q->checked));
    if (st != NICGPU_OK) return st;
    q->chk_gen = gen;
    ++q->checks_scanned;
  }
  const uint64_t* f = q->hp_chk + 5;
  *verdict = f[0] == q->chk_gen ? -1 : (f[1] == q->chk_gen ? 0 : 1);
  return NICGPU_OK;
}

int nicgpu_qp_check_async(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, unsigned flags, void* stream) {
  if (!q || ntx > q->cap_tx || nrx > q->cap_rx || (flags & ~NICGPU_QP_CHECK_WHOLE)) return NICGPU_ERR_INVALID;
  const bool segmented = q->nseg && !(flags & NICGPU_QP_CHECK_WHOLE);
  DeviceGuard g(q->device);
  if (q->chk_on) {  // an unwaited earlier check: its flags land before these are reused
    q->chk_on = false;
    if (hipEventSynchronize(q->checked) != hipSuccess) return NICGPU_ERR_HIP;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (segmented && (ntx != q->seg_ntx || nrx != q->seg_nrx)) return NICGPU_ERR_INVALID;
  const unsigned long long gen = ++q->gen;
  // the simple form first (no scan: every RX span nonempty); a ring with an
  // empty span makes nicgpu_qp_check_wait run the scan form behind it
  const int st = qp_check_enqueue(q, mem_size, ntx, nrx, segmented, true, s, gen);
  if (st != NICGPU_OK) return st;
  q->chk_gen = gen;
  q->chk_on = true;
  q->chk_args = nicgpu_qp::CheckArgs{mem_size, (uint64_t) ntx, (uint64_t) nrx, segmented, s};
  return NICGPU_OK;
}

int nicgpu_qp_resolve_start(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, uint64_t max_mtu,
                            uint16_t queue_id, void* stream) {
  if (!q || ntx > q->cap_tx || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  q->res = nicgpu_qp::Pending{};
  if (q->nseg && (ntx != q->seg_ntx || nrx != q->seg_nrx)) return NICGPU_ERR_INVALID;
  QpCtx C{queue_id, max_mtu, mem_size, q->plans, q->piece_csum, q->piece_cs4, q->tx, q->rx, (uint64_t) nrx};
  const QpSegs S = qp_segs(q);
  const unsigned grid = qp_tx_grid(q, ntx + 1);
  uint64_t* tail = q->partials + (size_t) grid * kQpStats;
  // first guess: every packet pops what it needs (rx_need).  The final pass
  // runs on it speculatively and reports the first packet that popped
  // otherwise; a batch that settles at once (uniform RX descriptors, no early
  // ends) needs no relaxation step and no host round trip before its DMA writes.
  hipLaunchKernelGGL(qp_need_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, (uint64_t) ntx, q->need,
                     reinterpret_cast<unsigned long long*>(tail + 1), q->gflags, q->plan_gen, S, 0u);
  int st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = qp_scan(q, q->need, q->pos, ntx + 1, s);
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_full_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->pos, (uint64_t) ntx, q->txc, q->rxc,
                     q->writes, q->partials, q->need, q->gflags, q->plan_gen, S, q->late, (uint64_t) 0);
  st = hip_status(hipGetLastError());
  if (st != NICGPU_OK) return st;
  hipLaunchKernelGGL(qp_reduce_kernel, dim3(1), dim3(kQpReduceThreads), 0, s, q->partials, grid, q->pos,
                     (uint64_t) ntx, true, q->gflags, q->plan_gen);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && q->nseg) st = qp_seg_finish(q, ntx, true, s);
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
  QpCtx C{R.queue_id, R.max_mtu, R.mem_size, q->plans, q->piece_csum, q->piece_cs4, q->tx, q->rx, R.nrx};
  const QpSegs S = qp_segs(q);
  const unsigned grid = R.grid;
  const uint64_t* part = q->hp;  // the tail, kQpTail words (page-locked)
  uint64_t* tail = q->partials + (size_t) grid * kQpStats;
  int st = hip_status(hipEventSynchronize(q->resolved));
  if (st != NICGPU_OK) return st;
  q->np = part[20];
  q->late_batch = part[21] != 0u;
  C.late = q->late_batch;  // (the relaxation's and the walk's resolves)
  q->late_used = 0;
  if (part[19] == 2u) return NICGPU_ERR_RANGE;  // a descriptor planned > 256 pieces: nothing resolved or settled
  if (part[19]) {  // the async plan did not fit its buffers: the same
    q->want_pieces = part[20] + part[20] / 4 + 64;
    return NICGPU_ERR_AGAIN;
  }
  uint64_t used = part[0];
  const unsigned long long first0 = (unsigned long long) part[1];
  const uint64_t settled = part[2];
  unsigned long long first = first0;
  uint64_t lim = ntx;
  if (first < ntx) {  // relax from the same guess (the speculative pass left `need` as it was)
    // everything from here waits on the stream, behind whatever was enqueued
    // after the start (a settled-prefix delivery reads none of what follows)
    auto relax = [&](bool scan_first) {
      for (int it = 0; st == NICGPU_OK; ++it) {
        if (it > 0 || scan_first) st = qp_scan(q, q->need, q->pos, ntx + 1, s);
        q->misc()[4] = ntx;  // page-locked source; the step below waits for the stream
        if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->scal, q->misc() + 4, sizeof(uint64_t), hipMemcpyHostToDevice, s));
        if (st != NICGPU_OK) break;
        hipLaunchKernelGGL(qp_relax_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->need, q->pos, ntx, q->scal, S);
        st = hip_status(hipGetLastError());
        if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->misc() + 3, q->scal, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
        if (st != NICGPU_OK) break;
        first = (unsigned long long) q->misc()[3];
        // pos is exact up to and including `first` (pops before it agreed)
        lim = first < ntx ? (uint64_t) first : ntx;
        if (first >= ntx || it + 1 == kQpRelaxSteps) break;
      }
    };
    relax(false);
    // not settled: the walk, then the ring's end relaxed
    if (st == NICGPU_OK && lim < ntx) {
      st = qp_walk(q, C, S, ntx, grid, s);
      if (st == NICGPU_OK) relax(true);
      if (st == NICGPU_OK) q->walks += 1;
    }
    // a segmented batch settles all or nothing (nothing was delivered: the
    // speculative pass's settled count was 0)
    if (st == NICGPU_OK && q->nseg && lim < ntx) return NICGPU_ERR_UNSETTLED;
    if (st == NICGPU_OK) {
      hipLaunchKernelGGL(qp_full_kernel, dim3(grid), dim3(kQpBlock), 0, s, C, q->pos, lim, q->txc, q->rxc, q->writes,
                         q->partials, static_cast<const uint32_t*>(nullptr), q->gflags, q->plan_gen, S, q->late,
                         q->late_batch ? (uint64_t) settled : (uint64_t) 0);  // (the settled prefix is delivered: its patches stay)
      st = hip_status(hipGetLastError());
    }
    if (st == NICGPU_OK) {
      hipLaunchKernelGGL(qp_reduce_kernel, dim3(1), dim3(kQpReduceThreads), 0, s, q->partials, grid, q->pos, ntx, false,
                         q->gflags, q->plan_gen);
      st = hip_status(hipGetLastError());
    }
    if (st == NICGPU_OK && q->nseg) st = qp_seg_finish(q, ntx, false, s);
    if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->hp, tail, kQpTail * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
    if (st != NICGPU_OK) return st;
    used = part[0];
  }
  std::memcpy(stats, part + 3, kQpStats * sizeof(uint64_t));
  if (q->nseg) used = q->seg_nrx;
  q->late_used = used;  // the completions the device resolved (deferred ones among them)  // every slot of the concatenated ring (the unused ones marked)
  *done = lim;
  *rx_used = used;
  if (rx_settled) *rx_settled = settled < used ? settled : used;
  return NICGPU_OK;
}

int nicgpu_qp_set_deferred_verify(nicgpu_qp* q, int on) {
  if (!q) return NICGPU_ERR_INVALID;
  q->defer_verify = on != 0;
  return NICGPU_OK;
}

int nicgpu_qp_set_delivery_reserve(nicgpu_qp* q, int cus) {
  if (!q) return NICGPU_ERR_INVALID;
  q->dlv_reserve = cus;
  return NICGPU_OK;
}

int nicgpu_qp_deferred(const nicgpu_qp* q, int* deferred) {
  if (!q || !deferred) return NICGPU_ERR_INVALID;
  *deferred = q->late_batch ? 1 : 0;
  return NICGPU_OK;
}

int nicgpu_qp_verify_fixups_async(nicgpu_qp* q, uint64_t* out, size_t nseg, void* stream) {
  if (!q || !out || nseg == 0 || nseg > NICGPU_QP_MAX_SEGMENTS) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  return hip_status(hipMemcpyAsync(out, q->fix, nseg * NICGPU_QP_FIXUPS * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                   static_cast<hipStream_t>(stream)));
}

int nicgpu_qp_walks(const nicgpu_qp* q, uint64_t* walks) {
  if (!q || !walks) return NICGPU_ERR_INVALID;
  *walks = q->walks;
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
  if (flags & ~(unsigned) (NICGPU_DELIVER_SETTLED | NICGPU_DELIVER_APPEND | NICGPU_DELIVER_RESET_HITS))
    return NICGPU_ERR_INVALID;
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
  const bool add_count = (flags & NICGPU_DELIVER_APPEND) != 0, add_hits = (flags & NICGPU_DELIVER_RESET_HITS) == 0;
  if (rx_end == rx_begin) {  // no launch: the resets by hand
    if (rss && !add_count) st = hip_status(hipMemsetAsync(q->scal + 3, 0, sizeof(uint64_t), s));
    if (rss && !add_hits && st == NICGPU_OK) st = hip_status(hipMemsetAsync(hits_dev, 0, ctx->table_n * sizeof(uint64_t), s));
    return st;
  }
  if (rss && ctx->table_n + 1 > q->c_dlv_acc) {  // once per table size: a zero accumulator
    if (q->dlv_acc) (void) hipFree(q->dlv_acc);
    q->dlv_acc = nullptr;
    q->c_dlv_acc = 0;
    if (hipMalloc(&q->dlv_acc, (ctx->table_n + 1) * sizeof(unsigned long long)) != hipSuccess) return NICGPU_ERR_NOMEM;
    q->c_dlv_acc = ctx->table_n + 1;
    st = hip_status(hipMemsetAsync(q->dlv_acc, 0, q->c_dlv_acc * sizeof(unsigned long long), s));
    if (st != NICGPU_OK) return st;
  }
  const DeviceInfo* di = nullptr;
  st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  DeliverParams P{};
  P.reserve = q->dlv_reserve;
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
  if (q->defer_verify) {  // (the kernel reads whether the plan deferred)
    P.late = q->late;
    P.lateflag = q->gflags + 7;
    P.late_gen = q->plan_gen;
    P.late_n = (flags & NICGPU_DELIVER_SETTLED) ? ~0ull : q->late_used;
    P.fix = q->fix;
    P.seg = q->nseg ? q->d_seg : nullptr;
    P.nseg = q->nseg;
  }
  if (rss) {
    P.rss.lut = ctx->d_lut;
    P.rss.table = ctx->d_table;
    P.rss.table_n = (uint32_t) ctx->table_n;
    P.rss.lut_words = 2u * (tuple_mode == NICGPU_TUPLE_RAW ? raw_len : 36u) * 16u;
    P.rx_hash = q->rx_hash;
    P.rx_queue = q->rx_queue;
    P.hits = reinterpret_cast<unsigned long long*>(hits_dev);
    P.count = reinterpret_cast<unsigned long long*>(q->scal + 3);
    P.acc = q->dlv_acc;
    P.done = q->dlv_done;
    P.add_count = add_count ? 1u : 0u;
    P.add_hits = add_hits ? 1u : 0u;
#ifdef NICGPU_HIST_REP
    if (P.rss.table_n <= (uint32_t) kHistLds) {
      P.rss.hits_rep = ctx->d_rep;
      P.rss.hits_done = ctx->d_done;
    }
#endif
  }
  return launch_deliver<0>(P, rss, di->cus, s);
}

int nicgpu_qp_set_segments(nicgpu_qp* q, const nicgpu_qp_segment* seg, size_t nseg, size_t ntx, void* stream) {
  if (!q || nseg > NICGPU_QP_MAX_SEGMENTS || (nseg && !seg)) return NICGPU_ERR_INVALID;
  if (nseg == 0) {
    q->nseg = 0;
    return NICGPU_OK;
  }
  // the segments partition [0, ntx) and the concatenated ring, in order
  uint64_t rx_end = 0;
  for (size_t k = 0; k < nseg; ++k) {
    if (seg[k].tx_begin > ntx || (k && seg[k].tx_begin < seg[k - 1].tx_begin) || seg[k].rx_begin != rx_end)
      return NICGPU_ERR_INVALID;
    rx_end += seg[k].nrx;
  }
  if (seg[0].tx_begin != 0 || ntx > q->cap_tx || rx_end > q->cap_rx) return NICGPU_ERR_INVALID;
  // the table the device holds already (a manager drains the same queue
  // layout again and again): nothing to upload
  if (q->seg_last.size() == nseg && q->seg_last_ntx == ntx && q->seg_grid &&
      std::memcmp(q->seg_last.data(), seg, nseg * sizeof(nicgpu_qp_segment)) == 0) {
    q->nseg = (uint32_t) nseg;
    q->seg_ntx = ntx;
    q->seg_nrx = rx_end;
    return NICGPU_OK;
  }
  q->seg_last.clear();
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // blocks in proportion to the segments' TX descriptors, at least one each
  const uint64_t want = std::max<uint64_t>((ntx + kQpBlock - 1) / kQpBlock, nseg);
  const uint64_t G = std::min<uint64_t>(std::max<uint64_t>(want, nseg), std::max<uint64_t>(q->grid, nseg));
  if (G > q->part_blocks()) return NICGPU_ERR_INVALID;  // partials hold part_blocks() blocks
  std::vector<QpBlk> blk;
  std::vector<uint32_t> fb(nseg);
  blk.reserve(G);
  const uint64_t spare = G - nseg;
  for (size_t k = 0; k < nseg; ++k) {
    const uint64_t e = k + 1 < nseg ? seg[k + 1].tx_begin : ntx;
    const uint64_t n = e - seg[k].tx_begin;
    const uint64_t nb = 1 + (ntx ? spare * n / ntx : 0);
    fb[k] = (uint32_t) blk.size();
    for (uint64_t r = 0; r < nb; ++r) blk.push_back(QpBlk{(uint32_t) k, (uint32_t) r, (uint32_t) nb, 0u});
  }
  int st = qp_grow(q->d_seg, q->c_seg, nseg);
  if (st == NICGPU_OK) st = qp_grow(q->d_blk, q->c_blk, blk.size());
  if (st == NICGPU_OK) st = qp_grow(q->d_fb, q->c_fb, nseg);
  if (st == NICGPU_OK) st = qp_grow(q->d_segout, q->c_segout, nseg * kQpSegOut);
  if (st != NICGPU_OK) return st;
  const size_t b_seg = nseg * sizeof(nicgpu_qp_segment), b_blk = blk.size() * sizeof(QpBlk), b_fb = nseg * 4;
  const size_t need = b_seg + b_blk + b_fb;
  if (need > q->c_seg_stage || nseg * kQpSegOut > q->c_seg_hp) {
    // the previous batch's copies out of the staging may still be in flight
    if (hipStreamSynchronize(s) != hipSuccess) return NICGPU_ERR_HIP;
    if (need > q->c_seg_stage) {
      if (q->seg_stage) (void) hipHostFree(q->seg_stage);
      q->seg_stage = nullptr;
      q->c_seg_stage = 0;
      if (hipHostMalloc(&q->seg_stage, need * 2) != hipSuccess) return NICGPU_ERR_NOMEM;
      q->c_seg_stage = need * 2;
    }
    if (nseg * kQpSegOut > q->c_seg_hp) {
      if (q->seg_hp) (void) hipHostFree(q->seg_hp);
      q->seg_hp = nullptr;
      q->c_seg_hp = 0;
      if (hipHostMalloc(reinterpret_cast<void**>(&q->seg_hp), nseg * kQpSegOut * sizeof(uint64_t)) != hipSuccess)
        return NICGPU_ERR_NOMEM;
      q->c_seg_hp = nseg * kQpSegOut;
    }
  } else if (hipStreamSynchronize(s) != hipSuccess) {  // the staging is reused: its last copies done
    return NICGPU_ERR_HIP;
  }
  auto* st8 = static_cast<uint8_t*>(q->seg_stage);
  std::memcpy(st8, seg, b_seg);
  std::memcpy(st8 + b_seg, blk.data(), b_blk);
  std::memcpy(st8 + b_seg + b_blk, fb.data(), b_fb);
  st = hip_status(hipMemcpyAsync(q->d_seg, st8, b_seg, hipMemcpyHostToDevice, s));
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->d_blk, st8 + b_seg, b_blk, hipMemcpyHostToDevice, s));
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(q->d_fb, st8 + b_seg + b_blk, b_fb, hipMemcpyHostToDevice, s));
  if (st != NICGPU_OK) return st;
  q->nseg = (uint32_t) nseg;
  q->seg_grid = (unsigned) blk.size();
  q->seg_ntx = ntx;
  q->seg_nrx = rx_end;
  q->seg_last.assign(seg, seg + nseg);
  q->seg_last_ntx = ntx;
  return NICGPU_OK;
}

int nicgpu_qp_segment_results(const nicgpu_qp* q, uint64_t* used, nicgpu_qp_stats* stats) {
  if (!q || !q->nseg || !used || !stats) return NICGPU_ERR_INVALID;
  for (uint32_t k = 0; k < q->nseg; ++k) {
    std::memcpy(&stats[k], q->seg_hp + (size_t) k * kQpSegOut, sizeof(nicgpu_qp_stats));
    used[k] = q->seg_hp[(size_t) k * kQpSegOut + kQpStats];
  }
  return NICGPU_OK;
}

int nicgpu_qp_segment_lists(nicgpu_qp* q, size_t nrx, size_t nq, uint32_t* split_host, void* stream) {
  if (!q || !q->nseg || !split_host || nrx > q->cap_rx || nq > 65536) return NICGPU_ERR_INVALID;
  const size_t ns = (size_t) (q->nseg + 1) * nq;
  if (ns == 0) return NICGPU_OK;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int st = qp_grow(q->d_split, q->c_split, ns);
  if (st != NICGPU_OK) return st;
  const QpSegs S = qp_segs(q);
  hipLaunchKernelGGL(qp_seg_split_kernel, dim3((unsigned) ((ns + kQpBlock - 1) / kQpBlock)), dim3(kQpBlock), 0, s, S,
                     (uint32_t) nq, q->queue_which, q->queue_start, q->queue_end, q->d_split);
  st = hip_status(hipGetLastError());
  if (st == NICGPU_OK && nrx) {
    hipLaunchKernelGGL(qp_seg_rel_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, S, q->queue_which,
                       reinterpret_cast<const unsigned long long*>(q->scal + 3));
    st = hip_status(hipGetLastError());
  }
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(split_host, q->d_split, ns * 4, hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  return st;
}

int nicgpu_qp_segment_hits(nicgpu_qp* q, size_t nrx, size_t table_n, uint64_t* hits_dev, void* stream) {
  if (!q || !q->nseg || !hits_dev || table_n == 0 || nrx > q->cap_rx) return NICGPU_ERR_INVALID;
  DeviceGuard g(q->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int st = hip_status(hipMemsetAsync(hits_dev, 0, (size_t) q->nseg * table_n * sizeof(uint64_t), s));
  if (st == NICGPU_OK && nrx && table_n <= kQpSegHitsLds) {
    // a few blocks of long ranges: ~1 K atomics of histogram bins per segment
    const uint64_t want = (nrx + 8191) / 8192;
    const unsigned grid = (unsigned) (want < 256 ? (want ? want : 1) : 256);
    hipLaunchKernelGGL(qp_seg_hits_kernel, dim3(grid), dim3(kQpBlock), 0, s, qp_segs(q), (uint64_t) nrx, q->rxc,
                       q->rx_hash, (uint64_t) table_n, reinterpret_cast<unsigned long long*>(hits_dev));
    st = hip_status(hipGetLastError());
  } else if (st == NICGPU_OK && nrx) {
    hipLaunchKernelGGL(qp_seg_hits_global_kernel, dim3(qp_grid(q, nrx)), dim3(kQpBlock), 0, s, qp_segs(q),
                       (uint64_t) nrx, q->rxc, q->rx_hash, (uint64_t) table_n,
                       reinterpret_cast<unsigned long long*>(hits_dev));
    st = hip_status(hipGetLastError());
  }
  return st;
}

}  // extern "C"

#ifdef NICGPU_TUNING
// tools/f1_deliver_bench.py: one delivery launch over a caller-built write
// list in a timing-only mode (kDlv*; 0 = production), RSS when ctx is given.
extern "C" int nicgpu_tune_deliver(int mode, uint8_t* mem, uint64_t mem_size, const nicgpu_segment_write* w,
                                   const nicgpu_completion* rxc, size_t n, const nicgpu_rss_ctx* ctx,
                                   uint32_t* rx_hash, uint16_t* rx_queue, uint64_t* hits, uint64_t* count,
                                   uint64_t alt_dst, void* stream) {
  if (n == 0) return NICGPU_OK;
  const DeviceInfo* di = nullptr;
  int st = current_device_info(&di);
  if (st != NICGPU_OK) return st;
  DeliverParams P{};
  P.reserve = -1;
  P.mem = mem;
  P.mem_size = mem_size;
  P.w = w;
  P.rxc = const_cast<nicgpu_completion*>(rxc);  // (tuning modes never write it)
  P.j0 = 0;
  P.n = n;
  P.alt_dst = alt_dst;
  const bool rss = ctx != nullptr;
  P.rss.mode = rss ? NICGPU_TUPLE_AUTO : NICGPU_TUPLE_NONE;
  if (rss) {
    P.rss.lut = ctx->d_lut;
    P.rss.table = ctx->d_table;
    P.rss.table_n = (uint32_t) ctx->table_n;
    P.rss.lut_words = 2u * 36u * 16u;
    P.rx_hash = rx_hash;
    P.rx_queue = rx_queue;
    P.hits = reinterpret_cast<unsigned long long*>(hits);
    P.count = reinterpret_cast<unsigned long long*>(count);
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (mode) {
    case 0: return launch_deliver<0>(P, rss, di->cus, s);
    case kDlvNoStore: return launch_deliver<kDlvNoStore>(P, rss, di->cus, s);
    case kDlvNoLoad: return launch_deliver<kDlvNoLoad>(P, rss, di->cus, s);
    case kDlvNoHash: return launch_deliver<kDlvNoHash>(P, rss, di->cus, s);
    case kDlvPackedDst: return launch_deliver<kDlvPackedDst>(P, rss, di->cus, s);
    case kDlvNoLoad | kDlvNoHash: return launch_deliver<kDlvNoLoad | kDlvNoHash>(P, rss, di->cus, s);
    case kDlvNoStore | kDlvNoHash: return launch_deliver<kDlvNoStore | kDlvNoHash>(P, rss, di->cus, s);
    case kDlvNoStore | kDlvNoLoad | kDlvNoHash: return launch_deliver<kDlvNoStore | kDlvNoLoad | kDlvNoHash>(P, rss, di->cus, s);
    case kDlvV1: return launch_deliver<kDlvV1>(P, rss, di->cus, s);
    case kDlvV1 | kDlvNoStore | kDlvNoLoad | kDlvNoHash:
      return launch_deliver<kDlvV1 | kDlvNoStore | kDlvNoLoad | kDlvNoHash>(P, rss, di->cus, s);
    case kDlvV1 | kDlvNoStore | kDlvNoHash: return launch_deliver<kDlvV1 | kDlvNoStore | kDlvNoHash>(P, rss, di->cus, s);
    case kDlvV1 | kDlvNoLoad | kDlvNoHash: return launch_deliver<kDlvV1 | kDlvNoLoad | kDlvNoHash>(P, rss, di->cus, s);
    default: return NICGPU_ERR_INVALID;
  }
}
#endif  // NICGPU_TUNING
