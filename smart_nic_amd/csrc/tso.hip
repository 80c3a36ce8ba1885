// tso.hip — row f2: the per-segment checksums of TSO/GSO frames
// (tso_checksum_kernel, QueuePair::build_segments + handle_rx_segment's
// verify, src/queue_pair.cpp:212-278, 434-447) and the materialised
// segmentation with VLAN insert/strip (tso_segment_kernel).  DESIGN.md §4.2, §4.5.

#include "common.h"
#include "host.h"

using namespace nicgpu_detail;

namespace {

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


// One dword of a segment at offset r0 from its start (4-aligned in memory),
// any overlap with the segment: bytes from the prefix / part A / part B,
// chosen with selects from unconditional LDS byte reads, and stored through a
// buffer resource over the segment's own bytes (`seg` = out + dst,
// num_records = size), so a byte outside the segment — or every byte of a
// lane with no edge dword (`on` false) — is an out-of-range store the
// hardware drops.  Returns its halfword sum (absolute positions).  (Round 5's
// form branched per byte: most of the kernel's scalar instructions,
// profiles/r06_tso_pmc.json.)
__device__ __forceinline__ uint32_t seg_dword_select(__amdgpu_buffer_rsrc_t seg, bool on, int r0, int sz, int pa, int pb,
                                                     uint32_t tag, const uint8_t* st_b, uint32_t a, uint32_t b) {
  // the prefix (81 00 tag-hi tag-lo) as a little-endian dword: byte r of it
  const uint32_t pfx = 0x81u | (((tag >> 8) & 0xFFu) << 16) | ((tag & 0xFFu) << 24);
  uint32_t o = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + q;
    const bool in = on && r >= 0 && r < sz;
    const uint32_t idx = r >= pb ? b + (uint32_t) (r - pb) : a + (uint32_t) (r - pa);
    const uint32_t lb = st_b[in && r >= pa ? idx : 0u];
    const uint32_t pv = (pfx >> (8u * ((uint32_t) r & 3u))) & 0xFFu;
    const uint32_t v = in ? (r < pa ? pv : lb) : 0u;
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t) v, seg, in ? r : -1, 0, 0);
    o |= v << (8 * q);
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
  // a uniform trip count, and no branch per block: a block outside part A /
  // part B (or past nblk) reads the stage's first dwords and stores at an
  // out-of-range offset of the blocks' buffer resource, which the hardware
  // drops; alignbyte by 0 is the low dword, so no select on the shift
  const __amdgpu_buffer_rsrc_t blks =
      __builtin_amdgcn_make_buffer_rsrc(out + D16, (short) 0, (int) (nblk * 16u), 0x00020000);
  const uint32_t iters = (nblk + kWave - 1) / kWave;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t j = it * kWave + lane;
    const int r0 = (int) (D16 - dst) + 16 * (int) j;
    const bool inB = r0 >= pb && r0 + 16 <= sz;
    const bool inA = r0 >= pa && r0 + 16 <= pb;
    const uint32_t okm = -(uint32_t) ((inA || inB) && j < nblk);  // all ones for a block to write
    // (masks, not selects: the compiler turned the selects into branches)
    const uint32_t srcA = a + (uint32_t) (r0 - pa), srcB = b + (uint32_t) (r0 - pb);
    const uint32_t src = (srcA ^ ((srcA ^ srcB) & -(uint32_t) inB)) & okm;
    const uint32_t k = src >> 2, sh = src & 3u;
    const uint32_t w0 = st[k], w1 = st[k + 1], w2 = st[k + 2], w3 = st[k + 3], w4 = st[k + 4];
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
    o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
    o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
    o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
    __builtin_amdgcn_raw_buffer_store_b128(o, blks, (int) ((16u * j) | ~okm), 0, 2);  // nt: as the f1 delivery
    const uint32_t s4 = add_halves(o.w, add_halves(o.z, add_halves(o.y, add_halves(o.x, 0u))));
    sum += s4 & okm;
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
    const bool on = size != 0 && !dup && !pass1 && A + 4 > dst && A < E;
    const __amdgpu_buffer_rsrc_t seg =
        __builtin_amdgcn_make_buffer_rsrc(out + dst, (short) 0, (int) size, 0x00020000);
    sum += seg_dword_select(seg, on, (int) ((int64_t) A - (int64_t) dst), sz, pa, pb, tag, st_b, a, b);
  }
  return sum;
}

// A segment whose prefix and part A together fit 64 B is first made one
// contiguous run in the stage: [prefix | part A] is written right before its
// part B (over bytes of the previous segment's payload, already stored, or —
// for the first segment — A over itself and the prefix into the pad before
// the frame), so the copy has one source and edges only at the segment's
// ends (seg_copy_one).  The pad: 64 B before the stage.
constexpr uint32_t kSegPadChunks = 4;

// Segment bytes out[dst, +size) = stage[s0, +size), one source: pass 1 as in
// seg_copy_stage over the 16-B blocks inside the segment, pass 2 the (at most
// two) partial blocks at its ends, byte-selected as in seg_dword_select.
__device__ __forceinline__ uint32_t seg_copy_one(uint8_t* out, uint64_t dst, uint32_t size, const uint8_t* st_b,
                                                 int s0, uint32_t lane) {
  const uint32_t* st = reinterpret_cast<const uint32_t*>(st_b);
  const uint64_t E = dst + size;
  const uint64_t D16 = (dst + 15) & ~15ull, E16 = E & ~15ull;
  const uint32_t nblk = E16 > D16 ? (uint32_t) ((E16 - D16) >> 4) : 0u;
  const __amdgpu_buffer_rsrc_t blks =
      __builtin_amdgcn_make_buffer_rsrc(out + D16, (short) 0, (int) (nblk * 16u), 0x00020000);
  const uint32_t iters = (nblk + kWave - 1) / kWave;
  const uint32_t base = (uint32_t) (s0 + (int) (D16 - dst));  // stage byte of block 0
  uint32_t sum = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t j = it * kWave + lane;
    const uint32_t okm = -(uint32_t) (j < nblk);
    const uint32_t src = (base + 16u * j) & okm;
    const uint32_t k = src >> 2, sh = src & 3u;
    const uint32_t w0 = st[k], w1 = st[k + 1], w2 = st[k + 2], w3 = st[k + 3], w4 = st[k + 4];
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
    o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
    o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
    o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
    __builtin_amdgcn_raw_buffer_store_b128(o, blks, (int) ((16u * j) | ~okm), 0, 2);  // nt: as the f1 delivery
    sum += add_halves(o.w, add_halves(o.z, add_halves(o.y, add_halves(o.x, 0u)))) & okm;
  }
  if (lane < 8u) {  // the first and the last block, when partial: 4 dwords each
    const uint64_t B = (lane < 4u ? dst : E - 1) & ~15ull;
    const bool dup = lane >= 4u && B == (dst & ~15ull);
    const bool full = B >= D16 && B < E16;
    const uint64_t A = B + 4ull * (lane & 3u);
    const bool on = size != 0 && !dup && !full && A + 4 > dst && A < E;
    const __amdgpu_buffer_rsrc_t seg = __builtin_amdgcn_make_buffer_rsrc(out + dst, (short) 0, (int) size, 0x00020000);
    const int r0 = (int) ((int64_t) A - (int64_t) dst);
    uint32_t o = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + q;
      const bool in = on && r >= 0 && r < (int) size;
      const uint32_t v = in ? (uint32_t) st_b[s0 + r] : 0u;
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t) v, seg, in ? r : -1, 0, 0);
      o |= v << (8 * q);
    }
    sum += (o & 0xFFFFu) + (o >> 16);
  }
  return sum;
}

__global__ __launch_bounds__(kBlock) void tso_segment_kernel(TsoSegParams P) {
  // +1: stage_u32's second dword; the pad before it: seg_copy_one's prefixes
  __shared__ uint4 stage_s[kWavesPerBlock][kSegPadChunks + kSegStageChunks + 1];
  const int w = __builtin_amdgcn_readfirstlane((int) (threadIdx.x / kWave));
  const uint32_t lane = lane_id();
  const uint64_t nwaves = (uint64_t) gridDim.x * kWavesPerBlock;
  uint4* stage = stage_s[w] + kSegPadChunks;
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
        // stage bytes indexed from the pad's start, so no index is negative
        uint8_t* st_b = reinterpret_cast<uint8_t*>(stage - kSegPadChunks);
        const int a = (int) (src_a - a0 + 16u * kSegPadChunks), b = (int) (src_b - a0 + 16u * kSegPadChunks);
        const int hb = (int) (pl + len_a);
        // [prefix | A] before B: the first segment's B follows A; a later
        // one's run must not reach back into A
        const bool one = hb <= 64 && (k == 0 ? b == a + (int) len_a : b - hb >= a + (int) len_a);
        if (one) {
          if (lane < 16u) {
            const uint32_t pfx = 0x81u | (((tag >> 8) & 0xFFu) << 16) | ((tag & 0xFFu) << 24);
            uint32_t v4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // read every byte first: the first segment writes A over itself
              const int i = (int) (4u * lane) + q;
              const uint32_t lb = st_b[a + (i < hb ? i : 0) - (int) pl];
              v4[q] = i < (int) pl ? (pfx >> (8 * (i & 3))) & 0xFFu : lb;
            }
            // bytes past the blob go to byte 0 of the pad (never read: a
            // prefix reaches back at most 4 bytes before the frame, at >= 60)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int i = (int) (4u * lane) + q;
              st_b[i < hb ? b - hb + i : 0] = (uint8_t) v4[q];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          sum = seg_copy_one(P.out, dst, (uint32_t) size, st_b, b - hb, lane);
        } else {
          sum = seg_copy_stage(P.out, dst, (uint32_t) size, (uint32_t) pl, tag, st_b, (uint32_t) a, (uint32_t) len_a,
                               (uint32_t) b, lane);
        }
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

}  // namespace

extern "C" {

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
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) blocks_per_cu(reinterpret_cast<const void*>(tso_checksum_kernel), kBlock, 0) * 2;
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(tso_checksum_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
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
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) blocks_per_cu(reinterpret_cast<const void*>(tso_segment_kernel), kBlock, 0);
  const unsigned grid = (unsigned) (want < cap ? want : cap);
  hipLaunchKernelGGL(tso_segment_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), P);
  return hip_status(hipGetLastError());
}

}  // extern "C"
