// icrc.hip — row f4: RoCEv2 ICRC (CRC-32C) over a batch of
// packets, nic::rocev2::IcrcCalculator (src/rocev2/packet.cpp:14-75).
// DESIGN.md §4.7.

#include "common.h"
#include "host.h"

#include <cstdlib>
#include <cstring>

using namespace nicgpu_detail;

namespace {

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

// ---------------------------------------------- lane-cooperative ICRC --
// Eight lanes per packet (a group; eight groups per wave), one 128-B line of
// the packet per step: lane `sub` loads the line's 16-B chunk `sub` — the
// group's loads cover whole lines, so a wave instruction reads eight lines
// instead of the 64 scattered lines of the lane-per-packet walk (92% of that
// kernel's time, profiles/r03_icrc_variants.jsonl).  CRC-32C is linear over
// GF(2): with A the state map of 16 zero bytes, a line's state is
//   S' = A^8 S ^ sum_sub A^(7 - sub) f(0, chunk_sub),
// f(s, c) the slice-by-4 chain over c from s.  Lane 0 runs its chain from S
// (f(S, c) = A S ^ f(0, c)), every lane shifts its result by A^(7 - sub)
// (operator tables: four byte lookups per power), and the group xor-reduces
// (three lane swaps).  Lines are aligned to the packet's END, so only the
// first line is partial: the packet is front-padded with Z zero bytes
// (chunks before the packet read as zeros, the chunk holding its first byte is
// masked) and the chain enters from kCrcLead128[Z], the state Z zero bytes
// take to 0xFFFFFFFF.
struct CrcLead128 {
  uint32_t s[128];
};
constexpr CrcLead128 make_crc_lead128() {
  const Crc32cTables T = make_crc32c_tables();
  uint32_t top_inv[256] = {};
  for (uint32_t k = 0; k < 256; ++k) top_inv[T.t[0][k] >> 24] = k;
  CrcLead128 R{};
  uint32_t s = 0xFFFFFFFFu;
  R.s[0] = s;
  for (int n = 1; n < 128; ++n) {
    const uint32_t k = top_inv[s >> 24];
    s = ((s ^ T.t[0][k]) << 8) | k;
    R.s[n] = s;
  }
  return R;
}
__constant__ CrcLead128 kCrcLead128 = make_crc_lead128();

// op[m][j][v] = A^m applied to (v << 8j): A^m s = xor_j op[m][j][byte j of s]
// (m = 1..4; A = 16 zero bytes: state = (state >> 8) ^ T0[state & 0xFF] per byte)
struct CrcShiftOps {
  uint32_t t[4][4][256];
};
constexpr CrcShiftOps make_crc_shift_ops() {
  const Crc32cTables T = make_crc32c_tables();
  CrcShiftOps O{};
  for (int m = 1; m <= 4; ++m)
    for (int j = 0; j < 4; ++j)
      for (uint32_t v = 0; v < 256; ++v) {
        uint32_t st = v << (8 * j);
        for (int b = 0; b < 16 * m; ++b) st = (st >> 8) ^ T.t[0][st & 0xFFu];
        O.t[m - 1][j][v] = st;
      }
  return O;
}
__constant__ CrcShiftOps kCrcShiftOps = make_crc_shift_ops();

constexpr int kCoopRing = 128;
#ifndef NICGPU_ICRC_LINES
#define NICGPU_ICRC_LINES 4
#endif
constexpr int kCoopLines = NICGPU_ICRC_LINES;  // lines of a packet in flight per group
constexpr uint32_t kOpsBytes = 4u * 4u * 256u * 4u;  // 16 KiB

__device__ __forceinline__ uint32_t crc_shift(const uint32_t* __restrict__ ops, uint32_t m, uint32_t s) {
  const uint32_t* o = ops + (m - 1u) * 1024u;
  return xor3(o[s & 0xFFu], o[256u + ((s >> 8) & 0xFFu)], o[512u + ((s >> 16) & 0xFFu)]) ^ o[768u + (s >> 24)];
}

template <int MODE>
__global__ __launch_bounds__(kIcrcThreads) void icrc_coop_kernel(IcrcParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t Tb[kB4Bytes];
  __shared__ uint32_t ops[kOpsBytes / 4u];
  __shared__ uint64_t ring_all[kIcrcWpb][kCoopRing];
  __shared__ uint4 lead_m[16];  // bytes >= p of a chunk kept
  if (threadIdx.x < 16u) {
    const int p = (int) threadIdx.x;
    lead_m[p] = make_uint4(dword_keep(p, 16, 0), dword_keep(p, 16, 1), dword_keep(p, 16, 2), dword_keep(p, 16, 3));
  }
  for (uint32_t q = threadIdx.x; q < kB4Bytes / 16u; q += kIcrcThreads) {
    const uint32_t o = q * 16u;
    const uint32_t j = 2u * (o >> 16) + ((o >> 7) & 1u), v = (o >> 8) & 255u;
    const uint32_t val = kCrc32c.t[3u - j][v];
    reinterpret_cast<uint4*>(Tb)[q] = make_uint4(val, val, val, val);
  }
  for (uint32_t q = threadIdx.x; q < kOpsBytes / 4u; q += kIcrcThreads) ops[q] = (&kCrcShiftOps.t[0][0][0])[q];
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint32_t sub = lane & 7u;
  const uint32_t cb = (lane & 31u) << 2;  // this lane's copy of the byte tables: bank lane % 32
  const uint32_t cbr = cb | ((cb + 128u) << 8) | (1u << 24);
  uint64_t* ring = ring_all[threadIdx.x / kWave];
  const uint64_t nwaves = (uint64_t) gridDim.x * kIcrcWpb;
  const uint64_t wave = (uint64_t) blockIdx.x * kIcrcWpb + threadIdx.x / kWave;
  const uint64_t per = (P.n + nwaves - 1) / nwaves;
  const uint64_t p0 = wave * per < P.n ? wave * per : P.n;
  const uint64_t p1 = p0 + per < P.n ? p0 + per : P.n;

  uint64_t loaded = p0;
  auto refill = [&]() __attribute__((always_inline)) {
    const uint64_t i = loaded + lane;
    ring[i & (kCoopRing - 1)] = i < p1 ? P.desc[i] : 0ull;
    loaded += kWave;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  };
  refill();
  refill();
  uint64_t next = p0 + 8u;
  uint64_t my = p0 + (lane >> 3);  // this group's packet
  // the group's packet (every lane of the group holds the same values):
  // span [off, end), T lines to go counting down, state S
  uint64_t off = 0, end = 0;
  uint32_t len = 0, tl = 0, S = 0xFFFFFFFFu;
  auto setup = [&]() __attribute__((always_inline)) {
    const uint64_t d = ring[my & (kCoopRing - 1)];
    off = d & kOffMask;
    len = (uint32_t) (d >> NICGPU_DESC_OFFSET_BITS);
    const uint32_t span = P.verify ? (len >= 4u ? len - 4u : 0u) : len;
    end = off + span;
    tl = (span + 127u) >> 7;
    S = kCrcLead128.s[(tl << 7) - span];
  };
  if (my < p1) setup();
  for (;;) {
    const bool active = my < p1;
    if (__ballot(active) == 0ull) break;
    if (active && tl != 0u) {
      // up to kCoopLines of the packet's lines per iteration, every load
      // issued before the first chain (a line's chunk `sub` ends
      // 128 * (tl - k - 1) bytes before the packet's end)
      const uint32_t nl = tl < (uint32_t) kCoopLines ? tl : (uint32_t) kCoopLines;
      u32x4 v[kCoopLines];
      int64_t av[kCoopLines];
#pragma unroll
      for (int k = 0; k < kCoopLines; ++k) {
        const uint32_t tk = (uint32_t) k < nl ? tl - (uint32_t) k : tl;
        const int64_t a = (int64_t) end - 128 * (int64_t) tk + 16 * (int64_t) sub;
        av[k] = a;
        const bool pad = a + 16 <= (int64_t) off;
        const int64_t la = pad ? (int64_t) off : (a < 0 ? 0 : a);
        __builtin_memcpy(&v[k], P.frames + la, 16);  // 16 B at any byte alignment
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < kCoopLines; ++k) {
        if ((uint32_t) k >= nl) break;
        const int64_t a = av[k];
        const bool pad = a + 16 <= (int64_t) off;
        u32x4 x = v[k];
        if (a < 0 && !pad) {  // (the packet starts within the image's first 16 B) bytes shifted up by -a
          const uint32_t d = (uint32_t) (-a) * 8u;
          uint64_t lo = ((uint64_t) x.y << 32) | x.x, hi = ((uint64_t) x.w << 32) | x.z;
          if (d < 64u) {
            hi = (hi << d) | (lo >> (64u - d));
            lo <<= d;
          } else {
            hi = lo << (d - 64u);
            lo = 0;
          }
          x = (u32x4){(uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32)};
        }
        if (pad) {
          x = (u32x4){0u, 0u, 0u, 0u};
        } else if (a < (int64_t) off) {
          const uint4 m = lead_m[(uint32_t) ((int64_t) off - a)];
          x.x &= m.x;
          x.y &= m.y;
          x.z &= m.z;
          x.w &= m.w;
        }
        uint32_t s = sub == 0u ? S : 0u;
        if constexpr (MODE == 1) {
          s ^= x.x ^ x.y ^ x.z ^ x.w;
        } else {
          s = b4_dword(Tb, cbr, s ^ x.x);
          s = b4_dword(Tb, cbr, s ^ x.y);
          s = b4_dword(Tb, cbr, s ^ x.z);
          s = b4_dword(Tb, cbr, s ^ x.w);
          // A^(7 - sub): A^4 when 7 - sub >= 4, then A^((7 - sub) & 3)
          const uint32_t r = 7u - sub;
          const uint32_t s4 = crc_shift(ops, 4u, s);
          s = (r & 4u) ? s4 : s;
          const uint32_t rr = r & 3u;
          const uint32_t sr = crc_shift(ops, rr ? rr : 1u, s);
          s = rr ? sr : s;
        }
        s ^= (uint32_t) __shfl_xor((int) s, 1);
        s ^= (uint32_t) __shfl_xor((int) s, 2);
        s ^= (uint32_t) __shfl_xor((int) s, 4);
        S = s;
      }
      tl -= nl;
    }
    const bool finished = active && tl == 0u;
    if (finished && sub == 0u) {
      const uint32_t crc = S ^ 0xFFFFFFFFu;
      if (P.out_crc) P.out_crc[my] = (P.verify && len < 4u) ? 0u : crc;
      if (P.verify) {
        uint32_t ok = 0;
        if (len >= 4u) {
          const uint8_t* t = P.frames + end;
          const uint32_t stored = ((uint32_t) t[0] << 24) | ((uint32_t) t[1] << 16) | ((uint32_t) t[2] << 8) | t[3];
          ok = stored == crc;
        }
        P.out_ok[my] = (uint8_t) ok;
      }
    }
    // finished groups take the next packets of the wave's range in group order
    const uint64_t m = __ballot(finished && sub == 0u);
    const uint32_t gl = lane & ~7u;
    const uint64_t below = gl ? (m & ((1ull << gl) - 1ull)) : 0ull;
    if (finished) my = next + (uint64_t) __builtin_popcountll(below);
    next += (uint64_t) __builtin_popcountll(m);
    if (finished && my < p1) setup();
    if (next + kWave > loaded && loaded < p1) refill();
  }
}


}  // namespace

extern "C" {

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
  // NICGPU_ICRC (tuning): b4 (default) the lane-per-packet kernel; coop the
  // lane-cooperative one; b4mem / coopmem: timing only, their loads without
  // the table work (results wrong)
  // (the cooperative kernel, measured slower: C2 591 / IMIX 1145 us against
  // 408 / 471 at 4 lines in flight per group, profiles/r04_icrc_coop.jsonl;
  // round 5's pipelined lane walk — two windows in flight per lane, exact
  // vmcnt waits — C2 437 / C3 515 us against 402 / 469, its loads alone 447 /
  // 420: profiles/r05_icrc_pipe_rejected.jsonl, code in git history; round 6's
  // LDS-staged line walk — whole lines moved into LDS by cooperative
  // global_load_lds, 16-copy tables — C2 / C3 442 / 547 against 404 / 477, its
  // loads alone 324 / 386 against 388 / 384, and the lane walk's loads with
  // sc1 / nt policies 604 / 689 and 1006 / 1036: profiles/r06_icrc_variants.jsonl,
  // code in git history, commit 5777fdb)
  static const int var = [] {
    const char* e = std::getenv("NICGPU_ICRC");
    if (!e) return 0;
    if (std::strcmp(e, "coop") == 0) return 2;
    if (std::strcmp(e, "b4mem") == 0) return 1;
    if (std::strcmp(e, "b4") == 0) return 0;
    if (std::strcmp(e, "coopmem") == 0) return 3;
    return 0;
  }();
  const uint64_t want = (n + kIcrcThreads - 1) / kIcrcThreads;
  const uint64_t cap = (uint64_t) di->cus * (uint64_t) blocks_per_cu(reinterpret_cast<const void*>(icrc_b4_kernel<8, 0>), kIcrcThreads, 0);
  const unsigned grid = (unsigned) (want < 1 ? 1 : (want < cap ? want : cap));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int v = var;
  if (v == 1) hipLaunchKernelGGL((icrc_b4_kernel<8, 1>), dim3(grid), dim3(kIcrcThreads), 0, s, P);
  else if (v == 0) hipLaunchKernelGGL((icrc_b4_kernel<8, 0>), dim3(grid), dim3(kIcrcThreads), 0, s, P);
  else if (v == 3) hipLaunchKernelGGL((icrc_coop_kernel<1>), dim3(grid), dim3(kIcrcThreads), 0, s, P);
  else hipLaunchKernelGGL((icrc_coop_kernel<0>), dim3(grid), dim3(kIcrcThreads), 0, s, P);
  return hip_status(hipGetLastError());
}

}  // extern "C"
