// qp_logic.h — the per-packet decisions of QueuePair::process_once
// (src/queue_pair.cpp:67-460) for the batched RX stage, in one
// source for both resolvers: the host one (host/rx_stage.cpp, fuzzed against
// the compiled reference QueuePair) and the device one (f1.hip).
//
// Plain templates over the descriptor, completion, write and stats types: the
// nic:: types on the host, their nicgpu_* C mirrors on the device (same field
// names and layouts, include/nicgpu.h).  No allocation, no exceptions, no
// library calls, so every function compiles for gfx950 as well.
//
// Byte-level facts the resolvers rest on (rx_stage.cpp's header comment):
// ones'-complement sums of pieces compose exactly (fold(a + b) is 0 only when
// a and b are), and a piece placed at an odd offset contributes its
// byte-swapped sum.
#pragma once

#include <stdint.h>

#if defined(__HIP__)
#define NICQP_HD __host__ __device__ inline
#else
#define NICQP_HD inline
#endif

namespace nicqp {

// A descriptor read whole: on the device, 16- or 8-B loads into registers
// (field-by-field reads of the 32-B TX / 24-B RX PODs cost seven memory
// instructions per descriptor); on the host, a plain copy.
template <class T>
NICQP_HD T desc_load(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  T v;
  if constexpr (sizeof(T) % 16 == 0) {
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      u4 w[sizeof(T) / 16];
#pragma unroll
      for (unsigned k = 0; k < sizeof(T) / 16; ++k) w[k] = reinterpret_cast<const u4*>(p)[k];
      __builtin_memcpy(&v, w, sizeof(T));
      return v;
    }
  }
  if constexpr (sizeof(T) % 8 == 0) {
    if ((reinterpret_cast<uintptr_t>(p) & 7u) == 0) {
      typedef unsigned int u2 __attribute__((ext_vector_type(2)));
      u2 w[sizeof(T) / 8];
#pragma unroll
      for (unsigned k = 0; k < sizeof(T) / 8; ++k) w[k] = reinterpret_cast<const u2*>(p)[k];
      __builtin_memcpy(&v, w, sizeof(T));
      return v;
    }
  }
#endif
  return *p;
}

constexpr uint32_t kRun = 65534;  // even, so every run of a plain packet starts at an even offset
constexpr uint64_t kMinMss = 1, kMaxMss = 9000, kMaxTsoSegments = 64;  // include/nic/offload.h:21-23
// CompletionCode (include/nic/tx_rx.h:26-35)
enum : uint32_t {
  kSuccess = 0,
  kBufferTooSmall = 1,
  kChecksumError = 2,
  kNoDescriptor = 3,
  kFault = 4,
  kMtuExceeded = 5,
  kInvalidMss = 6,
  kTooManySegments = 7,
};
// PacketPlan::Kind (include/nic/rx_stage.h)
enum : uint32_t { kNoBytes = 0, kPlain = 1, kSegmented = 2, kPlainSplit = 3 };

NICQP_HD uint32_t add1c(uint32_t a, uint32_t b) {
  const uint32_t x = a + b;
  return (x & 0xFFFFu) + (x >> 16);
}
NICQP_HD uint32_t swap16(uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }
NICQP_HD uint32_t at_offset(uint32_t s, uint64_t off) { return (off & 1) ? swap16(s) : s; }
NICQP_HD uint64_t min64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// SimpleHostMemory::translate_view bounds rule (simple_host_memory.cpp:85-93)
NICQP_HD bool dma_ok(uint64_t mem_size, uint64_t addr, uint64_t len) { return addr <= mem_size && len <= mem_size - addr; }

struct SegDecision {
  bool segmented;  // build_segments produced chunks
  bool invalid_mss;
  bool too_many;
  uint32_t nseg;
  uint32_t H;
};

// build_segments (queue_pair.cpp:212-278) without the copies.
template <class Tx>
NICQP_HD SegDecision decide_segments(const Tx& t) {
  SegDecision d{false, false, false, 1u, 0u};
  const uint64_t L = t.length;
  const bool enabled = (t.tso_enabled || t.gso_enabled) && t.mss > 0 && L > t.mss;
  if (!enabled) return d;
  if (t.mss < kMinMss || t.mss > kMaxMss) {
    d.invalid_mss = true;
    return d;
  }
  if (t.header_length > L) {
    d.invalid_mss = true;
    return d;
  }
  d.H = t.header_length;
  if (d.H >= L) return d;  // degenerate: one unsegmented copy (:250-252)
  const uint64_t n = (L - d.H + t.mss - 1) / t.mss;
  if (n > kMaxTsoSegments) {
    d.too_many = true;
    return d;
  }
  d.segmented = true;
  d.nseg = (uint32_t) n;
  return d;
}

template <class Tx>
NICQP_HD bool tx_verify_needed(const Tx& t) {
  return !t.checksum_offload && (uint32_t) t.checksum != 0u;  // :105 (ChecksumMode::None == 0)
}

// One TX descriptor's plan: the byte pieces whose sums the TX verify
// (:105-116) and the RX verifies (:434-447) need; put(addr, len) receives
// them in order.  Returns the number of pieces (0: no decision reads bytes).
//   kPlain      [0, min(4, L)) then [4, L) in runs of <= kRun bytes
//   kPlainSplit (split4) [0, L) in runs of <= kRun bytes: one piece per
//               packet below 64 KiB, the first one's sum split into its first
//               min(4, len) bytes and the rest (PacketSums::cs4)
//   kSegmented  H >= 4: [0, 4), [4, H), then chunk k = [H + k*mss, +len_k)
//               H < 4:  [0, H), then per chunk [.., +min(4 - H, len_k)) and its rest
template <class Tx, class Plan, class Put>
NICQP_HD uint32_t plan_packet(uint64_t max_mtu, uint64_t mem_size, const Tx& t, Plan& pp, Put&& put,
                              bool split4 = false) {
  uint32_t np = 0;
  pp.kind = static_cast<decltype(pp.kind)>(kNoBytes);
  pp.nseg = 0;
  pp.npieces = 0;
  pp.hdr_len = 0;
  pp.mss = 0;
  const uint64_t L = t.length;
  if (!dma_ok(mem_size, t.buffer_address, L)) return 0;  // read fault: no bytes
  const bool verify = tx_verify_needed(t);
  const bool mtu_drop = L > max_mtu;
  const SegDecision d = decide_segments(t);
  const bool dropped = mtu_drop || d.invalid_mss || d.too_many;
  if (dropped && !verify) return 0;
  const uint64_t a = t.buffer_address;
  if ((!d.segmented || dropped) && split4) {
    pp.kind = static_cast<decltype(pp.kind)>(kPlainSplit);
    put(a, min64(kRun, L));
    ++np;
    for (uint64_t o = kRun; o < L; o += kRun) {
      put(a + o, min64(kRun, L - o));
      ++np;
    }
  } else if (!d.segmented || dropped) {
    pp.kind = static_cast<decltype(pp.kind)>(kPlain);
    put(a, min64(4, L));
    ++np;
    for (uint64_t o = 4; o < L; o += kRun) {
      put(a + o, min64(kRun, L - o));
      ++np;
    }
  } else {
    pp.kind = static_cast<decltype(pp.kind)>(kSegmented);
    pp.nseg = d.nseg;
    pp.hdr_len = d.H;
    pp.mss = t.mss;
    if (d.H >= 4) {
      put(a, 4);
      put(a + 4, d.H - 4);
      np += 2;
      for (uint32_t k = 0; k < d.nseg; ++k) {
        const uint64_t o = d.H + (uint64_t) k * t.mss;
        put(a + o, min64(t.mss, L - o));
        ++np;
      }
    } else {
      put(a, d.H);
      ++np;
      for (uint32_t k = 0; k < d.nseg; ++k) {
        const uint64_t o = d.H + (uint64_t) k * t.mss;
        const uint64_t len = min64(t.mss, L - o);
        const uint64_t n0 = min64(4 - d.H, len);
        put(a + o, n0);
        put(a + o + n0, len - n0);
        np += 2;
      }
    }
  }
  pp.npieces = np;
  return np;
}

// Sums a resolve step needs, for one TX packet.  cs = compute_checksum of
// each piece, i.e. ~fold(sum); with cs4 (split sums, the device's piece pass)
// cs covers each piece's bytes past its first 4 and cs4 its first min(4, len):
// both exact, so a piece's sum is add1c of the two and a kPlainSplit packet's
// first4 / rest need no 4-byte piece of their own.
template <class Plan>
struct PacketSums {
  const Plan* p;
  const uint16_t* cs;
  const uint16_t* cs4;  // null: cs covers whole pieces
  uint64_t L;

  NICQP_HD uint32_t r(uint32_t k) const { return (uint32_t) (uint16_t) ~cs[p->first_piece + k]; }
  NICQP_HD uint32_t h(uint32_t k) const { return (uint32_t) (uint16_t) ~cs4[p->first_piece + k]; }
  // whole piece k (the rest starts 4 bytes in: same byte parity)
  NICQP_HD uint32_t s(uint32_t k) const { return cs4 ? add1c(h(k), r(k)) : r(k); }
  NICQP_HD uint32_t chunk_len(uint32_t k) const {
    const uint64_t o = (uint64_t) p->hdr_len + (uint64_t) k * p->mss;
    return (uint32_t) min64(p->mss, L - o);
  }
  // whole packet, as compute_checksum(packet) sums it
  NICQP_HD uint32_t whole() const {
    uint32_t acc = 0;
    if ((uint32_t) p->kind == kPlain || (uint32_t) p->kind == kPlainSplit) {
      for (uint32_t i = 0; i < p->npieces; ++i) acc = add1c(acc, s(i));  // all runs start at even offsets
      return acc;
    }
    const uint32_t H = p->hdr_len;
    if (H >= 4) {
      acc = add1c(s(0), s(1));
      for (uint32_t k = 0; k < p->nseg; ++k) acc = add1c(acc, at_offset(s(2 + k), H + (uint64_t) k * p->mss));
    } else {
      acc = s(0);
      for (uint32_t k = 0; k < p->nseg; ++k) {
        const uint64_t o = H + (uint64_t) k * p->mss;
        const uint32_t n0 = (uint32_t) min64(4 - H, chunk_len(k));
        acc = add1c(acc, at_offset(s(1 + 2 * k), o));
        acc = add1c(acc, at_offset(s(2 + 2 * k), o + n0));
      }
    }
    return acc;
  }
  // segment k: sum of its first 4 bytes and of the rest (rest placed at offset 4)
  NICQP_HD void segment(uint32_t k, uint32_t& first4, uint32_t& rest) const {
    if ((uint32_t) p->kind == kPlainSplit) {
      first4 = h(0);
      rest = r(0);
      for (uint32_t i = 1; i < p->npieces; ++i) rest = add1c(rest, s(i));
      return;
    }
    if ((uint32_t) p->kind == kPlain) {
      first4 = s(0);
      rest = 0;
      for (uint32_t i = 1; i < p->npieces; ++i) rest = add1c(rest, s(i));
      return;
    }
    const uint32_t H = p->hdr_len;
    if (H >= 4) {
      first4 = s(0);
      rest = add1c(s(1), at_offset(s(2 + k), H - 4));
    } else {
      first4 = add1c(s(0), at_offset(s(1 + 2 * k), H));
      rest = s(2 + 2 * k);
    }
  }
};

// What the resolve of one batch sees.
template <class Tx, class Rx, class Plan>
struct Ctx {
  uint16_t queue_id;
  uint64_t max_mtu;
  uint64_t mem_size;
  const Plan* plans;    // plans[i] for tx[i]
  const uint16_t* cs;   // piece checksums
  const uint16_t* cs4;  // their first-4-byte parts (split sums), or null
  const Tx* tx;
  const Rx* rx;
  uint64_t nrx;
  // deferred RX verify (the device's f1 path, batches where no decision that
  // moves ring positions reads a sum: no TX verify, one segment per packet):
  // the :434-447 check is taken to pass and the completion marked for the
  // delivery, which sums the bytes it writes and patches the failures
  bool late = false;
  // host resolve on a HostMemory with faults modelled (host_memory_faults):
  // each DMA write's verdict is the memory's own translate(address, length)
  // (DMAEngine::write, dma_engine.cpp:23-32), asked here in posting order;
  // null: the bounds rule alone.  Never set on the device.
  const void* wcheck = nullptr;
  bool (*wcheck_fn)(const void*, uint64_t, uint64_t) = nullptr;
};

// The memory's verdict on a DMA write the bounds rule allows (Ctx::wcheck).
template <class C_>
NICQP_HD bool write_allowed(const C_& C, uint64_t addr, uint64_t len) {
#if defined(__HIP_DEVICE_COMPILE__)
  (void) C;
  (void) addr;
  (void) len;
  return true;
#else
  return C.wcheck_fn == nullptr || C.wcheck_fn(C.wcheck, addr, len);
#endif
}

// A deferred completion's bits (the delivery's stats correction on a failure)
enum : uint32_t { kLateDeferred = 1, kLateStripBase = 2, kLateVlanInsert = 4 };

// sink.rx_late(e, w, bits) for a sink that records deferred completions, else
// sink.rx(e, w)
template <class Sink, class Comp, class Write>
NICQP_HD auto sink_rx_late(Sink& s, const Comp& e, const Write* w, uint32_t bits, int)
    -> decltype(s.rx_late(e, w, bits), void()) {
  s.rx_late(e, w, bits);
}
template <class Sink, class Comp, class Write>
NICQP_HD void sink_rx_late(Sink& s, const Comp& e, const Write* w, uint32_t, long) {
  s.rx(e, w);
}

template <class Comp>
NICQP_HD Comp make_completion(uint16_t qid, uint16_t idx, uint32_t st) {  // :150-158
  Comp e;
  e.queue_id = qid;
  e.descriptor_index = idx;
  e.status = st;
  e.checksum_offloaded = false;
  e.checksum_verified = false;
  e.tso_performed = false;
  e.gso_performed = false;
  e.vlan_inserted = false;
  e.vlan_stripped = false;
  e.gro_aggregated = false;
  e.segments_produced = 1;
  e.vlan_tag = 0;
  return e;
}

template <class Comp, class Tx>
NICQP_HD Comp make_tx(uint16_t qid, const Tx& t, uint32_t st, uint64_t segs, bool tso, bool gso) {  // :160-177
  Comp e = make_completion<Comp>(qid, t.descriptor_index, st);
  e.checksum_offloaded = t.checksum_offload;
  e.tso_performed = tso;
  e.gso_performed = gso;
  e.segments_produced = (uint16_t) min64(segs, 0xFFFFu);
  if (t.vlan_insert) {
    e.vlan_inserted = true;
    e.vlan_tag = t.vlan_tag;
  }
  return e;
}

// RX descriptors TX descriptor i pops when the ring has enough of them and no
// RX-side check aborts it early: 0 when it is dropped before the RX stage
// (read fault, TX checksum, MTU, invalid mss, too many segments).
// rx_need of a packet that needs no TX verify (or passed it): the MTU and
// segmentation checks only
template <class Tx>
NICQP_HD uint32_t rx_need_unverified(const Tx& t, uint64_t mem_size, uint64_t max_mtu) {
  const uint64_t L = t.length;
  if (!dma_ok(mem_size, t.buffer_address, L)) return 0;
  if (L > max_mtu) return 0;
  const SegDecision d = decide_segments(t);
  if (d.invalid_mss || d.too_many) return 0;
  return d.nseg;
}

template <class Tx, class Rx, class Plan>
NICQP_HD uint32_t rx_need(const Ctx<Tx, Rx, Plan>& C, uint64_t i) {
  const Tx t = desc_load(C.tx + i);
  const uint64_t L = t.length;
  if (!dma_ok(C.mem_size, t.buffer_address, L)) return 0;
  if (tx_verify_needed(t)) {
    const PacketSums<Plan> ps{&C.plans[i], C.cs, C.cs4, L};
    if ((uint16_t) (~ps.whole() & 0xFFFFu) != t.checksum_value) return 0;
  }
  return rx_need_unverified(t, C.mem_size, C.max_mtu);
}

// QueuePair::process_once (queue_pair.cpp:67-460) for TX descriptor i with
// the RX ring's consumer at rc: posts its completions through `sink` in the
// reference's order (sink.tx(entry, fires_interrupt), sink.rx(entry, write
// or nullptr)), adds to `stats`, returns the RX descriptors it popped.
template <class Comp, class Write, class Tx, class Rx, class Plan, class Stats, class Sink>
NICQP_HD uint64_t resolve_packet(const Ctx<Tx, Rx, Plan>& C, uint64_t i, uint64_t rc, Stats& stats, Sink& sink) {
  const uint16_t qid = C.queue_id;
  const Tx t = desc_load(C.tx + i);
  const PacketSums<Plan> ps{&C.plans[i], C.cs, C.cs4, (uint64_t) t.length};
  const uint64_t L = t.length;
  const uint64_t rc0 = rc;
  // :75-83 no RX descriptor at all
  if (rc == C.nrx) {
    sink.tx(make_tx<Comp>(qid, t, kNoDescriptor, 0, false, false), true);
    stats.drops_no_rx_desc += 1;
    return 0;
  }
  // :86-92 DMA read
  if (!dma_ok(C.mem_size, t.buffer_address, L)) {
    sink.tx(make_tx<Comp>(qid, t, kFault, 0, false, false), true);
    return 0;
  }
  // :94-105 TX checksum verify
  if (tx_verify_needed(t)) {
    const uint16_t computed = (uint16_t) (~ps.whole() & 0xFFFFu);
    if (computed != t.checksum_value) {
      sink.tx(make_tx<Comp>(qid, t, kChecksumError, 0, false, false), true);
      stats.drops_checksum += 1;
      return 0;
    }
  }
  // :195-210 MTU
  if (L > C.max_mtu) {
    sink.tx(make_tx<Comp>(qid, t, kMtuExceeded, 0, false, false), true);
    stats.drops_mtu_exceeded += 1;
    return 0;
  }
  // :212-278 segmentation
  const SegDecision d = decide_segments(t);
  if (d.invalid_mss) {
    sink.tx(make_tx<Comp>(qid, t, kInvalidMss, 0, false, false), true);
    stats.drops_invalid_mss += 1;
    return 0;
  }
  if (d.too_many) {
    sink.tx(make_tx<Comp>(qid, t, kTooManySegments, 0, false, false), true);
    stats.drops_too_many_segments += 1;
    return 0;
  }
  const uint32_t total = d.nseg;
  const bool tso = t.tso_enabled && total > 1;
  const bool gso = t.gso_enabled && total > 1;
  // :293-303 enough RX descriptors for every segment
  if (C.nrx - rc < total) {
    sink.tx(make_tx<Comp>(qid, t, kNoDescriptor, 0, tso, gso), true);
    stats.drops_no_rx_desc += 1;
    return 0;
  }
  for (uint32_t k = 0; k < total; ++k) {
    const auto xr = desc_load(C.rx + rc++);
    const bool x_present = xr.vlan_present || t.vlan_insert;  // :320-322
    // base segment = header || chunk k (or the whole packet)
    uint64_t src_a = t.buffer_address, src_b = 0;
    uint32_t len_a, len_b = 0;
    if (d.segmented) {
      len_a = d.H;
      src_b = t.buffer_address + d.H + (uint64_t) k * t.mss;
      len_b = ps.chunk_len(k);
    } else {
      len_a = (uint32_t) L;
    }
    const uint64_t base_len = (uint64_t) len_a + len_b;
    // :324-331 VLAN insert, :389-395 strip
    uint64_t size = base_len + (t.vlan_insert ? 4 : 0);
    const bool has_vlan = t.vlan_insert || x_present;
    const bool strip = xr.vlan_strip && has_vlan && size >= 4;
    if (strip) size -= 4;
    const bool prefix = t.vlan_insert && !strip;
    const bool strip_base = strip && !t.vlan_insert;  // the base segment loses its first 4 bytes
    // :397-414 buffer too small
    if (xr.buffer_length < size) {
      sink.tx(make_tx<Comp>(qid, t, kSuccess, total, tso, gso), false);
      Comp e = make_completion<Comp>(qid, xr.descriptor_index, kBufferTooSmall);
      e.vlan_stripped = xr.vlan_strip && has_vlan;
      if (e.vlan_stripped) e.vlan_tag = t.vlan_insert ? t.vlan_tag : xr.vlan_tag;
      sink.rx(e, (const Write*) nullptr);
      stats.drops_buffer_small += 1;
      return rc - rc0;
    }
    // :416-426 DMA write
    if (!dma_ok(C.mem_size, xr.buffer_address, size) || !write_allowed(C, xr.buffer_address, size)) {
      sink.tx(make_tx<Comp>(qid, t, kFault, total, tso, gso), false);
      sink.rx(make_completion<Comp>(qid, xr.descriptor_index, kFault), (const Write*) nullptr);
      return rc - rc0;
    }
    Write w;
    w.dst = xr.buffer_address;
    w.prefix = 0;
    w.prefix_len = 0;
    if (prefix) {
      const uint32_t tag = t.vlan_tag;
      w.prefix = 0x81u | (0x00u << 8) | (((tag >> 8) & 0xFFu) << 16) | ((tag & 0xFFu) << 24);
      w.prefix_len = 4;
    }
    if (strip_base) {  // drop the first 4 bytes of header || chunk
      const uint32_t from_a = len_a < 4 ? len_a : 4u;
      src_a += from_a;
      len_a -= from_a;
      src_b += 4 - from_a;
      len_b -= 4 - from_a;
    }
    w.src_a = src_a;
    w.len_a = len_a;
    w.src_b = src_b;
    w.len_b = len_b;

    Comp e = make_completion<Comp>(qid, xr.descriptor_index, kSuccess);
    e.gro_aggregated = xr.gro_enabled;
    if (e.gro_aggregated) stats.rx_gro_aggregated += 1;
    // :434-447 RX checksum verify of the delivered bytes
    bool deferred = false;
    if (xr.checksum_offload && (uint32_t) xr.checksum != 0u && C.late) {
      // (its sum is that of the bytes w writes: the delivery's)
      e.checksum_verified = true;
      stats.rx_checksum_verified += 1;
      deferred = true;
    } else if (xr.checksum_offload && (uint32_t) xr.checksum != 0u) {
      e.checksum_verified = true;
      stats.rx_checksum_verified += 1;
      uint32_t first4, rest;
      ps.segment(k, first4, rest);
      uint32_t sum = strip_base ? rest : add1c(first4, rest);
      if (prefix) sum = add1c(add1c(0x8100u, t.vlan_tag), sum);
      if ((~sum & 0xFFFFu) != 0) {
        e.status = kChecksumError;
        sink.rx(e, &w);
        sink.tx(make_tx<Comp>(qid, t, kSuccess, total, tso, gso), false);
        stats.drops_checksum += 1;
        return rc - rc0;
      }
    }
    e.vlan_stripped = xr.vlan_strip && has_vlan;
    if (e.vlan_stripped) {
      e.vlan_tag = t.vlan_insert ? t.vlan_tag : xr.vlan_tag;
      stats.rx_vlan_strips += 1;
    }
    if (deferred)
      sink_rx_late(sink, e, &w,
                   kLateDeferred | (strip_base ? kLateStripBase : 0u) | (t.vlan_insert ? kLateVlanInsert : 0u), 0);
    else
      sink.rx(e, &w);
    stats.rx_packets += 1;
    stats.rx_bytes += size;
  }
  // :280-301 finalize_tx_success
  sink.tx(make_tx<Comp>(qid, t, kSuccess, total, tso, gso), true);
  stats.tx_packets += total;
  stats.tx_bytes += L;
  if (tso) stats.tx_tso_segments += total;
  if (gso) stats.tx_gso_segments += total;
  if (t.vlan_insert) stats.tx_vlan_insertions += total;
  return rc - rc0;
}

}  // namespace nicqp
