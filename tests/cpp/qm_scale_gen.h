// qm_scale_gen.h — the input of the 16-queue-pair QueueManager fixture at scale
// (tests/golden/qm16_scale.json), made from a seed on both sides: by
// oracle/gen_golden.cpp against the compiled reference QueueManager
// (src/queue_manager.cpp:54-78 over src/queue_pair.cpp:67-460), and by
// tests/cpp/qm_test.cpp (`scale` mode) for nic::BatchedQueueManager.  The
// fixture is too large to commit as bytes (≈ 70 K descriptors, a ≈ 190 MB
// memory image), so it holds the seed and digests: per round and queue pair
// the FNV-1a-64 of the TX and RX completions in posting order, the MSI-X
// vector sequence's FNV, the stats, and the memory image's FNV.
//
// TEST INFRASTRUCTURE ONLY.  Plain data generation; uses the nic:: descriptor
// types of whichever side includes it (the reference's or this build's drop-in
// declarations, which are layout-identical).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace qm_scale {

struct Rng {
  std::uint64_t s;
  std::uint64_t next() {  // splitmix64
    std::uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  std::uint32_t u32() { return static_cast<std::uint32_t>(next() >> 32); }
  std::uint32_t below(std::uint32_t n) { return static_cast<std::uint32_t>((next() >> 32) % n); }
  std::uint8_t byte() { return static_cast<std::uint8_t>(next() >> 56); }
};

// ones'-complement sum of big-endian 16-bit words (odd tail byte high), folded
inline std::uint32_t fold_sum(const std::uint8_t* p, std::size_t n) {
  std::uint64_t s = 0;
  for (std::size_t i = 0; i + 1 < n; i += 2) s += (std::uint32_t{p[i]} << 8) | p[i + 1];
  if (n & 1) s += std::uint32_t{p[n - 1]} << 8;
  while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
  return static_cast<std::uint32_t>(s);
}

// compute_checksum's value (src/checksum.cpp:10-34: the complement of the sum)
inline std::uint16_t checksum(const std::uint8_t* p, std::size_t n) {
  return static_cast<std::uint16_t>(~fold_sum(p, n) & 0xFFFF);
}

inline std::uint64_t fnv(std::uint64_t h, const void* p, std::size_t n) {
  const auto* b = static_cast<const std::uint8_t*>(p);
  for (std::size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
  return h;
}
constexpr std::uint64_t kFnv0 = 0xcbf29ce484222325ull;

// one completion's 12 recorded fields, each as a little-endian u64
template <class C>
std::uint64_t fnv_completion(std::uint64_t h, const C& c) {
  const std::uint64_t f[12] = {c.queue_id, c.descriptor_index, static_cast<std::uint64_t>(c.status),
                               c.checksum_offloaded, c.checksum_verified, c.tso_performed, c.gso_performed,
                               c.vlan_inserted, c.vlan_stripped, c.gro_aggregated, c.segments_produced, c.vlan_tag};
  return fnv(h, f, sizeof f);
}

template <class Tx, class Rx>
struct Case {
  std::size_t Q = 16, R = 2;
  std::uint32_t max_mtu = 9000;
  std::vector<std::uint8_t> weights;
  std::vector<std::vector<std::size_t>> ntx, nrx;  // [round][queue]
  std::vector<std::vector<std::vector<Tx>>> tx;    // [round][queue]
  std::vector<std::vector<std::vector<Rx>>> rx;
  std::vector<std::uint8_t> image;
  bool etx(std::size_t q) const { return q % 2 == 0; }
  bool erx(std::size_t q) const { return q % 3 != 2; }
};

// 16 queue pairs, two rounds.  Round 0: 4096 TX descriptors per queue pair
// (queue pair 5 idle, so the scheduler skips it), RX rings of 4096-4696 buffers
// (queue pair 7 runs dry at 2000); round 1: 256 + 37 q each, 300 more buffers.
// Frames in C3-like proportions (64 / 576 / 1518 B) plus tiny, 9000 B TSO/GSO
// and over-MTU ones; two in three with offload on, one in six with a wrong
// checksum, RX buffers small, 1600 B or 9224 B; every queue pair's TX and RX
// buffers in regions of their own (the queues are disjoint).
template <class Tx, class Rx, class ModeNone, class ModeL3, class ModeL4>
Case<Tx, Rx> make_case(std::uint64_t seed, ModeNone none, ModeL3 l3, ModeL4 l4) {
  Case<Tx, Rx> c;
  Rng r{seed};
  const std::size_t Q = c.Q;
  c.weights = {1, 2, 3, 1, 4, 1, 2, 1, 3, 1, 1, 2, 5, 1, 2, 1};
  c.ntx.assign(c.R, std::vector<std::size_t>(Q));
  c.nrx.assign(c.R, std::vector<std::size_t>(Q));
  for (std::size_t q = 0; q < Q; ++q) {
    c.ntx[0][q] = q == 5 ? 0 : 4096;
    c.nrx[0][q] = q == 7 ? 2000 : 4096 + 300 * (q % 3);
    c.ntx[1][q] = 256 + 37 * q;
    c.nrx[1][q] = 300;
  }
  c.tx.assign(c.R, std::vector<std::vector<Tx>>(Q));
  c.rx.assign(c.R, std::vector<std::vector<Rx>>(Q));
  auto& img = c.image;
  for (std::size_t k = 0; k < c.R; ++k)
    for (std::size_t q = 0; q < Q; ++q) {
      for (std::size_t i = 0; i < c.ntx[k][q]; ++i) {
        const std::uint32_t pick = r.below(32);
        std::size_t L = pick < 14 ? 64 : pick < 22 ? 576 : pick < 28 ? 1518 : pick == 28 ? r.below(60)
                        : pick == 29 ? 9000 : pick == 30 ? 9001 + r.below(200) : 64 + r.below(1436);
        img.resize(img.size() + r.below(8));
        const std::size_t at = img.size();
        img.resize(at + L);
        std::uint8_t* f = img.data() + at;
        for (std::size_t b = 0; b < L; ++b) f[b] = r.byte();
        if (L >= 34) {  // Ethernet + IPv4 (protocol TCP or UDP)
          f[12] = 0x08; f[13] = 0x00; f[14] = 0x45; f[15] = 0;
          f[23] = r.below(2) ? 6 : 17;
        }
        if (L >= 64 && r.below(4) != 0) {  // balanced: the whole frame sums to 0xFFFF
          f[40] = f[41] = 0;
          const std::uint32_t w = 0xFFFF - fold_sum(f, L);
          f[40] = static_cast<std::uint8_t>(w >> 8);
          f[41] = static_cast<std::uint8_t>(w);
        }
        Tx t{};
        t.buffer_address = at;
        t.length = static_cast<std::uint32_t>(L);
        t.descriptor_index = static_cast<std::uint16_t>(i);
        const std::uint32_t cm = r.below(5);
        t.checksum = cm < 2 ? none : (cm < 4 ? l4 : l3);
        t.checksum_offload = r.below(3) != 0;
        const std::uint16_t good = checksum(f, L);
        t.checksum_value = r.below(6) == 0 ? static_cast<std::uint16_t>(good ^ (1u + r.below(0xFFFE))) : good;
        if (L > 1518 && r.below(3) != 0) {
          (r.below(2) ? t.tso_enabled : t.gso_enabled) = true;
          t.mss = r.below(10) == 0 ? static_cast<std::uint16_t>(1 + r.below(30)) : static_cast<std::uint16_t>(1448);
          t.header_length = 54;
        }
        if (r.below(8) == 0) { t.vlan_insert = true; t.vlan_tag = static_cast<std::uint16_t>(r.u32()); }
        c.tx[k][q].push_back(t);
      }
      img.resize((img.size() + 63) & ~std::size_t{63});
      for (std::size_t j = 0; j < c.nrx[k][q]; ++j) {
        const std::uint32_t bp = r.below(16);
        const std::uint32_t blen = bp == 0 ? 64 : bp == 1 ? r.below(1600) : bp == 2 ? 9224 : 1600;
        img.resize(img.size() + r.below(4));
        Rx x{};
        x.buffer_address = img.size();
        x.buffer_length = blen;
        img.resize(img.size() + blen);
        x.descriptor_index = static_cast<std::uint16_t>(j);
        x.checksum_offload = r.below(4) == 0;
        const std::uint32_t cm = r.below(5);
        x.checksum = cm == 0 ? none : (cm < 3 ? l4 : l3);
        x.vlan_strip = r.below(3) == 0;
        x.vlan_present = r.below(4) == 0;
        x.vlan_tag = static_cast<std::uint16_t>(r.u32());
        x.gro_enabled = r.below(5) == 0;
        c.rx[k][q].push_back(x);
      }
    }
  img.resize(img.size() + 64);
  return c;
}

}  // namespace qm_scale
