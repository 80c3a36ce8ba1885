// gen_golden.cpp — writes tests/golden/ from the COMPILED REFERENCE.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile (target `golden`) in the
// container where /root/reference exists: it links the reference's own
// src/checksum.cpp, src/rss.cpp and the QueuePair pipeline sources by path
// (nothing is copied into this repo) and records what they compute.  The
// outputs are plain data (JSON + little-endian .bin arrays); the GPU box only
// ever sees those files.
//
// Expected values come from:
//   nic::compute_checksum           src/checksum.cpp:10-34
//   nic::RssEngine::hash/select     src/rss.cpp:43-61 (+ stats, :45, :56-58)
//   nic::QueuePair::process_once    src/queue_pair.cpp:67-460 (statuses, TSO)
// The tuple fed to select_queue is extracted with oracle_extract_tuple (the
// build's own parser definition — the reference has none).

#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "nic/checksum.h"
#include "nic/completion_queue.h"
#include "nic/doorbell.h"
#include "nic/dma_engine.h"
#include "nic/interrupt_dispatcher.h"
#include "nic/msix.h"
#include "nic/queue_manager.h"
#include "nic/queue_pair.h"
#include "nic/rss.h"
#include "nic/simple_host_memory.h"
#include "nic/tx_rx.h"
#include "oracle.h"
#include "../tests/cpp/qm_scale_gen.h"
#include "../tests/cpp/fault_model.h"

using namespace nic;

namespace {

std::string g_out = "tests/golden";

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

std::uint16_t ref_csum(const std::uint8_t* p, std::size_t n) {
  return nic::compute_checksum(std::span<const std::byte>(reinterpret_cast<const std::byte*>(p), n));
}

std::string hex(const std::uint8_t* p, std::size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (std::size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

template <class T>
void write_bin(const std::string& name, const std::vector<T>& v) {
  std::ofstream f(g_out + "/" + name, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(T)));
}

template <class T>
std::string json_arr(const std::vector<T>& v) {
  std::ostringstream o;
  o << "[";
  for (std::size_t i = 0; i < v.size(); ++i) o << (i ? "," : "") << static_cast<std::uint64_t>(v[i]);
  o << "]";
  return o.str();
}

const std::vector<std::uint8_t> kMsKey = {
    // tests/tutorial_lesson8_test.cpp:56-60 (the Microsoft RSS verification key)
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa,
};

std::vector<std::uint8_t> default_key() {
  std::vector<std::uint8_t> k(20);
  oracle_default_key(k.data());
  return k;
}

// ---------------------------------------------------------------- checksum --
void gen_checksum() {
  std::ostringstream js;
  js << "{\n \"source\": \"nic::compute_checksum, src/checksum.cpp:10-34 (compiled reference)\",\n";
  js << " \"cases\": [\n";
  std::vector<std::vector<std::uint8_t>> cases = {
      {},
      {0xFF, 0xFF, 0xFF, 0xFF},  // tests/coverage_test.cpp:53-56 (asserts 0)
      {0x01, 0x02, 0x03},        // coverage_test.cpp:60-62
      {0xFF, 0xFF, 0xFF},        // coverage_test.cpp:64-66
      {0xFF, 0xFF},              // tx_rx_test.cpp:855
      {0x00, 0x00, 0x00, 0x00},
      {0x00},
      {0x80},
      {0xFF},
      {0x00, 0x01},
      {0xFF, 0xFE},
  };
  // tests/tx_rx_test.cpp:103-110 make_payload(i & 0xFF) at the lengths the tests use.
  for (std::size_t L : {1, 2, 3, 6, 8, 10, 12, 16, 63, 64, 65, 576, 1514, 1518, 9000, 9216}) {
    std::vector<std::uint8_t> v(L);
    for (std::size_t i = 0; i < L; ++i) v[i] = static_cast<std::uint8_t>(i & 0xFF);
    cases.push_back(v);
  }
  // all-0xFF buffers: the sum is a multiple of 0xFFFF (checks the zero/0xFFFF corner)
  for (std::size_t L : {2, 4, 6, 7, 130, 1518}) cases.emplace_back(L, 0xFF);
  for (std::size_t i = 0; i < cases.size(); ++i) {
    const auto& c = cases[i];
    js << "  {\"hex\": \"" << hex(c.data(), c.size()) << "\", \"len\": " << c.size()
       << ", \"csum\": " << ref_csum(c.data(), c.size()) << "}" << (i + 1 < cases.size() ? "," : "")
       << "\n";
  }
  js << " ]\n}\n";
  std::ofstream(g_out + "/checksum_kat.json") << js.str();

  // Length/alignment sweep: every length 0..300, then random lengths up to 9216,
  // placed at random (not only 16-B aligned) offsets with random gap bytes.
  Rng r{1};
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  std::vector<std::uint16_t> csum;
  std::vector<std::size_t> lens;
  for (std::size_t L = 0; L <= 300; ++L) lens.push_back(L);
  for (int i = 0; i < 64; ++i) lens.push_back(r.below(9217));
  for (std::size_t L : {1518, 9000, 9216, 9215, 4095, 4096, 4097}) lens.push_back(L);
  for (std::size_t L : lens) {
    std::size_t gap = r.below(4) == 0 ? r.below(16) : (16 - frames.size() % 16) % 16;
    for (std::size_t g = 0; g < gap; ++g) frames.push_back(r.byte());
    std::uint64_t off = frames.size();
    int pattern = static_cast<int>(r.below(4));
    for (std::size_t i = 0; i < L; ++i) {
      std::uint8_t b = pattern == 0 ? 0xFF : pattern == 1 ? static_cast<std::uint8_t>(i) : r.byte();
      frames.push_back(b);
    }
    desc.push_back(off | (static_cast<std::uint64_t>(L) << 40));
    csum.push_back(ref_csum(frames.data() + off, L));
  }
  for (int g = 0; g < 32; ++g) frames.push_back(r.byte());
  while (frames.size() % 16) frames.push_back(0);
  write_bin("checksum_sweep.frames.bin", frames);
  write_bin("checksum_sweep.desc.bin", desc);
  write_bin("checksum_sweep.csum.bin", csum);
}

// --------------------------------------------------------------------- RSS --
struct RssCase {
  std::vector<std::uint8_t> key;  // empty = engine default
  std::vector<std::uint16_t> table;
  std::vector<std::vector<std::uint8_t>> data;
  std::string note;
};

std::vector<std::uint8_t> tuple12(std::uint32_t s, std::uint32_t d, std::uint16_t sp, std::uint16_t dp) {
  return {static_cast<std::uint8_t>(s >> 24), static_cast<std::uint8_t>(s >> 16),
          static_cast<std::uint8_t>(s >> 8),  static_cast<std::uint8_t>(s),
          static_cast<std::uint8_t>(d >> 24), static_cast<std::uint8_t>(d >> 16),
          static_cast<std::uint8_t>(d >> 8),  static_cast<std::uint8_t>(d),
          static_cast<std::uint8_t>(sp >> 8), static_cast<std::uint8_t>(sp),
          static_cast<std::uint8_t>(dp >> 8), static_cast<std::uint8_t>(dp)};
}

std::uint32_t ip(int a, int b, int c, int d) {
  return (static_cast<std::uint32_t>(a) << 24) | (static_cast<std::uint32_t>(b) << 16) |
         (static_cast<std::uint32_t>(c) << 8) | static_cast<std::uint32_t>(d);
}

void gen_rss() {
  std::vector<RssCase> cases;
  // tests/queue_manager_rss_test.cpp:263-285 / :287-313 / :34-50 (default 20-B key)
  cases.push_back({{}, {0, 1, 2, 3}, {{0xAA, 0xBB, 0xCC, 0xDD}, {0x10, 0x20, 0x30, 0x40}, {0x01, 0x00, 0x00, 0x01}}, "queue_manager_rss_test.cpp:263-285"});
  cases.push_back({{}, {0, 1}, {{0x00, 0x00, 0x00, 0x01}, {0xFF, 0xEE, 0xDD, 0xCC}, {0x12, 0x34, 0x56, 0x78}}, "queue_manager_rss_test.cpp:287-313"});
  cases.push_back({{}, {2, 2, 2, 2}, {{0x01, 0x02, 0x03, 0x04}}, "queue_manager_rss_test.cpp:34-50"});
  cases.push_back({{}, {}, {{}}, "queue_manager_rss_test.cpp:315-330 (empty data, default table)"});
  // tests/tutorial_lesson8_test.cpp:94-160 (MS key, 8-entry table)
  cases.push_back({kMsKey, {0, 1, 2, 3, 0, 1, 2, 3},
                   {tuple12(0xC0A80164, 0xC0A80101, 8080, 80), tuple12(0xC0A80101, 0xC0A80164, 80, 8080)},
                   "tutorial_lesson8_test.cpp:94-160"});
  // docs/users_guide.md:2000-2020 (key = forty 0x6D)
  cases.push_back({std::vector<std::uint8_t>(40, 0x6D), {0, 1, 2, 3},
                   {tuple12(0xC0A80164, 0xC0A80101, 8080, 80)}, "users_guide.md:2000-2020"});
  // Microsoft RSS verification suite, IPv4 rows (TCP 12-B tuple and IP-only 8-B tuple)
  {
    RssCase c{kMsKey, {0, 1, 2, 3}, {}, "Microsoft RSS verification suite (IPv4)"};
    struct Row { std::uint32_t s, d; std::uint16_t sp, dp; };
    Row rows[] = {{ip(66, 9, 149, 187), ip(161, 142, 100, 80), 2794, 1766},
                  {ip(199, 92, 111, 2), ip(65, 69, 140, 83), 14230, 4739},
                  {ip(24, 19, 198, 95), ip(12, 22, 207, 184), 12898, 38024},
                  {ip(38, 27, 205, 30), ip(209, 142, 163, 6), 48228, 2217},
                  {ip(153, 39, 163, 191), ip(202, 188, 127, 2), 44251, 1303}};
    for (auto& w : rows) {
      auto t = tuple12(w.s, w.d, w.sp, w.dp);
      c.data.push_back(t);
      c.data.emplace_back(t.begin(), t.begin() + 8);
    }
    cases.push_back(c);
  }
  // Key-wrap: 36-B inputs i*7+1 against the 20-B default key (wraps) and the MS key.
  {
    std::vector<std::uint8_t> d(36);
    for (int i = 0; i < 36; ++i) d[i] = static_cast<std::uint8_t>(i * 7 + 1);
    cases.push_back({{}, {0, 1, 2}, {d}, "key wrap, default 20-B key"});
    cases.push_back({kMsKey, {0, 1, 2}, {d}, "36-B input, MS key"});
  }
  // Random data of many lengths x several keys (incl. short keys: 1, 4, 5 B) and table sizes.
  {
    Rng r{7};
    std::vector<std::vector<std::uint8_t>> keys = {{}, kMsKey, {0xA5}, {1, 2, 3, 4}, {9, 8, 7, 6, 5}, std::vector<std::uint8_t>(52, 0x3C)};
    for (std::size_t ki = 0; ki < keys.size(); ++ki) {
      std::vector<std::uint16_t> table(1 + r.below(300));
      for (auto& e : table) e = static_cast<std::uint16_t>(r.below(65536));
      RssCase c{keys[ki], table, {}, "random data"};
      for (int j = 0; j < 40; ++j) {
        std::vector<std::uint8_t> d(r.below(65));
        for (auto& b : d) b = r.byte();
        c.data.push_back(d);
      }
      cases.push_back(c);
    }
  }

  std::ostringstream js;
  js << "{\n \"source\": \"nic::RssEngine::hash/select_queue/stats, src/rss.cpp:17-114 (compiled reference)\",\n";
  js << " \"default_key\": \"" << hex(default_key().data(), 20) << "\",\n \"cases\": [\n";
  for (std::size_t ci = 0; ci < cases.size(); ++ci) {
    auto& c = cases[ci];
    RssConfig cfg;
    cfg.key = c.key;
    cfg.table = c.table;
    RssEngine eng{cfg};  // ctor applies ensure_defaults (rss.cpp:22-25, 96-108)
    std::vector<std::uint32_t> hashes;
    std::vector<std::uint16_t> queues;
    std::vector<std::uint32_t> tidx;
    for (auto& d : c.data) {
      std::uint32_t h = eng.hash(std::span<const std::uint8_t>(d));
      auto q = eng.select_queue(std::span<const std::uint8_t>(d));
      hashes.push_back(h);
      queues.push_back(*q);
      tidx.push_back(static_cast<std::uint32_t>(h % eng.config().table.size()));
    }
    js << "  {\"note\": \"" << c.note << "\", \"key\": \"" << hex(eng.config().key.data(), eng.config().key.size())
       << "\", \"table\": " << json_arr(eng.config().table) << ",\n   \"data\": [";
    for (std::size_t j = 0; j < c.data.size(); ++j) js << (j ? "," : "") << "\"" << hex(c.data[j].data(), c.data[j].size()) << "\"";
    js << "],\n   \"hash\": " << json_arr(hashes) << ", \"queue\": " << json_arr(queues)
       << ", \"tidx\": " << json_arr(tidx) << ",\n   \"stats_hashes\": " << eng.stats().hashes
       << ", \"stats_queue_hits\": " << json_arr(eng.stats().queue_hits) << "}"
       << (ci + 1 < cases.size() ? "," : "") << "\n";
  }
  js << " ]\n}\n";
  std::ofstream(g_out + "/rss_kat.json") << js.str();

  // queue_hits guard (rss.cpp:56-58): set_table to a larger table after construction.
  {
    RssEngine eng;  // default: 128-entry table, queue_hits sized 128
    std::vector<std::uint16_t> big(200);
    for (std::size_t i = 0; i < big.size(); ++i) big[i] = static_cast<std::uint16_t>(i % 5);
    eng.set_table(big);
    Rng r{11};
    std::vector<std::uint32_t> tidx;
    std::ostringstream data;
    for (int j = 0; j < 64; ++j) {
      std::vector<std::uint8_t> d(12);
      for (auto& b : d) b = r.byte();
      auto q = eng.select_queue(std::span<const std::uint8_t>(d));
      (void) q;
      tidx.push_back(eng.hash(std::span<const std::uint8_t>(d)) % 200);
      data << (j ? "," : "") << "\"" << hex(d.data(), d.size()) << "\"";
    }
    std::ofstream(g_out + "/rss_hits_guard.json")
        << "{\"note\": \"set_table(200) after default ctor; queue_hits stays 128 (rss.cpp:56-58,107)\",\n"
        << " \"table\": " << json_arr(big) << ",\n \"data\": [" << data.str() << "],\n \"tidx\": " << json_arr(tidx)
        << ",\n \"stats_hashes\": " << eng.stats().hashes << ", \"stats_queue_hits\": " << json_arr(eng.stats().queue_hits) << "}\n";
  }
}

// ------------------------------------------------------------ frame builder --
// Eth/IPv4/TCP|UDP and IPv6 frames laid out as src/packet_generator.cpp:46-166;
// IPv4 header checksum and L4 pseudo-header checksums as :200-305, 342-360.
std::uint16_t inet_sum_be(const std::uint8_t* p, std::size_t n, std::uint32_t sum = 0) {
  for (std::size_t i = 0; i < n; i += 2) {
    std::uint32_t w = static_cast<std::uint32_t>(p[i]) << 8;
    if (i + 1 < n) w |= p[i + 1];
    sum += w;
  }
  while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
  return static_cast<std::uint16_t>(sum);
}

struct FrameSpec {
  int l3 = 4;          // 4, 6 or 0 (ARP)
  int proto = 6;       // 6 TCP, 17 UDP, other
  int vlan_tags = 0;   // 0..2
  int ihl = 5;
  bool frag = false;
  std::size_t total = 64;  // frame length (may truncate headers)
  bool balance = true;     // adjust src-MAC bytes 10..11 so compute_checksum(frame) == 0
};

std::vector<std::uint8_t> build_frame(Rng& r, const FrameSpec& s) {
  std::vector<std::uint8_t> f;
  auto put16 = [&](unsigned v) { f.push_back(static_cast<std::uint8_t>(v >> 8)); f.push_back(static_cast<std::uint8_t>(v)); };
  for (int i = 0; i < 12; ++i) f.push_back(r.byte());  // dst + src MAC
  unsigned et = s.l3 == 4 ? 0x0800 : s.l3 == 6 ? 0x86DD : 0x0806;
  if (s.vlan_tags == 2) { put16(0x88A8); put16(r.below(4096)); put16(0x8100); put16(r.below(4096)); }
  if (s.vlan_tags == 1) { put16(0x8100); put16(r.below(4096)); }
  put16(et);
  std::size_t l3 = f.size();
  std::size_t l4 = l3;
  if (s.l3 == 4) {
    f.push_back(static_cast<std::uint8_t>(0x40 | s.ihl));
    f.push_back(0);
    put16(0);  // total length, patched below
    put16(r.below(65536));
    put16(s.frag ? (r.below(2) ? 0x2000 : (0x4000 | (1 + r.below(100)))) : 0x4000);
    f.push_back(64);
    f.push_back(static_cast<std::uint8_t>(s.proto));
    put16(0);
    for (int i = 0; i < 8; ++i) f.push_back(r.byte());
    for (int i = 20; i < s.ihl * 4; ++i) f.push_back(1);  // NOP options
    l4 = f.size();
  } else if (s.l3 == 6) {
    f.push_back(0x60); f.push_back(0); put16(r.below(65536));
    put16(0);  // payload length
    f.push_back(static_cast<std::uint8_t>(s.proto));
    f.push_back(64);
    for (int i = 0; i < 32; ++i) f.push_back(r.byte());
    l4 = f.size();
  } else {
    for (int i = 0; i < 28; ++i) f.push_back(r.byte());  // ARP body
    l4 = f.size();
  }
  if (s.l3 != 0) {
    put16(1024 + r.below(64512));
    put16(1 + r.below(65535));
    if (s.proto == 6) {
      for (int i = 0; i < 8; ++i) f.push_back(r.byte());
      f.push_back(0x50); f.push_back(0x18); put16(r.below(65536)); put16(0); put16(0);
    } else if (s.proto == 17) {
      put16(0); put16(0);
    }
  }
  while (f.size() < s.total) f.push_back(r.byte());
  f.resize(s.total);
  // Patch lengths and checksums when the headers are complete.
  if (s.l3 == 4 && f.size() >= l3 + 20) {
    std::size_t iplen = f.size() - l3;
    f[l3 + 2] = static_cast<std::uint8_t>(iplen >> 8); f[l3 + 3] = static_cast<std::uint8_t>(iplen);
    if (f.size() >= l3 + static_cast<std::size_t>(s.ihl) * 4) {
      std::uint16_t c = static_cast<std::uint16_t>(~inet_sum_be(&f[l3], static_cast<std::size_t>(s.ihl) * 4));
      f[l3 + 10] = static_cast<std::uint8_t>(c >> 8); f[l3 + 11] = static_cast<std::uint8_t>(c);
    }
  }
  if (s.l3 == 6 && f.size() >= l3 + 40) {
    std::size_t pl = f.size() - l3 - 40;
    f[l3 + 4] = static_cast<std::uint8_t>(pl >> 8); f[l3 + 5] = static_cast<std::uint8_t>(pl);
  }
  bool l4full = (s.proto == 6 && f.size() >= l4 + 20) || (s.proto == 17 && f.size() >= l4 + 8);
  if (s.l3 != 0 && l4full && !s.frag) {
    std::size_t seglen = f.size() - l4;
    if (s.proto == 17) { f[l4 + 4] = static_cast<std::uint8_t>(seglen >> 8); f[l4 + 5] = static_cast<std::uint8_t>(seglen); }
    std::uint8_t ph[40];
    std::size_t phl;
    if (s.l3 == 4) {
      std::memcpy(ph, &f[l3 + 12], 8); ph[8] = 0; ph[9] = static_cast<std::uint8_t>(s.proto);
      ph[10] = static_cast<std::uint8_t>(seglen >> 8); ph[11] = static_cast<std::uint8_t>(seglen); phl = 12;
    } else {
      std::memcpy(ph, &f[l3 + 8], 32); ph[32] = 0; ph[33] = 0; ph[34] = static_cast<std::uint8_t>(seglen >> 8);
      ph[35] = static_cast<std::uint8_t>(seglen); ph[36] = 0; ph[37] = 0; ph[38] = 0; ph[39] = static_cast<std::uint8_t>(s.proto); phl = 40;
    }
    std::size_t co = l4 + (s.proto == 6 ? 16 : 6);
    std::uint32_t psum = inet_sum_be(ph, phl);
    std::uint16_t c = static_cast<std::uint16_t>(~inet_sum_be(&f[l4], seglen, psum));
    if (s.proto == 17 && c == 0) c = 0xFFFF;  // packet_generator.cpp:304
    f[co] = static_cast<std::uint8_t>(c >> 8); f[co + 1] = static_cast<std::uint8_t>(c);
  }
  if (s.balance && f.size() >= 12) {
    // Choose src-MAC bytes 10..11 so the whole-frame checksum (the RX verify of
    // queue_pair.cpp:437-438) is 0: the ones'-complement sum must be 0xFFFF.
    f[10] = 0; f[11] = 0;
    std::uint16_t rest = inet_sum_be(f.data(), f.size());
    std::uint16_t w = static_cast<std::uint16_t>(0xFFFF - rest);
    if (w == 0) w = 0xFFFF;  // 0xFFFF + x == x in ones' complement, keeps the total 0xFFFF
    if (rest == 0) w = 0xFFFF;
    f[10] = static_cast<std::uint8_t>(w >> 8); f[11] = static_cast<std::uint8_t>(w);
  }
  return f;
}

FrameSpec random_spec(Rng& r) {
  FrameSpec s;
  int kind = static_cast<int>(r.below(14));
  static const std::size_t sizes[] = {64, 64, 64, 64, 64, 64, 64, 576, 576, 576, 576, 1518};
  s.total = r.below(5) == 0 ? 14 + r.below(1600) : sizes[r.below(12)];
  if (r.below(40) == 0) s.total = 9000;
  if (r.below(40) == 0) s.total = 9216;
  switch (kind) {
    case 0: s.proto = 6; break;
    case 1: s.proto = 17; break;
    case 2: s.vlan_tags = 1; s.proto = 6; break;
    case 3: s.vlan_tags = 2; s.proto = 17; break;
    case 4: s.ihl = 6 + static_cast<int>(r.below(10)); s.proto = 6; s.vlan_tags = static_cast<int>(r.below(3)); break;
    case 5: s.frag = true; s.proto = 17; break;
    case 6: s.proto = 1; break;
    case 7: s.l3 = 6; s.proto = 6; break;
    case 8: s.l3 = 6; s.proto = 17; s.vlan_tags = static_cast<int>(r.below(3)); break;
    case 9: s.l3 = 6; s.proto = 58; break;
    case 10: s.l3 = 0; break;
    case 11: s.total = r.below(60); s.proto = r.below(2) ? 6 : 17; s.vlan_tags = static_cast<int>(r.below(2)); break;
    default: s.total = s.total > 200 ? s.total : 200; break;  // plain TCP, bigger
  }
  s.balance = r.below(10) != 0;
  return s;
}

// ----------------------------------------------------------------- RX mix --
void gen_rx_mix() {
  Rng r{42};
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  const int N = 3000;
  for (int i = 0; i < N; ++i) {
    FrameSpec s = random_spec(r);
    auto f = build_frame(r, s);
    std::size_t gap = r.below(8) == 0 ? r.below(16) : (16 - frames.size() % 16) % 16;
    for (std::size_t g = 0; g < gap; ++g) frames.push_back(r.byte());
    std::uint64_t off = frames.size();
    frames.insert(frames.end(), f.begin(), f.end());
    desc.push_back(off | (static_cast<std::uint64_t>(f.size()) << 40));
  }
  for (int g = 0; g < 32; ++g) frames.push_back(r.byte());
  while (frames.size() % 16) frames.push_back(0);
  write_bin("rx_mix.frames.bin", frames);
  write_bin("rx_mix.desc.bin", desc);

  std::vector<std::uint16_t> csum(N);
  for (int i = 0; i < N; ++i) {
    std::uint64_t off = desc[i] & ((1ull << 40) - 1);
    csum[i] = ref_csum(frames.data() + off, static_cast<std::size_t>(desc[i] >> 40));
  }
  write_bin("rx_mix.csum.bin", csum);

  struct Cfg { std::string name; std::vector<std::uint8_t> key; std::vector<std::uint16_t> table; int mode; int raw_off; int raw_len; };
  std::vector<std::uint16_t> t4(128), t16(128), t7(7);
  for (int i = 0; i < 128; ++i) { t4[i] = static_cast<std::uint16_t>(i % 4); t16[i] = static_cast<std::uint16_t>(i % 16); }
  for (int i = 0; i < 7; ++i) t7[i] = static_cast<std::uint16_t>(100 + i);
  std::vector<Cfg> cfgs = {
      {"ms_q4", kMsKey, t4, ORACLE_TUPLE_AUTO, 0, 0},
      {"ms_q16", kMsKey, t16, ORACLE_TUPLE_AUTO, 0, 0},
      {"default_key_t7", {}, t7, ORACLE_TUPLE_AUTO, 0, 0},
      {"default_engine", {}, {}, ORACLE_TUPLE_AUTO, 0, 0},
      {"raw26x36_default_key", {}, {0, 1, 2, 3}, ORACLE_TUPLE_RAW, 26, 36},
      {"raw0x64_ms", kMsKey, t16, ORACLE_TUPLE_RAW, 0, 64},
      {"raw30x12_key52", std::vector<std::uint8_t>(52, 0x3C), t7, ORACLE_TUPLE_RAW, 30, 12},
  };
  std::ostringstream js;
  js << "{\n \"source\": \"compute_checksum (src/checksum.cpp) + RssEngine::select_queue (src/rss.cpp) on oracle_extract_tuple\",\n";
  js << " \"n\": " << N << ",\n \"configs\": [\n";
  for (std::size_t ci = 0; ci < cfgs.size(); ++ci) {
    auto& c = cfgs[ci];
    RssConfig rc;
    rc.key = c.key;
    rc.table = c.table;
    RssEngine eng{rc};
    std::vector<std::uint32_t> hash(N), tidx(N);
    std::vector<std::uint16_t> queue(N);
    std::uint8_t tuple[64];
    for (int i = 0; i < N; ++i) {
      std::uint64_t off = desc[i] & ((1ull << 40) - 1);
      std::size_t len = static_cast<std::size_t>(desc[i] >> 40);
      std::size_t tl = oracle_extract_tuple(frames.data() + off, len, c.mode, static_cast<std::size_t>(c.raw_off),
                                            static_cast<std::size_t>(c.raw_len), tuple);
      std::span<const std::uint8_t> sp(tuple, tl);
      auto q = eng.select_queue(sp);
      queue[i] = *q;
      RssEngine probe{eng.config()};
      hash[i] = probe.hash(sp);
      tidx[i] = static_cast<std::uint32_t>(hash[i] % eng.config().table.size());
    }
    write_bin("rx_mix." + c.name + ".hash.bin", hash);
    write_bin("rx_mix." + c.name + ".queue.bin", queue);
    write_bin("rx_mix." + c.name + ".tidx.bin", tidx);
    js << "  {\"name\": \"" << c.name << "\", \"key\": \"" << hex(eng.config().key.data(), eng.config().key.size())
       << "\", \"table\": " << json_arr(eng.config().table) << ", \"mode\": " << c.mode << ", \"raw_off\": " << c.raw_off
       << ", \"raw_len\": " << c.raw_len << ",\n   \"stats_hashes\": " << eng.stats().hashes
       << ", \"stats_queue_hits\": " << json_arr(eng.stats().queue_hits) << "}" << (ci + 1 < cfgs.size() ? "," : "") << "\n";
  }
  js << " ]\n}\n";
  std::ofstream(g_out + "/rx_mix.json") << js.str();
}

// --------------------------------------------------------- QueuePair runs --
struct PipeResult {
  std::uint32_t tx_status = 0;
  std::uint16_t tx_segments = 0;
  std::vector<std::uint32_t> rx_status;
  std::vector<std::uint8_t> rx_verified;
  std::vector<std::uint16_t> seg_csum;  // compute_checksum of each delivered RX buffer
  std::vector<std::uint32_t> seg_len;
  std::uint64_t drops_checksum = 0;
  std::uint64_t rx_packets = 0;
};

// One TX descriptor through QueuePair::process_once with `nrx` RX descriptors.
PipeResult run_pipeline(const std::vector<std::uint8_t>& pkt, bool tso, std::uint16_t mss, std::uint16_t hdr,
                        bool rx_csum, ChecksumMode mode, std::size_t nrx) {
  const std::size_t slot = 9216 + 64;
  HostMemoryConfig mc{.size_bytes = slot * (nrx + 2), .page_size = 4096, .iommu_enabled = false};
  SimpleHostMemory mem{mc};
  DMAEngine dma{mem};
  QueuePairConfig qc{
      .queue_id = 0,
      .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = 4, .base_address = 0, .queue_id = 0, .host_backed = false},
      .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = 0, .queue_id = 0, .host_backed = false},
      .tx_completion = {.ring_size = 4, .queue_id = 0},
      .rx_completion = {.ring_size = nrx + 1, .queue_id = 0},
  };
  QueuePair qp{qc, dma};
  auto bytes = std::as_bytes(std::span<const std::uint8_t>(pkt));
  assert(mem.write(0, bytes).ok());
  TxDescriptor tx{.buffer_address = 0, .length = static_cast<std::uint32_t>(pkt.size()), .checksum = ChecksumMode::None,
                  .descriptor_index = 1, .checksum_value = 0, .tso_enabled = tso, .mss = mss, .header_length = hdr};
  std::vector<std::byte> tb(sizeof(TxDescriptor));
  std::memcpy(tb.data(), &tx, sizeof(tx));
  assert(qp.tx_ring().push_descriptor(tb).ok());
  for (std::size_t i = 0; i < nrx; ++i) {
    RxDescriptor rx{.buffer_address = slot * (i + 1), .buffer_length = static_cast<std::uint32_t>(slot), .checksum = mode,
                    .descriptor_index = static_cast<std::uint16_t>(10 + i), .checksum_offload = rx_csum};
    std::vector<std::byte> rb(sizeof(RxDescriptor));
    std::memcpy(rb.data(), &rx, sizeof(rx));
    assert(qp.rx_ring().push_descriptor(rb).ok());
  }
  qp.process_once();
  PipeResult res;
  auto tc = qp.tx_completion().poll_completion();
  if (tc) { res.tx_status = tc->status; res.tx_segments = tc->segments_produced; }
  std::size_t k = 0;
  while (auto rc = qp.rx_completion().poll_completion()) {
    res.rx_status.push_back(rc->status);
    res.rx_verified.push_back(rc->checksum_verified ? 1 : 0);
    ++k;
  }
  // Delivered segment bytes (only meaningful when every segment was delivered).
  std::size_t H = (tso && mss > 0 && pkt.size() > mss) ? std::min<std::size_t>(hdr, pkt.size()) : pkt.size();
  for (std::size_t i = 0; i < k; ++i) {
    std::size_t seglen;
    if (!(tso && mss > 0 && pkt.size() > mss) || H >= pkt.size()) seglen = pkt.size();
    else seglen = H + std::min<std::size_t>(mss, pkt.size() - H - i * mss);
    std::vector<std::byte> out(seglen);
    assert(mem.read(slot * (i + 1), out).ok());
    res.seg_csum.push_back(nic::compute_checksum(out));
    res.seg_len.push_back(static_cast<std::uint32_t>(seglen));
  }
  res.drops_checksum = qp.stats().drops_checksum;
  res.rx_packets = qp.stats().rx_packets;
  return res;
}

void gen_c1() {
  // C1: 64 x 64 B Eth/IPv4/UDP, RX checksum offload Layer4, RSS MS key + table {0,1,2,3}.
  Rng r{64};
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  std::vector<std::uint16_t> csum, queue;
  std::vector<std::uint32_t> hash, status;
  RssConfig rc;
  rc.key = kMsKey;
  rc.table = {0, 1, 2, 3};
  RssEngine eng{rc};
  for (int i = 0; i < 64; ++i) {
    FrameSpec s;
    s.proto = 17;
    s.total = 64;
    s.balance = (i % 8) != 3;  // some frames fail the whole-frame verify
    auto f = build_frame(r, s);
    desc.push_back(frames.size() | (64ull << 40));
    frames.insert(frames.end(), f.begin(), f.end());
    csum.push_back(ref_csum(f.data(), f.size()));
    std::uint8_t tuple[64];
    std::size_t tl = oracle_extract_tuple(f.data(), f.size(), ORACLE_TUPLE_AUTO, 0, 0, tuple);
    std::span<const std::uint8_t> sp(tuple, tl);
    auto q = eng.select_queue(sp);
    RssEngine probe{eng.config()};
    hash.push_back(probe.hash(sp));
    queue.push_back(*q);
    auto pr = run_pipeline(f, false, 0, 0, true, ChecksumMode::Layer4, 1);
    status.push_back(pr.rx_status.empty() ? 0xFFFFFFFFu : pr.rx_status[0]);
  }
  write_bin("c1_udp64.frames.bin", frames);
  write_bin("c1_udp64.desc.bin", desc);
  std::ofstream(g_out + "/c1_udp64.json")
      << "{\"note\": \"C1: 64 x 64 B UDP; csum = compute_checksum, rx_status = QueuePair RX completion status "
         "(queue_pair.cpp:434-447, Layer4 offload), queue = RssEngine::select_queue (MS key, table {0,1,2,3})\",\n"
      << " \"key\": \"" << hex(kMsKey.data(), kMsKey.size()) << "\", \"table\": [0,1,2,3],\n"
      << " \"csum\": " << json_arr(csum) << ",\n \"hash\": " << json_arr(hash) << ",\n \"queue\": " << json_arr(queue)
      << ",\n \"rx_status\": " << json_arr(status) << ",\n \"stats_hashes\": " << eng.stats().hashes
      << ", \"stats_queue_hits\": " << json_arr(eng.stats().queue_hits) << "}\n";
}

void gen_tso() {
  Rng r{9000};
  struct Case { std::size_t L; std::uint16_t H; std::uint16_t mss; bool tso; bool random_bytes; };
  std::vector<Case> cs = {
      {9000, 54, 1448, true, true},  {9000, 54, 1448, true, false}, {9000, 55, 1448, true, true},
      {9000, 54, 1447, true, true},  {9000, 53, 1001, true, true},  {9000, 0, 1448, true, true},
      {9000, 66, 8934, true, true},  {1518, 54, 1460, true, true},  {1518, 54, 100, true, true},
      {4000, 54, 63, true, true},    {3000, 41, 17, true, true},    {200, 20, 5, true, true},
      {12, 0, 6, true, false},       {10, 2, 3, true, false},       {100, 100, 10, true, true},
      {100, 101, 10, true, true},    {9000, 54, 100, true, true},   {9000, 54, 9001, true, true},
      {1518, 54, 1518, true, true},  {1518, 54, 0, true, true},     {700, 54, 1448, false, true},
      {9000, 14, 140, true, true},   {9000, 54, 141, true, true},
  };
  std::ostringstream js;
  js << "{\n \"source\": \"QueuePair::process_once TSO (src/queue_pair.cpp:195-460) + compute_checksum of each delivered RX segment\",\n \"cases\": [\n";
  std::vector<std::uint8_t> frames;
  for (std::size_t ci = 0; ci < cs.size(); ++ci) {
    auto& c = cs[ci];
    std::vector<std::uint8_t> pkt(c.L);
    if (c.random_bytes) {
      FrameSpec s; s.total = c.L; s.balance = false;
      pkt = build_frame(r, s);
    } else {
      for (std::size_t i = 0; i < c.L; ++i) pkt[i] = static_cast<std::uint8_t>(i & 0xFF);
    }
    std::uint64_t off = frames.size();
    frames.insert(frames.end(), pkt.begin(), pkt.end());
    while (frames.size() % 16) frames.push_back(r.byte());
    // Pass 1: no RX checksum offload -> every segment delivered; csum of each.
    auto all = run_pipeline(pkt, c.tso, c.mss, c.H, false, ChecksumMode::None, 70);
    // Pass 2: RX offload Layer4 -> statuses with the first-failure short-circuit.
    auto ver = run_pipeline(pkt, c.tso, c.mss, c.H, true, ChecksumMode::Layer4, 70);
    js << "  {\"off\": " << off << ", \"len\": " << c.L << ", \"hdr\": " << c.H << ", \"mss\": " << c.mss
       << ", \"tso\": " << (c.tso ? 1 : 0) << ",\n   \"tx_status\": " << all.tx_status << ", \"tx_segments\": " << all.tx_segments
       << ", \"seg_csum\": " << json_arr(all.seg_csum) << ", \"seg_len\": " << json_arr(all.seg_len)
       << ",\n   \"verify_tx_status\": " << ver.tx_status << ", \"verify_tx_segments\": " << ver.tx_segments
       << ", \"verify_rx_status\": " << json_arr(ver.rx_status) << ", \"verify_drops_checksum\": " << ver.drops_checksum
       << ", \"verify_rx_packets\": " << ver.rx_packets << "}" << (ci + 1 < cs.size() ? "," : "") << "\n";
  }
  js << " ]\n}\n";
  write_bin("tso.frames.bin", frames);
  std::ofstream(g_out + "/tso.json") << js.str();
}


// ------------------------------------------------- batched QueuePair runs --
// Randomised multi-descriptor batches through the reference QueuePair
// (queue_pair.cpp:67-460): every TX descriptor is processed by process_once in
// ring order against a shared RX ring, as the batched RX stage
// must reproduce.  Recorded: the initial host-memory image, the raw TX/RX
// descriptor PODs, every TX and RX CompletionEntry in posting order, the
// QueuePairStats, the RX descriptors consumed and an FNV-1a-64 of every RX
// buffer region after the run (what the DMA writes left there).
std::uint64_t fnv1a(const std::byte* p, std::size_t n) {
  std::uint64_t h = 0xcbf29ce484222325ull;
  for (std::size_t i = 0; i < n; ++i) { h ^= static_cast<std::uint8_t>(p[i]); h *= 0x100000001b3ull; }
  return h;
}

std::string completion_json(const CompletionEntry& e) {
  std::ostringstream o;
  o << "[" << e.queue_id << "," << e.descriptor_index << "," << e.status << "," << int(e.checksum_offloaded) << ","
    << int(e.checksum_verified) << "," << int(e.tso_performed) << "," << int(e.gso_performed) << ","
    << int(e.vlan_inserted) << "," << int(e.vlan_stripped) << "," << int(e.gro_aggregated) << ","
    << e.segments_produced << "," << e.vlan_tag << "]";
  return o.str();
}

// SimpleHostMemory that records every successful write in order: the RX
// segment DMA writes of QueuePair::handle_rx_segment (:416-426), i.e. each
// delivered frame's bytes as written, before any later write lands on them.
class RecordingMemory final : public HostMemory {
public:
  explicit RecordingMemory(HostMemoryConfig c, SimpleHostMemory::AddressTranslator tr = {},
                           SimpleHostMemory::FaultInjector fi = {})
      : mem_(c, std::move(tr), std::move(fi)) {}
  HostMemoryConfig config() const noexcept override { return mem_.config(); }
  HostMemoryResult translate(HostAddress a, std::size_t n, HostMemoryView& v) override { return mem_.translate(a, n, v); }
  HostMemoryResult translate_const(HostAddress a, std::size_t n, ConstHostMemoryView& v) const override {
    return mem_.translate_const(a, n, v);
  }
  HostMemoryResult read(HostAddress a, std::span<std::byte> b) const override { return mem_.read(a, b); }
  HostMemoryResult write(HostAddress a, std::span<const std::byte> d) override {
    HostMemoryResult r = mem_.write(a, d);
    if (r.ok() && recording) {
      const auto* p = reinterpret_cast<const std::uint8_t*>(d.data());
      writes.emplace_back(p, p + d.size());
    }
    return r;
  }
  bool recording = false;
  std::vector<std::vector<std::uint8_t>> writes;

private:
  SimpleHostMemory mem_;
};

// The reference QueuePair over one batch and the fixture it leaves (shared by
// the plain, fault and ring cases).  ring_tx_at / ring_rx_at (not ~0): the
// rings are host-backed at those addresses (DescriptorRing pushes and pops by
// DMA, descriptor_ring.cpp:48-110) and the saved image holds them as pushed.
void emit_qp_case(const std::string& name, const std::vector<TxDescriptor>& txs,
                  const std::vector<RxDescriptor>& rxs, std::vector<std::uint8_t> image, std::size_t mem_size,
                  std::size_t tx_end, int faults, std::uint64_t ring_tx_at = ~0ull, std::uint64_t ring_rx_at = ~0ull) {
  const std::size_t ntx = txs.size(), nrx = rxs.size();
  const bool rings = ring_tx_at != ~0ull;
  HostMemoryConfig mc{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = faults == faultfx::kIommu};
  faultfx::Model fm;
  fm.kind = static_cast<faultfx::Kind>(faults);
  RecordingMemory mem = faults ? RecordingMemory{mc, fm.translator(), fm.injector()} : RecordingMemory{mc};
  (void) tx_end;
  assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(image))).ok());
  mem.recording = true;
  *fm.armed = true;
  DMAEngine dma{mem};
  QueuePairConfig qc{
      .queue_id = 5,
      .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = ntx + 1, .base_address = rings ? ring_tx_at : 0,
                  .queue_id = 5, .host_backed = rings},
      .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = rings ? ring_rx_at : 0,
                  .queue_id = 5, .host_backed = rings},
      .tx_completion = {.ring_size = ntx + 1, .queue_id = 5},
      .rx_completion = {.ring_size = 70 * ntx + 1, .queue_id = 5},
  };
  QueuePair qp{qc, dma};
  for (auto& t : txs) {
    std::vector<std::byte> b(sizeof(TxDescriptor));
    std::memcpy(b.data(), &t, sizeof(t));
    assert(qp.tx_ring().push_descriptor(b).ok());
  }
  for (auto& x : rxs) {
    std::vector<std::byte> b(sizeof(RxDescriptor));
    std::memcpy(b.data(), &x, sizeof(x));
    assert(qp.rx_ring().push_descriptor(b).ok());
  }
  if (rings) {  // the image the batch starts from holds the pushed rings
    mem.recording = false;
    std::vector<std::byte> pushed(mem_size);
    assert(mem.read(0, pushed).ok());
    std::memcpy(image.data(), pushed.data(), mem_size);
    mem.writes.clear();  // (the pushes' DMA writes are not RX deliveries)
    mem.recording = true;
  }
  while (qp.process_once()) {
  }
  const std::size_t rx_consumed = nrx - qp.rx_ring().available();
  std::ostringstream js;
  js << "{\n \"source\": \"QueuePair::process_once over a batch (src/queue_pair.cpp:67-460)\",\n"
     << " \"queue_id\": 5, \"max_mtu\": 9000, \"mem_size\": " << mem_size << ", \"ntx\": " << ntx << ", \"nrx\": " << nrx
     << ", \"rx_consumed\": " << rx_consumed << ",\n \"tx_completions\": [";
  bool first = true;
  while (auto c = qp.tx_completion().poll_completion()) { js << (first ? "" : ",") << "\n  " << completion_json(*c); first = false; }
  js << "],\n \"rx_completions\": [";
  first = true;
  std::vector<CompletionEntry> rxc;
  while (auto c = qp.rx_completion().poll_completion()) {
    js << (first ? "" : ",") << "\n  " << completion_json(*c);
    first = false;
    rxc.push_back(*c);
  }
  // RSS of every frame delivered with Success (the reference RssEngine, MS
  // 40-B key, 128-entry table i % 16, on oracle_extract_tuple AUTO of the
  // bytes written for it); writes pair with the RX completions that carry one
  // (Success and ChecksumError: handle_rx_segment writes, then verifies)
  const std::vector<std::uint8_t>& ms_key = kMsKey;
  std::vector<std::uint16_t> rss_table(128);
  for (int i = 0; i < 128; ++i) rss_table[i] = static_cast<std::uint16_t>(i % 16);
  RssEngine rss_eng{RssConfig{ms_key, rss_table}};
  std::vector<std::uint32_t> rx_hash(rxc.size(), 0);
  std::vector<std::uint32_t> rx_queue(rxc.size(), 0xFFFFu);
  std::size_t wk = 0;
  for (std::size_t j = 0; j < rxc.size(); ++j) {
    const auto status = static_cast<CompletionCode>(rxc[j].status);
    if (status != CompletionCode::Success && status != CompletionCode::ChecksumError) continue;
    assert(wk < mem.writes.size());
    const std::vector<std::uint8_t>& bytes = mem.writes[wk++];
    if (status != CompletionCode::Success) continue;
    std::uint8_t t[64];
    const std::size_t tl = oracle_extract_tuple(bytes.data(), bytes.size(), ORACLE_TUPLE_AUTO, 0, 0, t);
    rx_hash[j] = RssEngine{RssConfig{ms_key, rss_table}}.hash(std::span<const std::uint8_t>(t, tl));
    rx_queue[j] = *rss_eng.select_queue(std::span<const std::uint8_t>(t, tl));
  }
  assert(wk == mem.writes.size());
  *fm.armed = false;  // read back whole
  const auto& st = qp.stats();
  js << "],\n \"stats\": [" << st.tx_packets << "," << st.rx_packets << "," << st.tx_bytes << "," << st.rx_bytes << ","
     << st.drops_checksum << "," << st.drops_no_rx_desc << "," << st.drops_buffer_small << "," << st.drops_mtu_exceeded
     << "," << st.drops_invalid_mss << "," << st.drops_too_many_segments << "," << st.tx_tso_segments << ","
     << st.tx_gso_segments << "," << st.tx_vlan_insertions << "," << st.rx_vlan_strips << "," << st.rx_checksum_verified
     << "," << st.rx_gro_aggregated << "],\n \"rx_region_fnv\": [";
  std::vector<std::byte> after(mem_size);
  assert(mem.read(0, after).ok());
  for (std::size_t j = 0; j < nrx; ++j) {
    const std::size_t a = std::min<std::size_t>(rxs[j].buffer_address, mem_size);
    const std::size_t n = std::min<std::size_t>(rxs[j].buffer_length, mem_size - a);
    js << (j ? "," : "") << "\"" << std::hex << fnv1a(after.data() + a, n) << std::dec << "\"";
  }
  js << "],\n \"mem_fnv\": \"" << std::hex << fnv1a(after.data(), mem_size) << std::dec << "\"";
  js << ",\n \"faults\": " << faults;
  if (rings) js << ",\n \"tx_ring_at\": " << ring_tx_at << ", \"rx_ring_at\": " << ring_rx_at;
  js << ",\n \"rss\": \"RssEngine{MS 40-B key, table i % 16 of 128}::select_queue on oracle_extract_tuple(AUTO) of each Success frame as written\"";
  js << ",\n \"rx_hash\": [";
  for (std::size_t j = 0; j < rx_hash.size(); ++j) js << (j ? "," : "") << rx_hash[j];
  js << "],\n \"rx_queue\": [";
  for (std::size_t j = 0; j < rx_queue.size(); ++j) js << (j ? "," : "") << rx_queue[j];
  js << "],\n \"rss_hashes\": " << rss_eng.stats().hashes << ",\n \"rss_queue_hits\": [";
  for (std::size_t i = 0; i < rss_eng.stats().queue_hits.size(); ++i) js << (i ? "," : "") << rss_eng.stats().queue_hits[i];
  js << "]\n}\n";
  std::ofstream(g_out + "/" + name + ".json") << js.str();
  write_bin(name + ".mem.bin", image);
  std::vector<std::uint8_t> tb(txs.size() * sizeof(TxDescriptor)), rb(rxs.size() * sizeof(RxDescriptor));
  std::memcpy(tb.data(), txs.data(), tb.size());
  std::memcpy(rb.data(), rxs.data(), rb.size());
  write_bin(name + ".tx.bin", tb);
  write_bin(name + ".rx.bin", rb);
}

// flavour 0: mixed sizes; 1: 9000 B TSO/GSO; 2: mixed sizes with overlapping
// buffers (recycled RX buffers, RX buffers straddling the previous one or
// lying inside TX buffers), where the reference's in-order writes decide.
// faults (faultfx::Kind): the memory's own DMA faults (tests/cpp/fault_model.h)
// through SimpleHostMemory's FaultInjector / AddressTranslator, armed once the
// memory is loaded and disarmed before it is read back.
void gen_qp_batch_case(const std::string& name, std::uint64_t seed, std::size_t ntx, std::size_t nrx, int flavour,
                       int faults = faultfx::kNone) {
  Rng r{seed};
  // TX region, then the RX buffers, then a guard tail; a few descriptors point
  // past the end (DMA fault).
  std::vector<TxDescriptor> txs;
  std::vector<std::vector<std::uint8_t>> pkts;
  std::size_t tx_end = 0;
  std::vector<std::uint64_t> tx_addr;
  for (std::size_t i = 0; i < ntx; ++i) {
    std::size_t L;
    const std::uint32_t pick = r.below(20);
    if (flavour == 1) L = 9000;                       // C5-like TSO batch
    else if (pick < 6) L = 64;
    else if (pick < 9) L = 576;
    else if (pick < 13) L = 1518;
    else if (pick < 15) L = r.below(80);             // tiny / empty / sub-header
    else if (pick < 17) L = 9000;
    else if (pick < 18) L = 9001 + r.below(300);     // over max_mtu
    else L = 64 + r.below(4000);
    FrameSpec fs;
    fs.total = L;
    fs.proto = (r.below(2) == 0) ? 6 : 17;
    fs.vlan_tags = (r.below(6) == 0) ? 1 : 0;
    fs.balance = r.below(4) != 0;
    std::vector<std::uint8_t> f = L >= 14 ? build_frame(r, fs) : std::vector<std::uint8_t>(L);
    if (L < 14) for (auto& b : f) b = r.byte();
    if (r.below(50) == 0) for (auto& b : f) b = 0;  // all-zero frame (checksum 0xFFFF)
    const std::size_t gap = r.below(3) == 0 ? r.below(16) : 0;
    tx_end += gap;
    tx_addr.push_back(tx_end);
    tx_end += L;
    pkts.push_back(std::move(f));
    TxDescriptor t{};
    t.buffer_address = tx_addr.back();
    t.length = static_cast<std::uint32_t>(L);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    const std::uint32_t cm = r.below(6);
    t.checksum = cm < 3 ? ChecksumMode::None : (cm < 5 ? ChecksumMode::Layer4 : ChecksumMode::Layer3);
    t.checksum_offload = r.below(3) != 0;
    const std::uint16_t good = ref_csum(pkts.back().data(), L);
    t.checksum_value = r.below(5) == 0 ? static_cast<std::uint16_t>(good ^ (1u + r.below(0xFFFE))) : good;
    const bool seg = flavour == 1 ? true : r.below(4) == 0;
    if (seg) {
      (r.below(2) ? t.tso_enabled : t.gso_enabled) = true;
      if (r.below(6) == 0) { t.tso_enabled = true; t.gso_enabled = true; }
      const std::uint32_t mp = r.below(12);
      t.mss = mp == 0 ? 0 : (mp == 1 ? static_cast<std::uint16_t>(9001 + r.below(100))
                                     : (mp == 2 ? static_cast<std::uint16_t>(1 + r.below(40))
                                                : static_cast<std::uint16_t>(100 + r.below(1500))));
      if (flavour == 1 && mp > 2) t.mss = r.below(3) == 0 ? 1447 : 1448;
      const std::uint32_t hp = r.below(10);
      t.header_length = hp == 0 ? 0 : (hp == 1 ? static_cast<std::uint16_t>(1 + r.below(5))
                                               : (hp == 2 ? static_cast<std::uint16_t>(L + r.below(2))
                                                          : static_cast<std::uint16_t>(54 + r.below(2))));
    }
    if (r.below(5) == 0) { t.vlan_insert = true; t.vlan_tag = static_cast<std::uint16_t>(r.u32()); }
    txs.push_back(t);
  }
  tx_end = (tx_end + 63) & ~std::size_t{63};
  std::vector<RxDescriptor> rxs;
  std::size_t rx_at = tx_end;
  for (std::size_t j = 0; j < nrx; ++j) {
    RxDescriptor x{};
    const std::uint32_t bp = r.below(10);
    std::uint32_t blen = bp == 0 ? r.below(1600) : (bp == 1 ? 64 : (bp < 7 ? 1600 : 9216 + 8));
    if (flavour == 1) blen = bp == 0 ? 1400 : 9216 + 8;
    x.buffer_address = rx_at + r.below(4);
    x.buffer_length = blen;
    rx_at = x.buffer_address + blen + r.below(8);
    x.descriptor_index = static_cast<std::uint16_t>(1000 + j);
    x.checksum_offload = flavour == 1 ? r.below(4) == 0 : r.below(4) != 0;
    const std::uint32_t cm = r.below(5);
    x.checksum = cm == 0 ? ChecksumMode::None : (cm < 3 ? ChecksumMode::Layer4 : ChecksumMode::Layer3);
    x.vlan_strip = r.below(3) == 0;
    x.vlan_present = r.below(4) == 0;
    x.vlan_tag = static_cast<std::uint16_t>(r.u32());
    x.gro_enabled = r.below(5) == 0;
    rxs.push_back(x);
  }
  if (flavour == 2) {
    for (std::size_t j = 1; j < nrx; ++j) {
      RxDescriptor& x = rxs[j];
      const std::uint32_t k = r.below(12);
      if (k < 3) {  // a recycled buffer
        const RxDescriptor& y = rxs[r.below(static_cast<std::uint32_t>(j))];
        x.buffer_address = y.buffer_address;
        if (r.below(2)) x.buffer_length = y.buffer_length;
      } else if (k < 5) {  // straddling the previous buffer
        x.buffer_address = rxs[j - 1].buffer_address + r.below(std::max<std::uint32_t>(1, rxs[j - 1].buffer_length));
      } else if (k < 7) {  // inside a TX buffer
        x.buffer_address = tx_addr[r.below(static_cast<std::uint32_t>(ntx))] + r.below(16);
      }
    }
  }
  const std::size_t mem_size = rx_at + 64;
  // DMA faults: a few descriptors addressed past the end of host memory
  // (past the end, or straddling it); RX fault addresses are distinct so no
  // two DMA writes can land on the same bytes
  for (std::size_t i = 0; i < ntx; ++i)
    if (r.below(60) == 0) txs[i].buffer_address = r.below(2) ? mem_size + 1 + i : mem_size - txs[i].length / 2;
  for (std::size_t j = 0; j < nrx; ++j)
    if (r.below(80) == 0) rxs[j].buffer_address = mem_size + 1 + j;

  std::vector<std::uint8_t> image(mem_size);
  for (std::size_t a = 0; a < tx_end; ++a) image[a] = r.byte();  // RX region starts zeroed
  for (std::size_t i = 0; i < ntx; ++i) std::memcpy(image.data() + tx_addr[i], pkts[i].data(), pkts[i].size());
  emit_qp_case(name, txs, rxs, std::move(image), mem_size, tx_end, faults);
}


// Host-backed rings that the batch's own DMA writes land on: some RX buffers
// are exactly a later TX or RX ring slot (buffer_length 32 / 24), so a frame
// of at most that size delivered there becomes the descriptor the reference
// pops from that slot later (descriptor_ring.cpp:97-106).  Every frame starts
// with a 32-byte head that reads as a sane TxDescriptor and RxDescriptor
// (bools 0/1, no checksum, no TSO, no VLAN, lengths <= 1600, buffers below the
// rings), a third of the frames are that head alone (24..32 B), and no
// original descriptor inserts or strips a VLAN tag (a shifted head would not
// read as one).
void gen_qp_ring_case(const std::string& name, std::uint64_t seed, std::size_t ntx, std::size_t nrx) {
  Rng r{seed};
  const std::size_t rx_len = 2048;
  // layout: TX frames | RX buffers | TX ring | RX ring | guard
  std::vector<std::size_t> lens(ntx);
  std::size_t tx_end = 0;
  std::vector<std::uint64_t> tx_addr(ntx);
  for (std::size_t i = 0; i < ntx; ++i) {
    const std::uint32_t pick = r.below(3);
    lens[i] = pick == 0 ? 16 + r.below(17) : (pick == 1 ? 64 + r.below(500) : 600 + r.below(1000));
    tx_addr[i] = tx_end;
    tx_end += lens[i] + r.below(8);
  }
  tx_end = (tx_end + 63) & ~std::size_t{63};
  const std::size_t rx_base = tx_end;
  const std::size_t ring_tx_at = rx_base + nrx * rx_len;
  const std::size_t ring_rx_at = ring_tx_at + ntx * sizeof(TxDescriptor);
  const std::size_t rings_start = ring_tx_at;
  const std::size_t mem_size = ring_rx_at + nrx * sizeof(RxDescriptor) + 256;
  auto head = [&](std::uint8_t* h) {  // 32 bytes, a sane TxDescriptor and RxDescriptor
    std::memset(h, 0, 32);
    const std::uint64_t a = r.below(static_cast<std::uint32_t>(rings_start - 2048));
    std::memcpy(h, &a, 8);                                       // buffer_address
    const std::uint32_t len = r.below(1601);
    std::memcpy(h + 8, &len, 4);                                 // length / buffer_length
    h[14] = r.byte();                                            // descriptor_index
    h[15] = r.byte();
    h[16] = static_cast<std::uint8_t>(r.below(2));               // TX checksum_value lo | RX checksum_offload
    h[18] = static_cast<std::uint8_t>(r.below(2));               // TX checksum_offload | RX vlan_present
    h[22] = static_cast<std::uint8_t>(r.below(2));               // TX mss lo | RX gro_enabled
    h[23] = r.byte();                                            // TX mss hi
    h[24] = r.byte();                                            // TX header_length
    h[25] = r.byte();
    h[28] = r.byte();                                            // TX vlan_tag | (past the RX descriptor)
    h[29] = r.byte();
  };
  std::vector<std::uint8_t> image(mem_size, 0);
  for (std::size_t a = 0; a < tx_end; ++a) image[a] = r.byte();
  std::vector<TxDescriptor> txs(ntx);
  for (std::size_t i = 0; i < ntx; ++i) {
    std::uint8_t* f = image.data() + tx_addr[i];
    std::uint8_t h[32];
    head(h);
    std::memcpy(f, h, std::min<std::size_t>(32, lens[i]));
    TxDescriptor& t = txs[i];
    t.buffer_address = tx_addr[i];
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    const std::uint32_t cm = r.below(6);
    t.checksum = cm < 4 ? ChecksumMode::None : ChecksumMode::Layer4;
    t.checksum_offload = r.below(3) != 0;
    const std::uint16_t good = ref_csum(f, lens[i]);
    t.checksum_value = r.below(5) == 0 ? static_cast<std::uint16_t>(good ^ 1u) : good;
    if (lens[i] > 400 && r.below(4) == 0) {  // segmentation, headers of at least 32 bytes
      (r.below(2) ? t.tso_enabled : t.gso_enabled) = true;
      t.mss = static_cast<std::uint16_t>(100 + r.below(400));
      t.header_length = static_cast<std::uint16_t>(32 + r.below(40));
    }
  }
  std::vector<RxDescriptor> rxs(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    RxDescriptor& x = rxs[j];
    x.buffer_address = rx_base + j * rx_len;
    x.buffer_length = static_cast<std::uint32_t>(rx_len);
    x.descriptor_index = static_cast<std::uint16_t>(1000 + j);
    x.checksum_offload = r.below(2) != 0;
    x.checksum = r.below(3) == 0 ? ChecksumMode::None : ChecksumMode::Layer4;
    x.vlan_present = r.below(4) == 0;
    x.gro_enabled = r.below(4) == 0;
    const std::uint32_t k = r.below(8);
    if (k == 0 && j + 100 < nrx) {  // a later RX ring slot (beyond the pops of any one packet)
      x.buffer_address = ring_rx_at + (j + 80 + r.below(static_cast<std::uint32_t>(std::min<std::size_t>(60, nrx - j - 80)))) *
                                          sizeof(RxDescriptor);
      x.buffer_length = sizeof(RxDescriptor);
    } else if (k == 1 && j + 40 < ntx) {  // a later TX ring slot
      x.buffer_address = ring_tx_at + (j + 10 + r.below(30)) * sizeof(TxDescriptor);
      x.buffer_length = sizeof(TxDescriptor);
    }
  }
  emit_qp_case(name, txs, rxs, std::move(image), mem_size, tx_end, faultfx::kNone, ring_tx_at, ring_rx_at);
}

void gen_qp_batch() {
  gen_qp_batch_case("qp_mix_a", 101, 300, 180, 0);    // RX ring runs dry part-way
  gen_qp_batch_case("qp_mix_b", 202, 400, 700, 0);    // ample RX descriptors
  gen_qp_batch_case("qp_tso", 303, 40, 300, 1);       // 9000 B TSO/GSO, odd mss, tiny headers
  gen_qp_batch_case("qp_alias", 404, 300, 400, 2);    // overlapping RX/RX and RX/TX buffers
  // the memory's own faults (SimpleHostMemory's injector / IOMMU translator)
  gen_qp_batch_case("qp_fault_inj", 505, 400, 700, 0, faultfx::kInjector);
  gen_qp_batch_case("qp_fault_iommu", 606, 400, 700, 0, faultfx::kIommu);
  gen_qp_batch_case("qp_fault_tso", 707, 40, 300, 1, faultfx::kInjector);
  // host-backed rings written over by the batch's own DMA writes
  gen_qp_ring_case("qp_ring", 808, 400, 600);
}

// ------------------------------------------------------------ QueueManager --
// SURVEY §8 f1, the caller of the batched QueuePair: QueueManager::process_once
// (src/queue_manager.cpp:54-78) drained — weighted round robin with credits,
// skips of queues whose TX ring is empty — over several queue pairs sharing
// one host memory and one InterruptDispatcher, in two rounds (the scheduler's
// index/credit and the RX descriptors a round left carry into the next).
// Recorded per round and queue: the TX/RX completions in posting order and the
// RX descriptors consumed; per round: the MSI-X vectors fired in order (queue
// q -> vector q, packet threshold 1, so one per InterruptDispatcher::
// on_completion) and the scheduler's advances/skips; at the end: every
// QueuePairStats, QueueManagerStats (aggregate_stats, :119-139) and an FNV of
// the memory.  flavour 1: some RX buffers of queue q lie in queue q+1's TX
// buffers, so the order the scheduler serves the queues decides the bytes.
struct QmRound {
  std::vector<std::vector<TxDescriptor>> tx;  // [queue]
  std::vector<std::vector<RxDescriptor>> rx;
};

void gen_qm_case(const std::string& name, std::uint64_t seed, const std::vector<std::uint8_t>& weights,
                 const std::vector<std::vector<std::size_t>>& ntx, const std::vector<std::vector<std::size_t>>& nrx,
                 int flavour) {
  Rng r{seed};
  const std::size_t Q = weights.size(), R = ntx.size();
  std::vector<QmRound> rounds(R);
  std::vector<std::uint8_t> image;
  std::vector<std::vector<std::uint64_t>> tx_addr(Q);  // every TX buffer of a queue (for flavour 1)
  // per round and queue: a TX region then an RX region, appended to the image
  for (std::size_t k = 0; k < R; ++k) {
    rounds[k].tx.resize(Q);
    rounds[k].rx.resize(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      for (std::size_t i = 0; i < ntx[k][q]; ++i) {
        const std::uint32_t pick = r.below(16);
        std::size_t L = pick < 5 ? 64 : pick < 8 ? 576 : pick < 11 ? 1518 : pick < 12 ? r.below(60)
                        : pick < 13 ? 9000 : pick < 14 ? 9001 + r.below(100) : 64 + r.below(3000);
        FrameSpec fs;
        fs.total = L;
        fs.proto = r.below(2) ? 6 : 17;
        fs.balance = r.below(4) != 0;
        std::vector<std::uint8_t> f = L >= 14 ? build_frame(r, fs) : std::vector<std::uint8_t>(L);
        if (L < 14) for (auto& b : f) b = r.byte();
        image.resize(image.size() + r.below(8));
        TxDescriptor t{};
        t.buffer_address = image.size();
        t.length = static_cast<std::uint32_t>(L);
        t.descriptor_index = static_cast<std::uint16_t>(100 * q + i);
        const std::uint32_t cm = r.below(5);
        t.checksum = cm < 2 ? ChecksumMode::None : (cm < 4 ? ChecksumMode::Layer4 : ChecksumMode::Layer3);
        t.checksum_offload = r.below(3) != 0;
        const std::uint16_t good = ref_csum(f.data(), L);
        t.checksum_value = r.below(6) == 0 ? static_cast<std::uint16_t>(good ^ (1u + r.below(0xFFFE))) : good;
        if (L > 1518 && r.below(2) == 0) {
          (r.below(2) ? t.tso_enabled : t.gso_enabled) = true;
          t.mss = r.below(8) == 0 ? static_cast<std::uint16_t>(1 + r.below(30)) : static_cast<std::uint16_t>(1448);
          t.header_length = 54;
        }
        if (r.below(6) == 0) { t.vlan_insert = true; t.vlan_tag = static_cast<std::uint16_t>(r.u32()); }
        image.insert(image.end(), f.begin(), f.end());
        tx_addr[q].push_back(t.buffer_address);
        rounds[k].tx[q].push_back(t);
      }
      image.resize((image.size() + 63) & ~std::size_t{63});
      for (std::size_t j = 0; j < nrx[k][q]; ++j) {
        RxDescriptor x{};
        const std::uint32_t bp = r.below(10);
        const std::uint32_t blen = bp == 0 ? r.below(1600) : (bp == 1 ? 64 : (bp < 7 ? 1600 : 9216 + 8));
        image.resize(image.size() + r.below(4));
        x.buffer_address = image.size();
        x.buffer_length = blen;
        image.resize(image.size() + blen);
        x.descriptor_index = static_cast<std::uint16_t>(1000 + 100 * q + j);
        x.checksum_offload = r.below(4) != 0;
        const std::uint32_t cm = r.below(5);
        x.checksum = cm == 0 ? ChecksumMode::None : (cm < 3 ? ChecksumMode::Layer4 : ChecksumMode::Layer3);
        x.vlan_strip = r.below(3) == 0;
        x.vlan_present = r.below(4) == 0;
        x.vlan_tag = static_cast<std::uint16_t>(r.u32());
        x.gro_enabled = r.below(5) == 0;
        rounds[k].rx[q].push_back(x);
      }
    }
  }
  if (flavour == 1)  // RX buffers of queue q inside queue q+1's TX buffers (any round)
    for (std::size_t k = 0; k < R; ++k)
      for (std::size_t q = 0; q < Q; ++q)
        for (RxDescriptor& x : rounds[k].rx[q]) {
          const auto& ta = tx_addr[(q + 1) % Q];
          if (!ta.empty() && r.below(3) == 0) x.buffer_address = ta[r.below(static_cast<std::uint32_t>(ta.size()))] + r.below(8);
        }
  image.resize(image.size() + 64);
  const std::size_t mem_size = image.size();
  HostMemoryConfig mc{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = false};
  SimpleHostMemory mem{mc};
  assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(image))).ok());
  DMAEngine dma{mem};
  std::vector<std::uint16_t> fired;
  MsixMapping mapping{Q, 0};
  for (std::size_t q = 0; q < Q; ++q) mapping.set_queue_vector(q, static_cast<std::uint16_t>(q));
  InterruptDispatcher irq{MsixTable{Q}, mapping, CoalesceConfig{1, 0},
                          [&](std::uint16_t v, std::uint32_t) { fired.push_back(v); }};
  std::size_t tot_tx = 0, tot_rx = 0;
  for (std::size_t k = 0; k < R; ++k)
    for (std::size_t q = 0; q < Q; ++q) { tot_tx += ntx[k][q]; tot_rx += nrx[k][q]; }
  QueueManagerConfig qmc;
  for (std::size_t q = 0; q < Q; ++q) {
    const auto id = static_cast<std::uint16_t>(q);
    QueuePairConfig c{
        .queue_id = id,
        .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = tot_tx + 1, .base_address = 0, .queue_id = id, .host_backed = false},
        .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = tot_rx + 1, .base_address = 0, .queue_id = id, .host_backed = false},
        .tx_completion = {.ring_size = tot_tx + 1, .queue_id = id},
        .rx_completion = {.ring_size = 70 * tot_tx + 1, .queue_id = id},
    };
    c.interrupt_dispatcher = &irq;
    c.weight = weights[q];
    c.max_mtu = 9000;
    c.enable_tx_interrupts = q % 2 == 0;
    c.enable_rx_interrupts = q % 3 != 2;
    qmc.queue_configs.push_back(c);
  }
  QueueManager qm{qmc, dma};
  std::ostringstream js;
  js << "{\n \"source\": \"QueueManager::process_once drained per round (src/queue_manager.cpp:54-78), stats :119-139\",\n"
     << " \"queues\": " << Q << ", \"weights\": " << json_arr(weights) << ", \"max_mtu\": 9000, \"mem_size\": " << mem_size
     << ",\n \"enable_tx_interrupts\": [";
  for (std::size_t q = 0; q < Q; ++q) js << (q ? "," : "") << int(q % 2 == 0);
  js << "], \"enable_rx_interrupts\": [";
  for (std::size_t q = 0; q < Q; ++q) js << (q ? "," : "") << int(q % 3 != 2);
  js << "],\n \"rounds\": [";
  std::vector<TxDescriptor> all_tx;
  std::vector<RxDescriptor> all_rx;
  std::uint64_t adv0 = 0, skip0 = 0;
  for (std::size_t k = 0; k < R; ++k) {
    for (std::size_t q = 0; q < Q; ++q) {
      QueuePair& qp = *qm.queue(q);
      for (const TxDescriptor& t : rounds[k].tx[q]) {
        std::vector<std::byte> b(sizeof(TxDescriptor));
        std::memcpy(b.data(), &t, sizeof(t));
        assert(qp.tx_ring().push_descriptor(b).ok());
        all_tx.push_back(t);
      }
      for (const RxDescriptor& x : rounds[k].rx[q]) {
        std::vector<std::byte> b(sizeof(RxDescriptor));
        std::memcpy(b.data(), &x, sizeof(x));
        assert(qp.rx_ring().push_descriptor(b).ok());
        all_rx.push_back(x);
      }
    }
    std::vector<std::size_t> avail0(Q);
    for (std::size_t q = 0; q < Q; ++q) avail0[q] = qm.queue(q)->rx_ring().available();
    fired.clear();
    while (qm.process_once()) {
    }
    const QueueManagerStats ms = qm.stats();
    js << (k ? "," : "") << "\n  {\"ntx\": " << json_arr(ntx[k]) << ", \"nrx\": " << json_arr(nrx[k])
       << ", \"advances\": " << ms.scheduler_advances - adv0 << ", \"skips\": " << ms.scheduler_skips - skip0
       << ", \"rx_consumed\": [";
    adv0 = ms.scheduler_advances;
    skip0 = ms.scheduler_skips;
    for (std::size_t q = 0; q < Q; ++q) js << (q ? "," : "") << avail0[q] - qm.queue(q)->rx_ring().available();
    js << "],\n   \"irq_vectors\": " << json_arr(fired) << ",\n   \"tx_completions\": [";
    for (std::size_t q = 0; q < Q; ++q) {
      js << (q ? "," : "") << "[";
      bool first = true;
      while (auto c = qm.queue(q)->tx_completion().poll_completion()) { js << (first ? "" : ",") << completion_json(*c); first = false; }
      js << "]";
    }
    js << "],\n   \"rx_completions\": [";
    for (std::size_t q = 0; q < Q; ++q) {
      js << (q ? "," : "") << "[";
      bool first = true;
      while (auto c = qm.queue(q)->rx_completion().poll_completion()) { js << (first ? "" : ",") << completion_json(*c); first = false; }
      js << "]";
    }
    js << "]}";
  }
  js << "],\n \"stats\": [";
  for (std::size_t q = 0; q < Q; ++q) {
    const QueuePairStats st = *qm.queue_stats(q);
    js << (q ? "," : "") << "\n  [" << st.tx_packets << "," << st.rx_packets << "," << st.tx_bytes << "," << st.rx_bytes
       << "," << st.drops_checksum << "," << st.drops_no_rx_desc << "," << st.drops_buffer_small << ","
       << st.drops_mtu_exceeded << "," << st.drops_invalid_mss << "," << st.drops_too_many_segments << ","
       << st.tx_tso_segments << "," << st.tx_gso_segments << "," << st.tx_vlan_insertions << "," << st.rx_vlan_strips
       << "," << st.rx_checksum_verified << "," << st.rx_gro_aggregated << "]";
  }
  const QueueManagerStats ms = qm.stats();
  js << "],\n \"qm_stats\": [" << ms.total_tx_packets << "," << ms.total_rx_packets << "," << ms.total_tx_bytes << ","
     << ms.total_rx_bytes << "," << ms.total_drops_checksum << "," << ms.total_drops_no_rx_desc << ","
     << ms.total_drops_buffer_small << "," << ms.total_tx_tso_segments << "," << ms.total_tx_gso_segments << ","
     << ms.total_tx_vlan_insertions << "," << ms.total_rx_vlan_strips << "," << ms.total_rx_checksum_verified << ","
     << ms.total_rx_gro_aggregated << "," << ms.scheduler_advances << "," << ms.scheduler_skips << "],\n"
     << " \"stats_summary\": \"" << qm.stats_summary() << "\",\n";
  std::vector<std::byte> after(mem_size);
  assert(mem.read(0, after).ok());
  js << " \"mem_fnv\": \"" << std::hex << fnv1a(after.data(), mem_size) << std::dec << "\"\n}\n";
  std::ofstream(g_out + "/" + name + ".json") << js.str();
  write_bin(name + ".mem.bin", image);
  std::vector<std::uint8_t> tb(all_tx.size() * sizeof(TxDescriptor)), rb(all_rx.size() * sizeof(RxDescriptor));
  std::memcpy(tb.data(), all_tx.data(), tb.size());
  std::memcpy(rb.data(), all_rx.data(), rb.size());
  write_bin(name + ".tx.bin", tb);
  write_bin(name + ".rx.bin", rb);
}

void gen_qm() {
  // 4 queues, weights 1/3/2/1: queue 3 has nothing to send in round 0, queue 1
  // runs its RX ring dry; round 1 carries the leftovers and the scheduler state
  gen_qm_case("qm_mix", 505, {1, 3, 2, 1}, {{40, 90, 25, 0}, {10, 0, 30, 20}}, {{60, 50, 80, 10}, {30, 20, 10, 40}}, 0);
  // weight 0 (served as 1, queue_manager.cpp:14-16), single-descriptor queues
  gen_qm_case("qm_weights", 606, {0, 5, 1}, {{1, 33, 7}, {12, 1, 0}}, {{5, 70, 20}, {30, 3, 2}}, 0);
  // cross-queue aliasing: the served order decides what is read and written
  gen_qm_case("qm_alias", 707, {2, 1, 3}, {{30, 25, 20}, {15, 15, 15}}, {{40, 40, 40}, {20, 20, 20}}, 1);
}

// QueueManager at scale: 16 queue pairs, ≈ 70 K TX descriptors over two rounds
// (tests/cpp/qm_scale_gen.h makes the input from the seed on both sides; the
// fixture holds the seed, the schedule counters and digests — see there).
void gen_qm_scale(std::uint64_t seed) {
  auto c = qm_scale::make_case<TxDescriptor, RxDescriptor>(seed, ChecksumMode::None, ChecksumMode::Layer3,
                                                           ChecksumMode::Layer4);
  const std::size_t Q = c.Q, mem_size = c.image.size();
  HostMemoryConfig mc{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = false};
  SimpleHostMemory mem{mc};
  assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(c.image))).ok());
  DMAEngine dma{mem};
  std::vector<std::uint16_t> fired;
  MsixMapping mapping{Q, 0};
  for (std::size_t q = 0; q < Q; ++q) mapping.set_queue_vector(q, static_cast<std::uint16_t>(q));
  InterruptDispatcher irq{MsixTable{Q}, mapping, CoalesceConfig{1, 0},
                          [&](std::uint16_t v, std::uint32_t) { fired.push_back(v); }};
  QueueManagerConfig qmc;
  for (std::size_t q = 0; q < Q; ++q) {
    std::size_t tt = 0, tr = 0;
    for (std::size_t k = 0; k < c.R; ++k) { tt += c.ntx[k][q]; tr += c.nrx[k][q]; }
    const auto id = static_cast<std::uint16_t>(q);
    QueuePairConfig qc{
        .queue_id = id,
        .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = tt + 1, .base_address = 0, .queue_id = id, .host_backed = false},
        .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = tr + 1, .base_address = 0, .queue_id = id, .host_backed = false},
        .tx_completion = {.ring_size = tt + 1, .queue_id = id},
        .rx_completion = {.ring_size = 8 * tt + 1, .queue_id = id},
    };
    qc.interrupt_dispatcher = &irq;
    qc.weight = c.weights[q];
    qc.max_mtu = c.max_mtu;
    qc.enable_tx_interrupts = c.etx(q);
    qc.enable_rx_interrupts = c.erx(q);
    qmc.queue_configs.push_back(qc);
  }
  QueueManager qm{qmc, dma};
  std::ostringstream js;
  js << "{\n \"source\": \"QueueManager::process_once drained per round (src/queue_manager.cpp:54-78), stats :119-139; "
        "input made by tests/cpp/qm_scale_gen.h from the seed\",\n"
     << " \"seed\": " << seed << ", \"queues\": " << Q << ", \"weights\": " << json_arr(c.weights)
     << ", \"max_mtu\": " << c.max_mtu << ", \"mem_size\": " << mem_size << ",\n \"rounds\": [";
  auto str_arr = [](const std::vector<std::string>& v) {
    std::string o = "[";
    for (std::size_t i = 0; i < v.size(); ++i) o += (i ? "," : "") + v[i];
    return o + "]";
  };
  std::uint64_t adv0 = 0, skip0 = 0;
  for (std::size_t k = 0; k < c.R; ++k) {
    for (std::size_t q = 0; q < Q; ++q) {
      QueuePair& qp = *qm.queue(q);
      for (const TxDescriptor& t : c.tx[k][q]) {
        std::vector<std::byte> b(sizeof(TxDescriptor));
        std::memcpy(b.data(), &t, sizeof(t));
        assert(qp.tx_ring().push_descriptor(b).ok());
      }
      for (const RxDescriptor& x : c.rx[k][q]) {
        std::vector<std::byte> b(sizeof(RxDescriptor));
        std::memcpy(b.data(), &x, sizeof(x));
        assert(qp.rx_ring().push_descriptor(b).ok());
      }
    }
    std::vector<std::size_t> avail0(Q);
    for (std::size_t q = 0; q < Q; ++q) avail0[q] = qm.queue(q)->rx_ring().available();
    fired.clear();
    while (qm.process_once()) {
    }
    const QueueManagerStats ms = qm.stats();
    std::vector<std::size_t> consumed(Q), ntc(Q), nrc(Q);
    std::vector<std::string> ftx(Q), frx(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      consumed[q] = avail0[q] - qm.queue(q)->rx_ring().available();
      std::uint64_t h = qm_scale::kFnv0;
      while (auto e = qm.queue(q)->tx_completion().poll_completion()) { h = qm_scale::fnv_completion(h, *e); ++ntc[q]; }
      std::ostringstream o;
      o << std::hex << h;
      ftx[q] = "\"" + o.str() + "\"";
      h = qm_scale::kFnv0;
      while (auto e = qm.queue(q)->rx_completion().poll_completion()) { h = qm_scale::fnv_completion(h, *e); ++nrc[q]; }
      o.str("");
      o << std::hex << h;
      frx[q] = "\"" + o.str() + "\"";
    }
    std::ostringstream fv;
    fv << std::hex << qm_scale::fnv(qm_scale::kFnv0, fired.data(), fired.size() * sizeof(std::uint16_t));
    js << (k ? "," : "") << "\n  {\"ntx\": " << json_arr(c.ntx[k]) << ", \"nrx\": " << json_arr(c.nrx[k])
       << ", \"advances\": " << ms.scheduler_advances - adv0 << ", \"skips\": " << ms.scheduler_skips - skip0
       << ", \"rx_consumed\": " << json_arr(consumed) << ",\n   \"irq_count\": " << fired.size() << ", \"irq_fnv\": \""
       << fv.str() << "\",\n   \"tx_count\": " << json_arr(ntc) << ", \"rx_count\": " << json_arr(nrc)
       << ",\n   \"tx_fnv\": " << str_arr(ftx) << ",\n   \"rx_fnv\": " << str_arr(frx) << "}";
    adv0 = ms.scheduler_advances;
    skip0 = ms.scheduler_skips;
  }
  js << "],\n \"stats\": [";
  for (std::size_t q = 0; q < Q; ++q) {
    const QueuePairStats st = *qm.queue_stats(q);
    js << (q ? "," : "") << "\n  [" << st.tx_packets << "," << st.rx_packets << "," << st.tx_bytes << "," << st.rx_bytes
       << "," << st.drops_checksum << "," << st.drops_no_rx_desc << "," << st.drops_buffer_small << ","
       << st.drops_mtu_exceeded << "," << st.drops_invalid_mss << "," << st.drops_too_many_segments << ","
       << st.tx_tso_segments << "," << st.tx_gso_segments << "," << st.tx_vlan_insertions << "," << st.rx_vlan_strips
       << "," << st.rx_checksum_verified << "," << st.rx_gro_aggregated << "]";
  }
  const QueueManagerStats ms = qm.stats();
  js << "],\n \"qm_stats\": [" << ms.total_tx_packets << "," << ms.total_rx_packets << "," << ms.total_tx_bytes << ","
     << ms.total_rx_bytes << "," << ms.total_drops_checksum << "," << ms.total_drops_no_rx_desc << ","
     << ms.total_drops_buffer_small << "," << ms.total_tx_tso_segments << "," << ms.total_tx_gso_segments << ","
     << ms.total_tx_vlan_insertions << "," << ms.total_rx_vlan_strips << "," << ms.total_rx_checksum_verified << ","
     << ms.total_rx_gro_aggregated << "," << ms.scheduler_advances << "," << ms.scheduler_skips << "],\n"
     << " \"stats_summary\": \"" << qm.stats_summary() << "\",\n";
  std::vector<std::byte> after(mem_size);
  assert(mem.read(0, after).ok());
  js << " \"mem_fnv\": \"" << std::hex << fnv1a(after.data(), mem_size) << std::dec << "\"\n}\n";
  std::ofstream(g_out + "/qm16_scale.json") << js.str();
}

// ------------------------------------------------------ L3/L4 verification --
// SURVEY §8 f3.  Frames from build_frame (valid IPv4 header and TCP/UDP
// checksums), then mutated.  Expected flags use the reference's own
// compute_checksum (src/checksum.cpp:10-34), which is the same algorithm as
// PacketGenerator::ipv4_checksum / tcp_checksum / udp_checksum
// (packet_generator.cpp:200-305, not buildable here: bit_fields): a valid IPv4
// header has compute_checksum(header) == 0, a valid L4 segment
// compute_checksum(pseudo-header || segment) == 0.
std::uint8_t ref_l34(const std::vector<std::uint8_t>& f) {
  const std::size_t len = f.size();
  if (len < 14) return 0;
  std::size_t l3 = 14;
  unsigned et = (f[12] << 8) | f[13];
  for (int t = 0; t < 2 && (et == 0x8100 || et == 0x88A8); ++t) {
    if (len < l3 + 4) return 0;
    et = (f[l3 + 2] << 8) | f[l3 + 3];
    l3 += 4;
  }
  if (et != 0x0800 || len < l3 + 20 || (f[l3] >> 4) != 4) return 0;
  const std::size_t ihl = (f[l3] & 15u) * 4u;
  if (ihl < 20 || l3 + ihl > len) return 0;
  std::uint8_t fl = ORACLE_L34_IPV4;
  if (ref_csum(&f[l3], ihl) == 0) fl |= ORACLE_L34_IPV4_OK;
  const unsigned proto = f[l3 + 9];
  const unsigned frag = ((f[l3 + 6] << 8) | f[l3 + 7]) & 0x3FFFu;
  const std::size_t total = (f[l3 + 2] << 8) | f[l3 + 3];
  if ((proto != 6 && proto != 17) || frag != 0 || total < ihl || l3 + total > len) return fl;
  const std::size_t seg = total - ihl;
  if (seg < (proto == 6 ? 20u : 8u)) return fl;
  fl |= ORACLE_L34_L4;
  const std::size_t l4 = l3 + ihl;
  if (proto == 17 && f[l4 + 6] == 0 && f[l4 + 7] == 0) return fl | ORACLE_L34_L4_OK | ORACLE_L34_UDP_NOCSUM;
  std::vector<std::uint8_t> ps(12 + seg);
  std::memcpy(ps.data(), &f[l3 + 12], 8);
  ps[8] = 0;
  ps[9] = static_cast<std::uint8_t>(proto);
  ps[10] = static_cast<std::uint8_t>(seg >> 8);
  ps[11] = static_cast<std::uint8_t>(seg);
  std::memcpy(ps.data() + 12, &f[l4], seg);
  if (ref_csum(ps.data(), ps.size()) == 0) fl |= ORACLE_L34_L4_OK;
  return fl;
}

void gen_l34() {
  Rng r{3434};
  std::vector<std::uint8_t> frames, flags;
  std::vector<std::uint64_t> desc;
  const std::size_t sizes[] = {60, 64, 66, 77, 128, 576, 1000, 1514, 1518, 4001, 9000};
  for (int i = 0; i < 3000; ++i) {
    FrameSpec s;
    const std::uint32_t k = r.below(20);
    s.l3 = k == 0 ? 6 : (k == 1 ? 0 : 4);
    s.proto = r.below(10) == 0 ? 1 : (r.below(2) ? 6 : 17);
    s.vlan_tags = r.below(8) == 0 ? 1 + r.below(2) : 0;
    s.ihl = r.below(6) == 0 ? 6 + r.below(10) : 5;
    s.frag = r.below(15) == 0;
    s.total = sizes[r.below(11)] + (r.below(3) == 0 ? r.below(9) : 0);
    s.balance = r.below(2);
    auto f = build_frame(r, s);
    const std::size_t l3 = 14 + 4 * s.vlan_tags;
    const std::uint32_t m = r.below(16);
    if (m == 0 && f.size() > 60) f[40 + r.below(static_cast<std::uint32_t>(f.size() - 40))] ^= 1 + r.below(255);  // payload bit error
    else if (m == 1 && f.size() >= l3 + 20) f[l3 + r.below(20)] ^= 1 + r.below(255);                           // IP header error
    else if (m == 2 && f.size() >= l3 + 28 && s.proto == 17) { f[l3 + s.ihl * 4 + 6] = 0; f[l3 + s.ihl * 4 + 7] = 0; }  // UDP no checksum
    else if (m == 3) for (std::uint32_t p = 1 + r.below(30); p--;) f.push_back(r.byte());                       // Ethernet padding / trailer
    else if (m == 4 && f.size() >= l3 + 4) { f[l3 + 3] = static_cast<std::uint8_t>(f[l3 + 3] + 1 + r.below(4)); }  // total length past the frame
    else if (m == 5 && f.size() >= l3 + 4) { f[l3 + 2] = 0; f[l3 + 3] = static_cast<std::uint8_t>(r.below(20)); }  // total < IHL
    else if (m == 6 && f.size() >= l3 + 1) f[l3] = static_cast<std::uint8_t>((f[l3] & 0xF0) | r.below(5));       // IHL < 5
    else if (m == 7) f.resize(r.below(static_cast<std::uint32_t>(f.size()) + 1));                               // truncation
    // frames at any byte offset
    const std::size_t gap = r.below(4) == 0 ? r.below(16) : (16 - frames.size() % 16) % 16;
    for (std::size_t g = 0; g < gap; ++g) frames.push_back(r.byte());
    desc.push_back(frames.size() | (static_cast<std::uint64_t>(f.size()) << 40));
    frames.insert(frames.end(), f.begin(), f.end());
    flags.push_back(ref_l34(f));
  }
  frames.resize(frames.size() + 64, 0);
  write_bin("l34.frames.bin", frames);
  write_bin("l34.desc.bin", desc);
  write_bin("l34.flags.bin", flags);
}

// -------------------------------------------- TSO + VLAN materialisation --
// the segments the reference QueuePair delivers into RX buffers
// for TSO/GSO frames with TX VLAN insert and RX VLAN strip/present
// (queue_pair.cpp:212-278, 320-331, 389-395), RX checksum offload off so that
// every segment is delivered.  Recorded per case: TX status, and for every
// delivered segment its length, compute_checksum and FNV-1a-64 of its bytes.
constexpr std::size_t kSlotHash = 9216 + 8;  // bytes of each RX slot hashed

void gen_tso_vlan() {
  Rng r{4242};
  std::ostringstream js;
  js << "{\n \"source\": \"QueuePair::process_once TSO/GSO + VLAN insert/strip (src/queue_pair.cpp:212-278, 320-331, 389-395); segments read back from the RX buffers\",\n \"cases\": [\n";
  std::vector<std::uint8_t> frames;
  const int ncase = 160;
  for (int ci = 0; ci < ncase; ++ci) {
    const std::size_t lens[] = {0, 3, 60, 64, 200, 1518, 3000, 9000, 9000, 9000};
    std::size_t L = lens[r.below(10)];
    std::vector<std::uint8_t> pkt(L);
    for (auto& b : pkt) b = r.byte();
    const bool tso = r.below(5) != 0;
    const bool gso = tso && r.below(3) == 0;
    const std::uint16_t mss = static_cast<std::uint16_t>(r.below(8) == 0 ? r.below(10) : (r.below(6) == 0 ? 9001 : 100 + r.below(1500)));
    const std::uint16_t H = static_cast<std::uint16_t>(r.below(6) == 0 ? r.below(5) : (r.below(8) == 0 ? L + r.below(2) : 14 + r.below(60)));
    const bool ins = r.below(2), strip = r.below(2), present = r.below(3) == 0;
    const std::uint16_t tag = static_cast<std::uint16_t>(r.u32());
    std::uint64_t off = frames.size();
    frames.insert(frames.end(), pkt.begin(), pkt.end());
    while (frames.size() % 16) frames.push_back(r.byte());
    frames.insert(frames.end(), 16 * r.below(2), 0xEE);

    const std::size_t slot = 9216 + 64, nrx = 70;
    HostMemoryConfig mc{.size_bytes = slot * (nrx + 2), .page_size = 4096, .iommu_enabled = false};
    SimpleHostMemory mem{mc};
    DMAEngine dma{mem};
    QueuePairConfig qc{
        .queue_id = 0,
        .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = 4, .base_address = 0, .queue_id = 0, .host_backed = false},
        .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = 0, .queue_id = 0, .host_backed = false},
        .tx_completion = {.ring_size = 4, .queue_id = 0},
        .rx_completion = {.ring_size = nrx + 1, .queue_id = 0},
    };
    QueuePair qp{qc, dma};
    assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(pkt))).ok());
    TxDescriptor tx{.buffer_address = 0, .length = static_cast<std::uint32_t>(L), .checksum = ChecksumMode::None,
                    .descriptor_index = 1, .checksum_value = 0, .tso_enabled = tso && !gso, .gso_enabled = gso,
                    .mss = mss, .header_length = H, .vlan_insert = ins, .vlan_tag = tag};
    std::vector<std::byte> tb(sizeof(TxDescriptor));
    std::memcpy(tb.data(), &tx, sizeof(tx));
    assert(qp.tx_ring().push_descriptor(tb).ok());
    for (std::size_t i = 0; i < nrx; ++i) {
      RxDescriptor rx{.buffer_address = slot * (i + 1), .buffer_length = static_cast<std::uint32_t>(slot),
                      .checksum = ChecksumMode::None, .descriptor_index = static_cast<std::uint16_t>(i),
                      .checksum_offload = false, .vlan_strip = strip, .vlan_present = present};
      std::vector<std::byte> rb(sizeof(RxDescriptor));
      std::memcpy(rb.data(), &rx, sizeof(rx));
      assert(qp.rx_ring().push_descriptor(rb).ok());
    }
    qp.process_once();
    auto tc = qp.tx_completion().poll_completion();
    std::size_t k = 0;
    while (qp.rx_completion().poll_completion()) ++k;
    // RX memory starts zeroed, so each slot holds its segment followed by
    // zeros: hash the whole slot (the test zero-pads its own segment the same
    // way); the checksum of the slot is the segment's (zeros are neutral);
    // rx_bytes pins the total delivered length.
    js << "  {\"off\": " << off << ", \"len\": " << L << ", \"hdr\": " << H << ", \"mss\": " << mss << ", \"tso\": "
       << int(tso) << ", \"insert\": " << int(ins) << ", \"tag\": " << tag << ", \"strip\": " << int(strip)
       << ", \"present\": " << int(present) << ", \"tx_status\": " << (tc ? tc->status : 99u)
       << ", \"segments\": " << k << ", \"rx_bytes\": " << qp.stats().rx_bytes << ", \"slot_fnv\": [";
    std::vector<std::uint16_t> cs;
    for (std::size_t i = 0; i < k; ++i) {
      std::vector<std::byte> buf(kSlotHash);
      assert(mem.read(slot * (i + 1), buf).ok());
      js << (i ? "," : "") << "\"" << std::hex << fnv1a(buf.data(), buf.size()) << std::dec << "\"";
      cs.push_back(nic::compute_checksum(buf));
    }
    js << "], \"seg_csum\": " << json_arr(cs) << "}" << (ci + 1 < ncase ? "," : "") << "\n";
  }
  js << " ]\n}\n";
  write_bin("tso_vlan.frames.bin", frames);
  std::ofstream(g_out + "/tso_vlan.json") << js.str();
}
}  // namespace

// ------------------------------------------- per-RSS-queue completion rings --
// The batched stage's RSS dispatch posts every Success RX completion into the
// CompletionQueue of its RSS queue (completion_queue.cpp:30-43, full rings
// refuse) and a consumer polls them (:45-53).  Reference CompletionQueues,
// one per queue (ring 64, doorbells recording every ring): three batches of
// completions with skewed queue ids, polls between the batches, a full drain
// at the end.  cq_rings.json.
void gen_cq() {
  constexpr std::size_t Q = 8, kRing = 64, kBatch = 300;
  std::mt19937_64 rng(4242);
  std::vector<std::vector<std::pair<std::uint32_t, std::uint32_t>>> rung(Q);  // per doorbell: (queue_id, data)
  std::vector<Doorbell> bells(Q);
  std::vector<std::unique_ptr<CompletionQueue>> cqs;
  std::vector<std::pair<std::uint32_t, std::uint32_t>> ring_log;  // in ring order across queues
  for (std::size_t q = 0; q < Q; ++q) {
    bells[q].set_callback([&ring_log](const DoorbellPayload& p) { ring_log.push_back({p.queue_id, p.data}); });
    cqs.push_back(std::make_unique<CompletionQueue>(
        CompletionQueueConfig{kRing, static_cast<std::uint16_t>(100 + q)}, &bells[q]));
  }
  auto entry_json = [](const CompletionEntry& e) {
    std::ostringstream o;
    o << "[" << e.queue_id << "," << e.descriptor_index << "," << e.status << "," << e.segments_produced << ","
      << e.vlan_tag << "," << (int) e.checksum_verified << "]";
    return o.str();
  };
  std::ostringstream js;
  js << "{\"ring_size\": " << kRing << ", \"queues\": " << Q << ", \"cq_queue_id_base\": 100, \"batches\": [";
  for (int b = 0; b < 3; ++b) {
    std::vector<std::uint32_t> status, queue, didx, qid, segs, vlan, ver, posted;
    ring_log.clear();
    for (std::size_t j = 0; j < kBatch; ++j) {
      CompletionEntry e;
      e.queue_id = static_cast<std::uint16_t>(rng() % 4);
      e.descriptor_index = static_cast<std::uint16_t>(b * 1000 + j);
      const auto r = rng() % 10;
      e.status = r < 8 ? 0u : static_cast<std::uint32_t>(1 + rng() % 7);
      e.segments_produced = static_cast<std::uint16_t>(1 + rng() % 3);
      e.vlan_tag = static_cast<std::uint16_t>(rng() % 4096);
      e.checksum_verified = (rng() & 1) != 0;
      // skewed RSS queues: queue 0 and 1 take most (their rings fill)
      const auto u = rng() % 16;
      const std::uint32_t q = u < 6 ? 0u : (u < 10 ? 1u : static_cast<std::uint32_t>(2 + rng() % (Q - 2)));
      bool ok = false;
      if (e.status == 0) ok = cqs[q]->post_completion(e);
      status.push_back(e.status);
      queue.push_back(q);
      didx.push_back(e.descriptor_index);
      qid.push_back(e.queue_id);
      segs.push_back(e.segments_produced);
      vlan.push_back(e.vlan_tag);
      ver.push_back(e.checksum_verified);
      posted.push_back(ok);
    }
    std::vector<std::uint32_t> bq, bd;
    for (const auto& [a, d] : ring_log) {
      bq.push_back(a);
      bd.push_back(d);
    }
    // the consumer polls some of every ring before the next batch
    std::vector<std::uint32_t> polls(Q);
    std::ostringstream polled;
    polled << "[";
    for (std::size_t q = 0; q < Q; ++q) {
      polls[q] = static_cast<std::uint32_t>(rng() % 48);
      polled << (q ? "," : "") << "[";
      for (std::uint32_t k = 0; k < polls[q]; ++k) {
        const auto e = cqs[q]->poll_completion();
        if (!e) break;
        polled << (k ? "," : "") << entry_json(*e);
      }
      polled << "]";
    }
    polled << "]";
    js << (b ? "," : "") << "{\"status\": " << json_arr(status) << ", \"rss_queue\": " << json_arr(queue)
       << ", \"descriptor_index\": " << json_arr(didx) << ", \"queue_id\": " << json_arr(qid)
       << ", \"segments\": " << json_arr(segs) << ", \"vlan\": " << json_arr(vlan) << ", \"verified\": " << json_arr(ver)
       << ", \"posted\": " << json_arr(posted) << ", \"doorbell_queue\": " << json_arr(bq)
       << ", \"doorbell_data\": " << json_arr(bd) << ", \"polls\": " << json_arr(polls) << ", \"polled\": " << polled.str()
       << "}";
  }
  js << "], \"available_end\": [";
  for (std::size_t q = 0; q < Q; ++q) js << (q ? "," : "") << cqs[q]->available();
  js << "], \"drain\": [";
  for (std::size_t q = 0; q < Q; ++q) {
    js << (q ? "," : "") << "[";
    bool first = true;
    while (auto e = cqs[q]->poll_completion()) {
      js << (first ? "" : ",") << entry_json(*e);
      first = false;
    }
    js << "]";
  }
  js << "]}";
  std::ofstream(g_out + "/cq_rings.json") << js.str();
}

int main(int argc, char** argv) {
  if (argc > 1) g_out = argv[1];
  // Sanity: the reference reproduces the Microsoft verification vector.
  {
    RssConfig rc;
    rc.key = kMsKey;
    RssEngine e{rc};
    auto t = tuple12(ip(66, 9, 149, 187), ip(161, 142, 100, 80), 2794, 1766);
    if (e.hash(std::span<const std::uint8_t>(t)) != 0x51ccc178u) { std::fprintf(stderr, "MS vector mismatch\n"); return 1; }
    if (e.hash(std::span<const std::uint8_t>(t.data(), 8)) != 0x323e8fc2u) { std::fprintf(stderr, "MS vector mismatch\n"); return 1; }
  }
  if (argc > 2 && std::string(argv[2]) == "cq") {  // only the completion-ring fixture
    gen_cq();
    std::printf("cq fixture written to %s\n", g_out.c_str());
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "qm") {  // only the QueueManager fixtures
    gen_qm();
    gen_qm_scale(808);
    std::printf("qm fixtures written to %s\n", g_out.c_str());
    return 0;
  }
  gen_checksum();
  gen_rss();
  gen_rx_mix();
  gen_c1();
  gen_tso();
  gen_qp_batch();
  gen_l34();
  gen_tso_vlan();
  gen_qm();
  gen_qm_scale(808);
  gen_cq();
  std::printf("golden fixtures written to %s\n", g_out.c_str());
  return 0;
}
