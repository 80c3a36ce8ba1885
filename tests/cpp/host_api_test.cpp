// host_api_test.cpp — the drop-in nic:: API on the CPU, assert-style like the
// reference's tests (tests/coverage_test.cpp:52-67, tests/queue_manager_rss_test.cpp,
// tests/tutorial_lesson8_test.cpp).  Cross-checked against the oracle
// restatement (oracle/oracle.c, pinned to the reference's golden vectors).
#undef NDEBUG
#include <cassert>
#include <cstdio>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "nic/checksum.h"
#include "nic/offload.h"
#include "nic/rss.h"
#include "nic/tx_rx.h"
#include "nicgpu.h"
#include "oracle.h"

using namespace nic;

namespace {

std::vector<std::byte> bytes(std::initializer_list<int> v) {
  std::vector<std::byte> out;
  for (int x : v) out.push_back(std::byte(static_cast<unsigned char>(x)));
  return out;
}

std::vector<std::byte> incrementing(std::size_t n) {
  std::vector<std::byte> d(n);
  for (std::size_t i = 0; i < n; ++i) d[i] = std::byte(static_cast<unsigned char>(i & 0xFF));
  return d;
}

void test_checksum_kats() {
  // tests/coverage_test.cpp:52-67
  auto even = bytes({0xFF, 0xFF, 0xFF, 0xFF});
  assert(compute_checksum(even) == 0x0000);
  assert(verify_checksum(even, 0));
  assert(!verify_checksum(even, 1));
  assert(compute_checksum(bytes({0x01, 0x02, 0x03})) == 0xFBFD);
  assert(compute_checksum(bytes({0xFF, 0xFF, 0xFF})) == 0x00FF);
  assert(compute_checksum(bytes({0xFF, 0xFF})) == 0x0000);  // tx_rx_test.cpp:855
  assert(compute_checksum({}) == 0xFFFF);                   // empty -> ChecksumError path
  assert(compute_checksum(bytes({0, 0, 0, 0})) == 0xFFFF);
  // incrementing payloads (tx_rx_test.cpp:103-110), values from the compiled reference
  const std::pair<std::size_t, std::uint16_t> inc[] = {{6, 0xF9F6},  {8, 0xF3EF},    {12, 0xE1DB},  {16, 0xC7BF},
                                                       {64, 0x1BFC}, {1518, 0x2D39}, {9000, 0x39B7}};
  for (auto [n, v] : inc) assert(compute_checksum(incrementing(n)) == v);
}

void test_checksum_random_vs_oracle() {
  std::mt19937_64 rng(1);
  for (int t = 0; t < 20000; ++t) {
    std::size_t n = rng() % 2100;
    if (t % 7 == 0) n = rng() % 20;
    std::vector<std::byte> d(n);
    const int pat = static_cast<int>(rng() % 4);
    for (auto& b : d) b = std::byte(static_cast<unsigned char>(pat == 0 ? 0xFF : pat == 1 ? 0 : rng()));
    const auto* p = reinterpret_cast<const std::uint8_t*>(d.data());
    assert(compute_checksum(d) == oracle_compute_checksum(p, n));
  }
}

void test_rss_reference_cases() {
  {  // queue_manager_rss_test.cpp:34-50
    RssConfig cfg{};
    cfg.table.assign(4, 2);
    RssEngine rss{cfg};
    std::uint8_t data[]{0x01, 0x02, 0x03, 0x04};
    auto q = rss.select_queue(std::span<const std::uint8_t>(data));
    assert(q.has_value() && *q == 2);
    assert(rss.stats().hashes == 1);
    assert(std::accumulate(rss.stats().queue_hits.begin(), rss.stats().queue_hits.end(), std::uint64_t{0}) == 1);
  }
  {  // queue_manager_rss_test.cpp:263-285 (default 20-B key)
    RssConfig cfg{};
    cfg.table = {0, 1, 2, 3};
    RssEngine rss{cfg};
    std::uint8_t d0[]{0xAA, 0xBB, 0xCC, 0xDD}, d1[]{0x10, 0x20, 0x30, 0x40}, d2[]{0x01, 0x00, 0x00, 0x01};
    RssEngine probe{cfg};
    assert(probe.hash(d0) == 0x7ECE5995u && probe.hash(d1) == 0x3FB73D4Au && probe.hash(d2) == 0x1F8C0605u);
    assert(*rss.select_queue(d0) == 1 && *rss.select_queue(d1) == 2 && *rss.select_queue(d2) == 1);
    assert(rss.stats().hashes == 3);
  }
  {  // queue_manager_rss_test.cpp:287-313
    RssConfig cfg{};
    cfg.table = {0, 1};
    RssEngine rss{cfg};
    std::uint8_t d0[]{0x00, 0x00, 0x00, 0x01}, d1[]{0xFF, 0xEE, 0xDD, 0xCC}, d2[]{0x12, 0x34, 0x56, 0x78};
    assert(*rss.select_queue(d0) == 1 && *rss.select_queue(d1) == 0 && *rss.select_queue(d2) == 0);
    assert(rss.stats().queue_hits.size() == 2 && rss.stats().queue_hits[0] == 2 && rss.stats().queue_hits[1] == 1);
  }
  {  // queue_manager_rss_test.cpp:315-330
    RssEngine rss;
    rss.set_key({});
    rss.set_table({});
    std::vector<std::uint8_t> empty;
    assert(rss.hash(empty) == 0);
    assert(rss.stats().hashes >= 1);
    rss.reset_stats();
    assert(rss.stats().hashes == 0);
    assert(rss.config().key.size() == 20 && rss.config().table.size() == 128);
  }
  {  // tutorial_lesson8_test.cpp:94-160 + Microsoft verification suite + users_guide.md:2000-2020
    const std::vector<std::uint8_t> ms = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
                                          0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
                                          0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
    RssConfig cfg{ms, {0, 1, 2, 3, 0, 1, 2, 3}};
    RssEngine rss{cfg};
    std::uint8_t fwd[]{192, 168, 1, 100, 192, 168, 1, 1, 0x1F, 0x90, 0x00, 0x50};
    std::uint8_t rev[]{192, 168, 1, 1, 192, 168, 1, 100, 0x00, 0x50, 0x1F, 0x90};
    assert(rss.hash(fwd) == 0x682DA0B1u);
    assert(*rss.select_queue(fwd) == 1 && *rss.select_queue(rev) == 3);
    std::uint8_t msv[]{66, 9, 149, 187, 161, 142, 100, 80, 0x0A, 0xEA, 0x06, 0xE6};
    assert(rss.hash(msv) == 0x51CCC178u);
    assert(rss.hash(std::span<const std::uint8_t>(msv, 8)) == 0x323E8FC2u);
    RssEngine m6d{RssConfig{std::vector<std::uint8_t>(40, 0x6D), {0, 1, 2, 3}}};
    assert(m6d.hash(fwd) == 0x3E3E3E3Eu && *m6d.select_queue(fwd) == 2);
  }
  {  // key wrap: 36-B input longer than the 20-B default key (rss.cpp:83-89)
    std::uint8_t d[36];
    for (int i = 0; i < 36; ++i) d[i] = static_cast<std::uint8_t>(i * 7 + 1);
    RssEngine rss;
    assert(rss.hash(d) == 0x9406BF72u);
  }
  {  // queue_hits guard: set_table grows the table, queue_hits stays 128 (rss.cpp:56-58, 107)
    RssEngine rss;
    std::vector<std::uint16_t> big(200);
    for (std::size_t i = 0; i < big.size(); ++i) big[i] = static_cast<std::uint16_t>(i % 5);
    rss.set_table(big);
    std::mt19937 rng(3);
    std::uint64_t counted = 0;
    for (int i = 0; i < 1000; ++i) {
      std::uint8_t d[12];
      for (auto& b : d) b = static_cast<std::uint8_t>(rng());
      const std::uint32_t idx = RssEngine{rss.config()}.hash(d) % 200;
      (void) rss.select_queue(d);
      if (idx < 128) ++counted;
    }
    assert(rss.stats().queue_hits.size() == 128);
    assert(std::accumulate(rss.stats().queue_hits.begin(), rss.stats().queue_hits.end(), std::uint64_t{0}) == counted);
    assert(rss.stats().hashes == 1000);
  }
}

void test_rss_random_vs_oracle() {
  std::mt19937_64 rng(2);
  for (int t = 0; t < 3000; ++t) {
    std::vector<std::uint8_t> key(1 + rng() % 80), data(rng() % 100);
    for (auto& b : key) b = static_cast<std::uint8_t>(rng());
    for (auto& b : data) b = static_cast<std::uint8_t>(rng());
    std::vector<std::uint16_t> table(1 + rng() % 300);
    for (auto& e : table) e = static_cast<std::uint16_t>(rng());
    RssEngine rss{RssConfig{key, table}};
    std::uint32_t h = 0, idx = 0;
    const std::uint16_t q = oracle_select_queue(key.data(), key.size(), table.data(), table.size(), data.data(),
                                                data.size(), &h, &idx);
    assert(rss.hash(data) == h);
    assert(*rss.select_queue(data) == q);
  }
}

// The GPU batch path's limits (include/nic/rss.h, select_queue_batch): a
// table over NICGPU_MAX_TABLE is refused with NICGPU_ERR_INVALID before any
// device work (so this runs without a GPU), while select_queue takes it, as
// the reference's does (src/rss.cpp:35-41, 49-61).
void test_batch_limits() {
  std::vector<std::uint16_t> table(static_cast<std::size_t>(NICGPU_MAX_TABLE) + 1);
  for (std::size_t i = 0; i < table.size(); ++i) table[i] = static_cast<std::uint16_t>(i * 7);
  RssEngine e{RssConfig{{}, table}};
  bool threw = false;
  try {
    e.select_queue_batch(DevicePacketBatch{nullptr, nullptr, 0}, TupleSpec{}, RxBatchOutputs{});
  } catch (const GpuError& g) {
    threw = g.status() == NICGPU_ERR_INVALID && std::string(g.what()).find("NICGPU_MAX_TABLE") != std::string::npos;
  }
  assert(threw);
  assert(e.stats().hashes == 0);
  const std::uint8_t tuple[12] = {192, 168, 1, 100, 192, 168, 1, 1, 0x1F, 0x90, 0, 80};
  std::uint32_t h = 0, idx = 0;
  const std::uint16_t q = oracle_select_queue(e.config().key.data(), e.config().key.size(), table.data(), table.size(),
                                              tuple, sizeof(tuple), &h, &idx);
  assert(*e.select_queue(tuple) == q && e.stats().hashes == 1);
  // keys longer than NICGPU_MAX_KEY hash like their first NICGPU_MAX_KEY bytes
  // for every tuple the GPU path can hand over (<= NICGPU_MAX_TUPLE bytes):
  // no key bit past 8 * 64 + 31 is read (what select_queue_batch relies on)
  std::mt19937_64 rng(5);
  for (int it = 0; it < 50; ++it) {
    std::vector<std::uint8_t> key(NICGPU_MAX_KEY + 1 + rng() % 300), data(1 + rng() % NICGPU_MAX_TUPLE);
    for (auto& b : key) b = static_cast<std::uint8_t>(rng());
    for (auto& b : data) b = static_cast<std::uint8_t>(rng());
    const std::vector<std::uint8_t> head(key.begin(), key.begin() + NICGPU_MAX_KEY);
    const RssEngine full{RssConfig{key, {1}}}, cut{RssConfig{head, {1}}};
    assert(full.hash(data) == cut.hash(data));
  }
}

void test_abi_layouts() {
  static_assert(sizeof(TxDescriptor) == 32 && sizeof(RxDescriptor) == 24);
  assert(kMaxTsoSegments == 64 && kMaxMss == 9000 && kJumboMtu == 9000 && kMaxJumboFrame == 9216);
  assert(static_cast<int>(CompletionCode::ChecksumError) == 2);
}

}  // namespace

int main() {
  test_checksum_kats();
  test_checksum_random_vs_oracle();
  test_rss_reference_cases();
  test_rss_random_vs_oracle();
  test_abi_layouts();
  test_batch_limits();
  std::puts("host_api_test: ok");
  return 0;
}
