// gpu_batch_test.cpp — the GPU batch entry points of the nic:: API against
// the same API's per-packet calls (and therefore against the reference
// semantics pinned by host_api_test).  Needs an MI355X.
//
// nic::compute_checksum_batch        vs nic::compute_checksum per frame
// nic::RssEngine::select_queue_batch vs nic::RssEngine::select_queue per tuple,
//                                       including RssStats after the batch.
// nic::RssEngine::select_queue_batch_enqueue (device count) + account_batch
//                                    vs select_queue_batch over that count.
#undef NDEBUG
#include <cassert>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "nic/checksum.h"
#include "nic/rss.h"
#include "nicgpu.h"
#include "oracle.h"

using namespace nic;

namespace {

struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(std::size_t n) { assert(nicgpu_malloc(&p, n ? n : 16) == NICGPU_OK); }
  ~DevBuf() { nicgpu_free(p); }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

template <class T>
void to_dev(const DevBuf& d, const std::vector<T>& v) {
  assert(nicgpu_memcpy_async(d.p, v.data(), v.size() * sizeof(T), nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
}

template <class T>
std::vector<T> from_dev(const DevBuf& d, std::size_t n) {
  std::vector<T> v(n);
  assert(nicgpu_memcpy_async(v.data(), d.p, n * sizeof(T), nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  return v;
}

// Eth/IPv4/TCP-ish frames with random fields, packed at random byte offsets.
void make_batch(std::mt19937_64& rng, std::size_t n, std::vector<std::uint8_t>& frames, std::vector<std::uint64_t>& desc) {
  frames.clear();
  desc.clear();
  for (std::size_t i = 0; i < n; ++i) {
    std::size_t len = (rng() % 3 == 0) ? rng() % 60 : 54 + rng() % 1500;
    if (rng() % 50 == 0) len = 0;
    const std::size_t gap = (rng() % 4 == 0) ? rng() % 16 : (16 - frames.size() % 16) % 16;
    for (std::size_t g = 0; g < gap; ++g) frames.push_back(static_cast<std::uint8_t>(rng()));
    const std::size_t off = frames.size();
    for (std::size_t b = 0; b < len; ++b) frames.push_back(static_cast<std::uint8_t>(rng()));
    if (len >= 38 && rng() % 4 != 0) {
      std::uint8_t* f = frames.data() + off;
      f[12] = 0x08; f[13] = 0x00; f[14] = 0x45; f[20] = 0x40; f[21] = 0; f[23] = (rng() & 1) ? 6 : 17;
    }
    desc.push_back(NICGPU_DESC(off, len));
  }
  frames.resize(frames.size() + 64, 0);
}

void test_checksum_batch(std::mt19937_64& rng) {
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  make_batch(rng, 5000, frames, desc);
  DevBuf f(frames.size()), d(desc.size() * 8), o(desc.size() * 2);
  to_dev(f, frames);
  to_dev(d, desc);
  compute_checksum_batch(DevicePacketBatch{f.as<std::byte>(), d.as<std::uint64_t>(), desc.size()}, o.as<std::uint16_t>());
  auto got = from_dev<std::uint16_t>(o, desc.size());
  for (std::size_t i = 0; i < desc.size(); ++i) {
    const std::size_t off = desc[i] & ((1ull << 40) - 1), len = desc[i] >> 40;
    const auto* p = reinterpret_cast<const std::byte*>(frames.data() + off);
    assert(got[i] == compute_checksum(std::span<const std::byte>(p, len)));
  }
}

void test_select_queue_batch(std::mt19937_64& rng, const std::vector<std::uint8_t>& key, std::vector<std::uint16_t> table,
                             TupleSpec tuple, bool grow_table = true) {
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  make_batch(rng, 4000, frames, desc);
  const std::size_t n = desc.size();
  DevBuf f(frames.size()), d(n * 8), cs(n * 2), hs(n * 4), qs(n * 2);
  to_dev(f, frames);
  to_dev(d, desc);
  RssEngine gpu_engine{RssConfig{key, table}};
  RssEngine cpu_engine{RssConfig{key, table}};
  const DevicePacketBatch batch{f.as<std::byte>(), d.as<std::uint64_t>(), n};
  gpu_engine.select_queue_batch(batch, tuple, RxBatchOutputs{cs.as<std::uint16_t>(), hs.as<std::uint32_t>(), qs.as<std::uint16_t>()});
  auto c = from_dev<std::uint16_t>(cs, n);
  auto h = from_dev<std::uint32_t>(hs, n);
  auto q = from_dev<std::uint16_t>(qs, n);
  RssEngine probe{RssConfig{key, table}};
  for (std::size_t i = 0; i < n; ++i) {
    const std::size_t off = desc[i] & ((1ull << 40) - 1), len = desc[i] >> 40;
    const std::uint8_t* p = frames.data() + off;
    std::uint8_t t[64];
    const std::size_t tl = oracle_extract_tuple(p, len, static_cast<int>(tuple.mode), tuple.raw_offset, tuple.raw_length, t);
    const std::span<const std::uint8_t> sp(t, tl);
    assert(c[i] == compute_checksum(std::span<const std::byte>(reinterpret_cast<const std::byte*>(p), len)));
    assert(h[i] == probe.hash(sp));
    assert(q[i] == *cpu_engine.select_queue(sp));
  }
  // stats identical to n sequential select_queue calls
  assert(gpu_engine.stats().hashes == cpu_engine.stats().hashes);
  assert(gpu_engine.stats().queue_hits == cpu_engine.stats().queue_hits);
  // a second batch accumulates
  gpu_engine.select_queue_batch(batch, tuple, RxBatchOutputs{nullptr, nullptr, qs.as<std::uint16_t>()});
  assert(gpu_engine.stats().hashes == 2 * n);
  if (!grow_table) return;
  // set_table invalidates the device table; queue_hits keeps its size
  const std::size_t hits_size = gpu_engine.stats().queue_hits.size();
  assert(hits_size == cpu_engine.config().table.size());
  std::vector<std::uint16_t> t2(hits_size + 50, 7);
  gpu_engine.set_table(t2);
  gpu_engine.select_queue_batch(batch, tuple, RxBatchOutputs{nullptr, nullptr, qs.as<std::uint16_t>()});
  auto q2 = from_dev<std::uint16_t>(qs, n);
  for (auto v : q2) assert(v == 7);
  assert(gpu_engine.stats().queue_hits.size() == hits_size);
}

// select_queue_batch_enqueue over a device count + account_batch equals
// select_queue_batch over the first `count` packets (outputs past the count
// untouched, stats identical).
void test_enqueue_count(std::mt19937_64& rng, const std::vector<std::uint8_t>& key, const std::vector<std::uint16_t>& table) {
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  make_batch(rng, 3000, frames, desc);
  const std::size_t n = desc.size();
  for (const std::size_t count : {std::size_t{0}, std::size_t{1}, std::size_t{63}, std::size_t{1777}, n}) {
    DevBuf f(frames.size()), d(n * 8), hs(n * 4), qs(n * 2), hs2(n * 4), qs2(n * 2), cnt(8), hits(table.size() * 8);
    to_dev(f, frames);
    to_dev(d, desc);
    to_dev(cnt, std::vector<std::uint64_t>{count});
    const std::vector<std::uint32_t> fill_h(n, 0xA5A5A5A5u);
    const std::vector<std::uint16_t> fill_q(n, 0x5A5Au);
    to_dev(hs, fill_h);
    to_dev(qs, fill_q);
    to_dev(hits, std::vector<std::uint64_t>(table.size(), 0));
    RssEngine a{RssConfig{key, table}}, b{RssConfig{key, table}};
    a.select_queue_batch_enqueue(DevicePacketBatch{f.as<std::byte>(), d.as<std::uint64_t>(), n}, cnt.as<std::uint64_t>(),
                                 TupleSpec{TupleMode::Auto, 0, 0},
                                 RxBatchOutputs{nullptr, hs.as<std::uint32_t>(), qs.as<std::uint16_t>()},
                                 hits.as<std::uint64_t>());
    const auto h_hits = from_dev<std::uint64_t>(hits, table.size());
    a.account_batch(count, h_hits);
    if (count)
      b.select_queue_batch(DevicePacketBatch{f.as<std::byte>(), d.as<std::uint64_t>(), count},
                           TupleSpec{TupleMode::Auto, 0, 0},
                           RxBatchOutputs{nullptr, hs2.as<std::uint32_t>(), qs2.as<std::uint16_t>()});
    const auto h = from_dev<std::uint32_t>(hs, n), h2 = from_dev<std::uint32_t>(hs2, n);
    const auto q = from_dev<std::uint16_t>(qs, n), q2 = from_dev<std::uint16_t>(qs2, n);
    for (std::size_t i = 0; i < n; ++i) {
      if (i < count) {
        assert(h[i] == h2[i] && q[i] == q2[i]);
      } else {
        assert(h[i] == 0xA5A5A5A5u && q[i] == 0x5A5Au);
      }
    }
    assert(a.stats().hashes == b.stats().hashes && a.stats().queue_hits == b.stats().queue_hits);
  }
}

void test_errors() {
  bool threw = false;
  try {
    compute_checksum_batch(DevicePacketBatch{reinterpret_cast<const std::byte*>(0x1), nullptr, 3}, nullptr);
  } catch (const GpuError& e) {
    threw = e.status() == NICGPU_ERR_INVALID;
  }
  assert(threw);
}

}  // namespace

int main() {
  assert(gpu_device_count() >= 1);
  std::mt19937_64 rng(11);
  test_checksum_batch(rng);
  const std::vector<std::uint8_t> ms = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
                                        0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
                                        0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
  std::vector<std::uint16_t> t16(128);
  for (int i = 0; i < 128; ++i) t16[i] = static_cast<std::uint16_t>(i % 16);
  test_select_queue_batch(rng, ms, t16, TupleSpec{TupleMode::Auto, 0, 0});
  test_enqueue_count(rng, ms, t16);
  test_select_queue_batch(rng, {}, {}, TupleSpec{TupleMode::Auto, 0, 0});         // reference defaults
  test_select_queue_batch(rng, {}, {0, 1, 2, 3, 4, 5, 6}, TupleSpec{TupleMode::Raw, 26, 36});  // key wrap
  std::vector<std::uint16_t> big(3000);
  for (std::size_t i = 0; i < big.size(); ++i) big[i] = static_cast<std::uint16_t>(i);
  test_select_queue_batch(rng, ms, big, TupleSpec{TupleMode::Auto, 0, 0});        // table > LDS histogram
  // keys past NICGPU_MAX_KEY (truncated for the device, exactly) and the
  // largest tuples; tables past the reference-typical sizes up to the limit
  std::vector<std::uint8_t> long_key(NICGPU_MAX_KEY + 77);
  for (auto& b : long_key) b = static_cast<std::uint8_t>(rng());
  test_select_queue_batch(rng, long_key, t16, TupleSpec{TupleMode::Raw, 0, 64});
  test_select_queue_batch(rng, std::vector<std::uint8_t>(long_key.begin(), long_key.begin() + NICGPU_MAX_KEY), t16,
                          TupleSpec{TupleMode::Auto, 0, 0});
  std::vector<std::uint16_t> t65537(65537);
  for (std::size_t i = 0; i < t65537.size(); ++i) t65537[i] = static_cast<std::uint16_t>(i * 3);
  test_select_queue_batch(rng, ms, t65537, TupleSpec{TupleMode::Auto, 0, 0});
  std::vector<std::uint16_t> tmax(NICGPU_MAX_TABLE);
  for (std::size_t i = 0; i < tmax.size(); ++i) tmax[i] = static_cast<std::uint16_t>(i ^ (i >> 16));
  test_select_queue_batch(rng, ms, tmax, TupleSpec{TupleMode::Raw, 0, 64}, false);
  test_errors();
  std::puts("gpu_batch_test: ok");
  return 0;
}
