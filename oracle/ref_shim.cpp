// ref_shim.cpp — extern "C" handle onto the COMPILED REFERENCE hot path.
//
// TEST / BASELINE INFRASTRUCTURE ONLY.  oracle/Makefile links this file with
// /root/reference/src/checksum.cpp and src/rss.cpp (by path, never copied) into
// oracle/_ref/libref.so.  tests/ use it to validate the oracle restatement;
// bench.py times it as the "reference" CPU baseline (cpu_baseline.kind) on the
// GPU box's host cores.  The product never loads it.

#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "nic/checksum.h"
#include "nic/rss.h"
#include "oracle.h"

extern "C" {

std::uint16_t ref_compute_checksum(const std::uint8_t* p, std::size_t n) {
  return nic::compute_checksum(std::span<const std::byte>(reinterpret_cast<const std::byte*>(p), n));
}

std::uint32_t ref_toeplitz(const std::uint8_t* key, std::size_t key_len, const std::uint8_t* data,
                           std::size_t n) {
  nic::RssConfig c;
  c.key.assign(key, key + key_len);
  nic::RssEngine e{c};
  return e.hash(std::span<const std::uint8_t>(data, n));
}

// The reference's RX path over a batch, one RssEngine per thread (rss.h:43 is
// not thread-safe): per packet compute_checksum(frame) then
// select_queue(tuple) with the oracle's tuple extraction (the reference has no
// parser).  Shards are contiguous packet ranges.  Returns the total hashes
// counted by the engines (== n).
std::uint64_t ref_rx_batch(const std::uint8_t* frames, const std::uint64_t* desc, std::size_t n,
                           int mode, const std::uint8_t* key, std::size_t key_len,
                           const std::uint16_t* table, std::size_t table_n, std::uint16_t* csum,
                           std::uint16_t* queue, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  std::vector<std::uint64_t> counts(static_cast<std::size_t>(nthreads), 0);
  auto work = [&](int t) {
    nic::RssConfig c;
    c.key.assign(key, key + key_len);
    c.table.assign(table, table + table_n);
    nic::RssEngine eng{c};
    std::size_t lo = n * static_cast<std::size_t>(t) / static_cast<std::size_t>(nthreads);
    std::size_t hi = n * static_cast<std::size_t>(t + 1) / static_cast<std::size_t>(nthreads);
    std::uint8_t tuple[64];
    for (std::size_t i = lo; i < hi; ++i) {
      std::uint64_t off = desc[i] & ((1ull << 40) - 1);
      std::size_t len = static_cast<std::size_t>(desc[i] >> 40);
      const std::uint8_t* f = frames + off;
      csum[i] = ref_compute_checksum(f, len);
      if (mode == ORACLE_TUPLE_NONE) continue;
      std::size_t tl = oracle_extract_tuple(f, len, mode, 0, 0, tuple);
      auto q = eng.select_queue(std::span<const std::uint8_t>(tuple, tl));
      queue[i] = *q;
    }
    counts[static_cast<std::size_t>(t)] = eng.stats().hashes;
  };
  if (nthreads == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < nthreads; ++t) ts.emplace_back(work, t);
    for (auto& th : ts) th.join();
  }
  std::uint64_t total = 0;
  for (auto c : counts) total += c;
  return total;
}
}
