// ref_qp_bench.cpp — CPU baseline of SURVEY §8 rows f1 and f2 (TEST/MEASUREMENT
// INFRASTRUCTURE ONLY): the reference's own QueuePair::process_once
// (src/queue_pair.cpp:67-460, compiled from /root/reference by
// `make -C oracle ref`; no reference source is copied) over the batches
// tools/bench_rx_stage.cpp and tools/bench_rows.py give the GPU:
//   c3     IMIX 64/576/1518 (7:4:1) frames, each balanced so the whole-frame
//          checksum verifies, TX checksum offload, RX descriptors with Layer4
//          checksum offload and 2 KiB buffers (row f1);
//   c5seg  9000 B frames with TSO (H 54, mss 1448 -> 7 segments), RX verify
//          off, 1600 B RX buffers: every segment built and DMA-written, the
//          reference's build_segments + handle_rx_segment (row f2,
//          materialised segmentation);
//   c5     the same frames with Layer4 RX verify on: random payloads fail the
//          first segment's checksum and end the packet there (row f1's C5).
// One thread (the reference is single-threaded).  Prints one JSON line:
// descriptors per second through push + process_once + poll.
//
//   ref_qp_bench [tx_descriptors] [reps] [c3|c5seg|c5]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "nic/dma_engine.h"
#include "nic/queue_pair.h"
#include "nic/simple_host_memory.h"

using namespace nic;

namespace {

std::uint16_t csum(const std::uint8_t* p, std::size_t n) {
  std::uint64_t s = 0;
  for (std::size_t i = 0; i + 1 < n; i += 2) s += (std::uint32_t{p[i]} << 8) | p[i + 1];
  if (n & 1) s += std::uint32_t{p[n - 1]} << 8;
  while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
  return static_cast<std::uint16_t>(~s);
}

}  // namespace

int main(int argc, char** argv) {
  const std::size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 18);
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  const bool c5v = argc > 3 && std::strcmp(argv[3], "c5") == 0;  // TSO, RX verify on
  const bool seg = c5v || (argc > 3 && std::strcmp(argv[3], "c5seg") == 0);
  std::mt19937_64 rng(7);
  std::vector<std::size_t> lens(n);
  for (auto& L : lens) {
    const auto r = rng() % 12;
    L = seg ? 9000 : (r < 7 ? 64 : (r < 11 ? 576 : 1518));
  }
  std::size_t tx_bytes = 0;
  for (auto L : lens) tx_bytes += (L + 15) & ~std::size_t{15};
  const std::size_t rx_buf = seg ? 1600 : 2048;
  const std::size_t nrx = seg ? n * 7 : n;
  const std::size_t mem_size = tx_bytes + nrx * rx_buf;
  std::vector<std::uint8_t> img(tx_bytes);
  std::vector<TxDescriptor> tx(n);
  std::size_t at = 0, frame_bytes = 0;
  for (std::size_t i = 0; i < n; ++i) {
    std::uint8_t* p = img.data() + at;
    for (std::size_t b = 0; b < lens[i]; b += 8) {
      const std::uint64_t r = rng();
      std::memcpy(p + b, &r, std::min<std::size_t>(8, lens[i] - b));
    }
    p[12] = 0x08;
    p[13] = 0x00;
    p[10] = p[11] = 0;
    const std::uint16_t c = csum(p, lens[i]);
    p[10] = static_cast<std::uint8_t>(c >> 8);
    p[11] = static_cast<std::uint8_t>(c);
    TxDescriptor& t = tx[i];
    t.buffer_address = at;
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum_offload = true;
    t.checksum = ChecksumMode::Layer4;
    if (seg) {
      t.tso_enabled = true;
      t.mss = 1448;
      t.header_length = 54;
    }
    at += (lens[i] + 15) & ~std::size_t{15};
    frame_bytes += lens[i];
  }
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    rx[j].buffer_address = tx_bytes + j * rx_buf;
    rx[j].buffer_length = static_cast<std::uint32_t>(rx_buf);
    rx[j].descriptor_index = static_cast<std::uint16_t>(j);
    rx[j].checksum_offload = !seg || c5v;
    rx[j].checksum = seg && !c5v ? ChecksumMode::None : ChecksumMode::Layer4;
  }
  SimpleHostMemory mem{HostMemoryConfig{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = false}};
  if (!mem.write(0, std::as_bytes(std::span<const std::uint8_t>(img))).ok()) return 1;
  DMAEngine dma{mem};
  std::vector<double> secs;
  std::size_t ok = 0;
  for (int r = 0; r < reps; ++r) {
    QueuePairConfig qc{
        .queue_id = 1,
        .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = n + 1, .base_address = 0, .queue_id = 1, .host_backed = false},
        .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = 0, .queue_id = 1, .host_backed = false},
        .tx_completion = {.ring_size = n + 1, .queue_id = 1},
        .rx_completion = {.ring_size = nrx + 1, .queue_id = 1},
    };
    QueuePair qp{qc, dma};
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::byte> b(sizeof(TxDescriptor));
    for (const auto& t : tx) {
      std::memcpy(b.data(), &t, sizeof(t));
      if (!qp.tx_ring().push_descriptor(b).ok()) return 2;
    }
    std::vector<std::byte> br(sizeof(RxDescriptor));
    for (const auto& x : rx) {
      std::memcpy(br.data(), &x, sizeof(x));
      if (!qp.rx_ring().push_descriptor(br).ok()) return 3;
    }
    while (qp.process_once()) {
    }
    ok = 0;
    while (auto c = qp.rx_completion().poll_completion()) ok += c->status == static_cast<std::uint32_t>(CompletionCode::Success);
    while (auto c = qp.tx_completion().poll_completion()) {
    }
    secs.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(secs.begin(), secs.end());
  const double med = secs[secs.size() / 2];
  if (c5v)
    std::printf("{\"row\": \"f1_c5\", \"value\": %.4f, \"unit\": \"Mpkt/s\", \"cores\": 1, \"kind\": \"reference\", "
                "\"gbs\": %.4f, \"rx_success\": %zu, \"sample\": \"%zu x 9000 B TSO frames (H 54, mss 1448) through the "
                "reference QueuePair::process_once with Layer4 RX verify: each ends at its first segment's checksum; median "
                "of %d\"}\n",
                n / med / 1e6, frame_bytes / med / 1e9, ok, n, reps);
  else if (seg)
    std::printf("{\"row\": \"tso_seg_c5\", \"value\": %.4f, \"unit\": \"Mpkt/s\", \"cores\": 1, \"kind\": \"reference\", "
                "\"gbs\": %.4f, \"rx_success\": %zu, \"sample\": \"%zu x 9000 B TSO frames (H 54, mss 1448, 7 segments each) "
                "through the reference QueuePair::process_once (push, process, poll): every segment built and written "
                "into 1600 B RX buffers, RX verify off; median of %d\"}\n",
                n / med / 1e6, frame_bytes / med / 1e9, ok, n, reps);
  else
    std::printf("{\"row\": \"f1_c3\", \"value\": %.4f, \"unit\": \"Mpkt/s\", \"cores\": 1, \"kind\": \"reference\", "
                "\"gbs\": %.4f, \"rx_success\": %zu, \"sample\": \"%zu IMIX TX descriptors (7:4:1 64/576/1518 B) "
                "through the reference QueuePair::process_once (push, process, poll), 2 KiB RX buffers, Layer4 RX "
                "verify; median of %d\"}\n",
                n / med / 1e6, frame_bytes / med / 1e9, ok, n, reps);
  return 0;
}
