// bench_rx_stage.cpp — nic::BatchedQueuePair throughput.
//
//   bench_rx_stage <workload: c3|c5|qm16> <tx_descriptors> <reps> [host_threads] [device|host] [pageable|pinned|device] [sync|pipelined] [host|device] [irq]
//   (device: BatchedQueuePair's device resolve, the default for disjoint
//   buffers; host: the host resolve, BatchedQueuePairConfig::device_resolve off;
//   pinned: the descriptor arrays in page-locked memory, as a descriptor ring
//   the device DMAs from would be, so they go up without staging; device: the
//   descriptor arrays already in device memory (DeviceDescriptors, as a
//   host-backed ring in the image would be), no upload at all; pipelined:
//   submit()/collect() with three batches in flight, reported per batch over
//   the whole run, against process_batch one batch at a time; the last
//   argument: results copied to the host vectors, or left in device memory
//   (BatchedQueuePairConfig::results_on_device)); irq: RX and TX interrupt
//   callbacks on (a counting callback, as an InterruptDispatcher delivers
//   them: queue_pair.cpp:371-383), replayed from the completions;
//   hostmem: the memory is a HostMemory (nic::FlatHostMemory, the reference
//   SimpleHostMemory's bounds rule) in host RAM, descriptors in page-locked
//   arrays — every batch stages its TX bytes up and writes its delivered bytes
//   back (process_batch(HostMemory&, ...)): the end-to-end rate from host
//   memory, PCIe included
//
// c3: IMIX 64/576/1518 (7:4:1) frames, each balanced so the whole-frame
//     checksum verifies; RX descriptors with Layer4 checksum offload, 2 KiB
//     buffers; RSS over the delivered frames (MS key, table i%16).
// The RX ring's buffers start on a 4-KiB boundary after the TX frames, as a
// driver's page-backed ring does (env NIC_BENCH_RX_ALIGN=16: right after them,
// 16-B aligned only — frames then start inside 64-B sectors, which costs the
// delivery a read-modify-write per partial sector).
// qm16: the c3 batch split over 16 queue pairs of a nic::BatchedQueueManager
//     (one process_batch drains them all; host descriptors only).
// c5: 9000-B frames with TSO (H = 54, mss = 1448 -> 7 segments), RX verify on:
//     random payloads fail on the first segment, so the batch exercises the
//     reference's first-failure abort (queue_pair.cpp:361-364).
// Host memory image and descriptors are prepared once; each rep runs
// process_batch on the same batch (the RX buffers are rewritten).  Prints one
// JSON line: packets/s, frame bytes/s and the per-phase split.
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <span>
#include <string>
#include <vector>

#include "nic/flat_host_memory.h"
#include "nic/rss.h"
#include "nic/rx_queue_manager.h"
#include "nic/rx_stage.h"
#include "nicgpu.h"

using namespace nic;

namespace {

std::uint16_t csum(const std::uint8_t* p, std::size_t n) {
  std::uint64_t s = 0;
  for (std::size_t i = 0; i + 1 < n; i += 2) s += (std::uint32_t{p[i]} << 8) | p[i + 1];
  if (n & 1) s += std::uint32_t{p[n - 1]} << 8;
  while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
  return static_cast<std::uint16_t>(~s);
}

void check(int st, const char* what) {
  if (st != NICGPU_OK) {
    std::fprintf(stderr, "%s: %s\n", what, nicgpu_strerror(st));
    std::exit(1);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const std::string wl = argc > 1 ? argv[1] : "c3";
  const std::size_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (1u << 18);
  const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
  std::mt19937_64 rng(7);
  std::vector<std::size_t> lens(n);
  for (auto& L : lens) {
    if (wl == "c5") L = 9000;
    else {
      const auto r = rng() % 12;
      L = r < 7 ? 64 : (r < 11 ? 576 : 1518);
    }
  }
  std::size_t tx_bytes = 0;
  for (auto L : lens) tx_bytes += (L + 15) & ~std::size_t{15};
  const std::size_t rx_buf = wl == "c5" ? 1600 : 2048;
  const std::size_t segs = wl == "c5" ? 7 : 1;
  const std::size_t nrx = n * segs;
  const char* ra = std::getenv("NIC_BENCH_RX_ALIGN");
  const std::size_t rx_align = ra ? std::max<std::size_t>(16, std::strtoull(ra, nullptr, 10)) : 4096;
  const std::size_t rx_base = (tx_bytes + rx_align - 1) / rx_align * rx_align;
  const std::size_t mem_size = rx_base + nrx * rx_buf;
  std::vector<std::uint8_t> tx_img(tx_bytes);
  std::vector<TxDescriptor> tx(n);
  std::size_t at = 0;
  for (std::size_t i = 0; i < n; ++i) {
    std::uint8_t* p = tx_img.data() + at;
    for (std::size_t b = 0; b < lens[i]; b += 8) {
      const std::uint64_t r = rng();
      std::memcpy(p + b, &r, std::min<std::size_t>(8, lens[i] - b));
    }
    p[12] = 0x08;
    p[13] = 0x00;
    if (wl != "c5") {  // balancing word in the source MAC: whole-frame checksum 0
      p[10] = p[11] = 0;
      const std::uint16_t c = csum(p, lens[i]);
      p[10] = static_cast<std::uint8_t>(c >> 8);
      p[11] = static_cast<std::uint8_t>(c);
    }
    TxDescriptor& t = tx[i];
    t.buffer_address = at;
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum_offload = true;
    t.checksum = ChecksumMode::Layer4;
    if (wl == "c5") {
      t.tso_enabled = true;
      t.mss = 1448;
      t.header_length = 54;
    }
    at += (lens[i] + 15) & ~std::size_t{15};
  }
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    rx[j].buffer_address = rx_base + j * rx_buf;
    rx[j].buffer_length = static_cast<std::uint32_t>(rx_buf);
    rx[j].descriptor_index = static_cast<std::uint16_t>(j);
    rx[j].checksum_offload = true;
    rx[j].checksum = ChecksumMode::Layer4;
  }
  void* mem = nullptr;
  check(nicgpu_malloc(&mem, (mem_size + 15) / 16 * 16), "nicgpu_malloc");
  check(nicgpu_memcpy_async(mem, tx_img.data(), tx_bytes, nullptr), "memcpy");
  check(nicgpu_memset_async(static_cast<std::uint8_t*>(mem) + tx_bytes, 0, mem_size - tx_bytes, nullptr), "memset");
  check(nicgpu_stream_synchronize(nullptr), "sync");

  const std::vector<std::uint8_t> ms_key = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67,
                                            0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb,
                                            0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30,
                                            0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
  std::vector<std::uint16_t> table(128);
  for (int i = 0; i < 128; ++i) table[i] = static_cast<std::uint16_t>(i % 16);
  RssEngine rss{RssConfig{ms_key, table}};
  BatchedQueuePairConfig cfg;
  cfg.queue_id = 1;
  cfg.rss = &rss;
  if (argc > 4) cfg.host_threads = static_cast<unsigned>(std::atoi(argv[4]));
  if (argc > 5) cfg.device_resolve = std::string(argv[5]) != "host";
  cfg.results_on_device = argc > 8 && std::string(argv[8]) == "device";
  if (const char* e = std::getenv("NIC_BENCH_OVERLAP"); e && *e == '1') cfg.overlap_resolve = true;  // A/B
  const bool irq = argc > 9 && std::string(argv[9]) == "irq";
  std::uint64_t irq_count = 0, irq_sum = 0;
  if (irq) {
    cfg.enable_tx_interrupts = true;
    cfg.enable_rx_interrupts = true;
    cfg.on_interrupt = [&irq_count, &irq_sum](std::uint16_t, const CompletionEntry& e) {
      ++irq_count;
      irq_sum += e.descriptor_index;
    };
  }
  const std::string desc_kind = argc > 6 ? argv[6] : "pageable";
  const bool hostmem = desc_kind == "hostmem";
  const bool pinned = desc_kind == "pinned" || hostmem, dev_desc = desc_kind == "device";
  std::unique_ptr<FlatHostMemory> hm;
  if (hostmem) {  // the same bytes in host RAM, behind the reference's HostMemory interface
    hm = std::make_unique<FlatHostMemory>(mem_size);
    std::memcpy(hm->data(), tx_img.data(), tx_bytes);
  }
  BatchedQueuePair qp{cfg};
  const DeviceHostMemory dm{static_cast<std::byte*>(mem), mem_size};
  std::span<const TxDescriptor> txs{tx};
  std::span<const RxDescriptor> rxs{rx};
  void *ptx = nullptr, *prx = nullptr;
  if (pinned) {
    check(nicgpu_host_alloc(&ptx, n * sizeof(TxDescriptor)), "nicgpu_host_alloc");
    check(nicgpu_host_alloc(&prx, nrx * sizeof(RxDescriptor)), "nicgpu_host_alloc");
    std::memcpy(ptx, tx.data(), n * sizeof(TxDescriptor));
    std::memcpy(prx, rx.data(), nrx * sizeof(RxDescriptor));
    txs = {static_cast<const TxDescriptor*>(ptx), n};
    rxs = {static_cast<const RxDescriptor*>(prx), nrx};
  }
  void *dtx = nullptr, *drx = nullptr;
  DeviceDescriptors dd;
  if (dev_desc) {
    check(nicgpu_malloc(&dtx, n * sizeof(TxDescriptor)), "nicgpu_malloc");
    check(nicgpu_malloc(&drx, nrx * sizeof(RxDescriptor)), "nicgpu_malloc");
    check(nicgpu_memcpy_async(dtx, tx.data(), n * sizeof(TxDescriptor), nullptr), "memcpy");
    check(nicgpu_memcpy_async(drx, rx.data(), nrx * sizeof(RxDescriptor), nullptr), "memcpy");
    check(nicgpu_stream_synchronize(nullptr), "sync");
    dd = {static_cast<const TxDescriptor*>(dtx), n, static_cast<const RxDescriptor*>(drx), nrx};
  }
  if (wl == "qm16") {
    // nic::BatchedQueueManager over 16 queue pairs, n / 16 C3 descriptors and
    // RX buffers each (weights 1, one RssEngine per queue pair): one
    // process_batch drains every queue, all 16 stages in flight at once
    constexpr std::size_t Q = 16;
    const std::size_t per = n / Q;
    std::vector<std::unique_ptr<RssEngine>> engines;
    BatchedQueueManagerConfig qc;
    for (std::size_t q = 0; q < Q; ++q) {
      engines.push_back(std::make_unique<RssEngine>(RssConfig{ms_key, table}));
      BatchedQueuePairConfig c = cfg;
      c.queue_id = static_cast<std::uint16_t>(q);
      c.rss = engines.back().get();
      c.on_interrupt = nullptr;
      c.enable_tx_interrupts = c.enable_rx_interrupts = false;
      qc.queue_configs.push_back(c);
    }
    BatchedQueueManager qm{qc};
    std::vector<QueueBatch> b(Q);
    for (std::size_t q = 0; q < Q; ++q) b[q] = QueueBatch{txs.subspan(q * per, per), rxs.subspan(q * per, per)};
    std::vector<DeviceQueueBatch> db(Q);  // descriptors in HBM
    if (dev_desc)
      for (std::size_t q = 0; q < Q; ++q)
        db[q] = DeviceQueueBatch{static_cast<const TxDescriptor*>(dtx) + q * per, per,
                                 static_cast<const RxDescriptor*>(drx) + q * per, per};
    std::vector<RxBatchResult> outs;
    std::vector<double> ts;
    std::uint64_t ok_q = 0;
    int fused = 0;
    for (int r = 0; r < reps + 2; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      if (dev_desc) qm.process_batch(dm, db, outs);
      else if (hostmem) qm.process_batch(*hm, b, outs);
      else qm.process_batch(dm, b, outs);
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 2) ts.push_back(us);
      fused += r >= 2 ? qm.last_fused() : 0;
    }
    for (const auto& o : outs) {
      if (o.timings.device && cfg.results_on_device) ok_q += o.dev.nrx;
      else for (const auto& c : o.rx_completions) ok_q += c.status == 0;
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2];
    std::size_t fb = 0;
    for (std::size_t i = 0; i < per * Q; ++i) fb += lens[i];
    std::printf("{\"row\": \"f1_queue_manager\", \"workload\": \"c3\", \"queue_pairs\": %zu, \"tx_per_queue\": %zu, "
                "\"descriptors\": \"%s\", \"results\": \"%s\", \"host_memory\": %s, \"rx_align\": %zu, \"rx_completions\": %llu, "
                "\"fused_drains\": %d, \"drains\": %d, \"us_median\": %.1f, \"mpkt_s\": %.3f, \"frame_GBps\": %.2f, "
                "\"phases_us\": {\"check\": %.1f, \"gpu_sums\": %.1f, \"resolve\": %.1f, \"gpu_gather\": %.1f, \"gpu_rss\": %.1f, \"copy\": %.1f}}\n",
                Q, per, desc_kind.c_str(), cfg.results_on_device ? "device" : "host", hostmem ? "true" : "false", rx_align,
                (unsigned long long) ok_q, fused, reps, med, per * Q / med, fb / med / 1e3, outs[0].timings.check_us,
                outs[0].timings.sums_us, outs[0].timings.resolve_us, outs[0].timings.gather_us, outs[0].timings.rss_us,
                outs[0].timings.copy_us);
    nicgpu_free(mem);
    if (ptx) nicgpu_host_free(ptx);
    if (prx) nicgpu_host_free(prx);
    return 0;
  }
  auto submit = [&] {
    if (dev_desc) qp.submit(dm, dd);
    else if (hostmem) qp.submit(*hm, txs, rxs);
    else qp.submit(dm, txs, rxs);
  };

  std::vector<std::pair<double, RxBatchResult::Timings>> tot;
  RxBatchResult last;
  const bool pipelined = argc > 7 && std::string(argv[7]) == "pipelined";
  if (pipelined) {
    // warm-up (every slot grows its buffers), then `reps` batches with three in
    // flight: per-batch time = the whole run / reps (the first upload and the
    // last download included)
    // (eight batches: the four result sets in rotation, the caller's and the
    // three slots', each take their first-touch page faults here)
    for (int w = 0; w < 8; ++w) {
      if (qp.pending() == 3) qp.collect(last);
      submit();
    }
    while (qp.collect(last)) {
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      if (qp.pending() == 3) qp.collect(last);
      submit();
    }
    while (qp.collect(last)) {
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    for (int r = 0; r < reps; ++r) tot.emplace_back(us, last.timings);
  }
  for (int r = 0; r < (pipelined ? 0 : reps + 1); ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    // one result object reused across batches
    if (dev_desc) qp.process_batch(dm, dd, last);
    else if (hostmem) qp.process_batch(*hm, txs, rxs, last);
    else qp.process_batch(dm, txs, rxs, last);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (r > 0) tot.emplace_back(us, last.timings);
    const auto& P = last.timings;
    std::fprintf(stderr, "rep %d: %.0f us (%s: check %.0f plan %.0f sums %.0f resolve %.0f gather %.0f rss %.0f copy %.0f)\n", r,
                 us, P.device ? "device" : "host", P.check_us, P.plan_us, P.sums_us, P.resolve_us, P.gather_us, P.rss_us,
                 P.copy_us);
  }
  std::sort(tot.begin(), tot.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  const double med = tot[tot.size() / 2].first;
  std::size_t ok = 0, frame_bytes = 0;
  if (last.timings.device && cfg.results_on_device) {  // the last batch's completions, copied down to count
    last.rx_completions.resize(last.dev.nrx);
    check(nicgpu_memcpy_async(last.rx_completions.data(), last.dev.rx_completions,
                              last.dev.nrx * sizeof(CompletionEntry), nullptr),
          "memcpy");
    check(nicgpu_stream_synchronize(nullptr), "sync");
  }
  // the interrupt callbacks' floor: the same replay over host arrays of the
  // last batch's completions, no GPU (what the irq row cannot go below)
  double floor_us = 0;
  const std::uint64_t irq_batches = irq_count;  // callbacks of the measured batches (the floor replays add more)
  if (irq) {
    std::vector<CompletionEntry> htc = last.tx_completions;
    if (last.timings.device && cfg.results_on_device) {
      htc.resize(last.dev.ntx);
      check(nicgpu_memcpy_async(htc.data(), last.dev.tx_completions, last.dev.ntx * sizeof(CompletionEntry), nullptr),
            "memcpy");
      check(nicgpu_stream_synchronize(nullptr), "sync");
    }
    std::vector<double> fl;
    for (int k = 0; k < 5; ++k) {
      const auto t0 = std::chrono::steady_clock::now();
      rx_stage_detail::replay_interrupts(cfg, htc, last.rx_completions);
      fl.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(fl.begin(), fl.end());
    floor_us = fl[fl.size() / 2];
  }
  for (const auto& c : last.rx_completions) ok += c.status == 0;
  for (auto L : lens) frame_bytes += L;
  if (hostmem) {  // the last batch's frames are in the host memory, byte for byte
    std::size_t bad = 0;
    for (std::size_t j = 0; j < std::min<std::size_t>(n, nrx) && !wl.compare("c3"); ++j)
      bad += std::memcmp(hm->data() + rx[j].buffer_address, tx_img.data() + tx[j].buffer_address, lens[j]) != 0;
    if (bad) {
      std::fprintf(stderr, "hostmem: %zu delivered frames differ in the host memory\n", bad);
      return 1;
    }
  }
  const auto& T = tot[tot.size() / 2].second;  // the median batch's phases
  std::printf(
      "{\"row\": \"f1_rx_stage\", \"workload\": \"%s\", \"resolve\": \"%s\", \"descriptors\": \"%s\", \"mode\": \"%s\", \"results\": \"%s\", \"host_threads\": %u, \"tx_descriptors\": %zu, \"rx_completions\": %zu, \"rx_align\": %zu, "
      "\"rx_success\": %zu, \"host_memory\": %s, \"tx_staged_whole\": %s, \"overlapped_resolve\": %s, \"overlap_redone\": %s, \"deferred\": %s, \"interrupts\": %s, \"irq_callbacks\": %llu, \"callback_floor_us\": %.1f, \"us_median\": %.1f, \"mpkt_s\": %.3f, \"frame_GBps\": %.2f, "
      "\"phases_us\": {\"check\": %.1f, \"plan\": %.1f, \"gpu_sums\": %.1f, \"resolve\": %.1f, \"gpu_gather\": %.1f, \"gpu_rss\": %.1f, \"copy\": %.1f, \"irq\": %.1f, \"irq_wait\": %.1f}}\n",
      wl.c_str(), T.device ? "device" : "host", desc_kind.c_str(), pipelined ? "pipelined" : "sync", cfg.results_on_device ? "device" : "host", cfg.host_threads, n, last.rx_completions.size(), rx_align, ok,
      T.host_image ? "true" : "false", T.staged_whole ? "true" : "false", T.overlapped ? "true" : "false",
      T.overlap_redone ? "true" : "false", T.deferred ? "true" : "false", irq ? "true" : "false", (unsigned long long) irq_batches, floor_us, med, n / med, frame_bytes / med / 1e3, T.check_us, T.plan_us, T.sums_us,
      T.resolve_us, T.gather_us, T.rss_us, T.copy_us, T.irq_us, T.irq_wait_us);
  nicgpu_free(mem);
  if (ptx) nicgpu_host_free(ptx);
  if (prx) nicgpu_host_free(prx);
  if (dtx) nicgpu_free(dtx);
  if (drx) nicgpu_free(drx);
  return 0;
}
