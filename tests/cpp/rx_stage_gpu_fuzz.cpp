// rx_stage_gpu_fuzz.cpp — nic::BatchedQueuePair's device resolve (nicgpu_qp_*,
// the path process_batch takes for batches whose buffers do not overlap)
// against its host resolve (rx_stage_detail::run_batch over the CPU backend of
// cpu_backend.h), which rx_stage_fuzz.cpp checks against the compiled
// reference QueuePair.  Random batches of every descriptor kind (TSO/GSO, VLAN,
// bad checksums, MTU, invalid mss, faults, RX rings that run short, buffers
// too small, failing segment checksums), small and large (several grid
// blocks, host tails).  Compared: every completion, the statistics, RX
// descriptors consumed, the memory image, RSS hash / queue per completion, the
// dispatch lists and the RSS engine's stats.  Odd seeds (here and in
// `pipeline`) hand the descriptors over in device memory (DeviceDescriptors);
// seeds with bit 1 set leave the results there (results_on_device) and
// compare them after copying them down.
// GPU only.
//
// `check` mode: nicgpu_qp_check (the device path's overlap check) against
// rx_stage_detail::buffers_disjoint on random layouts — ascending rings with
// and without TX/RX and RX/RX overlaps (touching ends included), shuffled
// rings, invalid and clipped descriptors.
//
//   rx_stage_gpu_fuzz <first_seed> <count>
//   rx_stage_gpu_fuzz full c3|c5 [dev] [keep]
//   rx_stage_gpu_fuzz check [count]
//   rx_stage_gpu_fuzz edges             (piece-count limit, descriptor rings inside the image)
//   rx_stage_gpu_fuzz pipeline [himg] [count]   (submit/collect vs process_batch in order)
//   rx_stage_gpu_fuzz qm [count]         (BatchedQueueManager's fused batch vs each queue pair alone)
#undef NDEBUG
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cpu_backend.h"
#include "nic/flat_host_memory.h"
#include "nic/rss.h"
#include "nic/rx_queue_manager.h"
#include "nic/rx_stage.h"
#include "nic/rss_rings.h"
#include "nicgpu.h"
#include "oracle.h"

using namespace nic;

namespace {

struct Rng {
  std::uint64_t s;
  std::uint64_t next() {
    std::uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  std::uint32_t below(std::uint32_t n) { return n ? static_cast<std::uint32_t>((next() >> 32) % n) : 0; }
  std::uint8_t byte() { return static_cast<std::uint8_t>(next() >> 56); }
};

bool same(const CompletionEntry& a, const CompletionEntry& b) {
  return a.queue_id == b.queue_id && a.descriptor_index == b.descriptor_index && a.status == b.status &&
         a.checksum_offloaded == b.checksum_offloaded && a.checksum_verified == b.checksum_verified &&
         a.tso_performed == b.tso_performed && a.gso_performed == b.gso_performed && a.vlan_inserted == b.vlan_inserted &&
         a.vlan_stripped == b.vlan_stripped && a.gro_aggregated == b.gro_aggregated &&
         a.segments_produced == b.segments_produced && a.vlan_tag == b.vlan_tag;
}

void balance(std::vector<std::uint8_t>& b, std::size_t at) {
  b[at] = b[at + 1] = 0;
  const std::uint16_t c = oracle_compute_checksum(b.data(), b.size());
  b[at] = static_cast<std::uint8_t>(c >> 8);
  b[at + 1] = static_cast<std::uint8_t>(c);
}

const std::vector<std::uint8_t> kMsKey = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67,
                                          0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb,
                                          0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30,
                                          0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};

std::size_t g_tail = 0, g_device = 0, g_short = 0, g_devdesc = 0;  // host tails, device batches, NoDescriptor, device descriptors
std::size_t g_late = 0, g_late_fail = 0;  // batches whose RX verifies the delivery made; ChecksumError completions in them
std::size_t g_himg = 0, g_himg_sparse = 0;  // batches run on a HostMemory (and staged per descriptor)
std::size_t g_irq = 0;  // interrupt callbacks compared

// BatchedQueuePairConfig::results_on_device: copy RxBatchResult::dev into the
// host vectors, as the host-result form fills them, so the comparisons apply.
// Called before the stage's next process_batch / submit (the view's lifetime).
std::size_t g_keep = 0;
bool materialize(RxBatchResult& o) {
  if (!o.timings.device) return o.dev.tx_completions == nullptr && o.dev.ntx == 0;
  if (!o.tx_completions.empty() || !o.rx_completions.empty() || !o.queues.empty()) return false;
  const auto& d = o.dev;
  if (d.ntx && !d.tx_completions) return false;
  if (d.nrx && !d.rx_completions) return false;
  o.tx_completions.resize(d.ntx);
  o.rx_completions.resize(d.nrx);
  o.rx_hash.assign(d.nrx, 0u);
  o.rx_queue.assign(d.nrx, RxBatchResult::kNoQueue);
  if (d.ntx)
    assert(nicgpu_memcpy_async(o.tx_completions.data(), d.tx_completions, d.ntx * sizeof(CompletionEntry), nullptr) ==
           NICGPU_OK);
  if (d.nrx)
    assert(nicgpu_memcpy_async(o.rx_completions.data(), d.rx_completions, d.nrx * sizeof(CompletionEntry), nullptr) ==
           NICGPU_OK);
  if (d.rx_hash && d.nrx) {
    assert(nicgpu_memcpy_async(o.rx_hash.data(), d.rx_hash, d.nrx * 4, nullptr) == NICGPU_OK);
    assert(nicgpu_memcpy_async(o.rx_queue.data(), d.rx_queue, d.nrx * 2, nullptr) == NICGPU_OK);
  }
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  if (d.queue_start.size() != d.queue_end.size() || (!d.queue_start.empty() && !d.queue_which)) return false;
  for (std::size_t q = 0; q < d.queue_start.size(); ++q) {
    std::vector<std::uint32_t> w(d.queue_end[q] - d.queue_start[q]);
    if (!w.empty())
      assert(nicgpu_memcpy_async(w.data(), d.queue_which + d.queue_start[q], w.size() * 4, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    o.queues.push_back(std::move(w));
  }
  ++g_keep;
  return true;
}

int run_case(std::uint64_t seed) {
  Rng r{seed * 104729 + 3};
  const bool large = r.below(8) == 0;
  const std::size_t ntx = large ? 20000 + r.below(60000) : 1 + r.below(300);
  const std::size_t nrx = r.below(4) == 0 ? r.below(static_cast<std::uint32_t>(ntx + 1)) : ntx * (1 + r.below(3));
  const std::size_t mtus[] = {9000, 1500, 3000, 65535};
  const std::size_t max_mtu = mtus[r.below(4)];
  const bool tso_heavy = r.below(4) == 0;
  // one seed in three: a batch the device resolves with its RX verifies
  // deferred to the delivery (no TX verify, one segment per packet; a quarter
  // of the frames unbalanced, so many of those verifies fail)
  const bool late_case = seed % 3 == 2;
  std::vector<TxDescriptor> tx(ntx);
  std::vector<std::uint8_t> image;
  std::size_t at = 0;
  std::vector<std::pair<std::size_t, std::vector<std::uint8_t>>> pkts;
  for (std::size_t i = 0; i < ntx; ++i) {
    const std::uint32_t pick = r.below(16);
    std::size_t L = pick < 4 ? r.below(70) : (pick < 10 ? 60 + r.below(1500) : (pick < 15 ? 9000 : 9000 + r.below(70000)));
    if (large && L > 9000) L = 1518;
    if (late_case && L > 9000) L = 9000;
    std::vector<std::uint8_t> p(L);
    const bool zero = r.below(40) == 0;
    for (auto& b : p) b = zero ? 0 : r.byte();
    if (L >= 16 && r.below(4) != 0) balance(p, 10);
    at += r.below(3) == 0 ? r.below(9) : 0;
    TxDescriptor& t = tx[i];
    t.buffer_address = at;
    t.length = static_cast<std::uint32_t>(L);
    t.descriptor_index = static_cast<std::uint16_t>(r.below(65536));
    t.checksum = static_cast<ChecksumMode>(r.below(3));
    t.checksum_offload = r.below(2);
    const std::uint16_t good = oracle_compute_checksum(p.data(), L);
    t.checksum_value = r.below(6) == 0 ? static_cast<std::uint16_t>(r.below(65536)) : good;
    if (r.below(tso_heavy ? 2 : 4) == 0) {
      t.tso_enabled = r.below(2);
      t.gso_enabled = !t.tso_enabled || r.below(3) == 0;
      const std::uint32_t mp = r.below(10);
      t.mss = static_cast<std::uint16_t>(mp == 0 ? 0 : (mp == 1 ? 9001 + r.below(3) : (mp < 3 ? 1 + r.below(9) : 50 + r.below(2000))));
      const std::uint32_t hp = r.below(8);
      t.header_length = static_cast<std::uint16_t>(hp == 0 ? r.below(4) : (hp == 1 ? L + r.below(2) : (hp == 2 ? r.below(12) : 14 + r.below(60))));
    }
    if (r.below(5) == 0) {
      t.vlan_insert = true;
      t.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
    }
    if (late_case) {
      t.checksum_offload = true;
      // TSO/GSO of at most one segment (header || one chunk when the mss is
      // at least the payload: the segmented write form)
      if ((t.tso_enabled || t.gso_enabled) && t.mss && L > t.header_length)
        t.mss = static_cast<std::uint16_t>(std::min<std::size_t>(9000, L - t.header_length + r.below(3)));
    }
    pkts.emplace_back(at, std::move(p));
    at += L;
  }
  at = (at + 15) & ~std::size_t{15};
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    RxDescriptor& x = rx[j];
    const std::uint32_t bp = r.below(10);
    x.buffer_length = bp == 0 ? r.below(200) : (bp < 5 ? 2000 : 9300);
    x.buffer_address = at + r.below(5);
    at = x.buffer_address + x.buffer_length + r.below(4);
    x.descriptor_index = static_cast<std::uint16_t>(r.below(65536));
    x.checksum = static_cast<ChecksumMode>(r.below(3));
    x.checksum_offload = r.below(3) != 0;
    x.vlan_strip = r.below(3) == 0;
    x.vlan_present = r.below(3) == 0;
    x.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
    x.gro_enabled = r.below(4) == 0;
  }
  const std::size_t mem_size = at + 32;
  for (std::size_t i = 0; i < ntx; ++i)
    if (r.below(60) == 0) tx[i].buffer_address = r.below(2) ? mem_size + 1 + i : mem_size - tx[i].length / 2;
  for (std::size_t j = 0; j < nrx; ++j)
    if (r.below(70) == 0) rx[j].buffer_address = mem_size + 1 + j;
  image.assign(mem_size, 0);
  for (auto& [a, p] : pkts) std::memcpy(image.data() + a, p.data(), p.size());
  std::vector<std::uint16_t> table(r.below(2) ? 128 : 1 + r.below(300));
  // mostly < 64 queues (the dispatch lists' counting sort), one batch in four
  // up to 300 (the radix-sort path)
  const std::uint64_t queues = r.below(4) == 0 ? 300 : 1 + r.below(63);
  for (auto& q : table) q = static_cast<std::uint16_t>(r.below(queues));
  const RssConfig rss_cfg{r.below(2) ? kMsKey : std::vector<std::uint8_t>{}, table};
  const std::uint16_t qid = static_cast<std::uint16_t>(r.below(8));

  BatchedQueuePairConfig cfg;
  cfg.queue_id = qid;
  cfg.max_mtu = max_mtu;
  if (!rx_stage_detail::buffers_disjoint(mem_size, tx, rx)) return 0;  // the host path's business (rx_stage_fuzz)
  // interrupt callbacks on most seeds: the host resolve fires them as it
  // posts; the device path replays them from the completions afterwards
  const bool irq = (seed % 4) != 3;
  cfg.enable_tx_interrupts = r.below(2);
  cfg.enable_rx_interrupts = r.below(4) != 0;
  std::vector<CompletionEntry> fired_host, fired_dev;
  if (irq)
    cfg.on_interrupt = [&fired_host](std::uint16_t, const CompletionEntry& e) { fired_host.push_back(e); };

  // host resolve
  RssEngine host_rss{rss_cfg};
  cfg.rss = &host_rss;
  std::vector<std::uint8_t> host_img = image;
  test::CpuBackend cpu{host_img, &host_rss, TupleSpec{}};
  RxBatchResult ho;
  QueuePairStats hs{};
  rx_stage_detail::BatchScratch scratch;
  rx_stage_detail::run_batch(cfg, mem_size, tx, rx, hs, ho, scratch, cpu);

  // device resolve
  RssEngine dev_rss{rss_cfg};
  cfg.rss = &dev_rss;
  // odd seeds hand the descriptors over in device memory (DeviceDescriptors),
  // placed in the same allocation past the image
  const bool dev_desc = seed & 1;
  const bool keep = (seed >> 1) & 1;  // results_on_device
  const std::size_t desc_at = (mem_size + 64 + 255) & ~std::size_t{255};
  const std::size_t rx_at = desc_at + ((ntx * sizeof(TxDescriptor) + 255) & ~std::size_t{255});
  void* d = nullptr;
  assert(nicgpu_malloc(&d, rx_at + nrx * sizeof(RxDescriptor) + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
  std::byte* base = static_cast<std::byte*>(d);
  if (ntx) assert(nicgpu_memcpy_async(base + desc_at, tx.data(), ntx * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
  if (nrx) assert(nicgpu_memcpy_async(base + rx_at, rx.data(), nrx * sizeof(RxDescriptor), nullptr) == NICGPU_OK);
  cfg.results_on_device = keep;
  if (irq) cfg.on_interrupt = [&fired_dev](std::uint16_t, const CompletionEntry& e) { fired_dev.push_back(e); };
  BatchedQueuePair qp{cfg};
  RxBatchResult go;
  if (dev_desc) {
    const DeviceDescriptors dd{reinterpret_cast<const TxDescriptor*>(base + desc_at), ntx,
                               reinterpret_cast<const RxDescriptor*>(base + rx_at), nrx};
    qp.process_batch(DeviceHostMemory{base, mem_size}, dd, go);
    g_devdesc += 1;
  } else {
    qp.process_batch(DeviceHostMemory{base, mem_size}, tx, rx, go);
  }
  bool irq_ok = fired_dev.size() == fired_host.size();
  std::size_t irq_at = 0;
  for (; irq_ok && irq_at < fired_host.size(); ++irq_at) irq_ok = same(fired_dev[irq_at], fired_host[irq_at]);
  if (!irq_ok) {
    // the first difference and how the batch was resolved; the completions
    // are compared below too, so the report says whether only the replay's
    // copy of them differed
    const auto& T = go.timings;
    std::fprintf(stderr,
                 "seed %llu: interrupt callbacks differ (%zu device, %zu host), first at %zu; device %s keep %d "
                 "walked %d host_tail %d ntx %zu nrx %zu irq_wait %.1f us\n",
                 (unsigned long long) seed, fired_dev.size(), fired_host.size(), irq_at ? irq_at - 1 : 0,
                 T.device ? "yes" : "no", (int) keep, (int) T.walked, (int) T.host_tail, ntx, nrx, T.irq_wait_us);
    if (irq_at && irq_at - 1 < fired_dev.size() && irq_at - 1 < fired_host.size()) {
      const CompletionEntry &a = fired_dev[irq_at - 1], &b = fired_host[irq_at - 1];
      std::fprintf(stderr, "  device: q %u idx %u status %u segs %u ver %u | host: q %u idx %u status %u segs %u ver %u\n",
                   a.queue_id, a.descriptor_index, a.status, a.segments_produced, (unsigned) a.checksum_verified,
                   b.queue_id, b.descriptor_index, b.status, b.segments_produced, (unsigned) b.checksum_verified);
    }
  }
  g_irq += irq ? fired_dev.size() : 0;
  if (keep && !materialize(go)) {
    std::fprintf(stderr, "results on the device: the view is not as documented\n");
    return 1;
  }
  std::vector<std::uint8_t> dev_img(mem_size);
  assert(nicgpu_memcpy_async(dev_img.data(), d, mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  nicgpu_free(d);
  if (!go.timings.device) {
    std::fprintf(stderr, "seed %llu: disjoint batch not resolved on the device\n", (unsigned long long) seed);
    return 1;
  }
  g_device += 1;
  if (go.timings.deferred) {
    g_late += 1;
    for (const CompletionEntry& e : ho.rx_completions) g_late_fail += e.status == static_cast<std::uint32_t>(CompletionCode::ChecksumError);
  }
  bool ok = go.tx_completions.size() == ho.tx_completions.size() && go.rx_completions.size() == ho.rx_completions.size();
  for (std::size_t i = 0; ok && i < ho.tx_completions.size(); ++i) ok = same(go.tx_completions[i], ho.tx_completions[i]);
  for (std::size_t i = 0; ok && i < ho.rx_completions.size(); ++i) ok = same(go.rx_completions[i], ho.rx_completions[i]);
  const bool comp_ok = ok;
  if (!irq_ok) {
    std::fprintf(stderr, "  completions (materialized after the batch) %s the host's\n", comp_ok ? "equal" : "differ from");
    return 1;
  }
  ok = ok && std::memcmp(&hs, &qp.stats(), sizeof(hs)) == 0;
  const bool stats_ok = ok;
  ok = ok && go.rx_consumed == ho.rx_consumed && go.tx_processed == ho.tx_processed;
  ok = ok && host_img == dev_img;
  const bool mem_ok = ok;
  ok = ok && go.rx_hash == ho.rx_hash && go.rx_queue == ho.rx_queue && go.queues == ho.queues;
  ok = ok && dev_rss.stats().hashes == host_rss.stats().hashes && dev_rss.stats().queue_hits == host_rss.stats().queue_hits;
  if (!ok) {
    std::fprintf(stderr,
                 "seed %llu: device resolve differs (ntx %zu nrx %zu: completions %d stats %d memory %d; tx %zu/%zu rx "
                 "%zu/%zu consumed %zu/%zu)\n",
                 (unsigned long long) seed, ntx, nrx, int(comp_ok), int(stats_ok), int(mem_ok), go.tx_completions.size(),
                 ho.tx_completions.size(), go.rx_completions.size(), ho.rx_completions.size(), go.rx_consumed,
                 ho.rx_consumed);
    return 1;
  }
  // seeds with bit 2 set (host descriptors): the same batch once more on a
  // HostMemory (the reference's interface, FlatHostMemory = SimpleHostMemory's
  // bounds rule): TX bytes staged up, delivered bytes written back, everything
  // equal to the host resolve's, the memory's bytes included
  if (!dev_desc && ((seed >> 2) & 1)) {
    FlatHostMemory hm(mem_size);
    std::memcpy(hm.data(), image.data(), mem_size);
    RssEngine hi_rss{rss_cfg};
    cfg.rss = &hi_rss;
    std::vector<CompletionEntry> fired_hi;
    if (irq) cfg.on_interrupt = [&fired_hi](std::uint16_t, const CompletionEntry& e) { fired_hi.push_back(e); };
    BatchedQueuePair hq{cfg};
    RxBatchResult hio;
    hq.process_batch(hm, tx, rx, hio);
    if (keep && !materialize(hio)) return 1;
    bool hok = hio.timings.host_image && hio.tx_completions.size() == ho.tx_completions.size() &&
               hio.rx_completions.size() == ho.rx_completions.size();
    for (std::size_t i = 0; hok && i < ho.tx_completions.size(); ++i) hok = same(hio.tx_completions[i], ho.tx_completions[i]);
    for (std::size_t i = 0; hok && i < ho.rx_completions.size(); ++i) hok = same(hio.rx_completions[i], ho.rx_completions[i]);
    hok = hok && std::memcmp(&hs, &hq.stats(), sizeof(hs)) == 0 && hio.rx_consumed == ho.rx_consumed;
    const bool hmem = std::memcmp(hm.data(), host_img.data(), mem_size) == 0;
    hok = hok && hmem && hio.rx_hash == ho.rx_hash && hio.rx_queue == ho.rx_queue && hio.queues == ho.queues;
    hok = hok && hi_rss.stats().hashes == host_rss.stats().hashes && hi_rss.stats().queue_hits == host_rss.stats().queue_hits;
    hok = hok && fired_hi.size() == fired_host.size();
    for (std::size_t i = 0; hok && i < fired_host.size(); ++i) hok = same(fired_hi[i], fired_host[i]);
    if (!hok) {
      std::fprintf(stderr, "seed %llu: HostMemory batch differs (memory %d, device %d)\n", (unsigned long long) seed,
                   int(hmem), int(hio.timings.device));
      return 1;
    }
    g_himg += 1;
    g_himg_sparse += !hio.timings.staged_whole;
  }
  if (go.timings.host_tail) g_tail += 1;
  for (const auto& c : ho.tx_completions)
    if (c.status == static_cast<std::uint32_t>(CompletionCode::NoDescriptor)) {
      g_short += 1;
      break;
    }
  return 0;
}

// Full-size f1 workloads (tools/bench_rx_stage.cpp's): C3 = 1 M IMIX frames
// (balanced so every RX verify passes), C5 = 131072 x 9000 B TSO (H 54, mss
// 1448; random payloads, so every packet ends at its first segment's
// checksum).  Device resolve against host resolve, everything compared;
// `dev` hands the descriptors over in device memory, `keep` leaves the results
// there (results_on_device).
int run_full(const char* wl, bool dev_desc, bool keep) {
  const bool c5 = std::strcmp(wl, "c5") == 0;
  const std::size_t n = c5 ? 131072 : (1u << 20);
  Rng r{c5 ? 55u : 33u};
  std::vector<std::size_t> lens(n);
  for (auto& L : lens) {
    const std::uint32_t k = r.below(12);
    L = c5 ? 9000 : (k < 7 ? 64 : (k < 11 ? 576 : 1518));
  }
  std::size_t tx_bytes = 0;
  for (auto L : lens) tx_bytes += (L + 15) & ~std::size_t{15};
  const std::size_t rx_buf = c5 ? 1600 : 2048, segs = c5 ? 7 : 1, nrx = n * segs;
  const std::size_t mem_size = tx_bytes + nrx * rx_buf;
  std::vector<std::uint8_t> image(mem_size, 0);
  std::vector<TxDescriptor> tx(n);
  std::size_t at = 0;
  for (std::size_t i = 0; i < n; ++i) {
    std::uint8_t* p = image.data() + at;
    for (std::size_t b = 0; b < lens[i]; ++b) p[b] = r.byte();
    p[12] = 0x08;
    p[13] = 0x00;
    if (!c5) {
      p[10] = p[11] = 0;
      const std::uint16_t c = oracle_compute_checksum(p, lens[i]);
      p[10] = static_cast<std::uint8_t>(c >> 8);
      p[11] = static_cast<std::uint8_t>(c);
    }
    TxDescriptor& t = tx[i];
    t.buffer_address = at;
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum_offload = true;
    t.checksum = ChecksumMode::Layer4;
    if (c5) {
      t.tso_enabled = true;
      t.mss = 1448;
      t.header_length = 54;
    }
    at += (lens[i] + 15) & ~std::size_t{15};
  }
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    rx[j].buffer_address = tx_bytes + j * rx_buf;
    rx[j].buffer_length = static_cast<std::uint32_t>(rx_buf);
    rx[j].descriptor_index = static_cast<std::uint16_t>(j);
    rx[j].checksum_offload = true;
    rx[j].checksum = ChecksumMode::Layer4;
  }
  std::vector<std::uint16_t> table(128);
  for (int i = 0; i < 128; ++i) table[i] = static_cast<std::uint16_t>(i % 16);
  const RssConfig rss_cfg{kMsKey, table};
  BatchedQueuePairConfig cfg;
  cfg.queue_id = 1;
  // RX and TX interrupt callbacks on: fired by the host resolve as it posts,
  // replayed by the device path from the completions
  cfg.enable_tx_interrupts = true;
  const bool irq = true;
  std::vector<CompletionEntry> fired_host, fired_dev;
  cfg.on_interrupt = [&fired_host](std::uint16_t, const CompletionEntry& e) { fired_host.push_back(e); };
  RssEngine host_rss{rss_cfg};
  cfg.rss = &host_rss;
  std::vector<std::uint8_t> host_img = image;
  test::CpuBackend cpu{host_img, &host_rss, TupleSpec{}};
  RxBatchResult ho;
  QueuePairStats hs{};
  rx_stage_detail::BatchScratch scratch;
  rx_stage_detail::run_batch(cfg, mem_size, tx, rx, hs, ho, scratch, cpu);
  RssEngine dev_rss{rss_cfg};
  cfg.rss = &dev_rss;
  const std::size_t ntx = tx.size();
  const std::size_t desc_at = (mem_size + 64 + 255) & ~std::size_t{255};
  const std::size_t rx_at = desc_at + ((ntx * sizeof(TxDescriptor) + 255) & ~std::size_t{255});
  void* d = nullptr;
  assert(nicgpu_malloc(&d, rx_at + nrx * sizeof(RxDescriptor) + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
  std::byte* base = static_cast<std::byte*>(d);
  if (ntx) assert(nicgpu_memcpy_async(base + desc_at, tx.data(), ntx * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
  if (nrx) assert(nicgpu_memcpy_async(base + rx_at, rx.data(), nrx * sizeof(RxDescriptor), nullptr) == NICGPU_OK);
  cfg.results_on_device = keep;
  if (irq) cfg.on_interrupt = [&fired_dev](std::uint16_t, const CompletionEntry& e) { fired_dev.push_back(e); };
  BatchedQueuePair qp{cfg};
  RxBatchResult go;
  if (dev_desc) {
    const DeviceDescriptors dd{reinterpret_cast<const TxDescriptor*>(base + desc_at), ntx,
                               reinterpret_cast<const RxDescriptor*>(base + rx_at), nrx};
    qp.process_batch(DeviceHostMemory{base, mem_size}, dd, go);
    g_devdesc += 1;
  } else {
    qp.process_batch(DeviceHostMemory{base, mem_size}, tx, rx, go);
  }
  bool irq_ok = fired_dev.size() == fired_host.size() && !fired_host.empty();
  for (std::size_t i = 0; irq_ok && i < fired_host.size(); ++i) irq_ok = same(fired_dev[i], fired_host[i]);
  if (!irq_ok) std::fprintf(stderr, "full %s: interrupt callbacks differ (%zu device, %zu host)\n", wl,
                            fired_dev.size(), fired_host.size());
  if (keep && !materialize(go)) {
    std::fprintf(stderr, "results on the device: the view is not as documented\n");
    return 1;
  }
  std::vector<std::uint8_t> dev_img(mem_size);
  assert(nicgpu_memcpy_async(dev_img.data(), d, mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  nicgpu_free(d);
  bool ok = go.timings.device && !go.timings.host_tail && go.tx_completions.size() == ho.tx_completions.size() &&
            go.rx_completions.size() == ho.rx_completions.size();
  for (std::size_t i = 0; ok && i < ho.tx_completions.size(); ++i) ok = same(go.tx_completions[i], ho.tx_completions[i]);
  for (std::size_t i = 0; ok && i < ho.rx_completions.size(); ++i) ok = same(go.rx_completions[i], ho.rx_completions[i]);
  ok = ok && std::memcmp(&hs, &qp.stats(), sizeof(hs)) == 0 && go.rx_consumed == ho.rx_consumed;
  ok = ok && host_img == dev_img && go.rx_hash == ho.rx_hash && go.rx_queue == ho.rx_queue && go.queues == ho.queues;
  ok = ok && dev_rss.stats().hashes == host_rss.stats().hashes && dev_rss.stats().queue_hits == host_rss.stats().queue_hits;
  ok = ok && irq_ok;
  std::size_t succ = 0;
  for (const auto& c : go.rx_completions) succ += c.status == 0;
  std::printf("rx_stage_gpu_fuzz full %s: %s (%zu TX, %zu RX completions, %zu Success, device %d, host tail %d, device "
              "descriptors %d, %zu interrupt callbacks)\n",
              wl, ok ? "ok" : "MISMATCH", go.tx_completions.size(), go.rx_completions.size(), succ,
              int(go.timings.device), int(go.timings.host_tail), int(dev_desc), fired_dev.size());
  return ok ? 0 : 1;
}

// submit()/collect() against process_batch in submission order: sequences
// of batches over one memory image, where later batches read bytes earlier
// ones wrote (TX buffers inside the RX ring), some batches overlap their own
// buffers (host path) and the RX windows wrap the ring.  Results, statistics,
// the image and the RSS engine's stats must all be equal.
std::size_t g_pipe_batches = 0, g_pipe_host = 0, g_pipe_devdesc = 0, g_pipe_himg = 0, g_pipe_late = 0;
bool g_force_himg = false;  // `pipeline himg`: every sequence's pipelined side on a HostMemory
std::size_t g_pipe_overlapped = 0, g_pipe_redone = 0;  // overlapped resolves that stood / were redone

int run_pipeline(std::uint64_t seed) {
  Rng r{seed * 7727 + 5};
  const std::size_t tx_region = 1u << 20, ring = 512, buf = 2048;
  const std::size_t mem_size = tx_region + ring * buf;
  std::vector<std::uint8_t> image(mem_size, 0);
  for (std::size_t i = 0; i < tx_region; ++i) image[i] = r.byte();
  // balanced frames at 2 KiB strides so some TX verifies pass
  for (std::size_t a = 0; a + 2048 <= tx_region; a += 2048) {
    std::vector<std::uint8_t> f(image.begin() + a, image.begin() + a + 1518);
    balance(f, 10);
    std::memcpy(image.data() + a, f.data(), f.size());
  }
  std::vector<std::uint16_t> table(128);
  for (auto& q : table) q = static_cast<std::uint16_t>(r.below(16));
  const RssConfig rss_cfg{kMsKey, table};
  const int nb = 5 + static_cast<int>(r.below(4));
  std::vector<std::vector<TxDescriptor>> txs(nb);
  std::vector<std::vector<RxDescriptor>> rxs(nb);
  std::size_t ring_at = 0;
  // one sequence in five reads no frame from the ring: every batch's
  // overlapped resolve then stands (the others mostly redo it behind the
  // earlier batches' writes)
  const bool quiet = seed % 5 == 0;
  // one sequence in four: batches the device resolves with their RX verifies
  // deferred to the delivery (the process_batch side sums them eagerly)
  const bool late_case = seed % 4 == 1;
  for (int b = 0; b < nb; ++b) {
    const std::size_t ntx = 1 + r.below(b % 3 == 0 ? 3000 : 300);
    const std::size_t nrx = std::min<std::size_t>(ring / 2, ntx * (1 + r.below(2)) + r.below(5));
    // one batch in four may also read its own RX window (overlap: the host path)
    const bool own = r.below(4) == 0;
    for (std::size_t i = 0; i < ntx; ++i) {
      TxDescriptor t{};
      if (r.below(6) == 0 && !quiet) {  // a frame an earlier batch delivered into the ring
        const std::size_t slot = own ? r.below(ring) : (ring_at + nrx + r.below(static_cast<std::uint32_t>(ring - nrx))) % ring;
        t.buffer_address = tx_region + slot * buf;
        t.length = 64 + r.below(1400);
      } else {
        t.buffer_address = r.below(static_cast<std::uint32_t>(tx_region / 2048)) * 2048;
        t.length = r.below(4) ? 1518 : 1 + r.below(2000);
      }
      t.descriptor_index = static_cast<std::uint16_t>(i);
      t.checksum = static_cast<ChecksumMode>(r.below(3));
      t.checksum_offload = late_case || r.below(4) != 0;
      if (r.below(8) == 0 && !late_case) {
        t.tso_enabled = true;
        t.mss = static_cast<std::uint16_t>(200 + r.below(1200));
        t.header_length = 54;
      }
      if (r.below(8) == 0) {
        t.vlan_insert = true;
        t.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
      }
      txs[b].push_back(t);
    }
    for (std::size_t j = 0; j < nrx; ++j) {
      RxDescriptor x{};
      x.buffer_address = tx_region + ((ring_at + j) % ring) * buf;
      x.buffer_length = static_cast<std::uint32_t>(r.below(10) ? buf : r.below(300));
      x.descriptor_index = static_cast<std::uint16_t>(j);
      x.checksum = static_cast<ChecksumMode>(r.below(3));
      x.checksum_offload = r.below(3) != 0;
      x.vlan_strip = r.below(4) == 0;
      rxs[b].push_back(x);
    }
    ring_at = (ring_at + nrx) % ring;
  }
  BatchedQueuePairConfig cfg;
  cfg.queue_id = 3;
  void *d_seq = nullptr, *d_pipe = nullptr;
  assert(nicgpu_malloc(&d_seq, mem_size + 64) == NICGPU_OK);
  assert(nicgpu_malloc(&d_pipe, mem_size + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d_seq, image.data(), mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d_pipe, image.data(), mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  const DeviceHostMemory m_seq{static_cast<std::byte*>(d_seq), mem_size}, m_pipe{static_cast<std::byte*>(d_pipe), mem_size};
  // host descriptors with bit 2 set (every seed under `pipeline himg`): the
  // pipelined side runs on a HostMemory — later batches read frames earlier
  // pending ones deliver, rings wrap onto buffers still being written back
  const bool himg = !(seed & 1) && (g_force_himg || ((seed >> 2) & 1));
  FlatHostMemory hm(himg ? mem_size : 0);
  if (himg) std::memcpy(hm.data(), image.data(), mem_size);

  RssEngine rss_seq{rss_cfg}, rss_pipe{rss_cfg};
  cfg.rss = &rss_seq;
  cfg.defer_rx_verify = false;  // the reference side: every batch's piece sums before its resolve
  cfg.enable_tx_interrupts = r.below(2);
  std::vector<CompletionEntry> irq_seq, irq_pipe;
  cfg.on_interrupt = [&irq_seq](std::uint16_t, const CompletionEntry& e) { irq_seq.push_back(e); };
  BatchedQueuePair seq{cfg};
  cfg.rss = &rss_pipe;
  cfg.on_interrupt = [&irq_pipe](std::uint16_t, const CompletionEntry& e) { irq_pipe.push_back(e); };
  const bool keep = (seed >> 1) & 1;  // results_on_device on the pipelined side
  cfg.results_on_device = keep;
  cfg.overlap_resolve = seed % 3 != 1;  // the overlapped resolve (opt-in) on two sequences in three
  cfg.defer_rx_verify = true;
  BatchedQueuePair pipe{cfg};
  bool view_ok = true;
  std::vector<RxBatchResult> want(nb), got;
  for (int b = 0; b < nb; ++b) seq.process_batch(m_seq, txs[b], rxs[b], want[b]);
  // odd seeds: the pipelined side gets its descriptors in device memory, and
  // runs a batch through process_batch now and then when nothing is pending
  const bool dev_desc = seed & 1;
  std::vector<DeviceDescriptors> dd(nb);
  void* d_desc = nullptr;
  // The descriptors are written to dd[] by a device-to-device copy enqueued on
  // the caller's stream just before each hand-over (a device-side producer),
  // from a staged copy; dd[] starts zeroed, so a stage that read them before
  // that copy landed would see empty rings.
  void* d_src = nullptr;
  std::size_t desc_bytes = 0;
  if (dev_desc) {
    std::size_t bytes = 0;
    for (int b = 0; b < nb; ++b) bytes += txs[b].size() * sizeof(TxDescriptor) + rxs[b].size() * sizeof(RxDescriptor);
    desc_bytes = bytes;
    assert(nicgpu_malloc(&d_desc, bytes + 64) == NICGPU_OK);
    assert(nicgpu_malloc(&d_src, bytes + 64) == NICGPU_OK);
    std::byte* p = static_cast<std::byte*>(d_src);
    for (int b = 0; b < nb; ++b) {
      assert(nicgpu_memcpy_async(p, txs[b].data(), txs[b].size() * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
      dd[b].tx = reinterpret_cast<const TxDescriptor*>(static_cast<std::byte*>(d_desc) + (p - static_cast<std::byte*>(d_src)));
      dd[b].ntx = txs[b].size();
      p += txs[b].size() * sizeof(TxDescriptor);
      assert(nicgpu_memcpy_async(p, rxs[b].data(), rxs[b].size() * sizeof(RxDescriptor), nullptr) == NICGPU_OK);
      dd[b].rx = reinterpret_cast<const RxDescriptor*>(static_cast<std::byte*>(d_desc) + (p - static_cast<std::byte*>(d_src)));
      dd[b].nrx = rxs[b].size();
      p += rxs[b].size() * sizeof(RxDescriptor);
    }
    assert(nicgpu_memset_async(d_desc, 0, bytes + 64, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  }
  // a slow producer: ~0.1 ms of other work on the stream ahead of the copy
  constexpr std::size_t kBusy = std::size_t{512} << 20;
  void* d_busy = nullptr;
  if (dev_desc) assert(nicgpu_malloc(&d_busy, kBusy) == NICGPU_OK);
  auto produce = [&](int b) {  // the producer: batch b's descriptors into dd[b], on the caller's stream
    assert(nicgpu_memset_async(d_busy, b & 0xFF, kBusy, nullptr) == NICGPU_OK);
    const std::size_t at = reinterpret_cast<const std::byte*>(dd[b].tx) - static_cast<std::byte*>(d_desc);
    const std::size_t len = dd[b].ntx * sizeof(TxDescriptor) + dd[b].nrx * sizeof(RxDescriptor);
    if (len) assert(nicgpu_memcpy_async(static_cast<std::byte*>(d_desc) + at, static_cast<std::byte*>(d_src) + at, len,
                                        nullptr) == NICGPU_OK);
  };
  (void) desc_bytes;
  RxBatchResult out;
  for (int b = 0; b < nb; ++b) {
    while (pipe.pending() == 3 || (pipe.pending() > 0 && r.below(3) == 0)) {
      assert(pipe.collect(out));
      if (keep) view_ok &= materialize(out);
      got.push_back(std::move(out));
      out = RxBatchResult{};
    }
    if (himg && pipe.pending() == 0 && r.below(4) == 0) {
      pipe.process_batch(hm, txs[b], rxs[b], out);
      if (keep) view_ok &= materialize(out);
      got.push_back(std::move(out));
      out = RxBatchResult{};
    } else if (himg) {
      pipe.submit(hm, txs[b], rxs[b]);
    } else if (!dev_desc) {
      pipe.submit(m_pipe, txs[b], rxs[b]);
    } else if (pipe.pending() == 0 && r.below(3) == 0) {
      produce(b);
      pipe.process_batch(m_pipe, dd[b], out);
      if (keep) view_ok &= materialize(out);
      got.push_back(std::move(out));
      out = RxBatchResult{};
    } else {
      produce(b);
      pipe.submit(m_pipe, dd[b]);
    }
  }
  while (pipe.collect(out)) {
    if (keep) view_ok &= materialize(out);
    got.push_back(std::move(out));
    out = RxBatchResult{};
  }
  bool ok = view_ok && static_cast<int>(got.size()) == nb;
  for (int b = 0; ok && b < nb; ++b) {
    const RxBatchResult &w = want[b], &g = got[b];
    ok = w.tx_completions.size() == g.tx_completions.size() && w.rx_completions.size() == g.rx_completions.size() &&
         w.rx_consumed == g.rx_consumed && w.tx_processed == g.tx_processed && w.rx_hash == g.rx_hash &&
         w.rx_queue == g.rx_queue && w.queues == g.queues && w.timings.device == g.timings.device &&
         g.timings.host_image == himg;
    for (std::size_t i = 0; ok && i < w.tx_completions.size(); ++i) ok = same(w.tx_completions[i], g.tx_completions[i]);
    for (std::size_t i = 0; ok && i < w.rx_completions.size(); ++i) ok = same(w.rx_completions[i], g.rx_completions[i]);
    if (!ok) {
      std::fprintf(stderr, "pipeline seed %llu: batch %d differs (deferred %d, device %d/%d, tx %zu/%zu rx %zu/%zu)\n",
                   (unsigned long long) seed, b, (int) g.timings.deferred, (int) w.timings.device,
                   (int) g.timings.device, w.tx_completions.size(), g.tx_completions.size(), w.rx_completions.size(),
                   g.rx_completions.size());
      for (std::size_t i = 0; i < std::min(w.rx_completions.size(), g.rx_completions.size()); ++i)
        if (!same(w.rx_completions[i], g.rx_completions[i])) {
          const CompletionEntry &x = w.rx_completions[i], &y = g.rx_completions[i];
          std::fprintf(stderr, "  rx %zu: in order status %u strip %u tag %u ver %u | pipelined status %u strip %u tag %u ver %u\n",
                       i, x.status, (unsigned) x.vlan_stripped, x.vlan_tag, (unsigned) x.checksum_verified, y.status,
                       (unsigned) y.vlan_stripped, y.vlan_tag, (unsigned) y.checksum_verified);
          break;
        }
      for (std::size_t i = 0; i < std::min(w.tx_completions.size(), g.tx_completions.size()); ++i)
        if (!same(w.tx_completions[i], g.tx_completions[i])) {
          std::fprintf(stderr, "  tx %zu: status %u / %u\n", i, w.tx_completions[i].status, g.tx_completions[i].status);
          break;
        }
      if (w.rx_hash != g.rx_hash || w.rx_queue != g.rx_queue) std::fprintf(stderr, "  RSS results differ\n");
    }
    g_pipe_host += !w.timings.device;
    g_pipe_overlapped += g.timings.overlapped && !g.timings.overlap_redone;
    g_pipe_redone += g.timings.overlap_redone;
    g_pipe_late += g.timings.deferred;
  }
  g_pipe_batches += nb;
  if (dev_desc) g_pipe_devdesc += nb;
  if (himg) g_pipe_himg += nb;
  if (std::memcmp(&seq.stats(), &pipe.stats(), sizeof(QueuePairStats)) != 0) {
    const auto* x = reinterpret_cast<const std::uint64_t*>(&seq.stats());
    const auto* y = reinterpret_cast<const std::uint64_t*>(&pipe.stats());
    std::fprintf(stderr, "pipeline seed %llu: stats differ:", (unsigned long long) seed);
    for (std::size_t k = 0; k < sizeof(QueuePairStats) / 8; ++k)
      if (x[k] != y[k]) std::fprintf(stderr, " [%zu] %llu/%llu", k, (unsigned long long) x[k], (unsigned long long) y[k]);
    std::fprintf(stderr, "\n");
    ok = false;
  }
  bool irq_ok = irq_seq.size() == irq_pipe.size();
  for (std::size_t i = 0; irq_ok && i < irq_seq.size(); ++i) irq_ok = same(irq_seq[i], irq_pipe[i]);
  if (!irq_ok) std::fprintf(stderr, "pipeline seed %llu: interrupt callbacks differ\n", (unsigned long long) seed);
  ok = ok && irq_ok;
  ok = ok && rss_seq.stats().hashes == rss_pipe.stats().hashes && rss_seq.stats().queue_hits == rss_pipe.stats().queue_hits;
  std::vector<std::uint8_t> a(mem_size), b(mem_size);
  assert(nicgpu_memcpy_async(a.data(), d_seq, mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_memcpy_async(b.data(), d_pipe, mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  if (himg) std::memcpy(b.data(), hm.data(), mem_size);  // the HostMemory itself, after every collect
  ok = ok && a == b;
  nicgpu_free(d_seq);
  nicgpu_free(d_pipe);
  if (d_desc) nicgpu_free(d_desc);
  if (d_src) nicgpu_free(d_src);
  if (d_busy) nicgpu_free(d_busy);
  if (!ok) {
    std::fprintf(stderr, "pipeline seed %llu: pipelined run differs from process_batch in order\n",
                 (unsigned long long) seed);
    return 1;
  }
  return 0;
}

// Device overlap check vs host buffers_disjoint (see the header comment).
int run_check(std::uint64_t count) {
  nicgpu_qp* q = nullptr;
  assert(nicgpu_qp_create(&q, 0) == NICGPU_OK);
  std::size_t decided = 0, overlaps = 0, undecided = 0, bad = 0;
  for (std::uint64_t seed = 1; seed <= count; ++seed) {
    Rng r{seed * 7919 + 11};
    const int kind = static_cast<int>(r.below(5));
    const bool big = r.below(10) == 0;
    const std::size_t nrx = big ? 50000 + r.below(200000) : r.below(400);
    const std::size_t ntx = big ? 50000 + r.below(200000) : r.below(400);
    std::vector<RxDescriptor> rx(nrx);
    std::vector<TxDescriptor> tx(ntx);
    // RX ring ascending from address 0 with random gaps (0 = touching)
    std::uint64_t at = 0;
    for (auto& d : rx) {
      at += r.below(3) == 0 ? 0 : r.below(64);
      d.buffer_address = at;
      d.buffer_length = 1 + r.below(2048);
      at += d.buffer_length;
    }
    const std::uint64_t rx_end = at;
    for (auto& t : tx) {  // TX buffers after the ring, touching it or not
      at += r.below(2) ? 0 : r.below(32);
      t.buffer_address = at;
      t.length = 1 + r.below(1600);
      at += t.length;
    }
    std::uint64_t mem_size = at + r.below(64);
    if (kind == 1 && ntx && nrx) {  // some TX buffers overlap an RX buffer (or just touch one)
      for (int k = 0, m = 1 + static_cast<int>(r.below(3)); k < m; ++k) {
        const RxDescriptor& d = rx[r.below(static_cast<std::uint32_t>(nrx))];
        TxDescriptor& t = tx[r.below(static_cast<std::uint32_t>(ntx))];
        switch (r.below(3)) {
          case 0: t.buffer_address = d.buffer_address + r.below(d.buffer_length); break;
          case 1: t.buffer_address = d.buffer_address + d.buffer_length; break;  // touches: no overlap
          default: t.buffer_address = d.buffer_address > t.length ? d.buffer_address - t.length : 0; break;
        }
      }
    } else if (kind == 2 && nrx > 1) {  // two neighbouring RX buffers overlap
      const std::size_t j = 1 + r.below(static_cast<std::uint32_t>(nrx - 1));
      rx[j].buffer_address = rx[j - 1].buffer_address + r.below(rx[j - 1].buffer_length);
    } else if (kind == 3 && nrx > 1) {  // shuffled ring
      for (std::size_t j = nrx - 1; j > 0; --j) std::swap(rx[j], rx[r.below(static_cast<std::uint32_t>(j + 1))]);
    } else if (kind == 4) {  // invalid / clipped descriptors, a smaller image
      mem_size = rx_end ? rx_end - r.below(static_cast<std::uint32_t>(std::min<std::uint64_t>(rx_end, 4096))) : 0;
      for (auto& d : rx)
        if (r.below(8) == 0) d.buffer_length = 0;
      for (auto& t : tx) {
        if (r.below(4) == 0) t.buffer_address = r.below(static_cast<std::uint32_t>(mem_size + 1));
        if (r.below(8) == 0) t.length = 0;
      }
    }
    nicgpu_qp_view v{};
    assert(nicgpu_qp_reserve(q, ntx, nrx, &v) == NICGPU_OK);
    if (ntx) assert(nicgpu_memcpy_async(v.tx, tx.data(), ntx * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
    if (nrx) assert(nicgpu_memcpy_async(v.rx, rx.data(), nrx * sizeof(RxDescriptor), nullptr) == NICGPU_OK);
    int verdict = 9;
    assert(nicgpu_qp_check(q, mem_size, ntx, nrx, &verdict, nullptr) == NICGPU_OK);
    const bool host = rx_stage_detail::buffers_disjoint(mem_size, tx, rx);
    // the check's bounds (nicgpu_qp_check_bounds): TX spans [min start, max
    // end); RX spans [first span's start, max end) — the least start when the
    // ring ascends (verdict >= 0)
    {
      std::uint64_t bnd[4];
      assert(nicgpu_qp_check_bounds(q, bnd) == NICGPU_OK);
      std::uint64_t tlo = ~0ull, thi = 0, rfirst = ~0ull, rlo = ~0ull, rhi = 0;
      for (const auto& t : tx)
        if (t.length && t.buffer_address <= mem_size && t.length <= mem_size - t.buffer_address) {  // dma_ok
          tlo = std::min<std::uint64_t>(tlo, t.buffer_address);
          thi = std::max<std::uint64_t>(thi, t.buffer_address + t.length);
        }
      for (const auto& d : rx)
        if (d.buffer_length && d.buffer_address < mem_size) {
          const std::uint64_t e = d.buffer_address + std::min<std::uint64_t>(d.buffer_length, mem_size - d.buffer_address);
          if (rfirst == ~0ull) rfirst = d.buffer_address;
          rlo = std::min<std::uint64_t>(rlo, d.buffer_address);
          rhi = std::max(rhi, e);
        }
      // RX bounds are documented for rings the device decided (verdict >= 0:
      // ascending), where the first span's start is the least
      const bool ok_b = bnd[0] == tlo && bnd[1] == thi &&
                        (verdict < 0 || (bnd[2] == rfirst && bnd[3] == rhi && (rfirst == rlo || rhi == 0)));
      if (!ok_b) {
        std::printf("check seed %llu kind %d: bounds %llx %llx %llx %llx, host %llx %llx %llx(%llx) %llx\n",
                    (unsigned long long) seed, kind, (unsigned long long) bnd[0], (unsigned long long) bnd[1],
                    (unsigned long long) bnd[2], (unsigned long long) bnd[3], (unsigned long long) tlo,
                    (unsigned long long) thi, (unsigned long long) rfirst, (unsigned long long) rlo,
                    (unsigned long long) rhi);
        ++bad;
      }
    }
    if (verdict < 0) {
      ++undecided;
      if (kind == 0 || kind == 1) {  // an ascending ring apart is always decided
        std::printf("check seed %llu kind %d: undecided on an ascending ring\n", (unsigned long long) seed, kind);
        ++bad;
      }
    } else {
      ++decided;
      overlaps += verdict == 0;
      if ((verdict == 1) != host) {
        std::printf("check seed %llu kind %d (ntx %zu nrx %zu): device %d host %d\n", (unsigned long long) seed, kind, ntx,
                    nrx, verdict, int(host));
        ++bad;
      }
    }
  }
  nicgpu_qp_destroy(q);
  if (bad) return 1;
  std::printf("rx_stage_gpu_fuzz check: ok (%llu layouts: %zu decided on the device, %zu of them overlapping; %zu "
              "left to the host sort)\n",
              (unsigned long long) count, decided, overlaps, undecided);
  return 0;
}

// Edge cases of the device path's limits:
//  - a TX descriptor whose plan has more pieces than 32-bit piece indices
//    allow per descriptor (a 17 MB plain packet, TX-verified, then dropped for
//    its MTU: one piece per 64 KiB) makes nicgpu_qp_plan return
//    NICGPU_ERR_RANGE; the batch must then go to the host path and still equal
//    the host resolve;
//  - device descriptor arrays inside the image that an RX buffer of the same
//    batch overlaps: not modelled, process_batch must throw before writing.
int run_edges() {
  const std::size_t big = 17u << 20;  // > 256 * 65534 B
  const std::size_t mem_size = big + (1u << 20);
  std::vector<std::uint8_t> image(mem_size);
  Rng r{777};
  for (auto& b : image) b = r.byte();
  std::vector<TxDescriptor> tx(8);
  for (std::size_t i = 0; i < tx.size(); ++i) {
    TxDescriptor& t = tx[i];
    t.buffer_address = i == 3 ? 0 : big + i * 2048;
    t.length = i == 3 ? static_cast<std::uint32_t>(big) : 1518;
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum = ChecksumMode::Layer4;
    t.checksum_offload = i == 3 ? false : true;  // descriptor 3: TX verify of 17 MB
    t.checksum_value = oracle_compute_checksum(image.data() + t.buffer_address, t.length);
  }
  std::vector<RxDescriptor> rx(8);
  for (std::size_t j = 0; j < rx.size(); ++j) {
    rx[j].buffer_address = big + 512 * 1024 + j * 2048;
    rx[j].buffer_length = 2048;
    rx[j].checksum = ChecksumMode::None;
  }
  BatchedQueuePairConfig cfg;
  cfg.max_mtu = 9000;
  std::vector<std::uint8_t> host_img = image;
  test::CpuBackend cpu{host_img, nullptr, TupleSpec{}};
  RxBatchResult ho;
  QueuePairStats hs{};
  rx_stage_detail::BatchScratch scratch;
  rx_stage_detail::run_batch(cfg, mem_size, tx, rx, hs, ho, scratch, cpu);
  void* d = nullptr;
  assert(nicgpu_malloc(&d, mem_size + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
  BatchedQueuePair qp{cfg};
  RxBatchResult go;
  qp.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, tx, rx, go);
  std::vector<std::uint8_t> dev_img(mem_size);
  assert(nicgpu_memcpy_async(dev_img.data(), d, mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  bool ok = !go.timings.device && go.tx_completions.size() == ho.tx_completions.size() &&
            go.rx_completions.size() == ho.rx_completions.size() && host_img == dev_img;
  for (std::size_t i = 0; ok && i < ho.tx_completions.size(); ++i) ok = same(go.tx_completions[i], ho.tx_completions[i]);
  for (std::size_t i = 0; ok && i < ho.rx_completions.size(); ++i) ok = same(go.rx_completions[i], ho.rx_completions[i]);
  ok = ok && std::memcmp(&hs, &qp.stats(), sizeof(hs)) == 0;
  ok = ok && ho.tx_completions[3].status == static_cast<std::uint32_t>(CompletionCode::MtuExceeded);
  if (!ok) std::fprintf(stderr, "edges: the over-range batch differs from the host resolve\n");
  // the piece-count limit itself, straight through the C-ABI
  {
    nicgpu_qp* q = nullptr;
    assert(nicgpu_qp_create(&q, 0) == NICGPU_OK);
    nicgpu_qp_view v{};
    assert(nicgpu_qp_reserve(q, tx.size(), rx.size(), &v) == NICGPU_OK);
    assert(nicgpu_memcpy_async(v.tx, tx.data(), tx.size() * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
    std::uint64_t np = 0;
    const int st = nicgpu_qp_plan(q, static_cast<const std::uint8_t*>(d), mem_size, tx.size(), 9000, &np, &v, nullptr);
    if (st != NICGPU_ERR_RANGE) {
      std::fprintf(stderr, "edges: nicgpu_qp_plan returned %d, want NICGPU_ERR_RANGE\n", st);
      ok = false;
    }
    tx[3].length = 1518;  // the same batch without the huge packet plans normally: one piece per packet
    assert(nicgpu_memcpy_async(v.tx, tx.data(), tx.size() * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
    ok = ok && nicgpu_qp_plan(q, static_cast<const std::uint8_t*>(d), mem_size, tx.size(), 9000, &np, &v, nullptr) ==
                   NICGPU_OK && np == tx.size();
    nicgpu_qp_destroy(q);
  }
  // descriptor arrays inside the image, overwritten by an RX buffer
  {
    std::byte* base = static_cast<std::byte*>(d);
    const std::size_t ring_at = big + 256 * 1024;  // TX descriptors here, RX ring after them
    assert(nicgpu_memcpy_async(base + ring_at, tx.data(), tx.size() * sizeof(TxDescriptor), nullptr) == NICGPU_OK);
    assert(nicgpu_memcpy_async(base + ring_at + 4096, rx.data(), rx.size() * sizeof(RxDescriptor), nullptr) ==
           NICGPU_OK);
    std::vector<RxDescriptor> rx2 = rx;
    const DeviceDescriptors dd{reinterpret_cast<const TxDescriptor*>(base + ring_at), tx.size(),
                               reinterpret_cast<const RxDescriptor*>(base + ring_at + 4096), rx.size()};
    BatchedQueuePair qp2{cfg};
    RxBatchResult o2;
    qp2.process_batch(DeviceHostMemory{base, mem_size}, dd, o2);  // rings apart from every RX buffer: fine
    rx2[5].buffer_address = ring_at + 64;  // now RX descriptor 5 writes over the TX descriptor ring
    assert(nicgpu_memcpy_async(base + ring_at + 4096, rx2.data(), rx2.size() * sizeof(RxDescriptor), nullptr) ==
           NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    // popped as the reference pops host-backed rings (descriptor_ring.cpp:
    // 97-106): the product path against the driver with RingSlots on the CPU
    // backend over a copy of the same image
    std::vector<std::uint8_t> host(mem_size), after(mem_size);
    assert(nicgpu_memcpy_async(host.data(), base, mem_size, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    BatchedQueuePairConfig ccfg = cfg;
    ccfg.rss = nullptr;
    ccfg.on_interrupt = nullptr;
    test::CpuBackend cpu{host, nullptr, TupleSpec{}};
    RxBatchResult co;
    QueuePairStats cst{};
    rx_stage_detail::BatchScratch cs;
    const rx_stage_detail::RingSlots slots{ring_at, ring_at + 4096};
    rx_stage_detail::run_batch(ccfg, mem_size, tx, rx2, cst, co, cs, cpu, -1, nullptr, &slots);
    BatchedQueuePair qp3{cfg};
    qp3.process_batch(DeviceHostMemory{base, mem_size}, dd, o2);
    assert(nicgpu_memcpy_async(after.data(), base, mem_size, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    bool eq = !o2.timings.device && o2.tx_completions.size() == co.tx_completions.size() &&
              o2.rx_completions.size() == co.rx_completions.size() &&
              std::memcmp(&qp3.stats(), &cst, sizeof(cst)) == 0 && after == host;
    for (std::size_t i = 0; eq && i < co.tx_completions.size(); ++i) eq = same(o2.tx_completions[i], co.tx_completions[i]);
    for (std::size_t i = 0; eq && i < co.rx_completions.size(); ++i) eq = same(o2.rx_completions[i], co.rx_completions[i]);
    if (!eq) std::fprintf(stderr, "edges: an RX buffer over the descriptor ring: the product path differs from the driver\n");
    ok = ok && eq;
  }
  // a batch of more TX descriptors than the device context's 32-bit piece
  // indices allow (NICGPU_QP_MAX_TX): refused by nicgpu_qp_reserve, so the
  // stage takes the host path (equal to the host resolve) instead of throwing
  {
    const std::size_t ntx = NICGPU_QP_MAX_TX + 1;
    {
      nicgpu_qp* q = nullptr;
      assert(nicgpu_qp_create(&q, 0) == NICGPU_OK);
      nicgpu_qp_view v{};
      if (nicgpu_qp_reserve(q, ntx, 4, &v) != NICGPU_ERR_INVALID) {
        std::fprintf(stderr, "edges: nicgpu_qp_reserve accepted %zu TX descriptors\n", ntx);
        ok = false;
      }
      nicgpu_qp_destroy(q);
    }
    std::vector<TxDescriptor> btx(ntx);
    for (std::size_t i = 0; i < ntx; ++i) {  // every descriptor sends the same 64-B frame
      TxDescriptor& t = btx[i];
      t.buffer_address = big;
      t.length = 64;
      t.descriptor_index = static_cast<std::uint16_t>(i);
    }
    std::vector<RxDescriptor> brx(4);
    for (std::size_t j = 0; j < brx.size(); ++j) {
      brx[j].buffer_address = big + 512 * 1024 + j * 2048;
      brx[j].buffer_length = 2048;
    }
    std::vector<std::uint8_t> himg = image;
    test::CpuBackend hcpu{himg, nullptr, TupleSpec{}};
    RxBatchResult bh;
    QueuePairStats bhs{};
    rx_stage_detail::BatchScratch bscratch;
    rx_stage_detail::run_batch(cfg, mem_size, btx, brx, bhs, bh, bscratch, hcpu);
    assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
    BatchedQueuePair bqp{cfg};
    RxBatchResult bg;
    bool threw = false;
    try {
      bqp.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, btx, brx, bg);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "edges: a batch of %zu TX descriptors threw: %s\n", ntx, e.what());
      threw = true;
    }
    bool same_all = !threw && !bg.timings.device && bg.tx_completions.size() == ntx &&
                    bg.rx_completions.size() == bh.rx_completions.size() &&
                    std::memcmp(&bhs, &bqp.stats(), sizeof(bhs)) == 0;
    for (std::size_t i = 0; same_all && i < ntx; ++i) same_all = same(bg.tx_completions[i], bh.tx_completions[i]);
    for (std::size_t i = 0; same_all && i < bh.rx_completions.size(); ++i)
      same_all = same(bg.rx_completions[i], bh.rx_completions[i]);
    if (!same_all) std::fprintf(stderr, "edges: the over-count batch differs from the host resolve\n");
    ok = ok && same_all;
  }
  // a first batch whose device plan outgrows the piece buffers the stage sizes
  // ahead (ntx + ntx / 4 + 64 pieces): TSO with a small mss, ~60 segments and
  // 62 pieces per descriptor.  The resolve finishes with NICGPU_ERR_AGAIN, the
  // stage redoes the batch once with the grown buffers (timings.replans == 1),
  // and the result equals the host resolve; the next batch fits at once.
  bool replanned = false;
  {
    const std::size_t ntx = 96, nrx = ntx * 64;
    std::vector<TxDescriptor> ttx(ntx);
    for (std::size_t i = 0; i < ntx; ++i) {
      TxDescriptor& t = ttx[i];
      t.buffer_address = big + (i % 8) * 2048;
      t.length = 1518;
      t.descriptor_index = static_cast<std::uint16_t>(i);
      t.tso_enabled = true;
      t.mss = static_cast<std::uint16_t>(24 + i % 3);
      t.header_length = 54;
      t.checksum_offload = true;
    }
    std::vector<RxDescriptor> trx(nrx);
    // distinct 80-B RX buffers after the TX frames (segments are 54 + <= 26 B)
    const std::size_t rx_base = big + 8 * 2048;
    for (std::size_t j = 0; j < nrx; ++j) {
      trx[j].buffer_address = rx_base + j * 80;
      trx[j].buffer_length = 80;
      trx[j].checksum = ChecksumMode::None;
    }
    assert(rx_base + nrx * 80 <= mem_size);
    std::vector<std::uint8_t> timg = image;
    test::CpuBackend tcpu{timg, nullptr, TupleSpec{}};
    RxBatchResult th;
    QueuePairStats ths{};
    rx_stage_detail::BatchScratch tscratch;
    rx_stage_detail::run_batch(cfg, mem_size, ttx, trx, ths, th, tscratch, tcpu);
    assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
    BatchedQueuePair tqp{cfg};
    RxBatchResult tg;
    tqp.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, ttx, trx, tg);
    std::vector<std::uint8_t> tdev(mem_size);
    assert(nicgpu_memcpy_async(tdev.data(), d, mem_size, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    replanned = tg.timings.device && tg.timings.replans == 1;
    bool eq = replanned && tg.tx_completions.size() == th.tx_completions.size() &&
              tg.rx_completions.size() == th.rx_completions.size() && tdev == timg &&
              std::memcmp(&ths, &tqp.stats(), sizeof(ths)) == 0;
    for (std::size_t i = 0; eq && i < th.tx_completions.size(); ++i) eq = same(tg.tx_completions[i], th.tx_completions[i]);
    for (std::size_t i = 0; eq && i < th.rx_completions.size(); ++i) eq = same(tg.rx_completions[i], th.rx_completions[i]);
    // the same stage again: its buffers now fit the plan
    RxBatchResult tg2;
    tqp.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, ttx, trx, tg2);
    eq = eq && tg2.timings.device && tg2.timings.replans == 0 && tg2.tx_completions.size() == th.tx_completions.size();
    if (!eq)
      std::fprintf(stderr, "edges: the outgrown plan (device %d, replans %u) differs from the host resolve\n",
                   int(tg.timings.device), tg.timings.replans);
    ok = ok && eq;
  }
  // positions the relaxation does not settle in 8 steps: 400 TSO packets of 3
  // segments against a ring where one buffer in three is too small for a
  // segment, so almost every packet ends early somewhere and shifts all the
  // later ones.  The stage walks the multi-descriptor packets (timings.walked)
  // and the result equals the host resolve, with no host tail.
  bool walked = false;
  {
    const std::size_t ntx = 400, nrx = ntx * 3;
    std::vector<TxDescriptor> wtx(ntx);
    for (std::size_t i = 0; i < ntx; ++i) {
      TxDescriptor& t = wtx[i];
      t.buffer_address = big + (i % 8) * 2048;
      t.length = 54 + 3 * 100;
      t.descriptor_index = static_cast<std::uint16_t>(i);
      t.tso_enabled = true;
      t.mss = 100;
      t.header_length = 54;
    }
    std::vector<RxDescriptor> wrx(nrx);
    const std::size_t rx_base = big + 8 * 2048;
    Rng wr{4242};
    for (std::size_t j = 0; j < nrx; ++j) {
      wrx[j].buffer_address = rx_base + j * 256;
      wrx[j].buffer_length = wr.below(3) == 0 ? 100 : 256;  // 100 B: a 154-B segment does not fit
      wrx[j].checksum = ChecksumMode::None;
    }
    assert(rx_base + nrx * 256 <= mem_size);
    std::vector<std::uint8_t> wimg = image;
    test::CpuBackend wcpu{wimg, nullptr, TupleSpec{}};
    RxBatchResult wh;
    QueuePairStats whs{};
    rx_stage_detail::BatchScratch wscratch;
    rx_stage_detail::run_batch(cfg, mem_size, wtx, wrx, whs, wh, wscratch, wcpu);
    assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
    BatchedQueuePair wqp{cfg};
    RxBatchResult wg;
    wqp.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, wtx, wrx, wg);
    std::vector<std::uint8_t> wdev(mem_size);
    assert(nicgpu_memcpy_async(wdev.data(), d, mem_size, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
    walked = wg.timings.device && wg.timings.walked && !wg.timings.host_tail;
    bool eq = walked && wg.tx_completions.size() == wh.tx_completions.size() &&
              wg.rx_completions.size() == wh.rx_completions.size() && wdev == wimg &&
              std::memcmp(&whs, &wqp.stats(), sizeof(whs)) == 0 && wg.rx_consumed == wh.rx_consumed;
    for (std::size_t i = 0; eq && i < wh.tx_completions.size(); ++i) eq = same(wg.tx_completions[i], wh.tx_completions[i]);
    for (std::size_t i = 0; eq && i < wh.rx_completions.size(); ++i) eq = same(wg.rx_completions[i], wh.rx_completions[i]);
    if (!eq)
      std::fprintf(stderr, "edges: the walked batch (device %d walked %d host_tail %d) differs from the host resolve\n",
                   int(wg.timings.device), int(wg.timings.walked), int(wg.timings.host_tail));
    ok = ok && eq;
  }
  nicgpu_free(d);
  if (ok)
    std::printf("rx_stage_gpu_fuzz edges: ok (over-range plan and over-count batch took the host path; ring "
                "overwrite refused; an outgrown plan was redone once: %d; unsettled positions walked: %d)\n",
                int(replanned), int(walked));
  return ok ? 0 : 1;
}

}  // namespace

// RSS dispatch into per-queue completion rings (nic::RssCompletionRings):
// two C3 batches of 64 K descriptors with RSS, their Success completions
// posted into 16 rings of 2048 entries (so the busy queues refuse), 1000
// entries polled from every ring between the batches, then every ring drained
// — from the device lists of a batch that kept its results in HBM and from
// the host lists of the same batch with host results, against
// nic::CompletionQueue's semantics restated here (src/completion_queue.cpp:30-53).
int run_rings() {
  const std::size_t n = 65536, Q = 16, kRing = 2048;
  Rng r{909};
  std::vector<std::size_t> lens(n);
  for (auto& L : lens) {
    const std::uint32_t k = r.below(12);
    L = k < 7 ? 64 : (k < 11 ? 576 : 1518);
  }
  std::size_t tx_bytes = 0;
  for (auto L : lens) tx_bytes += (L + 15) & ~std::size_t{15};
  const std::size_t mem_size = tx_bytes + n * 2048;
  std::vector<std::uint8_t> image(mem_size, 0);
  std::vector<TxDescriptor> tx(n);
  std::size_t at = 0;
  for (std::size_t i = 0; i < n; ++i) {
    std::uint8_t* p = image.data() + at;
    for (std::size_t b = 0; b < lens[i]; ++b) p[b] = r.byte();
    p[12] = 0x08;
    p[13] = 0x00;
    TxDescriptor& t = tx[i];
    t.buffer_address = at;
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum_offload = true;
    t.checksum = ChecksumMode::None;
    at += (lens[i] + 15) & ~std::size_t{15};
  }
  std::vector<RxDescriptor> rx(n);
  for (std::size_t j = 0; j < n; ++j) {
    rx[j].buffer_address = tx_bytes + j * 2048;
    rx[j].buffer_length = 2048;
    rx[j].descriptor_index = static_cast<std::uint16_t>(j);
    // a few short buffers: BufferTooSmall completions stay out of the rings
    if (r.below(16) == 0) rx[j].buffer_length = 60;
  }
  std::vector<std::uint16_t> table(128);
  for (int i = 0; i < 128; ++i) table[i] = static_cast<std::uint16_t>(i % Q);
  RssEngine rss_a{RssConfig{kMsKey, table}}, rss_b{RssConfig{kMsKey, table}};
  void* d = nullptr;
  assert(nicgpu_malloc(&d, mem_size + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
  const DeviceHostMemory dm{static_cast<std::byte*>(d), mem_size};
  BatchedQueuePairConfig ca, cb;
  ca.rss = &rss_a;
  cb.rss = &rss_b;
  cb.results_on_device = true;
  BatchedQueuePair qa{ca}, qb{cb};
  RssCompletionRings ring_host{Q, kRing}, ring_dev{Q, kRing};
  // CompletionQueue restated: a ring per queue
  struct Sim {
    std::vector<CompletionEntry> e;
    std::size_t prod = 0, cons = 0, count = 0, refused = 0;
  };
  std::vector<Sim> sim(Q);
  for (auto& x : sim) x.e.resize(kRing);
  bool ok = true;
  auto same_entry = [](const CompletionEntry& a, const CompletionEntry& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; };
  std::size_t posted_total = 0, refused_total = 0;
  for (int batch = 0; batch < 2 && ok; ++batch) {
    RxBatchResult ra, rb;
    qa.process_batch(dm, tx, rx, ra);
    qb.process_batch(dm, tx, rx, rb);
    ok = ok && ra.timings.device && rb.timings.device && rb.dev.queue_which != nullptr;
    // expected: Success completions in posting order into their queue's ring
    for (std::size_t j = 0; j < ra.rx_completions.size(); ++j) {
      if (ra.rx_completions[j].status != 0) continue;
      Sim& x = sim[ra.rx_queue[j]];
      if (x.count == kRing) {
        ++x.refused;
        ++refused_total;
        continue;
      }
      x.e[x.prod] = ra.rx_completions[j];
      x.prod = (x.prod + 1) % kRing;
      ++x.count;
      ++posted_total;
    }
    ring_host.post(ra);
    ring_dev.post(rb);
    for (std::size_t q = 0; q < Q && ok; ++q) {
      const auto sh = ring_host.state(q), sd = ring_dev.state(q);
      ok = sh.producer == sim[q].prod && sh.count == sim[q].count && sh.refused == sim[q].refused &&
           sd.producer == sh.producer && sd.consumer == sh.consumer && sd.count == sh.count && sd.refused == sh.refused;
      if (!ok) std::fprintf(stderr, "rings: batch %d queue %zu state differs\n", batch, q);
    }
    // the consumer takes 1000 from every ring (all of them after the last batch)
    for (std::size_t q = 0; q < Q && ok; ++q) {
      const std::size_t k = batch == 0 ? 1000 : kRing;
      const auto a = ring_host.poll(q, k), b = ring_dev.poll(q, k);
      ok = a.size() == b.size() && a.size() == std::min(k, sim[q].count);
      for (std::size_t i = 0; ok && i < a.size(); ++i) {
        ok = same_entry(a[i], sim[q].e[(sim[q].cons + i) % kRing]) && same_entry(b[i], a[i]);
      }
      if (!ok) std::fprintf(stderr, "rings: batch %d queue %zu polled entries differ\n", batch, q);
      sim[q].cons = (sim[q].cons + a.size()) % kRing;
      sim[q].count -= a.size();
    }
  }
  nicgpu_free(d);
  if (!ok) return 1;
  std::printf("rx_stage_gpu_fuzz rings: ok (%zu queues x %zu entries, %zu completions posted, %zu refused by full rings; "
              "device lists and host lists equal the CompletionQueue semantics)\n",
              Q, kRing, posted_total, refused_total);
  return 0;
}

// BatchedQueueManager's fused batch (every queue pair's batch and ring in one
// device batch, segments with their own queue id, MTU and ring) against each
// queue pair's batch run alone through the host resolve (run_batch over the
// CPU backend, which rx_stage_fuzz pins to the reference QueuePair): random
// queue counts, per-queue MTUs, rings that run short or are empty, TSO, VLAN,
// faults, every queue's buffers in a region of its own (queues disjoint).
// RSS through one shared engine or one engine per queue pair (equal configs);
// results on the host or left on the device; one sequence in three on a
// HostMemory.  Two rounds per seed (ring leftovers carried over).
std::size_t g_qm_fused = 0, g_qm_rounds = 0, g_qm_himg = 0, g_qm_late = 0;
int run_qm(std::uint64_t seed) {
  Rng r{seed * 6151 + 17};
  const std::size_t Q = 1 + r.below(12);
  const std::size_t region = 1u << 20;
  const std::size_t mem_size = Q * region;
  std::vector<std::uint8_t> image(mem_size);
  for (auto& b : image) b = r.byte();
  const bool shared_engine = r.below(2) == 0, rss_on = r.below(5) != 0, keep = r.below(3) == 0;
  const bool himg = r.below(3) == 0;
  // one manager in three: drains the fused batch resolves with its RX
  // verifies deferred to the delivery (no TX verify, no TSO)
  const bool late_case = seed % 3 == 2;
  std::vector<std::uint16_t> table(64 + r.below(100));
  for (auto& t : table) t = static_cast<std::uint16_t>(r.below(24));
  const RssConfig rss_cfg{kMsKey, table};
  std::vector<std::unique_ptr<RssEngine>> dev_eng, ref_eng;
  for (std::size_t q = 0; q < (shared_engine ? 1 : Q); ++q) {
    dev_eng.push_back(std::make_unique<RssEngine>(rss_cfg));
    ref_eng.push_back(std::make_unique<RssEngine>(rss_cfg));
  }
  std::vector<BatchedQueuePairConfig> cfg(Q);
  const std::size_t mtus[] = {9000, 1500, 3000};
  for (std::size_t q = 0; q < Q; ++q) {
    cfg[q].queue_id = static_cast<std::uint16_t>(r.below(9));
    cfg[q].max_mtu = mtus[r.below(3)];
    cfg[q].weight = static_cast<std::uint8_t>(r.below(4));
    cfg[q].results_on_device = keep;
  }
  std::vector<std::uint8_t> ref_img = image;
  void* d = nullptr;
  assert(nicgpu_malloc(&d, mem_size + 64) == NICGPU_OK);
  assert(nicgpu_memcpy_async(d, image.data(), mem_size, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  FlatHostMemory hm(himg ? mem_size : 0);
  if (himg) std::memcpy(hm.data(), image.data(), mem_size);
  std::vector<BatchedQueuePairConfig> dcfg = cfg;
  for (std::size_t q = 0; q < Q; ++q) dcfg[q].rss = rss_on ? dev_eng[shared_engine ? 0 : q].get() : nullptr;
  BatchedQueueManager qm{BatchedQueueManagerConfig{dcfg}};
  std::vector<QueuePairStats> ref_st(Q);
  std::vector<std::vector<RxDescriptor>> ring(Q);
  bool ok = true;
  for (int round = 0; round < 2 && ok; ++round) {
    std::vector<std::vector<TxDescriptor>> tx(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      const std::size_t base = q * region;
      const std::size_t ntx = r.below(5) == 0 ? 0 : 1 + r.below(r.below(4) == 0 ? 3000 : 200);
      for (std::size_t i = 0; i < ntx; ++i) {
        TxDescriptor t{};
        const std::size_t L = r.below(8) == 0 ? r.below(60) : (r.below(3) ? 64 + r.below(1500) : 1518);
        t.buffer_address = base + r.below(static_cast<std::uint32_t>(region / 2 - 2048));
        if (r.below(80) == 0) t.buffer_address = mem_size + 1;  // a DMA read fault
        t.length = static_cast<std::uint32_t>(L);
        t.descriptor_index = static_cast<std::uint16_t>(i);
        t.checksum = static_cast<ChecksumMode>(r.below(3));
        t.checksum_offload = late_case || r.below(4) != 0;
        t.checksum_value = static_cast<std::uint16_t>(r.below(65536));
        if (r.below(8) == 0 && !late_case) {
          t.tso_enabled = true;
          t.mss = static_cast<std::uint16_t>(100 + r.below(1400));
          t.header_length = static_cast<std::uint16_t>(14 + r.below(60));
        }
        if (r.below(8) == 0) {
          t.vlan_insert = true;
          t.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
        }
        tx[q].push_back(t);
      }
      // the ring: leftovers first, then new descriptors in the upper half
      const std::size_t add = r.below(4) == 0 ? r.below(static_cast<std::uint32_t>(ntx + 1)) : ntx + r.below(20);
      const std::size_t at0 = base + region / 2 + (round ? region / 4 : 0);
      for (std::size_t j = 0; j < add; ++j) {
        RxDescriptor x{};
        const std::size_t slot = (region / 4) / std::max<std::size_t>(add, 1);
        x.buffer_address = at0 + j * std::min<std::size_t>(slot, 2048);
        x.buffer_length = static_cast<std::uint32_t>(r.below(10) ? std::min<std::size_t>(slot, 2048) : r.below(200));
        x.descriptor_index = static_cast<std::uint16_t>(j);
        x.checksum = static_cast<ChecksumMode>(r.below(3));
        x.checksum_offload = r.below(3) != 0;
        x.vlan_strip = r.below(4) == 0;
        x.vlan_present = r.below(4) == 0;
        x.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
        x.gro_enabled = r.below(4) == 0;
        ring[q].push_back(x);
      }
    }
    // the reference: each queue pair alone, host resolve over the CPU backend
    std::vector<RxBatchResult> want(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      BatchedQueuePairConfig c = cfg[q];
      c.rss = rss_on ? ref_eng[shared_engine ? 0 : q].get() : nullptr;
      c.results_on_device = false;
      test::CpuBackend cpu{ref_img, c.rss, TupleSpec{}};
      rx_stage_detail::BatchScratch scratch;
      rx_stage_detail::run_batch(c, mem_size, tx[q], ring[q], ref_st[q], want[q], scratch, cpu);
    }
    std::vector<QueueBatch> b(Q);
    for (std::size_t q = 0; q < Q; ++q) b[q] = QueueBatch{tx[q], ring[q]};
    std::vector<RxBatchResult> got;
    if (himg) qm.process_batch(hm, b, got);
    else qm.process_batch(DeviceHostMemory{static_cast<std::byte*>(d), mem_size}, b, got);
    g_qm_fused += qm.last_fused();
    g_qm_rounds += 1;
    if (qm.last_fused() && !got.empty() && got[0].timings.deferred) g_qm_late += 1;
    for (std::size_t q = 0; q < Q && ok; ++q) {
      RxBatchResult& g = got[q];
      if (keep && !materialize(g)) {
        std::fprintf(stderr, "qm seed %llu: results on the device not as documented\n", (unsigned long long) seed);
        ok = false;
        break;
      }
      const RxBatchResult& w = want[q];
      bool e = g.tx_completions.size() == w.tx_completions.size() && g.rx_completions.size() == w.rx_completions.size() &&
               g.rx_consumed == w.rx_consumed;
      for (std::size_t i = 0; e && i < w.tx_completions.size(); ++i) e = same(g.tx_completions[i], w.tx_completions[i]);
      for (std::size_t i = 0; e && i < w.rx_completions.size(); ++i) e = same(g.rx_completions[i], w.rx_completions[i]);
      const QueuePairStats gs = *qm.queue_stats(q);
      e = e && std::memcmp(&ref_st[q], &gs, sizeof(QueuePairStats)) == 0;
      if (rss_on) e = e && g.rx_hash == w.rx_hash && g.rx_queue == w.rx_queue && g.queues == w.queues;
      if (!e) {
        std::fprintf(stderr, "qm seed %llu round %d queue %zu/%zu differs (fused %d, tx %zu/%zu rx %zu/%zu)\n",
                     (unsigned long long) seed, round, q, Q, qm.last_fused(), g.tx_completions.size(),
                     w.tx_completions.size(), g.rx_completions.size(), w.rx_completions.size());
        ok = false;
      }
    }
    for (std::size_t q = 0; q < Q; ++q) ring[q].erase(ring[q].begin(), ring[q].begin() + want[q].rx_consumed);
  }
  if (ok && rss_on)
    for (std::size_t k = 0; k < dev_eng.size(); ++k)
      ok = ok && dev_eng[k]->stats().hashes == ref_eng[k]->stats().hashes &&
           dev_eng[k]->stats().queue_hits == ref_eng[k]->stats().queue_hits;
  std::vector<std::uint8_t> after(mem_size);
  if (himg) {
    std::memcpy(after.data(), hm.data(), mem_size);
    g_qm_himg += 1;
  } else {
    assert(nicgpu_memcpy_async(after.data(), d, mem_size, nullptr) == NICGPU_OK);
    assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  }
  if (ok && after != ref_img) {
    std::fprintf(stderr, "qm seed %llu: memory differs\n", (unsigned long long) seed);
    ok = false;
  }
  if (!ok && rss_on) std::fprintf(stderr, "qm seed %llu: (engines %s)\n", (unsigned long long) seed, shared_engine ? "shared" : "own");
  nicgpu_free(d);
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  assert(gpu_device_count() >= 1);
  if (argc > 1 && std::strcmp(argv[1], "rings") == 0) return run_rings();
  if (argc > 1 && std::strcmp(argv[1], "check") == 0) return run_check(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 400);
  if (argc > 1 && std::strcmp(argv[1], "edges") == 0) return run_edges();
  if (argc > 1 && std::strcmp(argv[1], "qm") == 0) {
    const std::uint64_t count = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 60;
    int bad = 0;
    for (std::uint64_t s = 1; s <= count; ++s) bad += run_qm(s);
    if (bad) return 1;
    if (count >= 20 && g_qm_late == 0) {
      std::fprintf(stderr, "qm: no fused drain deferred its RX verifies\n");
      return 1;
    }
    std::printf("rx_stage_gpu_fuzz qm: ok (%llu managers, %zu of %zu drains fused, %zu on a HostMemory, %zu fused "
                "drains with the RX verifies deferred)\n",
                (unsigned long long) count, g_qm_fused, g_qm_rounds, g_qm_himg, g_qm_late);
    return 0;
  }
  if (argc > 1 && std::strcmp(argv[1], "pipeline") == 0) {
    int a = 2;
    if (argc > a && std::strcmp(argv[a], "himg") == 0) {
      g_force_himg = true;
      ++a;
    }
    const std::uint64_t count = argc > a ? std::strtoull(argv[a], nullptr, 10) : 40;
    int bad = 0;
    for (std::uint64_t s = 1; s <= count; ++s) bad += run_pipeline(s);
    if (bad) return 1;
    // both kinds of overlapped resolve happened (unless every sequence ran on a HostMemory)
    if (!g_force_himg && count >= 10 && (g_pipe_overlapped == 0 || g_pipe_redone == 0)) {
      std::fprintf(stderr, "pipeline: %zu overlapped resolves stood, %zu redone: both paths expected\n",
                   g_pipe_overlapped, g_pipe_redone);
      return 1;
    }
    if (count >= 10 && g_pipe_late == 0) {
      std::fprintf(stderr, "pipeline: no batch deferred its RX verifies\n");
      return 1;
    }
    std::printf("rx_stage_gpu_fuzz pipeline: ok (%llu sequences, %zu batches, %zu of them on the host path, %zu "
                "with device descriptors, %zu on a HostMemory, %zu results left on the device; overlapped "
                "resolves: %zu stood, %zu redone behind earlier writes; %zu with the RX verifies deferred)\n",
                (unsigned long long) count, g_pipe_batches, g_pipe_host, g_pipe_devdesc, g_pipe_himg, g_keep,
                g_pipe_overlapped, g_pipe_redone, g_pipe_late);
    return 0;
  }
  if (argc > 1 && std::strcmp(argv[1], "full") == 0) {
    bool dev = false, keep = false;
    for (int a = 3; a < argc; ++a) {
      dev |= std::strcmp(argv[a], "dev") == 0;
      keep |= std::strcmp(argv[a], "keep") == 0;
    }
    return run_full(argc > 2 ? argv[2] : "c3", dev, keep);
  }
  const std::uint64_t first = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
  const std::uint64_t count = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 300;
  int bad = 0;
  for (std::uint64_t s = first; s < first + count; ++s) bad += run_case(s);
  if (bad) return 1;
  if (count >= 30 && (g_late == 0 || g_late_fail == 0)) {
    std::fprintf(stderr, "fuzz: %zu batches deferred their RX verifies (%zu failed): both expected\n", g_late, g_late_fail);
    return 1;
  }
  std::printf("rx_stage_gpu_fuzz: ok (%llu batches, %zu resolved on the device, %zu of them with a host tail, %zu "
              "running out of RX descriptors, %zu with device descriptors, %zu with results left on the device, "
              "%zu interrupt callbacks equal, %zu also on a HostMemory (%zu staged per descriptor); %zu with the RX "
              "verifies deferred to the delivery, %zu of those failing)\n",
              (unsigned long long) count, g_device, g_tail, g_short, g_devdesc, g_keep, g_irq, g_himg, g_himg_sparse,
              g_late, g_late_fail);
  return 0;
}
