// rx_stage_fuzz.cpp — randomised batches through the reference QueuePair
// (src/queue_pair.cpp:67-460, compiled from /root/reference in this
// container) and through nic::BatchedQueuePair's driver
// (rx_stage_detail::run_batch with the CPU backend of cpu_backend.h: piece
// sums from the oracle), in the same process.  Compared per batch: every
// TX/RX CompletionEntry in posting order, QueuePairStats, RX descriptors
// consumed, interrupts delivered (the reference's InterruptDispatcher with a
// packet threshold of 1), the whole memory image after the DMA writes, and the
// RSS hash/queue of every frame delivered with Success against the bytes the
// reference's DMA engine wrote for it (recorded as they are written, so a
// buffer that a later segment overwrites is hashed as delivered).
// One batch in three makes RX buffers overlap: recycled buffers, buffers
// straddling the previous one, and buffers inside the TX region.
//
//   rx_stage_fuzz <first_seed> <count>
#undef NDEBUG
#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nic/dma_engine.h"
#include "nic/interrupt_dispatcher.h"
#include "nic/queue_pair.h"
#include "nic/rx_stage.h"
#include "nic/simple_host_memory.h"
#include "cpu_backend.h"
#include "fault_model.h"
#include "oracle.h"

using namespace nic;

namespace {

std::size_t g_overlapping = 0, g_split = 0, g_snap = 0;  // batches that took each careful step
std::size_t g_faulty = 0;  // batches on a memory with its own DMA faults
int g_steps_max = 0;                                        // most relaxation steps a batch needed
std::size_t g_split_pieces_saved = 0;                       // pieces the split plans did without

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

bool same(const QueuePairStats& a, const QueuePairStats& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

// SimpleHostMemory that records every successful write (the RX segment DMA
// writes of QueuePair::handle_rx_segment, :416-426) in order.
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

// Balance a buffer so that compute_checksum(buf) == 0 by adjusting the 16-bit
// word at even offset `at` (needs at + 2 <= size).
void balance(std::vector<std::uint8_t>& b, std::size_t at) {
  b[at] = b[at + 1] = 0;
  const std::uint16_t c = oracle_compute_checksum(b.data(), b.size());  // ~sum
  b[at] = static_cast<std::uint8_t>(c >> 8);
  b[at + 1] = static_cast<std::uint8_t>(c);
}

// Pairwise definition of rx_stage_detail::buffers_disjoint.
bool disjoint_brute(std::size_t mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx) {
  auto rxs = [&](const RxDescriptor& x, std::uint64_t& a, std::uint64_t& b) {
    if (x.buffer_address >= mem || x.buffer_length == 0) return false;
    a = x.buffer_address;
    b = a + std::min<std::uint64_t>(x.buffer_length, mem - a);
    return true;
  };
  for (std::size_t j = 0; j < rx.size(); ++j) {
    std::uint64_t a, b, c, d;
    if (!rxs(rx[j], a, b)) continue;
    for (std::size_t k = j + 1; k < rx.size(); ++k)
      if (rxs(rx[k], c, d) && c < b && a < d) return false;
    for (const TxDescriptor& t : tx) {
      if (t.length == 0 || t.buffer_address > mem || t.length > mem - t.buffer_address) continue;
      if (t.buffer_address < b && a < t.buffer_address + t.length) return false;
    }
  }
  return true;
}

// buffers_disjoint on batches large enough to run as parallel chunks (the
// fuzz batches run as one), against a sort-based check: ring layouts, an
// overlap at a random place (often a chunk seam), unsorted and invalid entries.
int check_disjoint_large() {
  Rng r{99};
  for (int it = 0; it < 60; ++it) {
    const std::size_t ntx = 1 + r.below(300000), nrx = 1 + r.below(300000);
    std::vector<TxDescriptor> tx(ntx);
    std::vector<RxDescriptor> rx(nrx);
    std::uint64_t at = 0;
    for (auto& t : tx) {
      t.buffer_address = at;
      t.length = r.below(10) == 0 ? 0 : 1 + r.below(2000);
      at += t.length + r.below(3);
    }
    for (auto& x : rx) {
      x.buffer_address = at;
      x.buffer_length = r.below(20) == 0 ? 0 : 1 + r.below(3000);
      at += x.buffer_length + r.below(3);
    }
    const std::size_t mem = at - r.below(2000);
    const std::uint32_t kind = r.below(6);
    if (kind == 1) {  // one RX buffer straddles its successor
      const std::size_t j = r.below(static_cast<std::uint32_t>(nrx));
      if (j + 1 < nrx) rx[j].buffer_length = static_cast<std::uint32_t>(rx[j + 1].buffer_address - rx[j].buffer_address + 1);
    } else if (kind == 2) {  // one RX buffer inside the TX region
      rx[r.below(static_cast<std::uint32_t>(nrx))].buffer_address = r.below(static_cast<std::uint32_t>(std::min<std::uint64_t>(at, 1u << 31)));
    } else if (kind == 3) {  // TX out of order
      std::swap(tx[r.below(static_cast<std::uint32_t>(ntx))], tx[r.below(static_cast<std::uint32_t>(ntx))]);
    } else if (kind == 4) {  // RX out of order (still disjoint)
      std::swap(rx[r.below(static_cast<std::uint32_t>(nrx))], rx[r.below(static_cast<std::uint32_t>(nrx))]);
    } else if (kind == 5) {  // invalid RX entries sprinkled in
      for (int k = 0; k < 50; ++k) rx[r.below(static_cast<std::uint32_t>(nrx))].buffer_address = mem + r.below(100);
    }
    // sort-based reference
    std::vector<std::pair<std::uint64_t, std::uint64_t>> rs, ts;
    for (const auto& x : rx)
      if (x.buffer_address < mem && x.buffer_length)
        rs.emplace_back(x.buffer_address, x.buffer_address + std::min<std::uint64_t>(x.buffer_length, mem - x.buffer_address));
    for (const auto& t : tx)
      if (t.length && t.buffer_address <= mem && t.length <= mem - t.buffer_address)
        ts.emplace_back(t.buffer_address, t.buffer_address + t.length);
    std::sort(rs.begin(), rs.end());
    bool expect = true;
    for (std::size_t i = 1; i < rs.size(); ++i) expect = expect && rs[i].first >= rs[i - 1].second;
    for (const auto& [a, b] : ts) {
      auto it = std::upper_bound(rs.begin(), rs.end(), std::pair<std::uint64_t, std::uint64_t>(a, ~std::uint64_t{0}));
      if (it != rs.begin() && std::prev(it)->second > a) expect = false;
      if (it != rs.end() && it->first < b) expect = false;
    }
    if (rx_stage_detail::buffers_disjoint(mem, tx, rx) != expect) {
      std::fprintf(stderr, "buffers_disjoint: large case %d (kind %u) differs\n", it, kind);
      return 1;
    }
  }
  return 0;
}

int run_case(std::uint64_t seed) {
  Rng r{seed * 7919 + 1};
  const std::size_t ntx = 1 + r.below(120);
  const std::size_t nrx = r.below(220);
  const std::size_t mtus[] = {9000, 1500, 3000, 65535};
  const std::size_t max_mtu = mtus[r.below(4)];
  std::vector<TxDescriptor> tx(ntx);
  std::vector<std::vector<std::uint8_t>> pkts(ntx);
  std::vector<std::uint64_t> addr(ntx);
  std::size_t at = 0;
  for (std::size_t i = 0; i < ntx; ++i) {
    const std::uint32_t pick = r.below(16);
    std::size_t L = pick < 4 ? r.below(70) : (pick < 9 ? 60 + r.below(1500) : (pick < 14 ? 9000 : 9000 + r.below(70000)));
    auto& p = pkts[i];
    p.resize(L);
    const bool zero = r.below(40) == 0;
    for (auto& b : p) b = zero ? 0 : r.byte();
    if (L >= 16 && r.below(2)) balance(p, 10);
    at += r.below(3) == 0 ? r.below(9) : 0;
    addr[i] = at;
    at += L;
    TxDescriptor& t = tx[i];
    t.buffer_address = addr[i];
    t.length = static_cast<std::uint32_t>(L);
    t.descriptor_index = static_cast<std::uint16_t>(r.below(65536));
    t.checksum = static_cast<ChecksumMode>(r.below(3));
    t.checksum_offload = r.below(2);
    const std::uint16_t good = oracle_compute_checksum(p.data(), L);
    t.checksum_value = r.below(4) == 0 ? static_cast<std::uint16_t>(r.below(65536)) : good;
    if (r.below(3) == 0) {
      t.tso_enabled = r.below(2);
      t.gso_enabled = !t.tso_enabled || r.below(3) == 0;
      const std::uint32_t mp = r.below(10);
      t.mss = static_cast<std::uint16_t>(mp == 0 ? 0 : (mp == 1 ? 9001 + r.below(3) : (mp < 4 ? 1 + r.below(9) : 50 + r.below(2000))));
      const std::uint32_t hp = r.below(8);
      t.header_length = static_cast<std::uint16_t>(hp == 0 ? r.below(4) : (hp == 1 ? L + r.below(2) : (hp == 2 ? r.below(12) : 14 + r.below(60))));
    }
    if (r.below(4) == 0) {
      t.vlan_insert = true;
      t.vlan_tag = static_cast<std::uint16_t>(r.below(65536));
    }
  }
  at = (at + 15) & ~std::size_t{15};
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    RxDescriptor& x = rx[j];
    const std::uint32_t bp = r.below(8);
    x.buffer_length = bp == 0 ? r.below(200) : (bp < 4 ? 2000 : 9300);
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
  // overlapping buffers: the reference writes them in order (last write wins)
  // and reads a TX buffer after the earlier segments' writes
  const bool alias = r.below(3) == 0;
  if (alias && nrx > 1) {
    for (std::size_t j = 1; j < nrx; ++j) {
      RxDescriptor& x = rx[j];
      const std::uint32_t k = r.below(12);
      if (k < 3) {  // a recycled buffer
        const RxDescriptor& y = rx[r.below(static_cast<std::uint32_t>(j))];
        x.buffer_address = y.buffer_address;
        if (r.below(2)) x.buffer_length = y.buffer_length;
      } else if (k < 5) {  // straddling the previous buffer
        x.buffer_address = rx[j - 1].buffer_address + r.below(std::max<std::uint32_t>(1, rx[j - 1].buffer_length));
      } else if (k < 7 && ntx) {  // inside a TX buffer (read by a later TX descriptor, or an earlier one)
        x.buffer_address = addr[r.below(static_cast<std::uint32_t>(ntx))] + r.below(16);
      }
    }
  }
  const std::size_t mem_size = at + 32;
  for (std::size_t i = 0; i < ntx; ++i)
    if (r.below(40) == 0) tx[i].buffer_address = r.below(2) ? mem_size + 1 + i : mem_size - tx[i].length / 2;
  for (std::size_t j = 0; j < nrx; ++j)
    if (r.below(50) == 0) rx[j].buffer_address = mem_size + 1 + j;
  std::vector<std::uint8_t> image(mem_size, 0);
  for (std::size_t i = 0; i < ntx; ++i) std::memcpy(image.data() + addr[i], pkts[i].data(), pkts[i].size());
  const bool tx_irq = r.below(2), rx_irq = r.below(4) != 0;
  const std::uint16_t qid = static_cast<std::uint16_t>(r.below(8));

  // RSS: the 40-B Microsoft key or the reference's 20-B default, 128 entries
  static const std::vector<std::uint8_t> ms_key = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67,
                                                   0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb,
                                                   0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30,
                                                   0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
  std::vector<std::uint16_t> rss_table(r.below(2) ? 128 : 1 + r.below(200));
  for (auto& q : rss_table) q = static_cast<std::uint16_t>(r.below(16));
  const RssConfig rss_cfg{r.below(2) ? ms_key : std::vector<std::uint8_t>{}, rss_table};

  // the memory's own DMA faults in a third of the cases (tests/cpp/fault_model.h:
  // SimpleHostMemory's FaultInjector or an IOMMU translator), which the stage
  // models with host_memory_faults' verdicts (checked_reads, DmaWriteCheck)
  faultfx::Model fm;
  fm.kind = r.below(3) == 0 ? static_cast<faultfx::Kind>(1 + r.below(2)) : faultfx::kNone;
  if (fm.kind != faultfx::kNone) g_faulty += 1;

  // ---- reference
  const HostMemoryConfig hmc{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = fm.kind == faultfx::kIommu};
  RecordingMemory mem = fm.kind ? RecordingMemory{hmc, fm.translator(), fm.injector()} : RecordingMemory{hmc};
  assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(image))).ok());
  mem.recording = true;
  *fm.armed = true;
  DMAEngine dma{mem};
  std::size_t ref_irq = 0;
  MsixTable table(8);
  InterruptDispatcher disp{table, MsixMapping(8, 0), CoalesceConfig{1, 0},
                           [&](std::uint16_t, std::uint32_t n) { ref_irq += n; }};
  QueuePairConfig qc{
      .queue_id = qid,
      .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = ntx + 1, .base_address = 0, .queue_id = qid, .host_backed = false},
      .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = 0, .queue_id = qid, .host_backed = false},
      .tx_completion = {.ring_size = ntx + 1, .queue_id = qid},
      .rx_completion = {.ring_size = 70 * ntx + 1, .queue_id = qid},
      .interrupt_dispatcher = &disp,
      .max_mtu = max_mtu,
      .enable_tx_interrupts = tx_irq,
      .enable_rx_interrupts = rx_irq,
  };
  QueuePair qp{qc, dma};
  for (auto& t : tx) {
    std::vector<std::byte> b(sizeof(TxDescriptor));
    std::memcpy(b.data(), &t, sizeof(t));
    assert(qp.tx_ring().push_descriptor(b).ok());
  }
  for (auto& x : rx) {
    std::vector<std::byte> b(sizeof(RxDescriptor));
    std::memcpy(b.data(), &x, sizeof(x));
    assert(qp.rx_ring().push_descriptor(b).ok());
  }
  while (qp.process_once()) {
  }
  std::vector<CompletionEntry> ref_tx, ref_rx;
  while (auto c = qp.tx_completion().poll_completion()) ref_tx.push_back(*c);
  while (auto c = qp.rx_completion().poll_completion()) ref_rx.push_back(*c);
  *fm.armed = false;
  std::vector<std::byte> ref_after(mem_size);
  assert(mem.read(0, ref_after).ok());

  // ---- batched stage: run_batch over the CPU backend
  using namespace rx_stage_detail;
  BatchedQueuePairConfig cfg;
  cfg.queue_id = qid;
  cfg.max_mtu = max_mtu;
  cfg.enable_tx_interrupts = tx_irq;
  cfg.enable_rx_interrupts = rx_irq;
  std::size_t our_irq = 0;
  std::vector<CompletionEntry> fired;  // what resolve's own firing delivered, in order
  cfg.on_interrupt = [&](std::uint16_t q, const CompletionEntry& e) {
    assert(q == qid);
    ++our_irq;
    fired.push_back(e);
  };
  RssEngine engine{rss_cfg};
  cfg.rss = &engine;
  std::vector<std::uint8_t> ours = image;
  test::CpuBackend dev{ours, &engine, TupleSpec{}};
  RxBatchResult out;
  QueuePairStats st{};
  BatchScratch scratch;
  if (fm.kind != faultfx::kNone) {
    // the verdicts of a memory with the same faults (its bytes do not matter)
    SimpleHostMemory verdicts{hmc, fm.translator(), fm.injector()};
    *fm.armed = true;
    struct Writes final : DmaWriteCheck {
      HostMemory* m;
      bool write_ok(std::uint64_t a, std::uint64_t n) const override {
        HostMemoryView v{};
        return m->translate(a, n, v).ok();
      }
    } wv;
    wv.m = &verdicts;
    std::vector<TxDescriptor> ctx;
    checked_reads(verdicts, tx, ctx);
    run_batch(cfg, mem_size, ctx, rx, st, out, scratch, dev, -1, &wv);
    *fm.armed = false;
  } else {
    run_batch(cfg, mem_size, tx, rx, st, out, scratch, dev);
  }
  if (buffers_disjoint(mem_size, tx, rx) != disjoint_brute(mem_size, tx, rx)) {
    std::fprintf(stderr, "seed %llu: buffers_disjoint differs from the pairwise check\n", (unsigned long long) seed);
    return 1;
  }
  if (!buffers_disjoint(mem_size, tx, rx)) g_overlapping += 1;
  if (dev.sum_calls > 1) g_split += 1;
  if (dev.snapshots) g_snap += 1;

  // the speculative parallel resolve (no interrupt callback, forced onto 4
  // threads even for these small batches) must equal the sequential one
  {
    const Plan plan = make_plan(cfg, mem_size, tx);
    std::vector<std::uint16_t> cs(plan.pieces.size());
    for (std::size_t i = 0; i < cs.size(); ++i) {
      assert(plan.pieces[i].len <= 65535u);
      cs[i] = oracle_compute_checksum(image.data() + plan.pieces[i].addr, plan.pieces[i].len);
    }
    RxBatchResult sout;
    QueuePairStats sst{};
    std::vector<SegmentWrite> writes;
    std::vector<std::int64_t> wof;
    BatchedQueuePairConfig scfg = cfg;
    scfg.on_interrupt = nullptr;
    resolve(scfg, mem_size, plan, cs, tx, rx, sst, sout, writes, wof, 1);
    const RxBatchResult& out = sout;
    const QueuePairStats& st = sst;
    BatchedQueuePairConfig pcfg = cfg;
    pcfg.on_interrupt = nullptr;
    RxBatchResult pout;
    QueuePairStats pst{};
    std::vector<SegmentWrite> pw;
    std::vector<std::int64_t> pwof;
    resolve(pcfg, mem_size, plan, cs, tx, rx, pst, pout, pw, pwof, 4);
    bool pok = pout.tx_completions.size() == out.tx_completions.size() &&
               pout.rx_completions.size() == out.rx_completions.size() && pw.size() == writes.size() &&
               pwof == wof && same(pst, st) && pout.rx_consumed == out.rx_consumed;
    for (std::size_t i = 0; pok && i < out.tx_completions.size(); ++i) pok = same(pout.tx_completions[i], out.tx_completions[i]);
    for (std::size_t i = 0; pok && i < out.rx_completions.size(); ++i) pok = same(pout.rx_completions[i], out.rx_completions[i]);
    for (std::size_t i = 0; pok && i < writes.size(); ++i)
      pok = std::memcmp(&pw[i], &writes[i], sizeof(SegmentWrite)) == 0;
    if (!pok) {
      std::fprintf(stderr, "seed %llu: parallel resolve differs from the sequential one\n", (unsigned long long) seed);
      return 1;
    }
    // the device resolve's algorithm (ring positions by relaxation, then the
    // settled prefix in parallel order): with steps enough it settles every
    // packet, with 2 steps a prefix, and either equals the sequential result
    for (const int max_steps : {2, 1 << 20}) {
      RxBatchResult rout;
      QueuePairStats rst{};
      std::vector<SegmentWrite> rw;
      std::vector<std::int64_t> rwof;
      std::size_t used = 0;
      int steps = 0;
      const std::size_t lim = resolve_relaxed(pcfg, mem_size, plan, cs, tx, rx, rst, rout, rw, rwof, max_steps, used, steps);
      bool rok = lim <= out.tx_completions.size() && used <= out.rx_completions.size() &&
                 rout.rx_completions.size() == used && (max_steps == 2 || lim == tx.size());
      for (std::size_t i = 0; rok && i < lim; ++i) rok = same(rout.tx_completions[i], out.tx_completions[i]);
      for (std::size_t i = 0; rok && i < used; ++i)
        rok = same(rout.rx_completions[i], out.rx_completions[i]) && rwof[i] == wof[i] &&
              std::memcmp(&rw[i], &writes[i], sizeof(SegmentWrite)) == 0;
      if (rok && lim == tx.size()) rok = same(rst, st) && used == out.rx_consumed;
      if (!rok) {
        std::fprintf(stderr, "seed %llu: relaxed resolve (%d steps max, %d taken, %zu settled) differs\n",
                     (unsigned long long) seed, max_steps, steps, lim);
        return 1;
      }
      if (max_steps > 2) g_steps_max = std::max(g_steps_max, steps);
    }
    // the device's split plans (one piece per plain packet, its sum taken as
    // its first 4 bytes | the rest, nicgpu_checksum_batch_split) resolve to
    // the same result
    {
      const Plan sp = make_plan(cfg, mem_size, tx, /*split4=*/true);
      const std::size_t m = sp.pieces.size();
      std::vector<std::uint16_t> scs(2 * m);
      for (std::size_t i = 0; i < m; ++i) {
        const Piece& pc = sp.pieces[i];
        const std::uint32_t h = pc.len < 4u ? pc.len : 4u;
        scs[i] = oracle_compute_checksum(image.data() + pc.addr + h, pc.len - h);
        scs[m + i] = oracle_compute_checksum(image.data() + pc.addr, h);
      }
      RxBatchResult xout;
      QueuePairStats xst{};
      std::vector<SegmentWrite> xw;
      std::vector<std::int64_t> xwof;
      resolve(scfg, mem_size, sp, scs, tx, rx, xst, xout, xw, xwof, 1);
      bool xok = m <= plan.pieces.size() && xout.tx_completions.size() == out.tx_completions.size() &&
                 xout.rx_completions.size() == out.rx_completions.size() && xwof == wof && same(xst, st);
      for (std::size_t i = 0; xok && i < out.tx_completions.size(); ++i) xok = same(xout.tx_completions[i], out.tx_completions[i]);
      for (std::size_t i = 0; xok && i < out.rx_completions.size(); ++i) xok = same(xout.rx_completions[i], out.rx_completions[i]);
      for (std::size_t i = 0; xok && i < writes.size(); ++i) xok = std::memcmp(&xw[i], &writes[i], sizeof(SegmentWrite)) == 0;
      if (!xok) {
        std::fprintf(stderr, "seed %llu: resolve over split piece sums differs\n", (unsigned long long) seed);
        return 1;
      }
      g_split_pieces_saved += plan.pieces.size() - m;
    }
  }

  // RSS of each frame delivered with Success, from the bytes the reference
  // wrote for it: recorded writes pair with RX completions that carry a write
  // (Success and ChecksumError: handle_rx_segment writes, then verifies)
  bool rss_ok = true;
  {
    std::size_t k = 0, delivered = 0;
    RssEngine expect{rss_cfg};
    for (std::size_t j = 0; j < ref_rx.size() && rss_ok; ++j) {
      const auto status = static_cast<CompletionCode>(ref_rx[j].status);
      if (status != CompletionCode::Success && status != CompletionCode::ChecksumError) continue;
      if (k >= mem.writes.size()) {
        rss_ok = false;
        break;
      }
      const std::vector<std::uint8_t>& bytes = mem.writes[k++];
      if (status != CompletionCode::Success) continue;
      ++delivered;
      std::uint8_t t[64];
      const std::size_t tl = oracle_extract_tuple(bytes.data(), bytes.size(), ORACLE_TUPLE_AUTO, 0, 0, t);
      const std::span<const std::uint8_t> tuple(t, tl);
      const std::uint32_t h = RssEngine{rss_cfg}.hash(tuple);
      const std::uint16_t q = *expect.select_queue(tuple);
      rss_ok = j < out.rx_hash.size() && out.rx_hash[j] == h && out.rx_queue[j] == q;
    }
    rss_ok = rss_ok && k == mem.writes.size();
    rss_ok = rss_ok && engine.stats().hashes == expect.stats().hashes && engine.stats().queue_hits == expect.stats().queue_hits;
    std::size_t listed = 0;
    for (std::size_t q = 0; q < out.queues.size() && rss_ok; ++q) {
      listed += out.queues[q].size();
      for (std::size_t i = 0; i < out.queues[q].size() && rss_ok; ++i)
        rss_ok = out.rx_queue[out.queues[q][i]] == q && (i == 0 || out.queues[q][i - 1] < out.queues[q][i]);
    }
    rss_ok = rss_ok && listed == delivered;
  }

  // the replay from the completions (what the device path and the pipelined
  // stage fire) delivers the same callbacks in the same order
  bool irq_ok = true;
  {
    std::vector<CompletionEntry> replayed;
    BatchedQueuePairConfig rcfg = cfg;
    rcfg.on_interrupt = [&](std::uint16_t q, const CompletionEntry& e) {
      irq_ok = irq_ok && q == qid;
      replayed.push_back(e);
    };
    replay_interrupts(rcfg, out.tx_completions, out.rx_completions);
    irq_ok = irq_ok && replayed.size() == fired.size();
    for (std::size_t i = 0; irq_ok && i < fired.size(); ++i) irq_ok = same(replayed[i], fired[i]);
    if (!irq_ok) std::fprintf(stderr, "seed %llu: replayed interrupts differ (%zu / %zu)\n", (unsigned long long) seed,
                              replayed.size(), fired.size());
  }
  bool ok = irq_ok && rss_ok && out.tx_completions.size() == ref_tx.size() && out.rx_completions.size() == ref_rx.size();
  for (std::size_t i = 0; ok && i < ref_tx.size(); ++i) ok = same(out.tx_completions[i], ref_tx[i]);
  for (std::size_t i = 0; ok && i < ref_rx.size(); ++i) ok = same(out.rx_completions[i], ref_rx[i]);
  ok = ok && same(st, qp.stats());
  ok = ok && out.rx_consumed == nrx - qp.rx_ring().available();
  ok = ok && our_irq == ref_irq;
  ok = ok && std::memcmp(ours.data(), ref_after.data(), mem_size) == 0;
  if (!ok) {
    std::fprintf(stderr, "seed %llu: mismatch (alias %d rss %d tx %zu/%zu rx %zu/%zu irq %zu/%zu)\n",
                 (unsigned long long) seed, int(alias), int(rss_ok), out.tx_completions.size(), ref_tx.size(),
                 out.rx_completions.size(), ref_rx.size(), our_irq, ref_irq);
    return 1;
  }
  return 0;
}


// Host-backed rings that the batch's own DMA writes land on (the reference
// pops each slot by a DMA read, descriptor_ring.cpp:97-106): RX buffers that
// are exactly a later TX or RX ring slot, frames whose first 32 bytes read as
// sane descriptors (bools 0/1, no checksum, no TSO, no VLAN, small lengths,
// buffers below the rings).  The reference QueuePair with host-backed rings
// against run_batch with RingSlots.
std::size_t g_ring_rereads = 0, g_ring_batches = 0;

int run_ring_case(std::uint64_t seed) {
  Rng r{seed * 104729 + 7};
  const std::size_t ntx = 1 + r.below(90), nrx = 1 + r.below(160);
  const std::size_t rx_len = 1600;
  std::vector<std::size_t> lens(ntx);
  std::vector<std::uint64_t> addr(ntx);
  std::size_t at = 0;
  for (std::size_t i = 0; i < ntx; ++i) {
    const std::uint32_t pick = r.below(3);
    lens[i] = pick == 0 ? 8 + r.below(25) : (pick == 1 ? 33 + r.below(300) : 400 + r.below(1100));
    addr[i] = at;
    at += lens[i] + r.below(4);
  }
  at = (at + 15) & ~std::size_t{15};
  const std::size_t rx_base = at;
  const std::size_t tx_at = rx_base + nrx * rx_len, rx_at = tx_at + ntx * sizeof(TxDescriptor);
  const std::size_t mem_size = rx_at + nrx * sizeof(RxDescriptor) + 64;
  std::vector<std::uint8_t> image(mem_size, 0);
  for (std::size_t a = 0; a < rx_base; ++a) image[a] = r.byte();
  std::vector<TxDescriptor> tx(ntx);
  for (std::size_t i = 0; i < ntx; ++i) {
    std::uint8_t* f = image.data() + addr[i];
    std::uint8_t h[32] = {};
    const std::uint64_t ba = r.below(static_cast<std::uint32_t>(std::max<std::size_t>(tx_at, 2048) - 1600));
    std::memcpy(h, &ba, 8);
    const std::uint32_t bl = r.below(1601);
    std::memcpy(h + 8, &bl, 4);
    h[14] = r.byte();
    h[15] = r.byte();
    h[16] = static_cast<std::uint8_t>(r.below(2));
    h[18] = static_cast<std::uint8_t>(r.below(2));
    h[22] = static_cast<std::uint8_t>(r.below(2));
    h[23] = r.byte();
    h[24] = r.byte();
    h[28] = r.byte();
    std::memcpy(f, h, std::min<std::size_t>(32, lens[i]));
    TxDescriptor& t = tx[i];
    t.buffer_address = addr[i];
    t.length = static_cast<std::uint32_t>(lens[i]);
    t.descriptor_index = static_cast<std::uint16_t>(i);
    t.checksum = r.below(4) == 0 ? ChecksumMode::Layer4 : ChecksumMode::None;
    t.checksum_offload = r.below(2);
    const std::uint16_t good = oracle_compute_checksum(f, lens[i]);
    t.checksum_value = r.below(4) == 0 ? static_cast<std::uint16_t>(good ^ 1u) : good;
    if (lens[i] > 300 && r.below(3) == 0) {
      (r.below(2) ? t.tso_enabled : t.gso_enabled) = true;
      t.mss = static_cast<std::uint16_t>(60 + r.below(300));
      t.header_length = static_cast<std::uint16_t>(32 + r.below(30));
    }
  }
  std::vector<RxDescriptor> rx(nrx);
  for (std::size_t j = 0; j < nrx; ++j) {
    RxDescriptor& x = rx[j];
    x.buffer_address = rx_base + j * rx_len;
    x.buffer_length = static_cast<std::uint32_t>(rx_len);
    x.descriptor_index = static_cast<std::uint16_t>(1000 + j);
    x.checksum_offload = r.below(2);
    x.checksum = r.below(3) == 0 ? ChecksumMode::None : ChecksumMode::Layer4;
    x.vlan_present = r.below(4) == 0;
    x.gro_enabled = r.below(4) == 0;
    const std::uint32_t k = r.below(5);
    if (k == 0 && j + 66 < nrx) {  // a later RX slot, past any one packet's pops
      x.buffer_address = rx_at + (j + 65 + r.below(static_cast<std::uint32_t>(nrx - j - 65))) * sizeof(RxDescriptor);
      x.buffer_length = sizeof(RxDescriptor);
    } else if (k == 1 && j + 2 < ntx) {  // a later TX slot
      x.buffer_address = tx_at + (j + 1 + r.below(static_cast<std::uint32_t>(ntx - j - 1))) * sizeof(TxDescriptor);
      x.buffer_length = sizeof(TxDescriptor);
    }
  }
  const std::uint16_t qid = static_cast<std::uint16_t>(r.below(8));
  // ---- reference, host-backed rings
  RecordingMemory mem{HostMemoryConfig{.size_bytes = mem_size, .page_size = 4096, .iommu_enabled = false}};
  assert(mem.write(0, std::as_bytes(std::span<const std::uint8_t>(image))).ok());
  DMAEngine dma{mem};
  QueuePairConfig qc{
      .queue_id = qid,
      .tx_ring = {.descriptor_size = sizeof(TxDescriptor), .ring_size = ntx + 1, .base_address = tx_at, .queue_id = qid, .host_backed = true},
      .rx_ring = {.descriptor_size = sizeof(RxDescriptor), .ring_size = nrx + 1, .base_address = rx_at, .queue_id = qid, .host_backed = true},
      .tx_completion = {.ring_size = ntx + 1, .queue_id = qid},
      .rx_completion = {.ring_size = 70 * ntx + 1, .queue_id = qid},
  };
  QueuePair qp{qc, dma};
  for (auto& t : tx) {
    std::vector<std::byte> b(sizeof(TxDescriptor));
    std::memcpy(b.data(), &t, sizeof(t));
    assert(qp.tx_ring().push_descriptor(b).ok());
  }
  for (auto& x : rx) {
    std::vector<std::byte> b(sizeof(RxDescriptor));
    std::memcpy(b.data(), &x, sizeof(x));
    assert(qp.rx_ring().push_descriptor(b).ok());
  }
  std::vector<std::byte> pushed(mem_size);
  assert(mem.read(0, pushed).ok());
  std::vector<std::uint8_t> ours(mem_size);
  std::memcpy(ours.data(), pushed.data(), mem_size);
  while (qp.process_once()) {
  }
  std::vector<CompletionEntry> ref_tx, ref_rx;
  while (auto c = qp.tx_completion().poll_completion()) ref_tx.push_back(*c);
  while (auto c = qp.rx_completion().poll_completion()) ref_rx.push_back(*c);
  std::vector<std::byte> ref_after(mem_size);
  assert(mem.read(0, ref_after).ok());
  // ---- the driver with the rings' offsets
  using namespace rx_stage_detail;
  BatchedQueuePairConfig cfg;
  cfg.queue_id = qid;
  test::CpuBackend dev{ours, nullptr, TupleSpec{}};
  RxBatchResult out;
  QueuePairStats st{};
  BatchScratch scratch;
  const RingSlots slots{tx_at, rx_at};
  run_batch(cfg, mem_size, tx, rx, st, out, scratch, dev, -1, nullptr, &slots);
  g_ring_batches += 1;
  g_ring_rereads += dev.refetches;
  bool ok = out.tx_completions.size() == ref_tx.size() && out.rx_completions.size() == ref_rx.size();
  for (std::size_t i = 0; ok && i < ref_tx.size(); ++i) ok = same(out.tx_completions[i], ref_tx[i]);
  for (std::size_t i = 0; ok && i < ref_rx.size(); ++i) ok = same(out.rx_completions[i], ref_rx[i]);
  ok = ok && same(st, qp.stats());
  ok = ok && std::memcmp(ours.data(), ref_after.data(), mem_size) == 0;
  if (!ok) {
    std::fprintf(stderr, "ring seed %llu: mismatch (tx %zu/%zu rx %zu/%zu)\n", (unsigned long long) seed,
                 out.tx_completions.size(), ref_tx.size(), out.rx_completions.size(), ref_rx.size());
    return 1;
  }
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  const std::uint64_t first = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
  const std::uint64_t count = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 200;
  int bad = check_disjoint_large();
  for (std::uint64_t s = first; s < first + count; ++s) bad += run_case(s);
  for (std::uint64_t s = first; s < first + count / 4; ++s) bad += run_ring_case(s);
  if (bad) return 1;
  std::printf("rx_stage_fuzz: ok (%llu batches; %zu with overlapping buffers, %zu split into sub-batches, %zu gathered "
              "from a copy; %zu on a memory with its own DMA faults; relaxation settled every batch in <= %d steps; split "
              "plans equal, %zu pieces fewer; %zu batches on host-backed rings their own writes land on, %zu re-reads)\n",
              (unsigned long long) count, g_overlapping, g_split, g_snap, g_faulty, g_steps_max, g_split_pieces_saved,
              g_ring_batches, g_ring_rereads);
  return 0;
}
