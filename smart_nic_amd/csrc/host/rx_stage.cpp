// rx_stage.cpp — nic::BatchedQueuePair: the reference's
// QueuePair::process_once (src/queue_pair.cpp:67-460) over a batch.
//
// 1. make_plan: per TX descriptor, the byte pieces whose ones'-complement sums
//    the TX verify (:105-116) and the RX verifies (:434-447) will need.
// 2. GPU: nicgpu_checksum_batch over all pieces (one pass over the TX bytes).
// 3. resolve: the reference's control flow, in order, from those sums.
//    Piece sums compose exactly: fold(a + b) is 0 only when a and b are, and
//    a piece placed at an odd offset contributes its byte-swapped sum.
// 4. GPU: nicgpu_segment_gather writes the delivered segments (the DMA writes
//    of :416-426) into the RX buffers.
// 5. GPU: RssEngine::select_queue_batch over the frames delivered with
//    Success -> per-queue dispatch lists.
// When buffers overlap (buffers_disjoint() false) run_batch goes through the
// batch in sub-batches (resolve_prefix) and applies each sub-batch's writes in
// layers (schedule_writes), so the in-order results of the reference hold.
#include "nic/rx_stage.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <limits>
#include <map>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>

#include <pthread.h>
#include <sched.h>

#include "nic/checksum.h"
#include "nicgpu.h"
#include "../qp_logic.h"

namespace nic {
namespace rx_stage_detail {
namespace {

using nicqp::dma_ok;

// The shared per-packet logic (qp_logic.h) over this library's types.
using Ctx = nicqp::Ctx<TxDescriptor, RxDescriptor, PacketPlan>;

// Worker placement: chunk c of a pass runs on the c-th allowed CPU after the
// calling thread's, so a batch's chunks stay on the same few neighbouring
// cores from pass to pass and batch to batch (their lines then stay in those
// cores' caches).  Empty when the affinity mask cannot be read.
std::vector<int> near_cpus(std::size_t k) {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return out;
  const int self = sched_getcpu();
  if (self < 0) return out;
  std::vector<int> allowed;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) allowed.push_back(c);
  const auto it = std::find(allowed.begin(), allowed.end(), self);
  const std::size_t at = it == allowed.end() ? 0 : static_cast<std::size_t>(it - allowed.begin());
  for (std::size_t i = 0; i < k && !allowed.empty(); ++i) out.push_back(allowed[(at + i) % allowed.size()]);
  return out;
}

void pin_to(const std::vector<int>& cpus, std::size_t c) {
  if (c >= cpus.size()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpus[c], &set);
  (void) pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

// Fixed partition of [0, n) into at most 16 contiguous chunks, run on
// std::threads when n is large enough to pay for them; f(chunk, begin, end).
// Both passes of a count/fill pair see the same partition.
struct Chunks {
  std::size_t n, k;
  explicit Chunks(std::size_t n_, std::size_t max_threads = 16, std::size_t grain = 32768) : n(n_) {
    const std::size_t hw = std::max(1u, std::thread::hardware_concurrency());
    k = std::max<std::size_t>(1, std::min<std::size_t>({hw, max_threads, n / grain}));
  }
  std::size_t begin(std::size_t c) const { return n * c / k; }
  template <class F>
  void run(F&& f) const {
    if (k == 1) {
      f(std::size_t{0}, std::size_t{0}, n);
      return;
    }
    std::vector<std::thread> th;
    th.reserve(k - 1);
    const std::vector<int> cpus = near_cpus(k);
    for (std::size_t c = 1; c < k; ++c)
      th.emplace_back([&, c] {
        pin_to(cpus, c);
        f(c, begin(c), begin(c + 1));
      });
    f(std::size_t{0}, std::size_t{0}, begin(1));
    for (auto& t : th) t.join();
  }
};

}  // namespace

namespace {

// One TX descriptor's plan (nicqp::plan_packet); writes its pieces to `out`
// unless it is null.  Returns the number of pieces.
std::uint32_t plan_packet(const BatchedQueuePairConfig& config, std::size_t mem_size, const TxDescriptor& t,
                          PacketPlan& pp, Piece* out, bool split4) {
  std::uint32_t k = 0;
  return nicqp::plan_packet(
      config.max_mtu, mem_size, t, pp,
      [&](std::uint64_t addr, std::uint64_t len) {
        if (out) out[k] = Piece{addr, static_cast<std::uint32_t>(len)};
        ++k;
      },
      split4);
}

}  // namespace

void replay_interrupts(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> txc,
                       std::span<const CompletionEntry> rxc) {
  if (!config.on_interrupt || (!config.enable_tx_interrupts && !config.enable_rx_interrupts)) return;
  InterruptCursor at;
  replay_interrupts(config, txc, rxc, at, txc.size());
}

namespace {
// The replay loop; ready_tx(i) / ready_rx(j) are called before TX completion i
// / RX completion j is first read (completions still landing in chunks).
template <class ReadyTx, class ReadyRx>
void replay_core(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> txc,
                 std::span<const CompletionEntry> rxc, InterruptCursor& at, std::size_t n, ReadyTx&& ready_tx,
                 ReadyRx&& ready_rx) {
  constexpr auto kOk = static_cast<std::uint32_t>(CompletionCode::Success);
  constexpr auto kFault = static_cast<std::uint32_t>(CompletionCode::Fault);
  const bool any = config.on_interrupt && (config.enable_tx_interrupts || config.enable_rx_interrupts);
  // a local copy of the callback and the flags: calls through `config` reload
  // the callable every time (the callback could reach `config`), ~25% of a
  // million-callback replay
  const std::function<void(std::uint16_t, const CompletionEntry&)> cb =
      any ? config.on_interrupt : std::function<void(std::uint16_t, const CompletionEntry&)>{};
  const bool rx_on = any && config.enable_rx_interrupts, tx_on = any && config.enable_tx_interrupts;
  const std::uint16_t q = config.queue_id;
  std::size_t j = at.rx;
  const std::size_t end = std::min(txc.size(), at.tx + n);
  const CompletionEntry* R = rxc.data();
  const std::size_t nr = rxc.size();
  for (std::size_t i = at.tx; i < end; ++i) {
    ready_tx(i);
    const CompletionEntry& t = txc[i];
    // the packets that popped RX descriptors: Success (all delivered, or an
    // RX-side abort), and a DMA write fault after some segment (segments_produced > 0)
    const bool popped = t.status == kOk || (t.status == kFault && t.segments_produced > 0);
    bool fires = !popped;
    if (popped) {
      fires = t.status == kOk;  // a faulted packet's TX completion fires none
      for (std::uint32_t k = 0; k < t.segments_produced && j < nr; ++k) {
        ready_rx(j);
        const CompletionEntry& e = R[j++];
        if (rx_on) cb(q, e);
        if (e.status != kOk) {  // the packet ends here and its TX completion fires none
          fires = false;
          break;
        }
      }
    }
    if (fires && tx_on) cb(q, t);
  }
  at.tx = end;
  at.rx = j;
}
}  // namespace

void replay_interrupts(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> txc,
                       std::span<const CompletionEntry> rxc, InterruptCursor& at, std::size_t n) {
  replay_core(config, txc, rxc, at, n, [](std::size_t) {}, [](std::size_t) {});
}

void replay_interrupts_chunked(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> txc,
                               std::span<const CompletionEntry> rxc, std::size_t chunk_tx, std::size_t chunk_rx,
                               const std::function<void(int, std::size_t)>& wait_chunk) {
  if (!config.on_interrupt || (!config.enable_tx_interrupts && !config.enable_rx_interrupts)) return;
  InterruptCursor at;
  std::size_t next_tx = 0, next_rx = 0;  // first index not yet known to have landed
  replay_core(
      config, txc, rxc, at, txc.size(),
      [&](std::size_t i) {
        if (i >= next_tx) {
          wait_chunk(0, i / chunk_tx);
          next_tx = (i / chunk_tx + 1) * chunk_tx;
        }
      },
      [&](std::size_t j) {
        if (j >= next_rx) {
          wait_chunk(1, j / chunk_rx);
          next_rx = (j / chunk_rx + 1) * chunk_rx;
        }
      });
}

// Count pass, prefix over the chunks, fill pass (each chunk in its own thread).
Plan make_plan(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               bool split4) {
  Plan plan;
  make_plan(config, mem_size, tx, plan, split4);
  return plan;
}

void make_plan(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               Plan& plan, bool split4) {
  plan.split4 = split4;
  plan.packets.resize(tx.size());
  const Chunks ch(tx.size(), config.host_threads ? config.host_threads : 16);
  std::vector<std::size_t> base(ch.k + 1, 0);
  ch.run([&](std::size_t c, std::size_t b, std::size_t e) {
    std::size_t n = 0;
    for (std::size_t i = b; i < e; ++i) n += plan_packet(config, mem_size, tx[i], plan.packets[i], nullptr, split4);
    base[c + 1] = n;
  });
  for (std::size_t c = 0; c < ch.k; ++c) base[c + 1] += base[c];
  // PacketPlan::first_piece is 32-bit (the device plan's layout)
  if (base[ch.k] > 0xFFFFFFFFull)
    throw GpuError("process_batch: more than 2^32 checksum pieces in one batch; split it", NICGPU_ERR_RANGE);
  plan.pieces.resize(base[ch.k]);
  ch.run([&](std::size_t c, std::size_t b, std::size_t e) {
    std::size_t at = base[c];
    for (std::size_t i = b; i < e; ++i) {
      PacketPlan& pp = plan.packets[i];
      const std::uint32_t np = plan_packet(config, mem_size, tx[i], pp, plan.pieces.data() + at, split4);
      pp.first_piece = static_cast<std::uint32_t>(at);
      at += np;
    }
  });
}

namespace {

void add_stats(QueuePairStats& a, const QueuePairStats& b) {
  a.tx_packets += b.tx_packets;
  a.rx_packets += b.rx_packets;
  a.tx_bytes += b.tx_bytes;
  a.rx_bytes += b.rx_bytes;
  a.drops_checksum += b.drops_checksum;
  a.drops_no_rx_desc += b.drops_no_rx_desc;
  a.drops_buffer_small += b.drops_buffer_small;
  a.drops_mtu_exceeded += b.drops_mtu_exceeded;
  a.drops_invalid_mss += b.drops_invalid_mss;
  a.drops_too_many_segments += b.drops_too_many_segments;
  a.tx_tso_segments += b.tx_tso_segments;
  a.tx_gso_segments += b.tx_gso_segments;
  a.tx_vlan_insertions += b.tx_vlan_insertions;
  a.rx_vlan_strips += b.rx_vlan_strips;
  a.rx_checksum_verified += b.rx_checksum_verified;
  a.rx_gro_aggregated += b.rx_gro_aggregated;
}

bool write_check_thunk(const void* w, std::uint64_t a, std::uint64_t n) {
  return static_cast<const DmaWriteCheck*>(w)->write_ok(a, n);
}

Ctx make_ctx(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
             std::span<const std::uint16_t> cs, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
             const DmaWriteCheck* wcheck = nullptr) {
  const std::size_t np = plan.pieces.size();
  if (cs.size() < (plan.split4 ? 2 * np : np)) throw std::invalid_argument("resolve: fewer piece sums than the plan's pieces");
  Ctx C{config.queue_id, config.max_mtu, mem_size,  plan.packets.data(), cs.data(),
        plan.split4 ? cs.data() + np : nullptr,   tx.data(), rx.data(), rx.size()};
  if (wcheck) {
    C.wcheck = wcheck;
    C.wcheck_fn = &write_check_thunk;
  }
  return C;
}

std::size_t rx_need(const Ctx& C, std::size_t i) { return nicqp::rx_need(C, i); }

template <class Sink>
std::size_t resolve_packet(const Ctx& C, std::size_t i, std::size_t rc, QueuePairStats& stats, Sink& sink) {
  return nicqp::resolve_packet<CompletionEntry, SegmentWrite>(C, i, rc, stats, sink);
}

// Appends, firing interrupts in posting order (:371-383).
struct AppendSink {
  const BatchedQueuePairConfig& config;
  RxBatchResult& out;
  std::vector<SegmentWrite>& writes;
  std::vector<std::int64_t>& write_of_rx;
  void tx(const CompletionEntry& e, bool fire) {
    out.tx_completions.push_back(e);
    if (fire && config.enable_tx_interrupts && config.on_interrupt) config.on_interrupt(config.queue_id, e);
  }
  void rx(const CompletionEntry& e, const SegmentWrite* w) {
    const std::int64_t j = static_cast<std::int64_t>(out.rx_completions.size());
    out.rx_completions.push_back(e);
    writes.push_back(w ? *w : SegmentWrite{});
    write_of_rx.push_back(w ? j : -1);
    if (config.enable_rx_interrupts && config.on_interrupt) config.on_interrupt(config.queue_id, e);
  }
};

// Writes at known positions (no interrupts: the parallel path runs only
// without an interrupt callback).
struct PlaceSink {
  CompletionEntry* txc;
  CompletionEntry* rxc;
  SegmentWrite* w;
  std::int64_t* wof;
  std::size_t ti = 0, rj = 0;  // next TX slot, next RX slot
  void tx(const CompletionEntry& e, bool) { txc[ti] = e; }
  void rx(const CompletionEntry& e, const SegmentWrite* sw) {
    rxc[rj] = e;
    w[rj] = sw ? *sw : SegmentWrite{};
    wof[rj] = sw ? static_cast<std::int64_t>(rj) : -1;
    ++rj;
  }
};

}  // namespace

void resolve(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
             std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
             std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
             std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx, unsigned max_threads,
             const DmaWriteCheck* wcheck) {
  const Ctx C = make_ctx(config, mem_size, plan, piece_csum, tx, rx, wcheck);
  const std::size_t n = tx.size();
  const std::size_t want = max_threads ? max_threads : (config.host_threads ? config.host_threads : 16);
  // (the memory's write verdicts are asked in posting order, on this thread)
  const Chunks ch(n, (config.on_interrupt || wcheck) ? 1 : want, max_threads ? 1 : 32768);
  std::size_t from = 0, rc = 0;  // first TX descriptor the sequential pass resolves, and its ring position
  std::size_t nmulti = 0;         // packets of more than one segment (only they can abort early)
  static thread_local std::vector<std::uint32_t> need_tl;
  static thread_local std::vector<std::size_t> pos_tl;
  // the calling thread's buffers, by reference: a worker naming need_tl
  // would get its own (empty) instance
  std::vector<std::uint32_t>& need = need_tl;
  std::vector<std::size_t>& pos = pos_tl;
  if (ch.k > 1) {
    // (1) RX descriptors each packet would pop, in parallel; (2) the ring
    // position of every packet by a scan, assuming no packet aborts before
    // its last segment; (3) every chunk resolved in parallel from its exact
    // position into its slots.  A chunk stops at the first packet that pops
    // a different number of descriptors (an RX-side abort before the last
    // segment); the batch is then finished sequentially from that packet.
    // (need, pos: per calling thread, reused, so steady batches take no page faults)
    need.resize(n);
    pos.resize(n + 1);
    std::vector<std::size_t> multi(ch.k, 0);
    ch.run([&](std::size_t c, std::size_t b, std::size_t e) {
      std::size_t m = 0;
      for (std::size_t i = b; i < e; ++i) {
        need[i] = static_cast<std::uint32_t>(rx_need(C, i));
        m += need[i] > 1;
      }
      multi[c] = m;
    });
    for (auto m : multi) nmulti += m;
  }
  // mostly multi-segment batches (TSO) are left to the sequential pass: every
  // early abort there would end the parallel prefix
  if (ch.k > 1 && (max_threads || nmulti * 8 <= n)) {
    std::size_t r = 0;
    for (std::size_t i = 0; i < n; ++i) {
      pos[i] = r;
      if (r != rx.size() && need[i] != 0 && rx.size() - r >= need[i]) r += need[i];
    }
    pos[n] = r;
    out.tx_completions.resize(n);
    out.rx_completions.resize(r);
    writes.resize(r);
    write_of_rx.resize(r);
    std::vector<std::size_t> stop(ch.k, 0);
    std::vector<QueuePairStats> cst(ch.k);
    ch.run([&](std::size_t c, std::size_t b, std::size_t e) {
      PlaceSink sink{out.tx_completions.data(), out.rx_completions.data(), writes.data(), write_of_rx.data()};
      QueuePairStats& S = cst[c];
      std::size_t i = b;
      for (; i < e; ++i) {
        sink.ti = i;
        sink.rj = pos[i];
        QueuePairStats d{};
        if (resolve_packet(C, i, pos[i], d, sink) != pos[i + 1] - pos[i]) break;
        add_stats(S, d);
      }
      stop[c] = i;
    });
    from = n;
    for (std::size_t c = 0; c < ch.k; ++c) {
      add_stats(stats, cst[c]);
      if (stop[c] != ch.begin(c + 1)) {
        from = stop[c];
        break;
      }
    }
    rc = pos[from];
    if (from == n) {
      rc = r;
    } else {
      out.tx_completions.resize(from);
      out.rx_completions.resize(rc);
      writes.resize(rc);
      write_of_rx.resize(rc);
    }
  } else {
    out.tx_completions.clear();
    out.rx_completions.clear();
    writes.clear();
    write_of_rx.clear();
  }
  if (from < n) {
    out.tx_completions.reserve(n);
    const std::size_t cap = std::min(n, rx.size());
    out.rx_completions.reserve(cap);
    writes.reserve(cap);
    write_of_rx.reserve(cap);
    AppendSink sink{config, out, writes, write_of_rx};
    for (std::size_t i = from; i < n; ++i) rc += resolve_packet(C, i, rc, stats, sink);
  }
  out.tx_processed = n;
  out.rx_consumed = rc;
}

namespace {
struct NullSink {
  void tx(const CompletionEntry&, bool) {}
  void rx(const CompletionEntry&, const SegmentWrite*) {}
};
struct PlaceAt {  // writes at known positions (resolve_relaxed)
  CompletionEntry* txc;
  CompletionEntry* rxc;
  SegmentWrite* w;
  std::int64_t* wof;
  std::size_t ti, rj;
  void tx(const CompletionEntry& e, bool) { txc[ti] = e; }
  void rx(const CompletionEntry& e, const SegmentWrite* sw) {
    rxc[rj] = e;
    w[rj] = sw ? *sw : SegmentWrite{};
    wof[rj] = sw ? static_cast<std::int64_t>(rj) : -1;
    ++rj;
  }
};
}  // namespace

std::size_t resolve_relaxed(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
                            std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
                            std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
                            std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx, int max_steps,
                            std::size_t& rx_used, int& steps) {
  const Ctx C = make_ctx(config, mem_size, plan, piece_csum, tx, rx);
  const std::size_t n = tx.size(), m = rx.size();
  std::vector<std::uint32_t> pops(n), pos(n + 1, 0);
  for (std::size_t i = 0; i < n; ++i) pops[i] = static_cast<std::uint32_t>(rx_need(C, i));
  std::size_t lim = n;
  steps = 0;
  for (int it = 0; it < max_steps; ++it) {
    ++steps;
    std::uint32_t r = 0;
    for (std::size_t i = 0; i < n; ++i) {
      pos[i] = r;
      r += pops[i];
    }
    pos[n] = r;
    std::size_t first = n;
    for (std::size_t i = 0; i < n; ++i) {  // one kernel launch: every packet against the same pos
      QueuePairStats d{};
      NullSink sink;
      const std::size_t rc = pos[i] < m ? pos[i] : m;
      const auto popped = static_cast<std::uint32_t>(resolve_packet(C, i, rc, d, sink));
      if (popped != pops[i]) {
        first = std::min(first, i);
        pops[i] = popped;
      }
    }
    lim = first;
    if (first == n) break;
  }
  rx_used = pos[lim];
  out.tx_completions.assign(lim, CompletionEntry{});
  out.rx_completions.assign(rx_used, CompletionEntry{});
  writes.assign(rx_used, SegmentWrite{});
  write_of_rx.assign(rx_used, -1);
  for (std::size_t i = 0; i < lim; ++i) {
    PlaceAt sink{out.tx_completions.data(), out.rx_completions.data(), writes.data(), write_of_rx.data(), i, pos[i]};
    resolve_packet(C, i, pos[i], stats, sink);
  }
  out.tx_processed = lim;
  out.rx_consumed = rx_used;
  return lim;
}

namespace {

struct Span64 {
  std::uint64_t a, b;  // [a, b)
};

// Sorted by start (sorting when needed); true when no two spans share a byte.
bool sort_disjoint(std::vector<Span64>& v, bool sorted) {
  if (!sorted) std::sort(v.begin(), v.end(), [](const Span64& x, const Span64& y) { return x.a < y.a; });
  for (std::size_t i = 1; i < v.size(); ++i)
    if (v[i].a < v[i - 1].b) return false;
  return true;
}

// Merged set of byte ranges.
class IntervalSet {
public:
  bool overlaps(std::uint64_t a, std::uint64_t b) const {
    if (a >= b) return false;
    auto it = m_.upper_bound(a);
    if (it != m_.begin() && std::prev(it)->second > a) return true;
    return it != m_.end() && it->first < b;
  }
  void add(std::uint64_t a, std::uint64_t b) {
    if (a >= b) return;
    auto it = m_.upper_bound(a);
    if (it != m_.begin() && std::prev(it)->second >= a) {
      --it;
      a = it->first;
      b = std::max(b, it->second);
      it = m_.erase(it);
    }
    while (it != m_.end() && it->first <= b) {
      b = std::max(b, it->second);
      it = m_.erase(it);
    }
    m_.emplace(a, b);
  }

private:
  std::map<std::uint64_t, std::uint64_t> m_;  // start -> end
};

inline std::uint64_t write_len(const SegmentWrite& w) {
  return static_cast<std::uint64_t>(w.prefix_len) + w.len_a + w.len_b;
}

}  // namespace

bool buffers_disjoint(std::size_t mem_size, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx) {
  // What an RX descriptor can receive: at most buffer_length bytes inside the
  // image (:397-426); what a TX descriptor is read from: its whole buffer.
  auto rx_span = [&](const RxDescriptor& x, Span64& sp) {
    if (x.buffer_address >= mem_size || x.buffer_length == 0) return false;
    sp = {x.buffer_address, x.buffer_address + std::min<std::uint64_t>(x.buffer_length, mem_size - x.buffer_address)};
    return true;
  };
  auto tx_span = [&](const TxDescriptor& x, Span64& sp) {
    if (x.length == 0 || !dma_ok(mem_size, x.buffer_address, x.length)) return false;
    sp = {x.buffer_address, x.buffer_address + x.length};
    return true;
  };
  // RX descriptors whose spans ascend and are disjoint (checked below) are
  // searched in place: first_after(a) = the first with an end past a, the
  // only one that can overlap a span starting at a (their ends ascend too).
  auto next_valid = [&](std::size_t j) {
    Span64 sp;
    while (j < rx.size() && !rx_span(rx[j], sp)) ++j;
    return j;
  };
  auto first_after = [&](std::uint64_t a) {
    std::size_t lo = 0, hi = rx.size();
    while (lo < hi) {
      const std::size_t mid = lo + (hi - lo) / 2, m = next_valid(mid);
      Span64 sp{};
      if (m == rx.size()) {
        hi = mid;
        continue;
      }
      (void) rx_span(rx[m], sp);
      if (sp.b <= a) lo = m + 1;
      else hi = mid;
    }
    return next_valid(lo);
  };
  // One parallel pass in the ring layout (no copies, no sort): chunk c checks
  // its share of the RX descriptors for ascending disjoint spans, and sweeps
  // its share of the TX spans (ascending within the chunk) against them.
  const Chunks ch(std::max(rx.size(), tx.size()));
  struct Part {
    bool rx_ok = true, tx_asc = true, hit = false, any_rx = false;
    Span64 rx_first{}, rx_last{};
  };
  std::vector<Part> part(ch.k);
  ch.run([&](std::size_t c, std::size_t, std::size_t) {
    Part& P = part[c];
    Span64 sp;
    for (std::size_t j = rx.size() * c / ch.k, e = rx.size() * (c + 1) / ch.k; j < e; ++j) {
      if (!rx_span(rx[j], sp)) continue;
      if (!P.any_rx) P.rx_first = sp;
      else if (sp.a < P.rx_last.b) P.rx_ok = false;
      P.any_rx = true;
      P.rx_last = sp;
    }
    std::size_t j = rx.size() + 1;  // not searched yet
    std::uint64_t last = 0;
    for (std::size_t i = tx.size() * c / ch.k, e = tx.size() * (c + 1) / ch.k; i < e && !P.hit; ++i) {
      if (!tx_span(tx[i], sp)) continue;
      if (j > rx.size()) {
        j = first_after(sp.a);
      } else if (sp.a < last) {
        P.tx_asc = false;
        return;
      }
      last = sp.a;
      Span64 r{};
      while (j < rx.size() && (!rx_span(rx[j], r) || r.b <= sp.a)) ++j;
      if (j < rx.size() && r.a < sp.b) P.hit = true;
    }
  });
  bool rx_ok = true, tx_asc = true, hit = false;
  const Span64* prev = nullptr;
  for (const Part& P : part) {
    rx_ok = rx_ok && P.rx_ok && (!P.any_rx || prev == nullptr || prev->b <= P.rx_first.a);
    if (P.any_rx) prev = &P.rx_last;
    tx_asc = tx_asc && P.tx_asc;
    hit = hit || P.hit;
  }
  if (rx_ok && tx_asc) return !hit;
  // general layouts: sort
  std::vector<Span64> r, t;
  Span64 sp;
  for (const RxDescriptor& x : rx)
    if (rx_span(x, sp)) r.push_back(sp);
  if (!sort_disjoint(r, false)) return false;
  for (const TxDescriptor& x : tx)
    if (tx_span(x, sp)) t.push_back(sp);
  std::sort(t.begin(), t.end(), [](const Span64& x, const Span64& y) { return x.a < y.a; });
  std::size_t j = 0;
  for (const Span64& x : t) {
    while (j < r.size() && r[j].b <= x.a) ++j;
    if (j == r.size()) break;
    if (r[j].a < x.b) return false;
  }
  return true;
}

std::size_t resolve_prefix(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
                           std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
                           std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
                           std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx,
                           const DmaWriteCheck* wcheck, const RingSlots* slots) {
  const Ctx C = make_ctx(config, mem_size, plan, piece_csum, tx, rx, wcheck);
  constexpr std::uint64_t kTxSlot = sizeof(TxDescriptor), kRxSlot = sizeof(RxDescriptor), kNone = ~0ull;
  const bool tx_ring = slots && slots->tx_at != kNone, rx_ring = slots && slots->rx_at != kNone;
  out.tx_completions.clear();
  out.rx_completions.clear();
  writes.clear();
  write_of_rx.clear();
  AppendSink sink{config, out, writes, write_of_rx};
  IntervalSet written;
  std::size_t rc = 0, i = 0;
  for (; i < tx.size(); ++i) {
    const PacketPlan& pp = plan.packets[i];
    bool reads_written = false;
    for (std::uint32_t k = 0; k < pp.npieces && !reads_written; ++k) {
      const Piece& q = plan.pieces[pp.first_piece + k];
      reads_written = written.overlaps(q.addr, q.addr + q.len);
    }
    if (reads_written) break;
    // ring slots in the image: the reference pops TX slot i, and the RX slots
    // from rc on, by DMA reads after the writes before (descriptor_ring.cpp:
    // 97-106) — a slot an earlier write touched is read again after it
    if (tx_ring && written.overlaps(slots->tx_at + kTxSlot * i, slots->tx_at + kTxSlot * (i + 1))) break;
    if (rx_ring && rc < rx.size()) {
      const std::uint64_t pops = std::min<std::uint64_t>(nicqp::decide_segments(tx[i]).nseg, rx.size() - rc);
      if (pops && written.overlaps(slots->rx_at + kRxSlot * rc, slots->rx_at + kRxSlot * (rc + pops))) break;
    }
    const std::size_t w0 = writes.size();
    const std::size_t rc0 = rc;
    rc += resolve_packet(C, i, rc, stats, sink);
    if (rx_ring)  // a segment's write over an RX slot a later segment of the same packet pops
      for (std::size_t k = 1; k < rc - rc0; ++k) {
        const std::uint64_t a = slots->rx_at + kRxSlot * (rc0 + k);
        for (std::size_t j = w0; j < w0 + k; ++j) {
          const std::uint64_t d = writes[j].dst, n = write_len(writes[j]);
          if (write_of_rx[j] >= 0 && n && d < a + kRxSlot && a < d + n)
            throw GpuError("process_batch: a segment's DMA write lands on an RX descriptor slot a later segment of the same "
                           "TX descriptor pops (not modelled)",
                           NICGPU_ERR_INVALID);
        }
      }
    for (std::size_t j = w0; j < writes.size(); ++j)
      if (write_of_rx[j] >= 0) written.add(writes[j].dst, writes[j].dst + write_len(writes[j]));
  }
  out.tx_processed = i;
  out.rx_consumed = rc;
  return i;
}

std::byte* checked_reads(const HostMemory& m, std::span<const TxDescriptor> tx, std::vector<TxDescriptor>& out) {
  const std::uint64_t size = m.config().size_bytes;
  out.assign(tx.begin(), tx.end());
  const std::byte* window = nullptr;
  for (TxDescriptor& t : out) {
    // DMAEngine::read -> HostMemory::read -> translate_const (dma_engine.cpp:12-21)
    ConstHostMemoryView v{};
    if (!m.translate_const(t.buffer_address, t.length, v).ok()) {
      t.buffer_address = size + 1;  // refused: a read fault (queue_pair.cpp:96-103)
      continue;
    }
    if (v.address != t.buffer_address)
      throw GpuError("host_memory_faults: a TX read is translated to another address (not modelled)", NICGPU_ERR_INVALID);
    const std::byte* w = v.data - t.buffer_address;
    if (window && w != window)
      throw GpuError("host_memory_faults: the memory's reads do not share one flat window", NICGPU_ERR_INVALID);
    window = w;
  }
  return const_cast<std::byte*>(window);
}

void schedule_writes(std::span<const SegmentWrite> writes, std::span<const std::int64_t> write_of_rx,
                     WriteSchedule& s) {
  s.order.clear();
  s.layer_begin.assign(1, 0);
  s.from_copy = false;
  // paint[start] = (end, layer of the last write covering [start, end)): that
  // write's layer is the highest of all the writes covering those bytes
  std::map<std::uint64_t, std::pair<std::uint64_t, std::uint32_t>> paint;
  std::vector<std::pair<std::uint32_t, std::uint32_t>> lj;  // (layer, j)
  std::vector<Span64> dst, src;
  for (std::size_t j = 0; j < writes.size(); ++j) {
    if (write_of_rx[j] < 0) continue;
    const SegmentWrite& w = writes[j];
    const std::uint64_t n = write_len(w);
    if (n == 0) continue;
    const std::uint64_t a = w.dst, b = a + n;
    auto it = paint.upper_bound(a);
    if (it != paint.begin() && std::prev(it)->second.first > a) --it;
    auto e = it;
    std::uint32_t layer = 0;
    for (; e != paint.end() && e->first < b; ++e) layer = std::max(layer, e->second.second + 1);
    if (it != e) {
      const std::uint64_t ls = it->first, re = std::prev(e)->second.first;
      const std::uint32_t ll = it->second.second, rl = std::prev(e)->second.second;
      paint.erase(it, e);
      if (ls < a) paint.emplace(ls, std::make_pair(a, ll));
      if (re > b) paint.emplace(b, std::make_pair(re, rl));
    }
    paint.emplace(a, std::make_pair(b, layer));
    lj.emplace_back(layer, static_cast<std::uint32_t>(j));
    dst.push_back({a, b});
    if (w.len_a) src.push_back({w.src_a, w.src_a + w.len_a});
    if (w.len_b) src.push_back({w.src_b, w.src_b + w.len_b});
  }
  // layers in order, posting order within each (stable by layer)
  std::stable_sort(lj.begin(), lj.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  s.order.reserve(lj.size());
  for (std::size_t i = 0; i < lj.size(); ++i) {
    if (i > 0 && lj[i].first != lj[i - 1].first) s.layer_begin.push_back(i);
    s.order.push_back(lj[i].second);
  }
  s.layer_begin.push_back(lj.size());
  if (lj.empty()) s.layer_begin.assign(1, 0);
  // does any destination land on any source?
  std::sort(src.begin(), src.end(), [](const Span64& x, const Span64& y) { return x.a < y.a; });
  std::vector<Span64> merged;
  for (const Span64& x : src) {
    if (!merged.empty() && x.a <= merged.back().b) merged.back().b = std::max(merged.back().b, x.b);
    else merged.push_back(x);
  }
  for (const Span64& d : dst) {
    auto it = std::upper_bound(merged.begin(), merged.end(), d.a, [](std::uint64_t v, const Span64& x) { return v < x.a; });
    if ((it != merged.begin() && std::prev(it)->b > d.a) || (it != merged.end() && it->a < d.b)) {
      s.from_copy = true;
      break;
    }
  }
}

void run_batch(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out, BatchScratch& S,
               Backend& dev, int disjoint_hint, const DmaWriteCheck* wcheck, const RingSlots* slots) {
  using clock = std::chrono::steady_clock;
  auto us_since = [](clock::time_point t) { return std::chrono::duration<double, std::micro>(clock::now() - t).count(); };
  constexpr auto kSuccess = static_cast<std::uint32_t>(CompletionCode::Success);
  // reset `out`, keeping its storage
  out.tx_processed = out.rx_consumed = 0;
  out.tx_completions.clear();
  out.rx_completions.clear();
  out.rx_hash.clear();
  out.rx_queue.clear();
  for (auto& q : out.queues) q.clear();
  out.queues.clear();
  out.timings = RxBatchResult::Timings{};

  auto t0 = clock::now();
  // descriptor arrays in the image that a write may land on: the sub-batch
  // path, over copies of the descriptors read again between sub-batches
  const bool rings = slots != nullptr && slots->any();
  if (rings) {
    S.ring_tx.assign(tx.begin(), tx.end());
    S.ring_rx.assign(rx.begin(), rx.end());
    tx = S.ring_tx;
    rx = S.ring_rx;
  }
  const bool disjoint = !rings && (disjoint_hint >= 0 ? disjoint_hint != 0 : buffers_disjoint(mem_size, tx, rx));
  out.timings.check_us = us_since(t0);
  // RSS of the frames part.rx_completions[which[..]] delivered with Success,
  // from the image as it is now.  The tuple lies in the first 82 bytes, so a
  // frame longer than NICGPU_MAX_PACKET (max_mtu above 65531) is hashed over
  // its first NICGPU_MAX_PACKET bytes: the same tuple, hash and queue.
  auto rss_of = [&](RxBatchResult& part) {
    const std::size_t m = S.which.size();
    if (m == 0) return;
    std::uint64_t* desc = dev.frame_desc(m);
    for (std::size_t i = 0; i < m; ++i) {
      const SegmentWrite& w = S.writes[S.which[i]];
      desc[i] = NICGPU_DESC(w.dst, std::min<std::uint64_t>(write_len(w), NICGPU_MAX_PACKET));
    }
    const std::uint32_t* h = nullptr;
    const std::uint16_t* q = nullptr;
    dev.rss(m, h, q);
    for (std::size_t i = 0; i < m; ++i) {
      part.rx_hash[S.which[i]] = h[i];
      part.rx_queue[S.which[i]] = q[i];
    }
  };

  std::size_t s = 0, r = 0;
  do {
    RxBatchResult& part = disjoint ? out : S.part;
    const auto txs = tx.subspan(s);
    const auto rxs = rx.subspan(r);
    auto t = clock::now();
    make_plan(config, mem_size, txs, S.plan);
    out.timings.plan_us += us_since(t);
    t = clock::now();
    const std::span<const std::uint16_t> cs = dev.piece_sums(S.plan.pieces);
    out.timings.sums_us += us_since(t);
    t = clock::now();
    std::size_t k;
    if (disjoint) {
      resolve(config, mem_size, S.plan, cs, txs, rxs, stats, part, S.writes, S.write_of_rx, 0, wcheck);
      k = txs.size();
    } else {
      RingSlots sub;  // the offsets of txs[0] / rxs[0]
      if (rings) {
        sub.tx_at = slots->tx_at == ~0ull ? ~0ull : slots->tx_at + sizeof(TxDescriptor) * s;
        sub.rx_at = slots->rx_at == ~0ull ? ~0ull : slots->rx_at + sizeof(RxDescriptor) * r;
      }
      k = resolve_prefix(config, mem_size, S.plan, cs, txs, rxs, stats, part, S.writes, S.write_of_rx, wcheck,
                         rings ? &sub : nullptr);
    }
    out.timings.resolve_us += us_since(t);
    const std::size_t nrx = part.rx_completions.size();
    part.rx_hash.assign(nrx, 0);
    part.rx_queue.assign(nrx, RxBatchResult::kNoQueue);
    if (disjoint) {
      // one parallel gather of every write (zero-length entries write nothing)
      t = clock::now();
      if (!S.writes.empty()) dev.gather(S.writes, false);
      out.timings.gather_us += us_since(t);
      t = clock::now();
      if (config.rss != nullptr) {
        S.which.clear();
        for (std::size_t j = 0; j < nrx; ++j)
          if (part.rx_completions[j].status == kSuccess) S.which.push_back(static_cast<std::uint32_t>(j));
        rss_of(part);
      }
      out.timings.rss_us += us_since(t);
    } else {
      t = clock::now();
      schedule_writes(S.writes, S.write_of_rx, S.schedule);
      const WriteSchedule& ws = S.schedule;
      if (ws.from_copy) dev.snapshot();
      out.timings.gather_us += us_since(t);
      for (std::size_t l = 0; l + 1 < ws.layer_begin.size(); ++l) {
        t = clock::now();
        S.layer.clear();
        for (std::size_t i = ws.layer_begin[l]; i < ws.layer_begin[l + 1]; ++i) S.layer.push_back(S.writes[ws.order[i]]);
        dev.gather(S.layer, ws.from_copy);
        out.timings.gather_us += us_since(t);
        t = clock::now();
        if (config.rss != nullptr) {
          S.which.clear();
          for (std::size_t i = ws.layer_begin[l]; i < ws.layer_begin[l + 1]; ++i)
            if (part.rx_completions[ws.order[i]].status == kSuccess) S.which.push_back(ws.order[i]);
          rss_of(part);
        }
        out.timings.rss_us += us_since(t);
      }
      // Success frames of zero bytes (no layer): hash of an empty tuple
      if (config.rss != nullptr) {
        S.which.clear();
        for (std::size_t j = 0; j < nrx; ++j)
          if (part.rx_completions[j].status == kSuccess && write_len(S.writes[j]) == 0)
            S.which.push_back(static_cast<std::uint32_t>(j));
        rss_of(part);
      }
      out.tx_completions.insert(out.tx_completions.end(), part.tx_completions.begin(), part.tx_completions.end());
      out.rx_completions.insert(out.rx_completions.end(), part.rx_completions.begin(), part.rx_completions.end());
      out.rx_hash.insert(out.rx_hash.end(), part.rx_hash.begin(), part.rx_hash.end());
      out.rx_queue.insert(out.rx_queue.end(), part.rx_queue.begin(), part.rx_queue.end());
    }
    s += k;
    r += part.rx_consumed;
    if (rings && s < tx.size()) {  // the descriptors not yet popped, as the writes left them
      auto t = clock::now();
      dev.descriptors(slots->tx_at == ~0ull ? ~0ull : slots->tx_at + sizeof(TxDescriptor) * s,
                      std::span<TxDescriptor>(S.ring_tx).subspan(s),
                      slots->rx_at == ~0ull ? ~0ull : slots->rx_at + sizeof(RxDescriptor) * r,
                      std::span<RxDescriptor>(S.ring_rx).subspan(r));
      out.timings.copy_us += us_since(t);
    }
  } while (s < tx.size());
  out.tx_processed = tx.size();
  out.rx_consumed = r;

  if (config.rss != nullptr) {
    auto t = clock::now();
    build_queue_lists(out);
    out.timings.rss_us += us_since(t);
  }
}

void Backend::descriptors(std::uint64_t, std::span<TxDescriptor>, std::uint64_t, std::span<RxDescriptor>) {
  throw std::logic_error("run_batch: this backend cannot read descriptors from the image (RingSlots)");
}

void build_queue_lists(RxBatchResult& out) {
  // per-queue dispatch lists of the Success frames, in posting order
  constexpr auto kSuccess = static_cast<std::uint32_t>(CompletionCode::Success);
  std::vector<std::size_t> cnt;
  for (std::size_t j = 0; j < out.rx_completions.size(); ++j) {
    if (out.rx_completions[j].status != kSuccess) continue;
    const std::uint16_t q = out.rx_queue[j];
    if (q >= cnt.size()) cnt.resize(static_cast<std::size_t>(q) + 1, 0);
    cnt[q] += 1;
  }
  out.queues.resize(cnt.size());
  for (std::size_t q = 0; q < cnt.size(); ++q) out.queues[q].reserve(cnt[q]);
  for (std::size_t j = 0; j < out.rx_completions.size(); ++j)
    if (out.rx_completions[j].status == kSuccess) out.queues[out.rx_queue[j]].push_back(static_cast<std::uint32_t>(j));
}

}  // namespace rx_stage_detail

namespace {

void check_at(int st, const char* what, int line) {
  if (st != NICGPU_OK)
    throw GpuError(std::string(what) + " (rx_stage.cpp:" + std::to_string(line) + "): " + nicgpu_strerror(st), st);
}
// (the call site in the message: one failing HIP call among many alike)
#define check(st, what) check_at((st), (what), __LINE__)

// BatchedQueuePairConfig::defer_rx_verify unless NIC_DEFER_VERIFY=0 (tuning A/B)
bool defer_env() {
  static const bool on = [] {
    const char* e = std::getenv("NIC_DEFER_VERIFY");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// The overlap check of a batch with no other in flight launched before the
// resolve on a normal-priority stream of its own (measured: one at a time
// 421-427 -> 413-415 us; with batches pending it only competes with the
// earlier delivery, 338-342 -> 345-347 us, so then it stays behind the plan),
// or NIC_CHECK_EARLY=0: never (tuning A/B)
bool check_early_env() {
  static const bool on = [] {
    const char* e = std::getenv("NIC_CHECK_EARLY");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// Host-image TX staging on its own stream (measured, profiles/r06_hostmem_ab.txt:
// behind the descriptor uploads on side_up, each batch's span copy started
// 1-2 ms late), or NIC_STAGE_STREAM=0: on side_up (tuning A/B)
bool stage_stream_env() {
  static const bool on = [] {
    const char* e = std::getenv("NIC_STAGE_STREAM");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// HostMemory mirrors in HBM for pipelined batches: 2, or NIC_IMAGE_MIRRORS=1
// (tuning A/B)
unsigned image_mirrors_env() {
  static const unsigned n = [] {
    const char* e = std::getenv("NIC_IMAGE_MIRRORS");
    return e && std::strcmp(e, "1") == 0 ? 1u : 2u;
  }();
  return n;
}

// One growable device buffer.
struct DevBuf {
  void* p = nullptr;
  std::size_t cap = 0;
  void* get(std::size_t n) {
    if (n > cap) {
      nicgpu_free(p);
      p = nullptr;
      cap = 0;
      check(nicgpu_malloc(&p, n), "nicgpu_malloc");
      cap = n;
    }
    return p;
  }
  ~DevBuf() { nicgpu_free(p); }
};

// One growable page-locked host buffer (staging for the H2D/D2H copies).
struct HostBuf {
  void* p = nullptr;
  std::size_t cap = 0;
  template <class T>
  T* get(std::size_t n) {
    const std::size_t bytes = n * sizeof(T);
    if (bytes > cap) {
      nicgpu_host_free(p);
      p = nullptr;
      cap = 0;
      check(nicgpu_host_alloc(&p, bytes), "nicgpu_host_alloc");
      cap = bytes;
    }
    return static_cast<T*>(p);
  }
  ~HostBuf() { nicgpu_host_free(p); }
};

}  // namespace

// Everything process_batch allocates, kept across batches (grown, never
// shrunk): the device buffers, pinned staging, and the host-side plan and
// write lists, so a steady stream of batches takes no page faults.
namespace {

// The stage's helper thread, started on first use and reused across batches
// (a thread per job costs tens of µs, a tenth of a small batch).  One job at
// a time: start() follows the previous job's wait().
class SideWorker {
public:
  ~SideWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  void start(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    job_ = std::move(f);
    done_ = false;
    done_flag_.store(false, std::memory_order_relaxed);
    cv_.notify_all();
  }
  // A job ends a batch the caller is waiting for: spin briefly before
  // sleeping, so the caller does not pay a thread wake-up (tens of µs) on the
  // batch's critical path.
  void wait() {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned i = 0; !done_flag_.load(std::memory_order_acquire); ++i) {
      if ((i & 63u) == 63u && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(1500)) break;
      std::this_thread::yield();
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return done_; });
  }

private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return stop_ || job_ != nullptr; });
      if (!job_) return;  // stopping, nothing queued
      std::function<void()> f = std::move(job_);
      job_ = nullptr;
      lk.unlock();
      f();
      lk.lock();
      done_ = true;
      done_flag_.store(true, std::memory_order_release);  // under the lock: a new job's start() cannot interleave
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  std::function<void()> job_;
  bool done_ = true, stop_ = false;
  std::atomic<bool> done_flag_{true};
};

// A pageable host<->device copy keeps the thread that issues it busy until the
// copy is staged, so copies meant to run beside the main stream's work are
// issued from the helper thread; errors come back to the caller at finish().
class SideJob {
public:
  explicit SideJob(SideWorker& w) : w_(w) {}
  template <class F>
  void start(F f) {
    w_.start([this, f] { f(*this); });
    running_ = true;
  }
  // records the first failure
  bool ok(int st, const char* what) {
    if (st != NICGPU_OK && status_ == NICGPU_OK) {
      status_ = st;
      what_ = what;
    }
    return status_ == NICGPU_OK;
  }
  void finish() {
    if (running_) w_.wait();
    running_ = false;
    check(status_, what_);
  }
  ~SideJob() {
    if (running_) w_.wait();
  }

private:
  SideWorker& w_;
  bool running_ = false;
  int status_ = NICGPU_OK;
  const char* what_ = "";
};

}  // namespace

namespace {

// In-order job runner: submit()'s batches are planned, resolved and enqueued
// on the device by this thread while the caller uploads the next batch.
class JobQueue {
public:
  ~JobQueue() { stop(); }
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!th_.joinable()) th_ = std::thread([this] { loop(); });
      q_.push_back(std::move(f));
    }
    cv_.notify_all();
  }
  // runs what is queued, then ends the thread (a later push starts another)
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = false;
  }

private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      std::function<void()> f = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      f();  // jobs catch their own exceptions
      lk.lock();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
};

}  // namespace

// One batch in flight on the device.  process_batch uses slot 0; submit()
// cycles through all of them, so batch k's buffers stay untouched while its
// results come down, batch k+1 is planned and resolved and batch k+2's
// descriptors go up.
namespace {
// host_memory_faults: a HostMemory's verdict on each DMA write, as
// DMAEngine::write reaches it (HostMemory::write -> translate,
// dma_engine.cpp:23-32, simple_host_memory.cpp:58-68): refused -> the
// reference's Fault completion; allowed -> the write lands where the window
// puts it (a translation elsewhere is not modelled).
struct MemWriteCheck final : rx_stage_detail::DmaWriteCheck {
  HostMemory* mem = nullptr;
  std::byte* window = nullptr;  // host address 0 (the registered window)
  bool write_ok(std::uint64_t a, std::uint64_t n) const override {
    HostMemoryView v{};
    if (!mem->translate(a, n, v).ok()) return false;
    if (v.address != a || window == nullptr || v.data != window + a)
      throw GpuError("host_memory_faults: an RX write is translated to another address (not modelled)",
                     NICGPU_ERR_INVALID);
    return true;
  }
};
}  // namespace

struct BatchedQueuePair::Slot {
  nicgpu_qp* qp = nullptr;   // device resolve context (same device as the Scratch streams)
  void* ev_tx = nullptr;     // TX descriptors uploaded
  void* ev_rx = nullptr;     // RX descriptors uploaded
  void* ev_resolved = nullptr;  // completions final
  void* ev_done = nullptr;      // DMA writes and RSS done
  void* ev_submit = nullptr;    // the caller's stream at submit (device descriptors handed over; frames produced)
  void* ev_gate = nullptr;      // overlapped resolve: the caller's stream, for a batch whose frames earlier batches write
  // overlapped resolve (submit/collect): the piece sums and the resolve on the
  // resolve stream, beside the earlier batches' DMA writes; rx_lo/hi_w: the
  // bytes this batch's DMA writes can touch ([0, ~0) unknown), for the later
  // batches' hazard test
  bool overlap = false;
  std::uint64_t rx_lo_w = 0, rx_hi_w = ~0ull;
  DevBuf hits;               // per-table-index RSS hits of the batch
  HostBuf h_meta, h_lists;   // pinned landing space of the downloads
  SideWorker worker;         // issues the downloads
  // the batch, between front() and finish()
  nicgpu_qp_view v{};
  std::size_t ntx = 0, nrx_total = 0, tn = 0, nq = 0;
  std::size_t settled = 0;  // completions [0, settled) delivered with the resolve
  bool relaxed = false;     // completions rewritten after the resolve's event
  bool rss = false;
  std::uint64_t* meta = nullptr;  // [count][hits tn]
  std::uint32_t *qs = nullptr, *qe = nullptr, *which = nullptr;
  std::optional<SideJob> down;
  std::promise<void> rss_recorded;  // ev_done is recorded (the download job waits for it)
  bool rss_released = false;
  double upload_us = 0;  // time upload() held its thread
  std::optional<SideJob> up;  // process_batch: the RX upload beside the plan
  // descriptors already in device memory (DeviceDescriptors): no upload; host
  // copies fetched only when a host step needs them
  const TxDescriptor* tx_dev = nullptr;
  const RxDescriptor* rx_dev = nullptr;
  std::size_t ntx_dev = 0, nrx_dev = 0;
  std::vector<TxDescriptor> htx;
  std::vector<RxDescriptor> hrx;
  bool fetched = false;
  // submit(): the batch, where its results land until collect(), its stats,
  // and the job that plans, resolves and enqueues it
  DeviceHostMemory mem{};
  std::span<const TxDescriptor> tx;
  std::span<const RxDescriptor> rx;
  void* stream = nullptr;
  RxBatchResult result;
  QueuePairStats stats{};
  bool on_device = false;
  std::promise<void> job_done;
  std::future<void> job;
  // host-image batch (HostMemory): the TX bytes' span / the RX buffers' box in
  // the memory, the earlier pending batches whose write-back the stage-in
  // (dep_stage) or the delivery (dep_rx) must follow, and the writes a
  // host-path batch made (written back from the device copy in wbuf)
  HostImage* image = nullptr;
  unsigned mirror = 0;        // which of the image's HBM mirrors the batch runs on
  void* ev_staged = nullptr;  // the batch's TX bytes are in the mirror
  void* ev_wb = nullptr;      // its delivered bytes are back in the host memory
  bool staged = false, stage_deferred = false, wb = false, whole = false;
  std::uint64_t tx_lo = 0, tx_hi = 0, tx_bytes = 0, rx_lo = 0, rx_hi = 0;
  std::vector<Slot*> dep_stage, dep_rx;
  std::vector<rx_stage_detail::SegmentWrite> applied;
  // host_memory_faults: the TX descriptors with refused reads moved out of
  // bounds (the batch runs on these), and the memory's write verdicts
  std::vector<TxDescriptor> checked_tx;
  MemWriteCheck mem_writes;
  const rx_stage_detail::DmaWriteCheck* wcheck = nullptr;
  DevBuf wbuf, stage_tx;
  HostBuf h_applied;
  // a manager's fused batch (process_queues): nseg queue pairs; their RSS
  // dispatch lists split per queue pair (split, (nseg + 1) x nq) and, when
  // they count into RssEngines of their own, their hits (seg_hits, nseg x tn)
  bool multi = false, seg_hits_on = false;
  std::size_t nseg = 0;
  HostBuf h_split, h_seg_hits;
  DevBuf seg_hits;
  // interrupt callbacks of a batch whose results stay on the device: its
  // completions come down in chunks into page-locked memory as soon as they
  // are final (side_irq), and the replay starts on the first chunk
  static constexpr int kIrqChunks = 16;
  void* ev_irq[2][kIrqChunks] = {};
  HostBuf h_itx, h_irx;
  bool irq_pending = false;
  std::size_t irq_ntx = 0, irq_nrx = 0;
  // deferred RX verify (nicgpu_qp_set_deferred_verify): the batch's completions
  // and statistics are final after its deliveries; its corrections (per
  // segment of a fused batch; the plan zeroes them on the device, so a batch
  // that failed after its deliveries leaves nothing for the next) come down
  // into h_fix
  bool late = false;
  HostBuf h_fix;
  // this batch's correction k of segment s
  std::uint64_t fix_delta(std::size_t s, unsigned k) const {
    return static_cast<const std::uint64_t*>(h_fix.p)[s * NICGPU_QP_FIXUPS + k];
  }

  void release_rss() {
    if (!rss_released) rss_recorded.set_value();
    rss_released = true;
  }
  void wait() {  // the batch's downloads, if any are running (errors dropped)
    if (down) {
      release_rss();
      down.reset();
    }
  }
  void release() {
    wait();
    up.reset();
    if (qp) (void) nicgpu_qp_destroy(qp);
    if (wb) (void) nicgpu_event_synchronize(ev_wb);  // no write-back may outlive the slot's buffers
    wb = false;
    for (auto& side : ev_irq)
      for (void*& e : side) {
        if (e && irq_pending) (void) nicgpu_event_synchronize(e);
        if (e) (void) nicgpu_event_destroy(e);
        e = nullptr;
      }
    irq_pending = false;
    for (void* e : {ev_tx, ev_rx, ev_resolved, ev_done, ev_submit, ev_staged, ev_wb, ev_gate})
      if (e) (void) nicgpu_event_destroy(e);
    qp = nullptr;
    ev_tx = ev_rx = ev_resolved = ev_done = ev_submit = ev_staged = ev_wb = ev_gate = nullptr;
  }
  void create(int dev) {
    check(nicgpu_qp_create(&qp, dev), "nicgpu_qp_create");
    for (void** e : {&ev_tx, &ev_rx, &ev_resolved, &ev_done, &ev_submit, &ev_staged, &ev_wb, &ev_gate})
      check(nicgpu_event_create(e), "nicgpu_event_create");
    for (auto& side : ev_irq)
      for (void*& e : side) check(nicgpu_event_create(&e), "nicgpu_event_create");
  }
  // the batch's bytes are in the host memory (host-image batches)
  void wait_writeback() {
    if (!wb) return;
    wb = false;
    check(nicgpu_event_synchronize(ev_wb), "nicgpu_event_synchronize");
  }
  ~Slot() { release(); }
};

// A HostMemory's flat window, page-locked and mapped for the device, and its
// mirror in HBM (the image every kernel of the stage works on).
struct BatchedQueuePair::HostImage {
  HostMemory* mem = nullptr;
  std::byte* host = nullptr;      // translate(0, size).data
  std::uint8_t* alias = nullptr;  // its device-visible address (nicgpu_host_register)
  bool owned = false;             // registered by this stage
  std::size_t size = 0;
  int device = -1;
  // two mirrors: pipelined batches alternate between them, so a batch's
  // delivery need not wait for the previous batch's write-back out of the
  // same bytes (the second is allocated by the first pipelined submit)
  DevBuf mirror[2];
  DeviceHostMemory view(unsigned m = 0) const {
    return DeviceHostMemory{static_cast<std::byte*>(mirror[m].p), size};
  }
  void release() {
    if (owned && host) (void) nicgpu_host_unregister(host);
    mem = nullptr;
    host = nullptr;
    alias = nullptr;
    owned = false;
    size = 0;
    device = -1;
  }
  ~HostImage() { release(); }
};

struct BatchedQueuePair::Scratch {
  DevBuf piece_desc, piece_csum, writes, rss_desc, rss_hash, rss_queue, copy;
  HostBuf h_desc, h_csum, h_writes, h_rss_desc, h_hash, h_queue;
  rx_stage_detail::BatchScratch host;
  std::vector<std::uint16_t> tail_cs;
  std::vector<CompletionEntry> irq_tx, irq_rx;  // completions fetched for the interrupt callbacks
  // device resolve: side streams for uploads beside the plan and downloads
  // beside the next steps, created with the slots on the current device
  int device = -1;
  void* side_up = nullptr;
  void* side_down = nullptr;
  void* side_plan = nullptr;  // plan and overlap check of a batch beside the earlier batch's writes
  void* side_wb = nullptr;    // host-image write-backs, beside the next batches' work
  void* side_irq = nullptr;   // completions for the interrupt callbacks, as soon as they are final
  void* side_res = nullptr;   // overlapped resolves: piece sums and resolve beside the earlier batches' DMA writes
  void* side_stage = nullptr; // host-image TX staging, apart from the descriptor uploads (see stage_stream)
  void* side_chk = nullptr;   // the overlap check launched early (check_early_env), at normal priority
  // the job thread's record of the two batches before the current one (their
  // DMA writes may still run): the bytes each can write, [0, ~0) unknown
  struct WriteBox {
    std::uint64_t lo = 0, hi = ~0ull;
  };
  WriteBox recent[2];
  unsigned n_recent = 0;
  std::uint64_t overlaps = 0, overlaps_redone = 0;
  std::shared_ptr<HostImage> img = std::make_shared<HostImage>();  // the HostMemory the host-image batches run against (shared by a manager's stages)
  SideWorker up_worker;  // process_batch: issues the RX descriptor uploads
  static constexpr unsigned kSlots = 3;
  Slot slot[kSlots];
  unsigned head = 0, pending = 0;  // submit(): oldest pending slot, batches pending
  std::atomic<unsigned> inflight{0};  // pending, as the job thread reads it (a later batch submitted?)
  JobQueue jobs;                   // submit(): plans, resolves and enqueues the batches in order
  void release() {
    for (Slot& sl : slot) sl.release();
    if (side_up) (void) nicgpu_stream_destroy(side_up);
    if (side_down) (void) nicgpu_stream_destroy(side_down);
    if (side_plan) (void) nicgpu_stream_destroy(side_plan);
    if (side_wb) (void) nicgpu_stream_destroy(side_wb);
    if (side_irq) (void) nicgpu_stream_destroy(side_irq);
    if (side_res) (void) nicgpu_stream_destroy(side_res);
    if (side_stage) (void) nicgpu_stream_destroy(side_stage);
    if (side_chk) (void) nicgpu_stream_destroy(side_chk);
    side_up = side_down = side_plan = side_wb = side_irq = side_res = side_stage = side_chk = nullptr;
    if (img.use_count() == 1) img->release();  // a manager's shared image is released by its last stage
    device = -1;
  }
  void ensure(int dev) {
    if (device == dev) return;
    release();
    check(nicgpu_stream_create(&side_up), "nicgpu_stream_create");
    check(nicgpu_stream_create(&side_down), "nicgpu_stream_create");
    static const int plan_low = [] {  // tuning A/B: NIC_PLAN_PRIORITY=high
      const char* e = std::getenv("NIC_PLAN_PRIORITY");
      return e && std::strcmp(e, "high") == 0 ? 0 : 1;
    }();
    check(nicgpu_stream_create_priority(&side_plan, plan_low), "nicgpu_stream_create_priority");
    check(nicgpu_stream_create(&side_wb), "nicgpu_stream_create");
    check(nicgpu_stream_create(&side_irq), "nicgpu_stream_create");
    check(nicgpu_stream_create_priority(&side_res, 0), "nicgpu_stream_create_priority");  // high: beside a DMA write
    check(nicgpu_stream_create(&side_stage), "nicgpu_stream_create");
    check(nicgpu_stream_create(&side_chk), "nicgpu_stream_create");
    for (Slot& sl : slot) sl.create(dev);
    device = dev;
  }
  ~Scratch() {
    jobs.stop();  // no job may still use a slot
    release();
  }
};

// The device mirrors (nicgpu.h) of the PODs the device resolve moves.
static_assert(sizeof(nicgpu_tx_descriptor) == sizeof(TxDescriptor) && sizeof(nicgpu_rx_descriptor) == sizeof(RxDescriptor));
static_assert(offsetof(nicgpu_tx_descriptor, length) == offsetof(TxDescriptor, length) &&
              offsetof(nicgpu_tx_descriptor, checksum) == offsetof(TxDescriptor, checksum) &&
              offsetof(nicgpu_tx_descriptor, descriptor_index) == offsetof(TxDescriptor, descriptor_index) &&
              offsetof(nicgpu_tx_descriptor, checksum_value) == offsetof(TxDescriptor, checksum_value) &&
              offsetof(nicgpu_tx_descriptor, checksum_offload) == offsetof(TxDescriptor, checksum_offload) &&
              offsetof(nicgpu_tx_descriptor, tso_enabled) == offsetof(TxDescriptor, tso_enabled) &&
              offsetof(nicgpu_tx_descriptor, gso_enabled) == offsetof(TxDescriptor, gso_enabled) &&
              offsetof(nicgpu_tx_descriptor, mss) == offsetof(TxDescriptor, mss) &&
              offsetof(nicgpu_tx_descriptor, header_length) == offsetof(TxDescriptor, header_length) &&
              offsetof(nicgpu_tx_descriptor, vlan_insert) == offsetof(TxDescriptor, vlan_insert) &&
              offsetof(nicgpu_tx_descriptor, vlan_tag) == offsetof(TxDescriptor, vlan_tag));
static_assert(offsetof(nicgpu_rx_descriptor, buffer_length) == offsetof(RxDescriptor, buffer_length) &&
              offsetof(nicgpu_rx_descriptor, checksum) == offsetof(RxDescriptor, checksum) &&
              offsetof(nicgpu_rx_descriptor, descriptor_index) == offsetof(RxDescriptor, descriptor_index) &&
              offsetof(nicgpu_rx_descriptor, checksum_offload) == offsetof(RxDescriptor, checksum_offload) &&
              offsetof(nicgpu_rx_descriptor, vlan_strip) == offsetof(RxDescriptor, vlan_strip) &&
              offsetof(nicgpu_rx_descriptor, vlan_present) == offsetof(RxDescriptor, vlan_present) &&
              offsetof(nicgpu_rx_descriptor, vlan_tag) == offsetof(RxDescriptor, vlan_tag) &&
              offsetof(nicgpu_rx_descriptor, gro_enabled) == offsetof(RxDescriptor, gro_enabled));
static_assert(sizeof(nicgpu_completion) == sizeof(CompletionEntry) &&
              offsetof(nicgpu_completion, status) == offsetof(CompletionEntry, status) &&
              offsetof(nicgpu_completion, checksum_offloaded) == offsetof(CompletionEntry, checksum_offloaded) &&
              offsetof(nicgpu_completion, gro_aggregated) == offsetof(CompletionEntry, gro_aggregated) &&
              offsetof(nicgpu_completion, segments_produced) == offsetof(CompletionEntry, segments_produced) &&
              offsetof(nicgpu_completion, vlan_tag) == offsetof(CompletionEntry, vlan_tag));
static_assert(sizeof(nicgpu_qp_stats) == sizeof(QueuePairStats));
static_assert(sizeof(nicgpu_segment_write) == sizeof(rx_stage_detail::SegmentWrite));

namespace {

// The GPU side of run_batch: every operation is a nicgpu_* launch on `stream`
// over the device-resident image, synchronised before returning.
class GpuBackend final : public rx_stage_detail::Backend {
public:
  GpuBackend(BatchedQueuePair::Scratch& s, const DeviceHostMemory& mem, const BatchedQueuePairConfig& config,
             void* stream, std::vector<rx_stage_detail::SegmentWrite>* applied = nullptr)
      : S(s), mem_(mem), config_(config), stream_(stream), applied_(applied) {}

  std::span<const std::uint16_t> piece_sums(std::span<const rx_stage_detail::Piece> pieces) override {
    const std::size_t np = pieces.size();
    std::uint16_t* csum = S.h_csum.get<std::uint16_t>(std::max<std::size_t>(np, 1));
    if (np == 0) return {};
    std::uint64_t* desc = S.h_desc.get<std::uint64_t>(np);
    rx_stage_detail::Chunks(np, config_.host_threads ? config_.host_threads : 16).run([&](std::size_t, std::size_t b, std::size_t e) {
      for (std::size_t i = b; i < e; ++i) desc[i] = NICGPU_DESC(pieces[i].addr, pieces[i].len);
    });
    void* d_desc = S.piece_desc.get(np * 8);
    void* d_cs = S.piece_csum.get(np * 2);
    check(nicgpu_memcpy_async(d_desc, desc, np * 8, stream_), "nicgpu_memcpy_async");
    check(nicgpu_checksum_batch(image(), static_cast<const std::uint64_t*>(d_desc), np, static_cast<std::uint16_t*>(d_cs),
                                stream_),
          "nicgpu_checksum_batch");
    check(nicgpu_memcpy_async(csum, d_cs, np * 2, stream_), "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream_), "nicgpu_stream_synchronize");
    return {csum, np};
  }

  void snapshot() override {
    void* c = S.copy.get(std::max<std::size_t>(mem_.size, 1));
    if (mem_.size) check(nicgpu_memcpy_async(c, mem_.base, mem_.size, stream_), "nicgpu_memcpy_async");
    have_copy_ = true;
  }

  void gather(std::span<const rx_stage_detail::SegmentWrite> writes, bool from_copy) override {
    const std::size_t nw = writes.size();
    if (nw == 0) return;
    if (from_copy && !have_copy_) throw GpuError("process_batch: gather from a copy that was never taken", NICGPU_ERR_INVALID);
    if (applied_)
      for (const auto& w : writes)
        if (rx_stage_detail::write_len(w)) applied_->push_back(w);
    auto* hw = S.h_writes.get<rx_stage_detail::SegmentWrite>(nw);
    std::memcpy(hw, writes.data(), nw * sizeof(rx_stage_detail::SegmentWrite));
    void* d_w = S.writes.get(nw * sizeof(rx_stage_detail::SegmentWrite));
    check(nicgpu_memcpy_async(d_w, hw, nw * sizeof(rx_stage_detail::SegmentWrite), stream_), "nicgpu_memcpy_async");
    const auto* src = from_copy ? static_cast<const std::uint8_t*>(S.copy.p) : image();
    check(nicgpu_segment_gather_from(image(), src, mem_.size, static_cast<const nicgpu_segment_write*>(d_w), nw, stream_),
          "nicgpu_segment_gather_from");
    check(nicgpu_stream_synchronize(stream_), "nicgpu_stream_synchronize");
  }

  std::uint64_t* frame_desc(std::size_t n) override { return S.h_rss_desc.get<std::uint64_t>(std::max<std::size_t>(n, 1)); }

  void descriptors(std::uint64_t tx_at, std::span<TxDescriptor> tx, std::uint64_t rx_at,
                   std::span<RxDescriptor> rx) override {
    if (tx_at != ~0ull && !tx.empty())
      check(nicgpu_memcpy_async(tx.data(), image() + tx_at, tx.size_bytes(), stream_), "nicgpu_memcpy_async");
    if (rx_at != ~0ull && !rx.empty())
      check(nicgpu_memcpy_async(rx.data(), image() + rx_at, rx.size_bytes(), stream_), "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream_), "nicgpu_stream_synchronize");
  }

  void rss(std::size_t m, const std::uint32_t*& hash, const std::uint16_t*& queue) override {
    void* d_desc = S.rss_desc.get(m * 8);
    void* d_h = S.rss_hash.get(m * 4);
    void* d_q = S.rss_queue.get(m * 2);
    check(nicgpu_memcpy_async(d_desc, S.h_rss_desc.p, m * 8, stream_), "nicgpu_memcpy_async");
    config_.rss->select_queue_batch(
        DevicePacketBatch{mem_.base, static_cast<const std::uint64_t*>(d_desc), m}, config_.tuple,
        RxBatchOutputs{nullptr, static_cast<std::uint32_t*>(d_h), static_cast<std::uint16_t*>(d_q)}, stream_, true);
    std::uint32_t* h = S.h_hash.get<std::uint32_t>(m);
    std::uint16_t* q = S.h_queue.get<std::uint16_t>(m);
    check(nicgpu_memcpy_async(h, d_h, m * 4, stream_), "nicgpu_memcpy_async");
    check(nicgpu_memcpy_async(q, d_q, m * 2, stream_), "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream_), "nicgpu_stream_synchronize");
    hash = h;
    queue = q;
  }

private:
  std::uint8_t* image() const { return reinterpret_cast<std::uint8_t*>(mem_.base); }
  BatchedQueuePair::Scratch& S;
  const DeviceHostMemory& mem_;
  const BatchedQueuePairConfig& config_;
  void* stream_;
  std::vector<rx_stage_detail::SegmentWrite>* applied_;
  bool have_copy_ = false;
};

}  // namespace

BatchedQueuePair::BatchedQueuePair(BatchedQueuePairConfig config)
    : config_(std::move(config)), quiet_(config_), scratch_(std::make_unique<Scratch>()) {
  quiet_.on_interrupt = nullptr;
}
BatchedQueuePair::~BatchedQueuePair() = default;
// The job thread's queued batches call back into the object that submitted
// them, so a move first lets them finish (their downloads and collect() need
// only the heap-held Scratch).
BatchedQueuePair::BatchedQueuePair(BatchedQueuePair&& o) noexcept {
  if (o.scratch_) o.scratch_->jobs.stop();
  config_ = std::move(o.config_);
  quiet_ = std::move(o.quiet_);
  stats_ = o.stats_;
  scratch_ = std::move(o.scratch_);
}
BatchedQueuePair& BatchedQueuePair::operator=(BatchedQueuePair&& o) noexcept {
  if (this != &o) {
    if (scratch_) scratch_->jobs.stop();
    if (o.scratch_) o.scratch_->jobs.stop();
    config_ = std::move(o.config_);
    quiet_ = std::move(o.quiet_);
    stats_ = o.stats_;
    scratch_ = std::move(o.scratch_);
  }
  return *this;
}

// Batches past the device context's 32-bit piece indices (nicgpu.h
// NICGPU_QP_MAX_TX) take the host path, as a descriptor planning too many
// pieces does (front(): NICGPU_ERR_RANGE).
static bool device_fits(std::size_t ntx, std::size_t nrx) noexcept {
  return ntx <= NICGPU_QP_MAX_TX && nrx <= NICGPU_QP_MAX_RX;
}

RxBatchResult BatchedQueuePair::process_batch(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                                              std::span<const RxDescriptor> rx, void* stream) {
  RxBatchResult out;
  process_batch(mem, tx, rx, out, stream);
  return out;
}

void BatchedQueuePair::process_batch(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                                     std::span<const RxDescriptor> rx, RxBatchResult& out, void* stream) {
  if (mem.base == nullptr && mem.size != 0) throw GpuError("process_batch: null host-memory image", NICGPU_ERR_INVALID);
  if (scratch_->pending) throw std::logic_error("process_batch: collect() the submitted batches first");
  // stats are committed only when the whole batch went through
  QueuePairStats st = stats_;
  int disjoint = -1;  // unknown; the device path checks on the device
  double check_us = 0;
  bool on_device = false;
  if (config_.device_resolve && device_fits(tx.size(), rx.size())) {
    int dev = 0;
    check(nicgpu_get_device(&dev), "nicgpu_get_device");
    scratch_->ensure(dev);
    Slot& sl = scratch_->slot[0];
    sl.tx_dev = nullptr;
    sl.rx_dev = nullptr;
    sl.image = nullptr;
    sl.staged = false;
    sl.multi = false;
    sl.overlap = false;
    sl.dep_stage.clear();
    sl.dep_rx.clear();
    upload(sl, tx, rx, true);
    on_device = front(sl, mem, tx, rx, st, out, stream, disjoint, check_us);
    if (on_device) {
      back(sl, mem, out, stream);
      finish(sl, out, &st);
    }
  }
  if (!on_device) on_host(mem, tx, rx, st, out, stream, disjoint, check_us);
  out.timings.check_us = check_us;
  stats_ = st;
  if (config_.on_interrupt) fire_interrupts(out, &scratch_->slot[0]);
}

void BatchedQueuePair::on_host(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                               std::span<const RxDescriptor> rx, QueuePairStats& st, RxBatchResult& out, void* stream,
                               int disjoint, double& check_us, std::vector<rx_stage_detail::SegmentWrite>* applied,
                               const rx_stage_detail::DmaWriteCheck* wcheck, const rx_stage_detail::RingSlots* slots) {
  using clock = std::chrono::steady_clock;
  out.dev = RxBatchResult::DeviceResults{};
  if (disjoint < 0) {
    const auto t0 = clock::now();
    disjoint = rx_stage_detail::buffers_disjoint(mem.size, tx, rx) ? 1 : 0;
    check_us += std::chrono::duration<double, std::micro>(clock::now() - t0).count();
  }
  GpuBackend dev{*scratch_, mem, config_, stream, applied};
  rx_stage_detail::run_batch(quiet_, mem.size, tx, rx, st, out, scratch_->host, dev, disjoint, wcheck, slots);
}

void BatchedQueuePair::process_batch(const DeviceHostMemory& mem, const DeviceDescriptors& d, RxBatchResult& out,
                                     void* stream) {
  if (mem.base == nullptr && mem.size != 0) throw GpuError("process_batch: null host-memory image", NICGPU_ERR_INVALID);
  if ((d.ntx && !d.tx) || (d.nrx && !d.rx)) throw GpuError("process_batch: null device descriptors", NICGPU_ERR_INVALID);
  if (scratch_->pending) throw std::logic_error("process_batch: collect() the submitted batches first");
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  scratch_->ensure(dev);
  Slot& sl = scratch_->slot[0];
  sl.tx_dev = d.tx;
  sl.rx_dev = d.rx;
  sl.ntx_dev = d.ntx;
  sl.nrx_dev = d.nrx;
  sl.fetched = false;
  sl.image = nullptr;
  sl.staged = false;
  sl.multi = false;
  sl.overlap = false;
  sl.dep_stage.clear();
  sl.dep_rx.clear();
  check(nicgpu_event_record(sl.ev_submit, stream), "nicgpu_event_record");  // a producer's writes before this call
  QueuePairStats st = stats_;
  int disjoint = -1;
  double check_us = 0;
  bool on_device = false;
  if (config_.device_resolve && device_fits(d.ntx, d.nrx)) {
    on_device = front(sl, mem, {}, {}, st, out, stream, disjoint, check_us);
    if (on_device) {
      back(sl, mem, out, stream);
      finish(sl, out, &st);
    }
  }
  if (!on_device) {
    rx_stage_detail::RingSlots rs;
    const bool rw = rings_written(sl, mem, stream, &rs);
    const auto [htx, hrx] = host_spans(sl, {}, {}, stream);
    on_host(mem, htx, hrx, st, out, stream, disjoint, check_us, nullptr, nullptr, rw ? &rs : nullptr);
  }
  out.timings.check_us = check_us;
  stats_ = st;
  if (config_.on_interrupt) fire_interrupts(out, &sl);
}

// Device descriptor arrays inside the image that an RX buffer of the batch
// overlaps: a DMA write there changes descriptors the reference pops later
// (descriptor_ring.cpp:97-106), so the batch goes to the host path with the
// arrays' image offsets in *slots, which re-reads them between sub-batches.
// An array that only partly lies in the image is refused (GpuError, before
// anything is written) when a buffer overlaps it.
bool BatchedQueuePair::rings_written(Slot& sl, const DeviceHostMemory& mem, void* stream,
                                     rx_stage_detail::RingSlots* slots) {
  if (!sl.tx_dev && !sl.rx_dev) return false;
  const auto b = reinterpret_cast<std::uintptr_t>(mem.base);
  struct Span {
    std::uint64_t lo, hi;
    bool whole;
  };
  Span rings[2];
  std::uint64_t* at[2] = {nullptr, nullptr};
  int nr = 0;
  rx_stage_detail::RingSlots rs;
  auto add = [&](const void* p, std::size_t bytes, std::uint64_t* where) {
    const auto a = reinterpret_cast<std::uintptr_t>(p);
    if (!bytes || a >= b + mem.size || a + bytes <= b) return;
    const std::uint64_t lo = a > b ? a - b : 0, hi = std::min<std::uint64_t>(a + bytes - b, mem.size);
    const bool whole = a >= b && a + bytes <= b + mem.size;
    at[nr] = where;
    rings[nr++] = Span{lo, hi, whole};
  };
  add(sl.tx_dev, sl.ntx_dev * sizeof(TxDescriptor), &rs.tx_at);
  add(sl.rx_dev, sl.nrx_dev * sizeof(RxDescriptor), &rs.rx_at);
  if (nr == 0) return false;
  const auto hrx = host_spans(sl, {}, {}, stream).second;
  bool hit[2] = {false, false};
  for (const RxDescriptor& d : hrx) {
    if (d.buffer_length == 0 || d.buffer_address >= mem.size) continue;
    const std::uint64_t lo = d.buffer_address, hi = std::min<std::uint64_t>(lo + d.buffer_length, mem.size);
    for (int k = 0; k < nr; ++k) hit[k] = hit[k] || (lo < rings[k].hi && rings[k].lo < hi);
  }
  bool any = false;
  for (int k = 0; k < nr; ++k) {
    if (!hit[k]) continue;
    if (!rings[k].whole)
      throw GpuError("process_batch: an RX buffer overlaps a descriptor array that lies only partly in the image",
                     NICGPU_ERR_INVALID);
    *at[k] = rings[k].lo;
    any = true;
  }
  if (any && slots) {
    // (both arrays' offsets when both lie in the image: a write may land on either)
    for (int k = 0; k < nr; ++k)
      if (rings[k].whole) *at[k] = rings[k].lo;
    *slots = rs;
  }
  return any;
}

// The batch's descriptors on the host: the caller's spans, or (device
// descriptors) copies fetched once, in stream order.
std::pair<std::span<const TxDescriptor>, std::span<const RxDescriptor>> BatchedQueuePair::host_spans(
    Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx, void* stream) {
  if (!sl.tx_dev && !sl.rx_dev) return {tx, rx};
  if (!sl.fetched) {
    sl.htx.resize(sl.ntx_dev);
    sl.hrx.resize(sl.nrx_dev);
    if (sl.ntx_dev)
      check(nicgpu_memcpy_async(sl.htx.data(), sl.tx_dev, sl.ntx_dev * sizeof(TxDescriptor), stream),
            "nicgpu_memcpy_async");
    if (sl.nrx_dev)
      check(nicgpu_memcpy_async(sl.hrx.data(), sl.rx_dev, sl.nrx_dev * sizeof(RxDescriptor), stream),
            "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");
    sl.fetched = true;
  }
  return {sl.htx, sl.hrx};
}

void BatchedQueuePair::submit(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                              std::span<const RxDescriptor> rx, void* stream) {
  enqueue(mem, tx, rx, nullptr, stream);
}

void BatchedQueuePair::submit(const DeviceHostMemory& mem, const DeviceDescriptors& d, void* stream) {
  if ((d.ntx && !d.tx) || (d.nrx && !d.rx)) throw GpuError("submit: null device descriptors", NICGPU_ERR_INVALID);
  enqueue(mem, {}, {}, &d, stream);
}

void BatchedQueuePair::enqueue(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                               std::span<const RxDescriptor> rx, const DeviceDescriptors* d, void* stream,
                               HostImage* img) {
  if (mem.base == nullptr && mem.size != 0) throw GpuError("submit: null host-memory image", NICGPU_ERR_INVALID);
  Scratch& S = *scratch_;
  if (S.pending == Scratch::kSlots) throw std::logic_error("submit: three batches pending; collect() one first");
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  if (S.pending == 0) S.ensure(dev);
  else if (S.device != dev) throw std::logic_error("submit: batches pending on another device");
  for (unsigned k = 0; k < S.pending; ++k)
    if (S.slot[(S.head + k) % Scratch::kSlots].image != img)
      throw std::logic_error("submit: HostMemory and DeviceHostMemory batches (or two memories) pending together");
  Slot& sl = S.slot[(S.head + S.pending) % Scratch::kSlots];
  sl.image = nullptr;
  sl.staged = false;
  sl.multi = false;
  sl.overlap = false;
  sl.dep_stage.clear();
  sl.dep_rx.clear();
  if (img) image_prepare(sl, *img, tx, rx);  // dependencies on the batches pending now
  sl.stats = QueuePairStats{};
  sl.on_device = false;
  sl.mem = mem;
  sl.tx = tx;
  sl.rx = rx;
  sl.stream = stream;
  sl.tx_dev = d ? d->tx : nullptr;
  sl.rx_dev = d ? d->rx : nullptr;
  sl.ntx_dev = d ? d->ntx : 0;
  sl.nrx_dev = d ? d->nrx : 0;
  sl.fetched = false;
  // host_memory_faults (checked image batches): the host resolve asks the
  // memory for every write's verdict (submit set the slot's descriptors)
  const bool checked = img && config_.host_memory_faults;
  sl.wcheck = checked ? &sl.mem_writes : nullptr;
  const bool device = !checked && config_.device_resolve &&
                      (d ? device_fits(d->ntx, d->nrx) : device_fits(tx.size(), rx.size()));
  // host descriptors go up now, on this thread, beside the earlier batches'
  // device work (device descriptors are copied in the job, in stream order);
  // the rest runs in submission order on the job thread
  if (device && !d) upload(sl, tx, rx, false);
  // what the caller enqueued before this call (descriptors, frames): the
  // overlapped resolve waits for it, not for the earlier batches' DMA writes
  if (device) check(nicgpu_event_record(sl.ev_submit, stream), "nicgpu_event_record");
  sl.overlap = device && !img && config_.overlap_resolve;
  sl.rx_lo_w = 0;
  sl.rx_hi_w = ~0ull;
  if (S.pending == 0) S.n_recent = 0;  // every earlier batch collected: their writes are done
  // a host-image batch's TX bytes go up now, beside the earlier batches' work,
  // unless they overlap bytes an earlier pending batch delivers: then its job
  // stages them after that batch's write-back (recorded by the earlier job)
  sl.stage_deferred = img && !sl.dep_stage.empty();
  if (img && !sl.stage_deferred) image_stage(sl, tx.size(), tx.data(), device ? sl.v.tx : nullptr, stage_stream());
  sl.job_done = std::promise<void>();
  sl.job = sl.job_done.get_future();
  auto run = [this, &sl, device, dev] {
    try {
      check(nicgpu_set_device(dev), "nicgpu_set_device");  // the HIP device is per thread
      int disjoint = -1;
      double check_us = 0;
      if (sl.stage_deferred) {
        for (Slot* p : sl.dep_stage) check(nicgpu_stream_wait_event(stage_stream(), p->ev_wb), "nicgpu_stream_wait_event");
        image_stage(sl, sl.tx.size(), sl.tx.data(), device ? sl.v.tx : nullptr, stage_stream());
      }
      if (device) {
        sl.on_device = front(sl, sl.mem, sl.tx, sl.rx, sl.stats, sl.result, sl.stream, disjoint, check_us);
        if (sl.on_device) back(sl, sl.mem, sl.result, sl.stream);
      }
      if (!sl.on_device && sl.image) {
        image_host_path(sl, sl.tx, sl.rx, sl.stats, sl.result, sl.stream, disjoint, check_us);
      } else if (!sl.on_device) {
        rx_stage_detail::RingSlots rs;
        const bool rw = rings_written(sl, sl.mem, sl.stream, &rs);
        const auto [htx, hrx] = host_spans(sl, sl.tx, sl.rx, sl.stream);
        on_host(sl.mem, htx, hrx, sl.stats, sl.result, sl.stream, disjoint, check_us, nullptr, nullptr, rw ? &rs : nullptr);
      }
      sl.result.timings.check_us = check_us;
      // this batch's writes, for the overlapped resolves of the next two
      Scratch& SS = *scratch_;
      const Scratch::WriteBox box{sl.on_device ? sl.rx_lo_w : 0, sl.on_device ? sl.rx_hi_w : ~0ull};
      SS.recent[1] = SS.recent[0];
      SS.recent[0] = box;
      SS.n_recent = std::min(SS.n_recent + 1, 2u);
      sl.job_done.set_value();
    } catch (...) {
      Scratch& SS = *scratch_;  // writes unknown
      SS.recent[1] = SS.recent[0];
      SS.recent[0] = Scratch::WriteBox{};
      SS.n_recent = std::min(SS.n_recent + 1, 2u);
      sl.job_done.set_exception(std::current_exception());
    }
  };
  ++S.pending;
  S.inflight.fetch_add(1);
  S.jobs.push(run);  // interrupt callbacks fire in collect(), on the caller's thread
}

bool BatchedQueuePair::collect(RxBatchResult& out) {
  Scratch& S = *scratch_;
  if (S.pending == 0) return false;
  Slot& sl = S.slot[S.head];
  // the slot is free again whatever the batch throws
  S.head = (S.head + 1) % Scratch::kSlots;
  --S.pending;
  S.inflight.fetch_sub(1);
  try {
    sl.job.get();  // the job's exception, if any
  } catch (...) {
    try {
      sl.wait_writeback();
    } catch (...) {
    }
    throw;
  }
  if (sl.on_device) finish(sl, sl.result, &sl.stats);
  else sl.wait_writeback();  // a host-path batch of a HostMemory: its bytes are back
  rx_stage_detail::add_stats(stats_, sl.stats);
  std::swap(out, sl.result);
  if (config_.on_interrupt) fire_interrupts(out, &sl);
  return true;
}

// Completions still on the device (results_on_device) come from the slot's
// chunked page-locked copies (back()), the replay waiting for each chunk as it
// reaches it; without them they are fetched first.
void BatchedQueuePair::fire_interrupts(RxBatchResult& r, Slot* sl) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  struct Timed {
    RxBatchResult& r;
    clock::time_point t0;
    ~Timed() { r.timings.irq_us = std::chrono::duration<double, std::micro>(clock::now() - t0).count(); }
  } timed{r, t0};
  if (!r.timings.device || !config_.results_on_device) {
    rx_stage_detail::replay_interrupts(config_, r.tx_completions, r.rx_completions);
    return;
  }
  if (sl && sl->irq_pending && sl->irq_ntx == r.dev.ntx && sl->irq_nrx == r.dev.nrx) {
    sl->irq_pending = false;
    const std::size_t ptx = std::max<std::size_t>(1, (sl->irq_ntx + Slot::kIrqChunks - 1) / Slot::kIrqChunks);
    const std::size_t prx = std::max<std::size_t>(1, (sl->irq_nrx + Slot::kIrqChunks - 1) / Slot::kIrqChunks);
    double wait_us = 0;
    const CompletionEntry* itx = sl->h_itx.get<CompletionEntry>(1);
    const CompletionEntry* irx = sl->h_irx.get<CompletionEntry>(1);
    rx_stage_detail::replay_interrupts_chunked(
        config_, std::span<const CompletionEntry>(itx, sl->irq_ntx), std::span<const CompletionEntry>(irx, sl->irq_nrx),
        ptx, prx, [sl, &wait_us](int side, std::size_t c) {
          const auto w = clock::now();
          check(nicgpu_event_synchronize(sl->ev_irq[side][std::min<std::size_t>(c, Slot::kIrqChunks - 1)]),
                "nicgpu_event_synchronize");
          wait_us += std::chrono::duration<double, std::micro>(clock::now() - w).count();
        });
    r.timings.irq_wait_us = wait_us;
    return;
  }
  Scratch& S = *scratch_;
  S.irq_tx.resize(r.dev.ntx);
  S.irq_rx.resize(r.dev.nrx);
  if (r.dev.ntx)
    check(nicgpu_memcpy_async(S.irq_tx.data(), r.dev.tx_completions, r.dev.ntx * sizeof(CompletionEntry), nullptr),
          "nicgpu_memcpy_async");
  if (r.dev.nrx)
    check(nicgpu_memcpy_async(S.irq_rx.data(), r.dev.rx_completions, r.dev.nrx * sizeof(CompletionEntry), nullptr),
          "nicgpu_memcpy_async");
  check(nicgpu_stream_synchronize(nullptr), "nicgpu_stream_synchronize");
  rx_stage_detail::replay_interrupts(config_, S.irq_tx, S.irq_rx);
}

std::size_t BatchedQueuePair::pending() const noexcept { return scratch_->pending; }

// The descriptors up on the upload stream, so they need not wait behind
// earlier batches' DMA writes and RSS on the caller's stream: TX first, alone
// on the link, then RX — issued from the helper thread when `rx_beside`, so
// the plan and piece sums (TX descriptors only) run while it goes up.
// (Descriptor arrays in page-locked memory upload without staging and without
// holding the issuing thread.)
void BatchedQueuePair::upload(Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                              bool rx_beside) {
  using clock = std::chrono::steady_clock;
  const auto t = clock::now();
  Scratch& S = *scratch_;
  const std::size_t ntx = tx.size(), nrx = rx.size();
  nicgpu_qp_view& v = sl.v;
  check(nicgpu_qp_reserve(sl.qp, ntx, nrx, &v), "nicgpu_qp_reserve");
  check(nicgpu_memcpy_async(v.tx, tx.data(), ntx * sizeof(TxDescriptor), S.side_up), "nicgpu_memcpy_async");
  check(nicgpu_event_record(sl.ev_tx, S.side_up), "nicgpu_event_record");
  if (rx_beside) {
    sl.up.emplace(S.up_worker);
    sl.up->start([&sl, &S, &v, rx](SideJob& j) {
      j.ok(nicgpu_set_device(S.device), "nicgpu_set_device") &&
          j.ok(nicgpu_memcpy_async(v.rx, rx.data(), rx.size() * sizeof(RxDescriptor), S.side_up),
               "nicgpu_memcpy_async") &&
          j.ok(nicgpu_event_record(sl.ev_rx, S.side_up), "nicgpu_event_record");
    });
  } else {
    check(nicgpu_memcpy_async(v.rx, rx.data(), nrx * sizeof(RxDescriptor), S.side_up), "nicgpu_memcpy_async");
    check(nicgpu_event_record(sl.ev_rx, S.side_up), "nicgpu_event_record");
  }
  sl.upload_us = std::chrono::duration<double, std::micro>(clock::now() - t).count();
}

// Disjoint buffers, no interrupt callback: plan, piece sums and the
// reference's control flow on the device (nicgpu_qp_*), the part after a
// descriptor whose RX side ends it early (or where the ring runs short)
// resolved here in order.  The host moves descriptors up; back() and finish()
// do the rest.
// A plan that outgrew the piece buffers (NICGPU_ERR_AGAIN: nothing resolved,
// settled or written) is redone once with the buffers it asked for; a second
// AGAIN would mean the sizing is broken, and is an error.
bool BatchedQueuePair::front(Slot& sl, const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                             std::span<const RxDescriptor> rx, QueuePairStats& st, RxBatchResult& out, void* stream,
                             int& disjoint, double& check_us) {
  for (int attempt = 0;; ++attempt) {
    int again = 0;
    const bool r = front_once(sl, mem, tx, rx, st, out, stream, disjoint, check_us, again);
    if (!again) {
      out.timings.replans = static_cast<unsigned>(attempt);
      return r;
    }
    if (attempt >= 1)
      throw GpuError("process_batch: the device plan outgrew its piece buffers twice", NICGPU_ERR_AGAIN);
  }
}

bool BatchedQueuePair::front_once(Slot& sl, const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                                  std::span<const RxDescriptor> rx, QueuePairStats& st, RxBatchResult& out,
                                  void* stream, int& disjoint, double& check_us, int& again) {
  using namespace rx_stage_detail;
  using clock = std::chrono::steady_clock;
  auto us_since = [](clock::time_point t) { return std::chrono::duration<double, std::micro>(clock::now() - t).count(); };
  Scratch& S = *scratch_;
  out.tx_processed = out.rx_consumed = 0;
  for (auto& q : out.queues) q.clear();
  out.queues.clear();
  out.timings = RxBatchResult::Timings{};
  out.timings.device = true;
  out.dev = RxBatchResult::DeviceResults{};
  const bool dev_desc = sl.tx_dev || sl.rx_dev;
  const std::size_t ntx = dev_desc ? sl.ntx_dev : tx.size(), nrx = dev_desc ? sl.nrx_dev : rx.size();
  nicgpu_qp_view& v = sl.v;
  auto t = clock::now();
  // The plan and the overlap check read descriptors only, so they run on the
  // side stream `ps` — beside the earlier batches' DMA writes and RSS still on
  // `stream` — unless the descriptors are device arrays inside the image
  // (those writes may change them: copied in stream order).  The piece sums
  // read the image and stay on `stream`.
  auto inside = [&](const void* p, std::size_t bytes) {
    const auto a = reinterpret_cast<std::uintptr_t>(p), b = reinterpret_cast<std::uintptr_t>(mem.base);
    return bytes && a < b + mem.size && b < a + bytes;
  };
  const bool side = !dev_desc || (!inside(sl.tx_dev, ntx * sizeof(TxDescriptor)) &&
                                  !inside(sl.rx_dev, nrx * sizeof(RxDescriptor)));
  // descriptor arrays in the image that a write of the batch lands on: the
  // host path, which pops them as the reference does (nothing written yet)
  if (!side && rings_written(sl, mem, stream, nullptr)) return false;
  void* ps = side ? S.side_plan : stream;
  if (dev_desc) {
    check(nicgpu_qp_reserve(sl.qp, ntx, nrx, &v), "nicgpu_qp_reserve");
    if (side) {
      // read in place (outside the image, so no write of the batch changes
      // them), after whatever the caller enqueued on `stream` before handing
      // them over — no copy to compete with the earlier batch's DMA writes
      check(nicgpu_stream_wait_event(ps, sl.ev_submit), "nicgpu_stream_wait_event");
      check(nicgpu_qp_bind(sl.qp, reinterpret_cast<const nicgpu_tx_descriptor*>(sl.tx_dev), ntx,
                           reinterpret_cast<const nicgpu_rx_descriptor*>(sl.rx_dev), nrx, &v),
            "nicgpu_qp_bind");
    } else {  // inside the image: copied in stream order, before this batch writes
      if (ntx) check(nicgpu_memcpy_async(v.tx, sl.tx_dev, ntx * sizeof(TxDescriptor), ps), "nicgpu_memcpy_async");
      if (nrx) check(nicgpu_memcpy_async(v.rx, sl.rx_dev, nrx * sizeof(RxDescriptor), ps), "nicgpu_memcpy_async");
    }
  } else {
    out.timings.copy_us += sl.upload_us;
    sl.upload_us = 0;  // counted once, also when the plan is redone
    check(nicgpu_stream_wait_event(ps, sl.ev_tx), "nicgpu_stream_wait_event");
  }
  // a host-image batch: the piece sums read the TX bytes staged into the mirror
  out.timings.host_image = sl.image != nullptr;
  out.timings.staged_whole = sl.image != nullptr && sl.whole;
  if (sl.staged) check(nicgpu_stream_wait_event(stream, sl.ev_staged), "nicgpu_stream_wait_event");
  // Overlapped resolve (submit/collect): the piece sums and the resolve on the
  // resolve stream `rs`, after what the caller enqueued before submit, beside
  // the earlier batches' DMA writes still on `stream`; the overlap check's
  // bounds then tell whether this batch's frames lie where those write (then
  // both are redone behind them).  The DMA writes stay on `stream`, in order.
  const bool ov = sl.overlap && side && sl.image == nullptr;
  void* rs = ov ? S.side_res : stream;
  if (ov) check(nicgpu_stream_wait_event(rs, sl.ev_submit), "nicgpu_stream_wait_event");
  // the plan and the piece sums enqueued without a wait: the piece buffers are
  // sized ahead (ntx + ntx / 4 pieces, or what an earlier batch needed); a
  // plan that does not fit them, or a descriptor planning more pieces than
  // 32-bit piece indices allow, makes the resolve settle nothing and its
  // finish return NICGPU_ERR_RANGE — that batch then takes the host path
  // (which refuses it if its total does not fit either), the next one fits
  check(nicgpu_qp_set_deferred_verify(sl.qp, config_.defer_rx_verify && defer_env() ? 1 : 0),
        "nicgpu_qp_set_deferred_verify");
  check(nicgpu_qp_plan_async(sl.qp, reinterpret_cast<const std::uint8_t*>(mem.base), mem.size, ntx, config_.max_mtu,
                             &v, ps, rs),
        "nicgpu_qp_plan_async");
  out.timings.sums_us += us_since(t);
  t = clock::now();
  if (sl.up) {
    sl.up->finish();
    sl.up.reset();
  }
  if (!dev_desc) {
    check(nicgpu_stream_wait_event(ps, sl.ev_rx), "nicgpu_stream_wait_event");
    if (side) check(nicgpu_stream_wait_event(rs, sl.ev_rx), "nicgpu_stream_wait_event");
  }
  out.timings.copy_us += us_since(t);
  // (NIC_CHECK_EARLY=1) the overlap check on its own normal-priority stream as
  // soon as the descriptors are in place — beside the earlier batch's
  // delivery — instead of behind the plan on the least-priority stream, where
  // it waits for wave slots until the resolve is over
  const bool early = side && check_early_env() && S.inflight.load() <= 1;
  if (early) {
    if (dev_desc) check(nicgpu_stream_wait_event(S.side_chk, sl.ev_submit), "nicgpu_stream_wait_event");
    else {
      check(nicgpu_stream_wait_event(S.side_chk, sl.ev_tx), "nicgpu_stream_wait_event");
      check(nicgpu_stream_wait_event(S.side_chk, sl.ev_rx), "nicgpu_stream_wait_event");
    }
    check(nicgpu_qp_check_async(sl.qp, mem.size, ntx, nrx, 0u, S.side_chk), "nicgpu_qp_check_async");
  }
  // the speculative resolve goes in behind the piece sums before the overlap
  // check's verdict (it writes only the context's completions and writes),
  // so the stream does not wait for this thread's round trip on the check.
  // For an overlapping or unsorted batch that pass (need/scan/full/reduce and
  // its small download) is wasted GPU time: the host path then redoes the
  // batch, and the context's resolve state stays set until the next start.
  // Results are unaffected; disjoint rings are the common case.
  t = clock::now();
  check(nicgpu_qp_resolve_start(sl.qp, mem.size, ntx, nrx, config_.max_mtu, config_.queue_id, rs),
        "nicgpu_qp_resolve_start");
  check(nicgpu_event_record(sl.ev_resolved, rs), "nicgpu_event_record");  // final unless relaxed / tail below
  out.timings.resolve_us += us_since(t);
  // overlapping buffers go to the host path before anything is written; a
  // ring whose RX buffers are not in ascending address order is sorted there.
  // The check synchronises `ps`: the descriptors are then in place for `stream`.
  t = clock::now();
  int verdict = -1;
  if (early) check(nicgpu_qp_check_wait(sl.qp, &verdict), "nicgpu_qp_check_wait");
  else check(nicgpu_qp_check(sl.qp, mem.size, ntx, nrx, &verdict, ps), "nicgpu_qp_check");
  const bool ascending = verdict >= 0;  // the device decided: RX spans in address order
  if (verdict < 0) {
    const auto [htx, hrx] = host_spans(sl, tx, rx, stream);
    verdict = buffers_disjoint(mem.size, htx, hrx) ? 1 : 0;
  }
  disjoint = verdict;
  check_us += us_since(t);
  if (ov) {
    // the overlapped pass must be over before anything else touches this
    // context's buffers, whatever happens next (the host path included)
    check(nicgpu_stream_wait_event(stream, sl.ev_resolved), "nicgpu_stream_wait_event");
  }
  if (!disjoint) return false;
  if (ov) {
    std::uint64_t bnd[4];
    check(nicgpu_qp_check_bounds(sl.qp, bnd), "nicgpu_qp_check_bounds");
    // this batch's writes stay inside its RX spans (ascending: the first
    // span's start is their least; unsorted rings: unknown)
    sl.rx_lo_w = !ascending ? 0 : bnd[3] > bnd[2] ? bnd[2] : 0;
    sl.rx_hi_w = !ascending ? ~0ull : bnd[3] > bnd[2] ? bnd[3] : 0;
    bool hazard = false;
    if (bnd[1] > bnd[0])  // frames to read: do the earlier batches' writes reach them?
      for (unsigned k = 0; k < S.n_recent; ++k) hazard |= S.recent[k].hi > bnd[0] && bnd[1] > S.recent[k].lo;
    out.timings.overlapped = true;
    ++S.overlaps;
    if (hazard) {
      // redo the sums and the resolve behind everything `stream` holds now
      // (the earlier batches' DMA writes included)
      out.timings.overlap_redone = true;
      ++S.overlaps_redone;
      check(nicgpu_event_record(sl.ev_gate, stream), "nicgpu_event_record");
      check(nicgpu_stream_wait_event(rs, sl.ev_gate), "nicgpu_stream_wait_event");
      check(nicgpu_qp_resum(sl.qp, reinterpret_cast<const std::uint8_t*>(mem.base), mem.size, rs), "nicgpu_qp_resum");
      check(nicgpu_qp_resolve_start(sl.qp, mem.size, ntx, nrx, config_.max_mtu, config_.queue_id, rs),
            "nicgpu_qp_resolve_start");
      check(nicgpu_event_record(sl.ev_resolved, rs), "nicgpu_event_record");
      check(nicgpu_stream_wait_event(stream, sl.ev_resolved), "nicgpu_stream_wait_event");
    }
  }
  t = clock::now();
  // the DMA writes and RSS of the completions the resolve settles (bounded on
  // the device) go in at once: the host waits for the resolve while they are
  // already queued, so the stream does not idle on this thread's round trip
  sl.tn = sl.nq = 0;
  const nicgpu_rss_ctx* rctx = nullptr;
  std::uint64_t* hits = nullptr;
  if (config_.rss != nullptr) {
    if (config_.tuple.mode == TupleMode::None)
      throw GpuError("process_batch: TupleMode::None cannot produce hashes", NICGPU_ERR_INVALID);
    const auto& table = config_.rss->config().table;
    sl.tn = table.size();
    for (const std::uint16_t q : table) sl.nq = std::max<std::size_t>(sl.nq, std::size_t{q} + 1);
    rctx = config_.rss->device_context(stream);
    hits = static_cast<std::uint64_t*>(sl.hits.get(std::max<std::size_t>(sl.tn, 1) * sizeof(std::uint64_t)));
  }
  out.timings.resolve_us += us_since(t);
  t = clock::now();
  // host image: the delivery rewrites RX bytes an earlier pending batch may
  // still be writing back from the mirror
  for (Slot* p : sl.dep_rx) check(nicgpu_stream_wait_event(stream, p->ev_wb), "nicgpu_stream_wait_event");
  deliver(sl, mem, 0, nrx, NICGPU_DELIVER_SETTLED | NICGPU_DELIVER_RESET_HITS, rctx, hits, stream);  // hits set, not added
  out.timings.gather_us += us_since(t);
  t = clock::now();
  std::uint64_t done = 0, used = 0, settled = 0;
  nicgpu_qp_stats ds{};
  std::uint64_t walks0 = 0, walks1 = 0;
  check(nicgpu_qp_walks(sl.qp, &walks0), "nicgpu_qp_walks");
  const int rst = nicgpu_qp_resolve_finish(sl.qp, &done, &used, &settled, &ds);
  check(nicgpu_qp_walks(sl.qp, &walks1), "nicgpu_qp_walks");
  out.timings.walked = out.timings.walked || walks1 != walks0;
  if (rst == NICGPU_ERR_AGAIN || rst == NICGPU_ERR_RANGE) {  // the plan did not fit: nothing resolved, settled or written
    out.timings.resolve_us += us_since(t);
    if (rst == NICGPU_ERR_RANGE) return false;
    again = 1;  // grown buffers: the redone plan fits
    return false;
  }
  check(rst, "nicgpu_qp_resolve_finish");
  int late = 0;
  check(nicgpu_qp_deferred(sl.qp, &late), "nicgpu_qp_deferred");
  sl.late = late != 0;
  out.timings.deferred = sl.late;
  if (ov) {  // the relaxation's rewrites (on rs) before the rest of this batch's work on `stream`
    check(nicgpu_event_record(sl.ev_resolved, rs), "nicgpu_event_record");
    check(nicgpu_stream_wait_event(stream, sl.ev_resolved), "nicgpu_stream_wait_event");
  }
  sl.settled = settled;
  sl.relaxed = done < ntx || settled < used;  // completions rewritten after ev_resolved
  out.timings.resolve_us += us_since(t);
  t = clock::now();
  const QueuePairStats d{ds.tx_packets,         ds.rx_packets,         ds.tx_bytes,
                         ds.rx_bytes,           ds.drops_checksum,     ds.drops_no_rx_desc,
                         ds.drops_buffer_small, ds.drops_mtu_exceeded, ds.drops_invalid_mss,
                         ds.drops_too_many_segments, ds.tx_tso_segments, ds.tx_gso_segments,
                         ds.tx_vlan_insertions, ds.rx_vlan_strips,     ds.rx_checksum_verified,
                         ds.rx_gro_aggregated};
  add_stats(st, d);
  std::size_t nrx_total = used;
  out.rx_consumed = used;
  if (config_.results_on_device) out.tx_completions.clear();
  else out.tx_completions.resize(ntx);
  if (done < ntx) {
    out.timings.host_tail = true;
    // the rest, in order, from ring position `used` (the host resolve; its
    // plan of tx[done..] lists the same pieces as the device's from piece_base[done])
    const auto [htx, hrx] = host_spans(sl, tx, rx, stream);
    const auto tail_tx = htx.subspan(done);
    const auto tail_rx = hrx.subspan(used);
    make_plan(config_, mem.size, tail_tx, S.host.plan, /*split4=*/true);
    std::uint32_t pb = 0;
    std::uint64_t np = 0;
    check(nicgpu_qp_piece_count(sl.qp, &np), "nicgpu_qp_piece_count");
    check(nicgpu_memcpy_async(&pb, v.piece_base + done, sizeof(pb), stream), "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");
    if (np - pb != S.host.plan.pieces.size()) throw GpuError("process_batch: device and host plans differ", NICGPU_ERR_INVALID);
    // a batch that deferred its RX verifies skipped the piece sums
    if (sl.late)
      check(nicgpu_qp_resum(sl.qp, reinterpret_cast<const std::uint8_t*>(mem.base), mem.size, stream), "nicgpu_qp_resum");
    // the device's split sums of those pieces: rests, then first-4 parts
    const std::size_t m = np - pb;
    S.tail_cs.resize(2 * m);
    check(nicgpu_memcpy_async(S.tail_cs.data(), v.piece_csum + pb, m * 2, stream), "nicgpu_memcpy_async");
    check(nicgpu_memcpy_async(S.tail_cs.data() + m, v.piece_cs4 + pb, m * 2, stream), "nicgpu_memcpy_async");
    check(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");
    RxBatchResult& part = S.host.part;
    resolve(quiet_, mem.size, S.host.plan, S.tail_cs, tail_tx, tail_rx, st, part, S.host.writes, S.host.write_of_rx);
    const std::size_t tr = part.rx_completions.size();
    check(nicgpu_memcpy_async(v.txc + done, part.tx_completions.data(), part.tx_completions.size() * sizeof(CompletionEntry),
                              stream),
          "nicgpu_memcpy_async");
    check(nicgpu_memcpy_async(v.rxc + used, part.rx_completions.data(), tr * sizeof(CompletionEntry), stream),
          "nicgpu_memcpy_async");
    check(nicgpu_memcpy_async(v.writes + used, S.host.writes.data(), tr * sizeof(SegmentWrite), stream),
          "nicgpu_memcpy_async");
    nrx_total += tr;
    out.rx_consumed += part.rx_consumed;
  }
  out.tx_processed = ntx;
  out.timings.resolve_us += us_since(t);
  sl.ntx = ntx;
  sl.nrx_total = nrx_total;
  return true;
}

// Everything here is enqueued without waiting.  The completions are final:
// they go down on the side stream at once, while this thread enqueues the DMA
// writes and the RSS list, launch, scatter and dispatch lists (their sizes
// read on the device); the RSS results follow them down.
// The DMA writes and RSS of completions [a, b) (NICGPU_DELIVER_SETTLED: b
// lowered on the device to the pending resolve's settled prefix).
void BatchedQueuePair::deliver(Slot& sl, const DeviceHostMemory& mem, std::size_t a, std::size_t b, unsigned flags,
                               const nicgpu_rss_ctx* rctx, std::uint64_t* hits, void* stream) {
  // a later batch already submitted plans and checks beside this delivery:
  // CUs left to it (f1 C3 1 M pipelined 371 -> 353 us with 32; one batch at a
  // time is fastest with none, profiles/r05_dlv_reserve.txt, r05_dlv_reserve_ab.txt)
  static const int pipe_reserve = [] {
    const char* e = std::getenv("NIC_DLV_RESERVE_PIPE");
    return e ? std::atoi(e) : 32;
  }();
  check(nicgpu_qp_set_delivery_reserve(sl.qp, scratch_->inflight.load() > 1 ? pipe_reserve : -1),
        "nicgpu_qp_set_delivery_reserve");
  check(nicgpu_qp_deliver_range(sl.qp, reinterpret_cast<std::uint8_t*>(mem.base), mem.size, a, b, flags, rctx,
                                rctx ? static_cast<int>(config_.tuple.mode) : NICGPU_TUPLE_NONE, config_.tuple.raw_offset,
                                config_.tuple.raw_length, rctx ? hits : nullptr, stream),
        "nicgpu_qp_deliver_range");
}

void BatchedQueuePair::back(Slot& sl, const DeviceHostMemory& mem, RxBatchResult& out, void* stream) {
  using clock = std::chrono::steady_clock;
  auto us_since = [](clock::time_point t) { return std::chrono::duration<double, std::micro>(clock::now() - t).count(); };
  Scratch& S = *scratch_;
  const nicgpu_qp_view& v = sl.v;
  const std::size_t ntx = sl.ntx, nrx_total = sl.nrx_total;
  auto t = clock::now();
  sl.rss = config_.rss != nullptr && nrx_total != 0;
  if (!sl.rss) sl.tn = sl.nq = 0;
  const std::size_t tn = sl.tn, nq = sl.nq;
  const bool rss = sl.rss;
  const bool keep = config_.results_on_device;  // results stay in the slot's device buffers
  if (keep) {
    out.rx_completions.clear();
    out.rx_hash.clear();
    out.rx_queue.clear();
    RxBatchResult::DeviceResults& d = out.dev;
    d.tx_completions = reinterpret_cast<const CompletionEntry*>(v.txc);
    d.rx_completions = reinterpret_cast<const CompletionEntry*>(v.rxc);
    d.ntx = ntx;
    d.nrx = nrx_total;
    d.rx_hash = rss ? v.rx_hash : nullptr;
    d.rx_queue = rss ? v.rx_queue : nullptr;
    d.queue_which = rss ? v.queue_which : nullptr;
  } else {
    out.rx_completions.resize(nrx_total);
    out.rx_hash.resize(nrx_total);
    out.rx_queue.resize(nrx_total);
  }
  // pinned landing space: [count][hits tn] u64, then [start nq][end nq][which nrx] u32
  sl.meta = sl.h_meta.get<std::uint64_t>(1 + tn);
  sl.qs = sl.h_lists.get<std::uint32_t>(2 * nq + nrx_total + 1);
  sl.qe = sl.qs + nq;
  sl.which = sl.qe + nq;
  sl.meta[0] = 0;
  std::uint64_t* hits = config_.rss ? static_cast<std::uint64_t*>(sl.hits.get(std::max<std::size_t>(sl.tn, 1) * 8)) : nullptr;
  sl.rss_recorded = std::promise<void>();
  sl.rss_released = false;
  std::shared_future<void> rss_ready = sl.rss_recorded.get_future().share();
  if (sl.relaxed) check(nicgpu_event_record(sl.ev_resolved, stream), "nicgpu_event_record");
  sl.irq_pending = false;
  const bool irq_down =
      keep && config_.on_interrupt && (config_.enable_tx_interrupts || config_.enable_rx_interrupts) && !sl.multi;
  // the completions for the callbacks, in chunks, page-locked, as soon as they
  // are final (ev_resolved; a deferred-verify batch's after its deliveries,
  // ev_done): collect() replays chunk c while chunk c + 1 lands
  auto irq_download = [&](void* final_ev) {
    check(nicgpu_stream_wait_event(S.side_irq, final_ev), "nicgpu_stream_wait_event");
    const std::size_t n2[2] = {ntx, nrx_total};
    CompletionEntry* dst[2] = {sl.h_itx.get<CompletionEntry>(std::max<std::size_t>(ntx, 1)),
                               sl.h_irx.get<CompletionEntry>(std::max<std::size_t>(nrx_total, 1))};
    const nicgpu_completion* src[2] = {v.txc, v.rxc};
    for (int side = 0; side < 2; ++side) {
      const std::size_t per = std::max<std::size_t>(1, (n2[side] + Slot::kIrqChunks - 1) / Slot::kIrqChunks);
      for (int c = 0; c < Slot::kIrqChunks; ++c) {
        const std::size_t a = std::min(n2[side], c * per), b = std::min(n2[side], a + per);
        if (b > a)
          check(nicgpu_memcpy_async(dst[side] + a, src[side] + a, (b - a) * sizeof(CompletionEntry), S.side_irq),
                "nicgpu_memcpy_async");
        check(nicgpu_event_record(sl.ev_irq[side][c], S.side_irq), "nicgpu_event_record");
      }
    }
    sl.irq_ntx = ntx;
    sl.irq_nrx = nrx_total;
    sl.irq_pending = true;
  };
  if (irq_down && !sl.late) irq_download(sl.ev_resolved);
  sl.down.emplace(sl.worker);
  // the dispatch lists are made here too, on the download stream: they read
  // this slot's buffers only, so the next batch's piece sums need not queue
  // behind them on `stream`
  sl.down->start([&sl, &S, &out, &v, ntx, nrx_total, tn, nq, rss, keep, hits, rss_ready](SideJob& j) {
    bool ok = j.ok(nicgpu_set_device(S.device), "nicgpu_set_device") &&
              j.ok(nicgpu_stream_wait_event(S.side_down, sl.ev_resolved), "nicgpu_stream_wait_event");
    auto completions_down = [&] {
      ok = j.ok(nicgpu_memcpy_async(out.tx_completions.data(), v.txc, ntx * sizeof(CompletionEntry), S.side_down),
                "nicgpu_memcpy_async") &&
           j.ok(nicgpu_memcpy_async(out.rx_completions.data(), v.rxc, nrx_total * sizeof(CompletionEntry), S.side_down),
                "nicgpu_memcpy_async");
    };
    if (ok && !keep && !sl.late) completions_down();
    rss_ready.wait();
    ok = ok && j.ok(nicgpu_stream_wait_event(S.side_down, sl.ev_done), "nicgpu_stream_wait_event");
    // a deferred-verify batch: its completions are final now, and its
    // statistics' corrections come down with them
    if (ok && !keep && sl.late) completions_down();
    if (ok && sl.late) {
      const std::size_t ns = sl.multi ? sl.nseg : 1;
      ok = j.ok(nicgpu_qp_verify_fixups_async(sl.qp, sl.h_fix.get<std::uint64_t>(ns * NICGPU_QP_FIXUPS), ns, S.side_down),
                "nicgpu_qp_verify_fixups_async");
    }
    // a fused batch: the lists split per queue pair (entries made relative to
    // each queue pair's ring), and its per-queue-pair hits when it needs them
    // (its per-queue-pair hits beside the lists, on the interrupt stream, which
    // a fused batch does not use)
    const bool seg_hits = ok && rss && sl.multi && sl.seg_hits_on;
    if (seg_hits) {
      auto* sh = static_cast<std::uint64_t*>(sl.seg_hits.get(sl.nseg * tn * sizeof(std::uint64_t)));
      ok = j.ok(nicgpu_stream_wait_event(S.side_irq, sl.ev_done), "nicgpu_stream_wait_event") &&
           j.ok(nicgpu_qp_segment_hits(sl.qp, nrx_total, tn, sh, S.side_irq), "nicgpu_qp_segment_hits") &&
           j.ok(nicgpu_memcpy_async(sl.h_seg_hits.get<std::uint64_t>(sl.nseg * tn), sh, sl.nseg * tn * 8, S.side_irq),
                "nicgpu_memcpy_async");
    }
    if (ok && rss)
      ok = j.ok(nicgpu_qp_group(sl.qp, nrx_total, nq, S.side_down), "nicgpu_qp_group");
    if (ok && rss && sl.multi)
      ok = j.ok(nicgpu_qp_segment_lists(sl.qp, nrx_total, nq, sl.h_split.get<std::uint32_t>((sl.nseg + 1) * std::max<std::size_t>(nq, 1)),
                                        S.side_down),
                "nicgpu_qp_segment_lists");
    if (seg_hits) ok = j.ok(nicgpu_stream_synchronize(S.side_irq), "nicgpu_stream_synchronize") && ok;
    // (a fused batch's lists are the split's, so no list bounds; its totals
    // only for one shared engine or for the dispatch list's download)
    if (ok && rss && !(sl.multi && keep && sl.seg_hits_on))
      ok = j.ok(nicgpu_memcpy_async(sl.meta, v.rss_count, sizeof(std::uint64_t), S.side_down), "nicgpu_memcpy_async") &&
           j.ok(nicgpu_memcpy_async(sl.meta + 1, hits, tn * sizeof(std::uint64_t), S.side_down), "nicgpu_memcpy_async");
    if (ok && rss && !sl.multi)
      ok = j.ok(nicgpu_memcpy_async(sl.qs, v.queue_start, nq * 4, S.side_down), "nicgpu_memcpy_async") &&
           j.ok(nicgpu_memcpy_async(sl.qe, v.queue_end, nq * 4, S.side_down), "nicgpu_memcpy_async");
    if (ok && rss && !keep)
      ok = j.ok(nicgpu_memcpy_async(out.rx_hash.data(), v.rx_hash, nrx_total * 4, S.side_down), "nicgpu_memcpy_async") &&
           j.ok(nicgpu_memcpy_async(out.rx_queue.data(), v.rx_queue, nrx_total * 2, S.side_down), "nicgpu_memcpy_async") &&
           j.ok(nicgpu_stream_synchronize(S.side_down), "nicgpu_stream_synchronize") &&
           j.ok(nicgpu_memcpy_async(sl.which, v.queue_which, sl.meta[0] * 4, S.side_down), "nicgpu_memcpy_async");
    // (with the results kept on the device this is where the batch is known done)
    ok = ok && j.ok(nicgpu_stream_synchronize(S.side_down), "nicgpu_stream_synchronize");
  });
  try {
    out.timings.copy_us += us_since(t);
    t = clock::now();
    // the rest of the DMA writes and RSS (the settled prefix went in with the
    // resolve), one launch: the headers hashed from the bytes the writes move
    if (sl.settled < nrx_total)
      deliver(sl, mem, sl.settled, nrx_total, NICGPU_DELIVER_APPEND,
              config_.rss ? config_.rss->device_context(stream) : nullptr, hits, stream);
    out.timings.gather_us += us_since(t);
    t = clock::now();
    check(nicgpu_event_record(sl.ev_done, stream), "nicgpu_event_record");
    if (irq_down && sl.late) irq_download(sl.ev_done);
    if (sl.image) {  // the delivered bytes back into the host memory, beside the next batches' work
      check(nicgpu_stream_wait_event(S.side_wb, sl.ev_done), "nicgpu_stream_wait_event");
      image_writeback(sl, v.writes, nrx_total, S.side_wb);
    }
  } catch (...) {
    sl.wait();  // the downloads must not outlive this batch's buffers
    throw;
  }
  sl.release_rss();
  out.timings.rss_us += us_since(t);
  if (!rss && !keep) {
    std::fill(out.rx_hash.begin(), out.rx_hash.end(), 0u);
    std::fill(out.rx_queue.begin(), out.rx_queue.end(), RxBatchResult::kNoQueue);
  }
}

// The deferred verifies of segment s that failed in the batch just finished:
// its statistics took them as delivered (queue_pair.cpp:434-447 counts a drop
// instead, and neither the RX nor the finalized TX counters).
void BatchedQueuePair::apply_fixups(Slot& sl, std::size_t s, QueuePairStats& st) {
  const std::uint64_t failed = sl.fix_delta(s, 0);
  st.drops_checksum += failed;
  st.rx_packets -= failed;
  st.tx_packets -= failed;
  st.rx_bytes -= sl.fix_delta(s, 1);
  st.rx_vlan_strips -= sl.fix_delta(s, 2);
  st.tx_bytes -= sl.fix_delta(s, 3);
  st.tx_vlan_insertions -= sl.fix_delta(s, 4);
}

// The downloads waited for everything the batch did on the caller's stream,
// so the image holds its writes once they are done.
void BatchedQueuePair::finish(Slot& sl, RxBatchResult& out, QueuePairStats* st) {
  using clock = std::chrono::steady_clock;
  const auto t = clock::now();
  struct Reset {  // the slot's job is over whatever finish() throws
    Slot& sl;
    ~Reset() { sl.down.reset(); }
  } reset{sl};
  sl.down->finish();
  sl.wait_writeback();
  if (sl.late && !sl.multi) {  // (a fused batch's, per queue pair, are process_queues')
    if (!st) throw std::logic_error("finish: a deferred-verify batch without its statistics");
    apply_fixups(sl, 0, *st);
  }
  if (sl.rss && !sl.multi) {  // (a fused batch's accounting and lists are process_queues')
    const std::uint64_t m = sl.meta[0];
    config_.rss->account_batch(m, std::span<const std::uint64_t>(sl.meta + 1, sl.tn));
    std::size_t used_q = 0;  // largest queue with frames + 1
    for (std::size_t q = 0; q < sl.nq; ++q)
      if (sl.qe[q] > sl.qs[q]) used_q = q + 1;
    if (config_.results_on_device) {
      out.dev.queue_start.assign(sl.qs, sl.qs + used_q);
      out.dev.queue_end.assign(sl.qe, sl.qe + used_q);
    } else {
      out.queues.resize(used_q);
      for (std::size_t q = 0; q < used_q; ++q) out.queues[q].assign(sl.which + sl.qs[q], sl.which + sl.qe[q]);
    }
  }
  out.timings.copy_us += std::chrono::duration<double, std::micro>(clock::now() - t).count();
}

// ------------------------------------------------------------------------
// The stage on the reference's HostMemory (host_memory.h:49-73): an HBM mirror
// of its flat window.  Per batch the TX buffers' bytes go up (QueuePair's DMA
// read, queue_pair.cpp:86-92), the stage runs on the mirror, and the bytes its
// DMA writes delivered (:416-426) come back — nothing else of the memory is
// read or written by the device.

BatchedQueuePair::HostImage& BatchedQueuePair::bind_image(HostMemory& m, bool checked, std::byte* window) {
  Scratch& S = *scratch_;
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  const std::size_t size = m.config().size_bytes;
  std::byte* host = nullptr;
  if (checked) {
    // host_memory_faults: the window the batch's allowed reads showed, else the
    // whole memory's translation when it is allowed; none when every access
    // so far is refused (then no byte is read, and none written)
    host = window;
    if (!host && size) {
      HostMemoryView v{};
      if (m.translate(0, size, v).ok() && v.address == 0 && v.length == size) host = v.data;
    }
    HostImage& I = *S.img;
    if (!host && I.mem == &m && I.size == size && I.device == dev) return I;  // keep the known window
    if (reinterpret_cast<std::uintptr_t>(host) & 15u)
      throw GpuError("process_batch: HostMemory window is not 16-B aligned", NICGPU_ERR_INVALID);
  } else if (size) {
    HostMemoryView v{};
    const HostMemoryResult r = m.translate(0, size, v);
    if (!r.ok() || v.data == nullptr || v.length != size)
      throw GpuError("process_batch: HostMemory::translate(0, size) is not a view of the whole memory (an address "
                     "translator or fault injector is not modelled)",
                     NICGPU_ERR_INVALID);
    host = v.data;
    // flat: the last and a middle byte translate where the window puts them
    for (const HostAddress a : {static_cast<HostAddress>(size - 1), static_cast<HostAddress>(size / 2)}) {
      HostMemoryView p{};
      if (!m.translate(a, 1, p).ok() || p.data != host + a)
        throw GpuError("process_batch: HostMemory window is not flat (address translation is not modelled)",
                       NICGPU_ERR_INVALID);
    }
    if (reinterpret_cast<std::uintptr_t>(host) & 15u)
      throw GpuError("process_batch: HostMemory window is not 16-B aligned", NICGPU_ERR_INVALID);
  }
  HostImage& I = *S.img;
  if (I.mem == &m && I.host == host && I.size == size && I.device == dev) return I;
  if (S.pending) throw std::logic_error("submit: another HostMemory while batches are pending");
  I.release();
  I.mem = &m;
  I.host = host;
  I.size = size;
  I.device = dev;
  if (size) {
    if (host) {
      void* alias = nullptr;
      int owned = 0;
      check(nicgpu_host_register(host, size, &alias, &owned), "nicgpu_host_register");
      I.alias = static_cast<std::uint8_t*>(alias);
      I.owned = owned != 0;
    }
    I.mirror[0].get((size + 15) / 16 * 16);
  }
  return I;
}

// The batch's TX span and bytes, its RX box, whether one copy of the span
// stages it (dense: at most 1.5 x its bytes + 64 KiB), and the pending
// batches it must follow: their RX boxes meet the span this batch stages
// (its stage-in waits for their write-back) or its own RX box (its delivery
// does).  Boxes are conservative: a wait that is not needed costs time, not
// results.
void BatchedQueuePair::image_prepare(Slot& sl, HostImage& img, std::span<const TxDescriptor> tx,
                                     std::span<const RxDescriptor> rx) {
  Scratch& S = *scratch_;
  const std::uint64_t size = img.size;
  struct Box {
    std::uint64_t lo = ~0ull, hi = 0, bytes = 0;
  };
  const rx_stage_detail::Chunks ct(tx.size(), config_.host_threads ? config_.host_threads : 16, 1u << 17);
  std::vector<Box> tb(ct.k), rb;
  ct.run([&](std::size_t c, std::size_t b, std::size_t e) {
    Box x;
    for (std::size_t i = b; i < e; ++i) {
      const std::uint64_t a = tx[i].buffer_address, n = tx[i].length;
      if (n == 0 || !nicqp::dma_ok(size, a, n)) continue;
      x.lo = std::min(x.lo, a);
      x.hi = std::max(x.hi, a + n);
      x.bytes += n;
    }
    tb[c] = x;
  });
  const rx_stage_detail::Chunks cr(rx.size(), config_.host_threads ? config_.host_threads : 16, 1u << 17);
  rb.resize(cr.k);
  cr.run([&](std::size_t c, std::size_t b, std::size_t e) {
    Box x;
    for (std::size_t j = b; j < e; ++j) {
      const std::uint64_t a = rx[j].buffer_address;
      if (rx[j].buffer_length == 0 || a >= size) continue;
      x.lo = std::min(x.lo, a);
      x.hi = std::max(x.hi, a + std::min<std::uint64_t>(rx[j].buffer_length, size - a));
    }
    rb[c] = x;
  });
  Box T, R;
  for (const Box& x : tb) {
    T.lo = std::min(T.lo, x.lo);
    T.hi = std::max(T.hi, x.hi);
    T.bytes += x.bytes;
  }
  for (const Box& x : rb) {
    R.lo = std::min(R.lo, x.lo);
    R.hi = std::max(R.hi, x.hi);
  }
  sl.image = &img;
  sl.tx_lo = T.hi > T.lo ? T.lo : 0;
  sl.tx_hi = T.hi > T.lo ? T.hi : 0;
  sl.tx_bytes = T.bytes;
  sl.rx_lo = R.hi > R.lo ? R.lo : 0;
  sl.rx_hi = R.hi > R.lo ? R.hi : 0;
  sl.whole = sl.tx_hi > sl.tx_lo && sl.tx_hi - sl.tx_lo <= T.bytes + T.bytes / 2 + (std::uint64_t{1} << 16);
  sl.dep_stage.clear();
  sl.dep_rx.clear();
  for (unsigned k = 0; k < S.pending; ++k) {
    Slot& p = S.slot[(S.head + k) % Scratch::kSlots];
    if (&p == &sl || p.image != &img || p.rx_hi <= p.rx_lo) continue;
    if (p.rx_lo < sl.tx_hi && sl.tx_lo < p.rx_hi) sl.dep_stage.push_back(&p);
    // the delivery may not overwrite bytes a write-back still reads
    if (p.mirror == sl.mirror && p.rx_lo < sl.rx_hi && sl.rx_lo < p.rx_hi) sl.dep_rx.push_back(&p);
  }
}

void* BatchedQueuePair::stage_stream() const {
  return stage_stream_env() ? scratch_->side_stage : scratch_->side_up;
}

// The TX bytes into the mirror on `stream`: one copy of the span when dense
// (the registered window goes up by DMA at the link's rate), else the gather
// kernel over the TX descriptors (tx_dev: the batch's descriptors on the
// device, in stream order; null: uploaded here).  Records ev_staged.
void BatchedQueuePair::image_stage(Slot& sl, std::size_t ntx, const TxDescriptor* tx_host, const void* tx_dev,
                                   void* stream) {
  HostImage& I = *sl.image;
  Scratch& S = *scratch_;
  if (sl.tx_hi > sl.tx_lo) {
    auto* mirror = static_cast<std::uint8_t*>(I.mirror[sl.mirror].p);
    if (sl.whole) {
      check(nicgpu_memcpy_async(mirror + sl.tx_lo, I.host + sl.tx_lo, sl.tx_hi - sl.tx_lo, stream), "nicgpu_memcpy_async");
    } else {
      // descriptors uploaded on side_up (ev_tx) unless uploaded here
      if (tx_dev && stream != S.side_up) check(nicgpu_stream_wait_event(stream, sl.ev_tx), "nicgpu_stream_wait_event");
      if (!tx_dev) {
        tx_dev = sl.stage_tx.get(ntx * sizeof(TxDescriptor));
        check(nicgpu_memcpy_async(const_cast<void*>(tx_dev), tx_host, ntx * sizeof(TxDescriptor), stream),
              "nicgpu_memcpy_async");
      }
      check(nicgpu_image_stage(mirror, I.alias, I.size, static_cast<const nicgpu_tx_descriptor*>(tx_dev), ntx, stream),
            "nicgpu_image_stage");
    }
  }
  check(nicgpu_event_record(sl.ev_staged, stream), "nicgpu_event_record");
  sl.staged = true;
}

// The bytes of writes_dev[0, n) from the mirror back into the memory, on
// `stream`; records ev_wb (finish() / collect() wait for it).
void BatchedQueuePair::image_writeback(Slot& sl, const nicgpu_segment_write* writes_dev, std::size_t n, void* stream) {
  HostImage& I = *sl.image;
  if (n)
    check(nicgpu_image_writeback(static_cast<const std::uint8_t*>(I.mirror[sl.mirror].p), I.alias, I.size, writes_dev, n, stream),
          "nicgpu_image_writeback");
  check(nicgpu_event_record(sl.ev_wb, stream), "nicgpu_event_record");
  sl.wb = true;
}

// Overlapping buffers or the host resolve, on a HostMemory: the host path over
// the mirror (its piece sums after the stage-in, its writes after the
// write-backs of earlier batches it rewrites), then every write it made back
// into the memory, on `stream`.
void BatchedQueuePair::image_host_path(Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                                       QueuePairStats& st, RxBatchResult& out, void* stream, int disjoint,
                                       double& check_us) {
  if (!sl.staged) image_stage(sl, tx.size(), tx.data(), nullptr, stream);
  check(nicgpu_stream_wait_event(stream, sl.ev_staged), "nicgpu_stream_wait_event");
  for (Slot* p : sl.dep_rx) check(nicgpu_stream_wait_event(stream, p->ev_wb), "nicgpu_stream_wait_event");
  sl.applied.clear();
  on_host(sl.image->view(sl.mirror), tx, rx, st, out, stream, disjoint, check_us, &sl.applied, sl.wcheck);
  out.timings.host_image = true;
  out.timings.staged_whole = sl.whole;
  const std::size_t n = sl.applied.size();
  void* d = sl.wbuf.get(std::max<std::size_t>(n, 1) * sizeof(rx_stage_detail::SegmentWrite));
  if (n) {
    // staged through page-locked memory (a full-rate copy of the write list)
    auto* h = sl.h_applied.get<rx_stage_detail::SegmentWrite>(n);
    std::memcpy(h, sl.applied.data(), n * sizeof(rx_stage_detail::SegmentWrite));
    check(nicgpu_memcpy_async(d, h, n * sizeof(rx_stage_detail::SegmentWrite), stream), "nicgpu_memcpy_async");
  }
  image_writeback(sl, static_cast<const nicgpu_segment_write*>(d), n, stream);
}

RxBatchResult BatchedQueuePair::process_batch(HostMemory& mem, std::span<const TxDescriptor> tx,
                                              std::span<const RxDescriptor> rx, void* stream) {
  RxBatchResult out;
  process_batch(mem, tx, rx, out, stream);
  return out;
}

void BatchedQueuePair::process_batch(HostMemory& m, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                                     RxBatchResult& out, void* stream) {
  Scratch& S = *scratch_;
  if (S.pending) throw std::logic_error("process_batch: collect() the submitted batches first");
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  S.ensure(dev);
  Slot& sl = S.slot[0];
  const bool checked = config_.host_memory_faults;
  std::byte* window = nullptr;
  if (checked) tx = checked_tx(sl, m, tx, window);  // the reads' verdicts, before anything is written
  HostImage& I = bind_image(m, checked, window);
  sl.mem_writes.mem = &m;
  sl.mem_writes.window = I.host;
  sl.wcheck = checked ? &sl.mem_writes : nullptr;
  sl.mirror = 0;
  const DeviceHostMemory mem = I.view();
  sl.tx_dev = nullptr;
  sl.rx_dev = nullptr;
  sl.multi = false;
  sl.overlap = false;
  image_prepare(sl, I, tx, rx);  // nothing pending: no dependencies
  sl.staged = false;
  QueuePairStats st = stats_;
  int disjoint = -1;
  double check_us = 0;
  bool on_device = false;
  try {
    if (!checked && config_.device_resolve && device_fits(tx.size(), rx.size())) {
      upload(sl, tx, rx, true);
      image_stage(sl, tx.size(), tx.data(), sl.v.tx, stage_stream());
      on_device = front(sl, mem, tx, rx, st, out, stream, disjoint, check_us);
      if (on_device) {
        back(sl, mem, out, stream);
        finish(sl, out, &st);
      }
    }
    if (!on_device) {
      image_host_path(sl, tx, rx, st, out, stream, disjoint, check_us);
      sl.wait_writeback();
    }
  } catch (...) {
    try {
      sl.wait_writeback();
    } catch (...) {
    }
    throw;
  }
  out.timings.check_us = check_us;
  stats_ = st;
  if (config_.on_interrupt) fire_interrupts(out, &sl);
}

void BatchedQueuePair::submit(HostMemory& m, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                              void* stream) {
  Scratch& S = *scratch_;
  if (S.pending == Scratch::kSlots) throw std::logic_error("submit: three batches pending; collect() one first");
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  if (S.pending == 0) S.ensure(dev);
  else if (S.device != dev) throw std::logic_error("submit: batches pending on another device");
  Slot& sl = S.slot[(S.head + S.pending) % Scratch::kSlots];
  const bool checked = config_.host_memory_faults;
  std::byte* window = nullptr;
  if (checked) tx = checked_tx(sl, m, tx, window);  // kept in the slot until collected
  HostImage& I = bind_image(m, checked, window);
  sl.mem_writes.mem = &m;
  sl.mem_writes.window = I.host;
  // alternate mirrors while batches are pending (NIC_IMAGE_MIRRORS=1: one, A/B)
  sl.mirror = 0;
  if (S.pending && image_mirrors_env() > 1 && I.size) {
    sl.mirror = 1u - S.slot[(S.head + S.pending - 1) % Scratch::kSlots].mirror;
    I.mirror[sl.mirror].get((I.size + 15) / 16 * 16);
  }
  enqueue(I.view(sl.mirror), tx, rx, nullptr, stream, &I);
}

std::span<const TxDescriptor> BatchedQueuePair::checked_tx(Slot& sl, HostMemory& m, std::span<const TxDescriptor> tx,
                                                           std::byte*& window) {
  window = rx_stage_detail::checked_reads(m, tx, sl.checked_tx);
  return sl.checked_tx;
}

// ------------------------------------------------------------------------
// BatchedQueueManager's fused batch (queue_manager.cpp:54-78 over queue pairs
// whose buffers do not meet): every queue pair's TX batch and RX ring back to
// back in one device context, resolved as one batch with per-queue-pair
// segments (nicgpu_qp_set_segments), delivered in one launch.

void BatchedQueuePair::share_image(const BatchedQueuePair& owner) { scratch_->img = owner.scratch_->img; }

// front_once's device path for a segmented batch (sizes from the caller, no
// host tail, no host sort): false = the batch does not fit the fused path.
bool BatchedQueuePair::front_multi(Slot& sl, const DeviceHostMemory& mem, std::size_t ntx, std::size_t nrx,
                                   RxBatchResult& out, void* stream, int& again, bool whole_check) {
  using clock = std::chrono::steady_clock;
  auto us_since = [](clock::time_point t) { return std::chrono::duration<double, std::micro>(clock::now() - t).count(); };
  Scratch& S = *scratch_;
  nicgpu_qp_view& v = sl.v;
  void* ps = S.side_plan;
  auto t = clock::now();
  check(nicgpu_stream_wait_event(ps, sl.ev_tx), "nicgpu_stream_wait_event");
  if (sl.staged) check(nicgpu_stream_wait_event(stream, sl.ev_staged), "nicgpu_stream_wait_event");
  check(nicgpu_qp_set_deferred_verify(sl.qp, defer_multi_ ? 1 : 0), "nicgpu_qp_set_deferred_verify");
  check(nicgpu_qp_plan_async(sl.qp, reinterpret_cast<const std::uint8_t*>(mem.base), mem.size, ntx, config_.max_mtu, &v,
                             ps, stream),
        "nicgpu_qp_plan_async");
  check(nicgpu_stream_wait_event(ps, sl.ev_rx), "nicgpu_stream_wait_event");
  check(nicgpu_stream_wait_event(stream, sl.ev_rx), "nicgpu_stream_wait_event");
  out.timings.sums_us += us_since(t);
  t = clock::now();
  check(nicgpu_qp_resolve_start(sl.qp, mem.size, ntx, nrx, config_.max_mtu, config_.queue_id, stream),
        "nicgpu_qp_resolve_start");
  check(nicgpu_event_record(sl.ev_resolved, stream), "nicgpu_event_record");
  out.timings.resolve_us += us_since(t);
  t = clock::now();
  // the overlap check behind the plan on its stream, beside the piece sums and
  // the speculative resolve (measured: run beside the plan instead, it slows
  // the plan and the sums more than it gains)
  int verdict = -1;
  check(nicgpu_qp_check_async(sl.qp, mem.size, ntx, nrx, whole_check ? NICGPU_QP_CHECK_WHOLE : 0u, ps),
        "nicgpu_qp_check_async");
  check(nicgpu_qp_check_wait(sl.qp, &verdict), "nicgpu_qp_check_wait");
  out.timings.check_us += us_since(t);
  if (verdict != 1) return false;  // overlapping, or a ring not in address order: per queue pair
  t = clock::now();
  sl.tn = sl.nq = 0;
  const nicgpu_rss_ctx* rctx = nullptr;
  std::uint64_t* hits = nullptr;
  if (config_.rss != nullptr) {
    const auto& table = config_.rss->config().table;
    sl.tn = table.size();
    for (const std::uint16_t q : table) sl.nq = std::max<std::size_t>(sl.nq, std::size_t{q} + 1);
    rctx = config_.rss->device_context(stream);
    hits = static_cast<std::uint64_t*>(sl.hits.get(std::max<std::size_t>(sl.tn, 1) * sizeof(std::uint64_t)));
  }
  deliver(sl, mem, 0, nrx, NICGPU_DELIVER_SETTLED | NICGPU_DELIVER_RESET_HITS, rctx, hits, stream);
  out.timings.gather_us += us_since(t);
  t = clock::now();
  std::uint64_t done = 0, used = 0, settled = 0;
  nicgpu_qp_stats ds{};
  std::uint64_t walks0 = 0, walks1 = 0;
  check(nicgpu_qp_walks(sl.qp, &walks0), "nicgpu_qp_walks");
  const int rst = nicgpu_qp_resolve_finish(sl.qp, &done, &used, &settled, &ds);
  check(nicgpu_qp_walks(sl.qp, &walks1), "nicgpu_qp_walks");
  out.timings.walked = out.timings.walked || walks1 != walks0;
  out.timings.resolve_us += us_since(t);
  int late = 0;
  check(nicgpu_qp_deferred(sl.qp, &late), "nicgpu_qp_deferred");
  sl.late = rst == NICGPU_OK && late != 0;
  out.timings.deferred = sl.late;
  if (rst == NICGPU_ERR_AGAIN) {
    again = 1;
    return false;
  }
  if (rst == NICGPU_ERR_RANGE || rst == NICGPU_ERR_UNSETTLED) return false;
  check(rst, "nicgpu_qp_resolve_finish");
  sl.settled = settled;
  sl.relaxed = settled < used;
  sl.ntx = ntx;
  sl.nrx_total = used;
  out.tx_processed = ntx;
  out.rx_consumed = used;
  if (config_.results_on_device) out.tx_completions.clear();
  else out.tx_completions.resize(ntx);
  return true;
}

bool BatchedQueuePair::process_queues(const DeviceHostMemory& mem_in, HostImage* img,
                                      std::span<const std::span<const TxDescriptor>> tx,
                                      std::span<const std::span<const RxDescriptor>> rx,
                                      std::span<const BatchedQueuePairConfig> configs, std::vector<RxBatchResult>& out,
                                      std::vector<QueuePairStats>& stats, void* stream, bool dev_desc,
                                      bool whole_check) {
  using clock = std::chrono::steady_clock;
  Scratch& S = *scratch_;
  if (S.pending) throw std::logic_error("process_queues: batches pending");
  const std::size_t Q = tx.size();
  if (Q == 0 || Q > NICGPU_QP_MAX_SEGMENTS || rx.size() != Q || configs.size() != Q) return false;
  std::vector<nicgpu_qp_segment> seg(Q);
  std::size_t ntx = 0, nrx = 0;
  for (std::size_t q = 0; q < Q; ++q) {
    seg[q] = nicgpu_qp_segment{ntx, nrx, rx[q].size(), configs[q].max_mtu, configs[q].queue_id, 0, 0, 0};
    ntx += tx[q].size();
    nrx += rx[q].size();
  }
  if (!device_fits(ntx, nrx) || ntx == 0 || (dev_desc && img)) return false;
  int dev = 0;
  check(nicgpu_get_device(&dev), "nicgpu_get_device");
  S.ensure(dev);
  const DeviceHostMemory mem = img ? img->view() : mem_in;
  Slot& sl = S.slot[0];
  sl.mirror = 0;
  sl.tx_dev = nullptr;
  sl.rx_dev = nullptr;
  sl.image = nullptr;
  sl.wcheck = nullptr;
  sl.staged = false;
  sl.dep_stage.clear();
  sl.dep_rx.clear();
  sl.multi = true;
  sl.overlap = false;
  sl.nseg = Q;
  RxBatchResult cat;
  cat.timings = RxBatchResult::Timings{};
  cat.timings.device = true;
  const auto t0 = clock::now();
  // descriptors up, queue pair by queue pair, into the concatenated arrays
  // (device arrays: copied after what the caller enqueued before the call)
  nicgpu_qp_view& v = sl.v;
  check(nicgpu_qp_reserve(sl.qp, ntx, nrx, &v), "nicgpu_qp_reserve");
  if (dev_desc) {
    check(nicgpu_event_record(sl.ev_submit, stream), "nicgpu_event_record");
    check(nicgpu_stream_wait_event(S.side_up, sl.ev_submit), "nicgpu_stream_wait_event");
  }
  if (dev_desc) {  // HBM to HBM: one gather launch per 64 arrays, not a copy per array
    std::vector<nicgpu_copy_range> cr;
    cr.reserve(2 * Q);
    for (std::size_t q = 0; q < Q; ++q)
      cr.push_back({v.tx + seg[q].tx_begin, tx[q].data(), tx[q].size() * sizeof(TxDescriptor)});
    for (std::size_t q = 0; q < Q; ++q)
      cr.push_back({v.rx + seg[q].rx_begin, rx[q].data(), rx[q].size() * sizeof(RxDescriptor)});
    for (std::size_t i = 0; i < cr.size(); i += NICGPU_COPY_BATCH_MAX)
      check(nicgpu_memcpy_batch(cr.data() + i, std::min<std::size_t>(NICGPU_COPY_BATCH_MAX, cr.size() - i), S.side_up),
            "nicgpu_memcpy_batch");
    check(nicgpu_event_record(sl.ev_tx, S.side_up), "nicgpu_event_record");
    check(nicgpu_event_record(sl.ev_rx, S.side_up), "nicgpu_event_record");
  } else {
    for (std::size_t q = 0; q < Q; ++q)
      check(nicgpu_memcpy_async(v.tx + seg[q].tx_begin, tx[q].data(), tx[q].size() * sizeof(TxDescriptor), S.side_up),
            "nicgpu_memcpy_async");
    check(nicgpu_event_record(sl.ev_tx, S.side_up), "nicgpu_event_record");
    for (std::size_t q = 0; q < Q; ++q)
      check(nicgpu_memcpy_async(v.rx + seg[q].rx_begin, rx[q].data(), rx[q].size() * sizeof(RxDescriptor), S.side_up),
            "nicgpu_memcpy_async");
    check(nicgpu_event_record(sl.ev_rx, S.side_up), "nicgpu_event_record");
  }
  if (img) {  // the TX bytes of every queue pair: their span, or a gather over the uploaded descriptors
    sl.image = img;
    std::uint64_t lo = ~0ull, hi = 0, bytes = 0, rlo = ~0ull, rhi = 0;
    for (std::size_t q = 0; q < Q; ++q) {
      for (const TxDescriptor& t : tx[q]) {
        if (t.length == 0 || !nicqp::dma_ok(img->size, t.buffer_address, t.length)) continue;
        lo = std::min<std::uint64_t>(lo, t.buffer_address);
        hi = std::max<std::uint64_t>(hi, t.buffer_address + t.length);
        bytes += t.length;
      }
      for (const RxDescriptor& x : rx[q]) {
        if (x.buffer_length == 0 || x.buffer_address >= img->size) continue;
        rlo = std::min<std::uint64_t>(rlo, x.buffer_address);
        rhi = std::max<std::uint64_t>(rhi, x.buffer_address + std::min<std::uint64_t>(x.buffer_length, img->size - x.buffer_address));
      }
    }
    sl.tx_lo = hi > lo ? lo : 0;
    sl.tx_hi = hi > lo ? hi : 0;
    sl.tx_bytes = bytes;
    sl.rx_lo = rhi > rlo ? rlo : 0;
    sl.rx_hi = rhi > rlo ? rhi : 0;
    sl.whole = sl.tx_hi > sl.tx_lo && sl.tx_hi - sl.tx_lo <= bytes + bytes / 2 + (std::uint64_t{1} << 16);
    image_stage(sl, ntx, nullptr, v.tx, stage_stream());
  }
  cat.timings.copy_us += std::chrono::duration<double, std::micro>(clock::now() - t0).count();
  check(nicgpu_qp_set_segments(sl.qp, seg.data(), Q, ntx, S.side_plan), "nicgpu_qp_set_segments");
  // RSS: the engines' configurations are equal (the manager checked): one
  // context hashes every queue pair's frames; separate engines count their own
  RssEngine* const rss0 = configs[0].rss;
  bool own_engines = false;
  for (std::size_t q = 1; q < Q; ++q) own_engines |= configs[q].rss != rss0;
  sl.seg_hits_on = rss0 != nullptr && own_engines;
  // deferred RX verify when this stage and every queue pair's configuration allow it
  defer_multi_ = config_.defer_rx_verify && defer_env();
  for (std::size_t q = 0; q < Q; ++q) defer_multi_ = defer_multi_ && configs[q].defer_rx_verify;
  bool ok = false;
  try {
    for (int attempt = 0;; ++attempt) {
      int again = 0;
      ok = front_multi(sl, mem, ntx, nrx, cat, stream, again, whole_check);
      if (!again) break;
      if (attempt >= 1) throw GpuError("process_queues: the device plan outgrew its piece buffers twice", NICGPU_ERR_AGAIN);
      cat.timings.replans += 1;
    }
    if (ok) {
      back(sl, mem, cat, stream);
      finish(sl, cat, nullptr);
    }
  } catch (...) {
    (void) nicgpu_qp_set_segments(sl.qp, nullptr, 0, 0, nullptr);
    sl.multi = false;
    try {
      sl.wait_writeback();
    } catch (...) {
    }
    throw;
  }
  if (!ok) {
    check(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");  // the wasted resolve is over
    check(nicgpu_qp_set_segments(sl.qp, nullptr, 0, 0, nullptr), "nicgpu_qp_set_segments");
    sl.multi = false;
    return false;
  }
  // split per queue pair
  std::vector<std::uint64_t> used(Q);
  std::vector<nicgpu_qp_stats> ds(Q);
  check(nicgpu_qp_segment_results(sl.qp, used.data(), ds.data()), "nicgpu_qp_segment_results");
  out.resize(Q);
  stats.assign(Q, QueuePairStats{});
  const bool keep = config_.results_on_device;
  const bool rss = sl.rss;
  const std::size_t nq = sl.nq, tn = sl.tn;
  const std::uint32_t* split = rss ? sl.h_split.get<std::uint32_t>((Q + 1) * std::max<std::size_t>(nq, 1)) : nullptr;
  const std::uint64_t* seg_hits = sl.seg_hits_on ? sl.h_seg_hits.get<std::uint64_t>(Q * tn) : nullptr;
  for (std::size_t q = 0; q < Q; ++q) {
    RxBatchResult& o = out[q];
    const std::size_t tb = seg[q].tx_begin, rb = seg[q].rx_begin, nt = tx[q].size(), nr = used[q];
    static_assert(sizeof(QueuePairStats) == sizeof(nicgpu_qp_stats));
    std::memcpy(static_cast<void*>(&stats[q]), &ds[q], sizeof(QueuePairStats));
    if (sl.late) apply_fixups(sl, q, stats[q]);
    o.tx_processed = nt;
    o.rx_consumed = nr;
    o.timings = cat.timings;
    o.timings.host_image = img != nullptr;
    o.timings.staged_whole = img != nullptr && sl.whole;
    o.dev = RxBatchResult::DeviceResults{};
    std::size_t used_q = 0;  // largest RSS queue with frames + 1
    if (rss)
      for (std::size_t r = 0; r < nq; ++r)
        if (split[(q + 1) * nq + r] > split[q * nq + r]) used_q = r + 1;
    if (keep) {
      o.tx_completions.clear();
      o.rx_completions.clear();
      o.rx_hash.clear();
      o.rx_queue.clear();
      o.queues.clear();
      RxBatchResult::DeviceResults& d = o.dev;
      d.tx_completions = reinterpret_cast<const CompletionEntry*>(v.txc) + tb;
      d.rx_completions = reinterpret_cast<const CompletionEntry*>(v.rxc) + rb;
      d.ntx = nt;
      d.nrx = nr;
      d.rx_hash = rss ? v.rx_hash + rb : nullptr;
      d.rx_queue = rss ? v.rx_queue + rb : nullptr;
      d.queue_which = rss ? v.queue_which : nullptr;
      if (rss) {
        d.queue_start.assign(split + q * nq, split + q * nq + used_q);
        d.queue_end.assign(split + (q + 1) * nq, split + (q + 1) * nq + used_q);
      }
    } else {
      o.tx_completions.assign(cat.tx_completions.begin() + tb, cat.tx_completions.begin() + tb + nt);
      o.rx_completions.assign(cat.rx_completions.begin() + rb, cat.rx_completions.begin() + rb + nr);
      o.rx_hash.assign(cat.rx_hash.begin() + rb, cat.rx_hash.begin() + rb + nr);
      o.rx_queue.assign(cat.rx_queue.begin() + rb, cat.rx_queue.begin() + rb + nr);
      for (auto& l : o.queues) l.clear();
      o.queues.resize(used_q);
      for (std::size_t r = 0; r < used_q; ++r) o.queues[r].assign(sl.which + split[q * nq + r], sl.which + split[(q + 1) * nq + r]);
    }
    if (rss && seg_hits) {  // queue pair q's engine counts its own frames
      std::uint64_t m = 0;
      for (std::size_t k = 0; k < tn; ++k) m += seg_hits[q * tn + k];
      configs[q].rss->account_batch(m, std::span<const std::uint64_t>(seg_hits + q * tn, tn));
    }
  }
  if (rss && !seg_hits) rss0->account_batch(sl.meta[0], std::span<const std::uint64_t>(sl.meta + 1, sl.tn));
  return true;
}

}  // namespace nic
