// queue_manager.cpp — nic::BatchedQueueManager (include/nic/rx_queue_manager.h):
// the reference's QueueManager (src/queue_manager.cpp) over batches.
#include "nic/rx_queue_manager.h"

#include <algorithm>
#include <cstring>
#include <exception>
#include <set>
#include <sstream>

#include "nicgpu.h"

namespace nic {

namespace {

constexpr std::size_t kStats = sizeof(QueuePairStats) / sizeof(std::uint64_t);
static_assert(sizeof(QueuePairStats) == kStats * sizeof(std::uint64_t), "QueuePairStats is u64 counters");

// out += a - b, counter by counter
void add_delta(QueuePairStats& out, const QueuePairStats& a, const QueuePairStats& b) {
  std::uint64_t o[kStats], x[kStats], y[kStats];
  std::memcpy(o, &out, sizeof(o));
  std::memcpy(x, &a, sizeof(x));
  std::memcpy(y, &b, sizeof(y));
  for (std::size_t i = 0; i < kStats; ++i) o[i] += x[i] - y[i];
  std::memcpy(&out, o, sizeof(o));
}

void clear_result(RxBatchResult& r) {
  r.tx_processed = r.rx_consumed = 0;
  r.tx_completions.clear();
  r.rx_completions.clear();
  r.rx_hash.clear();
  r.rx_queue.clear();
  r.queues.clear();
  r.dev = RxBatchResult::DeviceResults{};
  r.timings = RxBatchResult::Timings{};
}

// part appended to out (its RX completion indices shifted past out's)
void append_result(RxBatchResult& out, const RxBatchResult& part) {
  const auto base = static_cast<std::uint32_t>(out.rx_completions.size());
  out.tx_processed += part.tx_processed;
  out.rx_consumed += part.rx_consumed;
  out.tx_completions.insert(out.tx_completions.end(), part.tx_completions.begin(), part.tx_completions.end());
  out.rx_completions.insert(out.rx_completions.end(), part.rx_completions.begin(), part.rx_completions.end());
  out.rx_hash.insert(out.rx_hash.end(), part.rx_hash.begin(), part.rx_hash.end());
  out.rx_queue.insert(out.rx_queue.end(), part.rx_queue.begin(), part.rx_queue.end());
  if (out.queues.size() < part.queues.size()) out.queues.resize(part.queues.size());
  for (std::size_t q = 0; q < part.queues.size(); ++q)
    for (const std::uint32_t j : part.queues[q]) out.queues[q].push_back(base + j);
  out.timings.check_us += part.timings.check_us;
  out.timings.plan_us += part.timings.plan_us;
  out.timings.sums_us += part.timings.sums_us;
  out.timings.resolve_us += part.timings.resolve_us;
  out.timings.gather_us += part.timings.gather_us;
  out.timings.rss_us += part.timings.rss_us;
  out.timings.copy_us += part.timings.copy_us;
}

struct Span {
  std::uint64_t lo, hi;
  std::uint32_t queue;
  bool rx;
};

// the largest span end seen so far from two different queues
struct Top2 {
  std::uint64_t hi1 = 0, hi2 = 0;
  std::uint32_t q1 = ~0u, q2 = ~0u;
  void add(std::uint64_t hi, std::uint32_t q) {
    if (q == q1) {
      hi1 = std::max(hi1, hi);
    } else if (hi > hi1) {
      hi2 = hi1;
      q2 = q1;
      hi1 = hi;
      q1 = q;
    } else if (q == q2 || hi > hi2) {
      hi2 = std::max(q == q2 ? hi2 : 0, hi);
      q2 = q;
    }
    if (hi2 > hi1) {  // keep hi1 the larger (q2's update may pass it)
      std::swap(hi1, hi2);
      std::swap(q1, q2);
    }
  }
  std::uint64_t other_than(std::uint32_t q) const { return q1 != q ? hi1 : hi2; }
};

}  // namespace

namespace qm_detail {

QueueSchedule schedule(std::span<const std::uint8_t> weights, std::span<const std::size_t> pending, std::size_t& index,
                       std::size_t& credit, bool want_runs) {
  QueueSchedule out;
  const std::size_t Q = weights.size();
  if (Q == 0) return out;
  std::vector<std::size_t> left(pending.begin(), pending.end());
  left.resize(Q, 0);
  for (;;) {  // one process_once per iteration (a run of them while the turn holds)
    // Without the runs, whole cycles are counted at once: from a fresh turn on
    // a nonempty queue, one trip round the ring serves weights[q] from every
    // nonempty queue and skips every empty one once, and comes back to the
    // same turn — as long as every nonempty queue has weights[q] left, and
    // more is served after it (the empty queues after the last serve are
    // skipped by the final call instead): k - 1 of the k possible cycles.
    if (!want_runs && left[index] > 0 && credit == weights[index]) {
      std::size_t k = ~std::size_t{0}, served_per = 0, empty = 0;
      for (std::size_t q = 0; q < Q; ++q) {
        if (left[q] == 0) {
          ++empty;
          continue;
        }
        k = std::min(k, left[q] / weights[q]);
        served_per += weights[q];
      }
      if (k > 1 && k != ~std::size_t{0}) {
        k -= 1;
        for (std::size_t q = 0; q < Q; ++q)
          if (left[q]) left[q] -= k * weights[q];
        out.advances += k * served_per;
        out.skips += k * empty;
      }
    }
    bool served = false;
    for (std::size_t tries = 0; tries < Q; ++tries) {
      if (left[index] > 0) {
        // process_once returns true for every descriptor of the batch: the
        // turn serves min(credit, left) of them, then passes when the credit ends
        const std::size_t k = std::min(credit, left[index]);
        if (!want_runs) {
        } else if (!out.runs.empty() && out.runs.back().queue == index) {
          out.runs.back().count += static_cast<std::uint32_t>(k);
        } else {
          out.runs.push_back({static_cast<std::uint32_t>(index), static_cast<std::uint32_t>(k)});
        }
        left[index] -= k;
        out.advances += k;
        if (k == credit) {
          index = (index + 1) % Q;
          credit = weights[index];
        } else {
          credit -= k;
        }
        served = true;
        break;
      }
      ++out.skips;  // an empty TX ring: skip it (queue_manager.cpp:72-75)
      index = (index + 1) % Q;
      credit = weights[index];
    }
    if (!served) break;  // every ring empty: process_once returned false
  }
  return out;
}

bool queues_disjoint(std::size_t mem_size, std::span<const QueueBatch> batches) {
  // Fast path, O(n): each queue's TX and RX spans inside bounding boxes; when
  // no queue's RX box meets another queue's TX or RX box no two spans can
  // overlap (the usual layout: every queue's buffers in a region of its own).
  // Otherwise the exact sweep below (a sort of every span).
  {
    struct Box {
      std::uint64_t lo = ~0ull, hi = 0;
      void add(std::uint64_t a, std::uint64_t b) {
        lo = std::min(lo, a);
        hi = std::max(hi, b);
      }
      bool meets(const Box& o) const { return lo < o.hi && o.lo < hi; }
    };
    std::vector<Box> tb(batches.size()), rb(batches.size());
    for (std::size_t q = 0; q < batches.size(); ++q) {
      for (const TxDescriptor& t : batches[q].tx)
        if (t.length && t.buffer_address < mem_size)
          tb[q].add(t.buffer_address, std::min<std::uint64_t>(t.buffer_address + t.length, mem_size));
      for (const RxDescriptor& x : batches[q].rx)
        if (x.buffer_length && x.buffer_address < mem_size)
          rb[q].add(x.buffer_address, std::min<std::uint64_t>(x.buffer_address + x.buffer_length, mem_size));
    }
    bool apart = true;
    for (std::size_t q = 0; q < batches.size() && apart; ++q)
      for (std::size_t r = 0; r < batches.size() && apart; ++r)
        if (q != r && (rb[q].meets(tb[r]) || rb[q].meets(rb[r]))) apart = false;
    if (apart) return true;
  }
  std::vector<Span> spans;
  auto add = [&](std::uint64_t a, std::uint64_t n, std::uint32_t q, bool rx) {
    if (n == 0 || a >= mem_size) return;  // nothing moved, or a DMA fault
    spans.push_back({a, std::min<std::uint64_t>(a + n, mem_size), q, rx});
  };
  for (std::uint32_t q = 0; q < batches.size(); ++q) {
    for (const TxDescriptor& t : batches[q].tx) add(t.buffer_address, t.length, q, false);
    for (const RxDescriptor& x : batches[q].rx) add(x.buffer_address, x.buffer_length, q, true);
  }
  std::sort(spans.begin(), spans.end(), [](const Span& a, const Span& b) { return a.lo < b.lo; });
  Top2 any, rx;  // ends of the spans so far (all / RX only), per queue
  for (const Span& s : spans) {
    // an earlier span (lo <= s.lo) of another queue overlaps s when it ends
    // past s.lo; a conflict needs an RX span on one side
    if ((s.rx ? any : rx).other_than(s.queue) > s.lo) return false;
    any.add(s.hi, s.queue);
    if (s.rx) rx.add(s.hi, s.queue);
  }
  return true;
}

}  // namespace qm_detail

struct BatchedQueueManager::Queue {
  BatchedQueuePairConfig config;           // as given (the interrupt callback is the manager's)
  BatchedQueuePair stage;                  // the device path, without the callback
  std::unique_ptr<BatchedQueuePair> host;  // interleaved replays: host path, made on first use
  QueuePairStats stats{};
  explicit Queue(const BatchedQueuePairConfig& c) : config(c), stage(quiet(c)) {}
  static BatchedQueuePairConfig quiet(BatchedQueuePairConfig c) {
    c.on_interrupt = nullptr;
    return c;
  }
  BatchedQueuePair& host_stage() {
    if (!host) {
      BatchedQueuePairConfig c = quiet(config);
      c.device_resolve = false;
      c.results_on_device = false;
      host = std::make_unique<BatchedQueuePair>(c);
    }
    return *host;
  }
};

// Every queue pair's batch runs on a stream of its own, forked from the
// caller's stream by an event and joined back into it, so the queue pairs'
// device work overlaps (one shared stream serialised 16 x 64 K batches).
struct BatchedQueueManager::Streams {
  int device = -1;
  void* fork = nullptr;           // recorded on the caller's stream
  std::vector<void*> s, joined;   // per queue pair: its stream and its end event
  ~Streams() { release(); }
  void release() {
    for (void* x : s) (void) nicgpu_stream_destroy(x);
    for (void* e : joined) (void) nicgpu_event_destroy(e);
    if (fork) (void) nicgpu_event_destroy(fork);
    s.clear();
    joined.clear();
    fork = nullptr;
    device = -1;
  }
  void ensure(std::size_t q) {
    int dev = 0;
    if (nicgpu_get_device(&dev) != NICGPU_OK) throw GpuError("BatchedQueueManager: no device", NICGPU_ERR_NO_DEVICE);
    if (dev != device) release();
    device = dev;
    auto ok = [](int st, const char* what) {
      if (st != NICGPU_OK) throw GpuError(std::string("BatchedQueueManager: ") + what, st);
    };
    if (!fork) ok(nicgpu_event_create(&fork), "nicgpu_event_create");
    while (s.size() < q) {
      void* x = nullptr;
      void* e = nullptr;
      ok(nicgpu_stream_create(&x), "nicgpu_stream_create");
      s.push_back(x);
      ok(nicgpu_event_create(&e), "nicgpu_event_create");
      joined.push_back(e);
    }
  }
};

BatchedQueueManager::BatchedQueueManager(BatchedQueueManagerConfig config) : streams_(std::make_unique<Streams>()) {
  for (BatchedQueuePairConfig& c : config.queue_configs) {
    if (c.weight == 0) c.weight = 1;  // queue_manager.cpp:14-16
    weights_.push_back(c.weight);
    qps_.push_back(std::make_unique<Queue>(c));
  }
  credit_ = weights_.empty() ? 0 : weights_.front();
  if (!qps_.empty()) {
    fused_ = std::make_unique<BatchedQueuePair>(Queue::quiet(qps_.front()->config));
    for (auto& qp : qps_) qp->stage.share_image(*fused_);  // one HBM mirror of a HostMemory for all
  }
}

// The fused batch needs the queue pairs' stage settings to agree: device
// resolve on, results kept alike, RSS off everywhere or engines whose key,
// table and tuple are equal (each still counts its own frames).
bool BatchedQueueManager::fusable() const {
  if (qps_.empty() || qps_.size() > NICGPU_QP_MAX_SEGMENTS) return false;
  const BatchedQueuePairConfig& c0 = qps_.front()->config;
  for (const auto& qp : qps_) {
    const BatchedQueuePairConfig& c = qp->config;
    if (!c.device_resolve || c.results_on_device != c0.results_on_device || (c.rss == nullptr) != (c0.rss == nullptr))
      return false;
    if (c.host_memory_faults) return false;  // the memory decides each access: per queue pair, on the host
    if (c.rss && c.rss != c0.rss) {
      if (c.tuple.mode != c0.tuple.mode || c.tuple.raw_offset != c0.tuple.raw_offset ||
          c.tuple.raw_length != c0.tuple.raw_length)
        return false;
      const RssConfig &a = c.rss->config(), &b = c0.rss->config();
      if (a.key != b.key || a.table != b.table) return false;
    } else if (c.rss && (c.tuple.mode != c0.tuple.mode || c.tuple.raw_offset != c0.tuple.raw_offset ||
                         c.tuple.raw_length != c0.tuple.raw_length)) {
      return false;
    }
  }
  return true;
}

BatchedQueueManager::~BatchedQueueManager() = default;

BatchedQueuePair* BatchedQueueManager::queue(std::size_t index) noexcept {
  return index < qps_.size() ? &qps_[index]->stage : nullptr;
}

std::optional<QueuePairStats> BatchedQueueManager::queue_stats(std::size_t index) const noexcept {
  if (index >= qps_.size()) return std::nullopt;
  return qps_[index]->stats;
}

QueueSchedule BatchedQueueManager::process_batch(const DeviceHostMemory& mem, std::span<const QueueBatch> batches,
                                                 std::vector<RxBatchResult>& out, void* stream) {
  return run(mem, nullptr, batches, out, stream);
}

QueueSchedule BatchedQueueManager::process_batch(HostMemory& mem, std::span<const QueueBatch> batches,
                                                 std::vector<RxBatchResult>& out, void* stream) {
  return run(DeviceHostMemory{}, &mem, batches, out, stream);
}

QueueSchedule BatchedQueueManager::process_batch(const DeviceHostMemory& mem, std::span<const DeviceQueueBatch> batches,
                                                 std::vector<RxBatchResult>& out, void* stream) {
  const std::size_t Q = qps_.size();
  if (batches.size() != Q) throw std::invalid_argument("BatchedQueueManager::process_batch: one batch per queue pair");
  for (const DeviceQueueBatch& b : batches)
    if ((b.ntx && !b.tx) || (b.nrx && !b.rx)) throw GpuError("process_batch: null device descriptors", NICGPU_ERR_INVALID);
  if (fusable()) {
    std::vector<std::span<const TxDescriptor>> txs(Q);
    std::vector<std::span<const RxDescriptor>> rxs(Q);
    std::vector<BatchedQueuePairConfig> cfgs(Q);
    std::vector<std::size_t> n(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      txs[q] = {batches[q].tx, batches[q].ntx};
      rxs[q] = {batches[q].rx, batches[q].nrx};
      cfgs[q] = qps_[q]->config;
      n[q] = batches[q].ntx;
    }
    for (RxBatchResult& r : out) clear_result(r);
    std::vector<QueuePairStats> st;
    if (fused_->process_queues(mem, nullptr, txs, rxs, cfgs, out, st, stream, /*dev_desc=*/true, /*whole_check=*/true)) {
      for (std::size_t q = 0; q < Q; ++q) add_delta(qps_[q]->stats, st[q], QueuePairStats{});
      std::size_t index = index_, credit = credit_;
      QueueSchedule sched = qm_detail::schedule(weights_, n, index, credit, interrupts());
      index_ = index;
      credit_ = credit;
      advances_ += sched.advances;
      skips_ += sched.skips;
      last_fused_ = 1;
      replay(sched, out, stream);
      return sched;
    }
  }
  // the host decides: the descriptors come down once
  std::vector<std::vector<TxDescriptor>> htx(Q);
  std::vector<std::vector<RxDescriptor>> hrx(Q);
  std::vector<QueueBatch> hb(Q);
  auto ok = [](int st, const char* what) {
    if (st != NICGPU_OK) throw GpuError(std::string("BatchedQueueManager: ") + what, st);
  };
  for (std::size_t q = 0; q < Q; ++q) {
    htx[q].resize(batches[q].ntx);
    hrx[q].resize(batches[q].nrx);
    if (batches[q].ntx)
      ok(nicgpu_memcpy_async(htx[q].data(), batches[q].tx, batches[q].ntx * sizeof(TxDescriptor), stream), "nicgpu_memcpy_async");
    if (batches[q].nrx)
      ok(nicgpu_memcpy_async(hrx[q].data(), batches[q].rx, batches[q].nrx * sizeof(RxDescriptor), stream), "nicgpu_memcpy_async");
  }
  ok(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");
  for (std::size_t q = 0; q < Q; ++q) hb[q] = QueueBatch{htx[q], hrx[q]};
  return run(mem, nullptr, hb, out, stream);
}

QueueSchedule BatchedQueueManager::run(const DeviceHostMemory& dmem, HostMemory* hmem, std::span<const QueueBatch> batches,
                                       std::vector<RxBatchResult>& out, void* stream) {
  const std::size_t Q = qps_.size();
  if (batches.size() != Q) throw std::invalid_argument("BatchedQueueManager::process_batch: one batch per queue pair");
  std::vector<std::size_t> n(Q);
  for (std::size_t q = 0; q < Q; ++q) n[q] = batches[q].tx.size();
  out.resize(Q);
  for (RxBatchResult& r : out) clear_result(r);
  // a HostMemory: the manager's one mirror of it (every stage shares it); with
  // host_memory_faults its window comes from the reads the memory allows
  bool checked = false;
  for (const auto& qp : qps_) checked = checked || qp->config.host_memory_faults;
  std::byte* window = nullptr;
  if (hmem && checked) {
    std::vector<TxDescriptor> scratch;
    for (std::size_t q = 0; q < Q && !window; ++q) window = rx_stage_detail::checked_reads(*hmem, batches[q].tx, scratch);
  }
  BatchedQueuePair::HostImage* img = hmem ? &fused_->bind_image(*hmem, checked, window) : nullptr;
  const std::size_t mem_size = hmem ? hmem->config().size_bytes : dmem.size;
  last_fused_ = 0;
  bool fused = false;
  int disjoint = -1;  // the queues' buffers apart from each other's (-1: not looked at yet)
  auto try_fused = [&](bool whole_check) {
    std::vector<std::span<const TxDescriptor>> txs(Q);
    std::vector<std::span<const RxDescriptor>> rxs(Q);
    std::vector<BatchedQueuePairConfig> cfgs(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      txs[q] = batches[q].tx;
      rxs[q] = batches[q].rx;
      cfgs[q] = qps_[q]->config;
    }
    std::vector<QueuePairStats> st;
    fused = fused_->process_queues(dmem, img, txs, rxs, cfgs, out, st, stream, false, whole_check);
    if (fused) {
      for (std::size_t q = 0; q < Q; ++q) add_delta(qps_[q]->stats, st[q], QueuePairStats{});
      last_fused_ = 1;
    }
  };
  // First the fused batch with the device checking the whole concatenation
  // (every queue's buffers against every other's too): no host pass over the
  // descriptors.  Rings laid out out of address order across queues fail that
  // check; then the host decides whether the queues are apart, and the fused
  // batch is tried once more, checked queue pair by queue pair.
  if (fusable()) try_fused(true);
  if (!fused) {
    disjoint = qm_detail::queues_disjoint(mem_size, batches) ? 1 : 0;
    if (disjoint && fusable()) try_fused(false);
  }
  // the runs of the schedule: for the reference's interleaving on the host
  // path and for the interrupts' order; the counters alone otherwise
  std::size_t index = index_, credit = credit_;
  QueueSchedule sched = qm_detail::schedule(weights_, n, index, credit, (!fused && !disjoint) || interrupts());
  if (fused) {
    // done: scheduler state and interrupts below
  } else if (disjoint && hmem) {
    // one mirror: the queue pairs one after another (their buffers are apart,
    // so the order does not matter)
    for (std::size_t q = 0; q < Q; ++q) {
      if (!n[q]) continue;
      const QueuePairStats b = qps_[q]->stage.stats();
      qps_[q]->stage.process_batch(*hmem, batches[q].tx, batches[q].rx, out[q], stream);
      add_delta(qps_[q]->stats, qps_[q]->stage.stats(), b);
    }
  } else if (disjoint) {
    const DeviceHostMemory& mem = dmem;
    // each queue pair's results do not depend on the interleaving: every
    // queue's batch on its own stage, all in flight at once — unless two share
    // an RssEngine (its statistics are not shared across job threads)
    std::set<const RssEngine*> engines;
    bool shared = false;
    for (std::size_t q = 0; q < Q; ++q)
      if (n[q] && qps_[q]->config.rss) shared |= !engines.insert(qps_[q]->config.rss).second;
    std::vector<QueuePairStats> before(Q);
    for (std::size_t q = 0; q < Q; ++q) before[q] = qps_[q]->stage.stats();
    if (!shared) {
      for (std::size_t q = 0; q < Q; ++q)  // contexts made on this thread before the jobs read them
        if (n[q] && qps_[q]->config.rss && qps_[q]->config.device_resolve) (void) qps_[q]->config.rss->device_context(stream);
      Streams& T = *streams_;
      T.ensure(Q);
      auto ok = [](int st, const char* what) {
        if (st != NICGPU_OK) throw GpuError(std::string("BatchedQueueManager: ") + what, st);
      };
      ok(nicgpu_event_record(T.fork, stream), "nicgpu_event_record");  // the caller's earlier work first
      std::vector<std::size_t> sent;
      std::exception_ptr err;
      for (std::size_t q = 0; q < Q && !err; ++q) {
        if (!n[q]) continue;
        try {
          ok(nicgpu_stream_wait_event(T.s[q], T.fork), "nicgpu_stream_wait_event");
          qps_[q]->stage.submit(mem, batches[q].tx, batches[q].rx, T.s[q]);
          sent.push_back(q);
        } catch (...) {
          err = std::current_exception();
        }
      }
      for (const std::size_t q : sent) {  // every submitted batch is collected, whatever throws
        try {
          qps_[q]->stage.collect(out[q]);
          // the caller's stream continues after every queue pair's work
          ok(nicgpu_event_record(T.joined[q], T.s[q]), "nicgpu_event_record");
          ok(nicgpu_stream_wait_event(stream, T.joined[q]), "nicgpu_stream_wait_event");
        } catch (...) {
          if (!err) err = std::current_exception();
        }
      }
      if (err) {
        // the stages whose batches went through advanced their own statistics
        // (a stage commits a batch's stats only when it completes): carry them
        // over before rethrowing; the scheduler state stays where it was, as
        // no schedule was completed
        for (std::size_t q = 0; q < Q; ++q) add_delta(qps_[q]->stats, qps_[q]->stage.stats(), before[q]);
        std::rethrow_exception(err);
      }
    } else {
      for (std::size_t q = 0; q < Q; ++q)
        if (n[q]) qps_[q]->stage.process_batch(mem, batches[q].tx, batches[q].rx, out[q], stream);
    }
    for (std::size_t q = 0; q < Q; ++q) add_delta(qps_[q]->stats, qps_[q]->stage.stats(), before[q]);
  } else {
    // the interleaving decides the bytes: the reference's order, run by run,
    // each run one host-path batch of its queue
    std::vector<std::size_t> ti(Q, 0), ri(Q, 0);
    RxBatchResult part;
    for (const QueueSchedule::Run& run : sched.runs) {
      Queue& qp = *qps_[run.queue];
      BatchedQueuePair& h = qp.host_stage();
      if (hmem) h.share_image(*fused_);
      const QueuePairStats b = h.stats();
      const QueueBatch& B = batches[run.queue];
      if (hmem) h.process_batch(*hmem, B.tx.subspan(ti[run.queue], run.count), B.rx.subspan(ri[run.queue]), part, stream);
      else h.process_batch(dmem, B.tx.subspan(ti[run.queue], run.count), B.rx.subspan(ri[run.queue]), part, stream);
      add_delta(qp.stats, h.stats(), b);
      append_result(out[run.queue], part);
      ti[run.queue] += run.count;
      ri[run.queue] += part.rx_consumed;
    }
  }
  index_ = index;
  credit_ = credit;
  advances_ += sched.advances;
  skips_ += sched.skips;
  replay(sched, out, stream);
  return sched;
}

bool BatchedQueueManager::interrupts() const {
  for (const auto& qp : qps_)
    if (qp->config.on_interrupt && (qp->config.enable_tx_interrupts || qp->config.enable_rx_interrupts)) return true;
  return false;
}

// interrupts in the order the reference's dispatcher sees them: run by run
void BatchedQueueManager::replay(const QueueSchedule& sched, const std::vector<RxBatchResult>& out, void* stream) {
  const std::size_t Q = qps_.size();
  if (interrupts()) {
    std::vector<std::vector<CompletionEntry>> htx(Q), hrx(Q);
    std::vector<std::span<const CompletionEntry>> txc(Q), rxc(Q);
    for (std::size_t q = 0; q < Q; ++q) {
      const RxBatchResult& r = out[q];
      if (r.timings.device && r.dev.tx_completions) {  // results_on_device: fetched for the callbacks
        htx[q].resize(r.dev.ntx);
        hrx[q].resize(r.dev.nrx);
        if (r.dev.ntx && nicgpu_memcpy_async(htx[q].data(), r.dev.tx_completions, r.dev.ntx * sizeof(CompletionEntry), stream) != NICGPU_OK)
          throw GpuError("process_batch: completion download", NICGPU_ERR_HIP);
        if (r.dev.nrx && nicgpu_memcpy_async(hrx[q].data(), r.dev.rx_completions, r.dev.nrx * sizeof(CompletionEntry), stream) != NICGPU_OK)
          throw GpuError("process_batch: completion download", NICGPU_ERR_HIP);
        if (nicgpu_stream_synchronize(stream) != NICGPU_OK) throw GpuError("process_batch: completion download", NICGPU_ERR_HIP);
        txc[q] = htx[q];
        rxc[q] = hrx[q];
      } else {
        txc[q] = r.tx_completions;
        rxc[q] = r.rx_completions;
      }
    }
    std::vector<rx_stage_detail::InterruptCursor> at(Q);
    for (const QueueSchedule::Run& run : sched.runs)
      rx_stage_detail::replay_interrupts(qps_[run.queue]->config, txc[run.queue], rxc[run.queue], at[run.queue], run.count);
  }
}

void BatchedQueueManager::reset() {
  index_ = 0;
  credit_ = weights_.empty() ? 0 : weights_.front();
  advances_ = skips_ = 0;
  for (auto& qp : qps_) {
    qp->stats = QueuePairStats{};
    qp->stage.reset_stats();
    if (qp->host) qp->host->reset_stats();
  }
}

QueueManagerStats BatchedQueueManager::stats() const {
  QueueManagerStats o{};
  for (const auto& qp : qps_) {  // aggregate_stats (:119-139): these 13 counters, then the scheduler's
    const QueuePairStats& s = qp->stats;
    o.total_tx_packets += s.tx_packets;
    o.total_rx_packets += s.rx_packets;
    o.total_tx_bytes += s.tx_bytes;
    o.total_rx_bytes += s.rx_bytes;
    o.total_drops_checksum += s.drops_checksum;
    o.total_drops_no_rx_desc += s.drops_no_rx_desc;
    o.total_drops_buffer_small += s.drops_buffer_small;
    o.total_tx_tso_segments += s.tx_tso_segments;
    o.total_tx_gso_segments += s.tx_gso_segments;
    o.total_tx_vlan_insertions += s.tx_vlan_insertions;
    o.total_rx_vlan_strips += s.rx_vlan_strips;
    o.total_rx_checksum_verified += s.rx_checksum_verified;
    o.total_rx_gro_aggregated += s.rx_gro_aggregated;
  }
  o.scheduler_advances = advances_;
  o.scheduler_skips = skips_;
  return o;
}

std::string BatchedQueueManager::stats_summary() const {
  const QueueManagerStats s = stats();
  std::ostringstream o;  // the text of queue_manager.cpp:102-117
  o << "qm tx_pkts=" << s.total_tx_packets << " rx_pkts=" << s.total_rx_packets << " tx_bytes=" << s.total_tx_bytes
    << " rx_bytes=" << s.total_rx_bytes << " drops_csum=" << s.total_drops_checksum
    << " drops_no_rx_desc=" << s.total_drops_no_rx_desc << " drops_buf_small=" << s.total_drops_buffer_small
    << " tx_tso_segs=" << s.total_tx_tso_segments << " tx_gso_segs=" << s.total_tx_gso_segments
    << " tx_vlan_ins=" << s.total_tx_vlan_insertions << " rx_vlan_strip=" << s.total_rx_vlan_strips
    << " rx_csum_ver=" << s.total_rx_checksum_verified << " rx_gro=" << s.total_rx_gro_aggregated
    << " sched_adv=" << s.scheduler_advances << " sched_skip=" << s.scheduler_skips;
  return o.str();
}

}  // namespace nic
