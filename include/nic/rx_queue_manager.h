// rx_queue_manager.h — nic::BatchedQueueManager: the reference's QueueManager
// (include/nic/queue_manager.h, src/queue_manager.cpp) over batches of the
// batched QueuePair stage (rx_stage.h).
//
// QueueManager::process_once (queue_manager.cpp:54-78) serves one TX
// descriptor of the queue pair at the scheduler's index — weighted round robin
// with credits: a queue keeps the turn for `weight` descriptors (0 counts as 1,
// :14-16) — and skips a queue whose process_once returns false (its TX ring is
// empty), counting scheduler_advances / scheduler_skips.  Draining it until it
// returns false over one batch per queue pair is what process_batch does:
//
//   * the schedule (which queue serves each descriptor, the advances, the
//     skips — including the final call that finds every ring empty, and the
//     index/credit carried to the next batch) is computed on the host from
//     the batch sizes alone: process_once returns true for every descriptor of
//     a batch (the stage's rings are not host-backed, so no pop or decode
//     fails);
//   * when no queue's RX buffer overlaps a byte another queue reads or writes,
//     each queue pair's results are independent of the order the scheduler
//     interleaves them in, so the queue pairs' batches are resolved as ONE
//     device batch: their TX batches and RX rings back to back, each queue
//     pair a segment with its own queue id, MTU and ring (the scan of the
//     ring positions restarted per segment), one plan / piece-sum / resolve /
//     delivery chain, the results, statistics and RSS dispatch lists split per
//     queue pair afterwards.  It needs the queue pairs' stage settings to agree
//     (device resolve on, results_on_device alike, RSS engines of equal key,
//     table and tuple — each engine still counts its own frames) and the
//     batch's buffers to be disjoint and settle on the device; otherwise each
//     queue's batch goes to its own BatchedQueuePair, all in flight at once;
//   * otherwise the interleaving decides the bytes (a queue writes into
//     another's TX buffer before or after it is read): the schedule is replayed
//     run by run, each run of one queue's consecutive descriptors a host-path
//     batch of that queue, in the reference's order;
//   * interrupt callbacks fire in the order the reference's single
//     InterruptDispatcher would see them: run by run, each run's descriptors
//     replayed from its queue's completions (rx_stage_detail::replay_interrupts).
//
// Statistics: queue_stats(i) is queue pair i's QueuePairStats, stats() their
// aggregate plus the scheduler counters exactly as aggregate_stats
// (:119-139), stats_summary() the same text as :102-117.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <optional>
#include <span>
#include <string>
#include <vector>

#include "nic/rx_stage.h"

#if __has_include("nic/queue_manager.h")
#include "nic/queue_manager.h"  // reference build: its QueueManagerStats
#else
namespace nic {
// Same members and order as include/nic/queue_manager.h:18-34.
struct QueueManagerStats {
  std::uint64_t total_tx_packets{0};
  std::uint64_t total_rx_packets{0};
  std::uint64_t total_tx_bytes{0};
  std::uint64_t total_rx_bytes{0};
  std::uint64_t total_drops_checksum{0};
  std::uint64_t total_drops_no_rx_desc{0};
  std::uint64_t total_drops_buffer_small{0};
  std::uint64_t total_tx_tso_segments{0};
  std::uint64_t total_tx_gso_segments{0};
  std::uint64_t total_tx_vlan_insertions{0};
  std::uint64_t total_rx_vlan_strips{0};
  std::uint64_t total_rx_checksum_verified{0};
  std::uint64_t total_rx_gro_aggregated{0};
  std::uint64_t scheduler_advances{0};
  std::uint64_t scheduler_skips{0};
};
}  // namespace nic
#endif

namespace nic {

/// QueueManagerConfig (queue_manager.h:14-16) for batched queue pairs.
struct BatchedQueueManagerConfig {
  std::vector<BatchedQueuePairConfig> queue_configs;
};

/// One queue pair's share of a batch: the TX descriptors to send and the
/// contents of its RX ring (rx[0] first; what a batch leaves unconsumed is the
/// caller's to pass again, first, with the next one).
struct QueueBatch {
  std::span<const TxDescriptor> tx;
  std::span<const RxDescriptor> rx;
};

/// The same with the descriptors already in device memory (a host-backed ring
/// in the image, a device-side producer): device pointers, read in stream
/// order after the caller's earlier work on the stream.
struct DeviceQueueBatch {
  const TxDescriptor* tx{nullptr};
  std::size_t ntx{0};
  const RxDescriptor* rx{nullptr};
  std::size_t nrx{0};
};

/// How one drain served the queues: runs of consecutive descriptors of one
/// queue, in order, and the scheduler counters it added.
struct QueueSchedule {
  struct Run {
    std::uint32_t queue;
    std::uint32_t count;
  };
  std::vector<Run> runs;
  std::uint64_t advances{0}, skips{0};
};

namespace qm_detail {
/// The scheduler of queue_manager.cpp:54-78 drained over `pending[q]`
/// descriptors per queue from (index, credit); both are advanced to where the
/// reference leaves them.  weights: already 0 -> 1.  want_runs false: only
/// the counters and (index, credit) — whole round-robin cycles are counted at
/// once instead of one run per turn (16 weight-1 queues of 64 K descriptors
/// make 1 M runs).
QueueSchedule schedule(std::span<const std::uint8_t> weights, std::span<const std::size_t> pending, std::size_t& index,
                       std::size_t& credit, bool want_runs = true);
/// No queue's RX buffer overlaps a byte another queue's TX or RX buffer
/// covers (clipped to the image, as the stage's own check).
bool queues_disjoint(std::size_t mem_size, std::span<const QueueBatch> batches);
}  // namespace qm_detail

class BatchedQueueManager {
public:
  explicit BatchedQueueManager(BatchedQueueManagerConfig config);
  ~BatchedQueueManager();
  BatchedQueueManager(const BatchedQueueManager&) = delete;
  BatchedQueueManager& operator=(const BatchedQueueManager&) = delete;

  [[nodiscard]] std::size_t queue_count() const noexcept { return qps_.size(); }
  /// The queue pair's stage (its config has no interrupt callback: the
  /// manager fires them, in the scheduler's order); nullptr past the end.
  /// Its own stats() count only the batches that ran per queue pair; the
  /// queue pair's statistics are queue_stats().
  [[nodiscard]] BatchedQueuePair* queue(std::size_t index) noexcept;
  [[nodiscard]] std::optional<QueuePairStats> queue_stats(std::size_t index) const noexcept;

  /// QueueManager::process_once until it returns false, over batches[q] for
  /// queue pair q (batches.size() == queue_count()); results into out[q]
  /// (resized).  Synchronises `stream`.  Returns the schedule it served
  /// (its runs only when they were needed: the queues' buffers overlap or an
  /// interrupt callback is set; the counters always).
  /// If a queue pair's batch throws, the statistics of the queue pairs whose
  /// batches completed are kept (their writes are in memory), the scheduler
  /// state (index, credit, advances, skips) is not advanced, and the
  /// exception propagates.
  QueueSchedule process_batch(const DeviceHostMemory& mem, std::span<const QueueBatch> batches,
                              std::vector<RxBatchResult>& out, void* stream = nullptr);
  /// The same against the reference's HostMemory (host_memory.h:49-73), as
  /// BatchedQueuePair::process_batch(HostMemory&, ...): one HBM mirror for all
  /// queue pairs, every queue's TX bytes staged up, the delivered bytes written
  /// back; when the fused batch does not apply, the queue pairs run one after
  /// another on it.
  QueueSchedule process_batch(HostMemory& mem, std::span<const QueueBatch> batches, std::vector<RxBatchResult>& out,
                              void* stream = nullptr);
  /// Descriptors in device memory: the fused batch when the device finds the
  /// whole concatenated batch disjoint (every queue pair's buffers apart from
  /// every other's); otherwise the descriptors come down once and the host
  /// path of process_batch above decides.
  QueueSchedule process_batch(const DeviceHostMemory& mem, std::span<const DeviceQueueBatch> batches,
                              std::vector<RxBatchResult>& out, void* stream = nullptr);
  /// How the last process_batch ran: 1 = one fused device batch, 0 = per
  /// queue pair (device stages or the reference's interleaving on the host).
  [[nodiscard]] int last_fused() const noexcept { return last_fused_; }

  /// Scheduler index/credit/counters and every queue pair's statistics
  /// (QueueManager::reset, :80-93; the rings are the caller's).
  void reset();
  [[nodiscard]] QueueManagerStats stats() const;
  [[nodiscard]] std::string stats_summary() const;

private:
  QueueSchedule run(const DeviceHostMemory& dmem, HostMemory* hmem, std::span<const QueueBatch> batches,
                    std::vector<RxBatchResult>& out, void* stream);
  bool fusable() const;
  void replay(const QueueSchedule& sched, const std::vector<RxBatchResult>& out, void* stream);
  bool interrupts() const;  // some queue pair has an interrupt callback that fires
  struct Queue;
  std::vector<std::unique_ptr<Queue>> qps_;
  std::unique_ptr<BatchedQueuePair> fused_;  // every queue pair's batch as one (queue 0's settings)
  int last_fused_{0};
  struct Streams;  // a stream per queue pair, forked from and joined into the caller's
  std::unique_ptr<Streams> streams_;
  std::vector<std::uint8_t> weights_;
  std::size_t index_{0}, credit_{0};
  std::uint64_t advances_{0}, skips_{0};
};

}  // namespace nic
