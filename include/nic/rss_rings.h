// rss_rings.h — RSS dispatch of the batched QueuePair stage
// into per-queue completion rings: nic::CompletionQueue
// (include/nic/completion_queue.h, src/completion_queue.cpp:30-53) once per
// RSS queue, on the device.  After a batch, every Success RX completion goes
// into the ring of its RSS queue in posting order, exactly as that queue's
// CompletionQueue::post_completion would take it one by one (a full ring
// refuses the entry and counts it); poll() is CompletionQueue::poll_completion.
// A batch whose results stayed in HBM (results_on_device) is posted from its
// device lists without leaving the device.
// Doorbells: the reference's post_completion rings Doorbell{queue_id,
// producer} after every post it accepts (completion_queue.cpp:30-41).  The
// device rings place a batch's entries in parallel; with set_doorbell() post()
// then rings the same sequence through a callback — one call per accepted
// entry, in the batch's posting order across queues, each with its queue's
// CompletionQueueConfig::queue_id and the producer index that post left.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <optional>
#include <span>
#include <utility>
#include <vector>

#include "nic/rx_stage.h"

struct nicgpu_cq_set;

namespace nic {

class RssCompletionRings {
public:
  struct State {
    std::uint32_t producer{0}, consumer{0}, count{0}, refused{0};
  };
  /// `queues` rings of `ring_size` entries on `device`.
  RssCompletionRings(std::size_t queues, std::size_t ring_size, int device = 0);
  ~RssCompletionRings();
  RssCompletionRings(const RssCompletionRings&) = delete;
  RssCompletionRings& operator=(const RssCompletionRings&) = delete;

  [[nodiscard]] std::size_t queues() const noexcept { return nq_; }
  [[nodiscard]] std::size_t ring_size() const noexcept { return ring_; }
  /// The Success RX completions of a batch with an RssEngine, queue by queue
  /// (RxBatchResult::dev lists when it kept its results on the device, else
  /// RxBatchResult::queues over rx_completions).  Queues past queues() throw.
  void post(const RxBatchResult& r, void* stream = nullptr);
  std::optional<CompletionEntry> poll(std::size_t q);
  std::vector<CompletionEntry> poll(std::size_t q, std::size_t max);
  [[nodiscard]] State state(std::size_t q) const;
  /// What Doorbell::ring receives per accepted post (DoorbellPayload{queue_id,
  /// data = producer}); queue_ids[q] is ring q's CompletionQueueConfig::queue_id
  /// (default q).  With a doorbell, post() synchronises `stream`.  An empty
  /// function turns it off.
  using DoorbellFn = std::function<void(std::uint16_t queue_id, std::uint32_t producer)>;
  void set_doorbell(DoorbellFn ring, std::vector<std::uint16_t> queue_ids = {});

private:
  DoorbellFn bell_;
  std::vector<std::uint16_t> bell_ids_;
  nicgpu_cq_set* cq_{nullptr};
  std::size_t nq_{0}, ring_{0};
  int device_{0};
  void* up_rxc_{nullptr};  // device copies of a host-result batch
  void* up_which_{nullptr};
  std::size_t cap_rxc_{0}, cap_which_{0};
};

namespace rss_rings_detail {
/// The doorbells one post rings: which[start[q] .. end[q]) are queue q's
/// completion indices in posting order (< n); before[q] its ring's state
/// before the post.  Entry k of list q is accepted while k < ring_size -
/// before[q].count and then rings (queue_ids[q], (before[q].producer + k + 1)
/// % ring_size); the doorbells come out in posting order (completion index),
/// as the reference's one-by-one posts ring them.
std::vector<std::pair<std::uint16_t, std::uint32_t>> doorbells(std::span<const std::uint32_t> which,
                                                               std::span<const std::uint32_t> start,
                                                               std::span<const std::uint32_t> end,
                                                               std::span<const RssCompletionRings::State> before,
                                                               std::size_t ring_size,
                                                               std::span<const std::uint16_t> queue_ids, std::size_t n);
}  // namespace rss_rings_detail

}  // namespace nic
