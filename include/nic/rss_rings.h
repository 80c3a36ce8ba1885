// rss_rings.h — RSS dispatch of the batched QueuePair stage
// into per-queue completion rings: nic::CompletionQueue
// (include/nic/completion_queue.h, src/completion_queue.cpp:30-53) once per
// RSS queue, on the device.  After a batch, every Success RX completion goes
// into the ring of its RSS queue in posting order, exactly as that queue's
// CompletionQueue::post_completion would take it one by one (a full ring
// refuses the entry and counts it); poll() is CompletionQueue::poll_completion.
// A batch whose results stayed in HBM (results_on_device) is posted from its
// device lists without leaving the device.
// No doorbell: the reference's post_completion rings Doorbell{queue_id,
// producer} after every post (completion_queue.cpp:38-39); the device rings do
// not.  A caller that needs the doorbell sequence derives it from the rings'
// producers (state()): the last doorbell of a batch on queue q carries
// state(q).producer.
#pragma once
#include <cstddef>
#include <cstdint>
#include <optional>
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

private:
  nicgpu_cq_set* cq_{nullptr};
  std::size_t nq_{0}, ring_{0};
  int device_{0};
  void* up_rxc_{nullptr};  // device copies of a host-result batch
  void* up_which_{nullptr};
  std::size_t cap_rxc_{0}, cap_which_{0};
};

}  // namespace nic
