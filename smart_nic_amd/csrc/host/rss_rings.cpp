// rss_rings.cpp — nic::RssCompletionRings (include/nic/rss_rings.h) over the
// C-ABI's device rings (nicgpu_cq_*, csrc/cq.hip).
#include "nic/rss_rings.h"

#include <algorithm>
#include <stdexcept>
#include <string>

#include "nic/gpu_batch.h"
#include "nicgpu.h"

namespace nic {

namespace {
void ok(int st, const char* what) {
  if (st != NICGPU_OK) throw GpuError(std::string("RssCompletionRings: ") + what + ": " + nicgpu_strerror(st), st);
}
static_assert(sizeof(CompletionEntry) == sizeof(nicgpu_completion), "CompletionEntry is the C-ABI record");

// The rings' device current for a scope (the staging buffers of post() live
// on it, whatever device the calling thread has selected).
struct OnDevice {
  int prev = -1;
  explicit OnDevice(int dev) {
    ok(nicgpu_get_device(&prev), "nicgpu_get_device");
    if (prev != dev) ok(nicgpu_set_device(dev), "nicgpu_set_device");
  }
  ~OnDevice() {
    int cur = -1;
    if (prev >= 0 && nicgpu_get_device(&cur) == NICGPU_OK && cur != prev) (void) nicgpu_set_device(prev);
  }
};
}  // namespace

RssCompletionRings::RssCompletionRings(std::size_t queues, std::size_t ring_size, int device)
    : nq_(queues), ring_(ring_size), device_(device) {
  ok(nicgpu_cq_create(&cq_, device, queues, ring_size), "nicgpu_cq_create");
}

RssCompletionRings::~RssCompletionRings() {
  int prev = -1;
  const bool switched = (up_rxc_ || up_which_) && nicgpu_get_device(&prev) == NICGPU_OK && prev != device_ &&
                        nicgpu_set_device(device_) == NICGPU_OK;
  if (up_rxc_) (void) nicgpu_free(up_rxc_);
  if (up_which_) (void) nicgpu_free(up_which_);
  if (switched) (void) nicgpu_set_device(prev);
  if (cq_) (void) nicgpu_cq_destroy(cq_);
}

namespace rss_rings_detail {
std::vector<std::pair<std::uint16_t, std::uint32_t>> doorbells(std::span<const std::uint32_t> which,
                                                               std::span<const std::uint32_t> start,
                                                               std::span<const std::uint32_t> end,
                                                               std::span<const RssCompletionRings::State> before,
                                                               std::size_t ring_size,
                                                               std::span<const std::uint16_t> queue_ids, std::size_t n) {
  // at[j] = the doorbell completion j rings (queue + 1, producer), 0: none
  std::vector<std::pair<std::uint32_t, std::uint32_t>> at(n, {0u, 0u});
  std::size_t rung = 0;
  for (std::size_t q = 0; q < start.size(); ++q) {
    const std::size_t room = ring_size > before[q].count ? ring_size - before[q].count : 0;
    const std::size_t m = std::min<std::size_t>(end[q] - start[q], room);
    for (std::size_t k = 0; k < m; ++k) {
      const std::uint32_t j = which[start[q] + k];
      if (j >= n) throw std::out_of_range("doorbells: completion index past the batch");
      at[j] = {static_cast<std::uint32_t>(q) + 1u, static_cast<std::uint32_t>((before[q].producer + k + 1) % ring_size)};
    }
    rung += m;
  }
  std::vector<std::pair<std::uint16_t, std::uint32_t>> out;
  out.reserve(rung);
  for (const auto& [q1, p] : at)
    if (q1) out.emplace_back(q1 - 1 < queue_ids.size() ? queue_ids[q1 - 1] : static_cast<std::uint16_t>(q1 - 1), p);
  return out;
}
}  // namespace rss_rings_detail

void RssCompletionRings::set_doorbell(DoorbellFn ring, std::vector<std::uint16_t> queue_ids) {
  if (!queue_ids.empty() && queue_ids.size() != nq_)
    throw std::invalid_argument("RssCompletionRings::set_doorbell: one queue id per ring");
  bell_ = std::move(ring);
  bell_ids_ = std::move(queue_ids);
}

void RssCompletionRings::post(const RxBatchResult& r, void* stream) {
  // with a doorbell: the rings' state before, then the accepted posts rung in
  // the batch's posting order once the entries are placed
  std::vector<State> before;
  if (bell_) {
    std::vector<std::uint32_t> s(4 * nq_);
    ok(nicgpu_cq_state(cq_, s.data(), stream), "nicgpu_cq_state");
    before.resize(nq_);
    for (std::size_t q = 0; q < nq_; ++q) before[q] = State{s[q], s[nq_ + q], s[2 * nq_ + q], s[3 * nq_ + q]};
  }
  auto ring_bells = [&](std::span<const std::uint32_t> which, std::span<const std::uint32_t> start,
                        std::span<const std::uint32_t> end, std::size_t n) {
    if (!bell_) return;
    for (const auto& [qid, p] : rss_rings_detail::doorbells(which, start, end, before, ring_, bell_ids_, n)) bell_(qid, p);
  };
  if (r.dev.rx_completions && r.dev.queue_which) {  // results in HBM: the device lists
    const std::size_t nl = r.dev.queue_start.size();
    if (nl > nq_) throw std::invalid_argument("RssCompletionRings::post: more RSS queues than rings");
    ok(nicgpu_cq_post(cq_, reinterpret_cast<const nicgpu_completion*>(r.dev.rx_completions), r.dev.queue_which,
                      r.dev.queue_start.data(), r.dev.queue_end.data(), nl, stream),
       "nicgpu_cq_post");
    if (bell_) {  // the lists come down for the order
      std::size_t m = 0;
      for (std::size_t q = 0; q < nl; ++q) m = std::max<std::size_t>(m, r.dev.queue_end[q]);
      std::vector<std::uint32_t> which(m);
      if (m) {
        ok(nicgpu_memcpy_async(which.data(), r.dev.queue_which, m * sizeof(std::uint32_t), stream), "nicgpu_memcpy_async");
        ok(nicgpu_stream_synchronize(stream), "nicgpu_stream_synchronize");
      }
      ring_bells(which, r.dev.queue_start, r.dev.queue_end, r.dev.nrx);
    }
    return;
  }
  // host results: the lists and completions go up once, into staging buffers
  // on the rings' device
  const OnDevice on(device_);
  const std::size_t nl = r.queues.size();
  if (nl > nq_) throw std::invalid_argument("RssCompletionRings::post: more RSS queues than rings");
  std::vector<std::uint32_t> which, start(nl), end(nl);
  for (std::size_t q = 0; q < nl; ++q) {
    start[q] = static_cast<std::uint32_t>(which.size());
    which.insert(which.end(), r.queues[q].begin(), r.queues[q].end());
    end[q] = static_cast<std::uint32_t>(which.size());
  }
  const std::size_t n = r.rx_completions.size();
  auto grow = [](void*& p, std::size_t& cap, std::size_t bytes) {
    if (bytes <= cap) return;
    if (p) (void) nicgpu_free(p);
    p = nullptr;
    cap = 0;
    ok(nicgpu_malloc(&p, bytes), "nicgpu_malloc");
    cap = bytes;
  };
  grow(up_rxc_, cap_rxc_, std::max<std::size_t>(n, 1) * sizeof(CompletionEntry));
  grow(up_which_, cap_which_, std::max<std::size_t>(which.size(), 1) * sizeof(std::uint32_t));
  if (n) ok(nicgpu_memcpy_async(up_rxc_, r.rx_completions.data(), n * sizeof(CompletionEntry), stream), "nicgpu_memcpy_async");
  if (!which.empty())
    ok(nicgpu_memcpy_async(up_which_, which.data(), which.size() * sizeof(std::uint32_t), stream), "nicgpu_memcpy_async");
  ok(nicgpu_cq_post(cq_, static_cast<const nicgpu_completion*>(up_rxc_), static_cast<const std::uint32_t*>(up_which_),
                    start.data(), end.data(), nl, stream),
     "nicgpu_cq_post");
  ring_bells(which, start, end, n);
}

std::optional<CompletionEntry> RssCompletionRings::poll(std::size_t q) {
  auto v = poll(q, 1);
  if (v.empty()) return std::nullopt;
  return v.front();
}

std::vector<CompletionEntry> RssCompletionRings::poll(std::size_t q, std::size_t max) {
  if (q >= nq_) throw std::out_of_range("RssCompletionRings::poll: no such queue");
  std::vector<CompletionEntry> out(std::min(max, ring_));
  std::size_t got = 0;
  ok(nicgpu_cq_poll(cq_, static_cast<std::uint32_t>(q), reinterpret_cast<nicgpu_completion*>(out.data()), out.size(), &got,
                    nullptr),
     "nicgpu_cq_poll");
  out.resize(got);
  return out;
}

RssCompletionRings::State RssCompletionRings::state(std::size_t q) const {
  if (q >= nq_) throw std::out_of_range("RssCompletionRings::state: no such queue");
  std::vector<std::uint32_t> s(4 * nq_);
  ok(nicgpu_cq_state(cq_, s.data(), nullptr), "nicgpu_cq_state");
  return State{s[q], s[nq_ + q], s[2 * nq_ + q], s[3 * nq_ + q]};
}

}  // namespace nic
