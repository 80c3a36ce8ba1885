// cq_doorbell_test.cpp — the doorbells of nic::RssCompletionRings against the
// reference CompletionQueue (tests/golden/cq_rings.json: gen_cq in
// oracle/gen_golden.cpp posts three skewed batches through reference
// CompletionQueues whose Doorbells record every ring, completion_queue.cpp:
// 30-41, with polls between the batches).
//
//   cq_doorbell_test cpu <flat.txt>   rss_rings_detail::doorbells over the
//       fixture's lists, ring states carried across batches and polls
//   cq_doorbell_test gpu <flat.txt>   RssCompletionRings::post with a doorbell
//       callback (device rings), then the polls the fixture makes
//
// flat.txt is the fixture flattened by tests/test_cq_rings.py.
#undef NDEBUG
#include <cassert>
#include <cstdio>
#include <fstream>
#include <string>
#include <utility>
#include <vector>

#include "nic/rss_rings.h"

using namespace nic;

namespace {

struct Batch {
  std::vector<std::uint32_t> status, rss_queue, didx, qid, segs, vlan, verified, posted, db_queue, db_data, polls;
};

struct Fixture {
  std::size_t Q = 0, R = 0, base = 0;
  std::vector<Batch> batches;
};

std::vector<std::uint32_t> read_arr(std::ifstream& f) {
  std::size_t n = 0;
  f >> n;
  std::vector<std::uint32_t> v(n);
  for (auto& x : v) f >> x;
  return v;
}

Fixture read_fixture(const char* path) {
  std::ifstream f(path);
  assert(f);
  Fixture F;
  std::size_t nb = 0;
  f >> F.Q >> F.R >> F.base >> nb;
  for (std::size_t b = 0; b < nb; ++b) {
    Batch B;
    for (auto* v : {&B.status, &B.rss_queue, &B.didx, &B.qid, &B.segs, &B.vlan, &B.verified, &B.posted, &B.db_queue,
                    &B.db_data, &B.polls})
      *v = read_arr(f);
    F.batches.push_back(std::move(B));
  }
  assert(f);
  return F;
}

// Success completions grouped by RSS queue in posting order (nicgpu_qp_group's lists)
void lists(const Fixture& F, const Batch& B, std::vector<std::uint32_t>& which, std::vector<std::uint32_t>& start,
           std::vector<std::uint32_t>& end) {
  which.clear();
  start.assign(F.Q, 0);
  end.assign(F.Q, 0);
  for (std::size_t q = 0; q < F.Q; ++q) {
    start[q] = static_cast<std::uint32_t>(which.size());
    for (std::size_t j = 0; j < B.status.size(); ++j)
      if (B.status[j] == 0 && B.rss_queue[j] == q) which.push_back(static_cast<std::uint32_t>(j));
    end[q] = static_cast<std::uint32_t>(which.size());
  }
}

void expect_bells(const Batch& B, const std::vector<std::pair<std::uint16_t, std::uint32_t>>& got, std::size_t b) {
  if (got.size() != B.db_queue.size()) {
    std::fprintf(stderr, "batch %zu: %zu doorbells, the reference rang %zu\n", b, got.size(), B.db_queue.size());
    assert(false);
  }
  for (std::size_t k = 0; k < got.size(); ++k)
    if (got[k].first != B.db_queue[k] || got[k].second != B.db_data[k]) {
      std::fprintf(stderr, "batch %zu doorbell %zu: (%u, %u) vs (%u, %u)\n", b, k, got[k].first, got[k].second,
                   B.db_queue[k], B.db_data[k]);
      assert(false);
    }
}

std::vector<std::uint16_t> ids(const Fixture& F) {
  std::vector<std::uint16_t> v(F.Q);
  for (std::size_t q = 0; q < F.Q; ++q) v[q] = static_cast<std::uint16_t>(F.base + q);
  return v;
}

int run_cpu(const Fixture& F) {
  std::vector<RssCompletionRings::State> st(F.Q);
  const auto qids = ids(F);
  std::size_t total = 0;
  for (std::size_t b = 0; b < F.batches.size(); ++b) {
    const Batch& B = F.batches[b];
    std::vector<std::uint32_t> which, start, end;
    lists(F, B, which, start, end);
    const auto got = rss_rings_detail::doorbells(which, start, end, st, F.R, qids, B.status.size());
    expect_bells(B, got, b);
    total += got.size();
    for (std::size_t q = 0; q < F.Q; ++q) {  // the post, then the consumer's polls
      const std::size_t acc = std::min<std::size_t>(end[q] - start[q], F.R - st[q].count);
      st[q].producer = static_cast<std::uint32_t>((st[q].producer + acc) % F.R);
      st[q].count += static_cast<std::uint32_t>(acc);
      st[q].count -= std::min<std::uint32_t>(st[q].count, B.polls[q]);
    }
  }
  std::printf("cq_doorbell_test cpu: ok (%zu doorbells in the reference's order)\n", total);
  return 0;
}

int run_gpu(const Fixture& F) {
  RssCompletionRings rings(F.Q, F.R, 0);
  std::vector<std::pair<std::uint16_t, std::uint32_t>> rung;
  rings.set_doorbell([&](std::uint16_t q, std::uint32_t p) { rung.emplace_back(q, p); }, ids(F));
  std::size_t total = 0;
  for (std::size_t b = 0; b < F.batches.size(); ++b) {
    const Batch& B = F.batches[b];
    RxBatchResult r;
    for (std::size_t j = 0; j < B.status.size(); ++j) {
      CompletionEntry e{};
      e.queue_id = static_cast<std::uint16_t>(B.qid[j]);
      e.descriptor_index = static_cast<std::uint16_t>(B.didx[j]);
      e.status = B.status[j];
      e.segments_produced = static_cast<std::uint16_t>(B.segs[j]);
      e.vlan_tag = static_cast<std::uint16_t>(B.vlan[j]);
      e.checksum_verified = B.verified[j] != 0;
      r.rx_completions.push_back(e);
    }
    std::vector<std::uint32_t> which, start, end;
    lists(F, B, which, start, end);
    r.queues.resize(F.Q);
    for (std::size_t q = 0; q < F.Q; ++q) r.queues[q].assign(which.begin() + start[q], which.begin() + end[q]);
    rung.clear();
    rings.post(r);
    expect_bells(B, rung, b);
    total += rung.size();
    for (std::size_t q = 0; q < F.Q; ++q) (void) rings.poll(q, B.polls[q]);
  }
  std::printf("cq_doorbell_test gpu: ok (%zu doorbells in the reference's order)\n", total);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s cpu|gpu flat.txt\n", argv[0]);
    return 2;
  }
  const Fixture F = read_fixture(argv[2]);
  return std::string(argv[1]) == "gpu" ? run_gpu(F) : run_cpu(F);
}
