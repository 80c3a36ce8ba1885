// cpu_backend.h — test-only CPU implementation of rx_stage_detail::Backend, so
// that run_batch (BatchedQueuePair's driver: sub-batches, write layers, RSS)
// runs without a GPU against the reference QueuePair.  Piece sums and tuples
// come from the oracle (test infrastructure, never the product path); RSS goes
// through the host RssEngine::select_queue, i.e. one reference-semantics call
// per frame.
//
// Gathers run a layer's writes in REVERSE posting order and read sources from
// the image as it was when the gather started (or from the snapshot): a layer
// that wrongly held two overlapping writes, or a missing snapshot, then shows
// up as a mismatch against the reference's in-order writes.
#pragma once

#include <cstring>
#include <span>
#include <vector>

#include "nic/rss.h"
#include "nic/rx_stage.h"
#include "oracle.h"

namespace nic::test {

class CpuBackend final : public rx_stage_detail::Backend {
public:
  CpuBackend(std::vector<std::uint8_t>& image, RssEngine* rss, TupleSpec tuple)
      : image_(image), rss_(rss), tuple_(tuple) {
    if (rss_) probe_ = *rss_;  // same key and table, for the hash values
  }

  std::span<const std::uint16_t> piece_sums(std::span<const rx_stage_detail::Piece> pieces) override {
    cs_.resize(pieces.size());
    for (std::size_t i = 0; i < pieces.size(); ++i) {
      if (pieces[i].len > 65535u) std::abort();
      cs_[i] = oracle_compute_checksum(image_.data() + pieces[i].addr, pieces[i].len);
    }
    ++sum_calls;
    return cs_;
  }

  void snapshot() override {
    copy_ = image_;
    ++snapshots;
  }

  void gather(std::span<const rx_stage_detail::SegmentWrite> writes, bool from_copy) override {
    if (from_copy && copy_.size() != image_.size()) std::abort();
    // the writes read the image as it was before any of them: a copy, unless
    // no write's destination meets another's source (small batches checked
    // pair by pair; the copy is the whole image)
    bool meet = false;
    if (!from_copy && writes.size() <= 256) {
      for (const auto& w : writes) {
        const std::uint64_t d0 = w.dst, d1 = w.dst + w.prefix_len + w.len_a + w.len_b;
        for (const auto& u : writes)
          meet |= (u.len_a && u.src_a < d1 && d0 < u.src_a + u.len_a) || (u.len_b && u.src_b < d1 && d0 < u.src_b + u.len_b);
      }
    } else {
      meet = !from_copy;
    }
    const std::vector<std::uint8_t> before = meet ? image_ : std::vector<std::uint8_t>();
    const std::vector<std::uint8_t>& src = from_copy ? copy_ : meet ? before : image_;
    for (std::size_t k = writes.size(); k-- > 0;) {
      const auto& w = writes[k];
      const std::uint64_t total = std::uint64_t{w.prefix_len} + w.len_a + w.len_b;
      if (w.dst > image_.size() || total > image_.size() - w.dst) continue;  // skipped, as the kernel does
      std::uint64_t d = w.dst;
      for (std::uint32_t j = 0; j < w.prefix_len; ++j) image_[d++] = static_cast<std::uint8_t>(w.prefix >> (8 * j));
      if (w.len_a) std::memcpy(image_.data() + d, src.data() + w.src_a, w.len_a);
      if (w.len_b) std::memcpy(image_.data() + d + w.len_a, src.data() + w.src_b, w.len_b);
    }
    ++gathers;
  }

  void descriptors(std::uint64_t tx_at, std::span<TxDescriptor> tx, std::uint64_t rx_at,
                   std::span<RxDescriptor> rx) override {
    if (tx_at != ~0ull && !tx.empty()) std::memcpy(static_cast<void*>(tx.data()), image_.data() + tx_at, tx.size_bytes());
    if (rx_at != ~0ull && !rx.empty()) std::memcpy(static_cast<void*>(rx.data()), image_.data() + rx_at, rx.size_bytes());
    ++refetches;
  }

  std::uint64_t* frame_desc(std::size_t n) override {
    desc_.resize(n);
    return desc_.data();
  }

  void rss(std::size_t n, const std::uint32_t*& hash, const std::uint16_t*& queue) override {
    h_.resize(n);
    q_.resize(n);
    const int mode = tuple_.mode == TupleMode::Raw ? ORACLE_TUPLE_RAW
                     : tuple_.mode == TupleMode::Auto ? ORACLE_TUPLE_AUTO
                                                       : ORACLE_TUPLE_NONE;
    for (std::size_t i = 0; i < n; ++i) {
      const std::uint64_t off = desc_[i] & ((1ull << 40) - 1), len = desc_[i] >> 40;
      std::uint8_t t[64];
      const std::size_t tl = oracle_extract_tuple(image_.data() + off, len, mode, tuple_.raw_offset, tuple_.raw_length, t);
      const std::span<const std::uint8_t> tuple(t, tl);
      h_[i] = probe_.hash(tuple);
      q_[i] = *rss_->select_queue(tuple);
    }
    hash = h_.data();
    queue = q_.data();
    ++rss_calls;
  }

  std::size_t sum_calls = 0, snapshots = 0, gathers = 0, rss_calls = 0, refetches = 0;

private:
  std::vector<std::uint8_t>& image_;
  RssEngine* rss_;
  TupleSpec tuple_;
  RssEngine probe_;
  std::vector<std::uint8_t> copy_;
  std::vector<std::uint16_t> cs_, q_;
  std::vector<std::uint32_t> h_;
  std::vector<std::uint64_t> desc_;
};

}  // namespace nic::test
