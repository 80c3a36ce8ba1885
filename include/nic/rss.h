// nic/rss.h — Toeplitz RSS engine of the smart_nic model.
//
// Drop-in for rosslwheeler/smart_nic include/nic/rss.h:13-48: the same
// RssConfig / RssStats / RssEngine public surface and semantics
// (src/rss.cpp:17-114) — 20-byte default key, 128-entry all-zero default
// table, queue = table[hash % table.size()], Toeplitz windows taken at key bit
// (bit + k) % key_bits (wraps for inputs longer than the key), stats counting
// every hash() and select_queue() call, queue_hits indexed by table index and
// sized only at construction / reset_stats().  Like the reference, the const
// methods update mutable stats, so one engine must not be shared by threads.
//
// Added: select_queue_batch(), the same classification for every packet of a
// device-resident batch in one GPU launch (fused with the RX checksum), with
// the stats updated exactly as the equivalent sequence of select_queue calls;
// select_queue_batch_enqueue() / account_batch(), the same split into an
// enqueue-only launch and a later stats update, for pipelines.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <optional>
#include <span>
#include <vector>

#include "nic/gpu_batch.h"

struct nicgpu_rss_ctx;  // nicgpu.h

namespace nic {

struct RssConfig {
  std::vector<std::uint8_t> key;     ///< Toeplitz key bytes
  std::vector<std::uint16_t> table;  ///< indirection table: hash % size -> queue id
};

struct RssStats {
  std::uint64_t hashes{0};
  std::vector<std::uint64_t> queue_hits;  ///< hits per table index
};

namespace detail {
struct RssGpuState;
struct RssHostLut;
}  // namespace detail

class RssEngine {
public:
  RssEngine();
  explicit RssEngine(RssConfig config);

  void set_key(std::vector<std::uint8_t> key);
  void set_table(std::vector<std::uint16_t> table);

  [[nodiscard]] std::uint32_t hash(std::span<const std::uint8_t> data) const;

  /// Queue for `data`; nullopt only for an empty table (never after construction).
  [[nodiscard]] std::optional<std::uint16_t> select_queue(std::span<const std::uint8_t> data) const;

  [[nodiscard]] const RssConfig& config() const noexcept { return config_; }
  [[nodiscard]] const RssStats& stats() const noexcept { return stats_; }
  void reset_stats() noexcept;

  /// GPU batch (new): for every packet i of `batch`, extract the tuple per
  /// `tuple`, then out.hash[i] = hash(tuple), out.queue[i] = table[hash % n],
  /// and out.checksum[i] = compute_checksum(frame i) in the same pass.  Runs on
  /// the current HIP device; stats are updated as if select_queue had been
  /// called once per packet (hashes += count, queue_hits[idx] += hits for
  /// idx < queue_hits.size()), which requires waiting for the launch: the call
  /// is synchronous on `stream` unless update_stats is false.  Throws
  /// nic::GpuError.  Any key length hashes as select_queue does (keys over
  /// NICGPU_MAX_KEY = 256 B are truncated for the device, which is exact); a
  /// table over NICGPU_MAX_TABLE = 2^24 entries throws (NICGPU_ERR_INVALID)
  /// before any device work, where select_queue would accept it.
  void select_queue_batch(const DevicePacketBatch& batch, const TupleSpec& tuple,
                          const RxBatchOutputs& out, void* stream = nullptr,
                          bool update_stats = true) const;

  /// Pipelined form (new): select_queue_batch over the first min(batch.count,
  /// *count_dev) packets, the count read on the device (a uint64 an earlier
  /// launch of `stream` wrote), enqueued without waiting.  Per-table-index hits
  /// are added into `hits_dev` (table size u64, caller-owned); the stats change
  /// only when the caller hands the downloaded count and hits to
  /// account_batch().  Throws nic::GpuError.
  void select_queue_batch_enqueue(const DevicePacketBatch& batch, const std::uint64_t* count_dev,
                                  const TupleSpec& tuple, const RxBatchOutputs& out,
                                  std::uint64_t* hits_dev, void* stream = nullptr) const;
  /// The stats of `count` select_queue calls whose table-index hits are
  /// `hits` (hashes += count, queue_hits[i] += hits[i] for i < queue_hits.size()).
  void account_batch(std::uint64_t count, std::span<const std::uint64_t> hits) const;

  /// The device key LUT + table on the current HIP device (created on first
  /// use; valid while the engine lives with this key and table), for fused
  /// launches such as nicgpu_qp_deliver.  Throws nic::GpuError.
  [[nodiscard]] const nicgpu_rss_ctx* device_context(void* stream = nullptr) const;

private:
  RssConfig config_;
  mutable RssStats stats_;
  mutable std::shared_ptr<detail::RssGpuState> gpu_;      // device key LUT + table (lazy)
  mutable std::shared_ptr<const detail::RssHostLut> lut_;  // host byte LUT (lazy)

  [[nodiscard]] std::uint32_t toeplitz_hash(std::span<const std::uint8_t> key,
                                            std::span<const std::uint8_t> data) const;
  void ensure_defaults();
  void ensure_gpu(void* stream) const;  // device key LUT + table on the current device
};

}  // namespace nic
