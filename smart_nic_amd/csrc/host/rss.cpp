// rss.cpp — nic::RssEngine (host per-packet path + GPU batch path).
//
// Semantics follow the reference src/rss.cpp:17-114 exactly (defaults, stats,
// the queue_hits guard, `(bit + k) % key_bits` key wrap); the host hash is
// computed with a per-key table of 32-bit key windows (W[b] = key bits
// b..b+31 mod key_bits) and a per-byte lookup table, not the reference's
// bit-serial loop: h = XOR over set data bits b of W[b mod key_bits].
#include "nic/rss.h"

#include <array>
#include <cstring>
#include <string>

#include "nicgpu.h"

namespace nic {
namespace {

constexpr std::uint8_t kDefaultKey[20] = {0x6D, 0x5A, 0x56, 0x6B, 0x65, 0x4E, 0x67, 0x6E, 0x67, 0x55,
                                          0x6A, 0x6B, 0x61, 0x4F, 0x6B, 0x65, 0x6F, 0x49, 0x4D, 0x42};
constexpr std::size_t kDefaultTableSize = 128;
constexpr std::size_t kLutBytes = 64;  // data positions served by the byte table

std::uint32_t window_at(std::span<const std::uint8_t> key, std::size_t bit) {
  const std::size_t kb = key.size() * 8;
  std::uint32_t w = 0;
  for (std::size_t k = 0; k < 32; ++k) {
    const std::size_t b = (bit + k) % kb;
    w = (w << 1) | ((key[b / 8] >> (7 - b % 8)) & 1u);
  }
  return w;
}

[[noreturn]] void throw_gpu(const char* what, int st) {
  throw GpuError(std::string(what) + ": " + nicgpu_strerror(st), st);
}

}  // namespace

namespace detail {

struct RssHostLut {
  std::vector<std::uint8_t> key;
  std::vector<std::uint32_t> window;                 // key_bits windows
  std::vector<std::array<std::uint32_t, 256>> byte;  // [position][byte value]
};

struct RssGpuState {
  int device = -1;
  nicgpu_rss_ctx* ctx = nullptr;
  std::uint64_t* hits = nullptr;  // device u64[table_n] scratch for the stats
  std::size_t hits_n = 0;
  ~RssGpuState() {
    if (hits) (void) nicgpu_free(hits);
    if (ctx) (void) nicgpu_rss_destroy(ctx);
  }
};

}  // namespace detail

namespace {

std::shared_ptr<const detail::RssHostLut> build_lut(const std::vector<std::uint8_t>& key) {
  auto lut = std::make_shared<detail::RssHostLut>();
  lut->key = key;
  const std::size_t kb = key.size() * 8;
  lut->window.resize(kb);
  for (std::size_t b = 0; b < kb; ++b) lut->window[b] = window_at(key, b);
  lut->byte.resize(kLutBytes);
  for (std::size_t pos = 0; pos < kLutBytes; ++pos) {
    std::uint32_t w[8];
    for (std::size_t i = 0; i < 8; ++i) w[i] = lut->window[(pos * 8 + i) % kb];
    for (std::size_t v = 0; v < 256; ++v) {
      std::uint32_t h = 0;
      for (std::size_t i = 0; i < 8; ++i)
        if ((v >> (7 - i)) & 1u) h ^= w[i];
      lut->byte[pos][v] = h;
    }
  }
  return lut;
}

}  // namespace

RssEngine::RssEngine() { ensure_defaults(); }

RssEngine::RssEngine(RssConfig config) : config_(std::move(config)) { ensure_defaults(); }

void RssEngine::set_key(std::vector<std::uint8_t> key) {
  config_.key = std::move(key);
  if (config_.key.empty()) config_.key.assign(std::begin(kDefaultKey), std::end(kDefaultKey));
  lut_.reset();
  gpu_.reset();
}

void RssEngine::set_table(std::vector<std::uint16_t> table) {
  config_.table = std::move(table);
  if (config_.table.empty()) config_.table.assign(kDefaultTableSize, 0);
  gpu_.reset();  // queue_hits keeps its size (rss.cpp:35-41 does not touch stats)
}

std::uint32_t RssEngine::hash(std::span<const std::uint8_t> data) const {
  stats_.hashes += 1;
  return toeplitz_hash(std::span<const std::uint8_t>(config_.key), data);
}

std::optional<std::uint16_t> RssEngine::select_queue(std::span<const std::uint8_t> data) const {
  if (config_.table.empty()) return std::nullopt;
  const std::uint32_t h = hash(data);
  const std::size_t idx = h % static_cast<std::uint32_t>(config_.table.size());
  if (idx < stats_.queue_hits.size()) stats_.queue_hits[idx] += 1;
  return config_.table[idx];
}

std::uint32_t RssEngine::toeplitz_hash(std::span<const std::uint8_t> key, std::span<const std::uint8_t> data) const {
  if (key.empty() || data.empty()) return 0;
  const bool own_key = key.data() == config_.key.data() && key.size() == config_.key.size();
  if (!own_key) {  // not the engine's key: direct window evaluation
    std::uint32_t h = 0;
    for (std::size_t bit = 0; bit < data.size() * 8; ++bit)
      if ((data[bit / 8] >> (7 - bit % 8)) & 1u) h ^= window_at(key, bit);
    return h;
  }
  if (!lut_) lut_ = build_lut(config_.key);
  const auto& L = *lut_;
  std::uint32_t h = 0;
  const std::size_t n = data.size() < kLutBytes ? data.size() : kLutBytes;
  for (std::size_t i = 0; i < n; ++i) h ^= L.byte[i][data[i]];
  const std::size_t kb = L.window.size();
  for (std::size_t i = kLutBytes; i < data.size(); ++i)
    for (std::size_t j = 0; j < 8; ++j)
      if ((data[i] >> (7 - j)) & 1u) h ^= L.window[(i * 8 + j) % kb];
  return h;
}

void RssEngine::ensure_defaults() {
  if (config_.key.empty()) config_.key.assign(std::begin(kDefaultKey), std::end(kDefaultKey));
  if (config_.table.empty()) config_.table.assign(kDefaultTableSize, 0);
  stats_.queue_hits.assign(config_.table.size(), 0);
}

void RssEngine::reset_stats() noexcept {
  stats_.hashes = 0;
  stats_.queue_hits.assign(config_.table.size(), 0);
}

void RssEngine::select_queue_batch(const DevicePacketBatch& batch, const TupleSpec& tuple, const RxBatchOutputs& out,
                                   void* stream, bool update_stats) const {
  if (tuple.mode == TupleMode::None) {
    if (out.hash || out.queue) throw GpuError("select_queue_batch: TupleMode::None cannot produce hashes", NICGPU_ERR_INVALID);
    if (out.checksum) {
      const int st = nicgpu_checksum_batch(reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc,
                                           batch.count, out.checksum, stream);
      if (st != NICGPU_OK) throw_gpu("nicgpu_checksum_batch", st);
    }
    return;
  }
  // The per-packet path takes any key and table (rss.cpp:27-41); an RSS
  // context holds at most NICGPU_MAX_KEY key bytes and NICGPU_MAX_TABLE
  // entries.  A longer key is truncated, which hashes identically: tuples are
  // <= NICGPU_MAX_TUPLE bytes, so no key bit past 8 * 64 + 31 is ever read and
  // neither key wraps.  A larger table is refused before any device work.
  static_assert(NICGPU_MAX_KEY * 8 > NICGPU_MAX_TUPLE * 8 + 31, "truncated keys must not wrap");
  if (config_.table.size() > NICGPU_MAX_TABLE)
    throw GpuError("select_queue_batch: indirection table of " + std::to_string(config_.table.size()) +
                       " entries exceeds the GPU limit of NICGPU_MAX_TABLE = " + std::to_string(NICGPU_MAX_TABLE),
                   NICGPU_ERR_INVALID);
  ensure_gpu(stream);
  int st = NICGPU_OK;
  std::uint64_t* hits = nullptr;
  const std::size_t tn = config_.table.size();
  if (update_stats) {
    if (gpu_->hits_n < tn) {
      if (gpu_->hits) (void) nicgpu_free(gpu_->hits);
      gpu_->hits = nullptr;
      gpu_->hits_n = 0;
      void* p = nullptr;
      st = nicgpu_malloc(&p, tn * sizeof(std::uint64_t));
      if (st != NICGPU_OK) throw_gpu("nicgpu_malloc", st);
      gpu_->hits = static_cast<std::uint64_t*>(p);
      gpu_->hits_n = tn;
    }
    hits = gpu_->hits;
    st = nicgpu_memset_async(hits, 0, tn * sizeof(std::uint64_t), stream);
    if (st != NICGPU_OK) throw_gpu("nicgpu_memset_async", st);
  }
  st = nicgpu_rx_offload(gpu_->ctx, reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc, batch.count,
                         static_cast<int>(tuple.mode), tuple.raw_offset, tuple.raw_length, out.checksum, out.hash,
                         out.queue, hits, stream);
  if (st != NICGPU_OK) throw_gpu("nicgpu_rx_offload", st);
  if (update_stats) {
    std::vector<std::uint64_t> h(tn);
    st = nicgpu_memcpy_async(h.data(), hits, tn * sizeof(std::uint64_t), stream);
    if (st == NICGPU_OK) st = nicgpu_stream_synchronize(stream);
    if (st != NICGPU_OK) throw_gpu("stats readback", st);
    account_batch(batch.count, h);
  }
}

void RssEngine::ensure_gpu(void* stream) const {
  const std::size_t key_len = config_.key.size() < NICGPU_MAX_KEY ? config_.key.size() : NICGPU_MAX_KEY;
  int dev = 0;
  int st = nicgpu_get_device(&dev);
  if (st != NICGPU_OK) throw_gpu("nicgpu_get_device", st);
  if (!gpu_ || gpu_->device != dev) {
    auto g = std::make_shared<detail::RssGpuState>();
    g->device = dev;
    st = nicgpu_rss_create(&g->ctx, dev);
    if (st != NICGPU_OK) throw_gpu("nicgpu_rss_create", st);
    st = nicgpu_rss_set_key(g->ctx, config_.key.data(), key_len, stream);
    if (st != NICGPU_OK) throw_gpu("nicgpu_rss_set_key", st);
    st = nicgpu_rss_set_table(g->ctx, config_.table.data(), config_.table.size(), stream);
    if (st != NICGPU_OK) throw_gpu("nicgpu_rss_set_table", st);
    gpu_ = std::move(g);
  }
}

void RssEngine::select_queue_batch_enqueue(const DevicePacketBatch& batch, const std::uint64_t* count_dev,
                                           const TupleSpec& tuple, const RxBatchOutputs& out,
                                           std::uint64_t* hits_dev, void* stream) const {
  if (config_.table.size() > NICGPU_MAX_TABLE)
    throw GpuError("select_queue_batch_enqueue: indirection table of " + std::to_string(config_.table.size()) +
                       " entries exceeds the GPU limit of NICGPU_MAX_TABLE = " + std::to_string(NICGPU_MAX_TABLE),
                   NICGPU_ERR_INVALID);
  if (count_dev == nullptr) throw GpuError("select_queue_batch_enqueue: null device count", NICGPU_ERR_INVALID);
  if (tuple.mode == TupleMode::None)
    throw GpuError("select_queue_batch_enqueue: TupleMode::None cannot produce hashes", NICGPU_ERR_INVALID);
  if (batch.count == 0) return;
  ensure_gpu(stream);
  const int st = nicgpu_rx_offload_count(gpu_->ctx, reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc,
                                         batch.count, count_dev, static_cast<int>(tuple.mode), tuple.raw_offset,
                                         tuple.raw_length, out.checksum, out.hash, out.queue, hits_dev, stream);
  if (st != NICGPU_OK) throw_gpu("nicgpu_rx_offload_count", st);
}

const nicgpu_rss_ctx* RssEngine::device_context(void* stream) const {
  if (config_.table.size() > NICGPU_MAX_TABLE)
    throw GpuError("device_context: indirection table of " + std::to_string(config_.table.size()) +
                       " entries exceeds the GPU limit of NICGPU_MAX_TABLE = " + std::to_string(NICGPU_MAX_TABLE),
                   NICGPU_ERR_INVALID);
  ensure_gpu(stream);
  return gpu_->ctx;
}

void RssEngine::account_batch(std::uint64_t count, std::span<const std::uint64_t> hits) const {
  // identical to `count` sequential select_queue calls (rss.cpp:45, 56-58)
  stats_.hashes += count;
  for (std::size_t i = 0; i < hits.size() && i < stats_.queue_hits.size(); ++i) stats_.queue_hits[i] += hits[i];
}

}  // namespace nic
