// flat_host_memory.h — a HostMemory (host_memory.h:49-73) over one contiguous,
// page-aligned buffer, with the bounds rule of the reference's
// SimpleHostMemory::translate_view (src/simple_host_memory.cpp:89-96) and no
// address translator or fault injector: what BatchedQueuePair's host-image
// path (rx_stage.h, process_batch(HostMemory&, ...)) registers and mirrors.
// For builds without the reference's simple_host_memory.cpp (benchmarks, the
// GPU tests); the reference's SimpleHostMemory works the same way.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <span>

#include "nic/rx_stage.h"

namespace nic {

class FlatHostMemory final : public HostMemory {
public:
  explicit FlatHostMemory(std::size_t size_bytes) : size_(size_bytes) {
    const std::size_t cap = (size_bytes + 4095) / 4096 * 4096 + 4096;
    buf_.reset(static_cast<std::byte*>(std::aligned_alloc(4096, cap)));
    if (!buf_) throw std::bad_alloc();
    std::memset(buf_.get(), 0, cap);
  }
  [[nodiscard]] HostMemoryConfig config() const noexcept override { return HostMemoryConfig{size_, 4096, false}; }
  [[nodiscard]] HostMemoryResult translate(HostAddress a, std::size_t n, HostMemoryView& v) override {
    if (!in_bounds(a, n)) return {HostMemoryError::OutOfBounds, 0};
    v = HostMemoryView{buf_.get() + a, n, a};
    return {HostMemoryError::None, n};
  }
  [[nodiscard]] HostMemoryResult translate_const(HostAddress a, std::size_t n, ConstHostMemoryView& v) const override {
    if (!in_bounds(a, n)) return {HostMemoryError::OutOfBounds, 0};
    v = ConstHostMemoryView{buf_.get() + a, n, a};
    return {HostMemoryError::None, n};
  }
  [[nodiscard]] HostMemoryResult read(HostAddress a, std::span<std::byte> out) const override {
    if (!in_bounds(a, out.size())) return {HostMemoryError::OutOfBounds, 0};
    if (!out.empty()) std::memcpy(out.data(), buf_.get() + a, out.size());
    return {HostMemoryError::None, out.size()};
  }
  [[nodiscard]] HostMemoryResult write(HostAddress a, std::span<const std::byte> in) override {
    if (!in_bounds(a, in.size())) return {HostMemoryError::OutOfBounds, 0};
    if (!in.empty()) std::memcpy(buf_.get() + a, in.data(), in.size());
    return {HostMemoryError::None, in.size()};
  }
  std::byte* data() noexcept { return buf_.get(); }
  const std::byte* data() const noexcept { return buf_.get(); }
  std::size_t size() const noexcept { return size_; }

private:
  bool in_bounds(HostAddress a, std::size_t n) const noexcept { return a <= size_ && n <= size_ - a; }
  struct Free {
    void operator()(std::byte* p) const noexcept { std::free(p); }
  };
  std::size_t size_;
  std::unique_ptr<std::byte, Free> buf_;
};

}  // namespace nic
