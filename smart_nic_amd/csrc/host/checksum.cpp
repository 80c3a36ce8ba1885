// checksum.cpp — nic::compute_checksum / verify_checksum (host, per packet) and
// nic::compute_checksum_batch (GPU, per batch).
//
// Bit-exact with the reference src/checksum.cpp:10-34 but not its loop: the
// reference folds the carry after every 16-bit add; here 32-bit little-endian
// words are summed into 64 bits and folded once.  Both give 0 only for an
// all-zero buffer and otherwise the unique value in [1, 0xFFFF] congruent to
// the word sum mod 0xFFFF (2^16 == 1 mod 0xFFFF), and summing little-endian
// halfwords yields the byte-swapped big-endian sum (RFC 1071 byte-order
// independence).  SURVEY §0 fact 9.
#include "nic/checksum.h"

#include <cstring>

#include "nicgpu.h"

namespace nic {
namespace {

inline std::uint32_t fold64(std::uint64_t s) {
  if (s == 0) return 0;
  const std::uint32_t r = static_cast<std::uint32_t>(s % 0xFFFFull);
  return r ? r : 0xFFFFu;
}

}  // namespace

std::uint16_t compute_checksum(std::span<const std::byte> buffer) {
  const auto* p = reinterpret_cast<const unsigned char*>(buffer.data());
  const std::size_t n = buffer.size();
  std::uint64_t a = 0, b = 0;  // two accumulators for ILP
  std::size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    std::uint32_t w0, w1;
    std::memcpy(&w0, p + i, 4);
    std::memcpy(&w1, p + i + 4, 4);
    a += w0;
    b += w1;
  }
  std::uint64_t s = a + b;
  for (; i + 2 <= n; i += 2) s += static_cast<std::uint32_t>(p[i]) | (static_cast<std::uint32_t>(p[i + 1]) << 8);
  if (i < n) s += p[i];  // odd trailing byte: low byte of a LE halfword = high byte of a BE word
  const std::uint32_t le = fold64(s);
  const std::uint32_t be = ((le & 0xFFu) << 8) | (le >> 8);
  return static_cast<std::uint16_t>(~be & 0xFFFFu);
}

bool verify_checksum(std::span<const std::byte> buffer, std::uint16_t expected) {
  return compute_checksum(buffer) == expected;
}

void compute_checksum_batch(const DevicePacketBatch& batch, std::uint16_t* out_device, void* stream) {
  const int st = nicgpu_checksum_batch(reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc, batch.count,
                                       out_device, stream);
  if (st != NICGPU_OK) throw GpuError(std::string("nicgpu_checksum_batch: ") + nicgpu_strerror(st), st);
}

int gpu_device_count() {
  const int n = nicgpu_device_count();
  return n < 0 ? 0 : n;
}

}  // namespace nic
