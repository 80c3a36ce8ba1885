// nic/gpu_batch.h — batched, GPU-resident RX offload for the nic:: API.
//
// New in this build (the reference processes one packet per call, on one
// thread): a batch of frames already resident in MI355X HBM, described by one
// 64-bit descriptor per packet (offset | length << 40, include/nicgpu.h), is
// checksummed and RSS-classified by one kernel launch.  These types are the
// C++ face of the C-ABI in include/nicgpu.h; the batch entry points live next
// to the functions they batch: nic::compute_checksum_batch (nic/checksum.h)
// and nic::RssEngine::select_queue_batch (nic/rss.h).
//
// Errors: every batch entry point throws nic::GpuError (never falls back to
// the CPU) — no GPU, a missing libnicgpu.so symbol, a HIP failure, bad args.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace nic {

/// A batch of frames in device memory.  `frames` must be 16-B aligned; every
/// 16-B chunk holding a packet byte must be readable.  desc[i] =
/// offset_i | (length_i << 40), length_i <= 65535.
struct DevicePacketBatch {
  const std::byte* frames{nullptr};
  const std::uint64_t* desc{nullptr};
  std::size_t count{0};
};

/// Which bytes of a frame feed the Toeplitz hash (the reference has no parser;
/// its callers pass the 12-byte src_ip|dst_ip|sport|dport tuple,
/// tests/tutorial_lesson8_test.cpp:20-35).
enum class TupleMode : int {
  None = 0,  ///< checksum only
  Auto = 1,  ///< Ethernet (+VLAN/QinQ) -> IPv4/IPv6 4-tuple (or IP pair), else empty
  Raw = 2,   ///< frame bytes [raw_offset, raw_offset + raw_length), <= 64
};

struct TupleSpec {
  TupleMode mode{TupleMode::Auto};
  std::uint32_t raw_offset{0};
  std::uint32_t raw_length{0};
};

/// Per-packet outputs in device memory; any pointer may be null.
struct RxBatchOutputs {
  std::uint16_t* checksum{nullptr};  ///< compute_checksum(frame); RX verify passes iff == 0
  std::uint32_t* hash{nullptr};      ///< Toeplitz hash of the tuple
  std::uint16_t* queue{nullptr};     ///< table[hash % table.size()]
};

class GpuError : public std::runtime_error {
public:
  GpuError(const std::string& what, int status) : std::runtime_error(what), status_(status) {}
  [[nodiscard]] int status() const noexcept { return status_; }

private:
  int status_;
};

/// Number of visible gfx950 devices (0 when none; throws only if the HIP
/// runtime itself cannot be queried).
int gpu_device_count();

}  // namespace nic
