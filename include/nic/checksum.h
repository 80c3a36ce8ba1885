// nic/checksum.h — ones'-complement checksum of the smart_nic model.
//
// Drop-in for rosslwheeler/smart_nic include/nic/checksum.h:9-12 (same two
// declarations, bit-exact with src/checksum.cpp:10-34), plus the GPU batch
// entry point that replaces one call per packet with one launch per batch.
#pragma once

#include <cstddef>
#include <cstdint>
#include <span>

#include "nic/gpu_batch.h"

namespace nic {

/// Ones'-complement sum of the buffer's big-endian 16-bit words (an odd final
/// byte is the high byte of a last word), complemented.  Empty -> 0xFFFF.
/// Host-side and synchronous: the per-packet calls of QueuePair stay cheap.
std::uint16_t compute_checksum(std::span<const std::byte> buffer);

/// compute_checksum(buffer) == expected.
bool verify_checksum(std::span<const std::byte> buffer, std::uint16_t expected);

/// out_device[i] = compute_checksum(frame i) for every packet of a
/// device-resident batch, on the GPU, asynchronously on `stream` (a
/// hipStream_t; nullptr = the default stream).  Throws nic::GpuError.
void compute_checksum_batch(const DevicePacketBatch& batch, std::uint16_t* out_device,
                            void* stream = nullptr);

}  // namespace nic
