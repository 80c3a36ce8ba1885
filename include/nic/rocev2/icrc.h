// nic/rocev2/icrc.h — RoCEv2 ICRC.
//
// IcrcCalculator is declared exactly as in the reference's
// include/nic/rocev2/packet.h:195-214, so libnic_host.so's definitions of
// calculate() / verify() satisfy either header: a reference build drops the
// IcrcCalculator definitions from src/rocev2/packet.cpp:14-75 and links this
// library.  Host calls stay per packet and synchronous; the
// batch functions below run one GPU launch over a device-resident batch
// (nicgpu_icrc_batch).  Include either this header or the reference's
// packet.h in a translation unit, not both.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <span>

#include "nic/gpu_batch.h"

namespace nic::rocev2 {

inline constexpr std::size_t kIcrcSize = 4;  // packet.h:22

/// Calculate ICRC (Invariant CRC) for RoCEv2 packets: CRC-32C (Castagnoli).
class IcrcCalculator {
public:
  /// CRC-32C of `data` (BTH through payload, excluding ICRC).
  [[nodiscard]] static std::uint32_t calculate(std::span<const std::byte> data);

  /// true iff data.size() >= 4 and calculate(all but the last 4 bytes) equals
  /// the last 4 bytes read big-endian.
  [[nodiscard]] static bool verify(std::span<const std::byte> data);

private:
  static const std::array<std::uint32_t, 256> kCrc32cTable;
  [[nodiscard]] static std::uint32_t update_crc(std::uint32_t crc, std::byte byte);
};

/// calculate() of every descriptor's span; out_device: u32[batch.count].
void icrc_calculate_batch(const DevicePacketBatch& batch, std::uint32_t* out_device, void* stream = nullptr);

/// verify() of every descriptor's span; ok_device: u8[batch.count] (0/1);
/// crc_device (optional): the CRC of all but the last 4 bytes (0 below 4 B).
void icrc_verify_batch(const DevicePacketBatch& batch, std::uint8_t* ok_device, std::uint32_t* crc_device = nullptr,
                       void* stream = nullptr);

}  // namespace nic::rocev2
