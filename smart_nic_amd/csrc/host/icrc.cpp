// icrc.cpp — nic::rocev2::IcrcCalculator (host, per packet) and the batch
// functions over nicgpu_icrc_batch.  Bit-exact with the reference
// src/rocev2/packet.cpp:14-75 (CRC-32C, init/xorout 0xFFFFFFFF) but
// slice-by-8 instead of one table lookup per byte.
#include "nic/rocev2/icrc.h"

#include <cstring>
#include <string>

#include "nicgpu.h"

namespace nic::rocev2 {
namespace {

struct Tables {
  std::uint32_t t[8][256];
  constexpr Tables() : t{} {
    for (std::uint32_t i = 0; i < 256; ++i) {
      std::uint32_t c = i;
      for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (int k = 1; k < 8; ++k)
      for (std::uint32_t i = 0; i < 256; ++i) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xFFu];
  }
};
constexpr Tables kT{};

std::array<std::uint32_t, 256> table0() {
  std::array<std::uint32_t, 256> a{};
  for (int i = 0; i < 256; ++i) a[i] = kT.t[0][i];
  return a;
}

}  // namespace

const std::array<std::uint32_t, 256> IcrcCalculator::kCrc32cTable = table0();

std::uint32_t IcrcCalculator::update_crc(std::uint32_t crc, std::byte byte) {
  return kT.t[0][static_cast<std::uint8_t>(crc ^ static_cast<std::uint8_t>(byte))] ^ (crc >> 8);
}

std::uint32_t IcrcCalculator::calculate(std::span<const std::byte> data) {
  const auto* p = reinterpret_cast<const unsigned char*>(data.data());
  std::size_t n = data.size();
  std::uint32_t crc = 0xFFFFFFFFu;
  while (n >= 8) {
    std::uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;  // little-endian host (x86-64 / the GPU box)
    crc = kT.t[7][lo & 0xFF] ^ kT.t[6][(lo >> 8) & 0xFF] ^ kT.t[5][(lo >> 16) & 0xFF] ^ kT.t[4][lo >> 24] ^
          kT.t[3][hi & 0xFF] ^ kT.t[2][(hi >> 8) & 0xFF] ^ kT.t[1][(hi >> 16) & 0xFF] ^ kT.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = kT.t[0][(crc ^ *p++) & 0xFFu] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}

bool IcrcCalculator::verify(std::span<const std::byte> data) {
  if (data.size() < kIcrcSize) return false;
  const auto* t = reinterpret_cast<const unsigned char*>(data.data()) + data.size() - kIcrcSize;
  const std::uint32_t stored = (std::uint32_t{t[0]} << 24) | (std::uint32_t{t[1]} << 16) | (std::uint32_t{t[2]} << 8) | t[3];
  return calculate(data.subspan(0, data.size() - kIcrcSize)) == stored;
}

void icrc_calculate_batch(const DevicePacketBatch& batch, std::uint32_t* out_device, void* stream) {
  const int st = nicgpu_icrc_batch(reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc, batch.count,
                                   NICGPU_ICRC_CALCULATE, out_device, nullptr, stream);
  if (st != NICGPU_OK) throw GpuError(std::string("nicgpu_icrc_batch: ") + nicgpu_strerror(st), st);
}

void icrc_verify_batch(const DevicePacketBatch& batch, std::uint8_t* ok_device, std::uint32_t* crc_device,
                       void* stream) {
  const int st = nicgpu_icrc_batch(reinterpret_cast<const std::uint8_t*>(batch.frames), batch.desc, batch.count,
                                   NICGPU_ICRC_VERIFY, crc_device, ok_device, stream);
  if (st != NICGPU_OK) throw GpuError(std::string("nicgpu_icrc_batch: ") + nicgpu_strerror(st), st);
}

}  // namespace nic::rocev2
