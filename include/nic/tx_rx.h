// nic/tx_rx.h — TX/RX descriptor and completion PODs of the smart_nic model.
//
// Drop-in for rosslwheeler/smart_nic include/nic/tx_rx.h:11-71.  Field order,
// types and defaults are what the reference's QueuePair memcpy-serialises
// (src/queue_pair.cpp:130-148), so the layouts are pinned below with
// static_asserts (x86-64).
#pragma once

#include <cstddef>
#include <cstdint>

#if __has_include("nic/host_memory.h")
#include "nic/host_memory.h"  // the model's HostMemory (reference build)
#endif
#include "nic/offload.h"

namespace nic {

// Same alias as include/nic/host_memory.h:9 (re-declaring an alias to the same
// type is well-formed, so both headers may be included together).
using HostAddress = std::uint64_t;

// Layer3 and Layer4 behave identically in the model (whole-buffer checksum).
enum class ChecksumMode : std::uint8_t { None, Layer3, Layer4 };

enum class CompletionCode : std::uint16_t {
  Success = 0,
  BufferTooSmall = 1,
  ChecksumError = 2,
  NoDescriptor = 3,
  Fault = 4,
  MtuExceeded = 5,
  InvalidMss = 6,
  TooManySegments = 7,
};

struct TxDescriptor {
  HostAddress buffer_address{0};
  std::uint32_t length{0};
  ChecksumMode checksum{ChecksumMode::None};
  std::uint16_t descriptor_index{0};
  std::uint16_t checksum_value{0};
  bool checksum_offload{false};
  bool tso_enabled{false};
  bool gso_enabled{false};
  std::uint16_t mss{0};
  std::uint16_t header_length{0};  // bytes kept verbatim at the front of every segment
  bool vlan_insert{false};
  std::uint16_t vlan_tag{0};
};

struct RxDescriptor {
  HostAddress buffer_address{0};
  std::uint32_t buffer_length{0};
  ChecksumMode checksum{ChecksumMode::None};
  std::uint16_t descriptor_index{0};
  bool checksum_offload{false};
  bool vlan_strip{false};
  bool vlan_present{false};
  std::uint16_t vlan_tag{0};
  bool gro_enabled{false};  // echoed back only (no aggregation in the model)
};

struct TxCompletion {
  std::uint16_t queue_id{0};
  std::uint16_t descriptor_index{0};
  CompletionCode status{CompletionCode::Success};
  bool checksum_offloaded{false};
  bool tso_performed{false};
  bool gso_performed{false};
  bool vlan_inserted{false};
  std::uint16_t segments_produced{1};
  std::uint16_t vlan_tag{0};
};

struct RxCompletion {
  std::uint16_t queue_id{0};
  std::uint16_t descriptor_index{0};
  CompletionCode status{CompletionCode::Success};
  bool checksum_verified{false};
  bool vlan_stripped{false};
  bool gro_aggregated{false};
  std::uint16_t vlan_tag{0};
};

// Layout pins (the reference ABI as the model memcpy's it).
static_assert(sizeof(TxDescriptor) == 32);
static_assert(offsetof(TxDescriptor, length) == 8);
static_assert(offsetof(TxDescriptor, checksum) == 12);
static_assert(offsetof(TxDescriptor, descriptor_index) == 14);
static_assert(offsetof(TxDescriptor, checksum_value) == 16);
static_assert(offsetof(TxDescriptor, checksum_offload) == 18);
static_assert(offsetof(TxDescriptor, tso_enabled) == 19);
static_assert(offsetof(TxDescriptor, gso_enabled) == 20);
static_assert(offsetof(TxDescriptor, mss) == 22);
static_assert(offsetof(TxDescriptor, header_length) == 24);
static_assert(offsetof(TxDescriptor, vlan_insert) == 26);
static_assert(offsetof(TxDescriptor, vlan_tag) == 28);
static_assert(sizeof(RxDescriptor) == 24);
static_assert(offsetof(RxDescriptor, buffer_length) == 8);
static_assert(offsetof(RxDescriptor, checksum) == 12);
static_assert(offsetof(RxDescriptor, descriptor_index) == 14);
static_assert(offsetof(RxDescriptor, checksum_offload) == 16);
static_assert(offsetof(RxDescriptor, vlan_strip) == 17);
static_assert(offsetof(RxDescriptor, vlan_present) == 18);
static_assert(offsetof(RxDescriptor, vlan_tag) == 20);
static_assert(offsetof(RxDescriptor, gro_enabled) == 22);

}  // namespace nic
