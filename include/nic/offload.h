// nic/offload.h — offload limits and enums of the smart_nic model.
//
// Drop-in for rosslwheeler/smart_nic include/nic/offload.h:9-42: the same
// names and values, so reference translation units (QueuePair, QueueManager)
// compile unchanged against this header.  The RX offload kernels use the frame
// and segment limits below (kMaxJumboFrame, kMaxTsoSegments).
#pragma once

#include <cstddef>
#include <cstdint>

namespace nic {

// Frame sizes (bytes).
constexpr std::size_t kMinEthernetFrame = 64;
constexpr std::size_t kStandardMtu = 1500;
constexpr std::size_t kJumboMtu = 9000;
constexpr std::size_t kMaxJumboFrame = 9216;  // headers included

// TSO/GSO limits; kMinMss is deliberately tiny (tests use mss = 3..6).
constexpr std::size_t kMaxTsoSegments = 64;
constexpr std::size_t kMinMss = 1;
constexpr std::size_t kMaxMss = 9000;

// 802.1Q / 802.1ad tagging.
constexpr std::size_t kVlanHeaderSize = 4;
constexpr std::uint16_t kVlanEthertype = 0x8100;
constexpr std::uint16_t kQinQEthertype = 0x88A8;

enum class OffloadError : std::uint8_t {
  None = 0,
  MtuExceeded,
  InvalidMss,
  InvalidHeaderLength,
  TooManySegments,
  VlanError,
  GroTimeout,
  GroFlowMismatch,
};

enum class GroState : std::uint8_t {
  Idle = 0,
  Aggregating,
  TimedOut,
  FlowChanged,
};

}  // namespace nic
