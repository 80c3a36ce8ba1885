// fault_model.h — the DMA faults of the qp_fault_* fixtures, shared by their
// generator (oracle/gen_golden.cpp, through the reference's SimpleHostMemory)
// and the tests that replay them (tests/cpp/rx_stage_test.cpp): a
// FaultInjector and an IOMMU AddressTranslator in the shape SimpleHostMemory
// takes them (include/nic/simple_host_memory.h:14-15, applied by
// translate_view, src/simple_host_memory.cpp:76-87).  Both are functions of
// (address, length) once armed — the memory is loaded through the same
// translate() before they are.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <optional>

namespace faultfx {

enum Kind : int { kNone = 0, kInjector = 1, kIommu = 2 };

inline std::uint64_t mix(std::uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// kInjector: about one access in nine refused (FaultInjected)
inline bool inject(std::uint64_t a, std::size_t n) { return mix(a * 0x100000001B3ull ^ n) % 9 == 0; }

// kIommu: every 1 KiB page mapped onto itself except about one in seven; an
// access touching an unmapped page is refused (IommuFault)
inline std::optional<std::uint64_t> iommu(std::uint64_t a, std::size_t n) {
  const std::uint64_t p0 = a >> 10, p1 = (a + (n ? n - 1 : 0)) >> 10;
  for (std::uint64_t p = p0; p <= p1; ++p)
    if (mix(p) % 7 == 0) return std::nullopt;
  return a;
}

// The pair for one fixture, switched on by `armed` after the memory is loaded.
struct Model {
  std::shared_ptr<bool> armed = std::make_shared<bool>(false);
  Kind kind = kNone;
  auto translator() const {
    return [armed = armed, k = kind](std::uint64_t a, std::size_t n) -> std::optional<std::uint64_t> {
      if (!*armed || k != kIommu) return a;
      return iommu(a, n);
    };
  }
  auto injector() const {
    return [armed = armed, k = kind](std::uint64_t a, std::size_t n) { return *armed && k == kInjector && inject(a, n); };
  }
};

}  // namespace faultfx
