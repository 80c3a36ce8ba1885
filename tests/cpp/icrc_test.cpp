// icrc_test.cpp — nic::rocev2::IcrcCalculator.
//   icrc_test cpu   host calculate/verify: published CRC-32C vectors, the
//                   reference's own test properties (tests/rocev2/packet_test.cpp:22-63)
//                   and random spans vs the oracle
//   icrc_test gpu   icrc_calculate_batch / icrc_verify_batch vs the host calls
#undef NDEBUG
#include <cassert>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "nic/rocev2/icrc.h"
#include "nicgpu.h"
#include "oracle.h"

using nic::rocev2::IcrcCalculator;

namespace {

std::span<const std::byte> sp(const std::vector<std::uint8_t>& v, std::size_t off = 0, std::size_t n = SIZE_MAX) {
  n = std::min(n, v.size() - off);
  return {reinterpret_cast<const std::byte*>(v.data() + off), n};
}

int run_cpu() {
  auto str = [](const char* s) { return std::vector<std::uint8_t>(s, s + std::strlen(s)); };
  assert(IcrcCalculator::calculate(sp(str("123456789"))) == 0xE3069283u);
  assert(IcrcCalculator::calculate(sp(std::vector<std::uint8_t>(32, 0))) == 0x8A9136AAu);
  assert(IcrcCalculator::calculate(sp(std::vector<std::uint8_t>(32, 0xFF))) == 0x62A8AB43u);
  std::vector<std::uint8_t> inc(32), dec(32);
  for (int i = 0; i < 32; ++i) { inc[i] = static_cast<std::uint8_t>(i); dec[i] = static_cast<std::uint8_t>(31 - i); }
  assert(IcrcCalculator::calculate(sp(inc)) == 0x46DD794Eu);
  assert(IcrcCalculator::calculate(sp(dec)) == 0x113FDB5Cu);
  assert(IcrcCalculator::calculate({}) == 0u);
  // reference properties (packet_test.cpp:22-63)
  const std::vector<std::uint8_t> d1 = {1, 2, 3, 4};
  assert(IcrcCalculator::calculate(sp(d1)) != 0 && IcrcCalculator::calculate(sp(d1)) == IcrcCalculator::calculate(sp(d1)));
  std::vector<std::uint8_t> pk = {0x11, 0x22, 0x33, 0x44, 0, 0, 0, 0};
  const std::uint32_t c = IcrcCalculator::calculate(sp(pk, 0, 4));
  pk[4] = c >> 24; pk[5] = c >> 16; pk[6] = c >> 8; pk[7] = c;
  assert(IcrcCalculator::verify(sp(pk)));
  pk[2] = 0xFF;
  assert(!IcrcCalculator::verify(sp(pk)));
  assert(!IcrcCalculator::verify(sp(pk, 0, 3)));
  std::mt19937_64 rng(5);
  for (int t = 0; t < 20000; ++t) {
    std::vector<std::uint8_t> b(1 + rng() % 3000);
    for (auto& x : b) x = static_cast<std::uint8_t>(rng());
    const std::size_t off = rng() % b.size(), n = rng() % (b.size() - off + 1);
    assert(IcrcCalculator::calculate(sp(b, off, n)) == oracle_icrc_calculate(b.data() + off, n));
    assert(IcrcCalculator::verify(sp(b, off, n)) == (oracle_icrc_verify(b.data() + off, n) != 0));
  }
  std::puts("icrc_test cpu: ok");
  return 0;
}

int run_gpu() {
  std::mt19937_64 rng(6);
  std::vector<std::uint8_t> frames;
  std::vector<std::uint64_t> desc;
  for (int i = 0; i < 20000; ++i) {
    std::size_t len = (i % 7 == 0) ? rng() % 8 : (i % 11 == 0 ? 4000 + rng() % 5500 : 20 + rng() % 1500);
    const std::size_t gap = rng() % 20;
    for (std::size_t g = 0; g < gap; ++g) frames.push_back(static_cast<std::uint8_t>(rng()));
    const std::size_t off = frames.size();
    for (std::size_t k = 0; k < len; ++k) frames.push_back(static_cast<std::uint8_t>(rng()));
    if (len >= 4 && rng() % 2) {  // a valid ICRC trailer on half of them
      const std::uint32_t c = IcrcCalculator::calculate(sp(frames, off, len - 4));
      frames[off + len - 4] = c >> 24; frames[off + len - 3] = c >> 16; frames[off + len - 2] = c >> 8; frames[off + len - 1] = c;
    }
    desc.push_back(NICGPU_DESC(off, len));
  }
  frames.resize(frames.size() + 64);
  const std::size_t n = desc.size();
  void *df, *dd, *dc, *dv, *dc2;
  assert(nicgpu_malloc(&df, frames.size()) == NICGPU_OK && nicgpu_malloc(&dd, n * 8) == NICGPU_OK);
  assert(nicgpu_malloc(&dc, n * 4) == NICGPU_OK && nicgpu_malloc(&dv, n) == NICGPU_OK && nicgpu_malloc(&dc2, n * 4) == NICGPU_OK);
  assert(nicgpu_memcpy_async(df, frames.data(), frames.size(), nullptr) == NICGPU_OK);
  assert(nicgpu_memcpy_async(dd, desc.data(), n * 8, nullptr) == NICGPU_OK);
  const nic::DevicePacketBatch batch{static_cast<const std::byte*>(df), static_cast<const std::uint64_t*>(dd), n};
  nic::rocev2::icrc_calculate_batch(batch, static_cast<std::uint32_t*>(dc));
  nic::rocev2::icrc_verify_batch(batch, static_cast<std::uint8_t*>(dv), static_cast<std::uint32_t*>(dc2));
  std::vector<std::uint32_t> crc(n), crc2(n);
  std::vector<std::uint8_t> ok(n);
  assert(nicgpu_memcpy_async(crc.data(), dc, n * 4, nullptr) == NICGPU_OK);
  assert(nicgpu_memcpy_async(crc2.data(), dc2, n * 4, nullptr) == NICGPU_OK);
  assert(nicgpu_memcpy_async(ok.data(), dv, n, nullptr) == NICGPU_OK);
  assert(nicgpu_stream_synchronize(nullptr) == NICGPU_OK);
  std::size_t nok = 0;
  for (std::size_t i = 0; i < n; ++i) {
    const std::size_t off = desc[i] & ((1ull << 40) - 1), len = desc[i] >> 40;
    assert(crc[i] == IcrcCalculator::calculate(sp(frames, off, len)));
    assert(ok[i] == (IcrcCalculator::verify(sp(frames, off, len)) ? 1 : 0));
    assert(crc2[i] == (len >= 4 ? IcrcCalculator::calculate(sp(frames, off, len - 4)) : 0u));
    nok += ok[i];
  }
  assert(nok > n / 3);
  // argument checks
  assert(nicgpu_icrc_batch(static_cast<const std::uint8_t*>(df), static_cast<const std::uint64_t*>(dd), n, 7,
                           static_cast<std::uint32_t*>(dc), nullptr, nullptr) == NICGPU_ERR_INVALID);
  assert(nicgpu_icrc_batch(static_cast<const std::uint8_t*>(df), static_cast<const std::uint64_t*>(dd), n,
                           NICGPU_ICRC_VERIFY, static_cast<std::uint32_t*>(dc), nullptr, nullptr) == NICGPU_ERR_INVALID);
  for (void* p : {df, dd, dc, dv, dc2}) nicgpu_free(p);
  std::printf("icrc_test gpu: ok (%zu spans, %zu verified)\n", n, nok);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  return mode == "gpu" ? run_gpu() : run_cpu();
}
