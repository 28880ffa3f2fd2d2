// frankie_crc32.hpp — drop-in replacement for tinykvpp's src/core/crc32.hpp (+ crc32.cpp).
//
// Keeps the reference's C++ surface exactly (/root/reference/src/core/crc32.hpp:9-49): namespace
// frankie::core, the kCRC32* constants, crc32_table, the constexpr generate_crc32_table(), and
// class crc32 with constexpr default ctor, [[nodiscard]] crc32& update(span<const byte>) noexcept,
// [[nodiscard]] uint32_t finalize() const noexcept and void reset() noexcept — so wal.cpp's
// `core::crc32{}.update({...}).finalize()` (wal.cpp:54-57, 89-92) and test/crc32_test.cpp compile
// unchanged. update() forwards to the C ABI (tkv_crc32_update, include/tkv_crc32.h), which runs the
// gfx950 HIP kernel, except for short spans (below).
//
// Short spans run on the calling core: spans of at most TKV_DROPIN_HOST_MAX bytes (default 65536) go
// to tkv_crc32_update_host (slicing-by-8 over tables built from the polynomial, product code with its
// own parity tests; not the oracle). That is the measured crossover of one call
// (profiles/r3/put_latency.jsonl): up to 64 KiB the host path is faster (36 B: 0.011 us against the
// reference's 0.040 us and 11 us for a GPU round trip; 64 KiB: 23 us against 31 us), from 128 KiB the
// GPU is (35 us against 46 us). So the reference's per-put record stamp (wal.cpp:54-57) costs less
// than in the reference. Longer spans go to the GPU (tkv_crc32_update). The reference's update is
// noexcept and has no failure mode (crc32.cpp:9-16), so when the GPU call returns an error (no device
// on this node, a HIP failure) the same span is recomputed on the host by tkv_crc32_update_fallback,
// which warns once per process on stderr and counts the call. update therefore never fails, at any
// span size, with or without a device. -DTKV_DROPIN_HOST_MAX=0 sends every span to the GPU first.
// tkv_debug_update_counts_n says which path the calling thread's calls took: [0] host span, [1] GPU,
// [2] host recompute after a GPU error.
//
// Build: add include/ to the include path and link libtkv_crc32.so.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <span>

#include "tkv_crc32.h"

#ifndef TKV_DROPIN_HOST_MAX
#define TKV_DROPIN_HOST_MAX 65536
#endif

namespace frankie::core {

constexpr std::uint32_t kCRC32DefaultValue{TKV_CRC32_DEFAULT_RAW};  // crc32.hpp:9
constexpr std::uint32_t kCRC32Bits{8};                               // crc32.hpp:10
constexpr std::uint32_t kCRC32Polynomial = TKV_CRC32_POLYNOMIAL;     // crc32.hpp:11

constexpr std::size_t kCRC32TableSize{256};                        // crc32.hpp:13
using crc32_table = std::array<std::uint32_t, kCRC32TableSize>;     // crc32.hpp:14

// Byte-at-a-time table of the reflected polynomial, usable in constant expressions
// (crc32_test.cpp:83 evaluates it with constexpr).
constexpr auto generate_crc32_table() noexcept -> crc32_table {
  crc32_table t{};
  for (std::size_t e = 0; e < t.size(); ++e) {
    std::uint32_t v = static_cast<std::uint32_t>(e);
    for (std::uint32_t k = 0; k < kCRC32Bits; ++k) v = (v >> 1) ^ ((v & 1u) != 0 ? kCRC32Polynomial : 0u);
    t[e] = v;
  }
  return t;
}

class crc32 final {
 public:
  constexpr crc32() = default;

  // Continues the stored register over `data` without XORing with 0xFFFFFFFF (crc32.cpp:9-16).
  [[nodiscard]] crc32 &update(std::span<const std::byte> data) noexcept {
    std::uint32_t next = crc_;
    const bool host = kHostSpanMax > 0 && data.size() <= kHostSpanMax;
    int rc = host ? tkv_crc32_update_host(crc_, data.data(), data.size(), &next)
                  : tkv_crc32_update(crc_, data.data(), data.size(), &next);
    if (rc != TKV_OK && !host) rc = tkv_crc32_update_fallback(rc, crc_, data.data(), data.size(), &next);
    if (rc != TKV_OK) {  // unreachable: the host path fails only on a null pointer, which a span cannot pass
      std::fprintf(stderr, "frankie::core::crc32::update: host CRC failed (status %d)\n", rc);
      std::abort();
    }
    crc_ = next;
    return *this;
  }

  // Stored register XOR 0xFFFFFFFF (crc32.cpp:19).
  [[nodiscard]] std::uint32_t finalize() const noexcept { return crc_ ^ kCRC32DefaultValue; }

  // Register back to 0xFFFFFFFF (crc32.cpp:22).
  void reset() noexcept { crc_ = kCRC32DefaultValue; }

 private:
  static constexpr const auto TABLE{generate_crc32_table()};  // crc32.hpp:46 (kept for layout parity)
  // Spans up to this many bytes take the host path (TKV_DROPIN_HOST_MAX; 0 = none, every span on the GPU).
  static constexpr std::size_t kHostSpanMax{TKV_DROPIN_HOST_MAX};

  std::uint32_t crc_{kCRC32DefaultValue};
};

}  // namespace frankie::core
