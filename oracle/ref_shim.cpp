// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// C entry points over the reference's own frankie::core::crc32 (compiled from
// /root/reference/src/core/crc32.cpp by oracle/Makefile into oracle/_ref/). Used to pin the
// oracle restatement and, in bench.py, as the "reference" CPU baseline. Never shipped.
#include <cstddef>
#include <cstdint>
#include <span>

#include "core/crc32.hpp"

using frankie::core::crc32;

extern "C" {

// crc32{}.update(bytes).finalize()  (/root/reference/src/core/crc32.hpp:32-49)
std::uint32_t ref_crc32(const unsigned char *p, std::size_t n) {
  return crc32{}.update(std::as_bytes(std::span<const unsigned char>(p, n))).finalize();
}

// Table entries from the reference's constexpr generator (crc32.hpp:16-30).
void ref_table(std::uint32_t *out) {
  constexpr auto t = frankie::core::generate_crc32_table();
  for (std::size_t i = 0; i < t.size(); ++i) out[i] = t[i];
}

// Incremental: chunked updates on one object (crc32_test.cpp:110-124 semantics).
std::uint32_t ref_crc32_chunked(const unsigned char *p, const std::size_t *cuts, std::size_t ncuts,
                                std::size_t n) {
  crc32 c;
  std::size_t prev = 0;
  for (std::size_t i = 0; i <= ncuts; ++i) {
    std::size_t end = i < ncuts ? cuts[i] : n;
    (void)c.update(std::as_bytes(std::span<const unsigned char>(p + prev, end - prev)));
    prev = end;
  }
  return c.finalize();
}

// Batch of equal-length blocks at a fixed stride, contiguous range [first, first+count).
void ref_crc32_blocks(const unsigned char *base, std::size_t stride, std::size_t len, std::size_t count,
                      std::uint32_t *out) {
  for (std::size_t i = 0; i < count; ++i) out[i] = ref_crc32(base + i * stride, len);
}

// Batch of blocks at arbitrary offsets and lengths: out[i] = crc of [base + off[i], + len[i]).
void ref_crc32_irregular(const unsigned char *base, const std::uint64_t *off, const std::uint32_t *len,
                         std::size_t count, std::uint32_t *out) {
  for (std::size_t i = 0; i < count; ++i) out[i] = ref_crc32(base + off[i], len[i]);
}

}  // extern "C"
