// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// C entry points over the reference's own frankie::core::crc32 (compiled from
// /root/reference/src/core/crc32.cpp by oracle/Makefile into oracle/_ref/). Used to pin the
// oracle restatement and, in bench.py, as the "reference" CPU baseline. Never shipped.
#include <cstddef>
#include <cstdint>
#include <cstring>
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

// The reference's recovery loop over a slurped WAL image, restated over its own crc32: wal_entry::
// decode (/root/reference/src/engine/wal.cpp:63-130) called until the image is used up, as
// engine::create does (engine.cpp:31-53). Returns 0 when every record decodes, 4 (corrupted) at
// the first record whose header size, record_len, CRC or key/value bounds fail; *good = records
// decoded before it, *stop = its offset (the end of the image when all decode). Lengths in 64 bits.
int ref_wal_verify(const unsigned char *w, std::size_t size, std::uint64_t *good, std::uint64_t *stop) {
  constexpr std::uint64_t kMeta = 26, kOff = 8;  // wal.hpp kMetadataSize, record_len + crc32 fields
  std::uint64_t p = 0, n = 0;
  int rc = 0;
  while (p < size) {
    const std::uint64_t rem = size - p;
    if (rem < kMeta) {
      rc = 4;
      break;
    }
    std::uint32_t rlen, stored, klen, vlen;
    std::memcpy(&rlen, w + p, 4);
    std::memcpy(&stored, w + p + 4, 4);
    if (rlen + kOff > rem) {
      rc = 4;
      break;
    }
    if (ref_crc32(w + p + kOff, rlen) != stored) {
      rc = 4;
      break;
    }
    std::memcpy(&klen, w + p + 18, 4);
    std::memcpy(&vlen, w + p + 22, 4);
    if (kMeta + static_cast<std::uint64_t>(klen) + vlen > kOff + rlen) {
      rc = 4;
      break;
    }
    p += kOff + rlen;
    ++n;
  }
  *good = n;
  *stop = p;
  return rc;
}

// wal_entry::encode's stamp (wal.cpp:54-58) over n records laid out in buf: CRC of [8, size) at 4.
void ref_wal_stamp(unsigned char *buf, const std::uint64_t *off, const std::uint32_t *size, std::size_t n) {
  for (std::size_t i = 0; i < n; ++i) {
    const std::uint32_t c = ref_crc32(buf + off[i] + 8, size[i] - 8);
    std::memcpy(buf + off[i] + 4, &c, 4);
  }
}

}  // extern "C"
