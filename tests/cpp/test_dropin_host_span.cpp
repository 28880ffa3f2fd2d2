// The drop-in header with the opt-in host path for short spans (built with -DTKV_DROPIN_HOST_MAX,
// by tests/test_host_span.py): the reference's crc32_test.cpp known answers (:81-124) and
// wal_entry::encode's record CRC (wal.cpp:54-57, tests/golden/wal.json) through
// frankie::core::crc32, every span at or below the threshold, so no GPU is touched.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <span>
#include <string>
#include <vector>

#include "frankie_crc32.hpp"

#if TKV_DROPIN_HOST_MAX < 64
#error "build with -DTKV_DROPIN_HOST_MAX=N, N >= 64"
#endif

using namespace frankie::core;

static int g_fail = 0;
#define CHECK_EQ(a, b)                                                                          \
  do {                                                                                          \
    const auto va = (a);                                                                        \
    const auto vb = (b);                                                                        \
    if (va != vb) {                                                                             \
      std::fprintf(stderr, "%s:%d CHECK_EQ(%s, %s) failed: %llx vs %llx\n", __FILE__, __LINE__, \
                   #a, #b, (unsigned long long)va, (unsigned long long)vb);                     \
      ++g_fail;                                                                                 \
    }                                                                                           \
  } while (0)

namespace {
std::span<const std::byte> bytes_of(const std::string& s) { return std::as_bytes(std::span{s}); }

void known_values() {
  CHECK_EQ(crc32{}.update({}).finalize(), 0x00000000u);
  CHECK_EQ(crc32{}.update(bytes_of("123456789")).finalize(), 0xCBF43926u);
  CHECK_EQ(crc32{}.update(bytes_of("The quick brown fox jumps over the lazy dog")).finalize(), 0x414FA339u);
}

void incremental_equals_single() {
  const std::string data = "Hello, World!";
  crc32 single;
  (void)single.update(bytes_of(data));
  crc32 chunked;
  (void)chunked.update(bytes_of(data.substr(0, 5)));
  (void)chunked.update(bytes_of(data.substr(5, 2)));
  (void)chunked.update(bytes_of(data.substr(7)));
  CHECK_EQ(single.finalize(), chunked.finalize());
  CHECK_EQ(single.finalize(), 0xEC4AC3D0u);  // tests/golden/kat.json "incremental"
  chunked.reset();
  CHECK_EQ(chunked.finalize(), 0u);
}

// wal_entry::encode's layout and CRC placement (wal.cpp:19-61): op 0, seq 42, "hello" -> "world".
void wal_record_crc() {
  const std::string k = "hello", v = "world";
  const std::uint32_t size = 26 + static_cast<std::uint32_t>(k.size() + v.size());
  std::vector<char> buf(size, 0);
  const std::uint32_t record_len = size - 8, klen = 5, vlen = 5;
  const std::uint64_t seq = 42;
  std::memcpy(buf.data(), &record_len, 4);
  std::memcpy(buf.data() + 9, &seq, 8);
  std::memcpy(buf.data() + 18, &klen, 4);
  std::memcpy(buf.data() + 22, &vlen, 4);
  std::memcpy(buf.data() + 26, k.data(), klen);
  std::memcpy(buf.data() + 31, v.data(), vlen);
  const std::uint32_t crc = crc32{}.update({reinterpret_cast<const std::byte*>(buf.data()) + 8, size - 8u}).finalize();
  CHECK_EQ(crc, 0x593B861Au);  // tests/golden/wal.json (the reference's crc32 over the same bytes)
}

// Every length up to the threshold against the byte-at-a-time definition (crc32.cpp:9-16).
void all_lengths() {
  constexpr auto T = generate_crc32_table();
  std::vector<std::byte> d(TKV_DROPIN_HOST_MAX);
  for (std::size_t i = 0; i < d.size(); ++i) d[i] = static_cast<std::byte>((i * 2654435761u) >> 11);
  for (std::size_t n = 0; n <= d.size(); n += (n < 130 ? 1 : 61)) {
    std::uint32_t r = 0xFFFFFFFFu;
    for (std::size_t i = 0; i < n; ++i) r = (r >> 8) ^ T[(r ^ static_cast<std::uint32_t>(d[i])) & 0xFFu];
    CHECK_EQ(crc32{}.update({d.data(), n}).finalize(), r ^ 0xFFFFFFFFu);
  }
}
}  // namespace

int main() {
  known_values();
  incremental_equals_single();
  wal_record_crc();
  all_lengths();
  std::printf("%s\n", g_fail ? "FAILED" : "ALL PASSED");
  return g_fail ? 1 : 0;
}
