// C++ parity tests written against the drop-in header include/frankie_crc32.hpp, the way tinykvpp's
// own test/crc32_test.cpp and test/wal_test.cpp use frankie::core::crc32. Known answers:
// crc32_test.cpp:81-124; WAL record layout and CRC coverage: wal.cpp:19-61, wal_test.cpp:96-118.
// Built by tests/test_cpp_header.py (g++ -std=c++20, linked to libtkv_crc32.so); run on a GPU.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <span>
#include <string>
#include <vector>

#include "frankie_crc32.hpp"
#include "tkv_crc32.h"

using namespace frankie::core;

static int g_fail = 0;
#define CHECK_EQ(a, b)                                                                           \
  do {                                                                                           \
    const auto va = (a);                                                                         \
    const auto vb = (b);                                                                         \
    if (va != vb) {                                                                              \
      std::fprintf(stderr, "%s:%d CHECK_EQ(%s, %s) failed: %llx vs %llx\n", __FILE__, __LINE__,  \
                   #a, #b, (unsigned long long)va, (unsigned long long)vb);                      \
      ++g_fail;                                                                                  \
    }                                                                                            \
  } while (0)

namespace {
std::span<const std::byte> bytes_of(const std::string& s) { return std::as_bytes(std::span{s}); }

// The table generator stays usable in constant expressions, as the reference test requires.
constexpr auto kTable = generate_crc32_table();
static_assert(kTable[0] == 0x00000000u && kTable[1] == 0x77073096u);
static_assert(kTable[2] == 0xEE0E612Cu && kTable[255] == 0x2D02EF8Du);
static_assert(sizeof(crc32) == sizeof(std::uint32_t), "crc32 stays a 4-byte value type");

void table_generation() {
  CHECK_EQ(kTable[1], 0x77073096u);
  CHECK_EQ(kTable[255], 0x2D02EF8Du);
}

void empty_input() {
  crc32 c;
  CHECK_EQ(c.finalize(), 0x00000000u);
  CHECK_EQ(crc32{}.update({}).finalize(), 0x00000000u);
}

void known_values() {
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
  chunked.reset();
  CHECK_EQ(chunked.finalize(), 0u);
}

// wal_entry::encode's layout and CRC placement (wal.cpp:19-61).
std::vector<char> wal_encode(std::uint8_t op, std::uint64_t seq, const std::string& k, const std::string& v,
                             std::uint8_t tomb) {
  const std::uint32_t size = 26 + static_cast<std::uint32_t>(k.size() + v.size());
  std::vector<char> buf(size, 0);
  const std::uint32_t record_len = size - 8, klen = static_cast<std::uint32_t>(k.size()),
                      vlen = static_cast<std::uint32_t>(v.size());
  char* c = buf.data();
  std::memcpy(c, &record_len, 4);
  std::memcpy(c + 8, &op, 1);
  std::memcpy(c + 9, &seq, 8);
  std::memcpy(c + 17, &tomb, 1);
  std::memcpy(c + 18, &klen, 4);
  std::memcpy(c + 22, &vlen, 4);
  std::memcpy(c + 26, k.data(), klen);
  std::memcpy(c + 26 + klen, v.data(), vlen);
  const std::uint32_t crc =
      crc32{}.update({reinterpret_cast<const std::byte*>(buf.data()) + 8, size - 8u}).finalize();
  std::memcpy(c + 4, &crc, 4);
  return buf;
}

void wal_record_crc() {
  const auto rec = wal_encode(0, 42, "hello", "world", 0);
  std::uint32_t stored;
  std::memcpy(&stored, rec.data() + 4, 4);
  CHECK_EQ(stored, 0x593B861Au);  // tests/golden/wal.json (reference crc32 over the same bytes)
  // batched verification of a slurped log: both records good, then corrupt the second CRC
  std::vector<char> log = rec;
  const auto rec2 = wal_encode(0, 1, "k", "v", 0);
  log.insert(log.end(), rec2.begin(), rec2.end());
  std::uint64_t good = 0, stop = 0;
  CHECK_EQ(tkv_wal_verify(reinterpret_cast<const std::uint8_t*>(log.data()), log.size(), &good, &stop), (int)TKV_OK);
  CHECK_EQ(good, 2u);
  log[rec.size() + 4] = static_cast<char>(~log[rec.size() + 4]);
  CHECK_EQ(tkv_wal_verify(reinterpret_cast<const std::uint8_t*>(log.data()), log.size(), &good, &stop),
           (int)TKV_CORRUPTED);
  CHECK_EQ(good, 1u);
  CHECK_EQ(stop, rec.size());
}

void batch_host() {
  std::vector<std::uint8_t> data(1 << 20);
  for (std::size_t i = 0; i < data.size(); ++i) data[i] = static_cast<std::uint8_t>(i * 2654435761u >> 13);
  std::vector<std::uint64_t> off;
  std::vector<std::uint32_t> len;
  for (std::uint32_t i = 0; i < 200; ++i) {
    off.push_back(i * 5000u + (i % 7));
    len.push_back((i * 37u) % 4999u);
  }
  std::vector<std::uint32_t> out(off.size());
  CHECK_EQ(tkv_crc32_batch_host(data.data(), off.data(), len.data(), nullptr, out.data(), off.size()), (int)TKV_OK);
  for (std::size_t i = 0; i < off.size(); ++i) {
    const auto want =
        crc32{}.update(std::as_bytes(std::span<const std::uint8_t>(data.data() + off[i], len[i]))).finalize();
    CHECK_EQ(out[i], want);
  }
}
}  // namespace

int main() {
  table_generation();
  empty_input();
  known_values();
  incremental_equals_single();
  wal_record_crc();
  batch_host();
  std::printf("%s\n", g_fail ? "FAILED" : "ALL PASSED");
  return g_fail ? 1 : 0;
}
