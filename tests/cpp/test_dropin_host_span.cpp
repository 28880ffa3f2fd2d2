// The drop-in header as a maintainer gets it (default TKV_DROPIN_HOST_MAX = 64 KiB, built by
// tests/test_host_span.py with no -D flag): the reference's crc32_test.cpp known answers (:81-124)
// and wal_entry::encode's record CRC (wal.cpp:54-57, tests/golden/wal.json) through
// frankie::core::crc32, every length up to the threshold, and the reference's contract: update never
// fails and touches no GPU for these spans (this runs on a machine without one; the per-thread
// counters of tkv_debug_update_counts_n show every call on the host path). It also times a 36-byte put
// (wal_entry::encode's {put, 42, "hello", "world"}) against the reference's byte loop
// (crc32.cpp:9-16, restated inline) on the same core.
//
// Spans above the threshold go to the GPU. The reference's update cannot fail, so on a node without
// a usable GPU (this container) the header recomputes them on the host after the GPU call's error
// (tkv_crc32_update_fallback): a 1 MiB span and a 128 KiB WAL record (a put with a 128 KiB value,
// wal.cpp:25) must return the byte loop's value without aborting, and the counters must show the GPU
// attempt and the host recompute (slot 2). With a GPU (tests/test_gpu_parity.py runs this binary
// too) the same spans take the GPU and slot 2 stays 0.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <span>
#include <string>
#include <vector>

#include "frankie_crc32.hpp"

#if TKV_DROPIN_HOST_MAX < 65536
#error "this test checks the default threshold (64 KiB)"
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

// A 36-byte put through the default header against the reference's byte loop, same bytes, same core.
void put_cost() {
  constexpr auto T = generate_crc32_table();
  std::vector<std::byte> rec(36 + 256);
  for (std::size_t i = 0; i < rec.size(); ++i) rec[i] = static_cast<std::byte>((i * 40503u) >> 3);
  using clk = std::chrono::steady_clock;
  constexpr int reps = 2000000;
  std::uint32_t sink = 0;
  auto t0 = clk::now();
  for (int i = 0; i < reps; ++i) sink ^= crc32{}.update({rec.data() + (i & 255), 36}).finalize();
  const double ours = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
  t0 = clk::now();
  for (int i = 0; i < reps; ++i) {
    std::uint32_t r = 0xFFFFFFFFu;  // crc32.cpp:9-16, one byte per step
    const std::byte* p = rec.data() + (i & 255);
    for (std::size_t k = 0; k < 36; ++k) r = (r >> 8) ^ T[(r ^ static_cast<std::uint32_t>(p[k])) & 0xFFu];
    sink ^= r ^ 0xFFFFFFFFu;
  }
  const double ref = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
  std::printf("put_cost_36B: drop-in %.4f us, reference byte loop %.4f us (sink %u)\n", ours, ref, sink & 1u);
  if (!(ours <= ref)) {
    std::fprintf(stderr, "a 36-byte put through the drop-in (%.4f us) is slower than the reference loop (%.4f us)\n",
                 ours, ref);
    ++g_fail;
  }
}

// Every length up to the threshold against the byte-at-a-time definition (crc32.cpp:9-16).
void all_lengths() {
  constexpr auto T = generate_crc32_table();
  std::vector<std::byte> d(TKV_DROPIN_HOST_MAX);
  for (std::size_t i = 0; i < d.size(); ++i) d[i] = static_cast<std::byte>((i * 2654435761u) >> 11);
  for (std::size_t n = 0; n <= d.size(); n += (n < 130 ? 1 : 611)) {
    std::uint32_t r = 0xFFFFFFFFu;
    for (std::size_t i = 0; i < n; ++i) r = (r >> 8) ^ T[(r ^ static_cast<std::uint32_t>(d[i])) & 0xFFu];
    CHECK_EQ(crc32{}.update({d.data(), n}).finalize(), r ^ 0xFFFFFFFFu);
  }
}
std::uint32_t byte_loop(const std::byte* p, std::size_t n) {
  constexpr auto T = generate_crc32_table();
  std::uint32_t r = 0xFFFFFFFFu;  // crc32.cpp:9-16
  for (std::size_t i = 0; i < n; ++i) r = (r >> 8) ^ T[(r ^ static_cast<std::uint32_t>(p[i])) & 0xFFu];
  return r ^ 0xFFFFFFFFu;
}

// Spans longer than the threshold: the GPU, or the host recompute after its error.
void long_spans() {
  std::uint64_t c0[3], c1[3];
  tkv_debug_update_counts_n(c0, 3);
  std::vector<std::byte> big(1u << 20);
  for (std::size_t i = 0; i < big.size(); ++i) big[i] = static_cast<std::byte>((i * 2246822519u) >> 13);
  CHECK_EQ(crc32{}.update({big.data(), big.size()}).finalize(), byte_loop(big.data(), big.size()));
  // wal_entry::encode (wal.cpp:19-61) of {put, seq 7, 16-byte key, 128 KiB value}; CRC over [8, size).
  const std::uint32_t klen = 16, vlen = 128u << 10, size = 26 + klen + vlen, record_len = size - 8;
  const std::uint64_t seq = 7;
  std::vector<std::byte> rec(size, std::byte{0});
  std::memcpy(rec.data(), &record_len, 4);
  std::memcpy(rec.data() + 9, &seq, 8);
  std::memcpy(rec.data() + 18, &klen, 4);
  std::memcpy(rec.data() + 22, &vlen, 4);
  for (std::uint32_t i = 0; i < klen + vlen; ++i) rec[26 + i] = static_cast<std::byte>((i * 40503u) >> 5);
  const std::uint32_t crc = crc32{}.update({rec.data() + 8, size - 8u}).finalize();
  CHECK_EQ(crc, byte_loop(rec.data() + 8, size - 8u));
  // chained: a short host span, then a long one, then a short one
  crc32 chained;
  (void)chained.update({rec.data() + 8, 100}).update({rec.data() + 108, 100000}).update({rec.data() + 100108, 7});
  CHECK_EQ(chained.finalize(), byte_loop(rec.data() + 8, 100107));
  tkv_debug_update_counts_n(c1, 3);
  const bool gpu = tkv_device_count() > 0;
  std::printf("long_spans: %s; GPU calls %llu, host recomputes %llu\n", gpu ? "GPU present" : "no GPU",
              (unsigned long long)(c1[1] - c0[1]), (unsigned long long)(c1[2] - c0[2]));
  CHECK_EQ(c1[1] - c0[1], 3u);  // every long span went to the GPU first
  CHECK_EQ(c1[2] - c0[2], gpu ? 0u : 3u);
  CHECK_EQ(c1[0] - c0[0], 2u);  // the two short spans of the chain
}
}  // namespace

int main() {
  std::uint64_t c0[3], c1[3];
  tkv_debug_update_counts_n(c0, 3);
  known_values();
  incremental_equals_single();
  wal_record_crc();
  all_lengths();
  {  // the threshold itself: a 64 KiB span is still a host span
    std::vector<std::byte> big(TKV_DROPIN_HOST_MAX, std::byte{7});
    (void)crc32{}.update({big.data(), big.size()}).finalize();
  }
  tkv_debug_update_counts_n(c1, 3);
  CHECK_EQ(c1[1] - c0[1], 0u);   // no call took the GPU path
  if (c1[0] - c0[0] < 200) {      // every update above was a host span
    std::fprintf(stderr, "only %llu host span calls counted\n", (unsigned long long)(c1[0] - c0[0]));
    ++g_fail;
  }
  long_spans();
  put_cost();
  std::printf("%s\n", g_fail ? "FAILED" : "ALL PASSED");
  return g_fail ? 1 : 0;
}
