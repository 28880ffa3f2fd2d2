// Per-put cost of the drop-in (not product code): frankie::core::crc32{}.update(record).finalize()
// through include/frankie_crc32.hpp (libtkv_crc32.so, the GPU path) next to the reference's own
// crc32.cpp (oracle/_ref/libref_crc32.so, loaded with dlopen; test-side only), for the WAL record
// sizes of wal_entry::encode (/root/reference/src/engine/wal.cpp:54-57), and the batched
// alternative: tkv_wal_stamp over N records (group commit). One JSON line per measurement.
// Build: make -C tools put_latency (needs oracle/_ref built from /root/reference).
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "frankie_crc32.hpp"

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const char* ref_path = argc > 1 ? argv[1] : "oracle/_ref/libref_crc32.so";
  void* h = dlopen(ref_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "cannot load %s: %s\n", ref_path, dlerror());
    return 1;
  }
  using ref_fn = std::uint32_t (*)(const unsigned char*, std::size_t);
  auto ref_crc32 = reinterpret_cast<ref_fn>(dlsym(h, "ref_crc32"));
  if (!ref_crc32 || tkv_set_device(0) != TKV_OK) return 1;
  std::mt19937_64 rng(1);
  std::vector<unsigned char> buf((2 << 20) + 256);
  for (auto& b : buf) b = static_cast<unsigned char>(rng());
  auto us_per = [](auto&& fn, int reps) {
    auto t0 = clk::now();
    for (int i = 0; i < reps; ++i) fn(i);
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
  };
  for (std::size_t n : {28ul, 36ul, 128ul, 1024ul, 4096ul, 16384ul, 65536ul, 131072ul, 262144ul, 1048576ul, 2097152ul}) {
    const auto* p = reinterpret_cast<const std::byte*>(buf.data());
    std::uint32_t sink = 0;
    // the GPU path itself (C ABI tkv_crc32_update), whatever the drop-in's threshold
    auto gpu = [&](int i) {
      std::uint32_t r = 0;
      (void)tkv_crc32_update(0xFFFFFFFFu, buf.data() + (i & 255), n, &r);
      sink ^= r;
    };
    for (int i = 0; i < 20; ++i) gpu(i);
    const int greps = n <= 16384 ? 2000 : 300;
    const double gpu_us = us_per(gpu, greps);
    const int rreps = static_cast<int>(std::max<std::size_t>(50, (std::size_t(200) << 20) / (n + 64)));
    const double ref_us = us_per([&](int i) { sink ^= ref_crc32(buf.data() + (i & 255), n); }, rreps);
    // the host span path (what the drop-in runs for spans <= TKV_DROPIN_HOST_MAX)
    const double host_us = us_per([&](int i) {
      std::uint32_t r = 0;
      (void)tkv_crc32_update_host(0xFFFFFFFFu, buf.data() + (i & 255), n, &r);
      sink ^= r;
    }, rreps);
    // the drop-in header as built (default threshold)
    const double dropin_us = us_per([&](int i) { sink ^= frankie::core::crc32{}.update({p + (i & 255), n}).finalize(); },
                                    n <= TKV_DROPIN_HOST_MAX ? rreps : greps);
    std::uint32_t hr = 0, gr = 0;
    (void)tkv_crc32_update_host(0xFFFFFFFFu, buf.data(), n, &hr);
    (void)tkv_crc32_update(0xFFFFFFFFu, buf.data(), n, &gr);
    const std::uint32_t want = ref_crc32(buf.data(), n);
    const bool same = frankie::core::crc32{}.update({p, n}).finalize() == want && (hr ^ 0xFFFFFFFFu) == want &&
                      (gr ^ 0xFFFFFFFFu) == want;
    std::printf("{\"row\": \"drop_in_update\", \"bytes\": %zu, \"gpu_us_per_call\": %.3f, \"host_span_us_per_call\": %.3f, "
                "\"drop_in_default_us_per_call\": %.3f, \"drop_in_host_max\": %d, \"reference_cpu_us_per_call\": %.3f, "
                "\"bit_exact\": %s, \"sink\": %u}\n", n, gpu_us, host_us, dropin_us, TKV_DROPIN_HOST_MAX, ref_us,
                same ? "true" : "false", sink & 1u);
    std::fflush(stdout);
  }
  // group commit: N records of 36 bytes stamped in one call (wal.cpp:54-58 per record)
  for (std::size_t nrec : {1ul, 16ul, 256ul, 4096ul}) {
    std::vector<std::uint64_t> off(nrec);
    std::vector<std::uint32_t> sz(nrec, 36);
    for (std::size_t i = 0; i < nrec; ++i) off[i] = 36 * i;
    std::vector<unsigned char> img(36 * nrec);
    std::memcpy(img.data(), buf.data(), img.size());
    for (int i = 0; i < 10; ++i) tkv_wal_stamp(img.data(), off.data(), sz.data(), nrec);
    const int reps = 200;
    auto t0 = clk::now();
    for (int i = 0; i < reps; ++i) tkv_wal_stamp(img.data(), off.data(), sz.data(), nrec);
    const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
    std::printf("{\"row\": \"group_commit_stamp\", \"records\": %zu, \"record_bytes\": 36, \"us_per_call\": %.2f, "
                "\"us_per_record\": %.3f}\n", nrec, us, us / nrec);
  }
  return 0;
}
