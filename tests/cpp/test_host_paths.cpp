// Host-runtime stress test of libtkv_crc32's host-memory paths, built with AddressSanitizer and
// UndefinedBehaviorSanitizer on the host side (tinykvpp_amd/csrc/Makefile target `sanitize`; the
// device code is not instrumented). SURVEY.md §5: the host shim runs worker threads (multi-device
// split, WAL chain walk, CRC phases, threaded field writes), so it is exercised here under the
// sanitizers, including concurrent callers on one device. Every result is checked against the test
// oracle (oracle/crc32_oracle.c, linked into this test only). Needs a GPU; prints ALL PASSED.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "tkv_crc32.h"

extern "C" {
uint32_t oracle_crc32(const uint8_t* p, size_t n);
uint32_t oracle_update(uint32_t raw, const uint8_t* p, size_t n);
uint32_t oracle_sst_stamp(const uint8_t* img, size_t size);
}

static int g_fail = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "%s:%d CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                               \
    }                                                                         \
  } while (0)

namespace {

std::vector<uint8_t> random_bytes(std::mt19937_64& rng, size_t n) {
  std::vector<uint8_t> v(n);
  for (size_t i = 0; i < n; i += 8) {
    const uint64_t r = rng();
    std::memcpy(v.data() + i, &r, std::min<size_t>(8, n - i));
  }
  return v;
}

struct Batch {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  std::vector<uint32_t> init;
  uint64_t bytes = 0;
};

// Irregular batch: lengths 0..maxlen (some huge), packed with gaps, ascending.
Batch make_batch(std::mt19937_64& rng, size_t n, uint32_t maxlen) {
  Batch b;
  uint64_t p = 3;
  for (size_t i = 0; i < n; ++i) {
    uint32_t l = static_cast<uint32_t>(rng() % (maxlen + 1));
    if (i % 97 == 0) l = static_cast<uint32_t>(rng() % 4);
    b.off.push_back(p);
    b.len.push_back(l);
    b.init.push_back(static_cast<uint32_t>(rng()));
    p += l + rng() % 16;
  }
  b.bytes = p + 64;
  return b;
}

void check_batch(const uint8_t* base, const Batch& b, const std::vector<uint32_t>& got, bool with_init) {
  for (size_t i = 0; i < b.off.size(); ++i) {
    const uint32_t want = with_init ? oracle_update(b.init[i], base + b.off[i], b.len[i]) ^ 0xFFFFFFFFu
                                    : oracle_crc32(base + b.off[i], b.len[i]);
    if (got[i] != want) {
      std::fprintf(stderr, "block %zu (len %u): %08x vs %08x\n", i, b.len[i], got[i], want);
      ++g_fail;
      return;
    }
  }
}

void host_batches(std::mt19937_64& rng) {
  const Batch b = make_batch(rng, 20000, 20000);
  std::vector<uint8_t> pageable = random_bytes(rng, b.bytes);
  uint8_t* pinned = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pinned), b.bytes, hipHostMallocDefault) == hipSuccess);
  std::memcpy(pinned, pageable.data(), b.bytes);
  std::vector<uint32_t> got(b.off.size());
  const int dev2[2] = {0, 0};
  for (const uint8_t* base : {static_cast<const uint8_t*>(pageable.data()), static_cast<const uint8_t*>(pinned)}) {
    CHECK(tkv_crc32_batch_host(base, b.off.data(), b.len.data(), nullptr, got.data(), got.size()) == TKV_OK);
    check_batch(base, b, got, false);
    CHECK(tkv_crc32_batch_host(base, b.off.data(), b.len.data(), b.init.data(), got.data(), got.size()) == TKV_OK);
    check_batch(base, b, got, true);
    CHECK(tkv_crc32_batch_host_multi(dev2, 2, base, b.off.data(), b.len.data(), nullptr, got.data(), got.size()) ==
          TKV_OK);
    check_batch(base, b, got, false);
  }
  CHECK(hipHostFree(pinned) == hipSuccess);
}

// Blocks of >= 1 MiB straddling device shares are cut and recombined (multi-device split path),
// with and without per-block initial registers, over 2-4 "devices" (device 0 repeated).
void split_batches(std::mt19937_64& rng) {
  Batch b;
  const uint32_t lens[] = {(3u << 20) + 1, 0, (2u << 20) + 77, 100, 1u << 20, (4u << 20) - 3, 9u << 20};
  uint64_t p = 5;
  for (uint32_t l : lens) {
    b.off.push_back(p);
    b.len.push_back(l);
    b.init.push_back(static_cast<uint32_t>(rng()));
    p += l + 3;
  }
  b.bytes = p + 64;
  std::vector<uint8_t> data = random_bytes(rng, b.bytes);
  std::vector<uint32_t> got(b.off.size());
  const int devs[4] = {0, 0, 0, 0};
  for (int nd = 2; nd <= 4; ++nd) {
    CHECK(tkv_crc32_batch_host_multi(devs, nd, data.data(), b.off.data(), b.len.data(), nullptr, got.data(),
                                     got.size()) == TKV_OK);
    check_batch(data.data(), b, got, false);
    CHECK(tkv_crc32_batch_host_multi(devs, nd, data.data(), b.off.data(), b.len.data(), b.init.data(), got.data(),
                                     got.size()) == TKV_OK);
    check_batch(data.data(), b, got, true);
  }
}

// Several host threads calling into the same device at once: update() on spans of every size
// (latency kernel up to 16 KiB, staged above), large host batches (staged pipeline), small host
// batches (one latency-kernel launch) and the host span path.
void concurrent_callers(std::mt19937_64& rng) {
  std::vector<std::vector<uint8_t>> data;
  for (int t = 0; t < 6; ++t) data.push_back(random_bytes(rng, (size_t(1) << 20) + 12345 * t));
  std::vector<int> bad(6, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < 6; ++t)
    th.emplace_back([&, t] {
      const auto& d = data[t];
      for (int it = 0; it < 20; ++it) {
        if (t % 3 == 0) {
          const size_t n = it % 2 ? (it * 7919 + 31 * t) % d.size() : (it * 977 + 31 * t) % 20000;
          uint32_t raw = 0;
          if (tkv_crc32_update(0xFFFFFFFFu, d.data(), n, &raw) != TKV_OK || (raw ^ 0xFFFFFFFFu) != oracle_crc32(d.data(), n))
            ++bad[t];
        } else if (t % 3 == 2) {
          std::vector<uint64_t> off;
          std::vector<uint32_t> len;
          for (int i = 0; i < 1 + (it * 37) % 256; ++i) {
            off.push_back((static_cast<uint64_t>(i) * 4099u + it) % (d.size() - 300));
            len.push_back(static_cast<uint32_t>((i * 13 + it) % 250));
          }
          std::vector<uint32_t> got(off.size());
          if (tkv_crc32_batch_host(d.data(), off.data(), len.data(), nullptr, got.data(), off.size()) != TKV_OK) ++bad[t];
          for (size_t i = 0; i < off.size(); ++i) {
            uint32_t hr = 0;
            if (got[i] != oracle_crc32(d.data() + off[i], len[i]) ||
                tkv_crc32_update_host(0xFFFFFFFFu, d.data() + off[i], len[i], &hr) != TKV_OK || (hr ^ 0xFFFFFFFFu) != got[i]) {
              ++bad[t];
              break;
            }
          }
        } else {
          std::vector<uint64_t> off;
          std::vector<uint32_t> len;
          for (size_t p = 0; p + 5000 < d.size(); p += 5000 + it) {
            off.push_back(p);
            len.push_back(static_cast<uint32_t>(1000 + (p % 4000)));
          }
          std::vector<uint32_t> got(off.size());
          if (tkv_crc32_batch_host(d.data(), off.data(), len.data(), nullptr, got.data(), off.size()) != TKV_OK) ++bad[t];
          for (size_t i = 0; i < off.size(); ++i)
            if (got[i] != oracle_crc32(d.data() + off[i], len[i])) {
              ++bad[t];
              break;
            }
        }
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < 6; ++t) CHECK(bad[t] == 0);
}

// A WAL image of >= 64 MiB (phased verify with helper threads), stamped and verified; then a
// corrupted record in a late phase.
void wal_roundtrip(std::mt19937_64& rng) {
  std::vector<uint8_t> wal;
  std::vector<uint64_t> off;
  std::vector<uint32_t> size;
  uint64_t seq = 0;
  while (wal.size() < (size_t(70) << 20)) {
    const uint32_t klen = rng() % 40, vlen = static_cast<uint32_t>(rng() % 3000);
    const uint32_t rec = 26 + klen + vlen, rlen = rec - 8;
    off.push_back(wal.size());
    size.push_back(rec);
    const size_t o = wal.size();
    wal.resize(o + rec);
    std::memcpy(&wal[o], &rlen, 4);
    std::memset(&wal[o + 4], 0, 4);
    wal[o + 8] = 0;
    std::memcpy(&wal[o + 9], &seq, 8);
    wal[o + 17] = 0;
    std::memcpy(&wal[o + 18], &klen, 4);
    std::memcpy(&wal[o + 22], &vlen, 4);
    for (uint32_t i = 26; i < rec; ++i) wal[o + i] = static_cast<uint8_t>(rng());
    ++seq;
  }
  CHECK(tkv_wal_stamp(wal.data(), off.data(), size.data(), off.size()) == TKV_OK);
  for (size_t i = 0; i < off.size(); i += off.size() / 50) {
    uint32_t stored;
    std::memcpy(&stored, &wal[off[i] + 4], 4);
    CHECK(stored == oracle_crc32(&wal[off[i] + 8], size[i] - 8));
  }
  uint64_t good = 0, stop = 0;
  CHECK(tkv_wal_verify(wal.data(), wal.size(), &good, &stop) == TKV_OK);
  CHECK(good == off.size() && stop == wal.size());
  const size_t bad = off.size() * 7 / 8;
  wal[off[bad] + 30] ^= 1;
  CHECK(tkv_wal_verify(wal.data(), wal.size(), &good, &stop) == TKV_CORRUPTED);
  CHECK(good == bad && stop == off[bad]);
}

void sst_roundtrip(std::mt19937_64& rng) {
  const size_t n = 40000, sz = 4096;
  std::vector<uint8_t> file = random_bytes(rng, n * sz);
  std::vector<uint64_t> off(n), size(n, sz);
  for (size_t i = 0; i < n; ++i) {
    off[i] = i * sz;
    file[off[i]] = 20;
  }
  CHECK(tkv_sst_stamp_blocks(file.data(), off.data(), size.data(), n) == TKV_OK);
  for (size_t i = 0; i < n; i += 997) {
    uint32_t stored;
    std::memcpy(&stored, &file[off[i] + TKV_SST_CRC_OFFSET], 4);
    CHECK(stored == oracle_sst_stamp(&file[off[i]], sz));
  }
  uint64_t nbad = 0, first = 0;
  CHECK(tkv_sst_verify_blocks(file.data(), off.data(), size.data(), n, &nbad, &first) == TKV_OK && nbad == 0);
  file[off[31337] + 100] ^= 4;
  CHECK(tkv_sst_verify_blocks(file.data(), off.data(), size.data(), n, &nbad, &first) == TKV_CORRUPTED);
  CHECK(nbad == 1 && first == 31337);
}

}  // namespace

int main() {
  if (tkv_device_count() < 1) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  std::mt19937_64 rng(2024);
  host_batches(rng);
  split_batches(rng);
  concurrent_callers(rng);
  wal_roundtrip(rng);
  sst_roundtrip(rng);
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("ALL PASSED\n");
  return 0;
}
