// Host latency path for one short span.
//
// tinykvpp's only live caller checksums one ~36-byte WAL record per put (wal_entry::encode,
// /root/reference/src/engine/wal.cpp:54-57). Through the GPU every such call is a launch and a
// round trip (~20 us); on the host core that already holds the record it is a few table lookups.
// This file is that host path: slicing-by-8 over tables built from the polynomial, the same
// register semantics as crc32::update (crc32.cpp:9-16: no init or xorout applied here). Nothing in
// the library calls it; the drop-in header uses it for spans up to TKV_DROPIN_HOST_MAX bytes
// (default 64 KiB, the measured crossover with the GPU round trip), and the C ABI exposes it as the
// separately named tkv_crc32[c]_update_host. The GPU entry points never route here, with or without
// a device. The drop-in header alone calls tkv_crc32[c]_update_fallback after a GPU update of a
// long span returned an error, because the reference's crc32::update cannot fail (crc32.cpp:9-16):
// that call recomputes the span here, warns once per process and is counted in a slot of its own.
// Each call is counted per thread (tkv_debug_update_counts).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "tkv_crc32.h"

namespace tkv {
// Calls of this thread: [0] host span path (this file), [1] GPU update path (tkv_crc32_host.cpp),
// [2] host recomputes after a failed GPU update (tkv_crc32[c]_update_fallback).
// Thread-local plain counters: an atomic add would cost a third of a 36-byte span.
thread_local std::uint64_t g_update_calls[3] = {0, 0, 0};
}  // namespace tkv

namespace {

// T[k][e]: register contribution of byte value e followed by k zero bytes (slicing-by-8 tables).
struct SpanTables {
  std::uint32_t t[8][256];
  explicit SpanTables(std::uint32_t poly) {
    for (std::uint32_t e = 0; e < 256; ++e) {
      std::uint32_t c = e;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? poly : 0u);
      t[0][e] = c;
    }
    for (std::uint32_t e = 0; e < 256; ++e)
      for (int k = 1; k < 8; ++k) t[k][e] = (t[k - 1][e] >> 8) ^ t[0][t[k - 1][e] & 0xFFu];
  }
};

const SpanTables& tables(std::uint32_t poly) {
  static const SpanTables crc(TKV_CRC32_POLYNOMIAL);
  static const SpanTables crcc(0x82F63B78u);
  return poly == TKV_CRC32_POLYNOMIAL ? crc : crcc;
}

std::uint32_t span_update(const SpanTables& T, std::uint32_t r, const unsigned char* p, std::size_t n) {
  while (n >= 8) {
    std::uint64_t w;
    std::memcpy(&w, p, 8);  // little-endian host (x86-64), as the device path assumes
    w ^= r;
    r = T.t[7][w & 0xFFu] ^ T.t[6][(w >> 8) & 0xFFu] ^ T.t[5][(w >> 16) & 0xFFu] ^ T.t[4][(w >> 24) & 0xFFu] ^
        T.t[3][(w >> 32) & 0xFFu] ^ T.t[2][(w >> 40) & 0xFFu] ^ T.t[1][(w >> 48) & 0xFFu] ^ T.t[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) r = (r >> 8) ^ T.t[0][(r ^ *p++) & 0xFFu];
  return r;
}

int update_host(std::uint32_t poly, std::uint32_t raw, const void* data, std::size_t len, std::uint32_t* out_raw) {
  if (out_raw == nullptr || (data == nullptr && len != 0)) return TKV_INVALID_ARGUMENT;
  ++tkv::g_update_calls[0];
  *out_raw = len ? span_update(tables(poly), raw, static_cast<const unsigned char*>(data), len) : raw;
  return TKV_OK;
}

std::atomic<bool> g_fallback_warned{false};

int update_fallback(std::uint32_t poly, int gpu_status, std::uint32_t raw, const void* data, std::size_t len,
                    std::uint32_t* out_raw) {
  if (out_raw == nullptr || (data == nullptr && len != 0)) return TKV_INVALID_ARGUMENT;
  ++tkv::g_update_calls[2];
  if (!g_fallback_warned.exchange(true, std::memory_order_relaxed))
    std::fprintf(stderr,
                 "libtkv_crc32: a GPU update of %zu bytes failed (status %d: %s); this and later failed "
                 "updates are recomputed on the host (warned once per process)\n",
                 len, gpu_status, tkv_last_error());
  *out_raw = len ? span_update(tables(poly), raw, static_cast<const unsigned char*>(data), len) : raw;
  return TKV_OK;
}

}  // namespace

extern "C" {

int tkv_crc32_update_host(uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  return update_host(TKV_CRC32_POLYNOMIAL, raw_state, data, len, out_raw);
}

int tkv_crc32c_update_host(uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  return update_host(0x82F63B78u, raw_state, data, len, out_raw);
}

int tkv_crc32_update_fallback(int gpu_status, uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  return update_fallback(TKV_CRC32_POLYNOMIAL, gpu_status, raw_state, data, len, out_raw);
}

int tkv_crc32c_update_fallback(int gpu_status, uint32_t raw_state, const void* data, size_t len,
                               uint32_t* out_raw) {
  return update_fallback(0x82F63B78u, gpu_status, raw_state, data, len, out_raw);
}

void tkv_debug_update_counts(uint64_t out[2]) {
  out[0] = tkv::g_update_calls[0];
  out[1] = tkv::g_update_calls[1];
}

size_t tkv_debug_update_counts_n(uint64_t* out, size_t n) {
  for (size_t i = 0; i < n && i < 3; ++i) out[i] = tkv::g_update_calls[i];
  return 3;
}

}  // extern "C"
