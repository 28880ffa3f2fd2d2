// Record formats around the CRC engine: WAL record verify/stamp (the reference's call sites,
// /root/reference/src/engine/wal.cpp:54-58, 63-130) and SSTable data-block stamping (SURVEY.md §8f
// rank 2, format defined in include/tkv_crc32.h). The host walks lengths and places fields; every
// checksum over record or block bytes runs on the GPU through the engine (tkv_engine.h).
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "tkv_crc32.h"
#include "tkv_engine.h"
#include "tkv_wal_device.h"

using namespace tkv;

namespace {
bool ptr_ok(const void* p) { return p != nullptr; }

// crc_0 of the 4 little-endian bytes of v followed by z zero bytes: the term that turns the CRC of an
// SSTable image with `v` in its crc32_ field into the CRC with the field read as zero (linearity of
// the CRC over GF(2); the same identity sst_fix applies on the device).
// Shift_(2^k bytes) as byte-sliced linear maps, k < 40: Shift_z(c) is one 4-lookup step per set bit
// of z (about 40 lookups for a 4 KiB image) instead of a bitwise GF(2) multiply per image.
struct PowTables {
  std::uint32_t t[40][4][256];
  PowTables() {
    for (int k = 0; k < 40; ++k)
      for (int j = 0; j < 4; ++j)
        for (std::uint32_t v = 0; v < 256; ++v) t[k][j][v] = shift_bytes(v << (8 * j), std::uint64_t(1) << k, kPoly);
  }
};
const PowTables& pow_tables() {
  static const PowTables* p = new PowTables();
  return *p;
}

std::uint32_t field_term(std::uint32_t v, std::uint64_t z) {
  std::uint32_t c = 0;
  for (int k = 0; k < 4; ++k) {
    c ^= (v >> (8 * k)) & 0xFFu;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
  }
  const PowTables& pt = pow_tables();
  for (int k = 0; z; ++k, z >>= 1)
    if (z & 1u)
      c = pt.t[k][0][c & 0xFFu] ^ pt.t[k][1][(c >> 8) & 0xFFu] ^ pt.t[k][2][(c >> 16) & 0xFFu] ^ pt.t[k][3][c >> 24];
  return c;
}

// ---- WAL record_len chain (wal.cpp:63-87) ----------------------------------------------------------
constexpr std::uint64_t kWalMeta = 26;  // wal.hpp:21-27 kMetadataSize

struct Chain {
  std::vector<std::uint64_t> pos;  // record starts, in order
  std::vector<std::uint32_t> len;  // their record_len (payload bytes after the 8-byte prefix)
  std::vector<std::uint32_t> crc;  // their stored crc32 (offset 4)
  std::vector<std::uint8_t> kv_ok; // 26 + klen + vlen fits the record (wal.cpp:118-121)
  std::uint64_t end = 0;           // first position after the last record (a record start >= limit)
  bool err = false;                // the chain hit a header that does not fit (wal.cpp:68-70, 82-87)

  void append(const Chain& o, std::size_t from) {
    pos.insert(pos.end(), o.pos.begin() + from, o.pos.end());
    len.insert(len.end(), o.len.begin() + from, o.len.end());
    crc.insert(crc.end(), o.crc.begin() + from, o.crc.end());
    kv_ok.insert(kv_ok.end(), o.kv_ok.begin() + from, o.kv_ok.end());
    end = o.end;
    err = o.err;
  }
};

// Sequential walk from `start` over the records that START before `limit`.
void walk(const std::uint8_t* w, std::uint64_t size, std::uint64_t start, std::uint64_t limit, Chain& c) {
  std::uint64_t p = start;
  while (p < limit) {
    if (size - p < kWalMeta) {
      c.err = true;
      break;
    }
    std::uint32_t rlen, crc, klen, vlen;
    std::memcpy(&rlen, w + p, 4);
    if (static_cast<std::uint64_t>(rlen) + 8 > size - p) {
      c.err = true;
      break;
    }
    std::memcpy(&crc, w + p + 4, 4);  // the header's other fields share its cache line
    std::memcpy(&klen, w + p + 18, 4);
    std::memcpy(&vlen, w + p + 22, 4);
    c.pos.push_back(p);
    c.len.push_back(rlen);
    c.crc.push_back(crc);
    c.kv_ok.push_back(kWalMeta + static_cast<std::uint64_t>(klen) + vlen <= 8 + static_cast<std::uint64_t>(rlen));
    p += 8 + static_cast<std::uint64_t>(rlen);
  }
  c.end = p;
}

// Host threads for CPU-side work: the CPUs this process may run on, capped by OMP_NUM_THREADS (the
// GPU boxes' per-job CPU share) and 16.
unsigned host_threads() {
  unsigned n = 16;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::min<unsigned>(n, static_cast<unsigned>(CPU_COUNT(&set)));
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const long v = std::strtol(e, nullptr, 10);
    if (v > 0) n = std::min<unsigned>(n, static_cast<unsigned>(v));
  }
  return std::max(1u, n);
}

// fn(i) for i in [0, n): on host threads when n is large (field writes scattered over a big image).
template <class F>
void parallel_for(std::uint64_t n, F fn) {
  const unsigned nt = n >= (1u << 14) ? host_threads() : 1u;
  if (nt == 1) {
    for (std::uint64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=] {
      for (std::uint64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) fn(i);
    });
  for (auto& t : th) t.join();
}

// A header the reference encoder would write (wal.cpp:19-61): record_len = 18 + klen + vlen and the
// two flag bytes are 0/1. Used only to choose speculative starting points; never trusted.
bool plausible(const std::uint8_t* w, std::uint64_t size, std::uint64_t p) {
  if (size - p < kWalMeta) return false;
  std::uint32_t rlen, klen, vlen;
  std::memcpy(&rlen, w + p, 4);
  std::memcpy(&klen, w + p + 18, 4);
  std::memcpy(&vlen, w + p + 22, 4);
  return w[p + 8] <= 1 && w[p + 17] <= 1 && static_cast<std::uint64_t>(rlen) == 18ull + klen + vlen &&
         static_cast<std::uint64_t>(rlen) + 8 <= size - p;
}

// The chain of the whole image, identical to a sequential walk from 0. Each record start depends on
// the previous one, so one thread walking a large WAL is bound by DRAM latency (one dependent miss
// per record). Here the image is cut into K pieces; the walker of piece k>0 starts at the first
// plausible header at or after the cut (speculation). Stitching is exact: piece k's chain is used
// from the true entry point e_k (where the verified chain of pieces < k crosses the cut) onward only
// if e_k is one of its record starts (chains that share a start coincide from there); otherwise
// piece k is walked again from e_k.
// Records that START in [start, limit); c.end is the first record start >= limit (or where the
// chain broke).
Chain wal_chain(const std::uint8_t* w, std::uint64_t size, std::uint64_t start, std::uint64_t limit) {
  constexpr std::uint64_t kPiece = std::uint64_t(8) << 20;
  const std::uint64_t span = limit > start ? limit - start : 0;
  const unsigned K = static_cast<unsigned>(
      std::min<std::uint64_t>(host_threads(), std::max<std::uint64_t>(1, span / kPiece)));
  std::vector<std::uint64_t> cut(K + 1);
  for (unsigned k = 0; k <= K; ++k) cut[k] = start + span * k / K;
  std::vector<Chain> part(K);
  auto run = [&](unsigned k) {
    Chain local;  // built thread-locally: the Chain headers in `part` share cache lines
    std::uint64_t p = cut[k];
    if (k > 0) {
      while (p < cut[k + 1] && !plausible(w, size, p)) ++p;
      if (p >= cut[k + 1]) {
        local.end = p;
        local.err = true;  // no usable start: forces a re-walk if the chain needs this piece
        part[k] = std::move(local);
        return;
      }
    }
    walk(w, size, p, cut[k + 1], local);
    part[k] = std::move(local);
  };
  if (K == 1) {
    run(0);
    return std::move(part[0]);
  }
  std::vector<std::thread> th;
  for (unsigned k = 0; k < K; ++k) th.emplace_back(run, k);
  for (auto& t : th) t.join();
  Chain c = std::move(part[0]);
  for (unsigned k = 1; k < K && !c.err; ++k) {
    const std::uint64_t e = c.end;  // true entry point into piece k (or beyond it)
    if (e >= cut[k + 1]) continue;  // one record spans piece k entirely
    const auto& pk = part[k].pos;
    const auto it = std::lower_bound(pk.begin(), pk.end(), e);
    if (it != pk.end() && *it == e) {
      c.append(part[k], static_cast<std::size_t>(it - pk.begin()));
    } else {
      Chain r;
      walk(w, size, e, cut[k + 1], r);
      c.append(r, 0);
    }
  }
  return c;
}

Chain wal_chain(const std::uint8_t* w, std::uint64_t size) { return wal_chain(w, size, 0, size); }

int wal_verify_host_walk(const uint8_t* h_wal, uint64_t size, uint64_t* n_good, uint64_t* stop_offset);

int sst_check(const std::uint64_t* h_sizes, std::uint64_t n) {
  for (std::uint64_t i = 0; i < n; ++i)
    if (h_sizes[i] < TKV_SST_MIN_IMAGE || h_sizes[i] > 0xFFFFFFFFull)
      return set_error(TKV_INVALID_ARGUMENT, "SSTable block image shorter than 22 bytes or 4 GiB and longer");
  return TKV_OK;
}
}  // namespace

extern "C" {

int tkv_wal_verify(const uint8_t* h_wal, uint64_t size, uint64_t* n_good, uint64_t* stop_offset) {
  if ((size && !ptr_ok(h_wal)) || !ptr_ok(n_good) || !ptr_ok(stop_offset))
    return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  // The image goes to the device once; the chain walk, the CRC batch and the first-corruption
  // search run there (tkv_wal_device.hip). The host walk below is the exact fallback for images the
  // device cannot hold or whose chain the speculative device walk could not settle.
  bool host_walk = false;
  const int rc = wal_verify_host_image_impl(h_wal, size, n_good, stop_offset, &host_walk);
  if (!host_walk) return rc;
  return wal_verify_host_walk(h_wal, size, n_good, stop_offset);
}

int tkv_wal_verify_device(const uint8_t* d_wal, uint64_t size, uint64_t* n_good, uint64_t* stop_offset,
                          void* stream) {
  if ((size && !ptr_ok(d_wal)) || !ptr_ok(n_good) || !ptr_ok(stop_offset))
    return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (size == 0) {
    *n_good = *stop_offset = 0;
    return TKV_OK;
  }
  bool host_walk = false;
  const int rc = wal_verify_device_impl(d_wal, size, n_good, stop_offset, static_cast<hipStream_t>(stream), &host_walk);
  if (!host_walk) return rc;
  // exact fallback: the image comes back to the host for the sequential-stitched host walk
  std::vector<std::uint8_t> h(size);
  if (hipMemcpy(h.data(), d_wal, size, hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(TKV_IO_ERROR, "WAL image copy to host failed");
  return wal_verify_host_walk(h.data(), size, n_good, stop_offset);
}

}  // extern "C"

namespace {
// The host-walk verify (exact for every image): the record_len chain walked on host threads, the
// CRCs checked on the GPU through the host batch API.
int wal_verify_host_walk(const uint8_t* h_wal, uint64_t size, uint64_t* n_good, uint64_t* stop_offset) {
  // The record_len chain (wal.cpp:63-87), walked in parallel (wal_chain): records are
  // [u32 record_len][u32 crc][payload of record_len bytes]. Large images go in phases: the CRC
  // batch of phase j runs (GPU, on a helper thread) while the host walks phase j+1.
  const unsigned J = size >= (std::uint64_t(64) << 20) ? 4u : 1u;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(TKV_IO_ERROR, "hipGetDevice failed");
  std::vector<Chain> phase;
  phase.reserve(J);  // helper threads read phase[j] while later phases are appended
  std::vector<std::vector<std::uint32_t>> got(J);
  std::vector<std::vector<std::uint64_t>> off(J);
  std::vector<int> rcs(J, TKV_OK);
  std::vector<std::thread> crc_th;
  std::uint64_t start = 0;
  for (unsigned j = 0; j < J; ++j) {
    const std::uint64_t limit = j + 1 == J ? size : std::max(start, size * (j + 1) / J);
    phase.push_back(wal_chain(h_wal, size, start, limit));
    const Chain& ch = phase.back();
    const std::size_t nrec = ch.pos.size();
    off[j].resize(nrec);
    got[j].resize(nrec);
    for (std::size_t i = 0; i < nrec; ++i) off[j][i] = ch.pos[i] + 8;
    if (nrec)
      crc_th.emplace_back([&, j, nrec] {
        if (hipSetDevice(dev) != hipSuccess) {
          rcs[j] = TKV_IO_ERROR;
          return;
        }
        rcs[j] = batch_host_impl(kAlgoCrc32, h_wal, off[j].data(), phase[j].len.data(), nullptr, got[j].data(), nrec);
      });
    start = ch.end;
    if (ch.err || start >= size) break;
  }
  for (auto& t : crc_th) t.join();
  for (unsigned j = 0; j < J; ++j)
    if (rcs[j] != TKV_OK) return set_error(rcs[j], "WAL verify: CRC batch failed");
  Chain ch = std::move(phase[0]);
  for (std::size_t j = 1; j < phase.size(); ++j) ch.append(phase[j], 0);
  std::vector<std::uint32_t> all;
  all.reserve(ch.pos.size());
  for (std::size_t j = 0; j < phase.size(); ++j) all.insert(all.end(), got[j].begin(), got[j].end());
  const std::size_t nrec = ch.pos.size();
  std::uint64_t good = 0;
  // first record whose CRC (wal.cpp:93-96) or key/value bounds (wal.cpp:118-121) fail
  while (good < nrec && all[good] == ch.crc[good] && ch.kv_ok[good]) ++good;
  *n_good = good;
  *stop_offset = good < nrec ? ch.pos[good] : ch.end;
  if (good < nrec || ch.err) return set_error(TKV_CORRUPTED, "corrupted WAL record");
  return TKV_OK;
}
}  // namespace

extern "C" {

int tkv_wal_stamp(uint8_t* h_buf, const uint64_t* h_offsets, const uint32_t* h_sizes, uint64_t n) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_buf) || !ptr_ok(h_offsets) || !ptr_ok(h_sizes)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  std::vector<std::uint64_t> off(n);
  std::vector<std::uint32_t> len(n), crc(n);
  for (std::uint64_t i = 0; i < n; ++i) {
    if (h_sizes[i] < 8) return set_error(TKV_INVALID_ARGUMENT, "WAL record shorter than its 8-byte prefix");
    off[i] = h_offsets[i] + 8;  // wal.cpp:54-57: CRC over [8, size)
    len[i] = h_sizes[i] - 8;
  }
  if (int rc = batch_host_impl(kAlgoCrc32, h_buf, off.data(), len.data(), nullptr, crc.data(), n)) return rc;
  parallel_for(n, [&](std::uint64_t i) { std::memcpy(h_buf + h_offsets[i] + 4, &crc[i], 4); });  // wal.cpp:58
  return TKV_OK;
}


int tkv_sst_stamp_blocks(uint8_t* h_file, const uint64_t* h_offsets, const uint64_t* h_sizes, uint64_t n) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_file) || !ptr_ok(h_offsets) || !ptr_ok(h_sizes)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (int rc = sst_check(h_sizes, n)) return rc;
  std::vector<std::uint32_t> len(n), crc(n);
  parallel_for(n, [&](std::uint64_t i) {
    std::memset(h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, 0, 4);  // the field reads as zero
    len[i] = static_cast<std::uint32_t>(h_sizes[i]);
  });
  if (int rc = batch_host_impl(kAlgoCrc32, h_file, h_offsets, len.data(), nullptr, crc.data(), n)) return rc;
  parallel_for(n, [&](std::uint64_t i) { std::memcpy(h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, &crc[i], 4); });
  return TKV_OK;
}

int tkv_sst_verify_blocks(const uint8_t* h_file, const uint64_t* h_offsets, const uint64_t* h_sizes, uint64_t n,
                          uint64_t* n_bad, uint64_t* first_bad) {
  if (!ptr_ok(n_bad) || !ptr_ok(first_bad)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  *n_bad = 0;
  *first_bad = n;
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_file) || !ptr_ok(h_offsets) || !ptr_ok(h_sizes)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (int rc = sst_check(h_sizes, n)) return rc;
  std::vector<std::uint32_t> len(n), got(n);
  for (std::uint64_t i = 0; i < n; ++i) len[i] = static_cast<std::uint32_t>(h_sizes[i]);
  if (int rc = batch_host_impl(kAlgoCrc32, h_file, h_offsets, len.data(), nullptr, got.data(), n)) return rc;
  // stored vs CRC with the field read as zero, on host threads for large files
  const unsigned nt = n >= (1u << 14) ? host_threads() : 1u;
  std::vector<std::uint64_t> bad(nt, 0), first(nt, n);
  auto part = [&](unsigned t) {
    for (std::uint64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
      std::uint32_t stored;
      std::memcpy(&stored, h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, 4);
      const std::uint32_t want = got[i] ^ field_term(stored, h_sizes[i] - TKV_SST_CRC_OFFSET - 4);
      if (want != stored) {
        if (bad[t] == 0) first[t] = i;
        ++bad[t];
      }
    }
  };
  pow_tables();
  if (nt == 1) {
    part(0);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(part, t);
    for (auto& t : th) t.join();
  }
  for (unsigned t = 0; t < nt; ++t) {
    if (bad[t] && *n_bad == 0) *first_bad = first[t];
    *n_bad += bad[t];
  }
  return *n_bad ? set_error(TKV_CORRUPTED, "corrupted SSTable data block") : TKV_OK;
}

int tkv_sst_block_crcs_device(uint8_t* d_file, const uint64_t* d_offsets, const uint32_t* d_sizes, uint32_t* d_out,
                              uint64_t n, int store, void* stream) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(d_file) || !ptr_ok(d_offsets) || !ptr_ok(d_sizes) || !ptr_ok(d_out))
    return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (int rc = batch_device_impl(kAlgoCrc32, d_file, d_offsets, d_sizes, nullptr, d_out, n, stream)) return rc;
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  const hipError_t e = launch_sst_fix(d_file, d_offsets, d_sizes, d_out, n, store, tabs, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e));
  return TKV_OK;
}

}  // extern "C"

namespace {
// CRC-32 of index image || footer[0, 16): one engine update over the index, chained into a second
// over the footer's fields (the raw register carries across, as crc32::update chaining does).
int footer_crc(const std::uint8_t* h_index, std::uint64_t index_size, const std::uint8_t* h_footer,
               std::uint32_t* crc) {
  if ((index_size && !ptr_ok(h_index)) || !ptr_ok(h_footer)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  std::uint32_t raw = 0xFFFFFFFFu;
  if (int rc = update_impl(kAlgoCrc32, raw, h_index, index_size, &raw)) return rc;
  if (int rc = update_impl(kAlgoCrc32, raw, h_footer, TKV_SST_FOOTER_CRC_OFFSET, &raw)) return rc;
  *crc = raw ^ 0xFFFFFFFFu;
  return TKV_OK;
}
}  // namespace

extern "C" {

int tkv_sst_stamp_footer(const uint8_t* h_index, uint64_t index_size, uint8_t* h_footer) {
  std::uint32_t crc = 0;
  if (int rc = footer_crc(h_index, index_size, h_footer, &crc)) return rc;
  std::memcpy(h_footer + TKV_SST_FOOTER_CRC_OFFSET, &crc, 4);
  return TKV_OK;
}

int tkv_sst_verify_footer(const uint8_t* h_index, uint64_t index_size, const uint8_t* h_footer) {
  std::uint32_t crc = 0, stored = 0;
  if (int rc = footer_crc(h_index, index_size, h_footer, &crc)) return rc;
  std::memcpy(&stored, h_footer + TKV_SST_FOOTER_CRC_OFFSET, 4);
  return stored == crc ? TKV_OK : set_error(TKV_CORRUPTED, "corrupted SSTable index or footer");
}

size_t tkv_debug_wal_chain(const uint8_t* h_wal, uint64_t size, uint64_t* out_pos, size_t cap, uint64_t* end,
                           int* err) {
  const Chain c = wal_chain(h_wal, size);
  if (out_pos) std::memcpy(out_pos, c.pos.data(), std::min(cap, c.pos.size()) * sizeof(std::uint64_t));
  if (end) *end = c.end;
  if (err) *err = c.err ? 1 : 0;
  return c.pos.size();
}

}  // extern "C"
