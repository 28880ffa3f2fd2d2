// Record formats around the CRC engine: WAL record verify/stamp (the reference's call sites,
// /root/reference/src/engine/wal.cpp:54-58, 63-130) and SSTable data-block stamping (SURVEY.md §8f
// rank 2, format defined in include/tkv_crc32.h). The host walks lengths and places fields; every
// checksum over record or block bytes runs on the GPU through the engine (tkv_engine.h).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "tkv_crc32.h"
#include "tkv_engine.h"

using namespace tkv;

namespace {
bool ptr_ok(const void* p) { return p != nullptr; }

// crc_0 of the 4 little-endian bytes of v followed by z zero bytes: the term that turns the CRC of an
// SSTable image with `v` in its crc32_ field into the CRC with the field read as zero (linearity of
// the CRC over GF(2); the same identity sst_fix applies on the device).
std::uint32_t field_term(std::uint32_t v, std::uint64_t z) {
  std::uint32_t c = 0;
  for (int k = 0; k < 4; ++k) {
    c ^= (v >> (8 * k)) & 0xFFu;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
  }
  return shift_bytes(c, z, kPoly);
}

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
  // Walk the record_len chain (wal.cpp:63-87): each record is [u32 record_len][u32 crc][payload].
  constexpr std::uint64_t kMeta = 26;  // wal.hpp:21-27 kMetadataSize
  std::vector<std::uint64_t> off;
  std::vector<std::uint32_t> len, stored;
  std::uint64_t pos = 0;
  bool structural_error = false;
  while (pos < size) {
    const std::uint64_t left = size - pos;
    if (left < kMeta) {
      structural_error = true;  // wal.cpp:68-70
      break;
    }
    std::uint32_t rlen, crc;
    std::memcpy(&rlen, h_wal + pos, 4);
    std::memcpy(&crc, h_wal + pos + 4, 4);
    if (static_cast<std::uint64_t>(rlen) + 8 > left) {
      structural_error = true;  // wal.cpp:82-87
      break;
    }
    off.push_back(pos + 8);
    len.push_back(rlen);
    stored.push_back(crc);
    pos += 8 + static_cast<std::uint64_t>(rlen);
  }
  std::vector<std::uint32_t> got(off.size());
  if (!off.empty()) {
    if (int rc = batch_host_impl(kAlgoCrc32, h_wal, off.data(), len.data(), nullptr, got.data(), off.size())) return rc;
  }
  std::uint64_t good = 0, stop = 0;
  for (; good < off.size(); ++good) {
    if (got[good] != stored[good]) break;  // wal.cpp:93-96
    // key/value bounds inside the payload (wal.cpp:118-121)
    const std::uint8_t* rec = h_wal + off[good] - 8;
    std::uint32_t klen, vlen;
    std::memcpy(&klen, rec + 18, 4);
    std::memcpy(&vlen, rec + 22, 4);
    if (kMeta + static_cast<std::uint64_t>(klen) + vlen > 8 + static_cast<std::uint64_t>(len[good])) break;
  }
  stop = good < off.size() ? off[good] - 8 : pos;
  *n_good = good;
  *stop_offset = stop;
  if (good < off.size() || structural_error) return set_error(TKV_CORRUPTED, "corrupted WAL record");
  return TKV_OK;
}

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
  for (std::uint64_t i = 0; i < n; ++i) std::memcpy(h_buf + h_offsets[i] + 4, &crc[i], 4);  // wal.cpp:58
  return TKV_OK;
}


int tkv_sst_stamp_blocks(uint8_t* h_file, const uint64_t* h_offsets, const uint64_t* h_sizes, uint64_t n) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_file) || !ptr_ok(h_offsets) || !ptr_ok(h_sizes)) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (int rc = sst_check(h_sizes, n)) return rc;
  std::vector<std::uint32_t> len(n), crc(n);
  for (std::uint64_t i = 0; i < n; ++i) {
    std::memset(h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, 0, 4);  // the field reads as zero
    len[i] = static_cast<std::uint32_t>(h_sizes[i]);
  }
  if (int rc = batch_host_impl(kAlgoCrc32, h_file, h_offsets, len.data(), nullptr, crc.data(), n)) return rc;
  for (std::uint64_t i = 0; i < n; ++i) std::memcpy(h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, &crc[i], 4);
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
  for (std::uint64_t i = 0; i < n; ++i) {
    std::uint32_t stored;
    std::memcpy(&stored, h_file + h_offsets[i] + TKV_SST_CRC_OFFSET, 4);
    const std::uint32_t want = got[i] ^ field_term(stored, h_sizes[i] - TKV_SST_CRC_OFFSET - 4);
    if (want != stored) {
      if (*n_bad == 0) *first_bad = i;
      ++*n_bad;
    }
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
