// Device-side WAL recovery verify (tkv_wal_device.hip), used by tkv_wal_verify and
// tkv_wal_verify_device (tkv_formats.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkv {

// One pass of the device verify over an image that starts with a record (tkv_wal_device.hip).
struct PassResult {
  std::uint64_t good = 0;  // records verified good from the pass's start
  std::uint64_t stop = 0;  // where decoding stopped (relative to the pass's start)
  bool corrupted = false;
  bool resume = false;     // the chain continues at `stop` (a true record start) beyond what was checked
};


// Verify the WAL image [d_wal, d_wal + size) in device memory on `st` (synchronous): the record
// chain walked on the device, one CRC batch, the first bad record. Same results as tkv_wal_verify.
// *needs_host_walk is set (and nothing else is decided) when the speculative walk could not settle
// the chain within its pass budget; the caller then runs the exact host walk.
int wal_verify_device_impl(const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                           std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk);

// Host image: copied into a device buffer kept per device (pinned sources in one copy, pageable ones
// through pinned staging slabs filled by host threads), then wal_verify_device_impl. Sets
// *needs_host_walk also when the device cannot hold the image.
int wal_verify_host_image_impl(const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk);

}  // namespace tkv
