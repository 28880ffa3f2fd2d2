// Device-side WAL recovery verify (tkv_wal_device.hip), used by tkv_wal_verify and
// tkv_wal_verify_device (tkv_formats.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkv {

// Verify the WAL image [d_wal, d_wal + size) in device memory on `st` (synchronous): one sweep that
// walks the record chain and folds every payload of at most 64 KiB, device fix-up rounds where a
// chunk's speculative entry was wrong, one CRC batch for longer payloads, the first bad record. Same
// results as tkv_wal_verify. *needs_host_walk is set (and nothing else is decided) when the fix-up
// rounds have not settled the chain within their budget (kRoundBudget); the caller then runs the
// exact host walk.
int wal_verify_device_impl(const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                           std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk);

// Host image: copied into a device buffer kept per device (pinned sources in one copy, pageable ones
// through pinned staging slabs filled by host threads), then wal_verify_device_impl. Sets
// *needs_host_walk also when the device cannot hold the image.
int wal_verify_host_image_impl(const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk);

}  // namespace tkv
