// Engine entry points shared by the C ABI files (tkv_crc32_host.cpp, tkv_formats.cpp). Each takes
// the checksum family (Algo) and works on the calling thread's current device; arguments and
// return codes are those of the matching tkv_crc32_* functions in include/tkv_crc32.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "tkv_crc32_internal.h"

namespace tkv {

int update_impl(int algo, std::uint32_t raw_state, const void* data, std::size_t len, std::uint32_t* out_raw);
int update_device_impl(int algo, std::uint32_t raw_state, const void* d_data, std::size_t len,
                       std::uint32_t* d_out_raw, void* stream);
int batch_device_impl(int algo, const std::uint8_t* d_base, const std::uint64_t* d_offsets,
                      const std::uint32_t* d_lengths, const std::uint32_t* d_init_raw, std::uint32_t* d_out_final,
                      std::uint64_t n, void* stream);
int batch_uniform_impl(int algo, const std::uint8_t* d_base, std::uint64_t stride, std::uint64_t len,
                       const std::uint32_t* d_init_raw, std::uint32_t* d_out_final, std::uint64_t n, void* stream);
int batch_host_impl(int algo, const std::uint8_t* h_base, const std::uint64_t* h_offsets,
                    const std::uint32_t* h_lengths, const std::uint32_t* h_init_raw, std::uint32_t* h_out_final,
                    std::uint64_t n);
int batch_host_multi_impl(int algo, const int* devices, int ndev, const std::uint8_t* h_base,
                          const std::uint64_t* h_offsets, const std::uint32_t* h_lengths,
                          const std::uint32_t* h_init_raw, std::uint32_t* h_out_final, std::uint64_t n);

// Record `msg` as this thread's tkv_last_error() text; returns `code`.
int set_error(int code, const char* msg);
// Constant tables of `algo` on the current device (creates the device context); nullptr on error.
const DeviceTables* device_tables(int algo);

// tkv_crc32_kernels.hip: SSTable stamp fix-up (see tkv_sst_block_crcs_device).
hipError_t launch_sst_fix(std::uint8_t* file, const std::uint64_t* offsets, const std::uint32_t* sizes,
                          std::uint32_t* out, std::uint64_t n, int store, const DeviceTables* tabs, hipStream_t st);

}  // namespace tkv
