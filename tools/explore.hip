// Variant explorer (not product code): the production row-kernel body instantiated with other
// pipeline shapes, a memory-only mode (same loads, XOR instead of CRC) and a plain coalesced
// streaming read, so one process can A/B them on the same buffer (cdna_hip_programming.md §5.4
// rule 24). Built by tools/Makefile into tools/libexplore.so; driven by tools/explore.py.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "tkv_crc32_device.h"

using namespace tkv;

template <int D, int I, int M>
__global__ __launch_bounds__(kThreads) void k_rows(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_rows_body<true, true, D, I, M>(a, lds);
}

// Ideal streaming read: every lane reads consecutive 16-byte words, XOR-reduces, one store per wave.
__global__ __launch_bounds__(256) void k_stream(const uint4* p, std::uint64_t n16, std::uint32_t* out) {
  std::uint32_t x = 0;
  for (std::uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
    const uint4 v = p[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;  // keep the loads alive
}

namespace {
DeviceTables* g_tabs = nullptr;
std::uint8_t* g_dummy = nullptr;
Seam* g_seams = nullptr;
int g_ncu = 0;

struct V {
  const char* name;
  void (*launch)(RowsArgs, hipStream_t);
};

template <int D, int I, int M>
void L(RowsArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_rows<D, I, M>), dim3(g_ncu), dim3(kThreads), 0, s, a);
}

const V kVariants[] = {
    {"crc D2 I1", L<2, 1, 0>}, {"crc D3 I1", L<3, 1, 0>}, {"crc D4 I1", L<4, 1, 0>},
    {"crc D4 I2", L<4, 2, 0>}, {"crc D6 I2", L<6, 2, 0>}, {"crc D6 I3", L<6, 3, 0>},
    {"mem D2 I1", L<2, 1, 1>}, {"mem D4 I1", L<4, 1, 1>}, {"mem D4 I2", L<4, 2, 1>},
    {"mem D8 I1", L<8, 1, 1>},
};
constexpr int kNV = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

namespace tkv {
void build_tables(DeviceTables* t);
std::uint32_t x8nmodp(std::uint64_t nbytes);
}  // namespace tkv

extern "C" int explore_count() { return kNV + 1; }
extern "C" const char* explore_name(int v) { return v < kNV ? kVariants[v].name : "stream read (ideal)"; }

extern "C" int explore_run(int v, const std::uint8_t* base, std::uint64_t n, std::uint32_t len, std::uint32_t* out,
                           void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!g_tabs) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    g_ncu = prop.multiProcessorCount;
    auto* h = new DeviceTables;
    build_tables(h);
    if (hipMalloc(&g_tabs, sizeof(DeviceTables)) != hipSuccess) return 1;
    hipMemcpy(g_tabs, h, sizeof(DeviceTables), hipMemcpyHostToDevice);
    delete h;
    hipMalloc(&g_dummy, 256);
    hipMemset(g_dummy, 0, 256);
    hipMalloc(&g_seams, sizeof(Seam) * 2 * g_ncu * kWavesPerWG);
  }
  if (v == kNV) {
    hipLaunchKernelGGL(k_stream, dim3(g_ncu * 8), dim3(256), 0, st, reinterpret_cast<const uint4*>(base),
                       n * len / 16, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  RowsArgs a{};
  a.base = base;
  a.stride = len;
  a.len = len;
  a.head_z = x8nmodp(head_len(len));
  a.init_default = 0xFFFFFFFFu;
  a.out_xor = 0xFFFFFFFFu;
  a.out = out;
  a.seams = g_seams;
  a.tabs = g_tabs;
  a.dummy = g_dummy;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.total_rows = static_cast<std::uint32_t>(n * rows_for_len(len));
  a.nwaves = g_ncu * kWavesPerWG;
  a.snap_blocks = 1;
  kVariants[v].launch(a, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
