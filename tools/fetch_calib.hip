// FETCH_SIZE calibration for the byte budget of the packed kernel (not product code).
// MI355X_MICROARCH.md calibrates FETCH_SIZE x 2 only for wide coalesced streaming reads; this probe
// reads the same 4 GiB in three load patterns with no CRC work, so a --pmc FETCH_SIZE pass over it
// gives the counter's reading of each pattern against a known byte count:
//   coal   - grid-stride, 16 B per lane, consecutive lanes on consecutive 16-byte pieces;
//   seg64  - the packed kernel's pattern: a wave owns a contiguous range of 4 KiB rows, lane l reads
//            bytes [64 l, 64 l + 64) of a row as four 16-byte loads, 4 rows in flight;
//   seg64c - seg64 with the product's pipeline tail: the loads past a wave's last row are clamped
//            to that row (re-read) instead of skipped.
// Each kernel runs 3 times; HIP events give its rate.
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__global__ __launch_bounds__(1024) void coal(const uint4* p, std::uint64_t n16, std::uint32_t* out) {
  std::uint32_t acc = 0;
  const std::uint64_t stride = static_cast<std::uint64_t>(gridDim.x) * blockDim.x;
  for (std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x; i < n16; i += stride) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // never true for the fill below; keeps the loads
}

template <bool CLAMP>
__global__ __launch_bounds__(1024) void seg64(const uint4* p, std::uint64_t nrows, std::uint32_t* out) {
  const std::uint64_t W = static_cast<std::uint64_t>(gridDim.x) * (blockDim.x / 64);
  const std::uint64_t w = blockIdx.x * static_cast<std::uint64_t>(blockDim.x / 64) + (threadIdx.x >> 6);
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint64_t r0 = w * nrows / W, r1 = (w + 1) * nrows / W;
  std::uint32_t acc = 0;
  constexpr int D = 4;
  for (std::uint64_t r = r0; r < r1; r += D) {
    uint4 v[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      std::uint64_t row = r + d;
      if (!CLAMP && row >= r1) continue;
      row = row < r1 ? row : r1 - 1;
      const uint4* q = p + row * 256 + lane * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[d][k] = q[k];
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (!CLAMP && r + d >= r1) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ void fill(std::uint32_t* p, std::uint64_t n) {
  for (std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<std::uint64_t>(gridDim.x) * blockDim.x)
    p[i] = static_cast<std::uint32_t>(i * 2654435761u) | 1u;
}

int main() {
  const std::uint64_t bytes = 4ull << 30;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  void* d = nullptr;
  std::uint32_t* out = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, static_cast<std::uint32_t*>(d), bytes / 4);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint4* p = static_cast<const uint4*>(d);
  for (int kind = 0; kind < 3; ++kind) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, 0));
      if (kind == 0)
        hipLaunchKernelGGL(coal, dim3(ncu * 8), dim3(1024), 0, 0, p, bytes / 16, out);
      else if (kind == 1)
        hipLaunchKernelGGL(seg64<false>, dim3(ncu), dim3(1024), 0, 0, p, bytes / 4096, out);
      else
        hipLaunchKernelGGL(seg64<true>, dim3(ncu), dim3(1024), 0, 0, p, bytes / 4096, out);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("{\"pattern\": \"%s\", \"rep\": %d, \"bytes\": %llu, \"ms\": %.4f, \"GBps\": %.1f}\n",
                  kind == 0 ? "coal" : kind == 1 ? "seg64" : "seg64c", rep, static_cast<unsigned long long>(bytes), ms,
                  bytes / (ms * 1e6));
    }
  }
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
