// Probe (not product code): the speculative record_len walk of a WAL image with the image streamed
// through LDS by LDS-DMA (global_load_lds_dwordx4), one wave per 16 KiB region, one lane per 256-byte
// piece: the lane finds its piece's first plausible header in LDS (wal_scan_head's test) and walks the
// records that start in its piece from there, writing their offsets to per-piece slots. No CRC.
// Measures whether a walk fed by coalesced loads beats the product's per-lane HBM walk (wal_spec,
// tinykvpp_amd/csrc/tkv_wal_device.hip), whose header chain alone took 405 us on 1 GiB of 59-byte
// records in round 3.
//
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/walk_probe.hip -o tools/ab/libwalk_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr std::uint32_t kP = 256;              // piece bytes (one lane)
constexpr std::uint32_t kNP = 64;              // pieces per region (one wave)
constexpr std::uint32_t kReg = kP * kNP;       // 16 KiB
constexpr std::uint32_t kLdsBytes = kReg + 1024;  // region + one more 1 KiB DMA: headers past the region end
constexpr std::uint32_t kSlots = 12;           // record starts kept per piece
constexpr std::uint32_t kNone = 0xFFFFFFFFu;
constexpr std::uint64_t kMeta = 26;

__device__ __forceinline__ std::uint32_t le1_bytes4(std::uint32_t d) {
  const std::uint32_t x = d & 0xFEFEFEFEu;
  const std::uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu) & 0x80808080u;
  return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

typedef std::uint32_t __attribute__((address_space(3))) lds_u32;

__device__ __forceinline__ std::uint32_t ld_al(const std::uint8_t* lds, std::uint32_t b) {
  return *reinterpret_cast<const std::uint32_t*>(lds + b);
}
__device__ __forceinline__ std::uint32_t ld_un(const std::uint8_t* lds, std::uint32_t b) {
  const std::uint32_t a = b & ~3u;
  return __builtin_amdgcn_alignbyte(ld_al(lds, a + 4), ld_al(lds, a), b & 3u);
}

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void walk_lds(const std::uint8_t* w, std::uint64_t size, std::uint32_t nreg,
                                                      std::uint32_t* S, std::uint32_t* X, std::uint32_t* cnt,
                                                      std::uint32_t* slots) {
  __shared__ __attribute__((aligned(16))) std::uint8_t lds_all[WAVES * kLdsBytes];
  const std::uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  std::uint8_t* lds = lds_all + wid * kLdsBytes;
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(w);
  const std::uintptr_t glast = (w0 + size - 1u) & ~static_cast<std::uintptr_t>(15);
  const std::uint32_t gw = blockIdx.x * WAVES + wid, nw = gridDim.x * WAVES;
  for (std::uint32_t r = gw; r < nreg; r += nw) {
    const std::uint64_t rs = static_cast<std::uint64_t>(r) * kReg;
    const std::uintptr_t al = (w0 + rs) & ~static_cast<std::uintptr_t>(15);
    const std::uint32_t o = static_cast<std::uint32_t>(w0 + rs - al);
#pragma unroll
    for (std::uint32_t i = 0; i < kLdsBytes / 1024u; ++i) {
      std::uintptr_t g = al + 1024u * i + 16u * lane;
      g = g < glast ? g : glast;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(g),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<std::uintptr_t>(lds + 1024u * i)),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const std::uint64_t k = static_cast<std::uint64_t>(r) * kNP + lane;
    const std::uint64_t ps = k * kP;
    auto lb = [&](std::uint64_t x) { return static_cast<std::uint32_t>(x - rs) + o; };  // LDS byte of image offset x
    std::uint32_t start = kNone;
    if (ps < size) {
      if (k == 0) {
        start = 0;
      } else {
        const std::uint64_t pe = size < kMeta ? 0 : (ps + kP < size - kMeta + 1 ? ps + kP : size - kMeta + 1);
        // 16 positions per step: marks of bytes x+8 and x+17 being 0 or 1 (op and tombstone, wal.cpp:30-52)
        for (std::uint64_t x0 = ps; x0 < pe && start == kNone; x0 += 16) {
          const std::uint32_t b = lb(x0);
          std::uint32_t m8 = 0, m17 = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            m8 |= le1_bytes4(ld_un(lds, b + 8u + 4u * q)) << (4 * q);
            m17 |= le1_bytes4(ld_un(lds, b + 17u + 4u * q)) << (4 * q);
          }
          std::uint32_t cand = m8 & m17;
          const std::uint64_t lim = pe - x0;
          if (lim < 16) cand &= (1u << lim) - 1u;
          while (cand) {
            const int j = __builtin_ctz(cand);
            const std::uint64_t x = x0 + j;
            const std::uint32_t bx = lb(x);
            const std::uint64_t rl = ld_un(lds, bx), kl = ld_un(lds, bx + 18u), vl = ld_un(lds, bx + 22u);
            if (rl == 18u + kl + vl && rl + 8u <= size - x) {
              start = static_cast<std::uint32_t>(x);
              break;
            }
            cand &= cand - 1u;
          }
        }
      }
    }
    std::uint32_t n = 0, broke = 0, p32 = start;
    if (start != kNone) {
      std::uint64_t p = start;
      const std::uint64_t lim = ps + kP;
      while (p < lim) {
        if (size - p < kMeta) {
          broke = 1;
          break;
        }
        const std::uint64_t rl = ld_un(lds, lb(p));
        if (rl + 8u > size - p) {
          broke = 1;
          break;
        }
        if (n < kSlots) slots[k * kSlots + n] = static_cast<std::uint32_t>(p);
        ++n;
        p += 8u + rl;
      }
      p32 = static_cast<std::uint32_t>(p);
    }
    if (ps < size) {
      S[k] = start;
      X[k] = p32;
      cnt[k] = n | (broke << 31);
    }
  }
}

}  // namespace

extern "C" int walk_probe(const std::uint8_t* d_img, std::uint64_t size, std::uint32_t* S, std::uint32_t* X,
                          std::uint32_t* cnt, std::uint32_t* slots, int waves_per_wg, int wgs_per_cu, void* stream) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 2;
  const std::uint32_t nreg = static_cast<std::uint32_t>((size + kReg - 1) / kReg);
  auto st = static_cast<hipStream_t>(stream);
  const unsigned grid = static_cast<unsigned>(ncu * wgs_per_cu);
  if (waves_per_wg == 1) hipLaunchKernelGGL(walk_lds<1>, dim3(grid), dim3(64), 0, st, d_img, size, nreg, S, X, cnt, slots);
  else if (waves_per_wg == 2) hipLaunchKernelGGL(walk_lds<2>, dim3(grid), dim3(128), 0, st, d_img, size, nreg, S, X, cnt, slots);
  else hipLaunchKernelGGL(walk_lds<4>, dim3(grid), dim3(256), 0, st, d_img, size, nreg, S, X, cnt, slots);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" std::uint32_t walk_probe_slots() { return kSlots; }
extern "C" std::uint32_t walk_probe_piece() { return kP; }
