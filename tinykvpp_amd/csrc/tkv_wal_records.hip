// Record-list check of a WAL image in HBM (tkv_wal_check_records_device, include/tkv_crc32.h):
// wal_entry::decode's per-record checks (/root/reference/src/engine/wal.cpp:63-127) for records whose
// start offsets are already known - the record list a walk produced, or the offsets a group-commit
// writer kept - with no lengths array and no prepass: each lane reads its record's header from the
// same 16-byte granules that hold its payload.
//
// One lane folds one record. The lane loads the NG aligned granules that cover the record's first
// 16 NG - 15 bytes at any alignment (the 8-byte header, key/value lengths at bytes 18-25, and the
// first payload bytes), realigns them in registers (two bitwise selects by the start's dword offset in
// its granule, then v_alignbyte by its byte offset, as the lane kernels do), and folds the payload
// from 0xFFFFFFFF with slicing-by-4 lookups into the LDS tables and Sarwate steps for the last 1-3
// bytes (crc32.cpp:9-16). A payload longer than the window continues 64 bytes at a time from fresh
// granules, the register carried over (rare for WAL records; every length is exact). Loads are clamped
// to the image's last granule, so no load leaves the image's pages whatever the offsets say.
//
// Per record (wal.cpp order): at least kMetadataSize = 26 bytes left (wal.cpp:68), record_len + 8
// within the image (:80), CRC-32 of the record_len payload bytes equal to the stored CRC (:89-96), key
// and value inside the payload (:118-121). A record failing any of them is corrupted; the first such
// record index is an atomic minimum.
//
// Pipeline (lane_phase's): offsets are fetched four steps ahead of their granules, granules two steps
// ahead of the fold, and nothing loaded is touched before use. Waves own contiguous ranges of records,
// 64 per step, with the packed kernels' issue priority from the work left.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "tkv_crc32.h"
#include "tkv_crc32_device.h"
#include "tkv_engine.h"
#include "tkv_wal_device.h"

namespace tkv {
namespace {

constexpr std::uint32_t kRecMeta = 26;  // wal.hpp kMetadataSize: 8-byte header + op, seq, tombstone, key/value lengths
constexpr unsigned kRecThreads = 1024;  // one workgroup per CU (128 KiB of LDS tables)

struct RecArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  const std::uint32_t* off;
  std::uint64_t n;
  std::uint32_t* crc;                  // nullable: computed CRC per record (0 when its length is bad)
  unsigned long long* first_bad;       // atomic minimum of bad record indices (preset to n)
  std::uint32_t nwaves;
  std::uint32_t defer;                 // payloads longer than this are not folded here (the verify pass
                                       // checks them through the irregular batch path); 0xFFFFFFFF: none
};

__global__ void rec_init(unsigned long long* first_bad, std::uint64_t n) { *first_bad = n; }

// The 4 NG little-endian dwords from byte p of the granules g (o = p & 15): d[k] = bytes [p + 4k, +4).
template <int NG>
__device__ __forceinline__ void rec_dwords(const uint4 (&g)[NG], std::uint32_t o, std::uint32_t (&d)[4 * NG - 4]) {
  std::uint32_t raw[4 * NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    raw[4 * i + 0] = g[i].x;
    raw[4 * i + 1] = g[i].y;
    raw[4 * i + 2] = g[i].z;
    raw[4 * i + 3] = g[i].w;
  }
  const std::uint32_t m8 = 0u - ((o >> 3) & 1u), m4 = 0u - ((o >> 2) & 1u);
#pragma unroll
  for (int i = 0; i < 4 * NG - 2; ++i) raw[i] ^= (raw[i] ^ raw[i + 2]) & m8;
#pragma unroll
  for (int i = 0; i < 4 * NG - 3; ++i) raw[i] ^= (raw[i] ^ raw[i + 1]) & m4;
#pragma unroll
  for (int k = 0; k < 4 * NG - 4; ++k) d[k] = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], o & 3u);
}

// Folds the payload bytes [0, n) of d (n <= 4 * ND) into register c (whole dwords, then Sarwate steps).
template <int ND>
__device__ __forceinline__ std::uint32_t rec_fold(const std::uint32_t* lds, const dev::LaneConst& kc, const std::uint32_t* d,
                                                  std::uint32_t n, std::uint32_t c) {
  dev::Reg r{c, 0};
  const std::uint32_t nf = n >> 2, tb = n & 3u;
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    if (static_cast<std::uint32_t>(k) < nf) dev::slice4(lds, r, d[k], kc);
    else if (static_cast<std::uint32_t>(k) == nf && tb != 0u) r = dev::Reg{dev::sarwate_bytes(lds, kc, r.value(), d[k], tb), 0};
  }
  if (nf == static_cast<std::uint32_t>(ND) && tb != 0u) r = dev::Reg{dev::sarwate_bytes(lds, kc, r.value(), d[ND], tb), 0};
  return r.value();
}

// NG granules per record window; AHEAD steps of granules in flight (2, or 1 for the wide window,
// whose three slots would spill at 16 waves per CU).
template <int NG, int AHEAD>
__global__ __launch_bounds__(kRecThreads) void wal_rec_lanes(RecArgs a, const DeviceTables* tabs) {
  constexpr int ND = 4 * NG - 4;      // realigned dwords of the window
  constexpr int NPAY = ND - 3;        // whole payload dwords folded from the window (payload at dword 2; one spare for the tail)
  constexpr int RING = 4;             // offsets are fetched RING steps ahead of their granules
  constexpr int DRING = AHEAD == 1 ? 2 : 4;
  static_assert(AHEAD == 1 || AHEAD == 2, "granules one or two steps ahead");
  __shared__ std::uint32_t lds[kLdsSliceWords];
  dev::fill_lds_slicing(tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const dev::LaneConst kc = dev::lane_const(lane);
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, n = a.n;
  const std::uint64_t TS = (n + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  if (ns == 0) return;
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(a.w);
  const std::uintptr_t glast = (w0 + a.size - 1u) & ~static_cast<std::uintptr_t>(15);  // the image's last granule
  auto gran = [&](std::uintptr_t p) { return dev::gload16(p < glast ? p : glast); };

  std::uint32_t d_off[RING];
  auto fetch = [&](std::uint32_t j, int slot) {
    const std::uint64_t b = (s0 + j) * 64u + lane;
    d_off[slot] = a.off[b < n ? b : n - 1u];  // clamped: every load stays inside the array
  };
  uint4 q[DRING][NG];
  std::uint32_t m_off[DRING];
  auto issue = [&](int slot, int dslot) {
    const std::uint32_t off = d_off[slot];
    const std::uintptr_t al = (w0 + off) & ~static_cast<std::uintptr_t>(15);
#pragma unroll
    for (int i = 0; i < NG; ++i) q[dslot][i] = gran(al + 16u * i);
    m_off[dslot] = off;
  };
  auto fold = [&](int slot, std::uint32_t j) {
    const std::uint64_t b = (s0 + j) * 64u + lane;
    const bool live = b < n;
    const std::uint32_t off = m_off[slot];
    const std::uintptr_t p = w0 + off;
    std::uint32_t d[ND];
    rec_dwords<NG>(q[slot], static_cast<std::uint32_t>(p & 15u), d);
    const std::uint32_t rlen = d[0], stored = d[1];
    const std::uint32_t klen = __builtin_amdgcn_alignbyte(d[5], d[4], 2u);
    const std::uint32_t vlen = __builtin_amdgcn_alignbyte(d[6], d[5], 2u);
    const std::uint64_t left = off < a.size ? a.size - off : 0u;
    const bool len_ok = left >= kRecMeta && static_cast<std::uint64_t>(rlen) + 8u <= left;  // wal.cpp:68, :80
    const bool deferred = len_ok && rlen > a.defer;
    const std::uint32_t L = live && len_ok && !deferred ? rlen : 0u;
    std::uint32_t c = rec_fold<NPAY>(lds, kc, d + 2, L < 4u * NPAY ? L : 4u * NPAY, 0xFFFFFFFFu);
    // payloads longer than the window: 64 bytes at a time from fresh granules, the register carried
    for (std::uint32_t done = 4u * NPAY; __ballot(L > done) != 0; done += 64u) {
      const std::uint32_t m = L > done ? std::min(L - done, 64u) : 0u;
      const std::uintptr_t ps = p + 8u + done;
      const std::uintptr_t al = ps & ~static_cast<std::uintptr_t>(15);
      uint4 g[dev::kLaneGran];
#pragma unroll
      for (int i = 0; i < dev::kLaneGran; ++i) g[i] = gran(m ? al + 16u * i : glast);
      std::uint32_t e[16];
      dev::lane_dwords<1>(g, static_cast<std::uint32_t>(ps & 15u), e);
      std::uint32_t e17[17];
#pragma unroll
      for (int k = 0; k < 16; ++k) e17[k] = e[k];
      e17[16] = 0u;
      c = rec_fold<16>(lds, kc, e17, m, c);
    }
    const std::uint32_t crc = c ^ 0xFFFFFFFFu;
    const bool kv_ok = static_cast<std::uint64_t>(klen) + vlen + (kRecMeta - 8u) <= rlen;  // wal.cpp:118-121
    if (live && a.crc) a.crc[b] = len_ok ? crc : 0u;
    if (live && (!len_ok || (crc != stored && !deferred) || !kv_ok))
      atomicMin(a.first_bad, static_cast<unsigned long long>(b));
  };

#pragma unroll
  for (int k = 0; k < RING; ++k) fetch(k, k);
#pragma unroll
  for (int k = 0; k < AHEAD; ++k) {
    issue(k, k % DRING);
    fetch(k + RING, k);
  }
  for (std::uint32_t t = 0; t < ns; t += RING) {
    dev::set_prio_from_left<3>(ns - t, ns);
#pragma unroll
    for (int k = 0; k < RING; ++k) {
      const int ahead = (k + AHEAD) % RING;  // step t+k+AHEAD: its offset arrived RING steps ago
      issue(ahead, (k + AHEAD) % DRING);
      fetch(t + k + AHEAD + RING, ahead);
      if (t + k < ns) fold(k % DRING, t + k);
    }
  }
}

int cu_count() {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = n;
  }
  return cached[dev];
}

// The record check over n records (first_bad preset to n by the caller's stream order).
void launch_records(RecArgs a, std::uint32_t max_payload, int ncu, const DeviceTables* tabs, hipStream_t st) {
  const std::uint64_t steps = (a.n + 63) / 64;
  const std::uint64_t grid =
      std::max<std::uint64_t>(1, std::min<std::uint64_t>(static_cast<std::uint64_t>(ncu), (steps + 15) / 16));
  a.nwaves = static_cast<std::uint32_t>(grid * 16);
  // window: NG granules hold the header, the key/value lengths and a payload of up to 16 NG - 26 bytes
  // at any alignment (36-byte payloads: 4 granules; 64: 6; 100: 8); longer ones continue 64 bytes at
  // a time. Wider windows keep one step of granules in flight instead of two (registers).
  const std::uint32_t ng =
      std::min<std::uint32_t>(8u, std::max<std::uint32_t>(4u, (std::min<std::uint32_t>(max_payload, 1024u) + 26u + 15u) / 16u));
  const dim3 g(static_cast<unsigned>(grid)), b(kRecThreads);
  switch (ng) {
    case 4: hipLaunchKernelGGL((wal_rec_lanes<4, 2>), g, b, 0, st, a, tabs); break;
    case 5: hipLaunchKernelGGL((wal_rec_lanes<5, 2>), g, b, 0, st, a, tabs); break;
    case 6: hipLaunchKernelGGL((wal_rec_lanes<6, 2>), g, b, 0, st, a, tabs); break;
    case 7: hipLaunchKernelGGL((wal_rec_lanes<7, 1>), g, b, 0, st, a, tabs); break;
    default: hipLaunchKernelGGL((wal_rec_lanes<8, 1>), g, b, 0, st, a, tabs); break;
  }
}

// ---- the verify pass with the image walked through LDS (wal_pass_lds) -------------------------------
// 1. wal_walk_lds: one wave per 16 KiB region, copied into LDS by LDS-DMA (17 global_load_lds_dwordx4,
//    the last KiB for headers past the region end), one lane per 256-byte piece. The lane searches its
//    piece for the first plausible header (wal_scan_head's test: op and tombstone bytes 0 or 1,
//    record_len = 18 + klen + vlen, fitting the image; piece 0 starts at 0) and walks the records that
//    start in the piece (wal.cpp:63-87: at least 26 bytes left, record_len + 8 within the image),
//    keeping each start as a byte offset into the piece (12 slots: records are at least 26 bytes; a
//    piece with more starts overflows and fails the stitch). All reads come from LDS, so the walk's
//    dependent reads cost LDS latency, and HBM sees only whole-region DMA reads.
// 2. wal_lds_stitch: the fast stitch of the round-3 pass in O(pieces): every piece with a start must
//    leave exactly at the next piece with a start (no start in between, at most kStitchSpan pieces
//    on), and the only piece whose chain ends (past the image or at a header that breaks) is the last
//    piece with a start. Piece 0 is entered at 0, so by induction every start is on the true chain.
// 3. record counts scanned (hipcub), one host sync for the verdict and the totals; when the stitch
//    fails, nothing is decided and the caller runs the round-3 pass.
// 4. wal_lds_compact: the records in chain order into one dense list of u32 offsets; payloads over
//    kLdsDefer bytes also into a list for the irregular batch path.
// 5. wal_rec_lanes over the list (tkv_wal_check_records_device's kernel), the deferred payloads through
//    batch_device_impl and wal_lds_big: the first bad record index, its start, one more host sync.
constexpr std::uint32_t kLdsPiece = 256;
constexpr std::uint32_t kLdsRegion = kLdsPiece * 64;
constexpr std::uint32_t kLdsBytes = kLdsRegion + 1024;
constexpr std::uint32_t kLdsSlots = 12;
constexpr std::uint32_t kLdsStitchSpan = 4096;      // pieces (1 MiB): a longer record fails the stitch
constexpr std::uint32_t kLdsDefer = 1024;           // longer payloads are checked through the irregular batch path
constexpr std::uint16_t kNoStart = 0xFFFFu;
constexpr std::uint8_t kBroke = 1, kOverflow = 2;

struct LdsArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  std::uint32_t K;         // pieces
  std::uint16_t* S;        // first plausible header, byte offset in the piece (kNoStart: none)
  std::uint32_t* X;        // exit of the piece's walk (or the start of the header that broke it)
  std::uint32_t* cnt;      // records walked from S
  std::uint32_t* base;     // exclusive scan of cnt
  std::uint8_t* flags;     // kBroke, kOverflow
  std::uint16_t* bigmask;  // slots whose payload is longer than kLdsDefer
  std::uint8_t* slots;     // kLdsSlots record starts per piece, byte offsets in the piece
  std::uint32_t* rec;      // dense record list (step 4)
  std::uint64_t* big_off;  // deferred payloads: offset, length, record index, stored CRC, computed CRC
  std::uint32_t* big_len;
  std::uint64_t* big_idx;
  std::uint32_t* big_crc;
  std::uint32_t* big_got;
  unsigned long long* res;  // [0] last piece with a start, [1] longest payload not deferred, [2] deferred
                            // payloads, [3] stitch failures, [4] first bad record, [5] deferred so far
};

__device__ __forceinline__ std::uint32_t le1_bytes4(std::uint32_t d) {  // bit i: byte i of d is 0 or 1
  const std::uint32_t x = d & 0xFEFEFEFEu;
  const std::uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu) & 0x80808080u;
  return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ std::uint32_t lds_al(const std::uint8_t* lds, std::uint32_t b) {
  return *reinterpret_cast<const std::uint32_t*>(lds + b);
}
__device__ __forceinline__ std::uint32_t lds_un(const std::uint8_t* lds, std::uint32_t b) {
  const std::uint32_t q = b & ~3u;
  return __builtin_amdgcn_alignbyte(lds_al(lds, q + 4), lds_al(lds, q), b & 3u);
}

__global__ __launch_bounds__(64) void wal_walk_lds(LdsArgs a, std::uint32_t nreg) {
  __shared__ __attribute__((aligned(16))) std::uint8_t lds[kLdsBytes];
  const std::uint32_t lane = threadIdx.x;
  const std::uint64_t size = a.size;
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(a.w);
  const std::uintptr_t glast = (w0 + size - 1u) & ~static_cast<std::uintptr_t>(15);
  std::uint32_t my_last = 0, my_max = 0, my_big = 0;
  bool any_start = false;
  for (std::uint32_t r = blockIdx.x; r < nreg; r += gridDim.x) {
    const std::uint64_t rs = static_cast<std::uint64_t>(r) * kLdsRegion;
    const std::uintptr_t al = (w0 + rs) & ~static_cast<std::uintptr_t>(15);
    const std::uint32_t o = static_cast<std::uint32_t>(w0 + rs - al);
#pragma unroll
    for (std::uint32_t i = 0; i < kLdsBytes / 1024u; ++i) {
      std::uintptr_t g = al + 1024u * i + 16u * lane;
      g = g < glast ? g : glast;  // inside the image's pages; bytes past its end are never trusted
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(g),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<std::uintptr_t>(lds + 1024u * i)),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const std::uint64_t k = static_cast<std::uint64_t>(r) * 64u + lane;
    const std::uint64_t ps = k * kLdsPiece;
    auto lb = [&](std::uint64_t x) { return static_cast<std::uint32_t>(x - rs) + o; };
    std::uint32_t start = kNoStart;
    if (ps < size) {
      if (k == 0) {
        start = 0;
      } else if (size >= kRecMeta) {
        const std::uint64_t pe = ps + kLdsPiece < size - kRecMeta + 1 ? ps + kLdsPiece : size - kRecMeta + 1;
        for (std::uint64_t x0 = ps; x0 < pe && start == kNoStart; x0 += 16) {  // 16 positions per step
          const std::uint32_t b = lb(x0);
          std::uint32_t m8 = 0, m17 = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            m8 |= le1_bytes4(lds_un(lds, b + 8u + 4u * q)) << (4 * q);
            m17 |= le1_bytes4(lds_un(lds, b + 17u + 4u * q)) << (4 * q);
          }
          std::uint32_t cand = m8 & m17;
          if (pe - x0 < 16) cand &= (1u << (pe - x0)) - 1u;
          while (cand) {
            const int j = __builtin_ctz(cand);
            const std::uint64_t x = x0 + static_cast<std::uint64_t>(j);
            const std::uint32_t bx = lb(x);
            const std::uint64_t rl = lds_un(lds, bx), kl = lds_un(lds, bx + 18u), vl = lds_un(lds, bx + 22u);
            if (rl == 18u + kl + vl && rl + 8u <= size - x) {
              start = static_cast<std::uint32_t>(x - ps);
              break;
            }
            cand &= cand - 1u;
          }
        }
      }
    }
    if (ps < size) {
      std::uint32_t n = 0;
      std::uint16_t big = 0;
      std::uint8_t fl = 0;
      std::uint64_t p = ps + start;
      if (start != kNoStart) {
        any_start = true;
        my_last = static_cast<std::uint32_t>(k);
        const std::uint64_t lim = ps + kLdsPiece < size ? ps + kLdsPiece : size;  // a chain that ends at
        while (p < lim) {                                                          // the image's end is clean
          if (size - p < kRecMeta) {
            fl |= kBroke;
            break;
          }
          const std::uint32_t rl = lds_un(lds, lb(p));
          if (static_cast<std::uint64_t>(rl) + 8u > size - p) {
            fl |= kBroke;
            break;
          }
          if (n == kLdsSlots) {
            fl |= kOverflow;
            break;
          }
          a.slots[k * kLdsSlots + n] = static_cast<std::uint8_t>(p - ps);
          if (rl > kLdsDefer) {
            big |= static_cast<std::uint16_t>(1u << n);
            ++my_big;
          } else {
            my_max = rl > my_max ? rl : my_max;
          }
          ++n;
          p += 8u + rl;
        }
      }
      a.S[k] = static_cast<std::uint16_t>(start);
      a.X[k] = static_cast<std::uint32_t>(p);
      a.cnt[k] = n;
      a.flags[k] = fl;
      a.bigmask[k] = big;
    }
  }
  // one atomic per wave for each result word
  std::uint32_t last = any_start ? my_last + 1u : 0u, mx = my_max, bg = my_big;
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) {
    last = std::max<std::uint32_t>(last, static_cast<std::uint32_t>(__shfl_xor(static_cast<int>(last), m, 64)));
    mx = std::max<std::uint32_t>(mx, static_cast<std::uint32_t>(__shfl_xor(static_cast<int>(mx), m, 64)));
    bg += static_cast<std::uint32_t>(__shfl_xor(static_cast<int>(bg), m, 64));
  }
  if (lane == 0) {
    if (last) atomicMax(&a.res[0], static_cast<unsigned long long>(last - 1u));
    atomicMax(&a.res[1], static_cast<unsigned long long>(mx));
    if (bg) atomicAdd(&a.res[2], static_cast<unsigned long long>(bg));
  }
}

__global__ void wal_lds_stitch(LdsArgs a) {
  const std::uint64_t k = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (k >= a.K || a.S[k] == kNoStart) return;
  const std::uint64_t X = a.X[k];
  const std::uint8_t fl = a.flags[k];
  bool ok = (fl & kOverflow) == 0;
  if ((fl & kBroke) || X >= a.size) {
    ok = ok && k == a.res[0];  // the chain ends here: no later piece may hold a start
  } else {
    const std::uint64_t q = X / kLdsPiece;
    ok = ok && q > k && q - k <= kLdsStitchSpan && a.S[q] != kNoStart && q * kLdsPiece + a.S[q] == X;
    for (std::uint64_t r = k + 1; ok && r < q; ++r) ok = a.S[r] == kNoStart;
  }
  if (!ok) atomicOr(&a.res[3], 1ull);
}

// Result words into the host's pinned block: res[0..3], the record total, the last start piece's exit
// and flags.
__global__ void wal_lds_publish(LdsArgs a, std::uint64_t* h) {
  const unsigned i = threadIdx.x;
  if (i < 4) h[i] = a.res[i];
  if (i == 4) h[4] = static_cast<std::uint64_t>(a.base[a.K - 1]) + a.cnt[a.K - 1];
  if (i == 5) h[5] = a.X[a.res[0] < a.K ? a.res[0] : 0];
  if (i == 6) h[6] = a.flags[a.res[0] < a.K ? a.res[0] : 0];
}

__global__ void wal_lds_compact(LdsArgs a) {
  const std::uint64_t k = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (k >= a.K) return;
  const std::uint32_t n = a.cnt[k];
  if (n == 0) return;
  const std::uint32_t b = a.base[k];
  const std::uint16_t big = a.bigmask[k];
  for (std::uint32_t i = 0; i < n; ++i) {
    const std::uint32_t off = static_cast<std::uint32_t>(k * kLdsPiece) + a.slots[k * kLdsSlots + i];
    a.rec[b + i] = off;
    if (big & (1u << i)) {
      const std::uint64_t j = atomicAdd(&a.res[5], 1ull);
      const std::uint32_t* h = reinterpret_cast<const std::uint32_t*>(a.w + off);  // (only read when big)
      std::uint32_t rl, st;
      std::memcpy(&rl, a.w + off, 4);
      std::memcpy(&st, a.w + off + 4, 4);
      (void)h;
      a.big_off[j] = static_cast<std::uint64_t>(off) + 8u;
      a.big_len[j] = rl;
      a.big_idx[j] = static_cast<std::uint64_t>(b) + i;
      a.big_crc[j] = st;
    }
  }
}

__global__ void wal_lds_big(LdsArgs a, std::uint64_t nbig) {
  const std::uint64_t j = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (j < nbig && a.big_got[j] != a.big_crc[j]) atomicMin(&a.res[4], a.big_idx[j]);
}

__global__ void wal_lds_final(LdsArgs a, std::uint64_t n, std::uint64_t* h) {
  const std::uint64_t f = a.res[4];
  h[7] = f;
  h[8] = f < n ? a.rec[f] : 0u;
}

struct LdsScratch {
  std::mutex mu;
  std::uint64_t cap_pieces = 0, cap_rec = 0, cap_big = 0;
  void* pieces = nullptr;
  std::uint32_t* rec = nullptr;
  void* bigs = nullptr;
  void* cub = nullptr;
  std::size_t cub_bytes = 0;
  unsigned long long* res = nullptr;
  std::uint64_t* h_res = nullptr;
  std::uint64_t* d_hres = nullptr;
};
std::mutex g_lds_mu;
LdsScratch* g_lds[64] = {};

#define LDS_HIP(call)                                                            \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e_)); \
  } while (0)

template <typename T>
int grow(T** p, std::uint64_t* cap, std::uint64_t want, std::uint64_t unit) {
  if (want <= *cap) return TKV_OK;
  const std::uint64_t c = std::max<std::uint64_t>(want, *cap * 2);
  LDS_HIP(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  LDS_HIP(hipMalloc(reinterpret_cast<void**>(p), c * unit));
  *cap = c;
  return TKV_OK;
}

}  // namespace

int g_wal_lds_walk = 1;

int wal_pass_lds(const std::uint8_t* w, std::uint64_t size, hipStream_t st, PassResult* r, bool* used) {
  *used = false;
  if (size == 0 || size > 0xFFFFFFFFull) return TKV_OK;
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  const int ncu = cu_count();
  if (ncu <= 0) return set_error(TKV_IO_ERROR, "no device");
  int dev = 0;
  LDS_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return set_error(TKV_INVALID_ARGUMENT, "device index out of range");
  LdsScratch* sp;
  {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    if (!g_lds[dev]) g_lds[dev] = new LdsScratch();
    sp = g_lds[dev];
  }
  LdsScratch& s = *sp;
  std::lock_guard<std::mutex> lk(s.mu);
  if (!s.res) {
    LDS_HIP(hipMalloc(reinterpret_cast<void**>(&s.res), 8 * sizeof(unsigned long long)));
    LDS_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_res), 16 * sizeof(std::uint64_t), hipHostMallocDefault));
    LDS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.d_hres), s.h_res, 0));
  }
  const std::uint32_t K = static_cast<std::uint32_t>((size + kLdsPiece - 1) / kLdsPiece);
  const std::uint32_t nreg = (K + 63u) / 64u;
  // per piece: S u16, bigmask u16, X u32, cnt u32, base u32, flags u8, slots 12 x u8 (+ padding)
  constexpr std::uint64_t kPer = 2 + 2 + 4 + 4 + 4 + 1 + kLdsSlots;
  std::uint8_t* pc = static_cast<std::uint8_t*>(s.pieces);
  if (int rc = grow(&pc, &s.cap_pieces, static_cast<std::uint64_t>(K) + 64, kPer)) return rc;
  s.pieces = pc;
  const std::uint64_t C = s.cap_pieces;
  LdsArgs a{};
  a.w = w;
  a.size = size;
  a.K = K;
  a.X = reinterpret_cast<std::uint32_t*>(pc);
  a.cnt = a.X + C;
  a.base = a.cnt + C;
  a.S = reinterpret_cast<std::uint16_t*>(a.base + C);
  a.bigmask = a.S + C;
  a.flags = reinterpret_cast<std::uint8_t*>(a.bigmask + C);
  a.slots = a.flags + C;
  a.res = s.res;
  std::size_t need = 0;
  LDS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need, a.cnt, a.base, K, st));
  if (need > s.cub_bytes) {
    LDS_HIP(hipStreamSynchronize(st));
    LDS_HIP(hipFree(s.cub));
    s.cub = nullptr;
    s.cub_bytes = 0;
    LDS_HIP(hipMalloc(&s.cub, need));
    s.cub_bytes = need;
  }
  // 1-3: walk, stitch, counts, one sync
  LDS_HIP(hipMemsetAsync(s.res, 0, 4 * sizeof(unsigned long long), st));
  LDS_HIP(hipMemsetAsync(s.res + 4, 0xFF, sizeof(unsigned long long), st));
  LDS_HIP(hipMemsetAsync(s.res + 5, 0, sizeof(unsigned long long), st));
  const unsigned grid = static_cast<unsigned>(std::min<std::uint64_t>(nreg, static_cast<std::uint64_t>(ncu) * 9u));
  hipLaunchKernelGGL(wal_walk_lds, dim3(grid), dim3(64), 0, st, a, nreg);
  hipLaunchKernelGGL(wal_lds_stitch, dim3((K + 255) / 256), dim3(256), 0, st, a);
  LDS_HIP(hipcub::DeviceScan::ExclusiveSum(s.cub, need, a.cnt, a.base, K, st));
  hipLaunchKernelGGL(wal_lds_publish, dim3(1), dim3(64), 0, st, a, s.d_hres);
  LDS_HIP(hipGetLastError());
  LDS_HIP(hipStreamSynchronize(st));
  if (s.h_res[3] != 0) return TKV_OK;  // the fast stitch does not hold: the caller runs the round-3 pass
  const std::uint64_t n = s.h_res[4], nbig = s.h_res[2], maxp = s.h_res[1];
  const std::uint64_t chain_end = s.h_res[5];
  const bool broke = (s.h_res[6] & kBroke) != 0;
  // 4-5: dense list, record check, deferred payloads, one sync
  if (n) {
    if (int rc = grow(&s.rec, &s.cap_rec, n, 4)) return rc;
    a.rec = s.rec;
    std::uint8_t* bg = static_cast<std::uint8_t*>(s.bigs);
    if (int rc = grow(&bg, &s.cap_big, std::max<std::uint64_t>(nbig, 1), 8 + 4 + 8 + 4 + 4)) return rc;
    s.bigs = bg;
    a.big_off = reinterpret_cast<std::uint64_t*>(bg);
    a.big_idx = a.big_off + s.cap_big;
    a.big_len = reinterpret_cast<std::uint32_t*>(a.big_idx + s.cap_big);
    a.big_crc = a.big_len + s.cap_big;
    a.big_got = a.big_crc + s.cap_big;
    hipLaunchKernelGGL(wal_lds_compact, dim3((K + 255) / 256), dim3(256), 0, st, a);
    RecArgs ra{w, size, s.rec, n, nullptr, s.res + 4, 0, kLdsDefer};
    launch_records(ra, static_cast<std::uint32_t>(maxp), ncu, tabs, st);
    if (nbig) {
      if (int rc = batch_device_impl(kAlgoCrc32, w, a.big_off, a.big_len, nullptr, a.big_got, nbig, st)) return rc;
      hipLaunchKernelGGL(wal_lds_big, dim3(static_cast<unsigned>((nbig + 255) / 256)), dim3(256), 0, st, a, nbig);
    }
    hipLaunchKernelGGL(wal_lds_final, dim3(1), dim3(1), 0, st, a, n, s.d_hres);
    LDS_HIP(hipGetLastError());
    LDS_HIP(hipStreamSynchronize(st));
  } else {
    s.h_res[7] = ~0ull;
  }
  const std::uint64_t first = std::min<std::uint64_t>(s.h_res[7], n);
  r->good = first;
  r->corrupted = first < n || broke;
  r->stop = first < n ? s.h_res[8] : chain_end;
  r->resume = false;
  *used = true;
  return TKV_OK;
}

}  // namespace tkv

extern "C" int tkv_wal_check_records_device(const uint8_t* d_img, uint64_t size, const uint32_t* d_rec_off, uint64_t n,
                                            uint32_t max_payload, uint32_t* d_crc, uint64_t* d_first_bad,
                                            void* stream) {
  using namespace tkv;
  if (!d_first_bad || (n && (!d_img || !d_rec_off))) return set_error(TKV_INVALID_ARGUMENT, "null pointer");
  if (size > 0xFFFFFFFFull + 1ull) return set_error(TKV_INVALID_ARGUMENT, "image larger than 4 GiB (u32 offsets)");
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  const int ncu = cu_count();
  if (ncu <= 0) return set_error(TKV_IO_ERROR, "no device");
  auto st = static_cast<hipStream_t>(stream);
  auto* fb = reinterpret_cast<unsigned long long*>(d_first_bad);
  // no records past an empty image can be good: the first record (if any) is the first bad one
  hipLaunchKernelGGL(rec_init, dim3(1), dim3(1), 0, st, fb, size ? n : 0);
  if (n && size) launch_records(RecArgs{d_img, size, d_rec_off, n, d_crc, fb, 0, 0xFFFFFFFFu}, max_payload, ncu, tabs, st);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e));
  return TKV_OK;
}

extern "C" int tkv_debug_set_wal_lds_walk(int enable) {
  const int prev = tkv::g_wal_lds_walk;
  tkv::g_wal_lds_walk = enable ? 1 : 0;
  return prev;
}
