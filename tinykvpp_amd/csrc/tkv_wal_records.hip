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

#include <algorithm>
#include <atomic>
#include <cstdint>

#include "tkv_crc32.h"
#include "tkv_crc32_device.h"
#include "tkv_engine.h"

namespace tkv {
namespace {

constexpr std::uint32_t kRecMeta = 26;  // wal.hpp kMetadataSize: 8-byte header + op, seq, tombstone, key/value lengths
// The granule kernel uses the 128 KiB table image with one 1024-thread workgroup per CU (narrow
// windows on the 64 KiB image with two 768-thread workgroups measured 3 % slower,
// profiles/r4/lanes16/rec_probe_rec16.jsonl).
constexpr unsigned kRecThreadsN = 1024;

struct RecArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  const std::uint32_t* off;
  std::uint64_t n;
  std::uint32_t* crc;                  // nullable: computed CRC per record (0 when its length is bad)
  unsigned long long* first_bad;       // atomic minimum of bad record indices (preset to n)
  std::uint32_t nwaves;
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
template <int ND, typename KC>
__device__ __forceinline__ std::uint32_t rec_fold(const std::uint32_t* lds, const KC& kc, const std::uint32_t* d,
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

// NG granules per record window; AHEAD steps of granules in flight: 3 at 5 granules, 2 at 6, 1 for
// the wide ones (whose three slots would spill at 16 waves per CU), none at 4 (4-granule windows load
// at the fold: in one process against 3 and 1 steps in flight, profiles/r4/lanes_r/rec4_probe.jsonl,
// 28-byte payloads 0.2946 -> 0.2851 ms, +3.3 %; wider windows lost with it, mixed 22-80 B -4.7 %).
template <int NG, int AHEAD>
__global__ __launch_bounds__(kRecThreadsN) void wal_rec_lanes(RecArgs a, const DeviceTables* tabs) {
  constexpr int ND = 4 * NG - 4;      // realigned dwords of the window
  constexpr int NPAY = ND - 3;        // whole payload dwords folded from the window (payload at dword 2; one spare for the tail)
  constexpr int RING = 4;             // offsets are fetched RING steps ahead of their granules
  constexpr int DRING = AHEAD == 1 ? 2 : 4;
  static_assert(AHEAD >= 0 && AHEAD <= 3, "granules up to three steps ahead");
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
    const std::uint32_t L = live && len_ok ? rlen : 0u;
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
    if (live && (!len_ok || crc != stored || !kv_ok)) atomicMin(a.first_bad, static_cast<unsigned long long>(b));
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

// The record check for narrow windows (4-5 granules) staged through LDS (round 4): a WAL image's
// records lie back to back, so the 64 records of a wave step span about 64 record lengths; the wave
// copies that span (3 KiB at most, else the step loads its granules as wal_rec_lanes does) into its
// own LDS buffer with coalesced LDS-DMA one step ahead, the step's offsets too (one 4-byte DMA per
// lane, two steps ahead, so no ordinary load is pending while the copies fly), and each lane reads
// its record's window from LDS (two reads per dword and v_alignbyte). Slicing tables: the 64 KiB
// image; 12 waves x (2 x 3 KiB + 2 x 256 B) of buffers.
constexpr unsigned kRecLdsThreads = 768;
constexpr std::uint32_t kRecLdsBuf = 3072;
__device__ __forceinline__ std::uint32_t umin32(std::uint32_t x, std::uint32_t y) { return x < y ? x : y; }
__device__ __forceinline__ std::uint32_t umax32(std::uint32_t x, std::uint32_t y) { return x > y ? x : y; }
__device__ __forceinline__ std::uint32_t wave_min_u32(std::uint32_t v) {
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0xB1, 0xF, 0xF, false)));
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0x4E, 0xF, 0xF, false)));
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0x141, 0xF, 0xF, false)));
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0x140, 0xF, 0xF, false)));
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0x142, 0xA, 0xF, false)));
  v = umin32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(~0u, v, 0x143, 0xC, 0xF, false)));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ std::uint32_t wave_max_u32(std::uint32_t v) {
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false)));
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false)));
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, false)));
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, false)));
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false)));
  v = umax32(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false)));
  return __builtin_amdgcn_readlane(v, 63);
}

template <int NG>
__global__ __launch_bounds__(kRecLdsThreads) void wal_rec_lds(RecArgs a, const DeviceTables* tabs) {
  constexpr int ND = 4 * NG - 4;  // realigned dwords of the window
  constexpr int NPAY = ND - 3;
  constexpr std::uint32_t kWaves = kRecLdsThreads / 64;
  constexpr std::uint32_t kTabBytes = kLdsSliceWords * 2;  // the 64 KiB image
  __shared__ std::uint32_t lds[(kTabBytes + kWaves * (2 * kRecLdsBuf + 2 * 256)) / 4];
  dev::fill_lds_slicing16(tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const dev::LaneConstX kc = dev::lane_const16(lane);
  const std::uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * kWaves + wid;
  const std::uint64_t W = a.nwaves, n = a.n;
  const std::uint64_t TS = (n + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  if (ns == 0) return;
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(a.w);
  const std::uintptr_t glast = (w0 + a.size - 1u) & ~static_cast<std::uintptr_t>(15);  // the image's last granule
  auto gran = [&](std::uintptr_t p) { return dev::gload16(p < glast ? p : glast); };
  std::uint8_t* l8 = reinterpret_cast<std::uint8_t*>(lds);
  const std::uint32_t data0 = kTabBytes + wid * 2u * kRecLdsBuf;             // byte offsets in LDS
  const std::uint32_t offs0 = kTabBytes + kWaves * 2u * kRecLdsBuf + wid * 512u;
  auto copy_offs = [&](std::uint32_t j) {  // step j's 64 offsets into offset buffer j & 1
    const std::uint64_t b = (s0 + j) * 64u + lane;
    const std::uint32_t* src = a.off + (b < n ? b : n - 1u);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(
                                         reinterpret_cast<std::uintptr_t>(src)),
                                     reinterpret_cast<__attribute__((address_space(3))) void*>(
                                         reinterpret_cast<std::uintptr_t>(l8 + offs0 + (j & 1u) * 256u)),
                                     4, 0, 0);
  };
  // per step (uniform): staged in LDS, the lowest offset and its place in the first granule
  bool st_staged0 = false, st_staged1 = false;  // (two named slots: no dynamically indexed arrays)
  std::uint32_t st_min0 = 0, st_min1 = 0, st_o0 = 0, st_o1 = 0;
  auto plan = [&](std::uint32_t j) {  // step j's offsets have landed: copy its span if it fits
    const std::uint32_t k = j & 1u;
    const std::uint32_t off = dev::lds_at(lds, offs0 + k * 256u + 4u * lane);
    const std::uint32_t mn = wave_min_u32(off), mx = wave_max_u32(off);
    const std::uintptr_t al = (w0 + mn) & ~static_cast<std::uintptr_t>(15);
    const std::uint32_t o = static_cast<std::uint32_t>(w0 + mn - al);
    const bool staged = static_cast<std::uint64_t>(mx - mn) + o + 16u * NG <= kRecLdsBuf;
    if (k) {
      st_staged1 = staged;
      st_min1 = mn;
      st_o1 = o;
    } else {
      st_staged0 = staged;
      st_min0 = mn;
      st_o0 = o;
    }
    if (staged) {
#pragma unroll
      for (std::uint32_t i = 0; i < kRecLdsBuf / 1024u; ++i) {
        std::uintptr_t g = al + 1024u * i + 16u * lane;
        g = g < glast ? g : glast;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(g),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<std::uintptr_t>(l8 + data0 + k * kRecLdsBuf + 1024u * i)),
                                         16, 0, 0);
      }
    }
  };

  copy_offs(0);
  if (ns > 1) copy_offs(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  plan(0);
  for (std::uint32_t j = 0; j < ns; ++j) {
    dev::set_prio_from_left<3>(ns - j, ns);
    // step j's span and step j+1's offsets have landed. With a result array, step j-1's result store
    // is the newest memory operation and need not be waited for (vmcnt counts stores too; waiting for
    // it measured 0.8 % slower, profiles/r4/storewait/)
    if (a.crc && j > 0u) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const std::uint32_t k = j & 1u;
    const std::uint32_t off = dev::lds_at(lds, offs0 + k * 256u + 4u * lane);  // (read before its buffer is reused)
    const bool staged = k ? st_staged1 : st_staged0;
    const std::uint32_t mn = k ? st_min1 : st_min0, o = k ? st_o1 : st_o0;
    if (j + 1u < ns) {
      plan(j + 1u);
      if (j + 2u < ns) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the offset read above is done with its buffer)
        copy_offs(j + 2u);
      }
    }
    const std::uint64_t b = (s0 + j) * 64u + lane;
    const bool live = b < n;
    const std::uintptr_t p = w0 + off;
    std::uint32_t d[ND + 1];
    if (staged) {
      const std::uint32_t qb = data0 + k * kRecLdsBuf + o + (off - mn);
      const std::uint32_t qa = qb & ~3u, sh = qb & 3u;
      std::uint32_t r[ND + 1];
#pragma unroll
      for (int i = 0; i <= ND; ++i) r[i] = dev::lds_at(lds, qa + 4u * i);
#pragma unroll
      for (int i = 0; i < ND; ++i) d[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
    } else {
      uint4 q[NG];
      const std::uintptr_t al = p & ~static_cast<std::uintptr_t>(15);
#pragma unroll
      for (int i = 0; i < NG; ++i) q[i] = gran(al + 16u * i);
      std::uint32_t e[4 * NG - 4];
      rec_dwords<NG>(q, static_cast<std::uint32_t>(p & 15u), e);
#pragma unroll
      for (int i = 0; i < ND; ++i) d[i] = e[i];
    }
    d[ND] = 0u;
    const std::uint32_t rlen = d[0], stored = d[1];
    const std::uint32_t klen = __builtin_amdgcn_alignbyte(d[5], d[4], 2u);
    const std::uint32_t vlen = __builtin_amdgcn_alignbyte(d[6], d[5], 2u);
    const std::uint64_t left = off < a.size ? a.size - off : 0u;
    const bool len_ok = left >= kRecMeta && static_cast<std::uint64_t>(rlen) + 8u <= left;  // wal.cpp:68, :80
    const std::uint32_t L = live && len_ok ? rlen : 0u;
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
      for (int i = 0; i < 16; ++i) e17[i] = e[i];
      e17[16] = 0u;
      c = rec_fold<16>(lds, kc, e17, m, c);
    }
    const std::uint32_t crc = c ^ 0xFFFFFFFFu;
    const bool kv_ok = static_cast<std::uint64_t>(klen) + vlen + (kRecMeta - 8u) <= rlen;  // wal.cpp:118-121
    if (live && a.crc) a.crc[b] = len_ok ? crc : 0u;
    if (live && (!len_ok || crc != stored || !kv_ok)) atomicMin(a.first_bad, static_cast<unsigned long long>(b));
  }
}

int cu_count() {
  static std::atomic<int> cached[64] = {};  // (concurrent first calls store the same value)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int c = cached[dev].load(std::memory_order_relaxed);
  if (c == 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

// The record check over n records (first_bad preset to n by the caller's stream order).
void launch_records(RecArgs a, std::uint32_t max_payload, int ncu, const DeviceTables* tabs, hipStream_t st) {
  const std::uint64_t steps = (a.n + 63) / 64;
  // window: NG granules hold the header, the key/value lengths and a first fold of 16 NG - 28 payload
  // bytes at any alignment (36-byte payloads: 4 granules; 68: 6; 100: 8); longer ones continue 64 bytes
  // at a time. Records are latency-bound like the lane kernel (profiles/r4/rec_check/).
  const std::uint32_t ng =
      std::min<std::uint32_t>(8u, std::max<std::uint32_t>(4u, (std::min<std::uint32_t>(max_payload, 1024u) + 28u + 15u) / 16u));
  // narrow windows with payloads of at least 32 bytes: staged through LDS (wal_rec_lds). One process
  // against wal_rec_lanes (profiles/r4/rec_lds/): 44-byte records (36-byte payloads) 2957 -> 3099 GB/s
  // of payload; 36-byte records (28-byte payloads) 2813 -> 2591, where the per-step cost (span
  // reduction, copy, full wait) outweighs what the copy saves, so shorter payloads keep wal_rec_lanes.
  if (ng <= 5 && max_payload >= 32u) {
    constexpr std::uint64_t waves = kRecLdsThreads / 64;
    const std::uint64_t grid =
        std::max<std::uint64_t>(1, std::min<std::uint64_t>(static_cast<std::uint64_t>(ncu), (steps + waves - 1) / waves));
    a.nwaves = static_cast<std::uint32_t>(grid * waves);
    if (ng == 4) hipLaunchKernelGGL((wal_rec_lds<4>), dim3(static_cast<unsigned>(grid)), dim3(kRecLdsThreads), 0, st, a, tabs);
    else hipLaunchKernelGGL((wal_rec_lds<5>), dim3(static_cast<unsigned>(grid)), dim3(kRecLdsThreads), 0, st, a, tabs);
    return;
  }
  const std::uint64_t waves = kRecThreadsN / 64;
  const std::uint64_t grid =
      std::max<std::uint64_t>(1, std::min<std::uint64_t>(static_cast<std::uint64_t>(ncu), (steps + waves - 1) / waves));
  a.nwaves = static_cast<std::uint32_t>(grid * waves);
  const dim3 g(static_cast<unsigned>(grid)), b(kRecThreadsN);
  switch (ng) {
    case 4: hipLaunchKernelGGL((wal_rec_lanes<4, 0>), g, b, 0, st, a, tabs); break;
    case 5: hipLaunchKernelGGL((wal_rec_lanes<5, 3>), g, b, 0, st, a, tabs); break;
    case 6: hipLaunchKernelGGL((wal_rec_lanes<6, 2>), g, b, 0, st, a, tabs); break;
    case 7: hipLaunchKernelGGL((wal_rec_lanes<7, 1>), g, b, 0, st, a, tabs); break;
    default: hipLaunchKernelGGL((wal_rec_lanes<8, 1>), g, b, 0, st, a, tabs); break;
  }
}

}  // namespace
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
  if (n && size) launch_records(RecArgs{d_img, size, d_rec_off, n, d_crc, fb, 0}, max_payload, ncu, tabs, st);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e));
  return TKV_OK;
}
