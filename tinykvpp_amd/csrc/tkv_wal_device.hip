// WAL recovery verify on the device: the record_len chain walk of
// wal_entry::decode (/root/reference/src/engine/wal.cpp:63-130) over a WAL image resident in HBM,
// the CRC check of every record (wal.cpp:89-96) and the key/value bounds check (wal.cpp:118-121),
// ending in the first corruption - without walking the chain on the host.
//
// The record chain is a linked list through the image (record i+1 starts 8 + record_len bytes after
// record i). The image is cut into regions of RS bytes (16 KiB - 1 MiB, about two per wave slot of
// the device), one wave per region (wal_region):
//  1. The wave streams its region in 2 KiB chunks, 32 bytes per lane, three chunks in flight. In each
//     chunk every lane takes the first plausible header of its 32 bytes (one the reference encoder
//     could have written, wal.cpp:19-61: op and tombstone bytes 0/1 found byte-parallel in registers,
//     then record_len = 18 + klen + vlen) and walks the one to three headers that start there (L2-hot
//     loads). The lane that holds the chain's current position starts there instead. Ballots then
//     check that every lane's exit is the next lane's start; when they all agree (every WAL without
//     fake headers in its values) the chain through the chunk is those lanes' records, otherwise a
//     scalar loop follows it lane by lane and re-walks a lane from its true entry. The region's first
//     record is its first plausible header (region 0: byte 0).
//  2. Records of at most kWalFold payload bytes queue in LDS and are folded 128 at a time, one lane
//     per record, with the slicing tables in LDS (the lane-block fold of the batch engine, DESIGN.md
//     §4.5); larger ones are appended to a big list for one CRC batch through the irregular path. A
//     region's walk stops at its first failing record (bounds or CRC).
//  3. wal_jump: next(k) = the region holding the exit of region k's walk. The true chain visits
//     regions 0, next(0), ...; pointer jumping (x4 per round) marks exactly those regions and
//     wal_link hands every one its entry E. A region whose entry is not its speculative start is
//     walked again from E (wal_region in exact mode). Entries are exact up to and including the first
//     region k* whose speculative exit was wrong; later regions are dropped, and when no record up to
//     k*'s exact exit fails, the next pass resumes there (a true record start).
//  4. One exclusive scan numbers the records; the first bad record is an atomic minimum of record
//     indices over the regions and the big list.
// Every step reads the image in HBM; the host only reads back a few counters.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "tkv_crc32.h"
#include "tkv_crc32_device.h"
#include "tkv_engine.h"
#include "tkv_wal_device.h"

namespace tkv {
namespace {

constexpr std::uint64_t kWalMeta = 26;      // wal.hpp:21-27 kMetadataSize
constexpr std::uint32_t kWalFold = 256;     // payloads up to this size are folded by wal_region's lanes
constexpr std::uint64_t kNone = ~0ull;
constexpr unsigned kRegThreads = 768;       // wal_region: 12 waves (LDS: tables + 12 chunk copies), one region each
constexpr unsigned kRegWaves = kRegThreads / 64;
constexpr std::uint64_t kChunk = 2048;      // bytes per wave step: 32 per lane (two 16-byte granules)
// A wave's LDS copy of its chunk carries the first kHalo bytes of the next one: every header that
// starts in the chunk, and every record with a payload of at most kWalFold bytes, lies whole in it.
constexpr std::uint32_t kHalo = 8 + kWalFold + 32;
constexpr std::uint32_t kHaloGran = kHalo / 16;   // 18 granules, loaded by lanes 0-17
// Good records (at least kWalMeta bytes each) that can start in one chunk.
constexpr std::uint32_t kChunkRecs = (kChunk + kWalMeta - 1) / kWalMeta + 1;
constexpr std::uint64_t kRegionMin = 16 << 10, kRegionMax = 1 << 20;
constexpr std::uint32_t kBigReserve = 64;   // big-list slots a wave reserves at a time

struct WalArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  std::uint64_t RS;          // region size (a multiple of kChunk)
  std::uint32_t K;           // regions
  // per region: the speculative walk
  std::uint64_t* S;          // speculative start (kNone: no plausible header)
  std::uint64_t* X;          // exit: the first record start at or past the region's end, or where the walk
                             //   stopped (a header that does not fit, or a failing record)
  std::uint8_t* broke;       // 0: ran to its exit, 1: a header that does not fit at X, 2: stopped at a failure
  std::uint64_t* spec_cnt;   // good records walked
  std::uint32_t* next;       // region of X (K: end of image, stopped, or no start)
  // per region: the walk the results come from (speculative, or exact from the entry)
  std::uint64_t* first_loc;  // first failing record (bounds or CRC of a folded payload): local index, kNone
  std::uint64_t* first_pos;  //   and its start
  std::uint32_t* Ja;         // pointer-jumping tables
  std::uint32_t* Jb;
  std::uint8_t* on;          // region is on the true chain
  std::uint8_t* recheck;     // entered off its speculative start: walked again in exact mode
  std::uint64_t* entry;      // true entry point of an on-path region
  std::uint64_t* cnt;        // good records of an on-path region from its entry (0 off the path)
  std::uint64_t* base;       // exclusive scan of cnt: index of the region's first record
  std::uint64_t* Xe;         // exit and break of the walk from the entry
  std::uint8_t* Be;
  std::uint64_t* bad_at;     // index of the region's first failing record
  // big list (payloads above kWalFold), appended in any order
  std::uint64_t cap_big;
  std::uint64_t* big_off;    // payload offset in the image
  std::uint64_t* big_key;    // (region << 32) | local record index
  std::uint32_t* big_len;
  std::uint32_t* big_crc;    // stored CRC
  std::uint32_t* got;        // engine CRC of each big payload (finalized)
  std::uint8_t* big_tag;     // 0: appended by the speculative walk, 1: by the exact walk
  const DeviceTables* tabs;
  std::uint64_t* res;        // [0] first region with a wrong speculative exit, [1] chain end and
                             // [2] chain broke (from the path's last region), [3] first bad record,
                             // [4] its start, [5] regions re-walked, [6] big records appended
};

__device__ __forceinline__ std::uint64_t gid() {
  return blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
}

__device__ __forceinline__ std::uint32_t le1_bytes4(std::uint32_t d) {
  // 4-bit mask: bit i set iff byte i of d is 0 or 1
  const std::uint32_t x = d & 0xFEFEFEFEu;
  const std::uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu) & 0x80808080u;
  return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// Slicing tables into LDS (the row kernels' lane-shift tables are not needed here).
__device__ __forceinline__ void fill_slices(const DeviceTables* tabs, std::uint32_t* lds) {
  for (std::uint32_t u = threadIdx.x; u < 1024u; u += blockDim.x) {
    const std::uint32_t pair = u >> 9, e = (u >> 1) & 255u, tt = u & 1u;
    const std::uint32_t v = tabs->slice[2 * pair + tt][e];
    uint4* dst = reinterpret_cast<uint4*>(lds + pair * 16384u + e * 64u + tt * 32u);
#pragma unroll
    for (std::uint32_t k = 0; k < 8u; ++k) dst[(k + u) & 7u] = make_uint4(v, v, v, v);
  }
  __syncthreads();
}

// The header fields of a record: record_len, the stored CRC, key and value lengths (wal.cpp:14-18).
struct Hdr {
  std::uint32_t rlen, stored;
  std::uint64_t klen, vlen;
};

// The fields from the wave's LDS copy of its chunk (byte b of the copy, b < kChunk; the copy holds
// the 32 bytes after the chunk too, so a header that starts in the chunk is whole in it), realigned
// with v_alignbyte.
__device__ __forceinline__ Hdr header_lds(const std::uint32_t* cb, std::uint32_t b) {
  const std::uint32_t* d = cb + (b >> 2);
  const std::uint32_t t = b & 3u;
  const std::uint32_t x0 = d[0], x1 = d[1], x2 = d[2], x4 = d[4], x5 = d[5], x6 = d[6], x7 = d[7];
  auto at = [&](std::uint32_t lo, std::uint32_t hi) { return t ? __builtin_amdgcn_alignbyte(hi, lo, t) : lo; };
  Hdr f;
  f.rlen = at(x0, x1);
  f.stored = at(x1, x2);
  const bool up = t >= 2u;
  const std::uint32_t o = (t + 2u) & 3u;
  auto at2 = [&](std::uint32_t lo, std::uint32_t hi) { return o ? __builtin_amdgcn_alignbyte(hi, lo, o) : lo; };
  f.klen = up ? at2(x5, x6) : at2(x4, x5);
  f.vlen = up ? at2(x6, x7) : at2(x5, x6);
  return f;
}

// The records that start in a lane's 32 bytes [.., hi) from s (wal.cpp:63-87: header size, then
// record_len against what is left; then the key/value bounds, wal.cpp:118-121). A good record is at
// least kWalMeta bytes long, so at most two start there, and a third step can only find a header
// that does not fit (status 1) or a failing record (status 2). X: the start after the last good
// record (or of the one that broke or failed).
struct LaneWalk {
  std::uint64_t X, p0, p1;
  std::uint32_t n, status, r0, r1, c0, c1;
};
__device__ __forceinline__ LaneWalk lane_walk(const WalArgs& a, const std::uint32_t* cb, std::int64_t cs, std::uint64_t s,
                                              std::uint64_t hi) {
  LaneWalk L{s, 0, 0, 0, 0, 0, 0, 0, 0};
  std::uint64_t p = s;
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    if (p >= hi || L.status != 0u) break;
    if (a.size - p < kWalMeta) {
      L.status = 1;
      break;
    }
    const Hdr f = header_lds(cb, static_cast<std::uint32_t>(static_cast<std::int64_t>(p) - cs));
    if (static_cast<std::uint64_t>(f.rlen) + 8 > a.size - p) {
      L.status = 1;
      break;
    }
    if (kWalMeta + f.klen + f.vlen > 8ull + f.rlen) {
      L.status = 2;
      break;
    }
    if (L.n == 0) {
      L.p0 = p;
      L.r0 = f.rlen;
      L.c0 = f.stored;
    } else {
      L.p1 = p;
      L.r1 = f.rlen;
      L.c1 = f.stored;
    }
    ++L.n;
    p += 8 + static_cast<std::uint64_t>(f.rlen);
  }
  L.X = p;
  return L;
}

__device__ __forceinline__ std::uint64_t readlane64(std::uint64_t v, std::uint32_t l) {
  const std::uint32_t lo = __builtin_amdgcn_readlane(static_cast<std::uint32_t>(v), l);
  const std::uint32_t hi = __builtin_amdgcn_readlane(static_cast<std::uint32_t>(v >> 32), l);
  return static_cast<std::uint64_t>(hi) << 32 | lo;
}

// The CRC of record k of a chunk's small records, one per lane (slot word: byte b of the record in
// the wave's LDS copy of its chunk | rlen << 11), from that copy: the payload [b + 8, b + 8 + rlen)
// folded from 0xFFFFFFFF a dword at a time with slicing-by-4 (read aligned and realigned with
// v_alignbyte) for as many dwords as the wave's longest payload has, then its last 1-3 bytes with
// Sarwate steps, and compared with the stored CRC at b + 4. Every step is predicated with selects
// rather than branched on: lanes differ in length, and per-lane branches cost more scalar
// instructions than the fold itself. live: the lane has a record. Returns whether it matches (true
// for a lane without one).
__device__ __forceinline__ bool fold_lds(const std::uint32_t* lds, const dev::LaneConst& kc, const std::uint32_t* cb,
                                         std::uint32_t word, bool live) {
  const std::uint32_t b = live ? word & 2047u : 0u, rl = live ? (word >> 11) & 511u : 0u;
  auto dw = [&](std::uint32_t byte) {  // little-endian u32 at any byte of the copy
    const std::uint32_t* d = cb + (byte >> 2);
    const std::uint32_t t = byte & 3u;
    return t ? __builtin_amdgcn_alignbyte(d[1], d[0], t) : d[0];
  };
  const std::uint32_t stored = dw(b + 4u);
  const std::uint32_t nf = rl >> 2;
  std::uint32_t mx = nf;  // the wave's longest payload, in whole dwords
#pragma unroll
  for (unsigned m = 32; m > 0; m >>= 1) mx = std::max(mx, static_cast<std::uint32_t>(__shfl_xor(static_cast<int>(mx), m, 64)));
  const std::uint32_t kmax = __builtin_amdgcn_readfirstlane(mx);
  const std::uint32_t s0 = b + 8u;
  const std::uint32_t* d = cb + (s0 >> 2);
  const std::uint32_t t = s0 & 3u;
  dev::Reg p{0xFFFFFFFFu, 0u};
  std::uint32_t lo = d[0];
  for (std::uint32_t k = 0; k < kmax; ++k) {
    const std::uint32_t hi = d[k + 1];
    const std::uint32_t w = t ? __builtin_amdgcn_alignbyte(hi, lo, t) : lo;
    lo = hi;
    dev::Reg np = p;
    dev::slice4(lds, np, w, kc);
    const bool on = k < nf;
    p.t = on ? np.t : p.t;
    p.u = on ? np.u : p.u;
  }
  // the last rl & 3 bytes
  const std::uint32_t tb = rl & 3u;
  const std::uint32_t wt = dw(s0 + 4u * nf);
  std::uint32_t c = p.value();
#pragma unroll
  for (std::uint32_t j = 0; j < 3u; ++j) {
    const std::uint32_t cn = (c >> 8) ^ dev::lds_at(lds, (((c ^ (wt >> (8 * j))) & 0xFFu) << 8) | kc.L0);
    c = j < tb ? cn : c;
  }
  return !live || (c ^ 0xFFFFFFFFu) == stored;
}

// A chunk's bytes in flight: lane l's 32 bytes, and for lanes 0-17 one granule of the next chunk's
// first kHalo bytes.
struct ChunkRegs {
  uint4 v0, v1, h;
};
__device__ __forceinline__ void chunk_issue(std::uintptr_t al, std::uint64_t lim, std::uint64_t c, std::uint32_t lane,
                                            ChunkRegs& k) {
  // lim: end of the image from al (the image's start rounded down to 16 bytes); only granules that
  // start before that end are read, so no load leaves the image's pages. A granule that does not
  // loads the image's first granule instead; those bytes are never used (every header, candidate and
  // record is bounded by the image's size), and no zeroing select may follow the loads here, or the
  // compiler waits for them at once.
  const std::uint64_t q = c * kChunk + 32u * lane;
  const std::uint64_t h = (c + 1) * kChunk + 16u * lane;
  k.v0 = dev::gload16(q < lim ? al + q : al);
  k.v1 = dev::gload16(q + 16 < lim ? al + q + 16 : al);
  k.h = dev::gload16(lane < kHaloGran && h < lim ? al + h : al);
}

// 1-2. One wave per region [k_lo, k_hi). exact = 0: every region from its first plausible header
// (region 0 from byte 0); exact = 1: only the regions flagged `recheck`, from their entry.
__global__ __launch_bounds__(kRegThreads) void wal_region(WalArgs a, std::uint64_t k_lo, std::uint64_t k_hi,
                                                          int exact) {
  __shared__ std::uint32_t lds[kLdsSliceWords];
  __shared__ uint4 chunkbuf[kRegWaves][(kChunk + kHalo) / 16];  // the wave's chunk and the next kHalo bytes
  __shared__ std::uint32_t slotbuf[kRegWaves][kChunkRecs];      // its small records, compacted
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t r = k_lo + static_cast<std::uint64_t>(blockIdx.x) * kRegWaves + wid;
  bool work = r < k_hi && (!exact || (a.on[r] && a.recheck[r]));
  if (__syncthreads_or(work ? 1 : 0) == 0) return;  // (uniform per workgroup)
  fill_slices(a.tabs, lds);
  if (!work) return;
  const dev::LaneConst kc = dev::lane_const(lane);
  uint4* cb4 = chunkbuf[wid];
  const std::uint32_t* cb = reinterpret_cast<const std::uint32_t*>(cb4);
  std::uint32_t* slots = slotbuf[wid];

  const std::uint64_t size = a.size;
  const std::uint64_t rb = r * a.RS;
  const std::uint64_t re = std::min(rb + a.RS, size);
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(a.w);
  const std::uintptr_t al = w0 & ~static_cast<std::uintptr_t>(15);
  const std::uint64_t off0 = w0 - al;
  const std::uint64_t lim = off0 + size;
  const std::int64_t size26 = static_cast<std::int64_t>(size) - static_cast<std::int64_t>(kWalMeta);

  std::uint64_t P = exact ? a.entry[r] : (r == 0 ? 0 : kNone);  // the chain's next record start
  std::uint64_t S = P;                                          // the region's first record start
  std::uint64_t nrec = 0;                                       // good records so far
  std::uint64_t fail_loc = kNone, fail_pos = 0;
  std::uint32_t brk = 0;
  bool done = false;

  // chunks: from the one holding the region's start (or its entry) to the one holding re - 1
  const std::uint64_t c_first = ((P == kNone ? rb : P) + off0) / kChunk;
  const std::uint64_t c_last = (re - 1 + off0) / kChunk;

  // Big-list slots are reserved kBigReserve at a time (one returning atomic per reservation, not per
  // chunk); unused ones are written as empty entries of no region.
  std::uint64_t res_base = 0;
  std::uint32_t res_left = 0;
  auto pad_big = [&](std::uint64_t b, std::uint32_t n) __attribute__((always_inline)) {
    if (lane < n && b + lane < a.cap_big) {
      a.big_off[b + lane] = 0;
      a.big_len[b + lane] = 0;
      a.big_crc[b + lane] = 0;
      a.big_key[b + lane] = kNone;
      a.big_tag[b + lane] = 0xFF;
    }
  };

  // One chunk: returns with P advanced past it (or done set).
  auto process = [&](std::uint64_t c, const ChunkRegs& k) __attribute__((always_inline)) {
    const std::int64_t cs = static_cast<std::int64_t>(c * kChunk) - static_cast<std::int64_t>(off0);  // image pos
    const std::int64_t ce = cs + static_cast<std::int64_t>(kChunk);
    if (P != kNone && static_cast<std::int64_t>(P) >= ce) return;  // inside a record that spans the chunk
    cb4[2 * lane] = k.v0;
    cb4[2 * lane + 1] = k.v1;
    if (lane < kHaloGran) cb4[kChunk / 16 + lane] = k.h;
    __builtin_amdgcn_wave_barrier();
    const std::int64_t sub = cs + 32 * static_cast<std::int64_t>(lane);
    const std::uint64_t sub_hi = static_cast<std::uint64_t>(std::max<std::int64_t>(sub + 32, 0));
    // lane e0 holds P; lanes before it take no part, lanes after it take their first plausible header
    const std::uint32_t e0 = P == kNone ? 0u : static_cast<std::uint32_t>((static_cast<std::int64_t>(P) - cs) >> 5);
    std::uint64_t start = kNone;
    if (P != kNone && lane == e0) start = P;
    if (lane > e0 || P == kNone) {
      std::uint32_t dw[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 v = cb4[2 * lane + i];
        dw[4 * i] = v.x;
        dw[4 * i + 1] = v.y;
        dw[4 * i + 2] = v.z;
        dw[4 * i + 3] = v.w;
      }
      std::uint64_t F = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) F |= static_cast<std::uint64_t>(le1_bytes4(dw[i])) << (4 * i);
      std::uint32_t cand = static_cast<std::uint32_t>((F >> 8) & (F >> 17));  // bytes j+8, j+17 are 0/1
      // positions: at or after the region's start (when searching for it), before re, header inside the image
      const std::int64_t lo = P == kNone ? static_cast<std::int64_t>(rb) : 0;
      const std::int64_t hi = std::min<std::int64_t>(static_cast<std::int64_t>(re), size26 + 1);
      const std::int64_t jlo = std::max<std::int64_t>(lo - sub, 0), jhi = std::min<std::int64_t>(hi - sub, 32);
      if (jhi <= jlo) {
        cand = 0;
      } else {
        cand &= (jhi >= 32 ? 0xFFFFFFFFu : (1u << jhi) - 1u) & ~((1u << jlo) - 1u);
      }
      while (cand) {
        const std::uint64_t p = static_cast<std::uint64_t>(sub + __builtin_ctz(cand));
        const Hdr f = header_lds(cb, static_cast<std::uint32_t>(static_cast<std::int64_t>(p) - cs));
        if (static_cast<std::uint64_t>(f.rlen) == 18ull + f.klen + f.vlen && f.rlen + 8ull <= size - p) {
          start = p;
          break;
        }
        cand &= cand - 1;
      }
    }
    std::uint64_t H = __ballot(start != kNone);
    if (P == kNone) {  // still looking for the region's first record
      if (H == 0) return;
      const std::uint32_t first = static_cast<std::uint32_t>(__builtin_ctzll(H));
      P = readlane64(start, first);
      S = P;
    }
    const std::uint64_t lane_hi = std::min<std::uint64_t>(sub_hi, re);
    LaneWalk L{start, 0, 0, 0, 0, 0, 0, 0, 0};
    if (start != kNone) L = lane_walk(a, cb, cs, start, lane_hi);
    // Fast path: every lane's exit is the start of the next lane with a start (or leaves the chunk,
    // for the last one), so the chain is exactly those lanes.
    const std::uint64_t above = lane == 63u ? 0ull : H & (~0ull << (lane + 1));
    const std::uint32_t nh = above ? static_cast<std::uint32_t>(__builtin_ctzll(above)) : 64u;
    const bool inside = L.status == 0u && L.X < static_cast<std::uint64_t>(ce) && L.X < re;
    const std::uint32_t lnx = inside ? static_cast<std::uint32_t>((static_cast<std::int64_t>(L.X) - cs) >> 5) : 64u;
    const std::uint64_t s_nh = __shfl(start, static_cast<int>(nh & 63u), 64);
    const bool ok = start == kNone || (lnx == nh && (nh == 64u || s_nh == L.X));
    std::uint64_t chain = H;
    if (__ballot(!ok) != 0) {
      // Slow path: follow the chain lane by lane from P, re-walking a lane whose start is not it.
      chain = 0;
      std::uint64_t pc = P;
      while (pc < static_cast<std::uint64_t>(ce) && pc < re) {
        const std::uint32_t l = __builtin_amdgcn_readfirstlane(
            static_cast<std::uint32_t>((static_cast<std::int64_t>(pc) - cs) >> 5));
        if (readlane64(start, l) != pc && lane == l) {
          start = pc;
          L = lane_walk(a, cb, cs, start, lane_hi);
        }
        chain |= 1ull << l;
        const std::uint32_t st = __builtin_amdgcn_readlane(L.status, l);
        pc = readlane64(L.X, l);
        if (st != 0u) break;
      }
    }
    const std::uint32_t lz = 63u - static_cast<std::uint32_t>(__builtin_clzll(chain));
    const std::uint64_t pexit = readlane64(L.X, lz);
    const std::uint32_t sexit = __builtin_amdgcn_readlane(L.status, lz);
    // The chain's good records, numbered: small ones folded here from the LDS copy, big ones appended
    // to the big list.
    const bool on = (chain >> lane) & 1ull;
    const bool g1 = on && L.n >= 1u, g2 = on && L.n >= 2u;
    const bool s1 = g1 && L.r0 <= kWalFold, s2 = g2 && L.r1 <= kWalFold;
    const bool b1 = g1 && !s1, b2 = g2 && !s2;
    const std::uint64_t lt = (1ull << lane) - 1ull;
    const std::uint64_t G1 = __ballot(g1), G2 = __ballot(g2);
    const std::uint64_t B1 = __ballot(b1), B2 = __ballot(b2);
    const std::uint64_t idx0 = nrec + __popcll(G1 & lt) + __popcll(G2 & lt);
    // Small records, compacted into consecutive lanes in chain order (slot word: byte in the copy |
    // rlen << 11 | rank among the chunk's good records << 20), folded one per lane.
    const std::uint64_t S1 = __ballot(s1), S2 = __ballot(s2);
    const std::uint32_t nsm = static_cast<std::uint32_t>(__popcll(S1) + __popcll(S2));
#ifndef TKV_WAL_PROBE_NOFOLD  // probe builds only (tools/build_variant.sh): the walk without the fold
    if (nsm != 0u) {
#else
    if (false) {
#endif
      const std::uint32_t sp = static_cast<std::uint32_t>(__popcll(S1 & lt) + __popcll(S2 & lt));
      const std::uint32_t rk = static_cast<std::uint32_t>(idx0 - nrec);
      if (s1)
        slots[sp] = static_cast<std::uint32_t>(static_cast<std::int64_t>(L.p0) - cs) | L.r0 << 11 | rk << 20;
      if (s2)
        slots[sp + (s1 ? 1u : 0u)] =
            static_cast<std::uint32_t>(static_cast<std::int64_t>(L.p1) - cs) | L.r1 << 11 | (rk + 1u) << 20;
      __builtin_amdgcn_wave_barrier();
      for (std::uint32_t k0 = 0; k0 < nsm; k0 += 64u) {
        const bool live = k0 + lane < nsm;
        const std::uint32_t word = live ? slots[k0 + lane] : 0u;
        const std::uint64_t bad = __ballot(!fold_lds(lds, kc, cb, word, live));
        if (bad) {  // the first failing record (slot order is record order)
          const std::uint32_t w = __builtin_amdgcn_readlane(word, static_cast<std::uint32_t>(__builtin_ctzll(bad)));
          const std::uint64_t loc = nrec + (w >> 20);
          if (loc < fail_loc) {
            fail_loc = loc;
            fail_pos = static_cast<std::uint64_t>(cs + static_cast<std::int64_t>(w & 2047u));
          }
          done = true;
          break;
        }
      }
    }
    const std::uint32_t nb = static_cast<std::uint32_t>(__popcll(B1) + __popcll(B2));
    if (nb) {
      if (nb > res_left) {  // a new reservation (the old one's unused slots become empty entries)
        pad_big(res_base, res_left);
        const std::uint32_t want = std::max(nb, kBigReserve);
        std::uint64_t got_base = 0;
        if (lane == 0)
          got_base = atomicAdd(reinterpret_cast<unsigned long long*>(&a.res[6]), static_cast<unsigned long long>(want));
        res_base = readlane64(got_base, 0);
        res_left = want;
      }
      const std::uint64_t bbase = res_base + __popcll(B1 & lt) + __popcll(B2 & lt);
      res_base += nb;
      res_left -= nb;
      const std::uint64_t key = r << 32;
      if (b1 && bbase < a.cap_big) {
        a.big_off[bbase] = L.p0 + 8;
        a.big_len[bbase] = L.r0;
        a.big_crc[bbase] = L.c0;
        a.big_key[bbase] = key | idx0;
        a.big_tag[bbase] = static_cast<std::uint8_t>(exact);
      }
      const std::uint64_t bb2 = bbase + (b1 ? 1u : 0u);
      if (b2 && bb2 < a.cap_big) {
        a.big_off[bb2] = L.p1 + 8;
        a.big_len[bb2] = L.r1;
        a.big_crc[bb2] = L.c1;
        a.big_key[bb2] = key | (idx0 + 1);
        a.big_tag[bb2] = static_cast<std::uint8_t>(exact);
      }
    }
    nrec += static_cast<std::uint64_t>(__popcll(G1) + __popcll(G2));
    P = pexit;
    if (sexit == 2u) {  // a record that fails its key/value bounds: the region's last
      if (nrec < fail_loc) {
        fail_loc = nrec;
        fail_pos = pexit;
      }
      done = true;
    } else if (sexit == 1u) {
      brk = 1;
      done = true;
    } else if (P >= re) {
      done = true;
    }
    __builtin_amdgcn_wave_barrier();  // this chunk's LDS reads before the next chunk's writes
  };

  // Two chunk buffers: while one is processed the other's loads are in flight. Unrolled by hand (a
  // buffer indexed at run time would live in scratch); two copies of the chunk step keep the kernel
  // inside the instruction cache (six copies, 104 KB of code, ran at half the speed). The loads are
  // issued unconditionally (clamped inside the image) so that the compiler's wait counting sees
  // straight-line code and waits for a buffer only when it is used.
  ChunkRegs ka, kb;
  auto step = [&](std::uint64_t c, const ChunkRegs& k) __attribute__((always_inline)) {
    if (c <= c_last && !done) process(c, k);
  };
  chunk_issue(al, lim, c_first, lane, ka);
  for (std::uint64_t c = c_first; c <= c_last && !done; c += 2) {
    chunk_issue(al, lim, c + 1, lane, kb);
    step(c, ka);
    chunk_issue(al, lim, c + 2, lane, ka);
    step(c + 1, kb);
  }
  pad_big(res_base, res_left);
  if (S == kNone) {  // no plausible header in the region
    if (!exact) {
      a.S[r] = kNone;
      a.X[r] = kNone;
      a.broke[r] = 0;
      a.spec_cnt[r] = 0;
      a.next[r] = a.K;
      a.first_loc[r] = kNone;
    }
    return;
  }
  if (fail_loc != kNone) brk = 2;
  if (lane == 0) {
    if (!exact) {
      a.S[r] = S;
      a.X[r] = P;
      a.broke[r] = static_cast<std::uint8_t>(brk);
      a.spec_cnt[r] = nrec;
      a.next[r] = (brk != 0 || P >= size) ? a.K : static_cast<std::uint32_t>(P / a.RS);
    } else {
      a.Xe[r] = P;
      a.Be[r] = static_cast<std::uint8_t>(brk);
      a.cnt[r] = nrec;
    }
    a.first_loc[r] = fail_loc;
    a.first_pos[r] = fail_pos;
  }
}

__global__ void wal_jump_init(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K) return;
  a.Ja[k] = a.next[k];
  a.on[k] = k == 0 ? 1 : 0;
  a.recheck[k] = 0;
  a.bad_at[k] = kNone;
}

// 3. One quadrupling round (J = next^(4^t)): every marked k marks J(k), J(J(k)) and J(J(J(k))), then
// J <- J o J o J o J. After round t the marks hold next^i(0) for every i < 4^(t+1), so
// ceil(log4 K) rounds mark the whole path: half the launches of doubling, for two more dependent
// loads per round. Marks set during the round by other threads are regions of the true path too,
// so reading them early is safe. K is the end of the path.
__global__ void wal_jump(const std::uint32_t* J, std::uint32_t* J2, std::uint8_t* on, std::uint32_t K) {
  const std::uint64_t k = gid();
  if (k >= K) return;
  const std::uint32_t j1 = J[k];
  const std::uint32_t j2 = j1 < K ? J[j1] : K;
  const std::uint32_t j3 = j2 < K ? J[j2] : K;
  J2[k] = j3 < K ? J[j3] : K;
  if (on[k]) {
    if (j1 < K) on[j1] = 1;
    if (j2 < K) on[j2] = 1;
    if (j3 < K) on[j3] = 1;
  }
}

// Entry points: each on-path region hands its exit to the region that holds it (one writer each:
// the path is a simple chain).
__global__ void wal_link(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K || !a.on[k]) return;
  if (k == 0) a.entry[0] = 0;
  const std::uint32_t n = a.next[k];
  if (n < a.K) a.entry[n] = a.X[k];
}

// 3'. Records of an on-path region from its entry: the speculative walk's when it started there;
// otherwise the region is flagged for the exact walk (res[5] counts them). Off-path regions count 0.
__global__ void wal_count(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K) return;
  if (!a.on[k]) {
    a.cnt[k] = 0;
    return;
  }
  if (a.entry[k] == a.S[k]) {
    a.cnt[k] = a.spec_cnt[k];
    a.Xe[k] = a.X[k];
    a.Be[k] = a.broke[k];
    if (a.next[k] >= a.K) {
      a.res[1] = a.X[k];
      a.res[2] = a.broke[k] == 1 ? 1 : 0;
    }
  } else {
    a.recheck[k] = 1;
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.res[5]), 1ull);
  }
}

// After the exact walks: res[0] = the first region whose speculative exit was wrong.
__global__ void wal_count_exact(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K || !a.on[k] || !a.recheck[k]) return;
  if (a.Xe[k] != a.X[k] || a.Be[k] != a.broke[k]) atomicMin(reinterpret_cast<unsigned long long*>(&a.res[0]), k);
  if (a.next[k] >= a.K) {
    a.res[1] = a.Xe[k];
    a.res[2] = a.Be[k] == 1 ? 1 : 0;
  }
}

// Regions past the first one with a wrong speculative exit are not on the true chain (or not known
// to be): drop them.
__global__ void wal_trim(WalArgs a, std::uint64_t kstar) {
  const std::uint64_t k = gid();
  if (k < a.K && k > kstar) a.cnt[k] = 0;
}

// 4. The first failing record of each counted region (bounds, or CRC of a folded payload), as a
// record index.
__global__ void wal_gather(WalArgs a, std::uint64_t kstar) {
  const std::uint64_t k = gid();
  if (k >= a.K || !a.on[k] || k > kstar) return;
  const std::uint64_t f = a.first_loc[k];
  if (f != kNone) {
    a.bad_at[k] = a.base[k] + f;
    atomicMin(reinterpret_cast<unsigned long long*>(&a.res[3]), a.base[k] + f);
  }
}

// A big-list entry counts when its region is counted and it comes from that region's final walk.
__device__ __forceinline__ bool big_valid(const WalArgs& a, std::uint64_t i, std::uint64_t kstar, std::uint64_t* idx) {
  const std::uint64_t key = a.big_key[i];
  const std::uint64_t k = key >> 32;
  if (k >= a.K || !a.on[k] || k > kstar || a.big_tag[i] != a.recheck[k]) return false;
  *idx = a.base[k] + (key & 0xFFFFFFFFull);
  return true;
}

__global__ void wal_check_big(WalArgs a, std::uint64_t n, std::uint64_t kstar) {
  const std::uint64_t i = gid();
  std::uint64_t idx;
  if (i < n && a.got[i] != a.big_crc[i] && big_valid(a, i, kstar, &idx))
    atomicMin(reinterpret_cast<unsigned long long*>(&a.res[3]), idx);
}

// Start of the first bad record (res[3]): from the region that found it, or from the big list.
__global__ void wal_bad_pos(WalArgs a, std::uint64_t n_big, std::uint64_t kstar) {
  const std::uint64_t i = gid();
  const std::uint64_t want = a.res[3];
  if (i < a.K && a.on[i] && i <= kstar && a.bad_at[i] == want) a.res[4] = a.first_pos[i];
  std::uint64_t idx;
  if (i < n_big && a.got[i] != a.big_crc[i] && big_valid(a, i, kstar, &idx) && idx == want) a.res[4] = a.big_off[i] - 8;
}

// Per-device scratch, grown by doubling and kept between calls (guarded by mu).
struct WalScratch {
  std::mutex mu;
  std::uint64_t cap_regions = 0, cap_big = 0;
  void* regions = nullptr;  // per region: 10 u64, 3 u32, 4 u8 (carve)
  void* bigs = nullptr;     // per big record: 2 u64, 3 u32, 1 u8
  void* cub = nullptr;
  std::size_t cub_bytes = 0;
  std::uint64_t* res = nullptr;
  std::uint64_t* h_res = nullptr;
  unsigned ncu = 0;              // the device's compute units (region sizing)
  // host images: device copy, pinned staging slabs for pageable sources, own stream
  std::uint8_t* d_img = nullptr;
  std::uint64_t cap_img = 0;
  std::uint8_t* slab[2] = {nullptr, nullptr};
  hipEvent_t slab_free[2] = {nullptr, nullptr};
  hipEvent_t landed[2] = {nullptr, nullptr};  // copy of a chunk done (copy stream -> compute stream)
  hipStream_t st = nullptr;   // copies of host images
  hipStream_t stc = nullptr;  // device work on host images (overlaps the copies)
  ~WalScratch() {
    if (st) (void)hipStreamSynchronize(st);
    if (stc) (void)hipStreamSynchronize(stc);
    for (int i = 0; i < 2; ++i)
      if (landed[i]) (void)hipEventDestroy(landed[i]);
    if (stc) (void)hipStreamDestroy(stc);
    (void)hipFree(d_img);
    for (int i = 0; i < 2; ++i) {
      (void)hipHostFree(slab[i]);
      if (slab_free[i]) (void)hipEventDestroy(slab_free[i]);
    }
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(regions);
    (void)hipFree(bigs);
    (void)hipFree(cub);
    (void)hipFree(res);
    (void)hipHostFree(h_res);
  }
};

std::mutex g_wal_mu;
WalScratch* g_wal[64] = {};

// What the calling thread's last WAL verify did (tkv_debug_wal_last).
thread_local std::uint64_t g_last[4] = {0, 0, 0, 0};  // passes, host walk needed, image copied, regions
// Region size forced by tkv_debug_wal_region (0: sized from the image and the device).
std::atomic<std::uint64_t> g_region_force{0};

#define WAL_HIP(call)                                                            \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e_)); \
  } while (0)

// About two regions per wave slot of the device (kRegWaves per CU), a power of two in
// [kRegionMin, kRegionMax].
std::uint64_t region_size(std::uint64_t size, unsigned ncu) {
  const std::uint64_t forced = g_region_force.load(std::memory_order_relaxed);
  if (forced) return forced;
  const std::uint64_t slots = std::max<std::uint64_t>(1, 2ull * ncu * kRegWaves);
  std::uint64_t rs = kRegionMin;
  while (rs < kRegionMax && 2 * rs * slots <= size) rs *= 2;
  return rs;
}

int grow_regions(WalScratch& s, std::uint64_t K) {
  if (K <= s.cap_regions) return TKV_OK;
  const std::uint64_t cap = std::max<std::uint64_t>(K, 2 * s.cap_regions);
  WAL_HIP(hipFree(s.regions));
  s.regions = nullptr;
  s.cap_regions = 0;
  WAL_HIP(hipMalloc(&s.regions, cap * (10 * 8 + 3 * 4 + 4)));
  s.cap_regions = cap;
  return TKV_OK;
}

int grow_big(WalScratch& s, std::uint64_t n) {
  if (n <= s.cap_big) return TKV_OK;
  const std::uint64_t cap = std::max<std::uint64_t>(n, 2 * s.cap_big);
  WAL_HIP(hipFree(s.bigs));
  s.bigs = nullptr;
  s.cap_big = 0;
  WAL_HIP(hipMalloc(&s.bigs, cap * (2 * 8 + 3 * 4 + 1)));
  s.cap_big = cap;
  return TKV_OK;
}

WalArgs carve(WalScratch& s, const std::uint8_t* w, std::uint64_t size, std::uint64_t RS, std::uint32_t K,
              const DeviceTables* tabs) {
  WalArgs a{};
  a.w = w;
  a.size = size;
  a.RS = RS;
  a.K = K;
  const std::uint64_t C = s.cap_regions;
  auto* p8 = static_cast<std::uint64_t*>(s.regions);
  std::uint64_t** u64s[] = {&a.S, &a.X, &a.spec_cnt, &a.first_loc, &a.first_pos, &a.entry, &a.cnt, &a.base, &a.Xe,
                            &a.bad_at};
  for (std::size_t i = 0; i < sizeof(u64s) / sizeof(u64s[0]); ++i) *u64s[i] = p8 + i * C;
  auto* p4 = reinterpret_cast<std::uint32_t*>(p8 + 10 * C);
  a.next = p4;
  a.Ja = p4 + C;
  a.Jb = p4 + 2 * C;
  auto* p1 = reinterpret_cast<std::uint8_t*>(p4 + 3 * C);
  a.broke = p1;
  a.on = p1 + C;
  a.Be = p1 + 2 * C;
  a.recheck = p1 + 3 * C;
  const std::uint64_t B = s.cap_big;
  a.cap_big = B;
  if (B) {
    auto* b8 = static_cast<std::uint64_t*>(s.bigs);
    a.big_off = b8;
    a.big_key = b8 + B;
    auto* b4 = reinterpret_cast<std::uint32_t*>(b8 + 2 * B);
    a.big_len = b4;
    a.big_crc = b4 + B;
    a.got = b4 + 2 * B;
    a.big_tag = reinterpret_cast<std::uint8_t*>(b4 + 3 * B);
  }
  a.tabs = tabs;
  a.res = s.res;
  return a;
}

unsigned blocks(std::uint64_t n, unsigned t) { return static_cast<unsigned>((n + t - 1) / t); }

// CRC batches of at most this many records (the irregular path's u32 block indices).
constexpr std::uint64_t kWalCrcChunk = std::uint64_t(1) << 31;

struct PassResult {
  std::uint64_t good = 0;  // records verified good from the pass's start
  std::uint64_t stop = 0;  // where decoding stopped (relative to the pass's start)
  bool corrupted = false;
  bool resume = false;     // the chain continues at `stop` (a true record start) beyond what was checked
  bool retry = false;      // the big list overflowed its scratch (now grown): run the pass again
};

// A pass over the image [w, w + size), which starts with a record (or is empty), in three parts:
// pass_begin (result words), pass_front over ranges of regions (the speculative walks; each range's
// bytes and the next kFrontMargin bytes must be resident), pass_tail.
int pass_begin(WalScratch& s, const std::uint8_t* w, std::uint64_t size, hipStream_t st, WalArgs* out) {
  const std::uint64_t RS = region_size(size, s.ncu);
  const std::uint32_t K = static_cast<std::uint32_t>((size + RS - 1) / RS);
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  if (int rc = grow_regions(s, K)) return rc;
  if (int rc = grow_big(s, std::max<std::uint64_t>(std::uint64_t(1) << 16, size >> 10))) return rc;
  WalArgs a = carve(s, w, size, RS, K, tabs);
  for (int i = 0; i < 8; ++i) s.h_res[i] = 0;
  s.h_res[0] = kNone;
  s.h_res[1] = size;
  s.h_res[3] = kNone;
  WAL_HIP(hipMemcpyAsync(s.res, s.h_res, 8 * sizeof(std::uint64_t), hipMemcpyHostToDevice, st));
  *out = a;
  return TKV_OK;
}

// Bytes past a region that its walk may read: the halo of its last chunk and the payloads of at
// most kWalFold bytes of its last records (header, 16-byte granules).
constexpr std::uint64_t kFrontTail = 2 * kChunk + kWalFold + 64;

void pass_front(const WalArgs& a, std::uint64_t k_lo, std::uint64_t k_hi, hipStream_t st) {
  if (k_hi <= k_lo) return;
  hipLaunchKernelGGL(wal_region, dim3(blocks(k_hi - k_lo, kRegWaves)), dim3(kRegThreads), 0, st, a, k_lo, k_hi, 0);
}

int pass_tail(WalScratch& s, WalArgs a, hipStream_t st, PassResult* r) {
  const std::uint8_t* w = a.w;
  const std::uint64_t size = a.size;
  const std::uint32_t K = a.K;
  // 3: the regions on the true chain and their entries
  hipLaunchKernelGGL(wal_jump_init, dim3(blocks(K, 256)), dim3(256), 0, st, a);
  std::uint32_t* J = a.Ja;
  std::uint32_t* J2 = a.Jb;
  for (std::uint64_t reach = 1; reach < K; reach <<= 2) {
    hipLaunchKernelGGL(wal_jump, dim3(blocks(K, 256)), dim3(256), 0, st, J, J2, a.on, K);
    std::swap(J, J2);
  }
  hipLaunchKernelGGL(wal_link, dim3(blocks(K, 256)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(wal_count, dim3(blocks(K, 256)), dim3(256), 0, st, a);
  // regions entered off their speculative start, walked again from the entry (most workgroups find
  // no such region among their eight and end before filling their tables)
  hipLaunchKernelGGL(wal_region, dim3(blocks(K, kRegWaves)), dim3(kRegThreads), 0, st, a, 0, K, 1);
  hipLaunchKernelGGL(wal_count_exact, dim3(blocks(K, 256)), dim3(256), 0, st, a);
  WAL_HIP(hipGetLastError());
  WAL_HIP(hipMemcpyAsync(s.h_res, s.res, 8 * sizeof(std::uint64_t), hipMemcpyDeviceToHost, st));
  WAL_HIP(hipStreamSynchronize(st));
  if (s.h_res[6] > s.cap_big) {  // the big list did not fit: grow it and run the pass again
    if (int rc = grow_big(s, s.h_res[6])) return rc;
    r->retry = true;
    return TKV_OK;
  }
  const std::uint64_t kstar = s.h_res[0];
  std::uint64_t chain_end = s.h_res[1];
  bool broke = s.h_res[2] != 0;
  const std::uint64_t n_big = s.h_res[6];
  const bool partial = kstar < K;
  if (partial) {
    hipLaunchKernelGGL(wal_trim, dim3(blocks(K, 256)), dim3(256), 0, st, a, kstar);
    std::uint8_t be = 0;
    WAL_HIP(hipMemcpyAsync(s.h_res + 1, a.Xe + kstar, 8, hipMemcpyDeviceToHost, st));
    WAL_HIP(hipMemcpyAsync(&be, a.Be + kstar, 1, hipMemcpyDeviceToHost, st));
    WAL_HIP(hipStreamSynchronize(st));
    chain_end = s.h_res[1];
    broke = be == 1;
  }
  // 4: record numbering, the first bad record (regions, then the CRC batch of the big ones)
  std::size_t need = 0;
  WAL_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need, a.cnt, a.base, K, st));
  if (need > s.cub_bytes) {
    WAL_HIP(hipStreamSynchronize(st));
    WAL_HIP(hipFree(s.cub));
    s.cub = nullptr;
    s.cub_bytes = 0;
    WAL_HIP(hipMalloc(&s.cub, need));
    s.cub_bytes = need;
  }
  WAL_HIP(hipcub::DeviceScan::ExclusiveSum(s.cub, need, a.cnt, a.base, K, st));
  const std::uint64_t ks = partial ? kstar : K;
  hipLaunchKernelGGL(wal_gather, dim3(blocks(K, 256)), dim3(256), 0, st, a, ks);
  WAL_HIP(hipGetLastError());
  for (std::uint64_t i = 0; i < n_big; i += kWalCrcChunk) {
    const std::uint64_t m = std::min(kWalCrcChunk, n_big - i);
    if (int rc = batch_device_impl(kAlgoCrc32, w, a.big_off + i, a.big_len + i, nullptr, a.got + i, m, st)) return rc;
  }
  if (n_big) hipLaunchKernelGGL(wal_check_big, dim3(blocks(n_big, 256)), dim3(256), 0, st, a, n_big, ks);
  hipLaunchKernelGGL(wal_bad_pos, dim3(blocks(std::max<std::uint64_t>(K, n_big), 256)), dim3(256), 0, st, a, n_big,
                     ks);
  WAL_HIP(hipGetLastError());
  WAL_HIP(hipMemcpyAsync(s.h_res + 3, s.res + 3, 2 * sizeof(std::uint64_t), hipMemcpyDeviceToHost, st));
  WAL_HIP(hipMemcpyAsync(s.h_res + 7, a.base + (K - 1), 8, hipMemcpyDeviceToHost, st));
  WAL_HIP(hipMemcpyAsync(s.h_res + 6, a.cnt + (K - 1), 8, hipMemcpyDeviceToHost, st));
  WAL_HIP(hipStreamSynchronize(st));
  const std::uint64_t n = s.h_res[7] + s.h_res[6];  // good records counted
  const bool bad = s.h_res[3] != kNone;
  r->good = bad ? std::min(s.h_res[3], n) : n;
  r->corrupted = bad || broke;
  r->stop = bad ? s.h_res[4] : chain_end;
  r->resume = !r->corrupted && partial && chain_end < size;
  return TKV_OK;
}

// A whole pass over a resident image.
int wal_pass(WalScratch& s, const std::uint8_t* w, std::uint64_t size, hipStream_t st, PassResult* r) {
  for (int attempt = 0; attempt < 3; ++attempt) {
    WalArgs a;
    if (int rc = pass_begin(s, w, size, st, &a)) return rc;
    pass_front(a, 0, a.K, st);
    *r = PassResult{};
    if (int rc = pass_tail(s, a, st, r)) return rc;
    if (!r->retry) return TKV_OK;
  }
  return set_error(TKV_IO_ERROR, "WAL verify: big-record list kept overflowing");
}

// The calling thread's device's scratch (created on first use, with its result words).
int scratch(WalScratch** out) {
  int dev = 0;
  WAL_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return set_error(TKV_INVALID_ARGUMENT, "device index out of range");
  WalScratch* sp;
  {
    std::lock_guard<std::mutex> lk(g_wal_mu);
    if (!g_wal[dev]) g_wal[dev] = new WalScratch();
    sp = g_wal[dev];
  }
  std::lock_guard<std::mutex> lk(sp->mu);
  if (!sp->res) {
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->res), 8 * sizeof(std::uint64_t)));
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_res), 8 * sizeof(std::uint64_t), hipHostMallocDefault));
    WAL_HIP(hipStreamCreateWithFlags(&sp->st, hipStreamNonBlocking));
    WAL_HIP(hipStreamCreateWithFlags(&sp->stc, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) WAL_HIP(hipEventCreateWithFlags(&sp->landed[i], hipEventDisableTiming));
    WAL_HIP(hipDeviceGetAttribute(reinterpret_cast<int*>(&sp->ncu), hipDeviceAttributeMultiprocessorCount, dev));
  }
  *out = sp;
  return TKV_OK;
}

int verify_locked(WalScratch& s, const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                  std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk,
                  const PassResult* first_pass = nullptr) {
  // Each pass checks the true chain at least through its first region; a pass that stops short of
  // the end without a verdict resumes at a true record start. Adversarial images that keep the
  // speculation wrong go to the exact host walk after kMaxPasses.
  constexpr int kMaxPasses = 8;
  std::uint64_t start = 0, good = 0;
  g_last[0] = g_last[1] = 0;
  {
    const std::uint64_t RS = region_size(size, s.ncu);
    g_last[3] = (size + RS - 1) / RS;
  }
  for (int pass = 0; pass < kMaxPasses; ++pass) {
    PassResult r;
    g_last[0] = static_cast<std::uint64_t>(pass) + 1;
    if (pass == 0 && first_pass && !first_pass->retry) r = *first_pass;
    else if (int rc = wal_pass(s, d_wal + start, size - start, st, &r)) return rc;
    good += r.good;
    if (!r.resume) {
      *n_good = good;
      *stop_offset = start + r.stop;
      return r.corrupted ? set_error(TKV_CORRUPTED, "corrupted WAL record") : TKV_OK;
    }
    start += r.stop;
  }
  *needs_host_walk = true;
  g_last[1] = 1;
  return TKV_OK;
}

// memcpy of a large range into pinned staging on several host threads.
void stage_copy(std::uint8_t* dst, const std::uint8_t* src, std::uint64_t n) {
  const unsigned nt = n >= (std::uint64_t(16) << 20) ? 8u : 1u;
  if (nt == 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=] {
      const std::uint64_t a = n * t / nt, e = n * (t + 1) / nt;
      std::memcpy(dst + a, src + a, e - a);
    });
  for (auto& t : th) t.join();
}

constexpr std::uint64_t kStageSlab = std::uint64_t(64) << 20;
constexpr std::uint64_t kMaxImage = std::uint64_t(1) << 46;  // regions stay below 2^32

}  // namespace

int wal_verify_device_impl(const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                           std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk) {
  *needs_host_walk = false;
  *n_good = 0;
  *stop_offset = 0;
  g_last[0] = g_last[1] = g_last[2] = g_last[3] = 0;
  if (size == 0) return TKV_OK;
  if (size >= kMaxImage) return set_error(TKV_INVALID_ARGUMENT, "WAL image too large for the device walk");
  WalScratch* sp = nullptr;
  if (int rc = scratch(&sp)) return rc;
  WalScratch& s = *sp;
  std::lock_guard<std::mutex> lk(s.mu);
  return verify_locked(s, d_wal, size, n_good, stop_offset, st, needs_host_walk);
}

int wal_verify_host_image_body(WalScratch& s, const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk);

// Device copies of host images above this size are freed after the verify (a multi-GiB recovery must
// not hold that much HBM for the rest of the process); smaller ones are kept for the next call.
constexpr std::uint64_t kKeepImage = std::uint64_t(1) << 30;

int wal_verify_host_image_impl(const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk) {
  *needs_host_walk = false;
  *n_good = 0;
  *stop_offset = 0;
  g_last[0] = g_last[1] = g_last[2] = g_last[3] = 0;
  if (size == 0) return TKV_OK;
  if (size >= kMaxImage) {
    *needs_host_walk = true;
    return TKV_OK;
  }
  WalScratch* sp = nullptr;
  if (int rc = scratch(&sp)) return rc;
  WalScratch& s = *sp;
  std::lock_guard<std::mutex> lk(s.mu);
  const int rc = wal_verify_host_image_body(s, h_wal, size, n_good, stop_offset, needs_host_walk);
  // Whatever happened, no copy that reads the caller's buffer or writes d_img is left in flight.
  const hipError_t e0 = hipStreamSynchronize(s.st), e1 = hipStreamSynchronize(s.stc);
  if (s.cap_img > kKeepImage) {
    (void)hipFree(s.d_img);
    s.d_img = nullptr;
    s.cap_img = 0;
  }
  if (rc == TKV_OK && (e0 != hipSuccess || e1 != hipSuccess))
    return set_error(TKV_IO_ERROR, hipGetErrorString(e0 != hipSuccess ? e0 : e1));
  return rc;
}

int wal_verify_host_image_body(WalScratch& s, const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk) {
  g_last[2] = 1;
  if (size > s.cap_img) {
    (void)hipStreamSynchronize(s.st);
    (void)hipFree(s.d_img);
    s.d_img = nullptr;
    s.cap_img = 0;
    if (hipMalloc(reinterpret_cast<void**>(&s.d_img), size) != hipSuccess) {
      (void)hipGetLastError();  // the image does not fit the device: exact host walk instead
      *needs_host_walk = true;
      g_last[1] = 1;
      return TKV_OK;
    }
    s.cap_img = size;
  }
  hipPointerAttribute_t attr;
  const bool pinned = hipPointerGetAttributes(&attr, h_wal) == hipSuccess && attr.type == hipMemoryTypeHost;
  if (!pinned) (void)hipGetLastError();
  if (!pinned) {
    for (int i = 0; i < 2; ++i) {
      if (!s.slab[i]) {
        WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.slab[i]), kStageSlab, hipHostMallocDefault));
        WAL_HIP(hipEventCreateWithFlags(&s.slab_free[i], hipEventDisableTiming));
      }
    }
  }
  // The image goes over in chunks on the copy stream (pageable sources through two pinned slabs that
  // host threads fill while the copy engine drains the other). As each chunk lands, the compute
  // stream walks the regions before it whose bytes are all resident (regions ending at least
  // kFrontTail bytes before the end of what has landed), so only the last chunk's regions and the
  // stitching remain once the copy is done.
  WalArgs a;
  if (int rc = pass_begin(s, s.d_img, size, s.stc, &a)) return rc;
  std::uint64_t fronted = 0;
  int k = 0;
  for (std::uint64_t off = 0; off < size; off += kStageSlab, k ^= 1) {
    const std::uint64_t m = std::min(kStageSlab, size - off);
    if (pinned) {
      WAL_HIP(hipMemcpyAsync(s.d_img + off, h_wal + off, m, hipMemcpyHostToDevice, s.st));
    } else {
      WAL_HIP(hipEventSynchronize(s.slab_free[k]));
      stage_copy(s.slab[k], h_wal + off, m);
      WAL_HIP(hipMemcpyAsync(s.d_img + off, s.slab[k], m, hipMemcpyHostToDevice, s.st));
      WAL_HIP(hipEventRecord(s.slab_free[k], s.st));
    }
    WAL_HIP(hipEventRecord(s.landed[k], s.st));
    WAL_HIP(hipStreamWaitEvent(s.stc, s.landed[k], 0));
    const bool last = off + m >= size;
    const std::uint64_t k_hi = last ? a.K : (off + m > kFrontTail ? (off + m - kFrontTail) / a.RS : 0);
    if (k_hi > fronted) {
      pass_front(a, fronted, k_hi, s.stc);
      fronted = k_hi;
    }
  }
  WAL_HIP(hipGetLastError());
  PassResult r;
  g_last[0] = 1;
  if (int rc = pass_tail(s, a, s.stc, &r)) return rc;
  return verify_locked(s, s.d_img, size, n_good, stop_offset, s.stc, needs_host_walk, &r);
}

}  // namespace tkv

extern "C" void tkv_debug_wal_last(uint64_t out[4]) {
  for (int i = 0; i < 4; ++i) out[i] = tkv::g_last[i];
}

extern "C" uint64_t tkv_debug_wal_region(uint64_t bytes) {
  // rounded up to whole chunks; 0 restores the automatic size
  const std::uint64_t rs = bytes ? (bytes + tkv::kChunk - 1) / tkv::kChunk * tkv::kChunk : 0;
  return tkv::g_region_force.exchange(rs);
}
