// WAL recovery verify on the device: the record_len chain walk of
// wal_entry::decode (/root/reference/src/engine/wal.cpp:63-130) over a WAL image resident in HBM,
// the CRC check of every record (wal.cpp:89-96) and the key/value bounds check (wal.cpp:118-121),
// ending in the first corruption - without walking the chain on the host.
//
// The record chain is a linked list through the image (record i+1 starts 8 + record_len bytes after
// record i), so it is walked speculatively in parallel and stitched exactly:
//  1. wal_scan_head: the image is cut into pieces of kWalPiece bytes, and the first plausible header
//     of every piece (one the reference encoder could have written, wal.cpp:19-61), searched from
//     the piece's front, becomes its speculative start S_k; piece 0 starts at 0.
//  2. wal_spec: one lane per piece walks the chain from S_k over the records that start in the
//     piece (X_k = the first record start at or past the piece's end, or the header that broke),
//     and checks them as it goes: key/value bounds, and the CRC of every payload of at most
//     kWalLaneMax bytes folded by the lane itself (slicing-by-4 lookups into the engine's tables in
//     LDS, the payload zero-padded in front to whole dwords). Larger records (at most two start in a
//     piece) wait in the piece's slots for one CRC batch through the engine's irregular path.
//  3. wal_jump: next(k) = the piece holding X_k. The true chain visits the pieces 0, next(0),
//     next(next(0)), ...; pointer jumping (x4 per round) marks exactly those pieces in
//     log4(#pieces) rounds, and wal_link hands every on-path piece its entry E = X of its predecessor.
//  4. wal_count: an on-path piece whose entry is its speculative start keeps its speculative walk
//     and checks; otherwise it walks again from E (and wal_recheck checks it again). Its speculative
//     exit was right when the exact walk leaves at the same X (and breaks, or not, the same way).
//     Entries are exact up to and including the first piece k* whose speculative exit was wrong (a
//     corrupted record_len, or a fake header in a key or value that led the speculation astray):
//     later pieces are dropped, and when no record up to k*'s exact exit fails, the next pass
//     resumes there (a true record start) as a new image.
//  5. one exclusive scan numbers the records; wal_gather turns each piece's first failing record
//     into a record index and moves the big-record slots into a dense list for the CRC batch;
//     wal_check_big checks those. The first bad record is an atomic minimum of record indices.
// Every step reads the image in HBM; the host only reads back a few counters.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
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

constexpr std::uint64_t kWalPiece = 2048;     // bytes of image per speculative walker
constexpr std::uint64_t kWalMeta = 26;        // wal.hpp:21-27 kMetadataSize
constexpr std::uint32_t kWalLaneMax = 1024;   // payloads up to this size are checked by their lane
constexpr std::uint64_t kNone = ~0ull;
constexpr unsigned kScanThreads = 256;        // wal_scan_head: 8 lanes per piece, 8 pieces per wave
constexpr unsigned kCheckThreads = 1024;      // wal_spec/wal_recheck
// A/B builds only (TKV_AB_WAL16=1): wal_spec/wal_recheck on the 64 KiB 16-replica table image with two
// workgroups per CU (32 waves, at most 64 VGPRs) where the 128 KiB image allows one: the walk is
// latency-bound (8 or 4 waves per CU instead of 16 were 15 % and 66 % slower).
#ifndef TKV_AB_WAL16
#define TKV_AB_WAL16 0
#endif
constexpr unsigned kCheckWgPerCu = TKV_AB_WAL16 ? 2 : 1;
constexpr unsigned kHres = 16;                // words of the pinned result block

struct WalArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  std::uint32_t K;           // pieces
  // per piece
  std::uint64_t* S;          // speculative start (kNone: no plausible header)
  std::uint64_t* X;          // exit of its speculative chain, or the start of the header that broke it
  std::uint64_t* spec_cnt;   // records of the speculative chain: (all << 32) | (larger than kWalLaneMax)
  std::uint32_t* next;       // piece of X (K: end of image, broken chain or no start)
  std::uint8_t* broke;       // the speculative chain hit a header that does not fit (at X)
  std::uint64_t* first_loc;  // first failing record of the piece's checked walk (local index, kNone)
  std::uint64_t* first_pos;  // and its start
  std::uint64_t* slot_off;   // two slots per piece: records larger than kWalLaneMax (payload offset,
  std::uint32_t* slot_len;   //   length, stored CRC, local index)
  std::uint32_t* slot_crc;
  std::uint32_t* slot_loc;
  std::uint32_t* Ja;         // pointer-jumping tables
  std::uint32_t* Jb;
  std::uint8_t* on;          // piece is on the true chain
  std::uint8_t* recheck;     // entered off its speculative start: walked and checked again
  std::uint64_t* entry;      // true entry point of an on-path piece
  std::uint64_t* cnt;        // records of an on-path piece from its entry, packed as spec_cnt
  std::uint64_t* base;       // exclusive scan of cnt: first record index (high), first big record (low)
  std::uint64_t* Xe;         // exit of its exact walk from the entry (or the header that broke it)
  std::uint8_t* Be;          // the exact walk broke
  std::uint64_t* bad_at;     // index of the piece's first failing record
  // per big record (dense, in record order)
  std::uint64_t* big_off;
  std::uint32_t* big_len;
  std::uint64_t* big_idx;
  std::uint32_t* big_crc;
  std::uint32_t* got;        // engine CRC of each big payload (finalized)
  const std::uint32_t* inj;  // inj[L] = Shift_L(0xFFFFFFFF), L <= kWalLaneMax: the init term
  const DeviceTables* tabs;
  std::uint64_t* res;        // [0] first piece with a wrong speculative exit, [1] chain end and
                             // [2] chain broke (from the path's last piece), [3] first bad record,
                             // [4] its start, [5] pieces re-checked
};

// Little-endian u32 at byte p of the image, p + 4 <= size: dword loads aligned to the absolute
// address, realigned with v_alignbyte. The second dword is read only when it starts inside the
// image, so no load touches a dword past the image's last byte (nor a page past its allocation);
// the first may start up to 3 bytes before w, inside the same aligned dword as w itself.
__device__ __forceinline__ std::uint32_t ld32(const std::uint8_t* w, std::uint64_t p, std::uint64_t size) {
  const std::uintptr_t q = reinterpret_cast<std::uintptr_t>(w) + p;
  const std::uintptr_t a = q & ~static_cast<std::uintptr_t>(3);
  const std::uintptr_t end = reinterpret_cast<std::uintptr_t>(w) + size;
  const std::uint32_t lo = *reinterpret_cast<const std::uint32_t*>(a);
  const std::uint32_t hi = (q & 3u) && a + 4 < end ? *reinterpret_cast<const std::uint32_t*>(a + 4) : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, static_cast<std::uint32_t>(q & 3u));
}

__device__ __forceinline__ std::uint64_t gid() {
  return blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
}

__device__ __forceinline__ std::uint32_t le1_bytes4(std::uint32_t d) {
  // 4-bit mask: bit i set iff byte i of d is 0 or 1
  const std::uint32_t x = d & 0xFEFEFEFEu;
  const std::uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu) & 0x80808080u;
  return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// 1. The first plausible header of every piece, searched from the piece's front with an early exit.
// A group of 8 lanes owns one piece and tests 224 positions per step. Lanes 0-6 each hold 32 bytes
// (two 16-byte loads) and report their 32 positions; lane 7 only lends its bytes. A header at p has
// its op and tombstone bytes (p+8, p+17) at 0 or 1 (wal.cpp:30-52): each lane marks which of its
// bytes are 0 or 1 with byte-parallel arithmetic, takes its right neighbour's marks by a cross-lane
// shift and so tests all 32 positions at once; only positions that pass get the full check
// (record_len = 18 + klen + vlen, fitting the image; re-read through L1). The group moves on only
// while no position of its piece passed. In a WAL of small records the first step finds the
// header, so about 256 bytes of every 2 KiB piece are read; a piece inside a large value is scanned
// whole. The earlier kernel scanned every position of the image in one coalesced pass: 1.11 ->
// 0.85 ms on 1 GiB of 59-byte records, Zipf image unchanged (profiles/r2/wal_head_scan/). Each
// piece has one owner, so the result is a plain store (S is preset to kNone; piece 0 starts at 0).
constexpr unsigned kHeadLanes = 8;                   // lanes per piece
constexpr unsigned kHeadChunks = 2 * (kHeadLanes - 1);  // 16-byte chunks reported per group and step
__global__ __launch_bounds__(kScanThreads) void wal_scan_head(WalArgs a, std::uint64_t k_lo, std::uint64_t k_hi) {
  const std::uintptr_t w0 = reinterpret_cast<std::uintptr_t>(a.w);
  const std::uintptr_t al = w0 & ~static_cast<std::uintptr_t>(15);
  const std::uint64_t off0 = w0 - al;
  const std::uintptr_t end = w0 + a.size;
  const std::uint32_t lane = threadIdx.x & 63u, g = lane / kHeadLanes, i = lane % kHeadLanes;
  const std::uint64_t k = k_lo + (gid() >> 6) * (64 / kHeadLanes) + g;
  const std::uint64_t ps = k * kWalPiece;
  // positions with a whole header inside the image and inside the piece: [ps, pe)
  const std::uint64_t pe = a.size < kWalMeta ? 0 : std::min<std::uint64_t>(ps + kWalPiece, a.size - kWalMeta + 1);
  bool active = k < k_hi && k != 0 && ps < pe;  // uniform within a group
  const std::uint64_t tg = (ps + off0) / 16;   // the chunk holding ps
  std::uint64_t found_at = kNone;
  for (std::uint64_t step = 0; __ballot(active) != 0; ++step) {
    const std::uint64_t t = tg + step * kHeadChunks + 2 * i;
    const std::uintptr_t c0 = al + 16 * t;
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
    if (active && c0 < end) v0 = *reinterpret_cast<const uint4*>(c0);
    if (active && c0 + 16 < end) v1 = *reinterpret_cast<const uint4*>(c0 + 16);
    const std::uint32_t f = le1_bytes4(v0.x) | le1_bytes4(v0.y) << 4 | le1_bytes4(v0.z) << 8 | le1_bytes4(v0.w) << 12 |
                            le1_bytes4(v1.x) << 16 | le1_bytes4(v1.y) << 20 | le1_bytes4(v1.z) << 24 |
                            le1_bytes4(v1.w) << 28;
    const std::uint32_t f1 = static_cast<std::uint32_t>(__shfl_down(static_cast<int>(f), 1, 64));
    const std::uint64_t F = f | static_cast<std::uint64_t>(f1) << 32;
    std::uint32_t cand = static_cast<std::uint32_t>((F >> 8) & (F >> 17));  // bytes j+8, j+17 are 0/1
    const std::int64_t p0 = static_cast<std::int64_t>(16 * t) - static_cast<std::int64_t>(off0);
    const std::int64_t lo = static_cast<std::int64_t>(ps) - p0, hi = static_cast<std::int64_t>(pe) - 1 - p0;
    if (!active || i + 1 == kHeadLanes || hi < 0 || lo > 31) {
      cand = 0;
    } else {
      const std::uint32_t jlo = lo < 0 ? 0u : static_cast<std::uint32_t>(lo);
      const std::uint32_t jhi = hi > 31 ? 31u : static_cast<std::uint32_t>(hi);
      cand &= (jhi == 31u ? 0xFFFFFFFFu : (2u << jhi) - 1u) & ~((1u << jlo) - 1u);
    }
    std::uint64_t best = kNone;
    while (cand) {
      const int j = __builtin_ctz(cand);
      const std::uint64_t p = static_cast<std::uint64_t>(p0 + j);
      const std::uint64_t rlen = ld32(a.w, p, a.size), klen = ld32(a.w, p + 18, a.size), vlen = ld32(a.w, p + 22, a.size);
      if (rlen == 18u + klen + vlen && rlen + 8 <= a.size - p) {
        best = p;
        break;
      }
      cand &= cand - 1;
    }
    // positions grow with the lane index inside a group: its first header is its lowest finder's
    const std::uint64_t bal = __ballot(best != kNone);
    const std::uint32_t gb = static_cast<std::uint32_t>(bal >> (g * kHeadLanes)) & ((1u << (kHeadLanes - 1)) - 1u);
    const std::uint32_t src = g * kHeadLanes + (gb ? static_cast<std::uint32_t>(__builtin_ctz(gb)) : 0u);
    const std::uint64_t first = __shfl(best, static_cast<int>(src), 64);
    const std::int64_t next_p0 = static_cast<std::int64_t>(16 * (tg + (step + 1) * kHeadChunks)) - static_cast<std::int64_t>(off0);
    if (active && gb) {
      found_at = first;
      active = false;
    } else if (next_p0 >= static_cast<std::int64_t>(pe)) {
      active = false;
    }
  }
  if (i == 0 && found_at != kNone) a.S[k] = found_at;
}

// One slicing-by-4 step of the lane's register over dword w (the engine's replicated LDS tables).
__device__ __forceinline__ void wal_fold(const std::uint32_t* lds, dev::Reg& r, std::uint32_t w, const dev::LaneConst& kc) {
  dev::slice4(lds, r, w, kc);
}

// CRC-32 (finalized) of the payload [q, q + L) in image bytes, L <= kWalLaneMax, folded by this
// lane alone with slicing-by-4 lookups into the LDS tables; the init register enters as
// inj[L] = Shift_L(0xFFFFFFFF) (crc_s(D) = Shift_|D|(s) ^ crc_0(D)). The payload is read as the
// 16-byte aligned granules that hold it, two at a time with the next two in flight: the bytes in
// front of the payload in its first granule are zeroed (leading zeros leave an init-0 register at
// 0), whole dwords are folded, and the last 0-3 bytes take Sarwate steps. A granule never crosses a
// page, so reading the whole of one that holds payload bytes cannot fault. Each lane reads its own
// part of the image, so a CU's lanes touch far more lines than its L1 holds; 16-byte reads take a
// quarter of the requests of the dword reads they replace (profiles/r2/wal_pmc/).
__device__ __forceinline__ std::uint32_t lane_crc(const std::uint32_t* lds, const dev::LaneConst& kc, const WalArgs& a,
                                                  std::uint64_t q, std::uint32_t L) {
  if (L == 0) return 0u;  // crc32 of nothing
  const std::uintptr_t s = reinterpret_cast<std::uintptr_t>(a.w) + q;
  const std::uintptr_t g0 = s & ~static_cast<std::uintptr_t>(15);
  const std::uint32_t h = static_cast<std::uint32_t>(s - g0);  // bytes in front, zeroed
  const std::uint32_t span = h + L;
  const std::uint32_t nd = span >> 2, tb = span & 3u;          // whole dwords, then tail bytes
  const std::uint32_t glast = (span - 1u) >> 4;                 // last granule with payload bytes
  auto G = [&](std::uint32_t m) { return *reinterpret_cast<const uint4*>(g0 + 16u * (m < glast ? m : glast)); };
  auto mask = [&](std::uint32_t k) -> std::uint32_t {  // bytes of dword k at or after the payload start
    const std::int32_t lead = static_cast<std::int32_t>(h) - static_cast<std::int32_t>(4u * k);
    return lead <= 0 ? 0xFFFFFFFFu : (lead >= 4 ? 0u : 0xFFFFFFFFu << (8 * lead));
  };
  dev::Reg r{0, 0};
  uint4 c0 = G(0), c1 = G(1);
  // Granule pairs [m, m + 2): the first one masks the head dwords, the ones wholly inside the
  // payload fold unguarded, the last one (<= 8 dwords left) is guarded and takes the tail bytes.
  auto pair = [&](std::uint32_t m, const uint4& x0, const uint4& x1, bool head, bool guarded) {
    const std::uint32_t d[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (std::uint32_t i = 0; i < 8; ++i) {
      const std::uint32_t k = 4u * m + i;
      const std::uint32_t w = head ? d[i] & mask(k) : d[i];
      if (!guarded || k < nd) {
        wal_fold(lds, r, w, kc);
      } else if (k == nd && tb) {  // the last 1-3 bytes
        std::uint32_t x = r.value(), b = w;
        for (std::uint32_t t = 0; t < tb; ++t, b >>= 8) x = (x >> 8) ^ dev::lds_at(lds, (((x ^ b) & 0xFFu) << 8) | kc.L0);
        r = dev::Reg{x, 0};
      }
    }
  };
  std::uint32_t m = 0;
  for (; 4u * m + 8u <= nd; m += 2) {  // pairs whose 8 dwords are all whole payload dwords
    const uint4 n0 = G(m + 2), n1 = G(m + 3);  // the next two granules, in flight
    if (m == 0) pair(0, c0, c1, true, false);
    else pair(m, c0, c1, false, false);
    c0 = n0;
    c1 = n1;
  }
  pair(m, c0, c1, m == 0, true);  // the last 0-7 whole dwords and the tail bytes
  return r.value() ^ a.inj[L] ^ 0xFFFFFFFFu;
}

// Slicing tables into LDS (the row kernels' lane-shift tables are not needed here).
__device__ __forceinline__ void fill_slices(const DeviceTables* tabs, std::uint32_t* lds) {
  if constexpr (TKV_AB_WAL16) {
    dev::fill_lds_slicing16(tabs, lds);
  } else {
    for (std::uint32_t u = threadIdx.x; u < 1024u; u += blockDim.x) {
      const std::uint32_t pair = u >> 9, e = (u >> 1) & 255u, tt = u & 1u;
      const std::uint32_t v = tabs->slice[2 * pair + tt][e];
      uint4* dst = reinterpret_cast<uint4*>(lds + pair * 16384u + e * 64u + tt * 32u);
#pragma unroll
      for (std::uint32_t k = 0; k < 8u; ++k) dst[(k + u) & 7u] = make_uint4(v, v, v, v);
    }
  }
  __syncthreads();
}

// The header fields of the record at p (p + 26 <= size): record_len, the stored CRC, key and value
// lengths (wal.cpp:14-18). header_load issues two dword-aligned 16-byte loads over [p & ~3, + 32),
// so the walk can put the next record's header in flight before it folds the current payload;
// header_fields realigns the fields in registers. Within 32 bytes of the image's end (where those
// loads could cross into the next page) nothing is loaded and the fields are read as dwords.
struct HdrRaw {
  uint4 u, v;
};
__device__ __forceinline__ bool header_window_ok(const WalArgs& a, std::uint64_t p) {
  const std::uintptr_t b = (reinterpret_cast<std::uintptr_t>(a.w) + p) & ~static_cast<std::uintptr_t>(3);
  return b + 32 <= reinterpret_cast<std::uintptr_t>(a.w) + a.size;
}
__device__ __forceinline__ HdrRaw header_load(const WalArgs& a, std::uint64_t p) {
  HdrRaw h{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  if (header_window_ok(a, p)) {
    const std::uintptr_t b = (reinterpret_cast<std::uintptr_t>(a.w) + p) & ~static_cast<std::uintptr_t>(3);
    h.u = *reinterpret_cast<const uint4*>(b);
    h.v = *reinterpret_cast<const uint4*>(b + 16);
  }
  return h;
}
__device__ __forceinline__ void header_fields(const WalArgs& a, std::uint64_t p, const HdrRaw& h, std::uint32_t* rlen,
                                              std::uint32_t* stored, std::uint64_t* klen, std::uint64_t* vlen) {
  if (!header_window_ok(a, p)) {
    *rlen = ld32(a.w, p, a.size);
    *stored = ld32(a.w, p + 4, a.size);
    *klen = ld32(a.w, p + 18, a.size);
    *vlen = ld32(a.w, p + 22, a.size);
    return;
  }
  const std::uint32_t t = static_cast<std::uint32_t>((reinterpret_cast<std::uintptr_t>(a.w) + p) & 3u);
  const std::uint32_t d[8] = {h.u.x, h.u.y, h.u.z, h.u.w, h.v.x, h.v.y, h.v.z, h.v.w};
  auto at = [&](std::uint32_t lo, std::uint32_t hi) { return t ? __builtin_amdgcn_alignbyte(hi, lo, t) : lo; };
  *rlen = at(d[0], d[1]);
  *stored = at(d[1], d[2]);
  // bytes p+18.. and p+22.. start in dword (t + 18) / 4 = 4 or 5 and (t + 22) / 4 = 5 or 6 of the
  // window, at byte (t + 2) & 3 of it
  const bool up = t >= 2u;
  const std::uint32_t o = (t + 2u) & 3u;
  auto at2 = [&](std::uint32_t lo, std::uint32_t hi) { return o ? __builtin_amdgcn_alignbyte(hi, lo, o) : lo; };
  *klen = up ? at2(d[5], d[6]) : at2(d[4], d[5]);
  *vlen = up ? at2(d[6], d[7]) : at2(d[5], d[6]);
}

// Walk piece k from `start` over the records that start in the piece (wal.cpp:63-87: header size,
// then record_len against what is left) and check each one: key/value bounds (wal.cpp:118-121) and,
// for payloads up to kWalLaneMax bytes, the CRC (wal.cpp:89-96) in this lane. Larger records (at most
// two start in a piece) are kept in the piece's two slots for the CRC batch. Writes the piece's exit,
// break, counts, first failing record (local index) and slots.
__device__ __forceinline__ void walk_check(const std::uint32_t* lds, const dev::LaneConst& kc, const WalArgs& a,
                                           std::uint64_t k, std::uint64_t start, std::uint64_t* exit_out,
                                           std::uint8_t* broke_out, std::uint64_t* cnt_out) {
  const std::uint64_t limit = (k + 1) * kWalPiece < a.size ? (k + 1) * kWalPiece : a.size;
  std::uint64_t p = start, n_all = 0, n_big = 0, first = kNone, first_pos = 0;
  bool bad_hdr = false;
  HdrRaw h = header_load(a, p);
  while (p < limit) {
    if (a.size - p < kWalMeta) {
      bad_hdr = true;
      break;
    }
    std::uint32_t rlen, stored;
    std::uint64_t klen, vlen;
    header_fields(a, p, h, &rlen, &stored, &klen, &vlen);
    if (static_cast<std::uint64_t>(rlen) + 8 > a.size - p) {
      bad_hdr = true;
      break;
    }
    const std::uint64_t np = p + 8 + static_cast<std::uint64_t>(rlen);
    if (np < limit && a.size - np >= kWalMeta) h = header_load(a, np);  // next header in flight during the fold
    bool bad = kWalMeta + klen + vlen > 8ull + rlen;
    if (rlen <= kWalLaneMax) {
      bad = bad || lane_crc(lds, kc, a, p + 8, rlen) != stored;
    } else {
      const std::uint64_t sl = 2 * k + (n_big & 1u);
      a.slot_off[sl] = p + 8;
      a.slot_len[sl] = rlen;
      a.slot_crc[sl] = stored;
      a.slot_loc[sl] = static_cast<std::uint32_t>(n_all);
      ++n_big;
    }
    if (bad && first == kNone) {
      first = n_all;
      first_pos = p;
    }
    ++n_all;
    p = np;
  }
  *exit_out = p;
  *broke_out = bad_hdr ? 1 : 0;
  *cnt_out = (n_all << 32) | n_big;
  a.first_loc[k] = first;
  a.first_pos[k] = first_pos;
}

// 2. Speculative walk and check of pieces [k_lo, k_hi) from their first plausible header (piece 0
// from 0).
__global__ __launch_bounds__(kCheckThreads) __attribute__((amdgpu_waves_per_eu(kCheckWgPerCu * kCheckThreads / 256))) void
wal_spec(WalArgs a, std::uint64_t k_lo, std::uint64_t k_hi) {
  __shared__ std::uint32_t lds[TKV_AB_WAL16 ? kLdsSliceWords / 2 : kLdsSliceWords];
  fill_slices(a.tabs, lds);
  const std::uint64_t k = k_lo + gid();
  if (k >= k_hi) return;
  const std::uint64_t s = k == 0 ? 0 : a.S[k];
  if (k == 0) a.S[0] = 0;
  if (s == kNone) {
    a.X[k] = kNone;
    a.next[k] = a.K;
    a.broke[k] = 0;
    a.spec_cnt[k] = 0;
    a.first_loc[k] = kNone;
    return;
  }
  const dev::LaneConst kc = TKV_AB_WAL16 ? dev::lane_const16(threadIdx.x & 63u) : dev::lane_const(threadIdx.x & 63u);
  std::uint64_t x, c;
  std::uint8_t br;
  walk_check(lds, kc, a, k, s, &x, &br, &c);
  a.X[k] = x;
  a.broke[k] = br;
  a.spec_cnt[k] = c;
  a.next[k] = (br || x >= a.size) ? a.K : static_cast<std::uint32_t>(x / kWalPiece);
}

__global__ void wal_jump_init(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K) return;
  a.Ja[k] = a.next[k];
  a.on[k] = k == 0 ? 1 : 0;
  a.recheck[k] = 0;
  a.bad_at[k] = kNone;
}

// 3 (fast path). Takes every piece with a speculative start (S != kNone) as on the true chain and
// entered at S, and checks that this holds: each such piece p must leave exactly into the next such
// piece q (next(p) == q and X_p == S_q), and the last one must end the chain (next == K). Piece 0
// is entered at 0, so by induction every such piece is then entered at S, and a piece with no
// plausible header holds no record start of the chain (a header the encoder wrote is plausible; a
// chain that reaches an implausible one breaks there, and next(p) == K contradicts a later piece
// with a start). Pieces further than kFastScan pieces from the next start fail the check. When it
// fails (res[6] = 1) the host runs the pointer-jumping stitch instead. Replaces wal_jump_init,
// ceil(log4 K) wal_jump launches and wal_link on every image whose speculation was right.
constexpr std::uint32_t kFastScan = 64;
__global__ void wal_fast(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K) return;
  const std::uint64_t s = a.S[k];
  const bool has = k == 0 || s != kNone;
  a.on[k] = has ? 1 : 0;
  a.entry[k] = k == 0 ? 0 : s;
  a.recheck[k] = 0;
  a.bad_at[k] = kNone;
  if (!has) return;
  std::uint64_t q = k + 1;
  while (q < a.K && q - k <= kFastScan && a.S[q] == kNone) ++q;
  bool ok;
  if (q >= a.K) ok = a.next[k] >= a.K;
  else ok = q - k <= kFastScan && a.next[k] == q && a.X[k] == a.S[q];
  if (!ok) a.res[6] = 1;
}

// Result words (res[0..6]) and the record scan's last entries into the host's pinned block.
__global__ void wal_publish(WalArgs a, std::uint64_t* h) {
  const unsigned i = threadIdx.x;
  if (i < 7) h[i] = a.res[i];
  if (i == 7) h[7] = a.base[a.K - 1];
  if (i == 8) h[8] = a.cnt[a.K - 1];
}

// 3. One quadrupling round (J = next^(4^t)): every marked k marks J(k), J(J(k)) and J(J(J(k))), then
// J <- J o J o J o J. After round t the marks hold next^i(0) for every i < 4^(t+1), so
// ceil(log4 K) rounds mark the whole path: half the launches of doubling, for two more dependent
// loads per round. Marks set during the round by other threads are pieces of the true path too,
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

// Entry points: each on-path piece hands its exit to the piece that holds it (one writer each:
// the path is a simple chain).
__global__ void wal_link(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K || !a.on[k]) return;
  if (k == 0) a.entry[0] = 0;
  const std::uint32_t n = a.next[k];
  if (n < a.K) a.entry[n] = a.X[k];
}

// 4. Records of an on-path piece from its entry: the speculative walk's when it started there;
// otherwise an exact walk (the records are checked again by wal_recheck). res[0] = the first piece
// whose speculative exit was wrong; res[5] counts re-checked pieces. Off-path pieces count 0.
__global__ void wal_count(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K) return;
  if (!a.on[k]) {
    a.cnt[k] = 0;
    return;
  }
  const std::uint64_t e = a.entry[k];
  std::uint64_t p, packed;
  bool bad;
  if (e == a.S[k]) {
    p = a.X[k];
    bad = a.broke[k] != 0;
    packed = a.spec_cnt[k];
  } else {
    const std::uint64_t limit = (k + 1) * kWalPiece < a.size ? (k + 1) * kWalPiece : a.size;
    std::uint64_t n_all = 0, n_big = 0;
    p = e;
    bad = false;
    while (p < limit) {  // wal.cpp:63-87
      if (a.size - p < kWalMeta) {
        bad = true;
        break;
      }
      const std::uint64_t rlen = ld32(a.w, p, a.size);
      if (rlen + 8 > a.size - p) {
        bad = true;
        break;
      }
      ++n_all;
      n_big += rlen > kWalLaneMax ? 1u : 0u;
      p += 8 + rlen;
    }
    packed = (n_all << 32) | n_big;
    a.recheck[k] = 1;
    atomicAdd(reinterpret_cast<unsigned long long*>(&a.res[5]), 1ull);
    if (p != a.X[k] || bad != (a.broke[k] != 0)) atomicMin(reinterpret_cast<unsigned long long*>(&a.res[0]), k);
  }
  a.cnt[k] = packed;
  a.Xe[k] = p;
  a.Be[k] = bad ? 1 : 0;
  if (a.next[k] >= a.K) {
    a.res[1] = p;
    a.res[2] = bad ? 1 : 0;
  }
}

// Pieces entered off their speculative start: check their records from the true entry.
__global__ __launch_bounds__(kCheckThreads) __attribute__((amdgpu_waves_per_eu(kCheckWgPerCu * kCheckThreads / 256))) void
wal_recheck(WalArgs a) {
  __shared__ std::uint32_t lds[TKV_AB_WAL16 ? kLdsSliceWords / 2 : kLdsSliceWords];
  fill_slices(a.tabs, lds);
  const std::uint64_t k = gid();
  if (k >= a.K || !a.recheck[k]) return;
  const dev::LaneConst kc = TKV_AB_WAL16 ? dev::lane_const16(threadIdx.x & 63u) : dev::lane_const(threadIdx.x & 63u);
  std::uint64_t x, c;
  std::uint8_t br;
  walk_check(lds, kc, a, k, a.entry[k], &x, &br, &c);
}

// Records past the first piece with a wrong speculative exit are not on the true chain (or not
// known to be): drop them.
__global__ void wal_trim(WalArgs a, std::uint64_t kstar) {
  const std::uint64_t k = gid();
  if (k < a.K && k > kstar) a.cnt[k] = 0;
}

// 5. Record numbering: the first failing record of each counted piece becomes a record index, and
// the big-record slots move to the dense list the CRC batch reads.
__global__ void wal_gather(WalArgs a) {
  const std::uint64_t k = gid();
  if (k >= a.K || a.cnt[k] == 0) return;
  const std::uint64_t b_all = a.base[k] >> 32, b_big = a.base[k] & 0xFFFFFFFFull;
  const std::uint64_t n_big = a.cnt[k] & 0xFFFFFFFFull;
  if (a.first_loc[k] != kNone) {
    a.bad_at[k] = b_all + a.first_loc[k];
    atomicMin(reinterpret_cast<unsigned long long*>(&a.res[3]), b_all + a.first_loc[k]);
  }
  for (std::uint64_t j = 0; j < n_big; ++j) {
    const std::uint64_t sl = 2 * k + j;
    a.big_off[b_big + j] = a.slot_off[sl];
    a.big_len[b_big + j] = a.slot_len[sl];
    a.big_crc[b_big + j] = a.slot_crc[sl];
    a.big_idx[b_big + j] = b_all + a.slot_loc[sl];
  }
}

__global__ void wal_check_big(WalArgs a, std::uint64_t n) {
  const std::uint64_t i = gid();
  if (i < n && a.got[i] != a.big_crc[i]) atomicMin(reinterpret_cast<unsigned long long*>(&a.res[3]), a.big_idx[i]);
}

// Start of the first bad record (res[3]): from the piece that found it, or from the big list.
__global__ void wal_bad_pos(WalArgs a, std::uint64_t n_big) {
  const std::uint64_t i = gid();
  const std::uint64_t want = a.res[3];
  if (i < a.K && a.cnt[i] != 0 && a.bad_at[i] == want) a.res[4] = a.first_pos[i];
  if (i < n_big && a.big_idx[i] == want) a.res[4] = a.big_off[i] - 8;
}

// Per-device scratch, grown by doubling and kept between calls (guarded by mu).
struct WalScratch {
  std::mutex mu;
  std::uint64_t cap_pieces = 0, cap_big = 0;
  void* pieces = nullptr;  // per piece: 13 u64, 9 u32, 4 u8 (carve)
  void* bigs = nullptr;    // per big record: 2 u64, 3 u32
  void* cub = nullptr;
  std::size_t cub_bytes = 0;
  std::uint64_t* res = nullptr;
  std::uint64_t* h_res = nullptr;  // pinned, kHres words
  std::uint64_t* d_hres = nullptr;  // device view of h_res (wal_publish)
  std::uint32_t* inj = nullptr;  // Shift_L(0xFFFFFFFF), L = 0..kWalLaneMax
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
    (void)hipFree(pieces);
    (void)hipFree(bigs);
    (void)hipFree(cub);
    (void)hipFree(res);
    (void)hipFree(inj);
    (void)hipHostFree(h_res);
  }
};

std::mutex g_wal_mu;
WalScratch* g_wal[64] = {};

// What the calling thread's last WAL verify did (tkv_debug_wal_last).
thread_local std::uint64_t g_last[4] = {0, 0, 0, 0};  // passes, host walk needed, image copied, fast stitch

#define WAL_HIP(call)                                                            \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e_)); \
  } while (0)

int grow_pieces(WalScratch& s, std::uint64_t K) {
  if (K <= s.cap_pieces) return TKV_OK;
  const std::uint64_t cap = std::max<std::uint64_t>(K, 2 * s.cap_pieces);
  WAL_HIP(hipFree(s.pieces));
  s.pieces = nullptr;
  s.cap_pieces = 0;
  WAL_HIP(hipMalloc(&s.pieces, cap * (13 * 8 + 9 * 4 + 4)));
  s.cap_pieces = cap;
  return TKV_OK;
}

int grow_big(WalScratch& s, std::uint64_t n) {
  if (n <= s.cap_big) return TKV_OK;
  const std::uint64_t cap = std::max<std::uint64_t>(n, 2 * s.cap_big);
  WAL_HIP(hipFree(s.bigs));
  s.bigs = nullptr;
  s.cap_big = 0;
  WAL_HIP(hipMalloc(&s.bigs, cap * (2 * 8 + 3 * 4)));
  s.cap_big = cap;
  return TKV_OK;
}

WalArgs carve(WalScratch& s, const std::uint8_t* w, std::uint64_t size, std::uint32_t K, const DeviceTables* tabs) {
  WalArgs a{};
  a.w = w;
  a.size = size;
  a.K = K;
  const std::uint64_t C = s.cap_pieces;
  auto* p8 = static_cast<std::uint64_t*>(s.pieces);
  std::uint64_t** u64s[] = {&a.S, &a.X, &a.spec_cnt, &a.first_loc, &a.first_pos, &a.entry, &a.cnt, &a.base, &a.Xe,
                            &a.bad_at};
  for (std::size_t i = 0; i < sizeof(u64s) / sizeof(u64s[0]); ++i) *u64s[i] = p8 + i * C;
  a.slot_off = p8 + 10 * C;  // 2C
  auto* p4 = reinterpret_cast<std::uint32_t*>(p8 + 13 * C);
  a.next = p4;
  a.Ja = p4 + C;
  a.Jb = p4 + 2 * C;
  a.slot_len = p4 + 3 * C;  // 2C each
  a.slot_crc = p4 + 5 * C;
  a.slot_loc = p4 + 7 * C;
  auto* p1 = reinterpret_cast<std::uint8_t*>(p4 + 9 * C);
  a.broke = p1;
  a.on = p1 + C;
  a.Be = p1 + 2 * C;
  a.recheck = p1 + 3 * C;
  const std::uint64_t B = s.cap_big;
  if (B) {
    auto* b8 = static_cast<std::uint64_t*>(s.bigs);
    a.big_off = b8;
    a.big_idx = b8 + B;
    auto* b4 = reinterpret_cast<std::uint32_t*>(b8 + 2 * B);
    a.big_len = b4;
    a.big_crc = b4 + B;
    a.got = b4 + 2 * B;
  }
  a.inj = s.inj;
  a.tabs = tabs;
  a.res = s.res;
  return a;
}

unsigned blocks(std::uint64_t n, unsigned t) { return static_cast<unsigned>((n + t - 1) / t); }

// CRC batches of at most this many records (the irregular path's u32 block indices).
constexpr std::uint64_t kWalCrcChunk = std::uint64_t(1) << 31;

// A pass over the image [w, w + size), which starts with a record (or is empty), in three parts:
// pass_begin (result words, speculative starts cleared), pass_front over ranges of pieces (scan and
// speculative walk; each range's bytes and the next 1 KiB + 26 bytes must be resident), pass_tail.
int pass_begin(WalScratch& s, const std::uint8_t* w, std::uint64_t size, hipStream_t st, WalArgs* out) {
  const std::uint32_t K = static_cast<std::uint32_t>((size + kWalPiece - 1) / kWalPiece);
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  if (int rc = grow_pieces(s, K)) return rc;
  WalArgs a = carve(s, w, size, K, tabs);
  s.h_res[0] = kNone;
  s.h_res[1] = size;
  s.h_res[2] = 0;
  s.h_res[3] = kNone;
  s.h_res[4] = 0;
  s.h_res[5] = 0;
  s.h_res[6] = 0;
  WAL_HIP(hipMemcpyAsync(s.res, s.h_res, 7 * sizeof(std::uint64_t), hipMemcpyHostToDevice, st));
  WAL_HIP(hipMemsetAsync(a.S, 0xFF, K * sizeof(std::uint64_t), st));
  *out = a;
  return TKV_OK;
}

void pass_front(const WalArgs& a, std::uint64_t k_lo, std::uint64_t k_hi, hipStream_t st) {
  if (k_hi <= k_lo) return;
  const std::uint64_t threads = (k_hi - k_lo + 64 / kHeadLanes - 1) / (64 / kHeadLanes) * 64;  // 8 pieces per wave
  hipLaunchKernelGGL(wal_scan_head, dim3(blocks(threads, kScanThreads)), dim3(kScanThreads), 0, st, a, k_lo, k_hi);
  hipLaunchKernelGGL(wal_spec, dim3(blocks(k_hi - k_lo, kCheckThreads)), dim3(kCheckThreads), 0, st, a, k_lo, k_hi);
}

int pass_tail(WalScratch& s, WalArgs a, hipStream_t st, PassResult* r) {
  const std::uint8_t* w = a.w;
  const std::uint64_t size = a.size;
  const std::uint32_t K = a.K;
  const DeviceTables* tabs = a.tabs;
  // 3: the pieces on the true chain and their entries, first by the fast path (wal_fast), with
  // record counts and their scan behind it, so one host sync reads the verdict and the totals
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
  auto count_and_publish = [&]() -> int {
    hipLaunchKernelGGL(wal_count, dim3(blocks(K, 256)), dim3(256), 0, st, a);
    WAL_HIP(hipcub::DeviceScan::ExclusiveSum(s.cub, need, a.cnt, a.base, K, st));
    hipLaunchKernelGGL(wal_publish, dim3(1), dim3(64), 0, st, a, s.d_hres);
    WAL_HIP(hipGetLastError());
    WAL_HIP(hipStreamSynchronize(st));
    return TKV_OK;
  };
  hipLaunchKernelGGL(wal_fast, dim3(blocks(K, 256)), dim3(256), 0, st, a);
  if (int rc = count_and_publish()) return rc;
  if (s.h_res[6]) g_last[3] = 0;  // the pointer-jumping stitch ran
  if (s.h_res[6]) {
    // the speculation was wrong somewhere: pointer jumping marks the pieces on the true chain
    // (wal_count above took the fast path's entries, which are speculative starts: it left res[0]
    // and res[5] alone, and the exact count below rewrites res[1], res[2] from the true last piece)
    hipLaunchKernelGGL(wal_jump_init, dim3(blocks(K, 256)), dim3(256), 0, st, a);
    std::uint32_t* J = a.Ja;
    std::uint32_t* J2 = a.Jb;
    for (std::uint64_t reach = 1; reach < K; reach <<= 2) {
      hipLaunchKernelGGL(wal_jump, dim3(blocks(K, 256)), dim3(256), 0, st, J, J2, a.on, K);
      std::swap(J, J2);
    }
    hipLaunchKernelGGL(wal_link, dim3(blocks(K, 256)), dim3(256), 0, st, a);
    // 4: record counts from the entries
    if (int rc = count_and_publish()) return rc;
  }
  const std::uint64_t kstar = s.h_res[0];
  std::uint64_t chain_end = s.h_res[1];
  bool broke = s.h_res[2] != 0;
  const bool partial = kstar < K;
  std::uint64_t tot = s.h_res[7] + s.h_res[8];  // (records << 32) | big records
  if (s.h_res[5]) hipLaunchKernelGGL(wal_recheck, dim3(blocks(K, kCheckThreads)), dim3(kCheckThreads), 0, st, a);
  if (partial) {
    hipLaunchKernelGGL(wal_trim, dim3(blocks(K, 256)), dim3(256), 0, st, a, kstar);
    WAL_HIP(hipcub::DeviceScan::ExclusiveSum(s.cub, need, a.cnt, a.base, K, st));
    hipLaunchKernelGGL(wal_publish, dim3(1), dim3(64), 0, st, a, s.d_hres);
    std::uint8_t be = 0;
    WAL_HIP(hipMemcpyAsync(s.h_res + 1, a.Xe + kstar, 8, hipMemcpyDeviceToHost, st));
    WAL_HIP(hipMemcpyAsync(&be, a.Be + kstar, 1, hipMemcpyDeviceToHost, st));
    WAL_HIP(hipStreamSynchronize(st));
    chain_end = s.h_res[1];
    broke = be != 0;
    tot = s.h_res[7] + s.h_res[8];
  }
  // 5: record numbering (the scan above), first failing in-lane record, the CRC batch of the big ones
  const std::uint64_t n = tot >> 32, n_big = tot & 0xFFFFFFFFull;
  std::uint64_t first = n;
  if (n) {
    if (int rc = grow_big(s, std::max<std::uint64_t>(n_big, 1))) return rc;
    a = carve(s, w, size, K, tabs);
    hipLaunchKernelGGL(wal_gather, dim3(blocks(K, 256)), dim3(256), 0, st, a);
    WAL_HIP(hipGetLastError());
    for (std::uint64_t i = 0; i < n_big; i += kWalCrcChunk) {
      const std::uint64_t m = std::min(kWalCrcChunk, n_big - i);
      if (int rc = batch_device_impl(kAlgoCrc32, w, a.big_off + i, a.big_len + i, nullptr, a.got + i, m, st)) return rc;
    }
    if (n_big) hipLaunchKernelGGL(wal_check_big, dim3(blocks(n_big, 256)), dim3(256), 0, st, a, n_big);
    hipLaunchKernelGGL(wal_bad_pos, dim3(blocks(std::max<std::uint64_t>(K, n_big), 256)), dim3(256), 0, st, a, n_big);
    WAL_HIP(hipGetLastError());
    hipLaunchKernelGGL(wal_publish, dim3(1), dim3(64), 0, st, a, s.d_hres);
    WAL_HIP(hipGetLastError());
    WAL_HIP(hipStreamSynchronize(st));
    first = std::min<std::uint64_t>(s.h_res[3], n);
  }
  r->good = first;
  r->corrupted = first < n || broke;
  r->stop = first < n ? s.h_res[4] : chain_end;
  r->resume = !r->corrupted && partial && chain_end < size;
  return TKV_OK;
}

// A whole pass over a resident image.
int wal_pass(WalScratch& s, const std::uint8_t* w, std::uint64_t size, hipStream_t st, PassResult* r) {
  WalArgs a;
  if (int rc = pass_begin(s, w, size, st, &a)) return rc;
  pass_front(a, 0, a.K, st);
  return pass_tail(s, a, st, r);
}

// The calling thread's device's scratch (created on first use, with its result words and the
// init-term table).
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
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_res), kHres * sizeof(std::uint64_t), hipHostMallocDefault));
    WAL_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&sp->d_hres), sp->h_res, 0));
    WAL_HIP(hipStreamCreateWithFlags(&sp->st, hipStreamNonBlocking));
    WAL_HIP(hipStreamCreateWithFlags(&sp->stc, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) WAL_HIP(hipEventCreateWithFlags(&sp->landed[i], hipEventDisableTiming));
    std::vector<std::uint32_t> inj(kWalLaneMax + 1);
    for (std::uint32_t L = 0; L <= kWalLaneMax; ++L) inj[L] = shift_bytes(kInit, L, kPoly);
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->inj), inj.size() * 4));
    WAL_HIP(hipMemcpy(sp->inj, inj.data(), inj.size() * 4, hipMemcpyHostToDevice));
  }
  *out = sp;
  return TKV_OK;
}

int verify_locked(WalScratch& s, const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                  std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk,
                  const PassResult* first_pass = nullptr) {
  // Each pass checks the true chain at least through its first piece; a pass that stops short of
  // the end without a verdict resumes at a true record start. Adversarial images that keep the
  // speculation wrong go to the exact host walk after kMaxPasses.
  constexpr int kMaxPasses = 8;
  std::uint64_t start = 0, good = 0;
  g_last[0] = g_last[1] = 0;
  for (int pass = 0; pass < kMaxPasses; ++pass) {
    PassResult r;
    g_last[0] = static_cast<std::uint64_t>(pass) + 1;
    if (pass == 0 && !first_pass) g_last[3] = 1;  // cleared by the first pass that needs the pointer-jumping stitch
    if (pass == 0 && first_pass) r = *first_pass;
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
// Device copies of host images up to this size stay allocated between verifies.
constexpr std::uint64_t kKeepImg = std::uint64_t(256) << 20;

int host_image_locked(WalScratch& s, const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                      std::uint64_t* stop_offset, bool* needs_host_walk);

}  // namespace

int wal_verify_device_impl(const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                           std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk) {
  *needs_host_walk = false;
  *n_good = 0;
  *stop_offset = 0;
  g_last[0] = g_last[1] = g_last[2] = g_last[3] = 0;
  if (size == 0) return TKV_OK;
  if ((size + kWalPiece - 1) / kWalPiece >= 0xFFFFFFFFull)
    return set_error(TKV_INVALID_ARGUMENT, "WAL image too large for the device walk");
  WalScratch* sp = nullptr;
  if (int rc = scratch(&sp)) return rc;
  WalScratch& s = *sp;
  std::lock_guard<std::mutex> lk(s.mu);
  return verify_locked(s, d_wal, size, n_good, stop_offset, st, needs_host_walk);
}

int wal_verify_host_image_impl(const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                               std::uint64_t* stop_offset, bool* needs_host_walk) {
  *needs_host_walk = false;
  *n_good = 0;
  *stop_offset = 0;
  g_last[0] = g_last[1] = g_last[2] = g_last[3] = 0;
  if (size == 0) return TKV_OK;
  if ((size + kWalPiece - 1) / kWalPiece >= 0xFFFFFFFFull) {
    *needs_host_walk = true;
    return TKV_OK;
  }
  WalScratch* sp = nullptr;
  if (int rc = scratch(&sp)) return rc;
  WalScratch& s = *sp;
  std::lock_guard<std::mutex> lk(s.mu);
  g_last[2] = 1;
  const int rc = host_image_locked(s, h_wal, size, n_good, stop_offset, needs_host_walk);
  // No copy that reads the caller's buffer, and no kernel on the device copy, may outlive the call
  // (an error return included). A device copy larger than kKeepImg is released, so one large
  // recovery does not keep its size of HBM from the caller's later allocations.
  (void)hipStreamSynchronize(s.st);
  (void)hipStreamSynchronize(s.stc);
  if (s.cap_img > kKeepImg) {
    (void)hipFree(s.d_img);
    s.d_img = nullptr;
    s.cap_img = 0;
  }
  return rc;
}

namespace {
int host_image_locked(WalScratch& s, const std::uint8_t* h_wal, std::uint64_t size, std::uint64_t* n_good,
                      std::uint64_t* stop_offset, bool* needs_host_walk) {
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
  // stream scans and speculatively walks the pieces before it whose records' bytes are all resident
  // (pieces ending at least kFrontMargin bytes before the end of what has landed), so only the last
  // chunk's pieces and the stitching remain once the copy is done.
  constexpr std::uint64_t kFrontMargin = kWalPiece + kWalLaneMax + 64;
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
    const std::uint64_t k_hi = last ? a.K : (off + m > kFrontMargin ? (off + m - kFrontMargin) / kWalPiece : 0);
    if (k_hi > fronted) {
      pass_front(a, fronted, k_hi, s.stc);
      fronted = k_hi;
    }
  }
  WAL_HIP(hipGetLastError());
  PassResult r;
  g_last[0] = 1;
  g_last[3] = 1;  // the first device pass starts here; cleared if it needs the pointer-jumping stitch
  if (int rc = pass_tail(s, a, s.stc, &r)) return rc;
  return verify_locked(s, s.d_img, size, n_good, stop_offset, s.stc, needs_host_walk, &r);
}
}  // namespace

}  // namespace tkv

extern "C" void tkv_debug_wal_last(uint64_t out[4]) {
  for (int i = 0; i < 4; ++i) out[i] = tkv::g_last[i];
}
