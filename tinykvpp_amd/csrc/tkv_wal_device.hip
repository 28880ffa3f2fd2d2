// WAL recovery verify on the device: the record_len chain walk of
// wal_entry::decode (/root/reference/src/engine/wal.cpp:63-130, driven by engine::create's recovery
// loop, /root/reference/src/engine/engine.cpp:31-53) over a WAL image resident in HBM, the CRC check
// of every record (wal.cpp:89-96) and the key/value bounds check (wal.cpp:118-121), ending in the first
// corruption. The image is read from HBM once (round 5).
//
// wal_sweep: every wave streams a contiguous chunk of the image, one region of kRegion = 7 KiB at a
// time. Regions are loaded a region ahead into registers (coalesced 16-byte buffer loads whose
// descriptor ends at the image's end) and written into the wave's LDS window together with the first
// kOver bytes of the next region, so a record that starts in the region and has a payload of at most
// kLaneFold bytes lies wholly in the window. Twelve waves (three per SIMD: 10 KiB regions with eight
// waves, and 5 KiB with sixteen, measured slower) share one copy of the 64 KiB slicing tables (16
// replicas, at LDS address 0). Positions are 32-bit for images below 4 GiB. Per region:
//  1. walk: lane l owns the piece [rs + kPiece l, + kPiece). The lane holding the region's entry E
//     (where the chain leaves the previous region) starts there; every later lane starts at the first
//     plausible header of its piece (one the reference encoder could have written, wal.cpp:19-61),
//     speculatively. Each lane walks the records that start in its piece (wal.cpp:63-87: at least 26
//     bytes left, record_len + 8 within the image), all reads from LDS.
//  2. link check: every lane with a start must be entered exactly where the previous such lane's walk
//     left (one shuffle per lane). Where a link fails, the chain from the last good lane is followed
//     exactly (the lane it lands in walks again from the landing point, the lanes it skips drop out),
//     so the region's chain is exact given E. Its exit is the next region's entry.
//  3. fold: the region's records are listed in chain order in LDS and folded one per lane from the
//     window (slicing-by-4 into the engine's conflict-free LDS tables), compared with the stored CRC
//     and checked for key/value bounds; the region keeps the index of its first bad record. Payloads
//     longer than kLaneFold go to a global list that one irregular CRC batch checks afterwards.
// The chunk's first region has no known entry: its wave takes the first plausible header it finds
// (a region without one "searches" on). After a break the wave searches again.
//
// Exactness across chunks (bounds_one in wal_after, wal_sweep in fix-up mode): wherever a region's entry did not
// come from its predecessor's exit in the same walk (chunk starts, search starts, fix-up starts),
// the predecessor's exit must land exactly on the entry, with only searching regions (no chain)
// between. A boundary that fails is walked again from the true exit by a fix-up wave, which stops as
// soon as its exit meets a stored entry (the chains coincide from there) or at the next failing
// boundary; the boundaries are checked again, and the first failing one moves forward every round.
// Nothing leaves the device but a few result words, and no image is walked on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "tkv_crc32.h"
#include "tkv_crc32_device.h"
#include "tkv_engine.h"
#include "tkv_wal_device.h"

namespace tkv {
namespace {

constexpr std::uint64_t kWalMeta = 26;          // wal.hpp:21-27 kMetadataSize
constexpr std::uint64_t kNone = ~0ull;
constexpr std::uint32_t kRegion = 7168;  // image bytes per region (one wave step)
constexpr int kRows = kRegion / 1024;           // 1 KiB load rows per region
constexpr std::uint32_t kPiece = kRegion / 64;  // bytes per lane piece
constexpr std::uint32_t kOver = 256;            // bytes of the next region behind the window
constexpr std::uint32_t kLaneFold = 240;        // payloads up to this long are folded by one lane from LDS
constexpr std::uint32_t kWin = 16 + kRegion + kOver;  // window: the region's aligned start, region, overlap
// listed records per region (see the list step), and behind them the region's fold ranges (12 bytes
// each: the carry range always fits behind the most records a region can hold)
constexpr std::uint32_t kList = kRegion / 26 + 16;
constexpr std::uint32_t kWinBytes = (kWin + 2 * kList + 15) & ~15u;
constexpr std::uint32_t kMedMax = 65536;  // payloads longer than kLaneFold and up to this: folded in the sweep
constexpr std::uint32_t kChunk = 112;     // bytes per lane of a range fold
static_assert(kRegion <= 64 * kChunk && kChunk <= kLaneFold, "a whole region is one round of chunks");
static_assert(2 * kList >= 2 * ((kRegion / 26 + 2) & ~1u) + 12, "the carry range fits behind a full list");
constexpr std::uint32_t kStore = kPiece / 26 + 2;  // starts a lane lists: its records up to the first tiny one
constexpr unsigned kSweepWaves = 12;            // waves per workgroup: the 64 KiB tables + 12 windows of LDS
constexpr unsigned kSweepThreads = 64 * kSweepWaves;
constexpr unsigned kHres = 16;                  // words of the pinned result block
constexpr std::uint32_t kMaxFix = 1u << 16;     // failing boundaries handled per fix-up round
static_assert(kRegion % 1024 == 0 && kPiece % 16 == 0, "region = whole 1 KiB load rows");
static_assert(kOver >= kLaneFold + 8 && kOver >= kWalMeta, "a lane-folded record ends inside the window");
static_assert(kList * 26 >= kRegion + 26 * 2, "records of >= 26 bytes fit the list");
static_assert(kLdsSliceWords * 2 + kSweepWaves * kWinBytes + 4 * (kLaneFold + 1) + 4 * 64 <= 163840, "LDS");
static_assert(kStore <= 8, "list counts per lane < 16");
static_assert(kList <= 512, "list indices fit 9 bits (range words, long-payload metadata)");

// Region flags (low byte of fl[]; the region's version, bumped by every fix-up rewrite, above it).
constexpr std::uint32_t kChain = 1;   // the region has chain state: E (entry, may lie past the region) and X
constexpr std::uint32_t kSpec = 2;    // its entry came from a search (speculative)
constexpr std::uint32_t kSearch = 4;  // no chain: the walk searched the region and found no header
constexpr std::uint32_t kBroke = 8;   // the chain broke in the region, at X (wal.cpp:68-70, 80-87)
constexpr std::uint32_t kEnd = 16;    // the chain reached the end of the image exactly (X == size)
constexpr std::uint32_t kFix = 32;    // its entry came from a fix-up task (checked like kSpec)
constexpr std::uint32_t kGiantHop = 64;  // the chain leaves it in a record longer than kMedMax (passed over)
constexpr std::uint32_t kFakeHop = 128;  // ... over more than kTrustHop regions from an implausible header
constexpr std::uint64_t kFakeHopBit = 1ull << 63;  // a failing boundary's exit (inc_x) from such a region
// kinds of fold range: the bytes in front of the region's entry (part of the record the chain is in
// when it enters; crc0), a payload wholly inside the region (initial register injected, checked here),
// the head of a payload that goes on past the region (initial register injected; finished by wal_fin_*)
constexpr std::uint32_t kRangeCarry = 0, kRangeWhole = 1, kRangeHead = 2;

// Result words (device, u64): see wal_fin_*.
enum : int { kResLongA = 0, kResIncons, kResFirst, kResP, kResQ, kResLidx, kResCnt, kResLongSeg, kResWalkMax,
             kResWalkSum, kResDone, kResWords = 11 };
static_assert(kResDone < kResWords, "result words");

struct SweepArgs {
  const std::uint8_t* w;
  std::uint64_t size;
  std::uintptr_t al0;         // w rounded down to 16 bytes
  std::uintptr_t gend;        // the end of the image's last 16-byte granule (loads stop there)
  std::uint32_t o;            // w - al0
  std::uint32_t nreg;
  std::uint32_t nwaves;       // sweep: chunks; fix-up: tasks
  std::uint32_t wsweep;       // the sweep's waves (segments of the long-payload list)
  const std::uint32_t* t_begin;  // fix-up task: first region, limit (exclusive), entry
  const std::uint32_t* t_limit;
  const std::uint64_t* t_entry;
  // per region
  std::uint64_t* E;
  std::uint64_t* X;
  std::uint64_t* B;           // start of the region's first bad record (kNone)
  std::uint32_t* cnt;         // chain records starting in the region
  std::uint32_t* bidx;        // index of the first bad one among them
  std::uint32_t* fl;
  // per region, the payloads folded in the sweep across region ends (kLaneFold < record_len <= kMedMax)
  std::uint32_t* carry;       // crc0 of [rs, min(E, re)): the record the chain is in when it enters
  std::uint32_t* cm_len;      // the region's crossing payload (its last record's, when it goes on past
  std::uint32_t* cm_crc;      //   re): record_len (0: none), stored CRC, the register after its bytes in
  std::uint32_t* cm_part;     //   the region (initial register included; ~0 when there are none), and
  std::uint32_t* cm_pos;      //   its start - rs | its list index << 16
  // records with payloads longer than kMedMax (checked by a CRC batch)
  std::uint64_t* l_off;
  std::uint32_t* l_len;
  std::uint32_t* l_crc;
  std::uint32_t* l_reg;
  std::uint32_t* l_meta;      // index in the region | version << 9
  std::uint64_t l_cap;        // entries; sweep wave w owns [w * l_seg, (w + 1) * l_seg), the rest is
  std::uint64_t l_seg;        //   taken by atomics (fix-ups, and sweep waves whose segment is full)
  std::uint32_t* l_cnt;       // per sweep wave: entries in its segment
  unsigned long long* res;
  const DeviceTables* tabs;
};

__device__ __forceinline__ std::uint32_t le1_marks(std::uint32_t d) {
  // bit 7 of byte i set iff byte i of d is 0 or 1 (bit 7 of (b & 0x7E) + 0x7F is clear iff no bit 1-6
  // of b is set; no byte carries into the next)
  return ~(((d & 0x7E7E7E7Eu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
}

// Little-endian u32 at byte b of the window (dword-aligned reads, v_alignbyte).
__device__ __forceinline__ std::uint32_t rd32(const std::uint8_t* win, std::uint32_t b) {
  const std::uint32_t q = b & ~3u;
  const std::uint32_t lo = *reinterpret_cast<const std::uint32_t*>(win + q);
  const std::uint32_t hi = *reinterpret_cast<const std::uint32_t*>(win + q + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, b & 3u);
}

// Image positions in the sweep: u32 for images of at most kPos32Max bytes (every position, the
// region ends and kNone fit), u64 beyond.
constexpr std::uint64_t kPos32Max = 0xFFFF0000ull;
template <typename P>
constexpr P kNoneP = static_cast<P>(~0ull);
template <typename P>
__device__ __forceinline__ std::uint64_t widen(P v) {
  return v == kNoneP<P> ? kNone : static_cast<std::uint64_t>(v);
}
__device__ __forceinline__ std::uint32_t shfl_pos(std::uint32_t v, std::uint32_t src) {
  return static_cast<std::uint32_t>(__shfl(static_cast<int>(v), static_cast<int>(src), 64));
}
__device__ __forceinline__ std::uint64_t shfl_pos(std::uint64_t v, std::uint32_t src) {
  const std::uint32_t lo = shfl_pos(static_cast<std::uint32_t>(v), src);
  const std::uint32_t hi = shfl_pos(static_cast<std::uint32_t>(v >> 32), src);
  return (static_cast<std::uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ std::uint32_t readlane_pos(std::uint32_t v, std::uint32_t l) {
  return static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(l)));
}
__device__ __forceinline__ std::uint64_t readlane_pos(std::uint64_t v, std::uint32_t l) { return dev::readlane64(v, l); }

using dev::lane_prefix;  // exclusive prefix sum over the 64 lanes (DPP scan) and its total


// The first plausible header in [ps, qe) (qe - ps <= 16 NG - 16: a whole piece at NG = 8; every
// position there has 26 bytes in the image): op and tombstone bytes (p+8, p+17) 0 or 1, then
// record_len = 18 + klen + vlen and record_len + 8 within the image. Byte-parallel over the window
// bytes from the 16-byte granule of ps + 8 (NG + 1 16-byte reads): z marks each byte that is 0 or 1
// (bit 7), c = z & (z 9 bytes on) marks the positions passing both, and the c of four dwords are packed
// into one word per 16 positions, transposed (bit 8 j + i = byte j of dword i; 4 shifts and 2 ORs, no
// multiply). ps + 8 is at the same granule offset sh in every lane (pieces are multiples of 16 bytes),
// so the mask of the positions in front of it is wave-uniform. Candidates are taken in position order
// and checked in full. One call covers a whole piece: searching it 48 positions at a time cost the
// wave a second step whenever any lane's first header lay further in (almost every region of small
// records) and three in every region inside a long payload.
static_assert(kPiece % 16 == 0 && kPiece + 15 + 9 < 16 * 9, "a piece's search fits nine granules");
template <typename P, int NG>
__device__ __forceinline__ P search_piece(const std::uint8_t* win, P rs, std::uint32_t o, P ps, P qe, P size) {
  static_assert(NG % 2 == 0, "groups of 16 positions in pairs (64-bit masks)");
  if (ps >= qe) return kNoneP<P>;
  const std::uint32_t b0 = static_cast<std::uint32_t>(ps - rs) + o + 8u;
  const std::uint32_t a16 = b0 & ~15u;
  const std::uint32_t sh = __builtin_amdgcn_readfirstlane(b0 & 15u);
  const uint4* g = reinterpret_cast<const uint4*>(win + a16);
  std::uint32_t z[4 * (NG + 1)];
#pragma unroll
  for (int i = 0; i <= NG; ++i) {
    const uint4 v = g[i];
    z[4 * i] = le1_marks(v.x);
    z[4 * i + 1] = le1_marks(v.y);
    z[4 * i + 2] = le1_marks(v.z);
    z[4 * i + 3] = le1_marks(v.w);
  }
  std::uint32_t y[NG];
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    std::uint32_t c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * gi + i;
      c[i] = z[k] & __builtin_amdgcn_alignbyte(z[k + 3], z[k + 2], 1u);
    }
    y[gi] = (c[0] >> 7) | (c[1] >> 6) | (c[2] >> 5) | (c[3] >> 4);
  }
  // positions p = 4 i + j < sh of the first group (wave-uniform)
  const std::uint32_t si = sh >> 2, sj = sh & 3u;
  y[0] &= ((0xFu << (si + 1u)) & 0xFu) * 0x01010101u | ((0x01010101u << (8u * sj)) << si);
  const std::uint32_t span = static_cast<std::uint32_t>(qe - ps);
  std::uint64_t m[NG / 2];
#pragma unroll
  for (int k = 0; k < NG / 2; ++k) m[k] = y[2 * k] | static_cast<std::uint64_t>(y[2 * k + 1]) << 32;
  for (;;) {
    std::uint64_t cur = 0;
    std::uint32_t sel = 0;
#pragma unroll
    for (int k = NG / 2 - 1; k >= 0; --k) {  // the first non-empty pair
      if (m[k] != 0) {
        cur = m[k];
        sel = static_cast<std::uint32_t>(k);
      }
    }
    if (cur == 0) break;
    const bool hw = static_cast<std::uint32_t>(cur) == 0u;
    const std::uint32_t yv = hw ? static_cast<std::uint32_t>(cur >> 32) : static_cast<std::uint32_t>(cur);
    const std::uint32_t gi = 2u * sel + (hw ? 1u : 0u);
    const std::uint32_t i = static_cast<std::uint32_t>(__builtin_ctz((yv | yv >> 8 | yv >> 16 | yv >> 24) & 0xFu));
    const std::uint32_t j = static_cast<std::uint32_t>(__builtin_ctz((yv >> i) & 0x01010101u)) >> 3;
    const std::uint32_t pos = 16u * gi + 4u * i + j - sh;  // from ps
    if (pos >= span) return kNoneP<P>;  // (every later candidate lies further on)
    const std::uint32_t b = b0 - 8u + pos;
    const std::uint64_t rl = rd32(win, b), kl = rd32(win, b + 18u), vl = rd32(win, b + 22u);
    const P q = ps + pos;
    if (rl == 18u + kl + vl && static_cast<P>(rl) <= size - q - 8u) return q;  // (size - q >= 26)
    const std::uint64_t bit = 1ull << ((hw ? 32u : 0u) + 8u * j + i);
#pragma unroll
    for (int k = 0; k < NG / 2; ++k)
      if (static_cast<std::uint32_t>(k) == sel) m[k] &= ~bit;
  }
  return kNoneP<P>;
}

// The records that start in [s, pe) from s (wal.cpp:63-87), read from the window. n: their count;
// st[j]: the offsets from rs of the first kStore; x: the first record start at or past pe, or where
// the chain broke (broke); tiny: the index of the first with record_len < 18 (bad for certain: its
// key/value fields cannot fit, wal.cpp:118-121), kStore if none among the stored ones. The records in
// front of a lane's first tiny one are at least 26 bytes long, so it is always among the stored.
template <typename P>
struct Walk {
  std::uint32_t st[kStore];
  std::uint32_t n, tiny;
  P x;
  P lr;  // the start of the last record walked
  bool broke;
};
template <typename P>
__device__ __forceinline__ void walk_piece(const std::uint8_t* win, P rs, std::uint32_t o, P s, P pe, P size, bool go,
                                           Walk<P>& wk) {
  P p = s;
  bool act = go && s != kNoneP<P>;
  if (go) {
    wk.n = 0;
    wk.tiny = kStore;
    wk.broke = false;
    wk.lr = kNoneP<P>;
  }
  auto step = [&](std::uint32_t j, bool store) {
    if (size - p < kWalMeta) {
      wk.broke = true;
      act = false;
    } else {
      const std::uint32_t rl = rd32(win, static_cast<std::uint32_t>(p - rs) + o);
      if (static_cast<P>(rl) > size - p - 8u) {  // (size - p >= 26)
        wk.broke = true;
        act = false;
      } else {
        if (store) {
          wk.st[j] = static_cast<std::uint32_t>(p - rs);
          if (rl < 18u && wk.tiny == kStore) wk.tiny = j;
        }
        wk.n += 1;
        wk.lr = p;
        p += 8u + static_cast<P>(rl);
      }
    }
  };
  bool more = true;
#pragma unroll
  for (std::uint32_t j = 0; j < kStore; ++j) {
    act = act && p < pe && p < size;  // (the chain ends where the image does: wal.cpp:63)
    if (__ballot(act) == 0) {
      more = false;
      break;
    }
    if (act) step(j, true);
  }
  // records past the stored ones (a chain of tiny records): walked, counted, not listed
  while (more) {
    act = act && p < pe && p < size;
    if (__ballot(act) == 0) break;
    if (act) step(0, false);
  }
  if (go) wk.x = p;
}


// CRC-32 (finalized) of the L <= kLaneFold window bytes at s, one record per lane. The record is read
// from s - z, z = 4 nd - L (nd = its dwords), so that it ends on a dword; the z bytes in front are
// zeroed in its first dword (leading zeros leave a zero register at 0). Every lane steps through the
// round's largest dword count, its register frozen after its own nd (selects, no branch: the LDS
// waits stay countable; exec-masked steps measured slower). Dword i is v_alignbyte of two
// dword-aligned window reads. The initial register enters as inj[L] = Shift_L(0xFFFFFFFF)
// (crc_s(D) = Shift_|D|(s) ^ crc_0(D)); slicing-by-4 into the 64 KiB table image (crc32.cpp:9-16
// restated). (Two or three records per lane at once, as independent chains, measured slower.)
// fold_raw is that fold from a zero register (crc0 of the bytes); callers add inj[L] ^ 0xFFFFFFFF.
__device__ __forceinline__ std::uint32_t fold_raw(const std::uint8_t* win, const std::uint32_t* tab, const dev::LaneConstX& kc,
                                                  std::uint32_t s, std::uint32_t L) {
  const std::uint32_t nd = (L + 3u) >> 2;
  const std::uint32_t nmax = dev::wave_max(nd);
  const std::uint32_t z = 4u * nd - L;
  const std::uint32_t b0 = s - z;  // (s >= 8: b0 >= 5)
  const std::uint32_t sh = b0 & 3u;
  const std::uint32_t* w = reinterpret_cast<const std::uint32_t*>(win + (b0 & ~3u));
  std::uint32_t lo = w[1];
  dev::Reg r{0u, 0u};
  dev::slice4(tab, r, __builtin_amdgcn_alignbyte(lo, w[0], sh) & (~0u << (8u * z)), kc);
  if (nd == 0u) r = dev::Reg{0u, 0u};
#pragma unroll 2
  for (std::uint32_t i = 1; i < nmax; ++i) {
    const std::uint32_t hi = w[i + 1u];
    dev::Reg t = r;
    dev::slice4(tab, t, __builtin_amdgcn_alignbyte(hi, lo, sh), kc);
    if (i < nd) r = t;
    lo = hi;
  }
  return r.value();
}

// a*b mod P (reflected, x^0 = bit 31) in few registers: the loop is kept rolled (fully unrolled, the
// shift chain of b is computed ahead and held, which spills the sweep).
__device__ __forceinline__ std::uint32_t mul_lean(std::uint32_t a, std::uint32_t b, std::uint32_t poly) {
  std::uint32_t p = 0;
#pragma unroll 4
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - (a >> 31));
    a <<= 1;
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

// x^(8n) mod P for n <= 2 kRow (head_shift[h][31] = Shift_h(x^0)), and reg moved past n zero bytes.
__device__ __forceinline__ std::uint32_t x8n(const DeviceTables* t, std::uint32_t n) {
  return n <= static_cast<std::uint32_t>(kRow)
             ? t->head_shift[n][31]
             : dev::multmodp(t->head_shift[n - kRow][31], t->head_shift[kRow][31], t->poly);
}
__device__ __forceinline__ std::uint32_t shift_n(const DeviceTables* t, std::uint32_t reg, std::uint32_t n) {
  return dev::multmodp(x8n(t, n), reg, t->poly);
}

// Fold ranges R[0, nr) of the window (3 words each: x | y << 16 window offsets, kk | kind << 9 |
// record offset << 16, and the result): every range cut into kChunk-byte chunks aligned to its end
// (the front chunk shorter), one chunk per lane (fold_raw from LDS), the chunk j from the end moved past
// the j kChunk bytes behind it by one multiply with K[j] = x^(8 kChunk j), and the chunks of a range
// XORed into its result word (LDS atomics). A range of kind kRangeWhole / kRangeHead starts from the
// initial register (the front chunk adds Shift_L(0xFFFFFFFF)), so its result is the CRC register after
// its bytes; a kRangeCarry range gives crc0. Whole wave; nr <= 64.
__device__ __forceinline__ void fold_ranges(const std::uint8_t* win, const std::uint32_t* tab, const std::uint32_t* inj,
                                            const std::uint32_t* K, std::uint32_t poly, const dev::LaneConstX& kc,
                                            std::uint32_t lane, std::uint32_t* R, std::uint32_t nr) {
  std::uint32_t xi = 0, yi = 0, ci = 0, ki = 0;
  if (lane < nr) {
    const std::uint32_t w0 = R[3 * lane];
    xi = w0 & 0xFFFFu;
    yi = w0 >> 16;
    ci = (yi - xi + kChunk - 1u) / kChunk;
    ki = (R[3 * lane + 1] >> 9) & 3u;
    R[3 * lane + 2] = 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  std::uint32_t total;
  const std::uint32_t pre = lane_prefix(ci, &total);
  for (std::uint32_t base = 0; base < total; base += 64u) {
    const std::uint32_t g = base + lane;
    const bool act = g < total;
    std::uint32_t r = 0;  // the range of chunk g: the last one whose first chunk is at most g
    for (std::uint32_t i = 1; i < nr; ++i) r = g >= static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pre), static_cast<int>(i))) ? i : r;
    const std::uint32_t x = shfl_pos(xi, r), y = shfl_pos(yi, r), c = shfl_pos(ci, r), p = shfl_pos(pre, r);
    const std::uint32_t kd = shfl_pos(ki, r);
    const std::uint32_t k = g - p;                 // chunk from the range's front
    const std::uint32_t j = act ? c - 1u - k : 0u;  // chunk from its end
    const std::uint32_t ce = y - j * kChunk;
    const std::uint32_t cs = ce > x + kChunk ? ce - kChunk : x;
    const std::uint32_t L = act ? ce - cs : 0u;
    std::uint32_t v = fold_raw(win, tab, kc, cs, L);
    if (k == 0u && kd != kRangeCarry) v ^= inj[L];
    v = mul_lean(K[j], v, poly);
    if (act) atomicXor(&R[3 * r + 2], v);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

constexpr int kAhead = 2;  // regions in registers: the current one and the next, in flight
constexpr std::uint32_t kTrustHop = 2;      // whole regions a hop from an implausible header may pass over

// The record at window offset (r - rs) + o has a header the encoder could have written (wal.cpp:19-61):
// op and tombstone bytes 0 or 1, record_len = 18 + key_len + value_len. Wave-uniform r.
template <typename P>
__device__ __forceinline__ bool plausible_at(const std::uint8_t* win, P rs, std::uint32_t o, P r) {
  if (r == kNoneP<P>) return false;
  const std::uint32_t b = static_cast<std::uint32_t>(r - rs) + o;
  const std::uint64_t rl = rd32(win, b), kl = rd32(win, b + 18u), vl = rd32(win, b + 22u);
  return (rd32(win, b + 8u) & 0xFFu) <= 1u && (rd32(win, b + 17u) & 0xFFu) <= 1u && rl == 18u + kl + vl;
}

// Region r's granules: 1 KiB load rows k = 0..kRows-1, lane l's 16 bytes at row offset 16 l, as
// buffer loads through a descriptor over the region's first `rows` rows, cut at the image's end: the
// hardware range check returns zeros past it and fetches nothing (regions the wave will not write
// into its window have rows = 0). Every load is issued, so the compiler counts them exactly.
__device__ __forceinline__ void load_region(const SweepArgs& a, std::uint64_t r, std::uint32_t lane, int rows, uint4 (&g)[kRows]) {
  const std::uint64_t ad = a.al0 + r * kRegion;
  const std::uint64_t base = static_cast<std::uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(ad))) |
                             static_cast<std::uint64_t>(static_cast<std::uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(ad >> 32)))) << 32;
  const std::uint64_t left = a.gend > base ? a.gend - base : 0u;
  const std::uint32_t nrec = __builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(std::min<std::uint64_t>(left, 1024u * static_cast<std::uint32_t>(rows))));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, nrec, 0x00020000);
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16u * lane + 1024u * k, 0, 0);
    g[k] = uint4{v[0], v[1], v[2], v[3]};
  }
}

// One wave: regions [r0, limit) from entry e (kNone: search). Fix-up mode stops where the exit meets
// the stored entry of the next region. No global load in the loop waits for a value except in fix-up
// mode (a wait on a load drains every prefetch issued before it).
template <bool FIXUP, typename P>
__device__ __forceinline__ void sweep_wave(const SweepArgs& a, std::uint8_t* win, std::uint16_t* list, const std::uint32_t* tab,
                                           const std::uint32_t* inj, const std::uint32_t* K, std::uint32_t r0, std::uint32_t limit,
                                           P e, std::uint32_t wave, bool hop_giant) {
  constexpr P kNo = kNoneP<P>;
  const std::uint32_t lane = threadIdx.x & 63u;
  const dev::LaneConstX kc = dev::lane_const16(lane);
  const P size = static_cast<P>(a.size);
  const std::uint32_t o = a.o;
  const std::uint32_t poly = a.tabs->poly;
  // the last region whose granules this wave writes into its window: limit (the overlap of limit - 1)
  const std::uint32_t rlast = limit;
  uint4 buf[kAhead][kRows];
  auto rows_of = [&](std::uint64_t r) -> int { return r < rlast ? kRows : r == rlast ? 1 : 0; };
#pragma unroll
  for (int k = 0; k < kAhead; ++k) {
    load_region(a, static_cast<std::uint64_t>(r0) + k, lane, rows_of(static_cast<std::uint64_t>(r0) + k), buf[k]);
    // in order: the loop's waits count the loads issued after the ones they wait for, on entry as well
    __builtin_amdgcn_sched_barrier(0);
  }
  std::uint32_t spec_next = e == kNo ? kSpec : (FIXUP ? kFix : 0u);  // flags the next entry carries
  std::uint64_t nlong = 0;  // long payloads listed in this wave's segment
  // window <- region rr and the head of rr + 1; the buffer refilled with region rr + kAhead
  auto put = [&](std::uint32_t rr, uint4 (&cur)[kRows], const uint4& head) {
#pragma unroll
    for (int j = 0; j < kRows; ++j) *reinterpret_cast<uint4*>(win + 1024u * j + 16u * lane) = cur[j];
    if (lane < (16u + kOver) / 16u) *reinterpret_cast<uint4*>(win + kRegion + 16u * lane) = head;
    const std::uint64_t nxt = static_cast<std::uint64_t>(rr) + kAhead;
    load_region(a, nxt, lane, rows_of(nxt), cur);
  };
  // regions [j0, j1) lie inside the record the chain is in (it leaves at x past them): stored without
  // being loaded or walked
  auto pass_over = [&](std::uint32_t j0, std::uint32_t j1, P x) {
    for (std::uint32_t j = j0 + lane; j < j1; j += 64u) {
      std::uint32_t v = 0;
      if constexpr (FIXUP) v = (a.fl[j] >> 8) + 1u;
      a.E[j] = widen(x);
      a.X[j] = widen(x);
      a.B[j] = kNone;
      a.cnt[j] = 0;
      a.bidx[j] = 0xFFFFFFFFu;
      a.fl[j] = kChain | (v << 8);
      a.cm_len[j] = 0;
    }
  };
  // the region body: the next region to walk (limit: the wave stops; fix-up converged)
  auto body = [&](std::uint32_t rr) -> std::uint32_t {
    {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const P rs = static_cast<P>(rr) * kRegion;
      const P re = rs + kRegion;
      std::uint32_t ver = 0;
      if constexpr (FIXUP) ver = (a.fl[rr] >> 8) + 1u;
      // ---- 1. starts ------------------------------------------------------------------------------
      const P ps = rs + static_cast<P>(kPiece) * lane, pe = ps + kPiece;
      const bool exact = e != kNo;
      std::uint32_t flags;
      P Er = e, Xout = e, Lr = kNo;
      std::uint32_t count = 0, bad_k = 0xFFFFFFFFu;
      P Bpos = kNo;
      std::uint32_t carry_v = 0, cm_len = 0, cm_crc = 0, cm_part = 0, cm_pos = 0;
      // the whole region (up to the image's end) as one carry range: a region inside a record
      auto carry_whole = [&]() {
        const std::uint32_t n = size - rs < static_cast<P>(kRegion) ? static_cast<std::uint32_t>(size - rs) : kRegion;
        std::uint32_t* R = reinterpret_cast<std::uint32_t*>(list);
        if (lane == 0) {
          R[0] = o | (o + n) << 16;
          R[1] = kRangeCarry << 9;
        }
        fold_ranges(win, tab, inj, K, poly, kc, lane, R, 1u);
        carry_v = R[2];
      };
      if (exact && (e >= re || e >= size)) {
        flags = kChain | spec_next;  // inside a record, or past the chain's end: no starts here
        if (e >= re && e < size) carry_whole();
      } else {
       do {  // (breaks out to the region record)
        const std::uint32_t le = exact ? static_cast<std::uint32_t>((e - rs) / kPiece) : 0u;
        P s = kNo;
        if (exact && lane == le) s = e;
        // the piece's first plausible header (the whole piece in one search)
        const P qend = size >= kWalMeta ? std::min<P>(pe, size - static_cast<P>(kWalMeta) + 1u) : 0u;
        if ((!exact || lane > le) && ps < qend) s = search_piece<P, 8>(win, rs, o, ps, qend, size);
        Walk<P> wk;
        walk_piece(win, rs, o, s, pe, size, true, wk);
        // ---- 2. link check ---------------------------------------------------------------------------
        std::uint64_t C = __ballot(s != kNo);
        const std::uint32_t f = exact ? le : (C ? static_cast<std::uint32_t>(__builtin_ctzll(C)) : 64u);
        if (f == 64u) {
          flags = kSearch;
          Er = Xout = kNo;
          carry_whole();  // (on the true chain, a region without a start lies inside a record)
          break;
        }
        {
          C &= ~((1ull << f) - 1ull);
          std::uint32_t cur = f;
          for (;;) {
            const std::uint64_t below = C & ((1ull << lane) - 1ull);
            const std::uint32_t prev = below ? 63u - static_cast<std::uint32_t>(__builtin_clzll(below)) : lane;
            const P xp = shfl_pos(wk.x, prev);
            const bool bp = __shfl(static_cast<int>(wk.broke), static_cast<int>(prev), 64) != 0;
            const bool mine = ((C >> lane) & 1ull) && lane > cur;
            const std::uint64_t fails = __ballot(mine && (bp || xp != s));
            std::uint32_t pv;  // the last lane known to be on the chain, whose exit must be followed
            if (fails) {
              const std::uint32_t l0 = static_cast<std::uint32_t>(__builtin_ctzll(fails));
              pv = 63u - static_cast<std::uint32_t>(__builtin_clzll(C & ((1ull << l0) - 1ull)));
            } else {
              pv = 63u - static_cast<std::uint32_t>(__builtin_clzll(C));  // every link holds: the last lane
            }
            const P xv = readlane_pos(wk.x, pv);
            const bool bv = __builtin_amdgcn_readlane(static_cast<int>(wk.broke), static_cast<int>(pv)) != 0;
            if (bv || xv >= re || xv >= size) {  // the chain breaks, leaves the region or ends at pv
              C &= (2ull << pv) - 1ull;
              break;
            }
            // otherwise the chain goes on inside the region, at a lane whose start is not xv
            const std::uint32_t q = static_cast<std::uint32_t>((xv - rs) / kPiece);
            C &= ~(((1ull << q) - 1ull) & ~((2ull << pv) - 1ull));  // lanes strictly between drop out
            C |= 1ull << q;
            const bool me = lane == q;
            if (me) s = xv;
            walk_piece(win, rs, o, s, pe, size, me, wk);
            cur = q;
          }
          const std::uint32_t last = 63u - static_cast<std::uint32_t>(__builtin_clzll(C));
          Xout = readlane_pos(wk.x, last);
          const bool broke = __builtin_amdgcn_readlane(static_cast<int>(wk.broke), static_cast<int>(last)) != 0;
          Er = exact ? e : readlane_pos(s, f);
          flags = kChain | spec_next | (broke ? kBroke : 0u) | (!broke && Xout == size ? kEnd : 0u);
          Lr = readlane_pos(wk.lr, last);
          // ---- 3. list and fold ------------------------------------------------------------------------
          const bool on = (C >> lane) & 1ull;
          (void)lane_prefix(on ? wk.n : 0u, &count);  // every chain record
          // listed: each lane's records up to its first tiny one (all stored), in chain order
          const std::uint32_t nn = on ? std::min<std::uint32_t>(wk.n, wk.tiny == kStore ? kStore : wk.tiny + 1u) : 0u;
          std::uint32_t nlist;
          const std::uint32_t pre = lane_prefix(nn, &nlist);
          const std::uint32_t t = on && wk.tiny < nn ? pre + wk.tiny : 0xFFFFFFFFu;
          const std::uint32_t tmin = dev::wave_min(t);
          const std::uint32_t nl = std::min<std::uint32_t>(std::min<std::uint32_t>(nlist, tmin == 0xFFFFFFFFu ? nlist : tmin + 1u), kList);
#pragma unroll
          for (std::uint32_t j = 0; j < kStore; ++j)
            if (j < nn && pre + j < nl) list[pre + j] = static_cast<std::uint16_t>(wk.st[j]);
          // fold ranges behind the list: the bytes in front of the entry first (the record the chain is
          // in when it enters the region), then the payloads longer than kLaneFold, in chain order
          std::uint32_t* R = reinterpret_cast<std::uint32_t*>(list + ((nl + 1u) & ~1u));
          const std::uint32_t rcap = (2u * kList - 2u * ((nl + 1u) & ~1u)) / 12u;
          std::uint32_t nr = 0;
          const std::uint32_t eo = static_cast<std::uint32_t>(Er - rs) + o;  // the entry's window offset
          // a carry of at most kLaneFold bytes (the tail of a short record, usually) is one more lane job of
          // the record fold below; a longer one is range 0 of the range fold
          const bool carry_lane = Er > rs && eo - o <= kLaneFold;
          if (Er > rs && !carry_lane) {
            if (lane == 0) {
              R[0] = o | eo << 16;
              R[1] = kRangeCarry << 9;
            }
            nr = 1;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          const std::uint32_t njobs = nl + (carry_lane ? 1u : 0u);
          for (std::uint32_t base = 0; base < njobs; base += 64u) {
            const std::uint32_t kk = base + lane;
            const bool act = kk < nl;
            const bool cj = carry_lane && kk == nl;  // this lane folds the carry
            const std::uint32_t so = act ? list[kk] : 0u;
            const std::uint32_t b = so + o;
            const std::uint32_t rl = rd32(win, b), stored = rd32(win, b + 4u);
            const std::uint32_t kl = rd32(win, b + 18u), vl = rd32(win, b + 22u);
            const bool kv_ok = kWalMeta + static_cast<std::uint64_t>(kl) + vl <= 8ull + rl;  // wal.cpp:118-121
            const bool lng = act && rl > kLaneFold;
            const std::uint32_t fn = cj ? eo - o : act && !lng ? rl : 0u;
            const std::uint32_t raw = fold_raw(win, tab, kc, cj ? o : b + 8u, fn);
            const std::uint32_t crc = raw ^ inj[fn] ^ 0xFFFFFFFFu;
            if (carry_lane && base + 64u > nl)
              carry_v = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(raw), static_cast<int>(nl - base)));
            const bool bad = act && (!kv_ok || (!lng && crc != stored));
            // payloads up to kMedMax: a fold range of their bytes in the region (wholly inside it, or the
            // head of one that goes on); longer ones, or ones the ranges have no room for: the batch
            bool gnt = lng && rl > kMedMax;
            const bool med = lng && !gnt;
            const std::uint64_t mb = __ballot(med);
            if (mb) {
              const std::uint32_t at = nr + __builtin_amdgcn_mbcnt_hi(static_cast<std::uint32_t>(mb >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo(static_cast<std::uint32_t>(mb), 0u));
              if (med) {
                if (at < rcap) {
                  const std::uint32_t rend = o + kRegion, pa = b + 8u, pz = b + 8u + rl;
                  R[3 * at] = std::min(pa, rend) | std::min(pz, rend) << 16;
                  R[3 * at + 1] = kk | (pz <= rend ? kRangeWhole : kRangeHead) << 9 | b << 16;
                } else {
                  gnt = true;
                }
              }
              nr = std::min<std::uint32_t>(nr + static_cast<std::uint32_t>(__builtin_popcountll(mb)), rcap);
            }
            const std::uint64_t lb = __ballot(gnt);
            if (lb) {
              const std::uint32_t nb = static_cast<std::uint32_t>(__builtin_popcountll(lb));
              std::uint64_t at;
              if (!FIXUP && nlong + nb <= a.l_seg) {  // the wave's own segment: no atomic, no wait
                at = static_cast<std::uint64_t>(wave) * a.l_seg + nlong;
                nlong += nb;
              } else {
                at = 0;
                if (lane == static_cast<std::uint32_t>(__builtin_ctzll(lb)))
                  at = atomicAdd(&a.res[kResLongA], static_cast<unsigned long long>(nb));
                at = a.l_seg * a.wsweep + dev::readlane64(at, static_cast<std::uint32_t>(__builtin_ctzll(lb)));
              }
              const std::uint64_t idx = at + __builtin_amdgcn_mbcnt_hi(static_cast<std::uint32_t>(lb >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo(static_cast<std::uint32_t>(lb), 0u));
              if (gnt && idx < a.l_cap) {
                a.l_off[idx] = static_cast<std::uint64_t>(rs) + so + 8u;
                a.l_len[idx] = rl;
                a.l_crc[idx] = stored;
                a.l_reg[idx] = rr;
                a.l_meta[idx] = kk | (ver << 9);  // (kk < 512)
              }
            }
            const std::uint64_t bk = __ballot(bad);
            if (bk && bad_k == 0xFFFFFFFFu) bad_k = base + static_cast<std::uint32_t>(__builtin_ctzll(bk));
          }
          if (nr) {
            fold_ranges(win, tab, inj, K, poly, kc, lane, R, nr);
            // results, one range per lane: the carry, whole payloads checked here, the crossing one kept
            std::uint32_t kd = 0, kki = 0, bo = 0, acc = 0, x = 0, y = 0;
            if (lane < nr) {
              x = R[3 * lane] & 0xFFFFu;
              y = R[3 * lane] >> 16;
              const std::uint32_t w1 = R[3 * lane + 1];
              kki = w1 & 0x1FFu;
              kd = (w1 >> 9) & 3u;
              bo = w1 >> 16;
              acc = R[3 * lane + 2];
            }
            if (Er > rs && !carry_lane) carry_v = static_cast<std::uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(acc)));
            const std::uint32_t st = lane < nr && kd != kRangeCarry ? rd32(win, bo + 4u) : 0u;
            const bool mbad = lane < nr && kd == kRangeWhole && (acc ^ 0xFFFFFFFFu) != st;
            const std::uint32_t mk = dev::wave_min(mbad ? kki : 0xFFFFFFFFu);
            bad_k = std::min(bad_k, mk);
            const std::uint64_t hb = __ballot(lane < nr && kd == kRangeHead);
            if (hb) {  // (at most one: the region's last record)
              const std::uint32_t h = static_cast<std::uint32_t>(__builtin_ctzll(hb));
              cm_len = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rd32(win, bo)), static_cast<int>(h)));
              cm_crc = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(st), static_cast<int>(h)));
              cm_part = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x == y ? 0xFFFFFFFFu : acc), static_cast<int>(h)));
              cm_pos = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>((bo - o) | kki << 16), static_cast<int>(h)));
            }
          }
          if (bad_k != 0xFFFFFFFFu) Bpos = rs + list[bad_k];
        }
       } while (false);
      }
      // ---- 4. region record, next entry --------------------------------------------------------------
      bool stop = false;
      P next_e = kNo;
      std::uint32_t next_spec = kSpec;
      if ((flags & kChain) && !(flags & kBroke)) {  // (after kEnd: size, past every later region)
        next_e = Xout;
        next_spec = 0u;
      }
      // A record that covers whole regions: longer than kMedMax, they are passed over (the batch checks
      // it); up to kMedMax, walked one by one (their bytes are folded as carries). A region inside one
      // (no record walked) continues the hop that led there.
      bool ghop = false;
      if ((flags & kChain) && !(flags & kBroke) && Xout < size && Xout / kRegion > static_cast<P>(rr) + 1u) {
        if (Lr != kNo) hop_giant = Xout - Lr - 8u > static_cast<P>(kMedMax);
        ghop = hop_giant;
      }
      if (ghop) flags |= kGiantHop;
      // A hop over more than kTrustHop regions from a header the encoder could not have written (a fake
      // chain reading a random record_len): see the pass-over below.
      const bool fake_hop = ghop && Lr != kNo && Xout / kRegion > static_cast<P>(rr) + 1u + kTrustHop &&
                            !plausible_at(win, rs, o, Lr);
      if (fake_hop) flags |= kFakeHop;
      if constexpr (FIXUP) {
        // converged: the next region's stored chain enters where this one leaves
        if (rr + 1u >= limit || (flags & (kBroke | kEnd)) || !(flags & kChain)) {
          stop = true;
        } else {
          const std::uint32_t nf = a.fl[rr + 1u];
          if ((nf & kChain) && a.E[rr + 1u] == widen(next_e)) stop = true;
        }
      }
      switch (lane) {
        case 0: a.E[rr] = widen(Er); break;
        case 1: a.X[rr] = widen(Xout); break;
        case 2: a.B[rr] = widen(Bpos); break;
        case 3: a.cnt[rr] = count; break;
        case 4: a.bidx[rr] = bad_k; break;
        case 5: a.fl[rr] = flags | (ver << 8); break;
        case 6: a.carry[rr] = carry_v; break;
        case 7: a.cm_len[rr] = cm_len; break;
        case 8: a.cm_crc[rr] = cm_crc; break;
        case 9: a.cm_part[rr] = cm_part; break;
        case 10: a.cm_pos[rr] = cm_pos; break;
        default: break;
      }
      e = next_e;
      spec_next = next_spec;
      std::uint32_t nx = stop ? limit : rr + 1u;
      if (!stop && (flags & kChain) && !(flags & kBroke)) {
        // the chain's current record covers whole regions: store them, go on where it ends
        const std::uint32_t qr = static_cast<std::uint32_t>(next_e / kRegion);
        const std::uint32_t q = next_e >= size || qr > limit ? limit : qr;
        if (q > rr + 1u && (next_e >= size || ghop)) {
          // A fake hop (kFakeHop) is not passed over: the regions behind it are walked from their own
          // searches, and the boundary check takes the hop's landing like a chunk's (its fix-up task waits
          // until it is the first failing boundary, whose exit is on the true chain; that task, whose entry
          // lies past its first region, passes over). In a fix-up task too: one that started from a fake
          // exit would otherwise store its landing in every region it jumps, and the true chain's task
          // could not meet a stored entry again before its limit.
          if (fake_hop && next_e < size) {
            e = kNo;
            spec_next = kSpec;
            return rr + 1u;
          }
          pass_over(rr + 1u, q, next_e);
          nx = q;
          if constexpr (FIXUP) {
            if (q < limit && (a.fl[q] & kChain) && a.E[q] == widen(next_e)) nx = limit;  // converged
          }
        }
      }
      return nx;
    }
  };
  bool done = false;
  std::uint32_t walked = 0;  // regions this wave walked (fix-up statistics)
  for (std::uint32_t r = r0; r < limit && !done; r += kAhead) {
#pragma unroll
    for (int k = 0; k < kAhead; ++k) {
      const std::uint32_t rr = r + static_cast<std::uint32_t>(k);
      if (done || rr >= limit) {
        done = true;
        break;
      }
      put(rr, buf[k], buf[(k + 1) % kAhead][0]);
      const std::uint32_t nx = body(rr);
      ++walked;
      if (nx >= limit) {
        done = true;
      } else if (nx != rr + 1u) {  // passed over regions: the pipeline restarts at nx
        load_region(a, nx, lane, rows_of(nx), buf[(k + 1) % kAhead]);
        load_region(a, static_cast<std::uint64_t>(nx) + 1u, lane, rows_of(static_cast<std::uint64_t>(nx) + 1u), buf[k]);
        r = nx - static_cast<std::uint32_t>(k) - 1u;
      }
    }
  }
  if (!FIXUP && lane == 0) a.l_cnt[wave] = static_cast<std::uint32_t>(nlong);
  if (FIXUP && lane == 0) {
    atomicMax(&a.res[kResWalkMax], static_cast<unsigned long long>(walked));
    atomicAdd(&a.res[kResWalkSum], static_cast<unsigned long long>(walked));
  }
}

template <bool FIXUP, typename P>
__global__ __launch_bounds__(kSweepThreads) void wal_sweep(SweepArgs a) {
  // one block with the tables at LDS address 0, so a lookup's v_perm result is its address
  __shared__ __attribute__((aligned(16))) std::uint8_t lds[kLdsSliceWords * 2 + kSweepWaves * kWinBytes + 4 * (kLaneFold + 1) + 4 * 64];
  std::uint32_t* tab = reinterpret_cast<std::uint32_t*>(lds);
  std::uint8_t (*wins)[kWinBytes] = reinterpret_cast<std::uint8_t (*)[kWinBytes]>(lds + kLdsSliceWords * 2);
  std::uint32_t* inj = reinterpret_cast<std::uint32_t*>(lds + kLdsSliceWords * 2 + kSweepWaves * kWinBytes);  // Shift_L(0xFFFFFFFF)
  std::uint32_t* K = inj + kLaneFold + 1;  // x^(8 kChunk j), j < 64
  dev::fill_lds_slicing16(a.tabs, tab);
  for (std::uint32_t i = threadIdx.x; i <= kLaneFold; i += blockDim.x) inj[i] = a.tabs->init_shift[i];
  if (threadIdx.x < 64u) K[threadIdx.x] = x8n(a.tabs, kChunk * threadIdx.x);
  __syncthreads();
  const std::uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t w = blockIdx.x * kSweepWaves + wv;
  if (w >= a.nwaves) return;
  std::uint8_t* win = wins[wv];
  std::uint16_t* list = reinterpret_cast<std::uint16_t*>(win + kWin);
  if constexpr (!FIXUP) {
    const std::uint32_t r0 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(w) * a.nreg / a.nwaves);
    const std::uint32_t r1 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(w + 1) * a.nreg / a.nwaves);
    sweep_wave<false, P>(a, win, list, tab, inj, K, r0, r1, r0 == 0 ? P(0) : kNoneP<P>, w, false);
  } else {
    const std::uint32_t b = a.t_begin[w];
    // a task whose entry lies past its first region continues its predecessor's hop
    const bool giant = b > 0u && (a.fl[b - 1u] & kGiantHop) != 0u;
    sweep_wave<true, P>(a, win, list, tab, inj, K, b, a.t_limit[w], static_cast<P>(a.t_entry[w]), w, giant);
  }
}

// Dense long-payload list for the CRC batch: the sweep waves' segments, then the atomic area.
// One block of kFinThreads threads scans the per-wave counts (block 0 of wal_after); every block of
// wal_long_gather copies its entries.
constexpr unsigned kFinThreads = 256;
__device__ void long_scan_block(const std::uint32_t* l_cnt, std::uint32_t W, std::uint64_t* l_base, unsigned long long* res) {
  __shared__ std::uint64_t part[kFinThreads];
  const std::uint32_t t = threadIdx.x;
  const std::uint32_t per = (W + kFinThreads - 1u) / kFinThreads;
  std::uint64_t s = 0;
  for (std::uint32_t i = 0; i < per; ++i) {
    const std::uint32_t w = t * per + i;
    if (w < W) s += l_cnt[w];
  }
  part[t] = s;
  __syncthreads();
  for (std::uint32_t d = 1; d < kFinThreads; d <<= 1) {
    const std::uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  std::uint64_t run = t ? part[t - 1] : 0;
  for (std::uint32_t i = 0; i < per; ++i) {
    const std::uint32_t w = t * per + i;
    if (w < W) {
      l_base[w] = run;
      run += l_cnt[w];
    }
  }
  if (t == kFinThreads - 1u) {
    l_base[W] = part[kFinThreads - 1u];
    res[kResLongSeg] = part[kFinThreads - 1u];
  }
}
// entry j of the dense list (d_*) <- wave w's segment / the atomic area
__global__ void wal_long_gather(SweepArgs a, const std::uint64_t* l_base, std::uint32_t W, const unsigned long long* res,
                                std::uint64_t* d_off, std::uint32_t* d_len, std::uint32_t* d_crc, std::uint32_t* d_reg,
                                std::uint32_t* d_meta) {
  const std::uint64_t nseg = l_base[W];
  const std::uint64_t n_atomic = std::min<std::uint64_t>(res[kResLongA], a.l_cap - a.l_seg * W);
  const std::uint64_t j = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (j >= nseg + n_atomic) return;
  std::uint64_t src;
  if (j < nseg) {
    std::uint32_t lo = 0, hi = W;  // the wave whose range holds j
    while (hi - lo > 1) {
      const std::uint32_t mid = (lo + hi) / 2;
      if (l_base[mid] <= j) lo = mid;
      else hi = mid;
    }
    src = static_cast<std::uint64_t>(lo) * a.l_seg + (j - l_base[lo]);
  } else {
    src = a.l_seg * W + (j - nseg);
  }
  // Entries of superseded walks (a stale version) or at or past the settled chain's first bad short
  // record / break (res P, Q of a fin pass without long payloads) are not folded: speculative chains
  // list records of any length, hundreds of MB each. They go to the batch empty and marked stale.
  const std::uint64_t off = a.l_off[src];
  const std::uint32_t reg = a.l_reg[src], meta = a.l_meta[src];
  const bool live = (meta >> 9) == (a.fl[reg] >> 8) && off - 8u < std::min<std::uint64_t>(res[kResP], res[kResQ]);
  d_off[j] = off;
  d_len[j] = live ? a.l_len[src] : 0u;
  d_crc[j] = a.l_crc[src];
  d_reg[j] = reg;
  d_meta[j] = live ? meta : 0xFFFFFFFFu;
}

// Boundary checks: region p ends a chain segment when the next region's entry did not come from p
// (it searched, or was entered by a search or a fix-up). Unless the chain ended in p, p's exit X must
// land exactly on the entry of region q = X / kRegion, and every region between must hold no chain
// (it searched) or be inside the same record (a chain region entered at X: a fix-up's, carried
// through the record). A chain region whose entry lies past its own end was carried there, so the
// rule is exact. Failing p go to the list.
__device__ void bounds_one(const SweepArgs& a, std::uint64_t p, std::uint32_t* inc_p, std::uint64_t* inc_x, std::uint32_t cap) {
  if (p + 1 >= a.nreg) return;
  const std::uint32_t f = a.fl[p] & 0xFFu;
  if (!(f & kChain) || (f & (kBroke | kEnd))) return;
  if (!(a.fl[p + 1] & (kSpec | kSearch | kFix))) return;
  const std::uint64_t x = a.X[p];
  const std::uint64_t q = x / kRegion;
  bool ok = q > p && q < a.nreg;
  for (std::uint64_t j = p + 1; ok && j < q; ++j) {
    const std::uint32_t fj = a.fl[j];
    ok = (fj & kSearch) || ((fj & kChain) && a.E[j] == x);
  }
  if (ok) ok = (a.fl[q] & kChain) && a.E[q] == x;
  if (!ok) {
    atomicMin(&a.res[kResFirst], static_cast<unsigned long long>(p));
    const unsigned long long i = atomicAdd(&a.res[kResIncons], 1ull);
    if (i < cap) {
      inc_p[i] = static_cast<std::uint32_t>(p);
      inc_x[i] = x | ((f & kFakeHop) ? kFakeHopBit : 0ull);
    }
  }
}

__global__ void wal_reset(unsigned long long* res, int lo, int hi) {
  const int i = lo + static_cast<int>(threadIdx.x);
  if (i < hi) res[i] = (i == kResP || i == kResQ || i == kResFirst) ? ~0ull : 0ull;
}

// The payload of region r's crossing record (kLaneFold < record_len <= kMedMax, going on past the
// region's end): its register after the region (cm_part) carried through the regions it covers,
// r' = Shift_n(r) ^ carry[q] for the n payload bytes of region q (carry[q] = crc0 of [rs_q, min(E_q, re_q)),
// and E_q = its end in the last one). A payload that starts past rs_q (the record's 8-byte prefix cut
// by the region end) has those prefix bytes h in front of it in carry[q]: crc0(h || p) =
// Shift_|p|(crc0(h)) ^ crc0(p), so r' = Shift_|p|(r ^ crc0(h)) ^ carry[q]. True when it fails its stored
// CRC (wal.cpp:86-93); *pos = the record's start, *idx = its index in the region's list.
__device__ bool crossing_bad(const SweepArgs& a, std::uint64_t r, std::uint64_t* pos, std::uint32_t* idx) {
  const std::uint32_t len = a.cm_len[r];
  if (len == 0u) return false;
  const std::uint32_t f = a.fl[r];
  if (!(f & kChain) || (f & kBroke)) return false;
  const DeviceTables* t = a.tabs;
  const std::uint32_t cp = a.cm_pos[r];
  const std::uint64_t s = r * kRegion + (cp & 0xFFFFu), A = s + 8u, B = A + len;
  std::uint32_t reg = a.cm_part[r];
  for (std::uint64_t q = r + 1u; q < a.nreg; ++q) {
    const std::uint64_t rsq = q * kRegion, req = rsq + kRegion, y = std::min(B, req);
    const std::uint32_t c = a.carry[q];
    if (A > rsq) {
      std::uint32_t h = 0;
      for (std::uint64_t i = rsq; i < A; ++i) h = (h >> 8) ^ t->slice[0][(h ^ a.w[i]) & 0xFFu];
      reg = shift_n(t, reg ^ h, static_cast<std::uint32_t>(y - A)) ^ c;
    } else {
      reg = shift_n(t, reg, static_cast<std::uint32_t>(y - rsq)) ^ c;
    }
    if (B <= req) break;
  }
  *pos = s;
  *idx = cp >> 16;
  return (reg ^ 0xFFFFFFFFu) != a.cm_crc[r];
}

// First bad record P (region lists, crossing payloads and, when their versions are current, the long
// payloads) and the chain's break Q.
__device__ void fin_min_one(const SweepArgs& a, std::uint64_t i, const std::uint32_t* got, std::uint64_t nlong) {
  if (i < a.nreg) {
    const std::uint32_t f = a.fl[i];
    if (f & kChain) {
      if (f & kBroke) atomicMin(&a.res[kResQ], static_cast<unsigned long long>(a.X[i]));
      const std::uint64_t b = a.B[i];
      if (b != kNone) atomicMin(&a.res[kResP], static_cast<unsigned long long>(b));
      std::uint64_t cpos;
      std::uint32_t cidx;
      if (crossing_bad(a, i, &cpos, &cidx)) atomicMin(&a.res[kResP], static_cast<unsigned long long>(cpos));
    }
  }
  if (i < nlong) {
    const std::uint32_t r = a.l_reg[i];
    if ((a.l_meta[i] >> 9) == (a.fl[r] >> 8) && got[i] != a.l_crc[i])
      atomicMin(&a.res[kResP], static_cast<unsigned long long>(a.l_off[i] - 8u));
  }
}

// After a sweep (one launch, kFinThreads per block): the long-payload scan (block 0, when scan), the
// boundary check of every region (bounds) and its share of P and Q (fmin).
struct AfterArgs {
  const std::uint32_t* l_cnt;
  std::uint32_t W;
  std::uint64_t* l_base;
  std::uint32_t* inc_p;
  std::uint64_t* inc_x;
  const std::uint32_t* got;
  std::uint64_t nlong;
  bool scan, bounds, fmin;
};
__global__ __launch_bounds__(kFinThreads) void wal_after(SweepArgs a, AfterArgs f) {
  std::uint32_t b = blockIdx.x;
  if (f.scan) {
    if (b == 0) {
      long_scan_block(f.l_cnt, f.W, f.l_base, a.res);
      return;
    }
    --b;
  }
  const std::uint64_t i = b * static_cast<std::uint64_t>(kFinThreads) + threadIdx.x;
  if (f.bounds) bounds_one(a, i, f.inc_p, f.inc_x, kMaxFix);
  if (f.fmin) fin_min_one(a, i, f.got, f.nlong);
}

__device__ __forceinline__ std::uint64_t res_load(const unsigned long long* r) {
  return __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Result words into the host's pinned block: [0] failing boundaries, [1] long payloads, [2] records
// good, [3] stop offset, [4] corrupted, [5] entries the atomic area was asked for, [6] the first failing
// boundary, [7]/[8] the fix-up walk statistics.
__device__ void publish_one(const SweepArgs& a, std::uint64_t* h) {
  const std::uint64_t P = res_load(&a.res[kResP]), Q = res_load(&a.res[kResQ]);
  h[0] = res_load(&a.res[kResIncons]);
  h[1] = res_load(&a.res[kResLongSeg]) + std::min<std::uint64_t>(res_load(&a.res[kResLongA]), a.l_cap - a.l_seg * a.wsweep);
  h[5] = res_load(&a.res[kResLongA]);
  h[6] = res_load(&a.res[kResFirst]);
  h[7] = res_load(&a.res[kResWalkMax]);
  h[8] = res_load(&a.res[kResWalkSum]);
  if (P < Q) {
    h[2] = res_load(&a.res[kResCnt]) + res_load(&a.res[kResLidx]);
    h[3] = P;
    h[4] = 1;
  } else {
    h[2] = res_load(&a.res[kResCnt]);
    h[3] = Q == kNone ? a.size : Q;
    h[4] = Q == kNone ? 0 : 1;
  }
}

// Records before the stop (block sums of cnt over the regions before it) and the first bad record's
// index within its region; the last block to finish publishes the result words.
__global__ __launch_bounds__(512) void wal_finish(SweepArgs a, const std::uint32_t* got, std::uint64_t nlong, std::uint64_t* h) {
  __shared__ unsigned long long part[8];
  __shared__ bool last;
  const std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  const std::uint64_t P = a.res[kResP], Q = a.res[kResQ];
  const bool bad = P < Q;
  const std::uint64_t stop = bad ? P : Q;
  const std::uint64_t rb = stop == kNone ? a.nreg : stop / kRegion;
  std::uint64_t c = 0;
  if (i < a.nreg) {
    const std::uint32_t f = a.fl[i];
    if ((f & kChain) && (i < rb || (i == rb && !bad))) c = a.cnt[i];
    if (bad && i == rb) {
      std::uint64_t cpos;
      std::uint32_t cidx;
      if (a.B[i] == P) atomicExch(&a.res[kResLidx], static_cast<unsigned long long>(a.bidx[i]));
      else if (crossing_bad(a, i, &cpos, &cidx) && cpos == P) atomicExch(&a.res[kResLidx], static_cast<unsigned long long>(cidx));
    }
  }
  if (bad && i < nlong) {
    const std::uint32_t r = a.l_reg[i];
    if ((a.l_meta[i] >> 9) == (a.fl[r] >> 8) && got[i] != a.l_crc[i] && a.l_off[i] - 8u == P)
      atomicExch(&a.res[kResLidx], static_cast<unsigned long long>(a.l_meta[i] & 0x1FFu));
  }
  // block sum
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) c += static_cast<std::uint64_t>(__shfl_xor(static_cast<long long>(c), m, 64));
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = c;
  __threadfence();  // every wave's Lidx exchange done and visible before the block counts itself in
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (unsigned k = 0; k < blockDim.x / 64u; ++k) s += part[k];
    if (s) atomicAdd(&a.res[kResCnt], s);
    __threadfence();
    last = atomicAdd(&a.res[kResDone], 1ull) == gridDim.x - 1u;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    publish_one(a, h);
    a.res[kResDone] = 0;
  }
}

// The result words alone (fix-up rounds).
__global__ void wal_publish(SweepArgs a, std::uint64_t* h) {
  if (threadIdx.x == 0) publish_one(a, h);
}

// Per-device scratch, grown by doubling and kept between calls (guarded by mu).
struct WalScratch {
  std::mutex mu;
  std::uint64_t cap_reg = 0, cap_raw = 0, cap_dense = 0;
  std::uint32_t cap_waves = 0;
  void* regs = nullptr;   // per region: E, X, B (u64), cnt, bidx, fl, carry, cm_len, cm_crc, cm_part, cm_pos (u32)
  void* raw = nullptr;    // long payloads as the sweep lists them: off (u64), len, crc, reg, meta (u32)
  void* dense = nullptr;  // the same, gathered for the CRC batch, and got (u32)
  std::uint32_t* l_cnt = nullptr;   // per sweep wave, then the scan's bases (u64)
  std::uint64_t* l_base = nullptr;
  unsigned long long* res = nullptr;
  std::uint64_t* h_res = nullptr;   // pinned, kHres words
  std::uint64_t* d_hres = nullptr;  // device view of h_res
  // failing boundaries (device) and fix-up tasks (pinned, read by the kernel in place)
  std::uint32_t* inc_p = nullptr;
  std::uint64_t* inc_x = nullptr;
  std::uint32_t* h_inc_p = nullptr;  // pinned copies for the host's pruning
  std::uint64_t* h_inc_x = nullptr;
  std::uint32_t* h_task = nullptr;   // pinned: begin[kMaxFix], limit[kMaxFix], entry (u64)[kMaxFix]
  std::uint32_t* d_task = nullptr;
  // host images: device copy, pinned staging slabs for pageable sources, own streams
  std::uint8_t* d_img = nullptr;
  std::uint64_t cap_img = 0;
  std::uint8_t* slab[2] = {nullptr, nullptr};
  hipEvent_t slab_free[2] = {nullptr, nullptr};
  hipStream_t st = nullptr;   // copies of host images
  hipStream_t stc = nullptr;  // device work on host images
  int ncu = 0;
  ~WalScratch() {
    if (st) (void)hipStreamSynchronize(st);
    if (stc) (void)hipStreamSynchronize(stc);
    if (stc) (void)hipStreamDestroy(stc);
    (void)hipFree(d_img);
    for (int i = 0; i < 2; ++i) {
      (void)hipHostFree(slab[i]);
      if (slab_free[i]) (void)hipEventDestroy(slab_free[i]);
    }
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(regs);
    (void)hipFree(raw);
    (void)hipFree(dense);
    (void)hipFree(l_cnt);
    (void)hipFree(l_base);
    (void)hipFree(res);
    (void)hipFree(inc_p);
    (void)hipFree(inc_x);
    (void)hipHostFree(h_res);
    (void)hipHostFree(h_inc_p);
    (void)hipHostFree(h_inc_x);
    (void)hipHostFree(h_task);
  }
};
// Fix-up rounds before the exact host walk takes over. The first failing boundary moves forward every
// round, so the rounds are bounded by the boundaries; none of the adversarial images needs more than a
// handful, and each round costs two host syncs.
constexpr std::uint64_t kRoundBudget = 256;

std::mutex g_wal_mu;
WalScratch* g_wal[64] = {};

// What the calling thread's last WAL verify did (tkv_debug_wal_last).
thread_local std::uint64_t g_last[4] = {0, 0, 0, 0};  // rounds, host walk needed, image copied, no fix-up
// per fix-up round of the calling thread's last verify: failing boundaries, tasks, the longest task's
// range and all tasks' ranges in regions, the most regions one task walked and all walked regions
// (tkv_debug_wal_rounds)
thread_local std::vector<std::uint64_t> g_rounds;

#define WAL_HIP(call)                                                            \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) return set_error(TKV_IO_ERROR, hipGetErrorString(e_)); \
  } while (0)

unsigned blocks(std::uint64_t n, unsigned t) { return static_cast<unsigned>((n + t - 1) / t); }

int grow(void** p, std::uint64_t* cap, std::uint64_t want, std::uint64_t unit) {
  if (want <= *cap) return TKV_OK;
  const std::uint64_t c = std::max<std::uint64_t>(want, 2 * *cap);
  WAL_HIP(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  WAL_HIP(hipMalloc(p, c * unit));
  *cap = c;
  return TKV_OK;
}

constexpr std::uint64_t kRawUnit = 8 + 4 * 4, kDenseUnit = 8 + 5 * 4;

// Long-payload arrays of the raw (sweep) or dense (batch) layout.
void long_view(void* base, std::uint64_t cap, SweepArgs* a, std::uint32_t** got) {
  auto* l8 = static_cast<std::uint64_t*>(base);
  a->l_off = l8;
  auto* l4 = reinterpret_cast<std::uint32_t*>(l8 + cap);
  a->l_len = l4;
  a->l_crc = l4 + cap;
  a->l_reg = l4 + 2 * cap;
  a->l_meta = l4 + 3 * cap;
  if (got) *got = l4 + 4 * cap;
}

SweepArgs carve(WalScratch& s, const std::uint8_t* w, std::uint64_t size, std::uint32_t nreg, std::uint32_t W,
                std::uint64_t seg, const DeviceTables* tabs) {
  SweepArgs a{};
  a.w = w;
  a.size = size;
  const std::uintptr_t wp = reinterpret_cast<std::uintptr_t>(w);
  a.al0 = wp & ~static_cast<std::uintptr_t>(15);
  a.gend = ((wp + size - 1) & ~static_cast<std::uintptr_t>(15)) + 16u;
  a.o = static_cast<std::uint32_t>(wp - a.al0);
  a.nreg = nreg;
  a.nwaves = W;
  a.wsweep = W;
  const std::uint64_t C = s.cap_reg;
  auto* p8 = static_cast<std::uint64_t*>(s.regs);
  a.E = p8;
  a.X = p8 + C;
  a.B = p8 + 2 * C;
  auto* p4 = reinterpret_cast<std::uint32_t*>(p8 + 3 * C);
  a.cnt = p4;
  a.bidx = p4 + C;
  a.fl = p4 + 2 * C;
  a.carry = p4 + 3 * C;
  a.cm_len = p4 + 4 * C;
  a.cm_crc = p4 + 5 * C;
  a.cm_part = p4 + 6 * C;
  a.cm_pos = p4 + 7 * C;
  long_view(s.raw, s.cap_raw, &a, nullptr);
  a.l_cap = s.cap_raw;
  a.l_seg = seg;
  a.l_cnt = s.l_cnt;
  a.res = s.res;
  a.tabs = tabs;
  return a;
}

// The calling thread's device's scratch (created on first use).
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
    hipDeviceProp_t prop;
    WAL_HIP(hipGetDeviceProperties(&prop, dev));
    sp->ncu = prop.multiProcessorCount;
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->inc_p), kMaxFix * sizeof(std::uint32_t)));
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->inc_x), kMaxFix * sizeof(std::uint64_t)));
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_inc_p), kMaxFix * sizeof(std::uint32_t), hipHostMallocDefault));
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_inc_x), kMaxFix * sizeof(std::uint64_t), hipHostMallocDefault));
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_task), kMaxFix * 16, hipHostMallocDefault));
    WAL_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&sp->d_task), sp->h_task, 0));
    WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&sp->h_res), kHres * sizeof(std::uint64_t), hipHostMallocDefault));
    WAL_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&sp->d_hres), sp->h_res, 0));
    WAL_HIP(hipStreamCreateWithFlags(&sp->st, hipStreamNonBlocking));
    WAL_HIP(hipStreamCreateWithFlags(&sp->stc, hipStreamNonBlocking));
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->res), kResWords * sizeof(unsigned long long)));
    const std::uint32_t wmax = static_cast<std::uint32_t>(sp->ncu) * kSweepWaves;
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->l_cnt), (wmax + 1) * sizeof(std::uint32_t)));
    WAL_HIP(hipMalloc(reinterpret_cast<void**>(&sp->l_base), (wmax + 1) * sizeof(std::uint64_t)));
    sp->cap_waves = wmax;
  }
  *out = sp;
  return TKV_OK;
}

// fin_min, fin_count, publish (long payloads from the dense list when nlong > 0).
// wal_after (scan: the long-payload scan; bounds: the boundary checks; P and Q always, with the long
// payloads from the dense list when nlong > 0), then, when finish, wal_finish (counts and the result words).
void launch_after(SweepArgs a, WalScratch& s, std::uint32_t W, std::uint64_t nlong, bool scan, bool bounds, bool finish,
                  hipStream_t st) {
  std::uint32_t* got = nullptr;
  if (nlong) long_view(s.dense, s.cap_dense, &a, &got);
  const std::uint64_t n = std::max<std::uint64_t>(a.nreg, nlong);
  const AfterArgs f{s.l_cnt, W, s.l_base, s.inc_p, s.inc_x, got, nlong, scan, bounds, true};
  hipLaunchKernelGGL(wal_after, dim3(blocks(n, kFinThreads) + (scan ? 1u : 0u)), dim3(kFinThreads), 0, st, a, f);
  if (finish) hipLaunchKernelGGL(wal_finish, dim3(blocks(n, 512)), dim3(512), 0, st, a, got, nlong, s.d_hres);
}

// The verify of [w, w + size) on `st` (synchronous). Caller holds s.mu.
int verify_locked(WalScratch& s, const std::uint8_t* w, std::uint64_t size, std::uint64_t* n_good,
                  std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk) {
  const DeviceTables* tabs = device_tables(kAlgoCrc32);
  if (!tabs) return TKV_IO_ERROR;
  const std::uint64_t nreg64 = (size + kRegion - 1) / kRegion;
  if (nreg64 >= 0xFFFFFFF0ull) return set_error(TKV_INVALID_ARGUMENT, "WAL image too large for the device walk");
  const std::uint32_t nreg = static_cast<std::uint32_t>(nreg64);
  if (int rc = grow(&s.regs, &s.cap_reg, nreg, 3 * 8 + 8 * 4)) return rc;
  const std::uint32_t W = static_cast<std::uint32_t>(std::min<std::uint64_t>(nreg, s.cap_waves));
  // a wave's segment holds the long payloads of its chunk's chain (>= kLaneFold + 8 bytes apart);
  // more (speculative chains) and the fix-ups' go to the atomic area behind the segments
  const std::uint64_t seg = (static_cast<std::uint64_t>((nreg + W - 1) / W) * kRegion) / (kLaneFold + 8) + 16;
  std::uint64_t atomic_area = nreg / 4 + 4096;
  for (;;) {  // (once, unless the long-payload list overflows)
    if (int rc = grow(&s.raw, &s.cap_raw, seg * W + atomic_area, kRawUnit)) return rc;
    SweepArgs a = carve(s, w, size, nreg, W, seg, tabs);
    hipLaunchKernelGGL(wal_reset, dim3(1), dim3(64), 0, st, s.res, 0, static_cast<int>(kResWords));
    if (size <= kPos32Max)
      hipLaunchKernelGGL((wal_sweep<false, std::uint32_t>), dim3(blocks(W, kSweepWaves)), dim3(kSweepThreads), 0, st, a);
    else
      hipLaunchKernelGGL((wal_sweep<false, std::uint64_t>), dim3(blocks(W, kSweepWaves)), dim3(kSweepThreads), 0, st, a);
    launch_after(a, s, W, 0, true, true, true, st);
    WAL_HIP(hipGetLastError());
    WAL_HIP(hipStreamSynchronize(st));
    std::uint64_t rounds = 1;
    const bool clean = s.h_res[0] == 0;
    g_rounds.clear();
    // fix-up rounds: every failing boundary is walked again from its true exit (race-free ranges)
    while (s.h_res[0] != 0) {
      const std::uint64_t ninc = std::min<std::uint64_t>(s.h_res[0], kMaxFix);
      WAL_HIP(hipMemcpyAsync(s.h_inc_p, s.inc_p, ninc * 4, hipMemcpyDeviceToHost, st));
      WAL_HIP(hipMemcpyAsync(s.h_inc_x, s.inc_x, ninc * 8, hipMemcpyDeviceToHost, st));
      WAL_HIP(hipStreamSynchronize(st));
      // failing boundaries (p, exit X; bit 63 of X: p's exit is a fake hop), in region order
      std::vector<std::pair<std::uint32_t, std::uint64_t>> v(ninc);
      for (std::uint64_t i = 0; i < ninc; ++i) v[i] = {s.h_inc_p[i], s.h_inc_x[i]};
      std::sort(v.begin(), v.end());
      if (v[0].first != s.h_res[6]) {  // (more than kMaxFix failed: the list holds an arbitrary part) the first
        const std::uint32_t p0 = static_cast<std::uint32_t>(s.h_res[6]);
        std::uint64_t x0 = 0;
        WAL_HIP(hipMemcpy(&x0, a.X + p0, 8, hipMemcpyDeviceToHost));
        v.insert(v.begin(), {p0, x0});
        v.resize(std::min<std::size_t>(v.size(), kMaxFix));
      }
      std::vector<bool> fake(v.size());
      for (std::size_t k = 0; k < v.size(); ++k) {
        fake[k] = (v[k].second & kFakeHopBit) != 0;
        v[k].second &= ~kFakeHopBit;
      }
      // Tasks. The first failing boundary's exit is on the true chain (every boundary before it holds,
      // back to region 0): its task runs up to the first boundary past the record it lands in (the
      // ones inside that jump are covered by it). Every later boundary gets a task up to the next one
      // (disjoint ranges: no two tasks write one region) unless its exit lies past that range, or is a
      // fake hop (a random record_len read from an implausible header): such a task would pass a stretch
      // of regions over and store its landing in each, which the true chain's task must then walk again
      // region by region (1 GiB of record-valued records: 137 ms against 3.3); it waits until it is the
      // first failing boundary.
      std::vector<std::pair<std::uint32_t, std::uint64_t>> bnd;  // boundaries whose ranges are taken
      std::vector<bool> bfake;
      const std::uint64_t reach0 = v[0].second / kRegion;
      bnd.push_back(v[0]);
      bfake.push_back(fake[0]);
      for (std::size_t k = 1; k < v.size(); ++k)
        if (static_cast<std::uint64_t>(v[k].first) + 1 > reach0) {
          bnd.push_back(v[k]);
          bfake.push_back(fake[k]);
        }
      std::vector<std::pair<std::uint32_t, std::uint64_t>> kept;
      std::vector<std::uint32_t> kept_lim;
      for (std::size_t k = 0; k < bnd.size(); ++k) {
        const std::uint32_t lim = k + 1 < bnd.size() ? bnd[k + 1].first + 1 : nreg;
        if (k > 0 && (bnd[k].second / kRegion >= lim || bfake[k])) continue;
        kept.push_back(bnd[k]);
        kept_lim.push_back(lim);
      }
      std::uint32_t* tb = s.h_task;
      std::uint32_t* tl = s.h_task + kMaxFix;
      auto* te = reinterpret_cast<std::uint64_t*>(s.h_task + 2 * kMaxFix);
      for (std::size_t k = 0; k < kept.size(); ++k) {
        tb[k] = kept[k].first + 1;
        tl[k] = kept_lim[k];
        te[k] = kept[k].second;
      }
      std::uint64_t span_max = 0, span_sum = 0;
      for (std::size_t k = 0; k < kept.size(); ++k) {
        span_max = std::max<std::uint64_t>(span_max, tl[k] - tb[k]);
        span_sum += tl[k] - tb[k];
      }
      const std::size_t at = g_rounds.size();
      g_rounds.insert(g_rounds.end(), {s.h_res[0], kept.size(), span_max, span_sum, 0, 0});
      SweepArgs f = a;
      f.nwaves = static_cast<std::uint32_t>(kept.size());
      f.t_begin = s.d_task;
      f.t_limit = s.d_task + kMaxFix;
      f.t_entry = reinterpret_cast<const std::uint64_t*>(s.d_task + 2 * kMaxFix);
      hipLaunchKernelGGL(wal_reset, dim3(1), dim3(64), 0, st, s.res, static_cast<int>(kResIncons), static_cast<int>(kResFirst) + 1);
      hipLaunchKernelGGL(wal_reset, dim3(1), dim3(64), 0, st, s.res, static_cast<int>(kResWalkMax), static_cast<int>(kResWalkSum) + 1);
      if (size <= kPos32Max)
        hipLaunchKernelGGL((wal_sweep<true, std::uint32_t>), dim3(blocks(f.nwaves, kSweepWaves)), dim3(kSweepThreads), 0, st, f);
      else
        hipLaunchKernelGGL((wal_sweep<true, std::uint64_t>), dim3(blocks(f.nwaves, kSweepWaves)), dim3(kSweepThreads), 0, st, f);
      const AfterArgs fb{s.l_cnt, W, s.l_base, s.inc_p, s.inc_x, nullptr, 0, false, true, false};
      hipLaunchKernelGGL(wal_after, dim3(blocks(nreg, kFinThreads)), dim3(kFinThreads), 0, st, a, fb);
      hipLaunchKernelGGL(wal_publish, dim3(1), dim3(64), 0, st, a, s.d_hres);
      WAL_HIP(hipGetLastError());
      WAL_HIP(hipStreamSynchronize(st));
      g_rounds[at + 4] = s.h_res[7];
      g_rounds[at + 5] = s.h_res[8];
      ++rounds;
      if (rounds > kRoundBudget) {  // (never seen) the exact host walk decides instead
        *needs_host_walk = true;
        g_last[0] = rounds;
        g_last[1] = 1;
        return TKV_OK;
      }
    }
    g_last[0] = rounds;
    g_last[3] = clean ? 1 : 0;
    if (s.h_res[5] > atomic_area) {  // atomic area overflow: a larger one, walk again
      atomic_area = 2 * s.h_res[5];
      continue;
    }
    const std::uint64_t nlong = s.h_res[1];
    if (nlong || !clean) {
      if (nlong) {
        if (int rc = grow(&s.dense, &s.cap_dense, nlong, kDenseUnit)) return rc;
        SweepArgs d = a;
        std::uint32_t* got = nullptr;
        long_view(s.dense, s.cap_dense, &d, &got);
        // P and Q without the long payloads, on the settled chain: the gather folds only live entries
        hipLaunchKernelGGL(wal_reset, dim3(1), dim3(64), 0, st, s.res, static_cast<int>(kResP), static_cast<int>(kResCnt) + 1);
        launch_after(a, s, W, 0, false, false, false, st);
        hipLaunchKernelGGL(wal_long_gather, dim3(blocks(nlong, 256)), dim3(256), 0, st, a, s.l_base, W, s.res, d.l_off,
                           d.l_len, d.l_crc, d.l_reg, d.l_meta);
        WAL_HIP(hipGetLastError());
        if (int rc = batch_device_impl(kAlgoCrc32, w, d.l_off, d.l_len, nullptr, got, nlong, st)) return rc;
      }
      hipLaunchKernelGGL(wal_reset, dim3(1), dim3(64), 0, st, s.res, static_cast<int>(kResP), static_cast<int>(kResCnt) + 1);
      launch_after(a, s, W, nlong, false, false, true, st);
      WAL_HIP(hipGetLastError());
      WAL_HIP(hipStreamSynchronize(st));
    }
    *n_good = s.h_res[2];
    *stop_offset = s.h_res[3];
    return s.h_res[4] ? set_error(TKV_CORRUPTED, "corrupted WAL record") : TKV_OK;
  }
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
  if (pinned) {
    WAL_HIP(hipMemcpyAsync(s.d_img, h_wal, size, hipMemcpyHostToDevice, s.st));
  } else {
    // pageable: host threads fill one pinned slab while the copy engine drains the other
    for (int i = 0; i < 2; ++i) {
      if (!s.slab[i]) {
        WAL_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.slab[i]), kStageSlab, hipHostMallocDefault));
        WAL_HIP(hipEventCreateWithFlags(&s.slab_free[i], hipEventDisableTiming));
      }
    }
    int k = 0;
    for (std::uint64_t off = 0; off < size; off += kStageSlab, k ^= 1) {
      const std::uint64_t m = std::min(kStageSlab, size - off);
      WAL_HIP(hipEventSynchronize(s.slab_free[k]));
      stage_copy(s.slab[k], h_wal + off, m);
      WAL_HIP(hipMemcpyAsync(s.d_img + off, s.slab[k], m, hipMemcpyHostToDevice, s.st));
      WAL_HIP(hipEventRecord(s.slab_free[k], s.st));
    }
  }
  WAL_HIP(hipStreamSynchronize(s.st));
  return verify_locked(s, s.d_img, size, n_good, stop_offset, s.stc, needs_host_walk);
}

}  // namespace

int wal_verify_device_impl(const std::uint8_t* d_wal, std::uint64_t size, std::uint64_t* n_good,
                           std::uint64_t* stop_offset, hipStream_t st, bool* needs_host_walk) {
  *needs_host_walk = false;
  *n_good = 0;
  *stop_offset = 0;
  g_last[0] = g_last[1] = g_last[2] = g_last[3] = 0;
  g_rounds.clear();
  if (size == 0) return TKV_OK;
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
  g_rounds.clear();
  if (size == 0) return TKV_OK;
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

}  // namespace tkv

extern "C" void tkv_debug_wal_last(uint64_t out[4]) {
  for (int i = 0; i < 4; ++i) out[i] = tkv::g_last[i];
}

extern "C" size_t tkv_debug_wal_rounds(uint64_t* out, size_t n) {
  const std::size_t k = std::min(n, tkv::g_rounds.size());
  for (std::size_t i = 0; i < k; ++i) out[i] = tkv::g_rounds[i];
  return tkv::g_rounds.size();
}
