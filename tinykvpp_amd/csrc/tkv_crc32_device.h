// Device-side building blocks of the CRC-32 row kernel (gfx950). Included by the product kernels
// (tkv_crc32_kernels.hip) and by the variant explorer, whose extra variants live in
// tools/explore_device.h. Everything here is instantiated by the product kernels.
//
// Notation: Shift_n(v) = CRC register after n zero bytes from v (= v * x^(8n) mod P, reflected);
// crc_s(D) = Shift_|D|(s) ^ crc_0(D) — the register is affine in its initial value s.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "tkv_crc32_internal.h"

namespace tkv {
namespace dev {

// Global (VMEM) and constant (SMEM) address-space views.
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1))) g_v4u;
typedef const std::uint32_t __attribute__((address_space(1))) g_u32;
typedef const std::uint32_t __attribute__((address_space(4))) c_u32;
typedef const std::uint64_t __attribute__((address_space(4))) c_u64;

__device__ __forceinline__ uint4 gload16(std::uintptr_t p) {
  const v4u v = *reinterpret_cast<g_v4u*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// Keeps every dword of a loaded window live up to this point (call it where the window is folded). A
// window dword that no fold reads is dead as soon as its load is issued, and the compiler then reuses
// its register while the load is in flight, which costs a vmcnt(0) wait in front of every step and so
// drains the whole load pipeline.
template <int N>
__device__ __forceinline__ void keep_live(const uint4 (&g)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(g[i].x), "v"(g[i].y), "v"(g[i].z), "v"(g[i].w));
}
__device__ __forceinline__ std::uint32_t sload32(const std::uint32_t* p, std::uint32_t i) {
  return reinterpret_cast<c_u32*>(reinterpret_cast<std::uintptr_t>(p))[i];
}
__device__ __forceinline__ std::uint64_t sload64(const std::uint64_t* p, std::uint32_t i) {
  return reinterpret_cast<c_u64*>(reinterpret_cast<std::uintptr_t>(p))[i];
}
__device__ __forceinline__ std::uint32_t lds_at(const std::uint32_t* lds, std::uint32_t byte_addr) {
  return *reinterpret_cast<const std::uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// Per-lane constants of the LDS table image (see kLds* in tkv_crc32_internal.h).
struct LaneConst {
  std::uint32_t L0, L1, L2, L3;  // slicing tables T0..T3: {byte0 = t*128 + c*4, byte2 = pair}
  std::uint32_t lsbase;          // byte address of LS[0][0][lane]
};

__device__ __forceinline__ LaneConst lane_const(std::uint32_t lane) {
  const std::uint32_t c4 = (lane & 31u) << 2;
  return {c4, 128u + c4, 0x10000u + c4, 0x10080u + c4, kLdsLaneBase + lane * 4u};
}
__device__ __forceinline__ std::uint32_t xor3(std::uint32_t a, std::uint32_t b, std::uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32 truth table 0x96 = a ^ b ^ c
}

// One slicing-by-4 step over a little-endian dword: crc ^= w; crc = T3[b0]^T2[b1]^T1[b2]^T0[b3].
// v_perm_b32 drops byte j of x into byte1 of Lk (entry*256), giving the LDS byte address directly.
// The register is carried split as crc = t ^ u so each step costs 2 v_bitop3 + 4 v_perm.
struct Reg {
  std::uint32_t t, u;
  __device__ __forceinline__ std::uint32_t value() const { return t ^ u; }
};

__device__ __forceinline__ void slice4(const std::uint32_t* lds, Reg& r, std::uint32_t w, const LaneConst& k) {
  const std::uint32_t x = xor3(r.t, r.u, w);
  const std::uint32_t a0 = __builtin_amdgcn_perm(x, k.L3, 0x0C020400u);
  const std::uint32_t a1 = __builtin_amdgcn_perm(x, k.L2, 0x0C020500u);
  const std::uint32_t a2 = __builtin_amdgcn_perm(x, k.L1, 0x0C020600u);
  const std::uint32_t a3 = __builtin_amdgcn_perm(x, k.L0, 0x0C020700u);
  r.t = xor3(lds_at(lds, a0), lds_at(lds, a1), lds_at(lds, a2));
  r.u = lds_at(lds, a3);
}

// The 16-replica image read without bank conflicts. ds_read_b32 banks are (a/4) mod 32 within each
// 32-lane group, and table t of replica c sits in bank (16 t + c) mod 32, so lanes l and l + 16 of a
// group collide whenever they look up the same table. Here the half with lane bit 4 set takes the
// bytes of each pair in the other order (byte j = i ^ 1 in lookup i): in every lookup instruction the
// two halves use tables of opposite parity, i.e. disjoint banks. Each lane still looks up all four
// bytes, and the XOR of the four lookups does not depend on their order.
// The 64 KiB image (fill_lds_slicing16): 16 replicas, all four tables in one 256-byte row per entry
// (table t at bytes 64 t + 4 c), so the entry * 256 addressing of slice4 holds. Lane shifts are not
// in it.
struct LaneConstX {
  std::uint32_t L[4];  // byte 0 of the address: 64 t + 4 c for the table of lookup i's byte
  std::uint32_t S[4];  // v_perm selector dropping that byte of x into byte 1 (entry * 256)
  std::uint32_t L0;    // T0's offset for this lane (Sarwate steps)
};
__device__ __forceinline__ LaneConstX lane_const16(std::uint32_t lane) {
  const std::uint32_t c4 = (lane & 15u) << 2, h = (lane >> 4) & 1u;
  LaneConstX k;
  k.L0 = c4;
#pragma unroll
  for (std::uint32_t i = 0; i < 4u; ++i) {
    const std::uint32_t j = i ^ h;       // byte j of x goes through T(3 - j)
    k.L[i] = 64u * (3u - j) + c4;
    k.S[i] = 0x0C020400u | (j << 8);
  }
  return k;
}
__device__ __forceinline__ void slice4(const std::uint32_t* lds, Reg& r, std::uint32_t w, const LaneConstX& k) {
  const std::uint32_t x = xor3(r.t, r.u, w);
  const std::uint32_t a0 = __builtin_amdgcn_perm(x, k.L[0], k.S[0]);
  const std::uint32_t a1 = __builtin_amdgcn_perm(x, k.L[1], k.S[1]);
  const std::uint32_t a2 = __builtin_amdgcn_perm(x, k.L[2], k.S[2]);
  const std::uint32_t a3 = __builtin_amdgcn_perm(x, k.L[3], k.S[3]);
  r.t = xor3(lds_at(lds, a0), lds_at(lds, a1), lds_at(lds, a2));
  r.u = lds_at(lds, a3);
}

// Shift_{(63-lane)*64}(p): 8 lookups into this lane's nibble tables.
__device__ __forceinline__ std::uint32_t lane_shift(const std::uint32_t* lds, std::uint32_t p, const LaneConst& k) {
  std::uint32_t l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) l[j] = lds_at(lds, k.lsbase + 4096u * j + (((p >> (4 * j)) & 15u) << 8));
  return xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), l[6] ^ l[7]);
}


// XOR of v over the 64 lanes, complete in lane 63 (DPP: within rows of 16, then row broadcasts).
__device__ __forceinline__ std::uint32_t wave_xor_to_lane63(std::uint32_t v) {
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, false);  // row_mirror
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1,3
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2,3
  return v;
}

// Maximum of v over the 64 lanes, wave-uniform (the DPP pattern of wave_xor_to_lane63, then lane 63):
// VALU only, no LDS round trips (a shuffle-based reduction costs six dependent ds_bpermute).
__device__ __forceinline__ std::uint32_t wave_max(std::uint32_t v) {
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false)));
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false)));
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x141, 0xF, 0xF, false)));
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x140, 0xF, 0xF, false)));
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xA, 0xF, false)));
  v = std::max(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xC, 0xF, false)));
  return static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// Dword k of a window with its bytes in front of window byte `lead` zeroed, lead8 = 8 max(lead, 0):
// min(lead8 -sat 32 k, 32) bits from the bottom (a saturating subtract, a min, a shift and an AND).
__device__ __forceinline__ std::uint32_t mask_front(std::uint32_t d, std::uint32_t lead8, int k) {
  const std::uint32_t x = __builtin_elementwise_sub_sat(lead8, static_cast<std::uint32_t>(32 * k));
  return d & static_cast<std::uint32_t>(0xFFFFFFFFull << (x < 32u ? x : 32u));
}

// Exclusive prefix sum over the 64 lanes (all active), and its total: an inclusive scan by DPP row
// shifts within rows of 16, then the row totals broadcast into the rows above (row_bcast:15 / :31).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ std::uint32_t dpp_add(std::uint32_t x) {
  return x + static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ std::uint32_t lane_prefix(std::uint32_t v, std::uint32_t* total) {
  std::uint32_t x = v;
  x = dpp_add<0x111, 0xF>(x);  // row_shr:1
  x = dpp_add<0x112, 0xF>(x);  // row_shr:2
  x = dpp_add<0x114, 0xF>(x);  // row_shr:4
  x = dpp_add<0x118, 0xF>(x);  // row_shr:8
  x = dpp_add<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
  x = dpp_add<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
  *total = static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
  return x - v;
}

// Minimum of v over the 64 lanes, wave-uniform (as wave_max; lanes past a row's edge read ~0).
__device__ __forceinline__ std::uint32_t wave_min(std::uint32_t v) {
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0xB1, 0xF, 0xF, false)));
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x4E, 0xF, 0xF, false)));
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x141, 0xF, 0xF, false)));
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x140, 0xF, 0xF, false)));
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x142, 0xA, 0xF, false)));
  v = std::min(v, static_cast<std::uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x143, 0xC, 0xF, false)));
  return static_cast<std::uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// a*b mod P in the reflected representation (x^0 = 0x80000000).
__device__ __forceinline__ std::uint32_t multmodp(std::uint32_t a, std::uint32_t b, std::uint32_t poly) {
  std::uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ poly : (b >> 1);
  }
  return p;
}

// reg * x^(8*kRow*k) mod P.
__device__ __forceinline__ std::uint32_t shift_rows(const DeviceTables* t, std::uint32_t reg, std::uint32_t k) {
  const std::uint32_t poly = t->poly;
  std::uint32_t m = 0x80000000u;  // x^0
  for (int i = 0; k != 0; ++i, k >>= 1)
    if (k & 1u) m = multmodp(m, t->row_pow[i], poly);
  return multmodp(m, reg, poly);
}

// reg * x^(8*kRow*k) mod P: one multiply for k < 4096 (rows_shift table), one more per set bit above.
__device__ __forceinline__ std::uint32_t shift_rows_tab(const DeviceTables* t, std::uint32_t reg, std::uint32_t k) {
  const std::uint32_t poly = t->poly;
  std::uint32_t m = sload32(t->rows_shift, k & 4095u);
  for (int i = 12; (k >> i) != 0u; ++i)
    if ((k >> i) & 1u) m = multmodp(m, sload32(t->row_pow, static_cast<std::uint32_t>(i)), poly);
  return multmodp(m, reg, poly);
}

struct Cursor {
  std::uint32_t b;          // block index
  std::uint32_t r;          // row within the block
  std::uint32_t R;          // rows of the block
  std::uint32_t n;          // bytes of the block
  const std::uint8_t* blk;  // block start
};

template <bool UNIFORM>
__device__ __forceinline__ void load_desc(const RowsArgs& a, Cursor& c, std::uint32_t nblk) {
  const std::uint32_t b = c.b < nblk ? c.b : nblk - 1;
  if constexpr (UNIFORM) {
    c.blk = a.base + static_cast<std::uint64_t>(b) * a.stride;
    c.n = a.len;
  } else {
    c.blk = a.base + sload64(a.offsets, b);
    c.n = sload32(a.lengths, b);
  }
  c.R = rows_for_len(c.n);
}

template <bool UNIFORM>
__device__ __forceinline__ void advance(const RowsArgs& a, Cursor& c, std::uint32_t nblk) {
  if (++c.r == c.R) {
    c.r = 0;
    ++c.b;
    load_desc<UNIFORM>(a, c, nblk);
  }
}

// Loads of one row for this lane: NP aligned 16-byte pieces covering its 64-byte segment, and (for
// irregular batches) its Shift_h constant when the row is a head row. Pieces outside the block and
// rows past the wave's range read the zero `dummy` buffer.
template <int NP>
struct RowBuf {
  uint4 q[NP];
  std::uint32_t hs;
};

template <int NP, bool UNIFORM>
__device__ __forceinline__ void issue_row(const RowsArgs& a, const Cursor& c, bool live, std::uint32_t lane,
                                          RowBuf<NP>& rb) {
  const std::int64_t rowstart =
      static_cast<std::int64_t>(c.n) - static_cast<std::int64_t>(c.R - c.r) * kRow;
  const std::uintptr_t blo = reinterpret_cast<std::uintptr_t>(c.blk);
  const std::uintptr_t bhi = blo + c.n;
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);
  const std::uintptr_t seg = static_cast<std::uintptr_t>(static_cast<std::int64_t>(blo) + rowstart) + lane * kSeg;
  if (NP == 4 || c.r == 0 || !live) {
    // 16-byte aligned pieces; pieces outside the block (head padding, dead rows) read `dummy`.
    const std::uintptr_t al = seg & ~static_cast<std::uintptr_t>(15);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const std::uintptr_t p = al + 16u * i;
      const bool ok = live && (p + 16 > blo) && (p < bhi);
      rb.q[i] = gload16(ok ? p : dmy);
    }
  } else {
    // Interior row of an unaligned block: the segment lies inside the block, so four dword-aligned
    // 16-byte loads (as fast as aligned ones on gfx950; byte-misaligned ones are 27 % slower) plus
    // one dword cover it; bytes read outside the block share an aligned dword with block bytes.
    const std::uintptr_t a4 = seg & ~static_cast<std::uintptr_t>(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) rb.q[i] = gload16(a4 + 16u * i);
    rb.q[NP - 1].x = *reinterpret_cast<g_u32*>((seg & 3u) ? a4 + 64u : dmy);
  }
  if constexpr (!UNIFORM) {
    const std::uintptr_t hp = reinterpret_cast<std::uintptr_t>(&a.tabs->head_shift[head_len(c.n)][lane & 31u]);
    rb.hs = *reinterpret_cast<g_u32*>((live && c.r == 0) ? hp : dmy);
  } else {
    rb.hs = 0;
  }
}

// The 16 little-endian dwords of this lane's 64-byte segment (realigned; head-row bytes in front of
// the block zeroed — whole pieces in front of it were already loaded from `dummy`).
template <bool ALIGNED, int NP>
__device__ __forceinline__ void segment_dwords(const Cursor& c, const RowBuf<NP>& rb, std::uint32_t lane,
                                               std::uint32_t (&dw)[16]) {
  if constexpr (ALIGNED) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dw[4 * i + 0] = rb.q[i].x;
      dw[4 * i + 1] = rb.q[i].y;
      dw[4 * i + 2] = rb.q[i].z;
      dw[4 * i + 3] = rb.q[i].w;
    }
  } else if (c.r != 0) {
    // interior row: dword-aligned loads (issue_row), only the byte shift t remains
    std::uint32_t raw[17];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      raw[4 * i + 0] = rb.q[i].x;
      raw[4 * i + 1] = rb.q[i].y;
      raw[4 * i + 2] = rb.q[i].z;
      raw[4 * i + 3] = rb.q[i].w;
    }
    raw[16] = rb.q[NP - 1].x;
    const std::uint32_t t = static_cast<std::uint32_t>((reinterpret_cast<std::uintptr_t>(c.blk) + c.n) & 3u);
#pragma unroll
    for (int k = 0; k < 16; ++k) dw[k] = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], t);
  } else {
    std::uint32_t raw[20];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      raw[4 * i + 0] = rb.q[i].x;
      raw[4 * i + 1] = rb.q[i].y;
      raw[4 * i + 2] = rb.q[i].z;
      raw[4 * i + 3] = rb.q[i].w;
    }
    // Every segment of a block has the same misalignment (segments start at end - k*64).
    const std::uint32_t s = static_cast<std::uint32_t>((reinterpret_cast<std::uintptr_t>(c.blk) + c.n) & 15u);
    const std::uint32_t t = s & 3u;
    if (s & 8u) {
#pragma unroll
      for (int i = 0; i < 18; ++i) raw[i] = raw[i + 2];
    }
    if (s & 4u) {
#pragma unroll
      for (int i = 0; i < 19; ++i) raw[i] = raw[i + 1];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) dw[k] = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], t);
    const std::int32_t rowstart = static_cast<std::int32_t>(c.n - c.R * static_cast<std::uint32_t>(kRow));
    if (c.r == 0 && rowstart < 0) {
      const std::int32_t off0 = rowstart + static_cast<std::int32_t>(lane * kSeg);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const std::int32_t before = -(off0 + 4 * k);  // bytes of this dword in front of the block
        const std::uint32_t sh = static_cast<std::uint32_t>(before < 0 ? 0 : (before > 4 ? 4 : before)) * 8u;
        dw[k] &= static_cast<std::uint32_t>(0xFFFFFFFFull << sh);
      }
    }
  }
}

// Per-wave state of the piece of a block the wave is folding.
struct WaveState {
  std::uint32_t B;          // running register of the current piece (Horner over rows)
  bool piece_has_row0;      // the current piece started at the block's head row
  bool first_piece;         // the current piece is the wave's first
  std::uint32_t s_block[2], s_part[2], s_after[2], s_flags[2];
  // uniform batches: whole blocks' results, gathered 64 at a time (lane k: the k-th since the last
  // store) and stored together: a store per block sits in the same vmcnt queue as the row loads
  // issued after it (3000-byte blocks +6 %, 6000-byte +13 %, profiles/r2/packed_small/)
  std::uint32_t k_val, k_idx, k_n;
};

// Horner step + init injection + DPP reduction for one row whose lane contributions are v; emits
// the block's result (or a seam record) when the row ends the block or the wave's range.
template <bool UNIFORM>
__device__ __forceinline__ void finish_row(const RowsArgs& a, const Cursor& c, std::uint32_t v, std::uint32_t hs,
                                           std::uint32_t hcon, std::uint32_t lane, bool last_of_range,
                                           WaveState& st) {
  const bool lo_half = lane < 32u;
  std::uint32_t init = 0;
  if (c.r == 0) {
    // per-block init of a compacted large block: its batch index is out_idx[c.b]
    init = a.init_raw ? sload32(a.init_raw, a.out_idx ? sload32(a.out_idx, c.b) : c.b) : a.init_default;
  }
  std::uint32_t hk = hcon;
  if constexpr (!UNIFORM) hk = lo_half ? hcon : hs;
  // lanes 0..31: bit l of B times Shift_4096(1<<l); lanes 32..63 on a head row: bit l-32 of init
  // times Shift_h(1<<(l-32)).
  const std::uint32_t sel = lo_half ? st.B : init;
  v ^= static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(sel), lane & 31u, 1)) & hk;
  const std::uint32_t Bn = __builtin_amdgcn_readlane(wave_xor_to_lane63(v), 63);
  if (c.r + 1 == c.R || last_of_range) {
    if (st.piece_has_row0 && c.r + 1 == c.R) {
      const std::uint32_t ob = a.out_idx ? sload32(a.out_idx, c.b) : c.b;
      if constexpr (UNIFORM) {
        st.k_val = lane == st.k_n ? Bn ^ a.out_xor : st.k_val;
        st.k_idx = lane == st.k_n ? ob : st.k_idx;
        if (++st.k_n == 64u) {
          a.out[st.k_idx] = st.k_val;
          st.k_n = 0;
        }
      } else {
        // (irregular: the three registers of the gather made the 768-thread kernel spill, 3.6 %
        // slower on a gapped Zipf batch; its whole blocks are the large ones, one store per >= 1 KiB)
        if (lane == 0) a.out[ob] = Bn ^ a.out_xor;
      }
    } else {
      // (explicit slots: a runtime index into these arrays would put them in scratch memory)
      const std::uint32_t flags = kSeamValid | (st.piece_has_row0 ? kSeamHasRow0 : 0u);
      if (UNIFORM && st.piece_has_row0) {
        // head piece of a block cut between waves: seed its result with xorout; crc_fixup XORs
        // every piece's shifted partial into it (this kernel precedes crc_fixup on the stream).
        // Irregular batches combine in this kernel instead (combine_seams).
        const std::uint32_t ob = a.out_idx ? sload32(a.out_idx, c.b) : c.b;
        if (lane == 0) a.out[ob] = a.out_xor;
      }
      if (st.first_piece) {
        st.s_block[0] = c.b;
        st.s_part[0] = Bn;
        st.s_after[0] = c.R - 1 - c.r;
        st.s_flags[0] = flags;
      } else {
        st.s_block[1] = c.b;
        st.s_part[1] = Bn;
        st.s_after[1] = c.R - 1 - c.r;
        st.s_flags[1] = flags;
      }
    }
    st.first_piece = false;
    st.piece_has_row0 = true;
    st.B = 0;
  } else {
    st.B = Bn;
  }
}

// Issue priority from the work a wave has left (`left` of `total` rows): the SIMD arbiter serves a
// SIMD's oldest wave first, so with equal ranges the first wave on each SIMD finishes long before
// the fourth. PRIO 1: levels 3..0 over the quarters of the range; PRIO p > 1:
// thresholds at 2^(1-p), 2^(-p), 2^(-1-p) of it left (3: 1/4, 1/8, 1/16, the product setting).
template <int PRIO>
__device__ __forceinline__ void set_prio_from_left(std::uint32_t left, std::uint32_t total) {
  const std::uint64_t rem = left;
  std::uint32_t lvl;
  if constexpr (PRIO == 1) {
    lvl = static_cast<std::uint32_t>(rem * 4u / (total + 1ull));
  } else {
    constexpr std::uint32_t sh = PRIO + 1;
    lvl = (rem << sh) > 4ull * total ? 3u : (rem << sh) > 2ull * total ? 2u : (rem << sh) > total ? 1u : 0u;
  }
  if (lvl >= 3u) __builtin_amdgcn_s_setprio(3);
  else if (lvl == 2u) __builtin_amdgcn_s_setprio(2);
  else if (lvl == 1u) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Small blocks of an irregular batch (defined below; runs inside the irregular row kernel).
__device__ __forceinline__ void small_phase(const RowsArgs& a, const std::uint32_t* lds);

// Fill the 160 KiB LDS table image (slicing tables replicated 32x, lane-shift nibble tables) with one
// global load per slicing entry: thread u owns (pair, entry, table) of u = 512 pair + 2 e + t and
// stores the 32 copies as eight 16-byte LDS writes, rotated by u so that a wave's writes spread over
// the banks; the lane-shift tables move as 16-byte pieces. Against one dword load and store per LDS
// word: +1.0 % on 1 M x 4 KiB, +0.2 to +0.4 % on 64 KiB blocks (profiles/r1/explore_wide_fill.txt).
__device__ __forceinline__ void fill_lds_slicing(const DeviceTables* tabs, std::uint32_t* lds) {
  for (std::uint32_t u = threadIdx.x; u < 1024u; u += blockDim.x) {
    const std::uint32_t pair = u >> 9, e = (u >> 1) & 255u, t = u & 1u;
    const std::uint32_t v = tabs->slice[2 * pair + t][e];
    uint4* dst = reinterpret_cast<uint4*>(lds + pair * 16384u + e * 64u + t * 32u);
#pragma unroll
    for (std::uint32_t k = 0; k < 8u; ++k) dst[(k + u) & 7u] = make_uint4(v, v, v, v);
  }
}

__device__ __forceinline__ void fill_lds_slicing16(const DeviceTables* tabs, std::uint32_t* lds) {
  for (std::uint32_t u = threadIdx.x; u < 1024u; u += blockDim.x) {
    const std::uint32_t e = u >> 2, t = u & 3u;
    const std::uint32_t v = tabs->slice[t][e];
    uint4* dst = reinterpret_cast<uint4*>(lds + e * 64u + t * 16u);
#pragma unroll
    for (std::uint32_t k = 0; k < 4u; ++k) dst[(k + u) & 3u] = make_uint4(v, v, v, v);
  }
}

__device__ __forceinline__ void fill_lds(const DeviceTables* tabs, std::uint32_t* lds) {
  fill_lds_slicing(tabs, lds);
  const uint4* ls = reinterpret_cast<const uint4*>(&tabs->lane_shift[0][0][0]);
  uint4* lds_ls = reinterpret_cast<uint4*>(lds + kLdsSliceWords);
  for (std::uint32_t i = threadIdx.x; i < kLdsLaneWords / 4u; i += blockDim.x) lds_ls[i] = ls[i];
}

// The generic row kernel's body (uniform batches of any length/stride/alignment, and irregular
// batches after the prepass). Irregular batches run their share of the small-block phase first.
// PRIO: issue priority from the rows a wave has left (set_prio_from_left).
template <bool ALIGNED, bool UNIFORM, int DEPTH, int ILP, int PRIO = 0>
__device__ __forceinline__ void crc_rows_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  constexpr int NP = ALIGNED ? 4 : 5;
  fill_lds(a.tabs, lds);

  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  std::uint32_t hcon = a.tabs->horner[lane];
  if constexpr (UNIFORM) {
    if (lane >= 32u) hcon = multmodp(a.head_z, 1u << (lane - 32u), a.tabs->poly);  // Shift_h(1 << (l-32))
  }
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (!UNIFORM) small_phase(a, lds);
  const std::uint64_t W = a.nwaves;

  // This wave's contiguous range of rows [g0, g1).
  std::uint32_t g0, g1;
  std::uint32_t nblk = a.nblocks;
  Cursor cur;
  if constexpr (UNIFORM) {
    const std::uint32_t R = rows_for_len(a.len);
    if (a.snap_blocks) {
      g0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(a.nblocks) / W) * R;
      g1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(a.nblocks) / W) * R;
    } else {
      g0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(a.total_rows) / W);
      g1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(a.total_rows) / W);
    }
    cur.b = g0 / R;
    cur.r = g0 - cur.b * R;
  } else {
    // large blocks only (compacted by the prepass); small ones are small_phase's
    nblk = sload32(a.counts, 0);
    const std::uint64_t TR = sload32(a.counts, 2);
    g0 = static_cast<std::uint32_t>(wave * TR / W);
    g1 = static_cast<std::uint32_t>((wave + 1) * TR / W);
    cur.b = g0 < g1 ? sload32(a.wave_start, wave) : 0u;
    cur.r = g0 < g1 ? g0 - sload32(a.row_scan, cur.b) : 0u;
  }

  WaveState st;
  st.B = 0;
  st.first_piece = true;
  st.k_val = st.k_idx = st.k_n = 0;
#pragma unroll
  for (int s = 0; s < 2; ++s) st.s_block[s] = st.s_part[s] = st.s_after[s] = st.s_flags[s] = 0;

  if (g0 < g1) {
    load_desc<UNIFORM>(a, cur, nblk);
    st.piece_has_row0 = cur.r == 0;

    // Lane contributions of n rows before the Horner step, Shift_{(63-l)*64}(crc_0(segment)), with
    // the rows' slicing chains interleaved (independent until the Horner step).
    auto lane_values = [&](auto n_const, const Cursor* cs, const RowBuf<NP>* rbs, std::uint32_t* v) {
      constexpr int n = decltype(n_const)::value;
      std::uint32_t d[n][16];
#pragma unroll
      for (int i = 0; i < n; ++i) segment_dwords<ALIGNED, NP>(cs[i], rbs[i], lane, d[i]);
      Reg p[n];
#pragma unroll
      for (int i = 0; i < n; ++i) p[i] = Reg{0, 0};
#pragma unroll
      for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int i = 0; i < n; ++i) slice4(lds, p[i], d[i][t], kc);
#pragma unroll
      for (int i = 0; i < n; ++i) v[i] = lane_shift(lds, p[i].value(), kc);
    };

    RowBuf<NP> buf[DEPTH];
    Cursor cq[DEPTH];
    Cursor lc = cur;  // cursor of the next row to load
    std::uint32_t gl = g0;
#pragma unroll
    for (int s = 0; s < DEPTH - ILP; ++s) {
      cq[s] = lc;
      issue_row<NP, UNIFORM>(a, lc, gl < g1, lane, buf[s]);
      advance<UNIFORM>(a, lc, nblk);
      ++gl;
    }
    for (std::uint32_t g = g0; g < g1; g += DEPTH) {
      if constexpr (PRIO != 0) set_prio_from_left<PRIO>(g1 - g, g1 - g0);
#pragma unroll
      for (int k = 0; k < DEPTH; k += ILP) {
        // refill the slots freed by the previous step
#pragma unroll
        for (int j = 0; j < ILP; ++j) {
          const int s = (k + DEPTH - ILP + j) % DEPTH;
          cq[s] = lc;
          issue_row<NP, UNIFORM>(a, lc, gl < g1, lane, buf[s]);
          advance<UNIFORM>(a, lc, nblk);
          ++gl;
        }
        const std::uint32_t gk = g + k;
        if (gk >= g1) break;
        if (gk + ILP <= g1) {
          std::uint32_t v[ILP];
          lane_values(std::integral_constant<int, ILP>{}, &cq[k], &buf[k], v);
#pragma unroll
          for (int i = 0; i < ILP; ++i)
            finish_row<UNIFORM>(a, cq[k + i], v[i], buf[k + i].hs, hcon, lane, gk + i + 1 == g1, st);
        } else {
#pragma unroll
          for (int i = 0; i < ILP; ++i) {  // tail: fewer than ILP rows left
            if (gk + i < g1) {
              std::uint32_t v[1];
              lane_values(std::integral_constant<int, 1>{}, &cq[k + i], &buf[k + i], v);
              finish_row<UNIFORM>(a, cq[k + i], v[0], buf[k + i].hs, hcon, lane, gk + i + 1 == g1, st);
            }
          }
        }
      }
    }
    if (UNIFORM && lane < st.k_n) a.out[st.k_idx] = st.k_val;  // the last gathered results
  }

  if constexpr (!UNIFORM) {
    // Irregular batches: the prepass zeroed the result of every block cut between waves, so each
    // piece XORs its partial, moved past the rows that follow it, straight into the result (the
    // head piece adds xorout): out = xorout ^ sum of pieces, in any order, with no fix-up launch.
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (st.s_flags[s] & kSeamValid) {
        const std::uint32_t contrib = shift_rows_tab(a.tabs, st.s_part[s], st.s_after[s]) ^
                                      ((st.s_flags[s] & kSeamHasRow0) ? a.out_xor : 0u);
        const std::uint32_t ob = a.out_idx ? sload32(a.out_idx, st.s_block[s]) : st.s_block[s];
        if (lane == 0) __hip_atomic_fetch_xor(a.out + ob, contrib, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if (lane == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Seam rec;
      rec.block = st.s_block[s];
      rec.partial = st.s_part[s];
      rec.rows_after = st.s_after[s];
      rec.flags = st.s_flags[s];
      a.seams[2 * static_cast<std::uint64_t>(wave) + s] = rec;
    }
  }
}


// Inclusive prefix XOR of v over the 64 lanes (DPP row shifts within rows of 16, then row
// broadcasts across rows).
__device__ __forceinline__ std::uint32_t wave_prefix_xor(std::uint32_t v) {
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v ^= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ __forceinline__ std::uint64_t readlane64(std::uint64_t v, std::uint32_t l) {
  const std::uint32_t lo = __builtin_amdgcn_readlane(static_cast<std::uint32_t>(v), l);
  const std::uint32_t hi = __builtin_amdgcn_readlane(static_cast<std::uint32_t>(v >> 32), l);
  return (static_cast<std::uint64_t>(hi) << 32) | lo;
}

// Stream-mode row partition: wave w (of W, 16 to a workgroup) walks rows [stream_row0(w), stream_row0(w+1))
// of the TR rows; stream_row0(W) = TR. Workgroup g gets rows [g*TR/G, (g+1)*TR/G) and shares them among
// its waves as crc_packed_body's SKEW partition does (slot class c = slot/4 weighted (SKEW/256)^c).
template <int SKEW>
__device__ __forceinline__ std::uint64_t stream_row0(std::uint64_t w, std::uint64_t TR, std::uint64_t W) {
  if constexpr (SKEW == 0) {
    return w * TR / W;
  } else {
    constexpr std::uint32_t w0 = 256, w1 = SKEW, w2 = w1 * SKEW / 256, w3 = w2 * SKEW / 256;
    constexpr std::uint32_t tot = 4 * (w0 + w1 + w2 + w3);
    const std::uint32_t k = static_cast<std::uint32_t>(w & 15u), c = k >> 2, m = k & 3u;
    const std::uint32_t pre = (c > 0 ? 4 * w0 : 0u) + (c > 1 ? 4 * w1 : 0u) + (c > 2 ? 4 * w2 : 0u) +
                              m * (c == 0 ? w0 : c == 1 ? w1 : c == 2 ? w2 : w3);
    const std::uint64_t g = w >> 4, G = W >> 4;
    const std::uint64_t r0 = g * TR / G, gn = (g + 1) * TR / G - r0;
    return r0 + gn * pre / tot;
  }
}
// Smallest wave w in [0, W] with row0[w] >= r, from the table row0[0..W] of stream_row0 (which is
// nondecreasing in w): a binary search of cached loads instead of 64-bit divisions.
__device__ __forceinline__ std::uint32_t stream_first_wave(const std::uint32_t* row0, std::uint64_t r, std::uint32_t W) {
  std::uint32_t lo = 0, hi = W;
  while (lo < hi) {
    const std::uint32_t mid = (lo + hi) >> 1;
    if (row0[mid] >= r) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// Byte-stream row walk of an irregular batch whose blocks lie back to back (stream mode, chosen by
// the prepass). The stream is cut into full 4 KiB rows from row 0 = its start
// rounded down to 16 bytes (bytes in front of it read as zero, bytes past its end are never used),
// so every row is aligned, no row is partial and there is no small-block phase. Waves own
// contiguous ranges of rows and fold them exactly as the packed kernel does, keeping
// B = crc_0(stream bytes from the wave's first row) by Horner over rows. Block ends do not stop
// the walk: for a block ending at E inside row g, in lane l's segment at byte r in (0, 64], the lane
// captures its chain register after floor(r/4) dwords during the fold, finishes the last r mod 4
// bytes with Sarwate steps (Q = crc_0 of its segment up to E), and the wave's prefix XOR of the
// lane values gives Y = Shift_4096(B) ^ (lanes before l, moved to the row end). Then
// crc_0(wave bytes up to E) = Shift_(rowend - E)^-1 (Y) ^ Q, which stream_finish turns into each
// block's CRC. Each wave stores (Y, Q) per block end it meets and its own B at the end of its range.
// The caller has filled the LDS tables (fill_lds + barrier): the body holds no barrier, so the waves
// of one workgroup may run different instantiations of it.
template <int PRIO, bool MANY = false>
__device__ __forceinline__ void crc_stream_body(const RowsArgs& a, std::uint32_t* lds) {
  constexpr int DEPTH = 4, ILP = 2;
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t hcon = a.tabs->horner[lane];  // Shift_4096(1 << l) for l < 32, else 0
  const bool lo_half = lane < 32u;
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t TR = sload32(a.counts, 2);
  const std::uint32_t g0 = sload32(a.s_row0, wave);
  const std::uint32_t g1 = sload32(a.s_row0, wave + 1);
  if (g0 >= g1) {
    if (lane == 0) a.s_wtot[wave] = 0u;
    return;
  }
  const std::uint32_t n = a.nblocks;
  const std::uint64_t s0rel = sload64(a.s_info, 1);
  const std::uintptr_t zrow = reinterpret_cast<std::uintptr_t>(a.base) + sload64(a.s_info, 0);
  const std::uintptr_t send = zrow + sload64(a.s_ends, n - 1);
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);
  const std::uint32_t nrows = g1 - g0;
  const std::uintptr_t lane_base = zrow + static_cast<std::uint64_t>(g0) * kRow + lane * kSeg;

  // block ends, 64 at a time: lane i of `win` holds E[bw + i]
  std::uint32_t b = sload32(a.wave_start, wave);  // first block ending in or after row g0
  std::uint32_t bw = b;
  auto load_win = [&](std::uint32_t from) -> std::uint64_t {
    const std::uint32_t i = from + lane;
    return i < n ? a.s_ends[i] : ~0ull;
  };
  // Two windows: the next one is loaded 64 ends ahead, so reading an end never waits on a load
  // issued behind the row loads in flight (a vmcnt wait drains every outstanding load before it).
  std::uint64_t win = load_win(bw), win2 = load_win(bw + 64u);
  std::uint32_t ci = 0;
  std::uint64_t e_next = readlane64(win, 0);

  // Per-end records (Y, Q) are gathered in registers, lane k of keep_y/keep_q holding block kb + k
  // (kmask: lanes filled), and written 64 at a time: a store in the row loop is counted by the
  // same vmcnt as the row loads behind it, so one store per end would stall the next row's wait on
  // its write acknowledgement (-4 % on cfg4). Ends too far past kb for the current window (a row
  // pair with more than 32 ends) are stored directly.
  std::uint32_t kb = b, keep_y = 0, keep_q = 0;
  std::uint64_t kmask = 0;
  auto flush = [&]() {
    if (kmask != 0) {
      if ((kmask >> lane) & 1u) {
        a.s_yq[kb + lane] = static_cast<std::uint64_t>(keep_y) | (static_cast<std::uint64_t>(keep_q) << 32);
        a.s_wv[kb + lane] = wave;
      }
      kmask = 0;
    }
  };

  // Block ends in the row [rs, rs + 4096): the lane whose segment holds one learns (r, block), and
  // keep lane b - kb learns which lane that is (src; rmask: keep lanes fed by this row).
  // MANY (probe): a row with many ends takes them all at once (lane-parallel capture).
  auto take_ends = [&](std::uint64_t rs, std::uint32_t& my_r, std::uint32_t& my_b, std::uint32_t& src,
                       std::uint64_t& rmask) -> bool {
    my_r = 0xFFu;  // no end in this lane's segment
    rmask = 0;
    const std::uint64_t lim = rs + kRow;
    if (e_next > lim) return false;
    // more than kManyEnds ends in the row (E[b + kManyEnds] inside it): take them all at once
    constexpr std::uint32_t kManyEnds = 8;
    const std::uint32_t probe = ci + kManyEnds;
    if (MANY && b + kManyEnds < n &&
        (probe < 64u ? readlane64(win, probe) : readlane64(win2, probe - 64u)) <= lim) {
      const bool in1 = lane >= ci && win <= lim;
      const std::uint32_t c1 = static_cast<std::uint32_t>(__popcll(__ballot(in1)));
      bool in2 = false;
      std::uint32_t cnt = c1;
      if (c1 == 64u - ci) {
        in2 = win2 <= lim;
        cnt += static_cast<std::uint32_t>(__popcll(__ballot(in2)));
      }
      {
        const std::uint32_t rel1 = static_cast<std::uint32_t>(win - rs), rel2 = static_cast<std::uint32_t>(win2 - rs);
        const std::uint32_t l1 = (rel1 + 63u) / 64u - 1u, r1 = rel1 - 64u * l1;
        const std::uint32_t l2 = (rel2 + 63u) / 64u - 1u, r2 = rel2 - 64u * l2;
        const std::uint64_t bit = (in1 ? 1ull << (l1 & 63u) : 0ull) | (in2 ? 1ull << (l2 & 63u) : 0ull);
        std::uint64_t S = bit;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) S |= __shfl_xor(S, m, 64);
        const std::uint32_t kr = static_cast<std::uint32_t>(__popcll(S & ((1ull << lane) - 1ull)));
        const std::uint32_t pos = ci + kr;
        const int pfrom = static_cast<int>((pos & 63u) << 2);
        const std::uint32_t pr1 = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(pfrom, static_cast<int>(r1)));
        const std::uint32_t pr2 = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(pfrom, static_cast<int>(r2)));
        if ((S >> lane) & 1u) {
          my_r = pos < 64u ? pr1 : pr2;
          my_b = b + kr;
        }
        const std::uint32_t kp = kb + lane - bw;
        const int kfrom = static_cast<int>((kp & 63u) << 2);
        const std::uint32_t pl1 = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(kfrom, static_cast<int>(l1)));
        const std::uint32_t pl2 = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(kfrom, static_cast<int>(l2)));
        const std::uint32_t k0 = b - kb;
        if (lane >= k0 && lane < k0 + cnt) src = kp < 64u ? pl1 : pl2;
        if (k0 < 64u) {
          const std::uint32_t k1 = k0 + cnt < 64u ? k0 + cnt : 64u;
          rmask = (k1 == 64u ? ~0ull : (1ull << k1) - 1ull) & ~((1ull << k0) - 1ull);
        }
        b += cnt;
        ci += cnt;
        if (ci >= 64u) {
          bw += 64u;
          win = win2;
          win2 = load_win(bw + 64u);
          ci -= 64u;
        }
        e_next = b < n ? readlane64(win, ci) : ~0ull;
        return true;
      }
    }
    while (e_next <= lim) {
      const std::uint32_t rel = static_cast<std::uint32_t>(e_next - rs);  // 1..4096
      const std::uint32_t l = (rel + 63u) / 64u - 1u;
      my_r = lane == l ? rel - 64u * l : my_r;
      my_b = lane == l ? b : my_b;
      const std::uint32_t k = b - kb;
      if (k < 64u) {
        src = lane == k ? l : src;
        rmask |= 1ull << k;
      }
      ++b;
      if (++ci == 64u) {
        bw += 64u;
        win = win2;
        win2 = load_win(bw + 64u);
        ci = 0;
      }
      e_next = b < n ? readlane64(win, ci) : ~0ull;
    }
    return true;
  };

  uint4 buf[DEPTH][4];
  // Row loads. Only the stream's last row can reach past its end; the wave that owns it walks it
  // after its main loop with guarded loads (pieces past the end read `dummy`).
  const bool owns_last = g1 == TR;
  const std::uint32_t nmain = nrows - (owns_last ? 1u : 0u);
  auto issue = [&](std::uint32_t j, uint4 (&q)[4]) {
    const std::uint32_t jc = j < nmain ? j : (nmain ? nmain - 1 : 0u);  // rows past the range reload
    const std::uintptr_t p = lane_base + static_cast<std::uint64_t>(jc) * kRow;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(nmain ? p + 16u * i : dmy);
  };
  auto issue_last = [&](uint4 (&q)[4]) {
    const std::uintptr_t p = lane_base + static_cast<std::uint64_t>(nrows - 1) * kRow;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(p + 16u * i < send ? p + 16u * i : dmy);
  };

  // The stream's first row, lane 0: bytes in front of the stream start read as zero (leading zeros
  // are free).
  auto head_mask = [&](uint4& q0) {
    if (lane == 0u) {
      const std::uint32_t s = static_cast<std::uint32_t>(s0rel);
      std::uint32_t* w = reinterpret_cast<std::uint32_t*>(&q0);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const std::int32_t before = static_cast<std::int32_t>(s) - 4 * d;  // bytes of dword d in front
        const std::uint32_t sh = static_cast<std::uint32_t>(before <= 0 ? 0 : (before >= 4 ? 4 : before)) * 8u;
        w[d] &= static_cast<std::uint32_t>(0xFFFFFFFFull << sh);
      }
    }
  };

  std::uint32_t B = 0;  // crc_0 of the wave's rows so far
  // Fold ILP rows (interleaved chains); with CAP each lane also keeps its chain register after
  // k = my_r / 4 dwords and dword k itself (k == 16: the whole segment).
  auto fold = [&](auto cap_const, const uint4 (*q)[4], const std::uint32_t* my_r, std::uint32_t* v,
                  std::uint32_t* capv, std::uint32_t* capd) {
    constexpr bool CAP = decltype(cap_const)::value;
    Reg p[ILP];
    std::uint32_t k[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      p[i] = Reg{0, 0};
      k[i] = my_r[i] >> 2;
      capv[i] = 0;
      capd[i] = 0;
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        const uint4& c = q[i][t >> 2];
        const std::uint32_t d = (t & 3) == 0 ? c.x : (t & 3) == 1 ? c.y : (t & 3) == 2 ? c.z : c.w;
        if constexpr (CAP) {
          const bool hit = k[i] == static_cast<std::uint32_t>(t);
          capv[i] = hit ? p[i].value() : capv[i];
          capd[i] = hit ? d : capd[i];
        }
        slice4(lds, p[i], d, kc);
      }
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      if constexpr (CAP) capv[i] = k[i] == 16u ? p[i].value() : capv[i];
      v[i] = lane_shift(lds, p[i].value(), kc);
    }
  };
  // Horner step over one row; at a row with block ends, the (Y, Q) of each end.
  auto finish = [&](std::uint32_t v, bool ends, std::uint32_t my_r, std::uint32_t my_b, std::uint32_t src,
                    std::uint64_t rmask, std::uint32_t capv, std::uint32_t capd) {
    const std::uint32_t term =
        lo_half ? static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(B), lane, 1)) & hcon : 0u;
    const std::uint32_t Bn = __builtin_amdgcn_readlane(wave_xor_to_lane63(v ^ term), 63);
    if (ends) {
      const std::uint32_t I = wave_prefix_xor(v);
      const std::uint32_t I63 = __builtin_amdgcn_readlane(I, 63);
      const std::uint32_t Y = Bn ^ I63 ^ I ^ v;  // Shift_4096(B) ^ lanes before this one
      const std::uint32_t m = my_r & 3u;
      std::uint32_t x = capv ^ (capd & static_cast<std::uint32_t>((1ull << (8 * m)) - 1ull));
#pragma unroll
      for (std::uint32_t j = 0; j < 3u; ++j)
        if (j < m) x = (x >> 8) ^ lds_at(lds, ((x & 0xFFu) << 8) | kc.L0);  // Sarwate step (T0)
      const std::uint32_t py = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src << 2), static_cast<int>(Y)));
      const std::uint32_t pq = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src << 2), static_cast<int>(x)));
      const bool mine = (rmask >> lane) & 1u;
      keep_y = mine ? py : keep_y;
      keep_q = mine ? pq : keep_q;
      kmask |= rmask;
      if (my_r != 0xFFu && my_b - kb >= 64u) {  // past the keep window: store now
        a.s_yq[my_b] = static_cast<std::uint64_t>(Y) | (static_cast<std::uint64_t>(x) << 32);
        a.s_wv[my_b] = wave;
      }
    }
    B = Bn;
  };
  // n (1 or ILP) rows at wave-local row jq from buffer slots q[0..n)
  auto rows = [&](int n, std::uint32_t jq, const uint4 (*q)[4]) {
    if (b - kb >= 32u) {  // room for the ends of this row pair in the keep window
      flush();
      kb = b;
    }
    std::uint32_t my_r[ILP], my_b[ILP] = {0, 0}, src[ILP] = {0, 0};
    std::uint64_t rmask[ILP] = {0, 0};
    bool ends[ILP];
    bool any = false;
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      my_r[i] = 0xFFu;
      ends[i] = false;
      if (i < n) {
        ends[i] = take_ends(static_cast<std::uint64_t>(g0 + jq + i) * kRow, my_r[i], my_b[i], src[i], rmask[i]);
        any = any || ends[i];
      }
    }
    std::uint32_t v[ILP], capv[ILP], capd[ILP];
    if (any) fold(std::true_type{}, q, my_r, v, capv, capd);
    else fold(std::false_type{}, q, my_r, v, capv, capd);
#pragma unroll
    for (int i = 0; i < ILP; ++i)
      if (i < n) finish(v[i], ends[i], my_r[i], my_b[i], src[i], rmask[i], capv[i], capd[i]);
  };

#pragma unroll
  for (int s = 0; s < DEPTH - ILP; ++s) issue(s, buf[s]);
  if (g0 == 0u && nmain) head_mask(buf[0][0]);  // the stream's first row
  for (std::uint32_t j = 0; j < nmain; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(nmain - j, nmain);
#pragma unroll
    for (int qd = 0; qd < DEPTH; qd += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + qd + DEPTH - ILP + i, buf[(qd + DEPTH - ILP + i) % DEPTH]);
      const std::uint32_t jq = j + qd;
      if (jq >= nmain) break;
      rows(jq + ILP <= nmain ? ILP : static_cast<int>(nmain - jq), jq, &buf[qd]);
    }
  }
  if (owns_last) {  // the stream's last row (it holds the last block's end)
    issue_last(buf[0]);
    if (nrows == 1 && g0 == 0u) head_mask(buf[0][0]);
    rows(1, nrows - 1, &buf[0]);
  }
  flush();
  if (lane == 0) a.s_wtot[wave] = B;
}

// Packed uniform fast path: block b = [base + b*len, +len) with len a multiple of kRow (4 KiB) and
// 16-byte aligned base, so every row is full, row g of the batch sits at base + g*kRow, and the head
// length is kRow (init injection constants = the Horner constants). Each wave owns the contiguous
// blocks [b0, b1) (no seams), keeps ILP rows' slicing chains interleaved and DEPTH-ILP rows in
// flight, and stores its results 64 at a time (lane k holds its k-th block). R1: one row per block
// (4 KiB blocks), so no Horner state at all. The SIMDs are issue-bound here (PMC: every SIMD issues
// ~96 % of cycles), so the loop is written for instruction count: incremental row addressing, no
// divisions, selects instead of divergent branches.
// SKEW (0: off): the waves of a 1024-thread workgroup share its equal slice of the batch in
// proportion to 256 * (SKEW/256)^(slot/4): slots 0-3 (the first wave on each SIMD) get the largest
// ranges, slots 12-15 the smallest, matching the issue arbitration that favours a SIMD's older waves.
// PRIO (0: off): set_prio_from_left<PRIO> once per DEPTH rows (the product uses 3, and SKEW 154 for
// blocks of more than one row; tkv_crc32_kernels.hip).
template <int DEPTH, int ILP, bool R1, int SKEW = 0, int PRIO = 0>
__device__ __forceinline__ void crc_packed_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t hcon = a.tabs->horner[lane & 31u];  // Shift_4096(1 << (l & 31))
  const bool lo_half = lane < 32u;
  // Init injection term for blocks without a per-block init: bit (l-32) of init * Shift_4096(...)
  const std::uint32_t inj_const =
      lo_half ? 0u
              : static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(a.init_default),
                                                                lane & 31u, 1)) & hcon;

  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves;
  const std::uint32_t R = R1 ? 1u : a.len / kRow;
  std::uint32_t b0, nb;
  if constexpr (SKEW != 0) {
    constexpr std::uint32_t w0 = 256, w1 = SKEW, w2 = w1 * SKEW / 256, w3 = w2 * SKEW / 256;
    constexpr std::uint32_t tot = 4 * (w0 + w1 + w2 + w3);
    const std::uint32_t k = wave & 15u, c = k >> 2, m = k & 3u;
    const std::uint32_t pre = (c > 0 ? 4 * w0 : 0u) + (c > 1 ? 4 * w1 : 0u) + (c > 2 ? 4 * w2 : 0u) +
                              m * (c == 0 ? w0 : c == 1 ? w1 : c == 2 ? w2 : w3);
    const std::uint32_t wk = c == 0 ? w0 : c == 1 ? w1 : c == 2 ? w2 : w3;
    const std::uint64_t g = wave >> 4, G = W >> 4;
    const std::uint64_t g0 = g * a.nblocks / G, gn = (g + 1) * a.nblocks / G - g0;
    b0 = static_cast<std::uint32_t>(g0 + gn * pre / tot);
    nb = static_cast<std::uint32_t>(g0 + gn * (pre + wk) / tot) - b0;
  } else {
    b0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(a.nblocks) / W);
    nb = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(a.nblocks) / W) - b0;
  }
  const std::uint32_t nrows = nb * R;  // wave-local rows j = 0 .. nrows-1, contiguous in memory
  const std::uintptr_t lane_base =
      reinterpret_cast<std::uintptr_t>(a.base) + static_cast<std::uint64_t>(b0) * R * kRow + lane * kSeg;

  uint4 buf[DEPTH][4];
  auto issue = [&](std::uint32_t j, uint4 (&q)[4]) {
    const std::uint32_t jc = j < nrows ? j : nrows - 1;  // rows past the range reload the last one
    const std::uintptr_t p = lane_base + static_cast<std::uint64_t>(jc) * kRow;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(p + 16u * i);
  };

  std::uint32_t B = 0;     // running register of the current block (Horner over its rows)
  std::uint32_t r = 0;     // row within the current block
  std::uint32_t k = 0;     // wave-local index of the current block
  std::uint32_t keep = 0;  // lane i: result of wave-local block (k & ~63) + i
  auto finish = [&](std::uint32_t v) {
    std::uint32_t term;
    const bool head = R1 || r == 0;
    if (head) {
      term = inj_const;
      if (a.init_raw) {
        const std::uint32_t init = sload32(a.init_raw, b0 + k);
        term = lo_half ? 0u : static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(init),
                                                                                lane & 31u, 1)) & hcon;
      }
    } else {
      term = lo_half ? static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(B), lane, 1)) & hcon
                     : 0u;
    }
    const std::uint32_t Bn = __builtin_amdgcn_readlane(wave_xor_to_lane63(v ^ term), 63);
    const bool last = R1 || ++r == R;
    if (last) {
      const std::uint32_t slot = k & 63u;
      keep = lane == slot ? (Bn ^ a.out_xor) : keep;
      if (slot == 63u || k + 1 == nb) {
        if (lane <= slot) a.out[b0 + k - slot + lane] = keep;
      }
      r = 0;
      ++k;
      B = 0;
    } else {
      B = Bn;
    }
  };

  // the first rows' loads go out before the table fill, so the fill (table loads from L2, LDS writes,
  // the barrier) overlaps their HBM latency instead of preceding it (round 4, profiles/r4/packed_early/)
  if (nb != 0) {
#pragma unroll
    for (int s = 0; s < DEPTH - ILP; ++s) issue(s, buf[s]);
  }
  fill_lds(a.tabs, lds);
  __syncthreads();
  if (nb == 0) return;
  for (std::uint32_t j = 0; j < nrows; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(nrows - j, nrows);
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + q + DEPTH - ILP + i, buf[(q + DEPTH - ILP + i) % DEPTH]);
      const std::uint32_t jq = j + q;
      if (jq >= nrows) break;
      if (jq + ILP <= nrows) {
        std::uint32_t v[ILP];
        Reg p[ILP];
#pragma unroll
        for (int i = 0; i < ILP; ++i) p[i] = Reg{0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].x, kc);
#pragma unroll
          for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].y, kc);
#pragma unroll
          for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].z, kc);
#pragma unroll
          for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].w, kc);
        }
#pragma unroll
        for (int i = 0; i < ILP; ++i) v[i] = lane_shift(lds, p[i].value(), kc);
#pragma unroll
        for (int i = 0; i < ILP; ++i) finish(v[i]);
      } else {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {  // tail: fewer than ILP rows left
          if (jq + i < nrows) {
            Reg p{0, 0};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              slice4(lds, p, buf[q + i][t].x, kc);
              slice4(lds, p, buf[q + i][t].y, kc);
              slice4(lds, p, buf[q + i][t].z, kc);
              slice4(lds, p, buf[q + i][t].w, kc);
            }
            finish(lane_shift(lds, p.value(), kc));
          }
        }
      }
    }
  }
}


// ---- packed small blocks: uniform batches of len = 64*G bytes (G = 1, 2, 4, ..., 32), stride == len,
// 16-byte aligned base. A 4 KiB row holds 64/G whole blocks; lane l folds its 64
// bytes as in crc_packed_body, its G-lane group (the lanes of one block) moves the partials to the
// block's end and XORs them together, so no row carries padding. The generic kernel gave every such
// block a whole zero-padded 4 KiB row (8x the table lookups of its bytes at 512 B).

// LDS image for G-lane groups: the slicing tables as fill_lds stores them, and in lane-shift column
// l the shift of lane l%G of a G-lane block, Shift_{(G-1-l%G)*64}, which is column 64-G+l%G of the
// device tables (LS[j][v][c] = Shift_{(63-c)*64}); every lane keeps a column of its own, so the
// lookups stay free of bank conflicts. G = 1 needs no lane shift.
template <int G>
__device__ __forceinline__ void fill_lds_group(const DeviceTables* tabs, std::uint32_t* lds) {
  fill_lds_slicing(tabs, lds);
  if constexpr (G >= 4) {
    const uint4* ls = reinterpret_cast<const uint4*>(&tabs->lane_shift[0][0][0]);
    uint4* lds_ls = reinterpret_cast<uint4*>(lds + kLdsSliceWords);
    for (std::uint32_t i = threadIdx.x; i < kLdsLaneWords / 4u; i += blockDim.x)
      lds_ls[i] = ls[(i & ~15u) + (64u - G + (4u * (i & 15u)) % G) / 4u];
  } else if constexpr (G == 2) {
    const std::uint32_t* ls = &tabs->lane_shift[0][0][0];
    std::uint32_t* lds_ls = lds + kLdsSliceWords;
    for (std::uint32_t i = threadIdx.x; i < static_cast<std::uint32_t>(kLdsLaneWords); i += blockDim.x)
      lds_ls[i] = ls[(i & ~63u) + 62u + (i & 1u)];
  }
}

// XOR over each G-lane group (G <= 32) with the first steps of wave_xor_to_lane63: for G <= 16 every
// lane of a group ends with the group's sum; for G = 32 lanes 16-31 and 48-63 do.
template <int G>
__device__ __forceinline__ std::uint32_t group_xor(std::uint32_t v) {
  if constexpr (G >= 2) v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (G >= 16) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, false); // row_mirror
  if constexpr (G >= 32) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1,3
  return v;
}

// Batch rows (4 KiB each, 64/G blocks) are split over the waves in contiguous ranges, with the
// packed kernel's pipeline and issue priority. Every block starts from init_default (per-block
// initial registers take the generic kernel): raw = Shift_len(init) ^ crc_0(block), with
// Shift_len(init) = head_z * init (head_z = x^(8 len)) added by the lane that stores the block.
template <int G, int DEPTH, int ILP, int PRIO = 0>
__device__ __forceinline__ void crc_packed_small_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(G >= 1 && G <= 32 && (G & (G - 1)) == 0, "G-lane groups of a power of two up to 32");
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  constexpr std::uint32_t kBpr = 64u / G;  // blocks per row
  fill_lds_group<G>(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t K = multmodp(a.head_z, a.init_default, a.tabs->poly) ^ a.out_xor;
  __syncthreads();

  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, TR = a.total_rows;
  const std::uint32_t r0 = static_cast<std::uint32_t>(wave * TR / W);
  const std::uint32_t nrows = static_cast<std::uint32_t>((wave + 1) * TR / W) - r0;
  if (nrows == 0) return;
  // Blocks of exactly 64 G bytes: row r is the batch's 4 KiB row r and holds blocks [r kBpr,
  // (r + 1) kBpr), lane g of a block's group reads its bytes [64 g, + 64), so the addressing is the
  // packed kernel's; in the batch's last row the lanes past its last block read that row's first
  // segment instead and store nothing. (Other multiples of 16 take crc_packed_small_gen's slots: the
  // zero-filled slot tails cost 6-10 % here, profiles/r6/small_uniform/lens.jsonl.)
  const std::uintptr_t row_base = reinterpret_cast<std::uintptr_t>(a.base) + static_cast<std::uint64_t>(r0) * kRow;
  const std::uint32_t lane_blk = lane / G;

  uint4 buf[DEPTH][4];
  auto issue = [&](std::uint32_t j, uint4 (&q)[4]) {
    const std::uint32_t jc = j < nrows ? j : nrows - 1;  // rows past the range reload the last one
    const bool live = static_cast<std::uint64_t>(r0 + jc) * kBpr + lane_blk < a.nblocks;
    const std::uintptr_t p = row_base + static_cast<std::uint64_t>(jc) * kRow + (live ? lane * kSeg : 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(p + 16u * i);
  };
  // G >= 2: the kBpr results of a row move into keep lanes ((j % G) * kBpr + block of the row), so
  // G rows fill all 64 and leave in one coalesced store; a store per row would sit in the same vmcnt
  // queue as the row loads issued after it. G = 1: each row's 64 results are one store already.
  std::uint32_t keep = 0;
  const std::uint32_t keep_src = ((lane % kBpr) * G + (G - 1u)) * 4u;  // byte address for ds_bpermute
  auto finish = [&](std::uint32_t j, std::uint32_t p) {
    std::uint32_t v = p;
    if constexpr (G > 1) {
      v = group_xor<G>(lane_shift(lds, v, kc)) ^ K;
      const std::uint32_t pulled = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(keep_src),
                                                                                          static_cast<int>(v)));
      const std::uint32_t slot = j % G;
      keep = lane / kBpr == slot ? pulled : keep;
      if (slot == G - 1u || j + 1u == nrows) {
        const std::uint64_t blk = static_cast<std::uint64_t>(r0 + j - slot) * kBpr + lane;
        if (lane < (slot + 1u) * kBpr && blk < a.nblocks) a.out[blk] = keep;
      }
    } else {
      const std::uint64_t blk = static_cast<std::uint64_t>(r0 + j) * kBpr + lane_blk;
      if (blk < a.nblocks) a.out[blk] = v ^ K;
    }
  };

#pragma unroll
  for (int s = 0; s < DEPTH - ILP; ++s) issue(s, buf[s]);
  for (std::uint32_t j = 0; j < nrows; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(nrows - j, nrows);
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + q + DEPTH - ILP + i, buf[(q + DEPTH - ILP + i) % DEPTH]);
      const std::uint32_t jq = j + q;
      if (jq >= nrows) break;
      Reg p[ILP];
#pragma unroll
      for (int i = 0; i < ILP; ++i) p[i] = Reg{0, 0};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].x, kc);
#pragma unroll
        for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].y, kc);
#pragma unroll
        for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].z, kc);
#pragma unroll
        for (int i = 0; i < ILP; ++i) slice4(lds, p[i], buf[q + i][t].w, kc);
      }
#pragma unroll
      for (int i = 0; i < ILP; ++i)
        if (jq + i < nrows) finish(jq + i, p[i].value());
    }
  }
}

// ---- lane blocks ------------------------------------------------------------------
// (declared here for crc_packed_small_gen_body below, defined with the lane kernels)
constexpr int kLaneGran = 5;  // granules covering 64 bytes at any alignment
template <int ALIGN>
__device__ __forceinline__ void lane_dwords(const uint4 (&g)[kLaneGran], std::uint32_t o, std::uint32_t (&d)[16]);

// ---- general small uniform blocks: 64 < L <= 64 G bytes (G = 2 .. 32 lanes per
// block), any stride (overlapping or gapped), any base alignment, optional per-block initial
// registers. The slot layout of crc_packed_small_body: block b sits right-aligned in a slot of 64 G
// bytes, lane g of its group folds [start_b + L - 64 G + 64 g, + 64), a row holds 64/G blocks. Each
// lane loads the five 16-byte granules covering its 64 bytes and realigns them in registers
// (lane_dwords); a granule holding no byte of the block reads the zero buffer, so no load leaves the
// block, and the bytes in front of the block in a straddling granule are masked (leading zeros leave
// an init-0 register at 0). The init term is spread over the group: lane g adds
// bit_i(init) * Shift_L(1 << i) for its 32/G bits i, before the group XOR.
// INIT: the batch has per-block initial registers (a.init_raw); without, the init term is one constant.
template <int G, bool INIT, int DEPTH, int ILP, int PRIO = 0>
__device__ __forceinline__ void crc_packed_small_gen_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(G >= 2 && G <= 32 && (G & (G - 1)) == 0, "G-lane groups of a power of two, 2 to 32");
  static_assert(DEPTH >= ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP (DEPTH - ILP steps in flight)");
  constexpr std::uint32_t kBpr = 64u / G;   // blocks per row
  constexpr int kBits = INIT ? 32 / G : 1;  // init bits per lane
  fill_lds_group<G>(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u, gl = lane % G, lane_blk = lane / G;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t L = a.len;
  std::uint32_t hsr[kBits];  // Shift_L(1 << i) for this lane's init bits
#pragma unroll
  for (int i = 0; i < kBits; ++i) hsr[i] = INIT ? a.tabs->head_shift[L][gl * kBits + i] : 0u;
  const std::uint32_t K = multmodp(a.head_z, a.init_default, a.tabs->poly) ^ a.out_xor;
  __syncthreads();

  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, TR = a.total_rows;
  const std::uint32_t r0 = static_cast<std::uint32_t>(wave * TR / W);
  const std::uint32_t nrows = static_cast<std::uint32_t>((wave + 1) * TR / W) - r0;
  if (nrows == 0) return;
  const std::uint64_t stride = a.stride;
  const std::int64_t c_lane = static_cast<std::int64_t>(L) - 64 * G + 64 * static_cast<std::int64_t>(gl);
  const std::uint64_t row_stride = static_cast<std::uint64_t>(kBpr) * stride;
  const std::uintptr_t blk_base = reinterpret_cast<std::uintptr_t>(a.base) +
                                  (static_cast<std::uint64_t>(r0) * kBpr + lane_blk) * stride;  // block of row 0
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);
  // bytes in front of the block, per dword k of the lane's 64: the low `before` bytes are zeroed
  std::uint32_t zmask[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const std::int64_t before = -(c_lane + 4 * k);
    const std::uint32_t sh = static_cast<std::uint32_t>(before < 0 ? 0 : (before > 4 ? 4 : before)) * 8u;
    zmask[k] = static_cast<std::uint32_t>(0xFFFFFFFFull << sh);
  }

  uint4 buf[DEPTH][kLaneGran];
  std::uint32_t o16[DEPTH], ini[INIT ? DEPTH : 1];
  auto issue = [&](std::uint32_t j, int slot) {
    const std::uint32_t jc = j < nrows ? j : nrows - 1;  // rows past the range reload the last one
    const bool live = static_cast<std::uint64_t>(r0 + jc) * kBpr + lane_blk < a.nblocks;
    if constexpr (INIT) {  // with the granules: a load issued at the fold would drain them all (vmcnt(0))
      const std::uint64_t blk = static_cast<std::uint64_t>(r0 + jc) * kBpr + lane_blk;
      ini[slot] = a.init_raw[blk < a.nblocks ? blk : a.nblocks - 1u];
    }
    const std::uintptr_t blo = blk_base + static_cast<std::uint64_t>(jc) * row_stride, bhi = blo + L;
    const std::uintptr_t p = static_cast<std::uintptr_t>(static_cast<std::int64_t>(blo) + c_lane);
    const std::uintptr_t al = p & ~static_cast<std::uintptr_t>(15);
#pragma unroll
    for (int i = 0; i < kLaneGran; ++i) {
      const std::uintptr_t q = al + 16u * i;
      buf[slot][i] = gload16(live && q + 16u > blo && q < bhi ? q : dmy);
    }
    o16[slot] = static_cast<std::uint32_t>(p & 15u);
  };
  std::uint32_t keep = 0;
  const std::uint32_t keep_src = ((lane % kBpr) * G + (G - 1u)) * 4u;  // byte address for ds_bpermute
  auto finish = [&](std::uint32_t j, std::uint32_t p, int bslot) {
    std::uint32_t v = lane_shift(lds, p, kc);
    if constexpr (INIT) {
      const std::uint32_t init = ini[bslot];
#pragma unroll
      for (int i = 0; i < kBits; ++i)
        v ^= static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(init), gl * kBits + i, 1)) & hsr[i];
      v = group_xor<G>(v) ^ a.out_xor;
    } else {
      v = group_xor<G>(v) ^ K;
    }
    const std::uint32_t pulled = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(keep_src),
                                                                                        static_cast<int>(v)));
    const std::uint32_t slot = j % G;
    keep = lane / kBpr == slot ? pulled : keep;
    if (slot == G - 1u || j + 1u == nrows) {
      const std::uint64_t ob = static_cast<std::uint64_t>(r0 + j - slot) * kBpr + lane;
      if (lane < (slot + 1u) * kBpr && ob < a.nblocks) a.out[ob] = keep;
    }
  };

#pragma unroll
  for (int s = 0; s < DEPTH - ILP; ++s) issue(s, s);
  for (std::uint32_t j = 0; j < nrows; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(nrows - j, nrows);
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + q + DEPTH - ILP + i, (q + DEPTH - ILP + i) % DEPTH);
      const std::uint32_t jq = j + q;
      if (jq >= nrows) break;
      std::uint32_t d[ILP][16];
      Reg p[ILP];
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        lane_dwords<1>(buf[q + i], o16[q + i], d[i]);
        p[i] = Reg{0, 0};
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) slice4(lds, p[i], d[i][k] & zmask[k], kc);
      }
#pragma unroll
      for (int i = 0; i < ILP; ++i)
        if (jq + i < nrows) finish(jq + i, p[i].value(), q + i);
    }
  }
}

// One lane folds one whole block of at most kLaneMax = 64 bytes. It starts from the block's own initial
// register and takes the bytes in the reference's order (crc32.cpp:9-16): whole dwords by slicing-by-4,
// the last len % 4 bytes by Sarwate steps. There is no GF(2) shift, no lane shift and no reduction, so
// a WAL record (26 + |k| + |v| bytes, wal.cpp:25) costs the lookups of its own bytes. The bytes come in
// as the 16-byte aligned granules that cover the block: a granule holding one of the block's bytes
// lies in a page the block maps, so no load can fault whatever the block's alignment. They are
// realigned in registers: two bitwise selects by the start's dword offset within its granule, then
// v_alignbyte by its byte offset. ALIGN 16 (every block start 16-byte aligned) needs neither, ALIGN 4
// (dword aligned) only the selects. (kLaneGran and lane_dwords are declared above.)

// ngr: granules worth loading (a wave-uniform bound; the granules past it are never read).
template <int ALIGN>
__device__ __forceinline__ void lane_issue(std::uintptr_t blk, std::uint32_t n, std::uintptr_t dmy,
                                           uint4 (&g)[kLaneGran], std::uint32_t ngr = kLaneGran) {
  constexpr int NG = ALIGN == 16 ? 4 : kLaneGran;
  const std::uintptr_t al = blk & ~static_cast<std::uintptr_t>(15);
  const std::uintptr_t last = (blk + n - 1u) & ~static_cast<std::uintptr_t>(15);  // used when n >= 1
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const std::uintptr_t p = al + 16u * i;
    // past the block's last granule: that granule again (an L1 hit); an empty block reads `dummy`
    if (static_cast<std::uint32_t>(i) < ngr) g[i] = gload16(n == 0 ? dmy : (p < last ? p : last));
    else g[i] = make_uint4(0, 0, 0, 0);
  }
}

// The 16 little-endian dwords d[k] = bytes [blk + 4k, blk + 4k + 4) from the granules (o = blk & 15).
template <int ALIGN>
__device__ __forceinline__ void lane_dwords(const uint4 (&g)[kLaneGran], std::uint32_t o, std::uint32_t (&d)[16]) {
  constexpr int NG = ALIGN == 16 ? 4 : kLaneGran;
  std::uint32_t raw[4 * kLaneGran];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    raw[4 * i + 0] = g[i].x;
    raw[4 * i + 1] = g[i].y;
    raw[4 * i + 2] = g[i].z;
    raw[4 * i + 3] = g[i].w;
  }
  if constexpr (ALIGN == 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = raw[k];
  } else {
    // bitwise selects: a ternary on a per-lane condition here becomes a dynamically indexed array
    const std::uint32_t m8 = 0u - ((o >> 3) & 1u), m4 = 0u - ((o >> 2) & 1u);
#pragma unroll
    for (int i = 0; i < 18; ++i) raw[i] ^= (raw[i] ^ raw[i + 2]) & m8;
#pragma unroll
    for (int i = 0; i < 17; ++i) raw[i] ^= (raw[i] ^ raw[i + 1]) & m4;
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = ALIGN == 4 ? raw[k] : __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], o & 3u);
  }
}

// Sarwate steps (crc32.cpp:12-14) over the low m <= 3 bytes of w, with T0 from the LDS image.
template <typename KC>
__device__ __forceinline__ std::uint32_t sarwate_bytes(const std::uint32_t* lds, const KC& kc, std::uint32_t c,
                                                       std::uint32_t w, std::uint32_t m) {
#pragma unroll
  for (std::uint32_t j = 0; j < 3u; ++j)
    if (j < m) c = (c >> 8) ^ lds_at(lds, (((c ^ (w >> (8 * j))) & 0xFFu) << 8) | kc.L0);
  return c;
}

// Folds NB blocks (dwords d[i], lengths n[i] <= 64, registers r[i] holding their initial values on
// entry and their final raw registers on return) with their chains interleaved. UNI: every block has
// the same length (uniform batches), so the bounds are wave-uniform and the branches scalar.
template <int NB, bool UNI, typename KC>
__device__ __forceinline__ void lane_fold(const std::uint32_t* lds, const KC& kc, const std::uint32_t (*d)[16],
                                          const std::uint32_t* n, std::uint32_t* r) {
  Reg p[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) p[i] = Reg{r[i], 0};
  if constexpr (UNI) {
    // one scalar branch per dword for all NB chains, so their lookups stay interleaved
    const std::uint32_t len = __builtin_amdgcn_readfirstlane(n[0]);
    const std::uint32_t nf = len >> 2, tb = len & 3u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (static_cast<std::uint32_t>(k) < nf) {
#pragma unroll
        for (int i = 0; i < NB; ++i) slice4(lds, p[i], d[i][k], kc);
      } else {
        if (static_cast<std::uint32_t>(k) == nf && tb != 0u) {
#pragma unroll
          for (int i = 0; i < NB; ++i) p[i] = Reg{sarwate_bytes(lds, kc, p[i].value(), d[i][k], tb), 0};
        }
        break;
      }
    }
  } else {
    std::uint32_t nf[NB], tb[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      nf[i] = n[i] >> 2;
      tb[i] = n[i] & 3u;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if (static_cast<std::uint32_t>(k) < nf[i]) {
          slice4(lds, p[i], d[i][k], kc);
        } else if (static_cast<std::uint32_t>(k) == nf[i] && tb[i] != 0u) {
          p[i] = Reg{sarwate_bytes(lds, kc, p[i].value(), d[i][k], tb[i]), 0};
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) r[i] = p[i].value();
}

// ---- uniform lane batches ---------------------------------------------------------------------------
// Uniform batches of blocks of at most kLaneMax bytes, any stride, alignment and initial registers:
// lane l of wave step s folds block 64 s + l. Waves own contiguous ranges of steps; DEPTH steps of
// loads are in flight and ILP steps fold with interleaved chains (crc_packed_body's pipeline and issue
// priority); each step's 64 results leave in one coalesced store.
// Waves of the round-3 kernel waited on memory (SQ_WAIT_ANY) 64 % of their cycles in uniform 36-byte
// batches and issued VALU 15 % (profiles/r4/lanes_pmc/summary.txt). A uniform batch's block length is
// known at launch, so the window here is exactly the NG granules a block can touch (NG = ceil((len +
// worst misalignment) / 16)) and the registers five-granule windows spent go to more blocks in flight:
// DEPTH 8 at NG <= 2, 6 at 3, 5 at 4. That lifted short blocks (26 B +8 %) but not 36 B: with 16 waves
// per CU (LDS-bound: one 1024-thread workgroup) the SIMDs' VALU is already ~52 % busy there, so more
// loads in flight leave the same issue-latency bound.
template <int ALIGN, int NG>
__device__ __forceinline__ void lane_issue_n(std::uintptr_t blk, std::uint32_t n, std::uintptr_t dmy, uint4 (&g)[NG]) {
  const std::uintptr_t al = blk & ~static_cast<std::uintptr_t>(15);
  const std::uintptr_t last = (blk + n - 1u) & ~static_cast<std::uintptr_t>(15);  // used when n >= 1
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const std::uintptr_t p = al + 16u * i;
    // past the block's last granule: that granule again (an L1 hit); an empty block reads `dummy`
    g[i] = gload16(n == 0 ? dmy : (p < last ? p : last));
  }
}

// d[k] = bytes [blk + 4k, +4) for k < 4 NG - (ALIGN == 16 ? 0 : 1) from the granules (o = blk & 15);
// the rest are don't-care.
template <int ALIGN, int NG>
__device__ __forceinline__ void lane_dwords_n(const uint4 (&g)[NG], std::uint32_t o, std::uint32_t (&d)[4 * NG]) {
  std::uint32_t raw[4 * NG + 3];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    raw[4 * i + 0] = g[i].x;
    raw[4 * i + 1] = g[i].y;
    raw[4 * i + 2] = g[i].z;
    raw[4 * i + 3] = g[i].w;
  }
  raw[4 * NG] = raw[4 * NG + 1] = raw[4 * NG + 2] = 0u;
  if constexpr (ALIGN == 16) {
#pragma unroll
    for (int k = 0; k < 4 * NG; ++k) d[k] = raw[k];
  } else {
    const std::uint32_t m8 = 0u - ((o >> 3) & 1u), m4 = 0u - ((o >> 2) & 1u);
#pragma unroll
    for (int i = 0; i < 4 * NG + 1; ++i) raw[i] ^= (raw[i] ^ raw[i + 2]) & m8;
#pragma unroll
    for (int i = 0; i < 4 * NG + 1; ++i) raw[i] ^= (raw[i] ^ raw[i + 1]) & m4;
#pragma unroll
    for (int k = 0; k < 4 * NG; ++k) d[k] = ALIGN == 4 ? raw[k] : __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], o & 3u);
  }
}

// Right-aligned lane walk for the default initial register, the length's whole-dword count NF a
// compile-time constant: each lane's window is the NF dwords that END at its block's end, starting
// lead = 4 NF - len bytes in front of the block. Those lead bytes (whatever lies there) are masked to
// zero in the first dword, and the NF dwords are folded from register 0, which leading zeros leave at
// 0; so every lane folds the same whole dwords, with no Sarwate tail for the last 1-3 bytes and no
// per-dword branch, and the initial register enters as one uniform term Shift_len(init) =
// head_z * init (head_z = x^(8 len)). ALIGN is the window start's alignment class (the block's when
// lead = 0, bytes otherwise); no load leaves the block's own granules.
template <int ALIGN, int NF, int NG, int DEPTH, int PRIO = 0>
__device__ __forceinline__ void crc_lanes_r_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(NF >= 1 && NF <= 16 && 4 * NF + (ALIGN == 16 ? 0 : ALIGN == 4 ? 12 : 15) <= 16 * NG,
                "the window's NG granules must cover NF dwords at the worst start offset");
  fill_lds_slicing(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t K = multmodp(a.head_z, a.init_default, a.tabs->poly) ^ a.out_xor;
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, nb = a.nblocks;
  const std::uint64_t TS = (nb + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  if (ns == 0) return;
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
    const std::uint32_t len = a.len;                 // 4 NF - 3 .. 4 NF
  const std::uint32_t lead = 4u * NF - len;        // bytes in front of the block in the first dword
  const std::uint32_t m0 = ~0u << (8u * lead);     // (lead <= 3)
  const std::uint64_t blk0 = s0 * 64u + lane;
  const std::uintptr_t lane_base = base + blk0 * a.stride;
  const std::uint64_t step_bytes = 64u * a.stride;
  const std::uintptr_t last_blk = base + (nb - 1u) * a.stride;  // lanes past the batch reload it, store nothing

  uint4 buf[DEPTH][NG];
  std::uint32_t o16[DEPTH];
  auto issue = [&](std::uint32_t j, int slot) {
    const std::uint32_t jc = j < ns ? j : ns - 1;  // steps past the range reload the last one
    const std::uint64_t b = blk0 + 64ull * jc;
    const std::uintptr_t blk = b < nb ? lane_base + jc * step_bytes : last_blk;
    const std::uintptr_t s = blk - lead;
    const std::uintptr_t al = s & ~static_cast<std::uintptr_t>(15);
    const std::uintptr_t first = blk & ~static_cast<std::uintptr_t>(15);
    const std::uintptr_t last = (blk + len - 1u) & ~static_cast<std::uintptr_t>(15);
    // granule 0 is never past the block's last granule, and lies in front of its first one only when
    // the lead bytes cross a granule boundary: it then reloads the first granule (its bytes are masked)
    buf[slot][0] = gload16(al < first ? first : al);
#pragma unroll
    for (int i = 1; i < NG; ++i) {
      const std::uintptr_t p = al + 16u * i;
      buf[slot][i] = gload16(p < last ? p : last);
    }
    o16[slot] = static_cast<std::uint32_t>(s & 15u);
  };
  auto fold = [&](int q, std::uint32_t j) {
    keep_live(buf[q]);
    std::uint32_t d[4 * NG];
    lane_dwords_n<ALIGN, NG>(buf[q], o16[q], d);
    Reg p{0u, 0u};
    slice4(lds, p, d[0] & m0, kc);
#pragma unroll
    for (int k = 1; k < NF; ++k) slice4(lds, p, d[k], kc);
    std::uint32_t v = p.value() ^ K;
    // computed by every lane: sunk into the store's divergent branch, the fold made the compiler
    // drain every load in flight (vmcnt(0)) in front of it
    asm volatile("" : "+v"(v));
    const std::uint64_t b = blk0 + 64ull * j;
    if (b < nb) a.out[b] = v;
  };

#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s) issue(s, s);
  for (std::uint32_t j = 0; j < ns; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(ns - j, ns);
#pragma unroll
    for (int q = 0; q < DEPTH; ++q) {
      issue(j + q + DEPTH - 1, (q + DEPTH - 1) % DEPTH);
      if (j + q >= ns) break;
      fold(q, j + q);
    }
  }
}

template <int ALIGN, int NG, int DEPTH, int ILP, int PRIO = 0, int R = 32>
__device__ __forceinline__ void crc_lanes_n_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH >= ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP (DEPTH - ILP steps in flight)");
  constexpr int ND = 4 * NG;
  static_assert(R == 32 || R == 16, "32- or 16-replica table image");
  if constexpr (R == 32) fill_lds_slicing(a.tabs, lds);
  else fill_lds_slicing16(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const auto kc = [lane] {
    if constexpr (R == 32) return lane_const(lane);
    else return lane_const16(lane);
  }();
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, nb = a.nblocks;
  const std::uint64_t TS = (nb + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  if (ns == 0) return;
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);
  const std::uint32_t len = a.len;
  const std::uint32_t nf = len >> 2, tb = len & 3u;  // whole dwords, tail bytes (uniform)
  const std::uint64_t blk0 = s0 * 64u + lane;
  const std::uintptr_t lane_base = base + blk0 * a.stride;
  const std::uint64_t step_bytes = 64u * a.stride;
  const std::uintptr_t last_blk = base + (nb - 1u) * a.stride;  // lanes past the batch reload it, store nothing

  uint4 buf[DEPTH][NG];
  std::uint32_t ini[DEPTH], o16[DEPTH];
  auto issue = [&](std::uint32_t j, int slot) {
    const std::uint32_t jc = j < ns ? j : ns - 1;  // steps past the range reload the last one
    const std::uint64_t b = blk0 + 64ull * jc;
    const std::uintptr_t blk = b < nb ? lane_base + jc * step_bytes : last_blk;
    lane_issue_n<ALIGN, NG>(blk, len, dmy, buf[slot]);
    o16[slot] = static_cast<std::uint32_t>(blk & 15u);
    ini[slot] = a.init_raw ? a.init_raw[b < nb ? b : nb - 1u] : a.init_default;
  };
  auto fold = [&](auto nb_const, int q, std::uint32_t j) {
    constexpr int NB = decltype(nb_const)::value;
    std::uint32_t d[NB][ND];
    Reg p[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      lane_dwords_n<ALIGN, NG>(buf[q + i], o16[q + i], d[i]);
      p[i] = Reg{ini[q + i], 0};
    }
    // one scalar branch per dword for all NB chains (the length is uniform)
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      if (static_cast<std::uint32_t>(k) < nf) {
#pragma unroll
        for (int i = 0; i < NB; ++i) slice4(lds, p[i], d[i][k], kc);
      } else {
        if (static_cast<std::uint32_t>(k) == nf && tb != 0u) {
#pragma unroll
          for (int i = 0; i < NB; ++i) p[i] = Reg{sarwate_bytes(lds, kc, p[i].value(), d[i][k], tb), 0};
        }
        break;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const std::uint64_t b = blk0 + 64ull * (j + i);
      if (b < nb) a.out[b] = p[i].value() ^ a.out_xor;
    }
  };

#pragma unroll
  for (int s = 0; s < DEPTH - ILP; ++s) issue(s, s);
  for (std::uint32_t j = 0; j < ns; j += DEPTH) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(ns - j, ns);
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + q + DEPTH - ILP + i, (q + DEPTH - ILP + i) % DEPTH);
      const std::uint32_t jq = j + q;
      if (jq >= ns) break;
      if (jq + ILP <= ns) {
        fold(std::integral_constant<int, ILP>{}, q, jq);
      } else {
#pragma unroll
        for (int i = 0; i < ILP; ++i)  // tail: fewer than ILP steps left
          if (jq + i < ns) fold(std::integral_constant<int, 1>{}, q + i, jq + i);
      }
    }
  }
}

// Uniform lane batches staged through LDS (round 4): a wave's 64 blocks of one step are 64 x stride
// contiguous bytes, so the wave copies them to its own LDS buffer with coalesced LDS-DMA
// (global_load_lds_dwordx4: lane l moves bytes [16 l, +16) of each KiB, no VGPRs) one step ahead of
// the fold, and each lane then reads its block's dwords from LDS (dword-aligned blocks: one ds_read
// per dword; others: two reads and v_alignbyte). Against crc_lanes_n this drops the per-lane 16-byte
// granule loads (each wave load touched ~36 lines for 36-byte blocks, three times per step) and the
// realignment selects. For strides up to kLanesLdsMaxStride (a step's bytes fit a 3 KiB buffer) and
// default initial registers; the slicing tables are the 64 KiB 16-replica image, which leaves 96 KiB
// for 16 waves x 2 buffers x 3 KiB.
constexpr std::uint32_t kLanesLdsBuf = 3072;                              // bytes per step buffer
constexpr std::uint32_t kLanesLdsMaxStride = (kLanesLdsBuf - 16u) / 64u;  // 47
template <bool RA, int NW, int KB, int PRIO = 0>
__device__ __forceinline__ void crc_lanes_lds_body(const RowsArgs& a, std::uint32_t* lds) {
  static_assert(NW >= 1 && NW <= 16, "a block's dwords (ceil(len / 4) <= NW)");
  static_assert(KB >= 1 && KB <= static_cast<int>(kLanesLdsBuf / 1024u), "KiB copied per step");
  constexpr std::uint32_t kTabWords = kLdsSliceWords / 2;  // the 64 KiB image
  fill_lds_slicing16(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConstX kc = lane_const16(lane);
  const std::uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + wid;
  const std::uint64_t W = a.nwaves, nb = a.nblocks;
  const std::uint64_t TS = (nb + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  if (ns == 0) return;
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  const std::uint64_t stride = a.stride;
  const std::uint32_t len = a.len;
  const std::uint32_t nf = len >> 2, tb = len & 3u;  // whole dwords, tail bytes (uniform)
  // the batch's last byte's granule: no copy reads past it (bytes beyond the last block are never used)
  const std::uintptr_t glast = (base + (nb - 1u) * stride + (len ? len : 1u) - 1u) & ~static_cast<std::uintptr_t>(15);
  // this wave's two step buffers, byte offsets in LDS
  const std::uint32_t buf0 = kTabWords * 4u + wid * 2u * kLanesLdsBuf;
  auto copy = [&](std::uint32_t j, std::uint32_t buf) {  // step j's bytes into buf (3 DMA instructions)
    const std::uint64_t b0 = (s0 + j) * 64u;
    const std::uintptr_t al = (base + b0 * stride) & ~static_cast<std::uintptr_t>(15);
#pragma unroll
    for (std::uint32_t i = 0; i < static_cast<std::uint32_t>(KB); ++i) {  // KB KiB: the step's bytes and slack
      std::uintptr_t g = al + 1024u * i + 16u * lane;
      g = g < glast ? g : glast;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const __attribute__((address_space(1))) void*>(g),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<std::uintptr_t>(reinterpret_cast<std::uint8_t*>(lds) + buf + 1024u * i)),
                                       16, 0, 0);
    }
  };
  auto lds32 = [&](std::uint32_t byte) { return lds_at(lds, byte); };
  // One step's copy in flight while the previous one folds (issuing and awaiting each step's copy at
  // its fold, or leaving the previous step's result store in flight at the wait, measured slower or
  // neutral: profiles/r4/storewait/, profiles/r4/lanes_lds/).
  copy(0, buf0);
  for (std::uint32_t j = 0; j < ns; ++j) {
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(ns - j, ns);
    const std::uint32_t cur = buf0 + (j & 1u) * kLanesLdsBuf;
    if (j + 1u < ns) {
      copy(j + 1u, buf0 + ((j + 1u) & 1u) * kLanesLdsBuf);
      // step j's copy has landed; step j+1's KB copies stay in flight (vmcnt counts in issue order)
      if constexpr (KB == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if constexpr (KB == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const std::uint64_t b0 = (s0 + j) * 64u;
    const std::uint32_t o = static_cast<std::uint32_t>((base + b0 * stride) & 15u);
    const std::uint32_t q = cur + o + lane * static_cast<std::uint32_t>(stride);  // this lane's block in LDS
    const std::uint32_t qa = q & ~3u, sh = q & 3u;
    (void)qa;
    (void)sh;
    // all NW words first (unconditional reads inside this lane's buffer: the bytes after a block are
    // don't-care), so one LDS round trip covers them before the lookup chain starts
    std::uint32_t w[NW];
    if constexpr (RA) {
      std::uint32_t r[NW + 1];
#pragma unroll
      for (int k = 0; k <= NW; ++k) r[k] = lds32(qa + 4u * k);
#pragma unroll
      for (int k = 0; k < NW; ++k) w[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], sh);
    } else {
#pragma unroll
      for (int k = 0; k < NW; ++k) w[k] = lds32(q + 4u * k);
    }
    Reg p{a.init_default, 0};
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      if (static_cast<std::uint32_t>(k) < nf) {
        slice4(lds, p, w[k], kc);
      } else {
        if (static_cast<std::uint32_t>(k) == nf && tb != 0u) p = Reg{sarwate_bytes(lds, kc, p.value(), w[k], tb), 0};
        break;
      }
    }
    const std::uint64_t b = b0 + lane;
    if (b < nb) a.out[b] = p.value() ^ a.out_xor;
  }
}

// Steps of data in flight ahead of the fold in the lane phase and the group walks (the ring holds
// four), and in the small phase's class-list walks. One step each: in one process against two (walks)
// and three (lists), the listed small-block batches ran 3.1-3.7 % faster (300-1000 B, 0-1024 B,
// 100-700 B, 180-400 B), the group passes up to 1.3 % (profiles/r4/walk_depth/); two list steps
// measured below both one and three. (Earlier in round 4 three list steps had beaten two by
// 0.7-1.6 %, profiles/r4/s12/; the lane phase and group passes spill at three.) 0 = no step ahead
// (10-15 % slower for every walk, profiles/r4/lanes_r/nopf_probe.jsonl).
constexpr int kWalkAhead = 1;
constexpr int kListAhead = 1;
static_assert(kWalkAhead >= 0 && kWalkAhead <= 3 && kListAhead >= 0 && kListAhead <= 3,
              "at most three steps ahead of a four-slot ring");

// Lane blocks of an irregular batch (len <= kLaneMax, in a scan tile the prepass marked dense), walked
// straight from the caller's offsets and lengths (the prepass lists them nowhere): wave w takes the
// blocks [w n / W, (w + 1) n / W) 64 at a time, lane l of step j the block b0 + 64 j + l, and folds it
// if it is such a lane block; other lanes idle.
// Runs in crc_stream's launch when the prepass chose the general path and counted lane blocks, with
// the slicing tables already in LDS. Descriptors are fetched four steps ahead of their data, data two
// steps ahead of the fold, and no loaded value is touched before use (small_phase's pipeline).
__device__ __forceinline__ void lane_phase(const RowsArgs& a, const std::uint32_t* lds) {
  constexpr int RING = 4;
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, n = a.nblocks;
  const std::uint64_t b0 = wave * n / W, b1 = (wave + 1) * n / W;
  if (b0 >= b1) return;
  const std::uint32_t ns = static_cast<std::uint32_t>((b1 - b0 + 63u) / 64u);
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);

  std::uint64_t d_off[RING];
  std::uint32_t d_len[RING];
  auto fetch = [&](std::uint32_t j, int slot) {
    const std::uint64_t b = b0 + 64ull * j + lane;
    const std::uint64_t bc = b < b1 ? b : b1 - 1u;  // clamped: every load stays inside the arrays
    d_off[slot] = a.l_off[bc];
    d_len[slot] = a.l_len[bc];
  };
  uint4 q[RING][kLaneGran];
  std::uint32_t m_len[RING], m_o[RING], m_init[RING];
  auto issue = [&](int slot, std::uint32_t j) {
    const std::uint64_t b = b0 + 64ull * j + lane;
    const bool live = j < ns && b < b1 && d_len[slot] <= kLaneMax && (a.l_tile[b / 4096u] & kTileLanes);
    const std::uint32_t len = live ? d_len[slot] : 0u;
    const std::uintptr_t blk = base + d_off[slot];
    lane_issue<1>(blk, len, dmy, q[slot]);
    m_len[slot] = live ? len : 0xFFFFFFFFu;  // 0xFFFFFFFF: nothing to store
    m_o[slot] = static_cast<std::uint32_t>(blk & 15u);
    m_init[slot] = a.init_raw ? a.init_raw[live ? b : b0] : a.init_default;
  };
  auto fold = [&](int slot, std::uint32_t j) {
    const std::uint32_t len = m_len[slot];
    const bool live = len != 0xFFFFFFFFu;
    if (__ballot(live) == 0) return;  // no lane block in this step
    std::uint32_t d[1][16], nn[1] = {live ? len : 0u}, r[1] = {m_init[slot]};
    lane_dwords<1>(q[slot], m_o[slot], d[0]);
    lane_fold<1, false>(lds, kc, d, nn, r);
    if (live) a.out[b0 + 64ull * j + lane] = r[0] ^ a.out_xor;
  };

#pragma unroll
  for (int k = 0; k < RING; ++k) fetch(k, k);
#pragma unroll
  for (int k = 0; k < kWalkAhead; ++k) {
    issue(k, k);
    fetch(k + RING, k);
  }
  for (std::uint32_t t = 0; t < ns; t += RING) {
#pragma unroll
    for (int k = 0; k < RING; ++k) {
      const int ahead = (k + kWalkAhead) % RING;  // step t+k+kWalkAhead: its descriptor arrived RING steps ago
      issue(ahead, t + k + kWalkAhead);
      fetch(t + k + kWalkAhead + RING, ahead);
      if (t + k < ns) fold(k, t + k);
    }
  }
}

// Group blocks of an irregular batch: a G-lane group folds one block right-aligned in a 64 G-byte
// slot (crc_packed_small_gen's layout), 64/G blocks per wave step. Two walks share the code:
//  * LIST = false, the group phase (tiles dense in a class): straight from the caller's offsets and
//    lengths over the same block range and pipeline as lane_phase (other groups idle). G = 4 takes
//    blocks of kLaneMax + 1 .. kGroupMax bytes, G = 8 up to kGroup8Max, each pass only the blocks of
//    its class in tiles flagged for it;
//  * LIST = true, the small-block phase: entries [lo, lo + cnt) of the prepass lists s_off/s_len/s_idx
//    (one class per list range, so every block but those of the shortest class fills over half its
//    slot), waves owning contiguous ranges of entries.
// Lane g loads the five granules covering its 64 bytes and realigns them (lane_dwords); granules
// holding no byte of the block read the zero buffer and the bytes in front of the block are masked.
// Lane shifts are column 64 - G + g of the LDS image (Shift_{(G-1-g)*64}); the init term is
// Shift_len(init), from init_shift[len] for the default register, or spread over the group (32/G bits
// per lane, head_shift[len]) for per-block registers; the group's sum comes from the first log2(G)
// DPP steps of the wave reduction. Pipeline: data of step t+2 is issued while step t folds;
// descriptors are fetched RING steps ahead of their data. The tables must already be in LDS.
template <int G, bool LIST>
__device__ __forceinline__ void group_walk(const RowsArgs& a, const std::uint32_t* lds, std::uint32_t lo,
                                           std::uint32_t cnt) {
  static_assert(G == 4 || G == 8 || (LIST && G == 16), "4- or 8-lane groups (16 for listed blocks)");
  // 16-lane groups take their fifth granule from the next lane: +2.9 % on 513-1024-byte and +3.9 % on
  // 300-1000-byte payloads in one process; with 4- and 8-lane groups the shuffle cost more than the
  // loads it saved (-6.5 %, -4.5 %; profiles/r4/group_shuf/)
  constexpr bool kShuf = G == 16;
  constexpr int RING = 4;
  constexpr int kAhead = LIST ? kListAhead : kWalkAhead;  // steps of data in flight
  constexpr std::uint32_t kSlot = 64u * G;
  constexpr std::uint32_t kLo = G == 4 ? kLaneMax : kGroupMax;  // the class: (kLo, kSlot]
  constexpr std::uint32_t kFlag = G == 4 ? kTileGroups : kTileGroups8;
  const std::uint32_t lane = threadIdx.x & 63u, gl = lane % G, grp = lane / G;
  LaneConst kc = lane_const(lane);
  kc.lsbase = kLdsLaneBase + (64u - G + gl) * 4u;
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves, n = LIST ? cnt : a.nblocks, first = LIST ? lo : 0u;
  const std::uint64_t b0 = first + wave * n / W, b1 = first + (wave + 1) * n / W;
  if (b0 >= b1) return;
  constexpr std::uint32_t kPer = 64u / G;  // blocks per step
  const std::uint32_t ns = static_cast<std::uint32_t>((b1 - b0 + kPer - 1u) / kPer);
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);

  std::uint64_t d_off[RING];
  std::uint32_t d_len[RING], d_idx[RING];
  auto fetch = [&](std::uint32_t j, int slot) {
    const std::uint64_t b = b0 + kPer * static_cast<std::uint64_t>(j) + grp;
    const std::uint64_t bc = b < b1 ? b : b1 - 1u;  // clamped: every load stays inside the arrays
    if constexpr (LIST) {
      d_off[slot] = a.s_off[bc];
      d_len[slot] = a.s_len[bc];
      d_idx[slot] = a.s_idx[bc];
    } else {
      d_off[slot] = a.l_off[bc];
      d_len[slot] = a.l_len[bc];
      d_idx[slot] = static_cast<std::uint32_t>(bc);
    }
  };
  uint4 q[RING][kLaneGran];
  std::uint32_t m_len[RING], m_o[RING], m_ishift[RING], m_idx[RING];
  std::int32_t m_lead[RING];
  auto issue = [&](int slot, std::uint32_t j) {
    const std::uint64_t b = b0 + kPer * static_cast<std::uint64_t>(j) + grp;
    const std::uint32_t len0 = d_len[slot];
    const bool live = j < ns && b < b1 && len0 <= kSlot && (LIST || (len0 > kLo && (a.l_tile[b / 4096u] & kFlag)));
    const std::uint32_t len = live ? len0 : 0u;
    const std::uintptr_t blo = base + d_off[slot], bhi = blo + len;
    const std::int32_t c_lane = static_cast<std::int32_t>(len) - static_cast<std::int32_t>(kSlot) +
                                64 * static_cast<std::int32_t>(gl);
    const std::uintptr_t p = static_cast<std::uintptr_t>(static_cast<std::int64_t>(blo) + c_lane);
    const std::uintptr_t al = p & ~static_cast<std::uintptr_t>(15);
    // SHUF: a lane's fifth granule is the next lane's first (the group's lanes cover adjacent 64-byte
    // ranges at the same offset), so only the group's last lane loads it and the others take it from
    // their neighbour at the fold (ds_bpermute): 4 + 1/G granule loads per lane instead of 5
#pragma unroll
    for (int i = 0; i < (kShuf ? kLaneGran - 1 : kLaneGran); ++i) {
      const std::uintptr_t g = al + 16u * i;
      q[slot][i] = gload16(live && g + 16u > blo && g < bhi ? g : dmy);
    }
    if constexpr (kShuf) {
      q[slot][kLaneGran - 1] = make_uint4(0u, 0u, 0u, 0u);
      if (gl == G - 1u) {
        const std::uintptr_t g = al + 16u * (kLaneGran - 1);
        q[slot][kLaneGran - 1] = gload16(live && g + 16u > blo && g < bhi ? g : dmy);
      }
    }
    m_len[slot] = live ? len : 0xFFFFFFFFu;  // 0xFFFFFFFF: nothing to fold or store
    m_o[slot] = static_cast<std::uint32_t>(p & 15u);
    m_lead[slot] = c_lane < 0 ? -8 * c_lane : 0;  // bits of the lane's window in front of the block
    if constexpr (LIST) m_idx[slot] = d_idx[slot];  // (a valid batch index even in a dead slot)
    m_ishift[slot] = a.tabs->init_shift[len];  // Shift_len(0xFFFFFFFF), the reference's init (crc32.hpp:39)
  };
  auto out_idx = [&](int slot, std::uint32_t j) -> std::uint64_t {  // the block's batch index (live slots)
    if constexpr (LIST) return m_idx[slot];
    return b0 + kPer * static_cast<std::uint64_t>(j) + grp;
  };
  auto fold = [&](int slot, std::uint32_t j) {
    const std::uint32_t len = m_len[slot];
    const bool live = len != 0xFFFFFFFFu;
    if (__ballot(live) == 0) return;  // no group block in this step
    if constexpr (kShuf) {
      const int src = static_cast<int>(((lane + 1u) & 63u) * 4u);
      const uint4 n0 = q[slot][0];
      const uint4 nb = make_uint4(static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(n0.x))),
                                  static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(n0.y))),
                                  static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(n0.z))),
                                  static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(n0.w))));
      if (gl != G - 1u) q[slot][kLaneGran - 1] = nb;
    }
    std::uint32_t d[16];
    lane_dwords<1>(q[slot], m_o[slot], d);
    const std::uint32_t lead8 = static_cast<std::uint32_t>(m_lead[slot]);
    Reg p{0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) slice4(lds, p, mask_front(d[k], lead8, k), kc);
    std::uint32_t v = lane_shift(lds, p.value(), kc);
    const std::uint32_t L = live ? len : 0u;
    if (a.init_raw) {
      // per-block registers (a rare path): loaded here rather than carried through the ring
      const std::uint32_t init = a.init_raw[live || LIST ? out_idx(slot, j) : b0];
#pragma unroll
      for (std::uint32_t i = 0; i < 32u / G; ++i) {
        const std::uint32_t bit = gl * (32u / G) + i;
        v ^= static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(init), bit, 1)) &
             a.tabs->head_shift[L][bit];
      }
    } else if (gl == 0u) {
      v ^= m_ishift[slot];
    }
    v = group_xor<G>(v);  // every lane of the group holds the group's sum
    if (live && gl == G - 1u) a.out[out_idx(slot, j)] = v ^ a.out_xor;
  };

#pragma unroll
  for (int k = 0; k < RING; ++k) fetch(k, k);
#pragma unroll
  for (int k = 0; k < kAhead; ++k) {
    issue(k, k);
    fetch(k + RING, k);
  }
  for (std::uint32_t t = 0; t < ns; t += RING) {
#pragma unroll
    for (int k = 0; k < RING; ++k) {
      const int ahead = (k + kAhead) % RING;  // step t+k+kAhead: its descriptor arrived RING steps ago
      issue(ahead, t + k + kAhead);
      fetch(t + k + kAhead + RING, ahead);
      if (t + k < ns) fold(k, t + k);
    }
  }
}

template <int G>
__device__ __forceinline__ void group_phase(const RowsArgs& a, const std::uint32_t* lds) {
  group_walk<G, false>(a, lds, 0u, 0u);
}

// Small blocks of an irregular batch (len <= kSmallMax = 1 KiB, listed by the prepass in
// s_off/s_len/s_idx by class): 4-lane groups for blocks of at most kGroupMax bytes, 8-lane groups up
// to kGroup8Max, 16-lane groups for the rest. Runs inside the irregular row kernel, before its rows,
// on the same partition of waves.
__device__ __forceinline__ void small_phase(const RowsArgs& a, const std::uint32_t* lds) {
  const std::uint32_t ns = sload32(a.counts, 1), n4 = sload32(a.counts, kCountSmall4);
  const std::uint32_t n8 = sload32(a.counts, kCountSmall8);
  if (n4) group_walk<4, true>(a, lds, 0u, n4);
  if (n8) group_walk<8, true>(a, lds, n4, n8);
  if (ns - n4 - n8) group_walk<16, true>(a, lds, n4 + n8, ns - n4 - n8);
}

// Combine the partials of blocks that were split between waves: one thread per seam record (two
// per wave) shifts its piece's partial past the rows that follow it in the block and XORs it into
// the block's result, which the head piece seeded with xorout. All pieces of a block combine in
// parallel (a block cut across thousands of waves - one huge span - costs one atomic each).
__device__ __forceinline__ void crc_fixup_body(const RowsArgs& a) {
  const std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (i >= 2ull * a.nwaves) return;
  const Seam s = a.seams[i];
  if ((s.flags & kSeamValid) == 0) return;
  const std::uint32_t contrib = shift_rows(a.tabs, s.partial, s.rows_after);
  const std::uint64_t ob = a.out_idx ? a.out_idx[s.block] : s.block;
  __hip_atomic_fetch_xor(a.out + ob, contrib, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dev
}  // namespace tkv