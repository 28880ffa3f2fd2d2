// CDNA4 (gfx950) kernels for batched CRC-32/ISO-HDLC — the hot path of tinykvpp's integrity code.
//
// Replaces the byte loop of frankie::core::crc32::update (/root/reference/src/core/crc32.cpp:9-16)
// for batches of independent blocks (WAL records, SSTable blocks). Bit-exact with the reference:
// reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF (crc32.hpp:9-11, crc32.cpp:19).
//
// Decomposition. Notation: Shift_n(v) = register after n zero bytes from v
// (= v * x^(8n) mod P); crc_s(D) = Shift_|D|(s) ^ crc_0(D) (the CRC register is affine in s).
//  * A block of n bytes is cut into 4 KiB "rows" aligned to the block END; row 0 (the head, h bytes)
//    may be partial and is zero-padded in front (leading zeros leave an init-0 register at 0).
//  * One wave folds one row: lane l owns the contiguous 64 bytes [l*64, l*64+64) of the row (four
//    16-byte global loads) and folds them with slicing-by-4 lookups into LDS tables replicated 32x,
//    so lane c of each 32-lane half always reads bank c (conflict-free ds_read_b32); each lookup
//    address is one v_perm_b32.
//  * Lane partials are moved to the row end with lane-specific nibble tables (Shift_{(63-l)*64}).
//    In the same DPP xor-reduction, lanes 0..31 add bit l of the running block register times
//    Shift_4096(1<<l) (Horner step over rows) and, on a head row, lanes 32..63 add bit l-32 of the
//    block's initial register times Shift_h(1<<(l-32)) — so the initial register never touches the
//    data and every length (0..3 bytes included) is exact.
//  * Waves own contiguous, balanced ranges of rows; a block cut between waves leaves "seam"
//    partials that crc_fixup combines with x^(8*4096*k) mod P products.
#include <hip/hip_runtime.h>

#include "tkv_crc32_internal.h"

namespace tkv {

namespace {

// Global (VMEM) and constant (SMEM) address-space views.
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1))) g_v4u;
typedef const std::uint32_t __attribute__((address_space(1))) g_u32;

__device__ __forceinline__ uint4 gload16(std::uintptr_t p) {
  const v4u v = *reinterpret_cast<g_v4u*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
typedef const std::uint32_t __attribute__((address_space(4))) c_u32;
typedef const std::uint64_t __attribute__((address_space(4))) c_u64;

__device__ __forceinline__ std::uint32_t sload32(const std::uint32_t* p, std::uint32_t i) {
  return reinterpret_cast<c_u32*>(reinterpret_cast<std::uintptr_t>(p))[i];
}
__device__ __forceinline__ std::uint64_t sload64(const std::uint64_t* p, std::uint32_t i) {
  return reinterpret_cast<c_u64*>(reinterpret_cast<std::uintptr_t>(p))[i];
}

__device__ __forceinline__ std::uint32_t lds_at(const std::uint32_t* lds, std::uint32_t byte_addr) {
  return *reinterpret_cast<const std::uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// One slicing-by-4 step over a little-endian dword: crc ^= w; crc = T3[b0]^T2[b1]^T1[b2]^T0[b3].
// Lk holds {byte0 = t*128 + c*4, byte2 = pair} of table k = 2*pair + t; v_perm_b32 drops byte j of
// x into byte1 (entry*256), giving the full LDS byte address in one instruction.
__device__ __forceinline__ std::uint32_t slice4(const std::uint32_t* lds, std::uint32_t crc, std::uint32_t w,
                                                std::uint32_t L0, std::uint32_t L1, std::uint32_t L2,
                                                std::uint32_t L3) {
  const std::uint32_t x = crc ^ w;
  const std::uint32_t a0 = __builtin_amdgcn_perm(x, L3, 0x0C020400u);
  const std::uint32_t a1 = __builtin_amdgcn_perm(x, L2, 0x0C020500u);
  const std::uint32_t a2 = __builtin_amdgcn_perm(x, L1, 0x0C020600u);
  const std::uint32_t a3 = __builtin_amdgcn_perm(x, L0, 0x0C020700u);
  return (lds_at(lds, a0) ^ lds_at(lds, a1)) ^ (lds_at(lds, a2) ^ lds_at(lds, a3));
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

// a*b mod P in the reflected representation (x^0 = 0x80000000).
__device__ __forceinline__ std::uint32_t d_multmodp(std::uint32_t a, std::uint32_t b) {
  std::uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
  }
  return p;
}

// reg * x^(8*kRow*k) mod P.
__device__ __forceinline__ std::uint32_t d_shift_rows(const DeviceTables* t, std::uint32_t reg, std::uint32_t k) {
  std::uint32_t m = 0x80000000u;  // x^0
  for (int i = 0; k != 0; ++i, k >>= 1)
    if (k & 1u) m = d_multmodp(m, t->row_pow[i]);
  return d_multmodp(m, reg);
}

struct Cursor {
  std::uint32_t b;          // block index
  std::uint32_t r;          // row within the block
  std::uint32_t R;          // rows of the block
  std::uint32_t n;          // bytes of the block
  const std::uint8_t* blk;  // block start
};

template <bool UNIFORM>
__device__ __forceinline__ void load_desc(const RowsArgs& a, Cursor& c) {
  const std::uint32_t b = c.b < a.nblocks ? c.b : a.nblocks - 1;
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
__device__ __forceinline__ void advance(const RowsArgs& a, Cursor& c) {
  if (++c.r == c.R) {
    c.r = 0;
    ++c.b;
    load_desc<UNIFORM>(a, c);
  }
}

// Issue the loads of this lane's 64-byte segment of row c.r: NP aligned 16-byte pieces, plus (for
// irregular batches) this lane's Shift_h constant when the row is a head row. Pieces that do not
// overlap the block and rows past the wave's range read the zero `dummy` buffer.
template <int NP, bool UNIFORM>
__device__ __forceinline__ void issue_row(const RowsArgs& a, const Cursor& c, bool live, std::uint32_t lane,
                                          uint4 (&buf)[NP], std::uint32_t& hs) {
  const std::int64_t rowstart =
      static_cast<std::int64_t>(c.n) - static_cast<std::int64_t>(c.R - c.r) * kRow;
  const std::uintptr_t blo = reinterpret_cast<std::uintptr_t>(c.blk);
  const std::uintptr_t bhi = blo + c.n;
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);
  const std::uintptr_t seg = static_cast<std::uintptr_t>(static_cast<std::int64_t>(blo) + rowstart) + lane * kSeg;
  const std::uintptr_t al = seg & ~static_cast<std::uintptr_t>(15);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const std::uintptr_t p = al + 16u * i;
    const bool ok = live && (p + 16 > blo) && (p < bhi);
    buf[i] = gload16(ok ? p : dmy);
  }
  if constexpr (!UNIFORM) {
    const std::uintptr_t hp =
        reinterpret_cast<std::uintptr_t>(&a.tabs->head_shift[head_len(c.n)][lane & 31u]);
    hs = *reinterpret_cast<g_u32*>((live && c.r == 0) ? hp : dmy);
  }
}

template <bool ALIGNED, bool UNIFORM>
__global__ __launch_bounds__(kThreads) void crc_rows(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  constexpr int NP = ALIGNED ? 4 : 5;

  // ---- prologue: replicate the tables into LDS --------------------------------------------------
  for (std::uint32_t i = threadIdx.x; i < kLdsSliceWords; i += kThreads) {
    const std::uint32_t pair = i >> 14, e = (i >> 6) & 255u, t = (i >> 5) & 1u;
    lds[i] = a.tabs->slice[2 * pair + t][e];
  }
  const std::uint32_t* ls = &a.tabs->lane_shift[0][0][0];
  for (std::uint32_t i = threadIdx.x; i < kLdsLaneWords; i += kThreads) lds[kLdsSliceWords + i] = ls[i];

  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t c4 = (lane & 31u) << 2;
  const std::uint32_t L0 = c4, L1 = 128u + c4, L2 = 0x10000u + c4, L3 = 0x10080u + c4;
  const std::uint32_t lsbase = kLdsLaneBase + lane * 4u;
  const bool lo_half = lane < 32u;
  // Horner constants (lanes 0..31); for uniform batches lanes 32..63 hold Shift_h(1 << (l-32)).
  std::uint32_t hcon = a.tabs->horner[lane];
  if constexpr (UNIFORM) {
    if (!lo_half) hcon = d_multmodp(a.head_z, 1u << (lane - 32u));
  }
  __syncthreads();

  const std::uint32_t wave = blockIdx.x * kWavesPerWG + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves;

  // ---- this wave's contiguous range of rows [g0, g1) --------------------------------------------
  std::uint32_t g0, g1;
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
    const std::uint64_t TR = sload32(a.row_scan, a.nblocks);
    g0 = static_cast<std::uint32_t>(wave * TR / W);
    g1 = static_cast<std::uint32_t>((wave + 1) * TR / W);
    cur.b = g0 < g1 ? sload32(a.wave_start, wave) : 0u;
    cur.r = g0 < g1 ? g0 - sload32(a.row_scan, cur.b) : 0u;
  }

  // Seam records (uniform state, written by lane 0 at the end).
  std::uint32_t s_block[2] = {0, 0}, s_part[2] = {0, 0}, s_after[2] = {0, 0}, s_flags[2] = {0, 0};

  if (g0 < g1) {
    load_desc<UNIFORM>(a, cur);
    std::uint32_t B = 0;           // running register of the current block piece (Horner over rows)
    bool piece_has_row0 = cur.r == 0;
    bool first_piece = true;

    auto process = [&](const Cursor& c, uint4 (&buf)[NP], std::uint32_t hs, std::uint32_t g) {
      std::uint32_t dw[16];
      if constexpr (ALIGNED) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dw[4 * i + 0] = buf[i].x;
          dw[4 * i + 1] = buf[i].y;
          dw[4 * i + 2] = buf[i].z;
          dw[4 * i + 3] = buf[i].w;
        }
      } else {
        std::uint32_t raw[20];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          raw[4 * i + 0] = buf[i].x;
          raw[4 * i + 1] = buf[i].y;
          raw[4 * i + 2] = buf[i].z;
          raw[4 * i + 3] = buf[i].w;
        }
        // Every segment of a block has the same misalignment (segments start at end - k*64).
        const std::uint32_t s =
            static_cast<std::uint32_t>((reinterpret_cast<std::uintptr_t>(c.blk) + c.n) & 15u);
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
        // Head row: zero the bytes in front of the block inside a piece that straddles its start
        // (whole pieces in front of it were loaded from `dummy`).
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

      // Fold this lane's 64 bytes from a zero register.
      std::uint32_t p = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) p = slice4(lds, p, dw[k], L0, L1, L2, L3);

      // Move the lane partial to the row end: Shift_{(63-lane)*64}(p) via 8 nibble lookups.
      std::uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) v ^= lds_at(lds, lsbase + 4096u * j + (((p >> (4 * j)) & 15u) << 8));

      // Horner step (lanes 0..31: Shift_4096(B)) and, on a head row, init injection (lanes 32..63:
      // Shift_h(init)): v ^= bit_(l&31)(sel) * hcon.
      std::uint32_t init = 0;
      if (c.r == 0) init = a.init_raw ? sload32(a.init_raw, c.b) : a.init_default;
      std::uint32_t hk = hcon;
      if constexpr (!UNIFORM) hk = lo_half ? hcon : hs;
      const std::uint32_t sel = lo_half ? B : init;
      v ^= static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(sel), lane & 31u, 1)) & hk;

      const std::uint32_t Bn = __builtin_amdgcn_readlane(wave_xor_to_lane63(v), 63);

      if (c.r + 1 == c.R || g + 1 == g1) {
        if (piece_has_row0 && c.r + 1 == c.R) {
          if (lane == 0) a.out[c.b] = Bn ^ a.out_xor;
        } else {
          const int slot = first_piece ? 0 : 1;
          s_block[slot] = c.b;
          s_part[slot] = Bn;
          s_after[slot] = c.R - 1 - c.r;
          s_flags[slot] = kSeamValid | (piece_has_row0 ? kSeamHasRow0 : 0u);
        }
        first_piece = false;
        piece_has_row0 = true;
        B = 0;
      } else {
        B = Bn;
      }
    };

    uint4 bufA[NP], bufB[NP];
    std::uint32_t hsA = 0, hsB = 0;
    issue_row<NP, UNIFORM>(a, cur, true, lane, bufA, hsA);
    Cursor nxt = cur;
    advance<UNIFORM>(a, nxt);
    for (std::uint32_t g = g0; g < g1; g += 2) {
      issue_row<NP, UNIFORM>(a, nxt, g + 1 < g1, lane, bufB, hsB);
      process(cur, bufA, hsA, g);
      if (g + 1 >= g1) break;
      Cursor n2 = nxt;
      advance<UNIFORM>(a, n2);
      issue_row<NP, UNIFORM>(a, n2, g + 2 < g1, lane, bufA, hsA);
      process(nxt, bufB, hsB, g + 1);
      cur = n2;
      nxt = n2;
      advance<UNIFORM>(a, nxt);
    }
  }

  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Seam rec;
      rec.block = s_block[s];
      rec.partial = s_part[s];
      rec.rows_after = s_after[s];
      rec.flags = s_flags[s];
      a.seams[2 * static_cast<std::uint64_t>(wave) + s] = rec;
    }
  }
}

// Combine the partials of blocks that were split between waves. One thread per wave; the thread
// whose wave holds a block's head row walks the following waves' first pieces.
__global__ void crc_fixup(RowsArgs a) {
  const std::uint64_t w = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (w >= a.nwaves) return;
  for (int slot = 0; slot < 2; ++slot) {
    const Seam s = a.seams[2 * w + slot];
    if ((s.flags & kSeamValid) == 0 || (s.flags & kSeamHasRow0) == 0) continue;
    std::uint32_t acc = d_shift_rows(a.tabs, s.partial, s.rows_after);
    std::uint32_t after = s.rows_after;
    for (std::uint64_t ww = w + 1; after != 0 && ww < a.nwaves; ++ww) {
      const Seam t = a.seams[2 * ww];
      if ((t.flags & kSeamValid) == 0) continue;  // wave with an empty row range
      acc ^= d_shift_rows(a.tabs, t.partial, t.rows_after);
      after = t.rows_after;
    }
    a.out[s.block] = acc ^ a.out_xor;
  }
}

}  // namespace

// ---- irregular-batch prepass: rows per block, exclusive scan, first block of every wave ------------
constexpr int kScanTile = 4096;  // blocks per scan workgroup (1024 threads x 4)

__global__ __launch_bounds__(1024) void rows_tile_scan(const std::uint32_t* lengths, std::uint32_t n,
                                                      std::uint32_t* row_scan, std::uint32_t* tile_sums) {
  __shared__ std::uint32_t part[1024];
  const std::uint64_t base = static_cast<std::uint64_t>(blockIdx.x) * kScanTile + threadIdx.x * 4u;
  std::uint32_t v[4], s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = (base + i < n) ? rows_for_len(lengths[base + i]) : 0u;
    s += v[i];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan of thread sums
    const std::uint32_t x = threadIdx.x >= static_cast<unsigned>(off) ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  std::uint32_t run = part[threadIdx.x] - s;  // exclusive
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base + i < n) row_scan[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 1023) tile_sums[blockIdx.x] = part[1023];
}

__global__ __launch_bounds__(1024) void rows_scan_tiles(std::uint32_t* tile_sums, std::uint32_t ntiles,
                                                       std::uint32_t* row_scan, std::uint32_t n) {
  __shared__ std::uint32_t part[1024];
  std::uint32_t carry = 0;
  for (std::uint32_t t0 = 0; t0 < ntiles; t0 += 1024) {
    const std::uint32_t i = t0 + threadIdx.x;
    const std::uint32_t x = i < ntiles ? tile_sums[i] : 0u;
    part[threadIdx.x] = x;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const std::uint32_t y = threadIdx.x >= static_cast<unsigned>(off) ? part[threadIdx.x - off] : 0u;
      __syncthreads();
      part[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < ntiles) tile_sums[i] = carry + part[threadIdx.x] - x;  // exclusive tile offset
    const std::uint32_t tot = part[1023];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) row_scan[n] = carry;  // total rows
}

__global__ void rows_finish(const std::uint32_t* lengths, std::uint32_t n, std::uint32_t* row_scan,
                            const std::uint32_t* tile_offs, std::uint32_t* wave_start, std::uint32_t W) {
  const std::uint64_t b = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (b >= n) return;
  const std::uint64_t lo = row_scan[b] + tile_offs[b / kScanTile];
  row_scan[b] = static_cast<std::uint32_t>(lo);
  const std::uint64_t hi = lo + rows_for_len(lengths[b]);
  const std::uint64_t TR = row_scan[n];
  // waves whose first row g0(w) = floor(w*TR/W) lies in [lo, hi): w in [ceil(lo*W/TR), ceil(hi*W/TR))
  const std::uint64_t wlo = (lo * W + TR - 1) / TR;
  const std::uint64_t whi = (hi * W + TR - 1) / TR;
  for (std::uint64_t w = wlo; w < whi && w < W; ++w) wave_start[w] = static_cast<std::uint32_t>(b);
}

// ---- synthetic data: byte j of block b = LE byte j%8 of
//      splitmix64((b << 24) ^ (j >> 3) ^ (seed << 56)). Test/bench input generation only. ----------
__device__ __forceinline__ std::uint64_t splitmix64(std::uint64_t x) {
  std::uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Uniform blocks, len % 8 == 0, block start 8-byte aligned: one 8-byte word per thread-iteration.
__global__ void fill_uniform(std::uint8_t* dst, std::uint64_t stride, std::uint64_t len, std::uint64_t first,
                             std::uint64_t nblocks, std::uint64_t seed) {
  const std::uint64_t words = len / 8;
  const std::uint64_t total = nblocks * words;
  for (std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<std::uint64_t>(gridDim.x) * blockDim.x) {
    const std::uint64_t bl = i / words, j8 = i - bl * words;
    const std::uint64_t b = first + bl;
    *reinterpret_cast<std::uint64_t*>(dst + bl * stride + j8 * 8) = splitmix64((b << 24) ^ j8 ^ (seed << 56));
  }
}

// Arbitrary blocks (offsets/lengths, any alignment): one workgroup per block, byte stores.
__global__ void fill_blocks(std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                            std::uint64_t first, std::uint64_t nblocks, std::uint64_t seed) {
  for (std::uint64_t bl = blockIdx.x; bl < nblocks; bl += gridDim.x) {
    const std::uint64_t b = first + bl;
    std::uint8_t* d = base + offsets[bl];
    const std::uint64_t n = lengths[bl];
    for (std::uint64_t j8 = threadIdx.x; j8 * 8 < n; j8 += blockDim.x) {
      const std::uint64_t w = splitmix64((b << 24) ^ j8 ^ (seed << 56));
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (j8 * 8 + k < n) d[j8 * 8 + k] = static_cast<std::uint8_t>(w >> (8 * k));
    }
  }
}

// ---- launchers (called from tkv_crc32_host.cpp) ----------------------------------------------------
hipError_t launch_rows(const RowsArgs& a, bool aligned, bool uniform, unsigned grid, hipStream_t st) {
  if (uniform) {
    if (aligned) hipLaunchKernelGGL((crc_rows<true, true>), dim3(grid), dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((crc_rows<false, true>), dim3(grid), dim3(kThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((crc_rows<false, false>), dim3(grid), dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_fixup(const RowsArgs& a, hipStream_t st) {
  const unsigned grid = (a.nwaves + 255u) / 256u;
  hipLaunchKernelGGL(crc_fixup, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_prepass(const std::uint32_t* lengths, std::uint32_t n, std::uint32_t* row_scan,
                          std::uint32_t* tile_sums, std::uint32_t* wave_start, std::uint32_t W, hipStream_t st) {
  const std::uint32_t ntiles = (n + kScanTile - 1) / kScanTile;
  hipLaunchKernelGGL(rows_tile_scan, dim3(ntiles), dim3(1024), 0, st, lengths, n, row_scan, tile_sums);
  hipLaunchKernelGGL(rows_scan_tiles, dim3(1), dim3(1024), 0, st, tile_sums, ntiles, row_scan, n);
  hipLaunchKernelGGL(rows_finish, dim3((n + 255) / 256), dim3(256), 0, st, lengths, n, row_scan, tile_sums,
                     wave_start, W);
  return hipGetLastError();
}

std::uint32_t prepass_tiles(std::uint32_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t launch_fill_uniform(std::uint8_t* dst, std::uint64_t stride, std::uint64_t len, std::uint64_t first,
                               std::uint64_t nblocks, std::uint64_t seed, hipStream_t st) {
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, st, dst, stride, len, first, nblocks, seed);
  return hipGetLastError();
}

hipError_t launch_fill_blocks(std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                              std::uint64_t first, std::uint64_t nblocks, std::uint64_t seed, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(nblocks < 65536 ? nblocks : 65536);
  if (grid) hipLaunchKernelGGL(fill_blocks, dim3(grid), dim3(256), 0, st, base, offsets, lengths, first, nblocks, seed);
  return hipGetLastError();
}

}  // namespace tkv
