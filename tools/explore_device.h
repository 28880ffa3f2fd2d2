// Explorer-only device code (not product): the variant bodies tools/explore.hip A/Bs against the
// product kernels. The product header (tinykvpp_amd/csrc/tkv_crc32_device.h) holds only what
// tkv_crc32_kernels.hip instantiates; the full-featured bodies below reduce to the product loops
// with their default template arguments (x_packed_body<D, I, R1> == crc_packed_body<D, I, R1>,
// x_rows_body<A, U, D, I, 0> == crc_rows_body<A, U, D, I>), so the explorer's "product" rows
// measure the same code.
#pragma once

#include "tkv_crc32_device.h"

namespace tkv {

// Kernel arguments of the explorer: the product's plus the fields only its variants use.
struct XArgs : RowsArgs {
  std::uint32_t* wg_ctr;          // per-workgroup / per-pool work counters, kCtrStride words apart
  unsigned long long* prog;       // per-wave progress stamps (x_packed_body PROG)
  const std::uint32_t* shift32;   // [j][v] = Shift_32(v << 4j), 128 words: joins two 32-byte half chains
};
constexpr std::uint32_t kProgSlots = 64;
constexpr std::uint32_t kCtrStride = 32;  // one work counter per 128-byte line

namespace dev {

// Non-temporal variant (global_load_dwordx4 ... nt): streamed bytes are read exactly once.
__device__ __forceinline__ uint4 gload16_nt(std::uintptr_t p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<g_v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Shift_32(p) from a 128-entry nibble table held in two VGPRs (lane i of s32[h] = entry 64h + i),
// read with ds_bpermute (LDS crossbar, no LDS memory): joins a lane's two 32-byte half chains.
__device__ __forceinline__ std::uint32_t shift32_bperm(std::uint32_t p, std::uint32_t s32lo, std::uint32_t s32hi) {
  std::uint32_t l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const std::uint32_t addr = (static_cast<std::uint32_t>((j & 3) * 16) + ((p >> (4 * j)) & 15u)) << 2;
    l[j] = static_cast<std::uint32_t>(
        __builtin_amdgcn_ds_bpermute(static_cast<int>(addr), static_cast<int>(j < 4 ? s32lo : s32hi)));
  }
  return xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), l[6] ^ l[7]);
}

// MODE 0: CRC. MODE 1 (explorer only): same loads, XOR of the data instead of the CRC (memory
// ceiling of this access pattern).
// SMALL (irregular batches): when a wave runs its share of the small-block phase. 0: before its
// rows; 1: even waves before their rows, odd waves after them, so the phase's latency-bound steps
// overlap other waves' row streaming instead of all waves idling the HBM at once; 2: after its rows.
// PRIO: issue priority from the rows a wave has left (as crc_packed_body).
template <bool ALIGNED, bool UNIFORM, int DEPTH, int ILP, int MODE, int SMALL = 0, int PRIO = 0>
__device__ __forceinline__ void x_rows_body(const XArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  constexpr int NP = ALIGNED ? 4 : 5;
  if constexpr (MODE == 0) fill_lds(a.tabs, lds);

  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  std::uint32_t hcon = a.tabs->horner[lane];
  if constexpr (UNIFORM) {
    if (lane >= 32u) hcon = multmodp(a.head_z, 1u << (lane - 32u), a.tabs->poly);  // Shift_h(1 << (l-32))
  }
  __syncthreads();
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool small_first = SMALL == 0 || (SMALL == 1 && (wave & 1u) == 0u);
  if constexpr (!UNIFORM && MODE == 0) {
    if (small_first) small_phase(a, lds);
  }
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
    // large blocks only (compacted by the prepass); small ones are crc_small's
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
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
          v[i] = 0;
#pragma unroll
          for (int t = 0; t < 16; ++t) v[i] ^= d[i][t];
        }
      } else {
        Reg p[n];
#pragma unroll
        for (int i = 0; i < n; ++i) p[i] = Reg{0, 0};
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
          for (int i = 0; i < n; ++i) slice4(lds, p[i], d[i][t], kc);
#pragma unroll
        for (int i = 0; i < n; ++i) v[i] = lane_shift(lds, p[i].value(), kc);
      }
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

  if constexpr (!UNIFORM && MODE == 0) {
    if (!small_first) small_phase(a, lds);
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

__device__ __forceinline__ void crc_small_body(const XArgs& a, std::uint32_t* lds) {
  fill_lds(a.tabs, lds);
  __syncthreads();
  small_phase(a, lds);
}

// Packed uniform fast path: block b = [base + b*len, +len) with len a multiple of kRow (4 KiB) and
// 16-byte aligned base, so every row is full, row g of the batch sits at base + g*kRow, and the head
// length is kRow (init injection constants = the Horner constants). Each wave owns the contiguous
// blocks [b0, b1) (no seams), keeps ILP rows' slicing chains interleaved and DEPTH-ILP rows in
// flight, and stores its results 64 at a time (lane k holds its k-th block). R1: one row per block
// (4 KiB blocks), so no Horner state at all. The SIMDs are issue-bound here (PMC: every SIMD issues
// ~96 % of cycles), so the loop is written for instruction count: incremental row addressing, no
// divisions, selects instead of divergent branches.
// CHK (explorer only, R1, nblocks a multiple of 64*waves): chunk-strided map - wave w owns chunks
// w, w+W, w+2W, ... of 2^CHK consecutive blocks instead of one contiguous range.
// PROG (explorer only): lane 0 stamps s_memrealtime into a.prog[wave * kProgSlots + s] after the table
// fill (s = 0), before every PROG-th row (s = 1 + j / PROG) and at the end (last slot used + 1).
// SUB: the caller has filled the LDS tables and passes the wave's block range [sub_b0, sub_b0 + sub_nb)
// (crc_packed_xq_body's static region).
// SKEW (0: off): the waves of a 1024-thread workgroup share its equal slice of the batch in
// proportion to 256 * (SKEW/256)^(slot/4): slots 0-3 (the first wave on each SIMD) get the largest
// ranges, slots 12-15 the smallest, matching the issue arbitration that favours a SIMD's older waves.
// PRIO (0: off): set_prio_from_left<PRIO> once per DEPTH rows (the product uses 3, and SKEW 154 for
// blocks of more than one row; tkv_crc32_kernels.hip).
// EARLY: a wave issues its first DEPTH-ILP row loads before the LDS table fill, so the fill and the
// first loads' latency overlap (explorer probe).
template <int DEPTH, int ILP, bool R1, bool SPLIT = false, std::uint32_t ROT = 0, int CHK = 0, int PROG = 0,
          bool SUB = false, int SKEW = 0, int PRIO = 0, bool EARLY = false>
__device__ __forceinline__ void x_packed_body(const XArgs& a, std::uint32_t* lds, std::uint32_t sub_b0 = 0,
                                                std::uint32_t sub_nb = 0) {
  static_assert(CHK == 0 || (R1 && ROT == 0 && CHK <= 6), "chunk-strided map: R1 only, chunks of <= 64 blocks");
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  static_assert(!EARLY || (!SUB && ROT == 0 && CHK == 0), "early issue: whole-kernel contiguous map only");
  if constexpr (!SUB && !EARLY) fill_lds(a.tabs, lds);
  const std::uint32_t lane = threadIdx.x & 63u;
  const LaneConst kc = lane_const(lane);
  const std::uint32_t hcon = a.tabs->horner[lane & 31u];  // Shift_4096(1 << (l & 31))
  const bool lo_half = lane < 32u;
  // Init injection term for blocks without a per-block init: bit (l-32) of init * Shift_4096(...)
  const std::uint32_t inj_const =
      lo_half ? 0u
              : static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(a.init_default),
                                                                lane & 31u, 1)) & hcon;
  std::uint32_t s32lo = 0, s32hi = 0;
  if constexpr (SPLIT) {
    s32lo = a.shift32[lane];
    s32hi = a.shift32[64 + lane];
  }
  if constexpr (!SUB && !EARLY) __syncthreads();

  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint64_t W = a.nwaves;
  const std::uint32_t R = R1 ? 1u : a.len / kRow;
  std::uint32_t b0, nb;
  if constexpr (SUB) {
    b0 = sub_b0;
    nb = sub_nb;
  } else if constexpr (SKEW != 0) {
    static_assert(CHK == 0 && ROT == 0, "skewed ranges: contiguous map only");
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
  if (!EARLY && nb == 0) return;  // EARLY: such a wave still fills its share of the tables
  const std::uint32_t nrows = nb * R;  // wave-local rows j = 0 .. nrows-1, contiguous in memory
  // CHK: global block of wave-local block j
  auto gblk = [&](std::uint32_t j) -> std::uint64_t {
    return (static_cast<std::uint64_t>(j >> CHK) * W + wave) * (1u << CHK) + (j & ((1u << CHK) - 1u));
  };
  const std::uintptr_t lane_base =
      reinterpret_cast<std::uintptr_t>(a.base) + static_cast<std::uint64_t>(b0) * R * kRow + lane * kSeg;
  // ROT != 0: the wave walks its blocks starting at block (wave*ROT) mod nb and wraps around, so at
  // any instant the waves sit at different offsets inside their ranges (address bits below the
  // range size differ from wave to wave instead of being equal).
  const std::uint32_t rot_b = ROT ? static_cast<std::uint32_t>((wave * static_cast<std::uint64_t>(ROT)) % nb) : 0u;
  auto stamp = [&](std::uint32_t slot) {
    if constexpr (PROG > 0) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (lane == 0 && slot < kProgSlots) a.prog[static_cast<std::uint64_t>(wave) * kProgSlots + slot] = t;
    }
  };
  stamp(0);
  const std::uint32_t rotr = rot_b * R;

  uint4 buf[DEPTH][4];
  auto issue = [&](std::uint32_t j, uint4 (&q)[4]) {
    std::uint32_t jc = j < nrows ? j : nrows - 1;  // rows past the range reload the last one
    if constexpr (ROT != 0) {
      jc += rotr;
      jc -= jc >= nrows ? nrows : 0u;
    }
    const std::uintptr_t p = CHK ? reinterpret_cast<std::uintptr_t>(a.base) + lane * kSeg + gblk(jc) * kRow
                                 : lane_base + static_cast<std::uint64_t>(jc) * kRow;
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
        std::uint32_t kk = k + rot_b;
        kk -= kk >= nb ? nb : 0u;
        const std::uint32_t init = sload32(a.init_raw, b0 + kk);
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
        std::uint32_t li = k - slot + lane + rot_b;  // wave-local block of lane's result
        li -= li >= nb ? nb : 0u;
        if (lane <= slot) a.out[CHK ? gblk(k - slot + lane) : b0 + li] = keep;
      }
      r = 0;
      ++k;
      B = 0;
    } else {
      B = Bn;
    }
  };

  if constexpr (EARLY) {
    if (nb != 0) {
#pragma unroll
      for (int s = 0; s < DEPTH - ILP; ++s) issue(s, buf[s]);
    }
    fill_lds(a.tabs, lds);
    __syncthreads();
    if (nb == 0) return;
  } else {
#pragma unroll
    for (int s = 0; s < DEPTH - ILP; ++s) issue(s, buf[s]);
  }
  for (std::uint32_t j = 0; j < nrows; j += DEPTH) {
    if constexpr (PROG > 0) {
      if (j % PROG == 0) stamp(1 + j / PROG);
    }
    if constexpr (PRIO != 0) set_prio_from_left<PRIO>(nrows - j, nrows);
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) issue(j + q + DEPTH - ILP + i, buf[(q + DEPTH - ILP + i) % DEPTH]);
      const std::uint32_t jq = j + q;
      if (jq >= nrows) break;
      if (jq + ILP <= nrows) {
        std::uint32_t v[ILP];
        if constexpr (SPLIT) {
          // two independent 32-byte chains per row: p = Shift_32(crc_0(dw 0..7)) ^ crc_0(dw 8..15)
          Reg pa[ILP], pb[ILP];
#pragma unroll
          for (int i = 0; i < ILP; ++i) pa[i] = pb[i] = Reg{0, 0};
#pragma unroll
          for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
              slice4(lds, pa[i], buf[q + i][t].x, kc);
              slice4(lds, pb[i], buf[q + i][t + 2].x, kc);
            }
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
              slice4(lds, pa[i], buf[q + i][t].y, kc);
              slice4(lds, pb[i], buf[q + i][t + 2].y, kc);
            }
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
              slice4(lds, pa[i], buf[q + i][t].z, kc);
              slice4(lds, pb[i], buf[q + i][t + 2].z, kc);
            }
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
              slice4(lds, pa[i], buf[q + i][t].w, kc);
              slice4(lds, pb[i], buf[q + i][t + 2].w, kc);
            }
          }
#pragma unroll
          for (int i = 0; i < ILP; ++i)
            v[i] = lane_shift(lds, shift32_bperm(pa[i].value(), s32lo, s32hi) ^ pb[i].value(), kc);
        } else {
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
        }
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
  if constexpr (PROG > 0) stamp(2 + (nrows - 1) / PROG);
}

// Packed kernel with dynamic work distribution inside each workgroup. The batch is cut into chunks
// of C whole blocks (CR = C*R rows, CR >= CROWS and a multiple of DEPTH; C <= 64); workgroup g owns
// a contiguous static range of chunks, and its waves take chunks from that range through one global
// atomic counter per workgroup. The statically partitioned body leaves the slowest waves of a CU
// running long after the median wave has finished (tools/wave_tail.py); here a wave that runs ahead
// takes more chunks.
// Pipeline: DEPTH rows in flight, ILP rows per step, chunk-aligned iterations of DEPTH rows. The id
// of chunk k+1 is requested when chunk k starts and read (v_readfirstlane) after iteration 0 of
// chunk k, whose row loads were issued after the atomic: the wait for those rows already covers
// the atomic's return, so the request never drains the row pipeline. In the last iteration of a
// chunk the issue cursor runs into the next chunk.
template <int DEPTH, int ILP, bool R1, int CROWS>
__device__ __forceinline__ void crc_packed_dyn_body(const XArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  static_assert(CROWS % DEPTH == 0 && CROWS >= 2 * DEPTH && CROWS <= 64, "chunk shape");
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t wpg = blockDim.x >> 6;
  std::uint32_t* ctr = a.wg_ctr + blockIdx.x * kCtrStride;
  if (threadIdx.x == 0) {
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);  // the reset has reached L2 before any wave of this group grabs
  }
  fill_lds(a.tabs, lds);
  const LaneConst kc = lane_const(lane);
  const std::uint32_t hcon = a.tabs->horner[lane & 31u];
  const bool lo_half = lane < 32u;
  const std::uint32_t inj_const =
      lo_half ? 0u
              : static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(a.init_default),
                                                                lane & 31u, 1)) & hcon;
  __syncthreads();

  const std::uint32_t R = R1 ? 1u : a.len / kRow;
  std::uint32_t C = R1 ? static_cast<std::uint32_t>(CROWS) : (CROWS + R - 1) / R;
  if (!R1)
    while ((C * R) % DEPTH) ++C;
  const std::uint32_t NIT = C * R / DEPTH;            // iterations per chunk (>= 2)
  const std::uint32_t NC = (a.nblocks + C - 1) / C;   // chunks in the batch; only the last is partial
  const std::uint32_t c0 = static_cast<std::uint32_t>(blockIdx.x * static_cast<std::uint64_t>(NC) / gridDim.x);
  const std::uint32_t ncw =
      static_cast<std::uint32_t>((blockIdx.x + 1) * static_cast<std::uint64_t>(NC) / gridDim.x) - c0;
  if (wid >= ncw) return;
  const std::uint64_t brow = static_cast<std::uint64_t>(R) * kRow;  // bytes per block
  const std::uintptr_t loff = lane * kSeg;

  // The counter address goes through an opaque VGPR zero: with a provably uniform address the
  // compiler's atomic optimizer rewrites the add into a wave-aggregated form that broadcasts the
  // result with v_readfirstlane at once, i.e. a vmcnt(0) drain of the row pipeline at every grab.
  std::uint32_t vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  std::uint32_t* const vctr = ctr + vzero;

  struct Chunk {
    std::uint32_t fb, nb, vrows;  // first block, blocks, rows holding data
    std::uintptr_t base;          // address of its first row
  };
  auto chunk = [&](std::uint32_t q) {
    Chunk c;
    c.fb = (c0 + q) * C;
    c.nb = a.nblocks - c.fb < C ? a.nblocks - c.fb : C;
    c.vrows = c.nb * R;
    c.base = reinterpret_cast<std::uintptr_t>(a.base) + static_cast<std::uint64_t>(c.fb) * brow;
    return c;
  };
  auto load_row = [&](std::uintptr_t rowp, uint4 (&q)[4]) {
    const std::uintptr_t p = rowp + loff;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(p + 16u * i);
  };

  Chunk cur = chunk(wid), nxt = cur;
  bool nvalid = false;
  auto grab = [&]() -> std::uint32_t {  // lane 0: wave-local id of the next chunk, minus wpg
    std::uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(vctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  std::uint32_t nv = grab();
  uint4 buf[DEPTH][4];
#pragma unroll
  for (int s = 0; s < DEPTH - ILP; ++s)
    load_row(cur.base + static_cast<std::uint64_t>(s < cur.vrows ? s : cur.vrows - 1) * kRow, buf[s]);

  // One flat loop over iterations of DEPTH rows (a nested chunk loop makes the compiler's wait
  // counters merge pessimistically at the inner loop head and drain the pipeline).
  std::uint32_t it = 0, B = 0, r = 0, kb = 0, keep = 0;
  for (;;) {
    const std::uint32_t row0 = it * DEPTH;
    const bool last_it = it + 1 == NIT;
    const std::uintptr_t clast = cur.base + static_cast<std::uint64_t>(cur.vrows - 1) * kRow;
#pragma unroll
    for (int q = 0; q < DEPTH; q += ILP) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        const int x = q + DEPTH - ILP + i;  // issue row row0 + x
        std::uintptr_t rp;
        if (x < DEPTH || !last_it) {
          const std::uint32_t ri = row0 + x;
          rp = ri < cur.vrows ? cur.base + static_cast<std::uint64_t>(ri) * kRow : clast;
        } else {
          const std::uint32_t ri = x - DEPTH;  // row of the next chunk
          const std::uint32_t rn = ri < nxt.vrows ? ri : nxt.vrows - 1;
          rp = nvalid ? nxt.base + static_cast<std::uint64_t>(rn) * kRow : clast;
        }
        load_row(rp, buf[x % DEPTH]);
      }
      // Keep the row loads ahead of this step's table work: left alone, the scheduler sinks them
      // below the first lookups (their scalar addresses come late), halving the rows in flight.
      __builtin_amdgcn_sched_barrier(0);
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
      for (int i = 0; i < ILP; ++i) {
        const std::uint32_t v = lane_shift(lds, p[i].value(), kc);
        if (row0 + q + i < cur.vrows) {
          std::uint32_t term;
          if (R1 || r == 0) {
            term = inj_const;
            if (a.init_raw) {
              const std::uint32_t init = sload32(a.init_raw, cur.fb + kb);
              term = lo_half ? 0u
                             : static_cast<std::uint32_t>(__builtin_amdgcn_sbfe(static_cast<std::int32_t>(init),
                                                                                lane & 31u, 1)) & hcon;
            }
          } else {
            term = lo_half ? static_cast<std::uint32_t>(
                                 __builtin_amdgcn_sbfe(static_cast<std::int32_t>(B), lane, 1)) & hcon
                           : 0u;
          }
          const std::uint32_t Bn = __builtin_amdgcn_readlane(wave_xor_to_lane63(v ^ term), 63);
          if (R1 || ++r == R) {
            keep = lane == kb ? (Bn ^ a.out_xor) : keep;
            ++kb;
            r = 0;
            B = 0;
          } else {
            B = Bn;
          }
        }
      }
      if (q == 0 && it == 1) {  // rows just processed were issued after the grab: its id is back
        const std::uint32_t qn = wpg + __builtin_amdgcn_readfirstlane(nv);
        nvalid = qn < ncw;
        if (nvalid) nxt = chunk(qn);
      }
    }
    if (last_it) {
      if (lane < cur.nb) a.out[cur.fb + lane] = keep;
      if (!nvalid) break;
      cur = nxt;
      nvalid = false;
      it = 0;
      kb = 0;
      nv = grab();
    } else {
      ++it;
    }
  }
}

}  // namespace dev
}  // namespace tkv
