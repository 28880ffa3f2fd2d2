// Variant explorer (not product code): the production row-kernel body instantiated with other
// pipeline shapes, a memory-only mode (same loads, XOR instead of CRC) and a plain coalesced
// streaming read, so one process can A/B them on the same buffer (cdna_hip_programming.md §5.4
// rule 24). Built by tools/Makefile into tools/libexplore.so; driven by tools/explore.py.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "explore_device.h"

using namespace tkv;

namespace tkv::dev {
// (explorer only; measured slower than the static packed body)
// Packed kernel with chip-wide dynamic work distribution (per-XCD queues with stealing). Two launches
// of the static body overlapped on two streams run 6 % faster than back to back
// (tools/overlap_probe.py), and per-wave progress stamps (tools/progress_probe.py) show why: a launch
// ends with ~140 us at half rate, while the waves that finished early (p10 at 0.6 of the span) leave
// their CUs idle. Here the batch is split in two regions:
// - static (SF/16 of the blocks; SF = 0: none): wave w owns a contiguous range, as crc_packed_body;
// - pool (the rest), cut into chunks of C whole blocks (C*R rows, >= CROWS, a multiple of DEPTH).
//   Chunk range y of 8 equal ranges is the pool of the workgroups with blockIdx % 8 == y (their
//   round-robin XCD, a label only); a wave whose pool is dry steals from the following pools.
// With SF = 0 a wave's first chunk is static (the pool's i-th chunk for its i-th wave). Chunk ids
// come from the pool's head counter, requested one chunk ahead and read after the first iteration
// of the current chunk (crc_packed_dyn_body), so the request never drains the row pipeline.
// ctr[y * kCtrStride] is pool y's head, ctr[8 * kCtrStride] counts finished waves; the last wave to
// finish zeroes them all for the next launch on this stream (they must be zero before the first).
// PERM != 0 (explorer): the pool's q-th chunk is chunk (q * PERM) mod pool size (sizes powers of 2).
// SD: SF is in 1/SD-ths of the blocks; SP: issue priority (set_prio_from_left<SP>) in the static region.
// LEAN: no exit counter and no blind walk over dry pools. The heads of this launch are a.wg_ctr; the
// host alternates two head sets between launches and passes the other one in a.prog, which
// workgroup 0 zeroes for the next launch. A wave whose pool ran dry reads all eight heads (one sc1
// load per lane 0-7) and grabs from the pool with the most chunks left, until none has any.
template <int DEPTH, int ILP, bool R1, int CROWS, std::uint32_t PERM = 0, int SF = 0, int SD = 16, int SP = 0,
          bool LEAN = false>
__device__ __forceinline__ void crc_packed_xq_body(const XArgs& a, std::uint32_t* lds) {
  static_assert(DEPTH > ILP && DEPTH % ILP == 0, "DEPTH must be a multiple of ILP and exceed it");
  static_assert(CROWS % DEPTH == 0 && CROWS >= 2 * DEPTH && CROWS <= 64, "chunk shape");
  static_assert(SF >= 0 && SF < SD, "static share in 1/SD-ths");
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t wpg = blockDim.x >> 6;
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
  const std::uint32_t G = gridDim.x;
  const std::uint32_t W = G * wpg;
  const std::uint32_t wave = blockIdx.x * wpg + wid;
  // static region [0, S): wave w owns [w*S/W, (w+1)*S/W); pool region [S, nblocks)
  const std::uint32_t S = SF ? static_cast<std::uint32_t>(static_cast<std::uint64_t>(a.nblocks) * SF / SD) : 0u;
  const std::uint32_t NC = (a.nblocks - S + C - 1) / C;  // pool chunks; only the last is partial
  const std::uint64_t brow = static_cast<std::uint64_t>(R) * kRow;  // bytes per block
  const std::uintptr_t loff = lane * kSeg;

  std::uint32_t vzero;  // opaque zero: keeps the atomic optimizer from draining (crc_packed_dyn_body)
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  std::uint32_t* const vctr = a.wg_ctr + vzero;
  auto plo = [&](std::uint32_t y) { return static_cast<std::uint32_t>(static_cast<std::uint64_t>(y) * NC / 8u); };
  auto psize = [&](std::uint32_t y) { return plo(y + 1) - plo(y); };
  // pool chunks handed out statically (SF = 0 only): one per wave of the pool's workgroups
  auto pstat = [&](std::uint32_t y) { return (SF == 0 && y < G) ? ((G - 1u - y) / 8u + 1u) * wpg : 0u; };
  const std::uint32_t xp = blockIdx.x & 7u;
  const std::uint32_t xi = (blockIdx.x >> 3) * wpg + wid;  // wave index inside its pool

  struct Chunk {
    std::uint32_t fb, nb, vrows, nit;  // first block, blocks, rows holding data, iterations
    std::uintptr_t base;               // address of its first row
  };
  auto span = [&](std::uint32_t fb, std::uint32_t nb) {
    Chunk c;
    c.fb = fb;
    c.nb = nb;
    c.vrows = nb * R;
    c.nit = (c.vrows + DEPTH - 1) / DEPTH;
    c.nit = c.nit < 2u ? 2u : c.nit;
    c.base = reinterpret_cast<std::uintptr_t>(a.base) + static_cast<std::uint64_t>(fb) * brow;
    return c;
  };
  auto pchunk = [&](std::uint32_t y, std::uint32_t q) {  // q-th chunk of pool y
    if constexpr (PERM != 0) q = static_cast<std::uint32_t>((static_cast<std::uint64_t>(q) * PERM) % psize(y));
    const std::uint32_t fb = S + (plo(y) + q) * C;
    return span(fb, a.nblocks - fb < C ? a.nblocks - fb : C);
  };
  auto load_row = [&](std::uintptr_t rowp, uint4 (&q)[4]) {
    const std::uintptr_t p = rowp + loff;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = gload16(p + 16u * i);
  };
  std::uint32_t gp = xp;   // pool the pending grab goes to
  std::uint32_t seen = 0;  // pools found exhausted
  auto grab = [&]() -> std::uint32_t {
    std::uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(vctr + gp * kCtrStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  // Blocking search from pool gp on (start, and after a pool runs dry): false once all 8 are dry.
  auto steal = [&](Chunk& out) -> bool {
    if constexpr (LEAN) {
      for (int tries = 0; tries < 64; ++tries) {
        std::int32_t left = -1;
        if (lane < 8u) {
          const std::uint32_t h = __hip_atomic_load(vctr + lane * kCtrStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          left = static_cast<std::int32_t>(psize(lane)) - static_cast<std::int32_t>(h);
        }
        std::int32_t best = 0;
        std::uint32_t by = 0;
#pragma unroll
        for (std::uint32_t y = 0; y < 8u; ++y) {
          const std::int32_t l = __builtin_amdgcn_readlane(left, y);
          if (l > best) {
            best = l;
            by = y;
          }
        }
        if (best <= 0) return false;
        gp = by;
        const std::uint32_t q = __builtin_amdgcn_readfirstlane(grab());
        if (q < psize(gp)) {
          out = pchunk(gp, q);
          return true;
        }
      }
      return false;
    }
    while (seen < 8u) {
      const std::uint32_t q = pstat(gp) + __builtin_amdgcn_readfirstlane(grab());
      if (q < psize(gp)) {
        out = pchunk(gp, q);
        return true;
      }
      ++seen;
      gp = (gp + 1u) & 7u;
    }
    return false;
  };

  Chunk cur{}, nxt{};
  bool live = true;
  if constexpr (LEAN) {
    if (blockIdx.x == 0 && threadIdx.x < 8u)
      __hip_atomic_store(reinterpret_cast<std::uint32_t*>(a.prog) + threadIdx.x * kCtrStride, 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (SF != 0) {  // static region: the packed loop itself (no per-row chunk bookkeeping)
    const std::uint32_t s0 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(wave) * S / W);
    const std::uint32_t s1 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(wave + 1) * S / W);
    if (s1 > s0) dev::x_packed_body<DEPTH, ILP, R1, false, 0, 0, 0, true, 0, SP>(a, lds, s0, s1 - s0);
  }
  if (!SF && xi < psize(xp)) cur = pchunk(xp, xi);
  else live = steal(cur);
  if (live) {
    std::uint32_t nv = grab();
    bool nvalid = false;
    uint4 buf[DEPTH][4];
    auto prologue = [&]() {
#pragma unroll
      for (int s = 0; s < DEPTH - ILP; ++s)
        load_row(cur.base + static_cast<std::uint64_t>(s < static_cast<int>(cur.vrows) ? s : cur.vrows - 1) * kRow,
                 buf[s]);
    };
    prologue();
    std::uint32_t it = 0, B = 0, r = 0, kb = 0, keep = 0;
    for (;;) {
      const std::uint32_t row0 = it * DEPTH;
      const bool last_it = it + 1 == cur.nit;
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
              keep = lane == (kb & 63u) ? (Bn ^ a.out_xor) : keep;
              ++kb;
              if ((kb & 63u) == 0u) a.out[cur.fb + kb - 64u + lane] = keep;  // 64 results at a time
              r = 0;
              B = 0;
            } else {
              B = Bn;
            }
          }
        }
        if (q == 0 && it == 1) {  // rows just processed were issued after the grab: its id is back
          const std::uint32_t qn = pstat(gp) + __builtin_amdgcn_readfirstlane(nv);
          nvalid = qn < psize(gp);
          if (nvalid) nxt = pchunk(gp, qn);
        }
      }
      if (last_it) {
        if (kb & 63u) {
          const std::uint32_t first = kb & ~63u;
          if (lane < (kb & 63u)) a.out[cur.fb + first + lane] = keep;
        }
        it = 0;
        kb = 0;
        if (nvalid) {
          cur = nxt;
          nvalid = false;
          nv = grab();
        } else {  // pool gp ran dry: search the others, then restart the row pipeline
          ++seen;
          if constexpr (!LEAN) gp = (gp + 1u) & 7u;
          if (!steal(cur)) break;
          nv = grab();
          prologue();
        }
      } else {
        ++it;
      }
    }
  }
  // The last wave out zeroes the pool heads and the exit count for the next launch.
  if (!LEAN && lane == 0) {
    std::uint32_t* done = vctr + 8u * kCtrStride;
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == W - 1u) {
#pragma unroll
      for (std::uint32_t y = 0; y < 8u; ++y)
        __hip_atomic_store(vctr + y * kCtrStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace tkv::dev

template <int D, int I, int M>
__global__ __launch_bounds__(kThreads) void k_rows(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::x_rows_body<true, true, D, I, M>(a, lds);
}

// Ideal streaming read: every lane reads consecutive 16-byte words, XOR-reduces, one store per wave.
template <int T = 256>
__global__ __launch_bounds__(T) void k_stream(const uint4* p, std::uint64_t n16, std::uint32_t* out) {
  std::uint32_t x = 0;
  for (std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(T) + threadIdx.x; i < n16;
       i += gridDim.x * static_cast<std::uint64_t>(T)) {
    const uint4 v = p[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;  // keep the loads alive
}


// Memory-pattern probe: uniform aligned batch, each wave owns a contiguous range of 4 KiB rows
// (same partition as crc_rows), DEPTH rows of 4 x 16-byte loads in flight per lane.
// PAT 0: lane l reads bytes [64l, 64l+64) of the row (the production segment layout)
// PAT 1: fully coalesced, load i reads [1024i + 16l, +16)
// PAT 2: lane l reads [2048(i/2) + 32l + 16(i%2), +16) (32-byte lane segments)
// FIN 0: XOR into a register, one store per wave; FIN 1: per-row DPP reduce + lane-0 store per row;
// FIN 2: per-row reduce, results kept in lane (row % 64) and stored 64 at a time (coalesced).
template <int PAT, int DEPTH, int FIN, int MIS = 0, int STR = 0>
__global__ __launch_bounds__(1024) void k_pat(const std::uint8_t* base, std::uint32_t nrows, std::uint32_t W,
                                              std::uint32_t* out) {
  base += MIS;  // byte misalignment of every load (unaligned global_load_dwordx4)
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wave = blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t g0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(nrows) / W);
  const std::uint32_t g1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(nrows) / W);
  auto addr = [&](std::uint32_t g, int i) -> std::uintptr_t {
    const std::uint32_t gl = g < g1 ? g : g0;
    // STR: the wave's j-th row is global row wave + j*W (all waves sweep one moving window)
    const std::uint64_t phys = STR ? static_cast<std::uint64_t>(gl - g0) * W + wave : gl;
    const std::uintptr_t rb = reinterpret_cast<std::uintptr_t>(base) + phys * 4096u;
    if constexpr (PAT >= 128) {
      // lane-contiguous segments of PAT bytes: a tile of 64*PAT bytes is PAT/64 rows; its j-th row
      // reads bytes [64j, 64j+64) of every lane's segment
      constexpr std::uint32_t J = PAT / 64;
      const std::uint64_t t = phys / J, j = phys % J;
      return reinterpret_cast<std::uintptr_t>(base) + t * 64u * PAT + lane * PAT + 64u * j + 16u * i;
    } else if constexpr (PAT == 0) return rb + 64u * lane + 16u * i;
    else if constexpr (PAT == 1) return rb + 1024u * i + 16u * lane;
    else return rb + 2048u * (i / 2) + 32u * lane + 16u * (i % 2);
  };
  uint4 buf[DEPTH][4];
  std::uint32_t acc = 0, keep = 0;
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g0 + s, i));
  for (std::uint32_t g = g0; g < g1; g += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int s = (k + DEPTH - 1) % DEPTH;
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g + k + DEPTH - 1, i));
      if (g + k >= g1) break;
      std::uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) x ^= buf[k][i].x ^ buf[k][i].y ^ buf[k][i].z ^ buf[k][i].w;
      if constexpr (FIN == 0) {
        acc ^= x;
      } else {
        const std::uint32_t r = __builtin_amdgcn_readlane(dev::wave_xor_to_lane63(x), 63);
        if constexpr (FIN == 1) {
          if (lane == 0) out[g + k] = r;
        } else {
          const std::uint32_t gi = g + k;
          if (lane == (gi & 63u)) keep = r;
          if ((gi & 63u) == 63u || gi + 1 == g1) {
            const std::uint32_t first = gi & ~63u;
            if (first + lane >= g0 && first + lane <= gi) out[first + lane] = keep;
          }
        }
      }
    }
  }
  if constexpr (FIN == 0) {
    if (acc == 0x9E3779B9u) out[0] = acc;
  }
}


// Block-per-lane probe (memory only): lane l of a wave walks 4 KiB block (64 t + l) of its tile t
// in steps of QB bytes (QB/16 loads of 16 bytes), DEPTH steps in flight; waves own contiguous tile
// ranges. A CRC kernel on this layout needs no lane shift and no wave reduction (each lane's chain
// is its block's CRC); the question is whether loads that touch 64 lines each keep the stream rate.
template <int QB, int DEPTH>
__global__ __launch_bounds__(1024) void k_blk(const std::uint8_t* base, std::uint32_t nrows, std::uint32_t W,
                                              std::uint32_t* out) {
  constexpr int NL = QB / 16;
  constexpr std::uint32_t SPT = 4096u / QB;  // steps per tile
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wave = blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t ntiles = (nrows + 1) / 64u;
  const std::uint32_t t0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(ntiles) / W);
  const std::uint32_t t1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(ntiles) / W);
  const std::uint32_t S = (t1 - t0) * SPT;
  if (S == 0) return;
  auto addr = [&](std::uint32_t s, int i) -> std::uintptr_t {
    const std::uint32_t sc = s < S ? s : S - 1;
    const std::uint64_t blk = static_cast<std::uint64_t>(t0 + sc / SPT) * 64u + lane;
    return reinterpret_cast<std::uintptr_t>(base) + blk * 4096u + (sc % SPT) * QB + 16u * i;
  };
  uint4 buf[DEPTH][NL];
  std::uint32_t acc = 0;
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
    for (int i = 0; i < NL; ++i) buf[s][i] = dev::gload16(addr(s, i));
  for (std::uint32_t g = 0; g < S; g += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int sl = (k + DEPTH - 1) % DEPTH;
#pragma unroll
      for (int i = 0; i < NL; ++i) buf[sl][i] = dev::gload16(addr(g + k + DEPTH - 1, i));
      if (g + k >= S) break;
#pragma unroll
      for (int i = 0; i < NL; ++i) acc ^= buf[k][i].x ^ buf[k][i].y ^ buf[k][i].z ^ buf[k][i].w;
    }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// Interference probe: the packed kernel's loads and pipeline (D4, seg64, batched stores), plus
// per row NLDS conflict-free ds_read_b32 in 4-wide dependent steps and/or NVALU dependent VALU
// ops, to see which pipe's activity slows the memory stream.
template <int NLDS, int NVALU>
__global__ __launch_bounds__(1024) void k_interf(const std::uint8_t* base, std::uint32_t nrows, std::uint32_t W,
                                                 std::uint32_t* out) {
  __shared__ std::uint32_t lds[kLdsWords];
  for (std::uint32_t i = threadIdx.x; i < kLdsWords; i += 1024) lds[i] = i * 2654435761u;
  __syncthreads();
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wave = blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t g0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(nrows) / W);
  const std::uint32_t g1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(nrows) / W);
  constexpr int DEPTH = 4;
  auto addr = [&](std::uint32_t g, int i) -> std::uintptr_t {
    return reinterpret_cast<std::uintptr_t>(base) + static_cast<std::uint64_t>(g < g1 ? g : g0) * 4096u +
           64u * lane + 16u * i;
  };
  uint4 buf[DEPTH][4];
  std::uint32_t keep = 0;
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g0 + s, i));
  for (std::uint32_t g = g0; g < g1; g += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int s = (k + DEPTH - 1) % DEPTH;
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g + k + DEPTH - 1, i));
      if (g + k >= g1) break;
      std::uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) x ^= buf[k][i].x ^ buf[k][i].y ^ buf[k][i].z ^ buf[k][i].w;
      std::uint32_t y = x;
#pragma unroll
      for (int j = 0; j < NLDS / 4; ++j) {
        const std::uint32_t a0 = ((y & 0xFFu) << 8) | (lane & 31u) << 2;
        y = dev::xor3(dev::lds_at(lds, a0), dev::lds_at(lds, a0 + 0x10000u), dev::lds_at(lds, a0 + 0x10080u)) ^
            dev::lds_at(lds, a0 + 128u);
      }
#pragma unroll
      for (int j = 0; j < NVALU / 2; ++j) y = __builtin_amdgcn_perm(y, y * 3u + j, 0x0C020500u) ^ x;
      const std::uint32_t r = __builtin_amdgcn_readlane(dev::wave_xor_to_lane63(y), 63);
      const std::uint32_t gi = g + k;
      if (lane == (gi & 63u)) keep = r;
      if ((gi & 63u) == 63u || gi + 1 == g1) {
        const std::uint32_t first = gi & ~63u;
        if (first + lane >= g0 && first + lane <= gi) out[first + lane] = keep;
      }
    }
  }
}



// Interference probe 2: NL lookups per row split over CH independent dependent chains, each lookup
// a conflict-free ds_read of WB bytes per lane (4 = ds_read_b32, 8 = ds_read_b64), same loads and
// pipeline as k_interf. Separates LDS bytes, LDS instruction count and chain latency.
template <int NL, int WB, int CH>
__global__ __launch_bounds__(1024) void k_interf2(const std::uint8_t* base, std::uint32_t nrows, std::uint32_t W,
                                                  std::uint32_t* out) {
  __shared__ std::uint32_t lds[kLdsWords];
  for (std::uint32_t i = threadIdx.x; i < kLdsWords; i += 1024) lds[i] = i * 2654435761u;
  __syncthreads();
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wave = blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t g0 = static_cast<std::uint32_t>(wave * static_cast<std::uint64_t>(nrows) / W);
  const std::uint32_t g1 = static_cast<std::uint32_t>((wave + 1) * static_cast<std::uint64_t>(nrows) / W);
  constexpr int DEPTH = 4;
  auto addr = [&](std::uint32_t g, int i) -> std::uintptr_t {
    return reinterpret_cast<std::uintptr_t>(base) + static_cast<std::uint64_t>(g < g1 ? g : g0) * 4096u +
           64u * lane + 16u * i;
  };
  uint4 buf[DEPTH][4];
  std::uint32_t keep = 0;
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g0 + s, i));
  for (std::uint32_t g = g0; g < g1; g += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int s = (k + DEPTH - 1) % DEPTH;
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[s][i] = dev::gload16(addr(g + k + DEPTH - 1, i));
      if (g + k >= g1) break;
      std::uint32_t y[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) y[c] = buf[k][c & 3].x ^ buf[k][(c + 1) & 3].w ^ c;
#pragma unroll
      for (int j = 0; j < NL / CH; ++j)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          // conflict-free: b32 lane c of each half reads bank c; b64 lane l reads banks 2l, 2l+1 (mod 64)
          const std::uint32_t a = WB == 4 ? (((y[c] & 0xFFu) << 8) | (lane & 31u) << 2)
                                          : (((y[c] & 0x7Fu) << 9) | (lane << 3));
          if constexpr (WB == 4) {
            y[c] = dev::lds_at(lds, a) ^ (y[c] >> 8);
          } else {
            const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(lds) + a);
            y[c] = v.x ^ v.y ^ (y[c] >> 8);
          }
        }
      std::uint32_t yy = 0;
#pragma unroll
      for (int c = 0; c < CH; ++c) yy ^= y[c];
      const std::uint32_t r = __builtin_amdgcn_readlane(dev::wave_xor_to_lane63(yy), 63);
      const std::uint32_t gi = g + k;
      if (lane == (gi & 63u)) keep = r;
      if ((gi & 63u) == 63u || gi + 1 == g1) {
        const std::uint32_t first = gi & ~63u;
        if (first + lane >= g0 && first + lane <= gi) out[first + lane] = keep;
      }
    }
  }
}

// Diagnostic: per-wave start/end s_memrealtime (100 MHz) of the production packed body.
__global__ __launch_bounds__(1024) void k_packed_stamped(XArgs a, unsigned long long* stamps) {
  __shared__ std::uint32_t lds[kLdsWords];
  const std::uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  dev::x_packed_body<4, 2, true>(a, lds);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    stamps[2 * wave] = t0;
    stamps[2 * wave + 1] = t1;
  }
}

template <int SK, int PR = 0>
__global__ __launch_bounds__(1024) void k_skew_stamped(XArgs a, unsigned long long* stamps) {
  __shared__ std::uint32_t lds[kLdsWords];
  const std::uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  dev::x_packed_body<4, 2, true, false, 0, 0, 0, false, SK, PR>(a, lds);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    stamps[2 * wave] = t0;
    stamps[2 * wave + 1] = t1;
  }
}

__global__ __launch_bounds__(1024) void k_dyn_stamped(XArgs a, unsigned long long* stamps) {
  __shared__ std::uint32_t lds[kLdsWords];
  const std::uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  dev::crc_packed_dyn_body<4, 2, true, 16>(a, lds);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    stamps[2 * wave] = t0;
    stamps[2 * wave + 1] = t1;
  }
}

namespace {
DeviceTables* g_tabs = nullptr;
std::uint8_t* g_dummy = nullptr;
Seam* g_seams = nullptr;
int g_ncu = 0;

struct V {
  const char* name;
  void (*launch)(XArgs, hipStream_t);
};

template <int D, int I, int M>
void L(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_rows<D, I, M>), dim3(g_ncu), dim3(kThreads), 0, s, a);
}

template <int PAT, int D, int F, int MIS = 0, int STR = 0>
void P(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_pat<PAT, D, F, MIS, STR>), dim3(g_ncu), dim3(1024), 0, s, a.base, a.total_rows - 1, a.nwaves,
                     a.out);
}

template <int QB, int D>
void BL(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_blk<QB, D>), dim3(g_ncu), dim3(1024), 0, s, a.base, a.total_rows - 1, a.nwaves, a.out);
}

template <int D, int I, bool R1, int T, bool SP, std::uint32_t ROT = 0, int CHK = 0>
__global__ __launch_bounds__(T) void k_packed(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::x_packed_body<D, I, R1, SP, ROT, CHK>(a, lds);
}

// chunk-strided block map (4 KiB blocks only; other lengths fall back to the product map)
template <int CHK>
void PC(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * 16;
  if (a.len == kRow && a.nblocks % (a.nwaves * 64u) == 0)
    hipLaunchKernelGGL((k_packed<4, 2, true, 1024, false, 0, CHK>), dim3(g_ncu), dim3(1024), 0, s, a);
  else hipLaunchKernelGGL((k_packed<4, 2, false, 1024, false>), dim3(g_ncu), dim3(1024), 0, s, a);
}

template <std::uint32_t ROT>
void PR(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * 16;
  if (a.len == kRow) hipLaunchKernelGGL((k_packed<4, 2, true, 1024, false, ROT>), dim3(g_ncu), dim3(1024), 0, s, a);
  else hipLaunchKernelGGL((k_packed<4, 2, false, 1024, false, ROT>), dim3(g_ncu), dim3(1024), 0, s, a);
}

template <int D, int I, bool R1, int T, int CR>
__global__ __launch_bounds__(T) void k_packed_dyn(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_packed_dyn_body<D, I, R1, CR>(a, lds);
}

std::uint32_t* g_ctr = nullptr;
std::uint32_t* g_shift32 = nullptr;  // explorer SPLIT variants

template <int D, int I, int CR, int T = 1024>
void PD(XArgs a, hipStream_t s) {
  a.wg_ctr = g_ctr;
  if (a.len == kRow) hipLaunchKernelGGL((k_packed_dyn<D, I, true, T, CR>), dim3(g_ncu), dim3(T), 0, s, a);
  else hipLaunchKernelGGL((k_packed_dyn<D, I, false, T, CR>), dim3(g_ncu), dim3(T), 0, s, a);
}

template <int D, int I, bool R1, int T, int CR, std::uint32_t PM, int SF, int SD, int SP, bool LN = false>
__global__ __launch_bounds__(T) void k_packed_xq(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_packed_xq_body<D, I, R1, CR, PM, SF, SD, SP, LN>(a, lds);
}

std::uint32_t* g_xq = nullptr;  // pool heads + exit count of the xq variants (zeroed once)
std::uint32_t* g_lean = nullptr;  // two head sets of the LEAN variants (zeroed once, then by the kernels)

// Static share SF/SD of the blocks as the product (priority 3, skew for multi-row blocks), then the
// rest in chunks of C blocks taken from eight heads (alternating head sets as PL), each chunk run by
// the product loop itself (crc_packed_body on the chunk's block range: a full pipeline per chunk, no
// per-row bookkeeping). A wave whose head is dry grabs from the fullest head.
template <int C, int SF, int SD, bool R1>
__global__ __launch_bounds__(1024) void k_packed_chunks(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::fill_lds(a.tabs, lds);
  __syncthreads();
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wpg = blockDim.x >> 6;
  const std::uint32_t wave = blockIdx.x * wpg + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t W = gridDim.x * wpg;
  if (blockIdx.x == 0 && threadIdx.x < 8u)
    __hip_atomic_store(reinterpret_cast<std::uint32_t*>(a.prog) + threadIdx.x * kCtrStride, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  const std::uint32_t S = static_cast<std::uint32_t>(static_cast<std::uint64_t>(a.nblocks) * SF / SD);
  const std::uint32_t s0 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(wave) * S / W);
  const std::uint32_t s1 = static_cast<std::uint32_t>(static_cast<std::uint64_t>(wave + 1) * S / W);
  if (s1 > s0) dev::x_packed_body<4, 2, R1, false, 0, 0, 0, true, 0, 3>(a, lds, s0, s1 - s0);
  const std::uint32_t NC = (a.nblocks - S + C - 1) / C;
  auto plo = [&](std::uint32_t y) { return static_cast<std::uint32_t>(static_cast<std::uint64_t>(y) * NC / 8u); };
  auto psize = [&](std::uint32_t y) { return plo(y + 1) - plo(y); };
  std::uint32_t vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  std::uint32_t* const vctr = a.wg_ctr + vzero;
  std::uint32_t gp = blockIdx.x & 7u;
  for (int tries = 0; tries < 1 << 20; ++tries) {
    std::uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(vctr + gp * kCtrStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const std::uint32_t q = __builtin_amdgcn_readfirstlane(v);
    if (q < psize(gp)) {
      const std::uint32_t fb = S + (plo(gp) + q) * C;
      dev::x_packed_body<4, 2, R1, false, 0, 0, 0, true, 0, 0>(a, lds, fb, a.nblocks - fb < C ? a.nblocks - fb : C);
      continue;
    }
    std::int32_t left = -1;
    if (lane < 8u) {
      const std::uint32_t h = __hip_atomic_load(vctr + lane * kCtrStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      left = static_cast<std::int32_t>(psize(lane)) - static_cast<std::int32_t>(h);
    }
    std::int32_t best = 0;
    std::uint32_t by = 0;
#pragma unroll
    for (std::uint32_t y = 0; y < 8u; ++y) {
      const std::int32_t l = __builtin_amdgcn_readlane(left, y);
      if (l > best) {
        best = l;
        by = y;
      }
    }
    if (best <= 0) break;
    gp = by;
  }
}

template <int C, int SF, int SD>
void PC2(XArgs a, hipStream_t s) {
  static int par = 0;
  par ^= 1;
  a.nwaves = g_ncu * 16;
  a.wg_ctr = g_lean + par * 8 * kCtrStride;
  a.prog = reinterpret_cast<unsigned long long*>(g_lean + (par ^ 1) * 8 * kCtrStride);
  if (a.len == kRow) hipLaunchKernelGGL((k_packed_chunks<C, SF, SD, true>), dim3(g_ncu), dim3(1024), 0, s, a);
  else hipLaunchKernelGGL((k_packed_chunks<C, SF, SD, false>), dim3(g_ncu), dim3(1024), 0, s, a);
}

template <int D, int I, int CR, int SF, int SD>
void PL(XArgs a, hipStream_t s) {
  static int par = 0;
  par ^= 1;
  a.wg_ctr = g_lean + par * 8 * kCtrStride;
  a.prog = reinterpret_cast<unsigned long long*>(g_lean + (par ^ 1) * 8 * kCtrStride);
  if (a.len == kRow)
    hipLaunchKernelGGL((k_packed_xq<D, I, true, 1024, CR, 0, SF, SD, 3, true>), dim3(g_ncu), dim3(1024), 0, s, a);
  else
    hipLaunchKernelGGL((k_packed_xq<D, I, false, 1024, CR, 0, SF, SD, 3, true>), dim3(g_ncu), dim3(1024), 0, s, a);
}

template <int D, int I, int CR, std::uint32_t PM = 0, int SF = 0, int T = 1024, int SD = 16, int SP = 0>
void PX(XArgs a, hipStream_t s) {
  a.wg_ctr = g_xq;
  if (a.len == kRow) hipLaunchKernelGGL((k_packed_xq<D, I, true, T, CR, PM, SF, SD, SP>), dim3(g_ncu), dim3(T), 0, s, a);
  else hipLaunchKernelGGL((k_packed_xq<D, I, false, T, CR, PM, SF, SD, SP>), dim3(g_ncu), dim3(T), 0, s, a);
}

// Start-stagger probe: before the production packed body, each wave (PERWAVE) or workgroup sleeps
// a pseudo-random 0..K-1 units of s_sleep 127 (~4 us each), so that waves do not all walk their
// ranges in lockstep from the same moment.
template <int K, bool PERWAVE>
__global__ __launch_bounds__(1024) void k_packed_stag(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  const std::uint32_t id = PERWAVE ? blockIdx.x * 16u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : blockIdx.x;
  const std::uint32_t n = ((id * 2654435761u) >> 16) % K;
  for (std::uint32_t i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  if (a.len == kRow) dev::x_packed_body<4, 2, true>(a, lds);
  else dev::x_packed_body<4, 2, false>(a, lds);
}

template <int K, bool PW>
void PS(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * 16;
  hipLaunchKernelGGL((k_packed_stag<K, PW>), dim3(g_ncu), dim3(1024), 0, s, a);
}

template <int SK, int PR, bool EA = false>
__global__ __launch_bounds__(1024) void k_packed_skew(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  if (a.len == kRow) dev::x_packed_body<4, 2, true, false, 0, 0, 0, false, SK, PR, EA>(a, lds);
  else dev::x_packed_body<4, 2, false, false, 0, 0, 0, false, SK, PR, EA>(a, lds);
}

template <int SK, int PR = 0, bool EA = false>
void PW(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * 16;
  hipLaunchKernelGGL((k_packed_skew<SK, PR, EA>), dim3(g_ncu), dim3(1024), 0, s, a);
}

// grid of M workgroups per CU (M rounds): a CU whose workgroup finishes early takes the next one
template <int M>
void PG(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * M * 16;
  if (a.len == kRow && a.nblocks >= a.nwaves)
    hipLaunchKernelGGL((k_packed<4, 2, true, 1024, false>), dim3(g_ncu * M), dim3(1024), 0, s, a);
  else hipLaunchKernelGGL((k_packed<4, 2, false, 1024, false>), dim3(g_ncu * M), dim3(1024), 0, s, a);
}

// Packed shapes with the product's work-left priority (no skew: it assumes 1024 threads).
template <int D, int I, bool R1, int T>
__global__ __launch_bounds__(T) void k_packed_pr(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::x_packed_body<D, I, R1, false, 0, 0, 0, false, 0, 3>(a, lds);
}

template <int D, int I, int T>
void PP(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * (T / 64);
  if (a.len == kRow) hipLaunchKernelGGL((k_packed_pr<D, I, true, T>), dim3(g_ncu), dim3(T), 0, s, a);
  else hipLaunchKernelGGL((k_packed_pr<D, I, false, T>), dim3(g_ncu), dim3(T), 0, s, a);
}

template <int D, int I, int T = 1024, bool SP = false>
void PK(XArgs a, hipStream_t s) {
  a.nwaves = g_ncu * (T / 64);
  if (a.len == kRow) hipLaunchKernelGGL((k_packed<D, I, true, T, SP>), dim3(g_ncu), dim3(T), 0, s, a);
  else hipLaunchKernelGGL((k_packed<D, I, false, T, SP>), dim3(g_ncu), dim3(T), 0, s, a);
}

template <int NL, int NV>
void IF(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_interf<NL, NV>), dim3(g_ncu), dim3(1024), 0, s, a.base, a.total_rows, a.nwaves, a.out);
}

template <int NL, int WB, int CH>
void IF2(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_interf2<NL, WB, CH>), dim3(g_ncu), dim3(1024), 0, s, a.base, a.total_rows, a.nwaves, a.out);
}

const V kVariants[] = {
    {"i2 L0", IF2<0, 4, 1>}, {"i2 L72 b32 ch1", IF2<72, 4, 1>}, {"i2 L72 b32 ch2", IF2<72, 4, 2>},
    {"i2 L72 b32 ch4", IF2<72, 4, 4>}, {"i2 L72 b32 ch8", IF2<72, 4, 8>}, {"i2 L36 b64 ch2", IF2<36, 8, 2>},
    {"i2 L72 b64 ch2", IF2<72, 8, 2>}, {"i2 L36 b32 ch2", IF2<36, 4, 2>}, {"i2 L144 b32 ch4", IF2<144, 4, 4>},
    {"i2 L144 b32 ch8", IF2<144, 4, 8>},
    {"interf L0 V0", IF<0, 0>}, {"interf L72 V0", IF<72, 0>}, {"interf L0 V128", IF<0, 128>},
    {"interf L72 V128", IF<72, 128>}, {"interf L36 V0", IF<36, 0>}, {"interf L144 V0", IF<144, 0>},
    {"interf L0 V256", IF<0, 256>},
    {"packed chunk64", PC<6>}, {"packed chunk16", PC<4>}, {"packed chunk4", PC<2>},
    {"packed rot1", PR<1>}, {"packed rot61", PR<61>}, {"packed rot16", PR<16>},
    {"dyn D4 I2 C8", PD<4, 2, 8>}, {"dyn D4 I2 C16", PD<4, 2, 16>}, {"dyn D4 I2 C32", PD<4, 2, 32>},
    {"dyn D4 I2 C64", PD<4, 2, 64>}, {"dyn T768 D4 I2 C16", PD<4, 2, 16, 768>},
    {"xq D4 I2 C16", PX<4, 2, 16>},
    {"hy S14 C8", PX<4, 2, 8, 0, 14>}, {"hy S12 C8", PX<4, 2, 8, 0, 12>}, {"hy S10 C8", PX<4, 2, 8, 0, 10>},
    {"hy S12 C16", PX<4, 2, 16, 0, 12>},
    {"tail S60/64 C8 p3", PX<4, 2, 8, 0, 60, 1024, 64, 3>}, {"tail S62/64 C8 p3", PX<4, 2, 8, 0, 62, 1024, 64, 3>},
    {"tail S63/64 C8 p3", PX<4, 2, 8, 0, 63, 1024, 64, 3>}, {"tail S60/64 C16 p3", PX<4, 2, 16, 0, 60, 1024, 64, 3>},
    {"tail S56/64 C8 p3", PX<4, 2, 8, 0, 56, 1024, 64, 3>},
    {"lean S56/64 C8", PL<4, 2, 8, 56, 64>}, {"lean S60/64 C8", PL<4, 2, 8, 60, 64>},
    {"lean S62/64 C8", PL<4, 2, 8, 62, 64>}, {"lean S60/64 C16", PL<4, 2, 16, 60, 64>},
    {"lean S48/64 C8", PL<4, 2, 8, 48, 64>}, {"lean S32/64 C16", PL<4, 2, 16, 32, 64>},
    {"chunks S60/64 C32", PC2<32, 60, 64>}, {"chunks S62/64 C32", PC2<32, 62, 64>},
    {"chunks S60/64 C64", PC2<64, 60, 64>}, {"chunks S56/64 C64", PC2<64, 56, 64>},
    {"chunks S62/64 C16", PC2<16, 62, 64>},
    {"chunks S60/64 C2", PC2<2, 60, 64>}, {"chunks S62/64 C2", PC2<2, 62, 64>}, {"chunks S60/64 C4", PC2<4, 60, 64>}, {"hy S12 C32", PX<4, 2, 32, 0, 12>}, {"hy S8 C16", PX<4, 2, 16, 0, 8>},
    {"pp T1024 D4 I2", PP<4, 2, 1024>}, {"pp T1024 D4 I1", PP<4, 1, 1024>}, {"pp T1024 D3 I1", PP<3, 1, 1024>},
    {"pp T768 D4 I2", PP<4, 2, 768>}, {"pp T768 D6 I2", PP<6, 2, 768>}, {"pp T768 D6 I3", PP<6, 3, 768>},
    {"pp T512 D8 I4", PP<8, 4, 512>}, {"pp T512 D6 I2", PP<6, 2, 512>}, {"pp T512 D8 I2", PP<8, 2, 512>},
    {"skew 0.8", PW<205>}, {"skew 0.6", PW<154>}, {"prio", PW<0, 1>}, {"prio skew 0.8", PW<205, 1>},
    {"prio skew 0.6", PW<154, 1>}, {"pri2", PW<0, 2>}, {"pri3", PW<0, 3>}, {"pri2 skew 0.6", PW<154, 2>},
    {"pri3 skew 0.6", PW<154, 3>}, {"pri4", PW<0, 4>}, {"pri5", PW<0, 5>}, {"pri4 skew 0.6", PW<154, 4>},
    {"pri5 skew 0.6", PW<154, 5>}, {"pri3 skew 0.5", PW<128, 3>}, {"pri3 skew 0.7", PW<179, 3>}, {"pri3 early", PW<0, 3, true>}, {"pri3 skew 0.6 early", PW<154, 3, true>},    {"stag wave 4", PS<4, true>}, {"stag wave 16", PS<16, true>}, {"stag wg 4", PS<4, false>},
    {"stag wg 16", PS<16, false>}, {"stag wave 1", PS<1, true>},
    {"grid x2", PG<2>}, {"grid x3", PG<3>}, {"grid x4", PG<4>}, {"grid x8", PG<8>}, {"grid x16", PG<16>},
    {"packed D4 I2", PK<4, 2>}, {"packed D4 I1", PK<4, 1>}, {"packed D3 I1", PK<3, 1>},
    {"packed T512 D8 I4", PK<8, 4, 512>}, {"packed T512 D6 I3", PK<6, 3, 512>},
    {"packed T768 D6 I2", PK<6, 2, 768>}, {"packed T768 D6 I3", PK<6, 3, 768>},
    {"packed T512 D6 I2", PK<6, 2, 512>}, {"packed D4 I2 split", PK<4, 2, 1024, true>},
    {"packed D4 I1 split", PK<4, 1, 1024, true>}, {"packed D3 I1 split", PK<3, 1, 1024, true>},
    {"packed T512 D8 I4 split", PK<8, 4, 512, true>}, {"packed T768 D6 I2 split", PK<6, 2, 768, true>},
    {"crc D2 I1", L<2, 1, 0>}, {"crc D3 I1", L<3, 1, 0>}, {"crc D4 I1", L<4, 1, 0>},
    {"crc D4 I2", L<4, 2, 0>}, {"crc D6 I2", L<6, 2, 0>},
    {"mem D2 I1", L<2, 1, 1>}, {"mem D4 I1", L<4, 1, 1>}, {"mem D4 I2", L<4, 2, 1>},
    {"mem D8 I1", L<8, 1, 1>},
    {"blk q64 D4", BL<64, 4>}, {"blk q128 D2", BL<128, 2>}, {"blk q128 D3", BL<128, 3>},
    {"blk q128 D4", BL<128, 4>}, {"blk q256 D2", BL<256, 2>},
    {"pat seg64 D4 fin0 strided", P<0, 4, 0, 0, 1>}, {"pat coal D4 fin0 strided", P<1, 4, 0, 0, 1>},
    {"pat seg64 D4 fin2 strided", P<0, 4, 2, 0, 1>}, {"stream T1024 ncu", nullptr},
    {"pat seg64 D4 fin2 mis0", P<0, 4, 2, 0>}, {"pat seg64 D4 fin2 mis4", P<0, 4, 2, 4>},
    {"pat seg64 D4 fin2 mis5", P<0, 4, 2, 5>}, {"pat seg64 D4 fin2 mis8", P<0, 4, 2, 8>},
    {"pat seg64 D2 fin0", P<0, 2, 0>}, {"pat seg64 D4 fin0", P<0, 4, 0>}, {"pat seg64 D4 fin1", P<0, 4, 1>},
    {"pat seg64 D4 fin2", P<0, 4, 2>}, {"pat coal D2 fin0", P<1, 2, 0>}, {"pat coal D4 fin0", P<1, 4, 0>},
    {"pat coal D4 fin1", P<1, 4, 1>}, {"pat coal D4 fin2", P<1, 4, 2>}, {"pat seg32 D4 fin0", P<2, 4, 0>},
    {"pat seg32 D4 fin2", P<2, 4, 2>}, {"pat coal D6 fin0", P<1, 6, 0>}, {"pat seg64 D6 fin0", P<0, 6, 0>},
    {"pat seg128 D4 fin0", P<128, 4, 0>}, {"pat seg256 D4 fin0", P<256, 4, 0>},
    {"pat seg1024 D4 fin0", P<1024, 4, 0>},
};
constexpr int kNV = sizeof(kVariants) / sizeof(kVariants[0]);

template <int D, int I, int T, int SM = 0, int PR = 0>
__global__ __launch_bounds__(T) void k_irr(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::x_rows_body<false, false, D, I, 0, SM, PR>(a, lds);
}

struct IV {
  const char* name;
  int threads;
  void (*launch)(XArgs, hipStream_t);
};

template <int D, int I, int T, int SM = 0, int PR = 0>
void LI(XArgs a, hipStream_t s) {
  hipLaunchKernelGGL((k_irr<D, I, T, SM, PR>), dim3(g_ncu), dim3(T), 0, s, a);
}

const IV kIrr[] = {
    {"irr T1024 D3 I1", 1024, LI<3, 1, 1024>}, {"irr T1024 D2 I1", 1024, LI<2, 1, 1024>},
    {"irr T1024 D4 I2", 1024, LI<4, 2, 1024>}, {"irr T512 D4 I2", 512, LI<4, 2, 512>},
    {"irr T512 D6 I2", 512, LI<6, 2, 512>}, {"irr T512 D6 I3", 512, LI<6, 3, 512>},
    {"irr T768 D4 I2", 768, LI<4, 2, 768>}, {"irr T512 D8 I4", 512, LI<8, 4, 512>},
    {"irr T768 D4 I2 prio", 768, LI<4, 2, 768, 0, 1>}, {"irr T768 D4 I2 pri3", 768, LI<4, 2, 768, 0, 3>}, {"irr T1024 D4 I2 prio", 1024, LI<4, 2, 1024, 0, 1>},
    {"irr T768 D4 I2 small-alt", 768, LI<4, 2, 768, 1>}, {"irr T768 D4 I2 small-last", 768, LI<4, 2, 768, 2>},
};
constexpr int kNIrr = sizeof(kIrr) / sizeof(kIrr[0]);
void* g_blob = nullptr;
std::uint64_t* g_scan64 = nullptr;
std::uint64_t* g_tiles64 = nullptr;
std::uint32_t* g_wstart = nullptr;
std::uint32_t* g_counts = nullptr;
std::uint32_t* g_tile_ok = nullptr;
PrepassOut g_po{};
std::uint64_t g_cap = 0;
}  // namespace

namespace tkv {
hipError_t launch_fixup(const RowsArgs& a, hipStream_t st);
hipError_t launch_prepass(const std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                          std::uint32_t n, std::uint64_t* scan, std::uint64_t* tile_sums, std::uint32_t* tile_ok,
                          std::uint32_t* counts, std::uint64_t* sinfo, std::uint64_t* ends, const PrepassOut& o,
                          std::uint32_t W, std::uint32_t ncu, std::uint32_t* out, std::uint32_t* row0,
                          hipStream_t st);
}  // namespace tkv

extern "C" int explore_count() { return kNV + 1; }
extern "C" const char* explore_name(int v) { return v < kNV ? kVariants[v].name : "stream read (ideal)"; }

extern "C" int explore_run(int v, const std::uint8_t* base, std::uint64_t n, std::uint32_t len, std::uint32_t* out,
                           void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!g_tabs) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    g_ncu = prop.multiProcessorCount;
    auto* h = new DeviceTables;
    build_tables(h);
    if (hipMalloc(&g_tabs, sizeof(DeviceTables)) != hipSuccess) return 1;
    hipMemcpy(g_tabs, h, sizeof(DeviceTables), hipMemcpyHostToDevice);
    delete h;
    hipMalloc(&g_dummy, 256);
    hipMemset(g_dummy, 0, 256);
    hipMalloc(&g_seams, sizeof(Seam) * 2 * g_ncu * kWavesPerWG);
    hipMalloc(&g_ctr, 4 * kCtrStride * g_ncu);
    hipMalloc(&g_xq, 4 * kCtrStride * 9);
    hipMemset(g_xq, 0, 4 * kCtrStride * 9);
    hipMalloc(&g_lean, 4 * kCtrStride * 16);
    hipMemset(g_lean, 0, 4 * kCtrStride * 16);
    std::uint32_t s32[128];  // [j][v] = Shift_32(v << 4j)
    for (int j = 0; j < 8; ++j)
      for (std::uint32_t v = 0; v < 16; ++v) s32[16 * j + v] = multmodp(x8nmodp(32), v << (4 * j));
    hipMalloc(&g_shift32, sizeof(s32));
    hipMemcpy(g_shift32, s32, sizeof(s32), hipMemcpyHostToDevice);
  }
  if (v == kNV) {
    hipLaunchKernelGGL(k_stream<256>, dim3(g_ncu * 8), dim3(256), 0, st, reinterpret_cast<const uint4*>(base),
                       n * len / 16, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  if (kVariants[v].launch == nullptr) {  // "stream T1024 ncu": the ideal read at the CRC kernels' shape
    hipLaunchKernelGGL(k_stream<1024>, dim3(g_ncu), dim3(1024), 0, st, reinterpret_cast<const uint4*>(base),
                       n * len / 16, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  XArgs a{};
  a.base = base;
  a.stride = len;
  a.len = len;
  a.head_z = x8nmodp(head_len(len));
  a.init_default = 0xFFFFFFFFu;
  a.out_xor = 0xFFFFFFFFu;
  a.out = out;
  a.seams = g_seams;
  a.tabs = g_tabs;
  a.dummy = g_dummy;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.total_rows = static_cast<std::uint32_t>(n * rows_for_len(len));
  a.nwaves = g_ncu * kWavesPerWG;
  a.snap_blocks = 1;
  a.shift32 = g_shift32;
  kVariants[v].launch(a, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int explore_irr_count() { return kNIrr; }
extern "C" const char* explore_irr_name(int v) { return kIrr[v].name; }

extern "C" int explore_run_irr(int v, const std::uint8_t* base, const std::uint64_t* off, const std::uint32_t* len,
                               std::uint64_t n, std::uint32_t* out, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!g_tabs) {
    std::uint32_t dummy_out;
    (void)dummy_out;
    if (explore_run(kNV, base, 0, 16, out, stream)) return 1;  // one-time init of tables etc.
  }
  if (n > g_cap) {
    hipFree(g_blob);
    const std::uint64_t nt = n / 4096 + 2;
    hipMalloc(&g_blob, 8 * (n + nt + 2 * n) + 4 * (5 * n + 1));
    auto* p8 = static_cast<std::uint64_t*>(g_blob);
    g_scan64 = p8;
    g_tiles64 = p8 + n;
    g_po.s_off = p8 + n + nt;
    g_po.big_off = p8 + 2 * n + nt;
    auto* p4 = reinterpret_cast<std::uint32_t*>(p8 + 3 * n + nt);
    g_po.s_len = p4;
    g_po.s_idx = p4 + n;
    g_po.big_len = p4 + 2 * n;
    g_po.big_idx = p4 + 3 * n;
    g_po.row_scan = p4 + 4 * n;
    if (!g_wstart) hipMalloc(&g_wstart, 4 * g_ncu * 16);
    if (!g_counts) hipMalloc(&g_counts, 64);
    hipFree(g_tile_ok);
    hipMalloc(&g_tile_ok, 4 * nt);
    g_po.wave_start = g_wstart;
    g_cap = n;
  }
  XArgs a{};
  a.base = base;
  a.offsets = g_po.big_off;
  a.lengths = g_po.big_len;
  a.out_idx = g_po.big_idx;
  a.row_scan = g_po.row_scan;
  a.wave_start = g_wstart;
  a.counts = g_counts;
  a.s_off = g_po.s_off;
  a.s_len = g_po.s_len;
  a.s_idx = g_po.s_idx;
  a.init_default = 0xFFFFFFFFu;
  a.out_xor = 0xFFFFFFFFu;
  a.out = out;
  a.seams = g_seams;
  a.tabs = g_tabs;
  a.dummy = g_dummy;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.nwaves = g_ncu * (kIrr[v].threads / 64);
  // The explorer's irregular variants run the general path only: on batches that qualify for stream
  // mode (blocks back to back, each >= 64 B) the prepass builds no small/large lists, so use them on
  // batches with gaps between blocks.
  launch_prepass(base, off, len, a.nblocks, g_scan64, g_tiles64, g_tile_ok, g_counts,
                 reinterpret_cast<std::uint64_t*>(g_counts + 4), g_po.big_off, g_po, a.nwaves, g_ncu, out,
                 reinterpret_cast<std::uint32_t*>(g_seams) + 16 * g_ncu, st);
  kIrr[v].launch(a, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int explore_stamped(const std::uint8_t* base, std::uint64_t n, std::uint32_t* out,
                               unsigned long long* stamps, void* stream, int dyn) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!g_tabs && explore_run(kNV, base, n, 4096, out, stream)) return 1;
  XArgs a{};
  a.base = base;
  a.stride = 4096;
  a.len = 4096;
  a.init_default = 0xFFFFFFFFu;
  a.out_xor = 0xFFFFFFFFu;
  a.out = out;
  a.seams = g_seams;
  a.tabs = g_tabs;
  a.dummy = g_dummy;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.nwaves = g_ncu * 16;
  a.wg_ctr = g_ctr;
  if (dyn == 4) hipLaunchKernelGGL((k_skew_stamped<0, 3>), dim3(g_ncu), dim3(1024), 0, st, a, stamps);
  else if (dyn == 2) hipLaunchKernelGGL(k_skew_stamped<154>, dim3(g_ncu), dim3(1024), 0, st, a, stamps);
  else if (dyn == 3) hipLaunchKernelGGL(k_skew_stamped<205>, dim3(g_ncu), dim3(1024), 0, st, a, stamps);
  else if (dyn) hipLaunchKernelGGL(k_dyn_stamped, dim3(g_ncu), dim3(1024), 0, st, a, stamps);
  else hipLaunchKernelGGL(k_packed_stamped, dim3(g_ncu), dim3(1024), 0, st, a, stamps);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Progress stamps of the production packed body (tools/progress_probe.py).
template <bool R1, int PROG>
__global__ __launch_bounds__(1024) void k_packed_prog(XArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::x_packed_body<4, 2, R1, false, 0, 0, PROG>(a, lds);
}

extern "C" int explore_prog(const std::uint8_t* base, std::uint64_t n, std::uint32_t len, std::uint32_t* out,
                            unsigned long long* stamps, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!g_tabs && explore_run(kNV, base, 0, 16, out, stream)) return 1;
  XArgs a{};
  a.base = base;
  a.stride = len;
  a.len = len;
  a.init_default = 0xFFFFFFFFu;
  a.out_xor = 0xFFFFFFFFu;
  a.out = out;
  a.tabs = g_tabs;
  a.dummy = g_dummy;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.nwaves = g_ncu * 16;
  a.prog = stamps;
  if (len == kRow) hipLaunchKernelGGL((k_packed_prog<true, 16>), dim3(g_ncu), dim3(1024), 0, st, a);
  else hipLaunchKernelGGL((k_packed_prog<false, 64>), dim3(g_ncu), dim3(1024), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
