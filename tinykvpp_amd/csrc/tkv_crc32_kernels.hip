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

#include "tkv_crc32_device.h"

namespace tkv {

namespace {

// Pipeline shape per variant: DEPTH row buffers per wave (DEPTH-ILP rows in flight
// while ILP rows are folded with interleaved chains). The unaligned variants carry a fifth 16-byte
// piece per row, so they keep fewer rows in registers.
// 768-thread workgroups (12 waves/CU, <= 168 VGPRs) with 2 rows folded together and 2 in flight
// measured best on cfg4 (tools/explore.py --irregular, profiles/r1/explore_irregular.txt).
template <bool ALIGNED>
struct Shape {
  static constexpr int kDepth = 4;
  static constexpr int kIlp = 2;
};

// ---- stream mode: every block's CRC from crc_stream's per-end and per-wave registers -----------------
// Run by crc_rows<false, false>, which is launched after crc_stream and has nothing else to do on a
// stream-mode batch: the finish rides on that launch instead of a launch of its own.
// x^(8d) mod P for any byte distance d: one table entry for d <= 4096, one GF(2) multiply more above.
__device__ __forceinline__ std::uint32_t stream_x8n(const DeviceTables* t, std::uint64_t d) {
  const std::uint32_t lo = t->head_shift[d & 4095u][31];
  const std::uint32_t k = static_cast<std::uint32_t>(d >> 12);
  return k == 0u ? lo : dev::shift_rows_tab(t, lo, k);
}

// Block b = [E[b-1], E[b]) of the stream (block 0 starts at the stream start s0; the bytes of row 0
// before it were read as zeros). Let S(e) = crc_0(stream bytes [0, e)), wave w hold rows
// [g0(w), g1(w)) with T_w = s_wtot[w] = crc_0 of those rows alone, and
// L(e) = crc_0(bytes of e's wave up to e) = Shift_(rowend - e)^-1 (Y) ^ Q from the row kernel. Then
// S(e) = Shift_(e - 4096 g0(w))(S(4096 g0(w))) ^ L(e), and S at a wave start is the sum of the earlier
// waves' T_v each shifted to that point, so with e' = E[b-1] in wave w' and e = E[b] in wave w:
//   crc_0(block) = L(e) ^ Shift_len(L(e')) ^ sum_{w' <= v < w} Shift_(e - 4096 g1(v))(T_v)
// (the wave sums before w' cancel). Most blocks lie in one wave and the last sum is empty. For
// block 0, L(s0) = 0 and w' = 0. The register from init is Shift_len(init) ^ crc_0(block).
//
// Lane l of a wave takes block w0 + l - 1 and computes its L(E) and loads E and its wave; lanes 1-63
// then finish their blocks with the predecessor's values pulled from the lane below (ds_bpermute), so
// each L costs one GF(2) multiply per block instead of two, and a block under 4 KiB needs no multiply
// for Shift_len: two multiplies per block in all (there were six, bitwise at 32 steps each). A wave
// advances 63 blocks per step.
__device__ __forceinline__ void stream_finish(const RowsArgs& a) {
  const DeviceTables* t = a.tabs;
  const std::uint32_t poly = t->poly;
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint64_t wave = (blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x) >> 6;
  const std::uint64_t nw = (static_cast<std::uint64_t>(gridDim.x) * blockDim.x) >> 6;
  const std::uint64_t n = a.nblocks;
  for (std::uint64_t w0 = wave * 63u; w0 < n; w0 += nw * 63u) {
    const std::uint64_t b = w0 + lane - 1u;  // lane 0 of the first step: b = ~0 (no block: L = 0)
    const bool have = (w0 + lane) != 0u && b < n;
    std::uint64_t e = a.s_info[1];  // the stream start, the end of "block -1"
    std::uint32_t Le = 0, w = 0;
    if (have) {
      e = a.s_ends[b];
      w = a.s_wv[b];
      const std::uint64_t yq = a.s_yq[b];
      const std::uint64_t rowend = ((e - 1) / kRow + 1) * kRow;
      Le = dev::multmodp(t->inv_shift[rowend - e], static_cast<std::uint32_t>(yq), poly) ^
           static_cast<std::uint32_t>(yq >> 32);
    }
    const int src = static_cast<int>((lane == 0u ? 0u : lane - 1u) * 4u);
    const std::uint32_t Lp = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(Le)));
    const std::uint32_t wp = static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(w)));
    const std::uint64_t ep =
        static_cast<std::uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(static_cast<std::uint32_t>(e)))) |
        (static_cast<std::uint64_t>(static_cast<std::uint32_t>(
             __builtin_amdgcn_ds_bpermute(src, static_cast<int>(static_cast<std::uint32_t>(e >> 32)))))
         << 32);
    if (lane == 0u || b >= n) continue;
    std::uint32_t crc0 = Le;
    for (std::uint32_t v = wp; v < w; ++v)
      crc0 ^= dev::multmodp(stream_x8n(t, e - static_cast<std::uint64_t>(a.s_row0[v + 1]) * kRow), a.s_wtot[v], poly);
    const std::uint32_t init = a.init_raw ? a.init_raw[b] : a.init_default;
    const std::uint32_t raw = dev::multmodp(stream_x8n(t, e - ep), init ^ Lp, poly) ^ crc0;
    a.out[b] = raw ^ a.out_xor;
  }
}

template <bool ALIGNED, bool UNIFORM>
__global__ __launch_bounds__(kRowsThreads) void crc_rows(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  if constexpr (!UNIFORM) {
    if (gate_closed(a.gate, a.gate_seq)) return;  // crc_list_lanes folded every block
    // irregular batch whose blocks lie back to back: the prepass chose the byte-stream row walk,
    // crc_stream (launched just before) has walked it, and this launch turns its registers into
    // block CRCs
    if (dev::sload32(a.counts, 3) == kModeStream) {
      stream_finish(a);
      return;
    }
  }
  // issue priority from the rows left (set_prio_from_left): +0.7 % on cfg4 (profiles/r1/launch_irr_pri3.txt)
  dev::crc_rows_body<ALIGNED, UNIFORM, Shape<ALIGNED>::kDepth, Shape<ALIGNED>::kIlp, 3>(a, lds);
}

// Byte-stream row walk of an irregular batch in stream mode: the packed kernel's
// shape, issue priority and skewed row partition; returns at once on general batches.
// Skewed row partition (stream_row0): +0.5 % on cfg4 against the even split (in-process A/B).
constexpr unsigned kStreamThreads = kThreads;
constexpr int kStreamSkew = 154;
__global__ __launch_bounds__(kStreamThreads) void crc_stream(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  if (gate_closed(a.gate, a.gate_seq)) return;  // crc_list_lanes folded every block
  if (dev::sload32(a.counts, 3) != kModeStream) {
    // General path: this launch folds the batch's lane and group blocks (len <= kGroup8Max, DESIGN.md
    // §4.5), each phase only if the prepass found its blocks; crc_rows follows with the rest. The
    // group passes (lane-shift column 64 - G + g) need the lane-shift tables, the lane phase not.
    const std::uint32_t ph = dev::sload32(a.counts, kCountPhases);
    if (ph == 0) return;
    if (ph & 6u) dev::fill_lds(a.tabs, lds);
    else dev::fill_lds_slicing(a.tabs, lds);
    __syncthreads();  // (the mode and ph are the same for the whole grid)
    if (ph & 1u) dev::lane_phase(a, lds);
    if (ph & 2u) dev::group_phase<4>(a, lds);
    if (ph & 4u) dev::group_phase<8>(a, lds);
    return;
  }
  dev::fill_lds(a.tabs, lds);
  __syncthreads();  // the one barrier of the stream walk
  // issue priority from the rows left: +0.8 % on cfg4 (in-process A/B). A wave whose rows hold more
  // than 8 block ends per row on average (blocks under ~500 bytes) takes them a row at a time
  // (MANY); the others keep the per-end loop, whose code the MANY path slows by up to 10 % when it
  // shares the loop (4 KiB blocks, profiles/r2/stream_many/). Neither body holds a barrier, so the
  // waves of a workgroup may mix them.
  const std::uint32_t wave = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t g0 = dev::sload32(a.s_row0, wave), g1 = dev::sload32(a.s_row0, wave + 1);
  const std::uint32_t e0 = dev::sload32(a.wave_start, wave);
  const std::uint32_t e1 = wave + 1 < a.nwaves ? dev::sload32(a.wave_start, wave + 1) : a.nblocks;
  const bool many = g1 > g0 && e1 > e0 && e1 - e0 > 8u * (g1 - g0);
  if (many) dev::crc_stream_body<3, true>(a, lds);
  else dev::crc_stream_body<3, false>(a, lds);
}

// Packed uniform batches (len % 4 KiB == 0, stride == len, 16-byte aligned): DESIGN.md §4.
// Issue priority follows the work a wave has left (PRIO); blocks of several rows also skew the
// workgroup's slice towards the SIMDs' older waves (SKEW 154/256 per slot class). Measured in one
// process against the plain static partition: +0.8 to +1.4 % on 4 KiB blocks (where the skew
// loses), +3.7 % on 64 KiB blocks (profiles/r1/launch_prio*_cfg*.txt).
constexpr int kPackedDepth = 4;
constexpr int kPackedIlp = 2;
constexpr int kPackedSkew = 154;
constexpr int kPackedPrio = 3;  // set_prio_from_left thresholds 1/4, 1/8, 1/16

template <bool R1>
__global__ __launch_bounds__(kThreads) void crc_packed(RowsArgs a) {
  static_assert(kThreads == 1024, "the skewed partition assumes 16 waves per workgroup");
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_packed_body<kPackedDepth, kPackedIlp, R1, R1 ? 0 : kPackedSkew, kPackedPrio>(a, lds);
}

// Packed small blocks (len = 64 G <= 2 KiB for a power of two G, stride == len, 16-byte aligned,
// default init): DESIGN.md §4.4.
template <int G>
__global__ __launch_bounds__(kThreads) void crc_packed_small(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_packed_small_body<G, kPackedDepth, kPackedIlp, kPackedPrio>(a, lds);
}

// General small uniform blocks (64 < len <= 2 KiB, any stride, alignment, initial registers):
// DESIGN.md §4.4. G-lane groups, five granules per lane. DEPTH 4 spills here; DEPTH 2 / ILP 1 measured
// 1-3 % faster than DEPTH 3 / ILP 1 in one process (profiles/r3/small_gen/ab_depth.jsonl).
constexpr int kGenDepth = 2;
constexpr int kGenIlp = 1;
template <int G, bool INIT>
__global__ __launch_bounds__(kThreads) void crc_packed_small_gen(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsWords];
  dev::crc_packed_small_gen_body<G, INIT, kGenDepth, kGenIlp, kPackedPrio>(a, lds);
}

// Uniform batches of blocks of at most kLaneMax bytes (any stride, alignment, initial registers): one
// lane per block, a window of exactly the NG granules a block can touch and DEPTH 8 at NG <= 2, 6 at
// NG 3, 5 at NG 4, 4 at NG 5, ILP 1. Only the slicing tables go to LDS (128 KiB).
// In one process against the five-granule DEPTH 3-4 kernel of round 3 (profiles/r4/lanes_ab/):
// 26 B 3544 -> 3825 GB/s, 16 B 3615 -> 3720, 28 B 3877 -> 4044, 36 B and 59 B unchanged.
// One 1024-thread workgroup per CU on the 128 KiB image (the 64 KiB 16-replica image with two
// workgroups per CU measured within -5..+2 %, profiles/r4/lanes16/). 5-granule windows keep no step
// in flight (+7-13 % at 52-60 B in one process against DEPTH 4, profiles/r4/lanes_r/nopf_probe.jsonl;
// the right-aligned kernel measured the same, crc_lanes_r).
template <int ALIGN, int NG>
__global__ __launch_bounds__(kThreads) void crc_lanes_n(RowsArgs a) {
  constexpr int DEPTH = NG <= 2 ? 8 : NG == 3 ? 6 : NG == 4 ? 5 : 1;
  __shared__ std::uint32_t lds[kLdsSliceWords];
  dev::crc_lanes_n_body<ALIGN, NG, DEPTH, 1, kPackedPrio>(a, lds);
}

// Uniform lane batches with the default initial register, right-aligned windows of NF whole dwords
// (crc_lanes_r_body); ALIGN is the window start's alignment class.
template <int ALIGN, int NF>
__global__ __launch_bounds__(kThreads) void crc_lanes_r(RowsArgs a) {
  constexpr int kMis = ALIGN == 16 ? 0 : ALIGN == 4 ? 12 : 15;
  constexpr int NG = (4 * NF + kMis + 15) / 16;
// 5-granule windows load no step ahead of their fold: in one process against DEPTH 4 / 3 / 2
// (profiles/r4/lanes_r/depth_probe.jsonl) 50-59 B ran 11-13 % faster with no step in flight and the
// same with one to three; narrow windows (5-27 B) want their steps in flight (+2 to +20 %).
  constexpr int DEPTH = NG <= 2 ? 8 : NG == 3 ? 6 : NG == 4 ? 5 : 1;
  __shared__ std::uint32_t lds[kLdsSliceWords];
  dev::crc_lanes_r_body<ALIGN, NF, NG, DEPTH, kPackedPrio>(a, lds);
}

// Uniform lane batches staged through LDS by LDS-DMA (crc_lanes_lds_body): strides up to
// kLanesLdsMaxStride, default initial registers. RA: blocks not dword-aligned (v_alignbyte reads).
template <bool RA, int NW, int KB>
__global__ __launch_bounds__(kThreads) void crc_lanes_lds(RowsArgs a) {
  __shared__ std::uint32_t lds[kLdsSliceWords / 2 + kThreads / 64 * 2 * dev::kLanesLdsBuf / 4];
  dev::crc_lanes_lds_body<RA, NW, KB, kPackedPrio>(a, lds);
}

__global__ void crc_fixup(RowsArgs a) { dev::crc_fixup_body(a); }

// ---- irregular batches of blocks up to 1 KiB in one pass ----------------------------------------------
// crc_list_lanes folds an irregular batch (default initial register) straight from the caller's
// (offset, length) arrays when no block is over kPackMax = 1 KiB, with no prepass: the general
// path's launches that follow it return at once unless it met a longer block (gate). Wave w takes
// 64-block steps [w TS / W, (w + 1) TS / W), in one of two modes:
//  * lanes (every block of the step at most kLaneMax bytes): one lane per block. A step's blocks
//    usually lie in a few KiB (WAL payloads); then its bytes [lo, hi) are loaded by coalesced 16-byte
//    buffer loads (a descriptor that ends at hi, so nothing past the last block is read), kListRows
//    rows per lane, kListRing steps ahead in registers, written into the wave's LDS window just before
//    the fold, and every lane folds its block from the window (the WAL sweep's fold,
//    tkv_wal_device.hip). A later step whose blocks do not fit one window, or are not in ascending
//    order from its first block, loads each block's granules per lane instead (correct for any batch).
//  * packed (pack_walk): from the first step that holds a longer block, or that is no window when it
//    is the wave's first, to the end of the wave's range (the steps before it are done): a block gets
//    ceil(len / 64) lanes of a per-wave lane stream, one 64-byte piece per lane (see pack_walk).
// A block over kPackMax bytes stops the kernel: the first wave of a workgroup to meet one writes the
// call's sequence number into the workgroup's flag, every wave polls the flags and leaves, and the
// general path then folds the whole batch (rows_tile_scan opens the gate from the flags). A workgroup
// any of whose waves took the packed mode says so in a second flag array (counts[kPackFlags + g],
// tkv_debug_irregular_path).
// The per-workgroup flags, polled by every wave: next() issues this lane's load of flag lane + 64 g
// (g taking the ceil(groups / 64) groups in turn, clamped to the last flag) and returns whether the
// load issued at the previous call found the call's number (seq is never 0). (An unconditional load
// whose value waits a step group: a conditional one, or one compared at once, made every check wait
// for all loads in flight.)
struct FlagPoll {
  const std::uint32_t* flags;
  std::uint32_t last, ngrp, lane, grp = 0, v = 0;
  __device__ FlagPoll(const std::uint32_t* f, std::uint32_t groups, std::uint32_t l)
      : flags(f), last(groups - 1u), ngrp((groups + 63u) / 64u), lane(l) {}
  __device__ __forceinline__ bool next(std::uint32_t seq) {
    const bool hit = v == seq;
    const std::uint32_t f = lane + 64u * grp;
    v = __hip_atomic_load(flags + (f < last ? f : last), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    grp = grp + 1u == ngrp ? 0u : grp + 1u;
    return hit;
  }
};

constexpr std::uint32_t kListSpan = 4096;          // bytes of one step's window
constexpr int kListRows = kListSpan / 1024;        // 1 KiB load rows per step
constexpr int kListRing = 3;                       // steps of data in registers (R - 1 ahead of the fold)
constexpr unsigned kListThreads = 1024;
constexpr unsigned kListWaves = kListThreads / 64;
constexpr std::uint32_t kListSlot = 32 + kListSpan + 96;  // a window slot: slack for reads before and after
constexpr std::uint32_t kPackMax = kSmallMax;             // 16 lanes at most per block
// LDS (one workgroup per CU): the 64 KiB 16-replica image, the packed mode's shift tables (8 KiB:
// word ((sh >> 1) * 8 + j) * 32 + (v | 16 (sh & 1)) = Shift_{64 sh}(v << 4 j), even shifts in the
// lower 16 banks, odd ones in the upper, so the pieces of one block split the banks),
// Shift_len(0xFFFFFFFF) ^ xorout for len <= kPackMax, then per wave its window slot or, in the packed
// mode, desc[2][64] (16 B), map[2048] (u8: accumulator buffer << 6 | block), acc[4][64], acc_chunk[4]
constexpr std::uint32_t kListLsp = kLdsSliceWords * 2;
constexpr std::uint32_t kListInj = kListLsp + 8 * 8 * 32 * 4;
constexpr std::uint32_t kListWaveArea = kListInj + 4 * (kPackMax + 4);
constexpr std::uint32_t kPackDesc = 0, kPackMap = 2048, kPackAcc = 4096, kPackAccQ = 5120;
constexpr std::uint32_t kListWaveBytes = 5136;
static_assert(kListWaveBytes >= kListSlot && kListWaveBytes >= kPackAccQ + 16, "wave area");
constexpr std::uint32_t kListLdsBytes = kListWaveArea + kListWaves * kListWaveBytes;
static_assert(kListLdsBytes + 8 <= 163840, "LDS");
static_assert(kPackFlags == kListFlags + static_cast<int>(kListMaxGroups), "pack flags follow the list flags");

// The packed mode of crc_list_lanes over steps (chunks) [s0, s0 + ns) of a wave: a block of len bytes
// gets k = ceil(len / 64) lanes of a per-wave lane stream: a chunk's k are scanned (DPP) into each
// block's first lane, and its block-lanes write their descriptor and a lane -> block map into the
// wave's LDS area. Substeps take the stream 64 lanes at a time, running from one chunk into the next
// (never further), so no substep is padded at a chunk's end: lane g of k folds the block's bytes
// [len - 64 (k - g), len - 64 (k - g - 1)) from zero (the bytes in front of the block masked: leading
// zeros leave an init-0 register at 0), moves the result to the block's end by Shift_{64 (k - 1 - g)}
// (nibble tables, one column per shift), and XORs it into the block's LDS accumulator, which the
// block-lane seeded with Shift_len(0xFFFFFFFF) ^ xorout (crc_s(D) = Shift_|D|(s) ^ crc_0(D)). After the
// substep that holds a chunk's last lane, its accumulators are the block CRCs. Against the 4-lane
// groups of the general path, a substep fills its 64 lanes with pieces whatever the length mix (a
// 128-byte block takes two lanes, not four, a 40-byte one one) and nothing is read twice:
// descriptors once, payload granules once per piece (5 granules for 64 bytes). A chunk with no lane
// (every block empty) is written when it is prepared.
// Pipeline: a substep's granules are issued one substep before its fold; a chunk is prepared (map,
// descriptors, accumulator seeds) when the stream first needs it as the chunk after the current one,
// its descriptors loaded two chunks earlier. Two descriptor buffers and a 2048-entry map ring (two
// chunks: at most 2 x 16 x 64 lanes), four accumulator buffers: a chunk's seeds never meet an unfolded
// substep of the chunk four before it (each substep spans two chunks at most).
__device__ __forceinline__ void pack_walk(const RowsArgs& a, std::uint8_t* lds, std::uint8_t* ws, std::uint64_t s0,
                                          std::uint32_t ns, std::uint32_t lane, const dev::LaneConstX& kc,
                                          FlagPoll& poll, std::uint32_t* wg_hit) {
  const std::uint64_t n = a.nblocks;
  const std::uint32_t seq = a.gate_seq;
  std::uint32_t* flags = const_cast<std::uint32_t*>(a.gate_flags);
  const std::uint32_t* tab = reinterpret_cast<const std::uint32_t*>(lds);
  const std::uint32_t* inj = reinterpret_cast<const std::uint32_t*>(lds + kListInj);
  uint4* desc = reinterpret_cast<uint4*>(ws + kPackDesc);
  std::uint8_t* map = ws + kPackMap;
  std::uint32_t* acc = reinterpret_cast<std::uint32_t*>(ws + kPackAcc);
  std::uint32_t* accq = reinterpret_cast<std::uint32_t*>(ws + kPackAccQ);
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  const std::uintptr_t dmy = reinterpret_cast<std::uintptr_t>(a.dummy);

  // descriptors of the next two chunks to prepare (c0: the next one)
  std::uint64_t c0_off, c1_off;
  std::uint32_t c0_len, c1_len;
  auto fetch = [&](std::uint32_t q, std::uint64_t& off, std::uint32_t& len) {
    const std::uint64_t b = (s0 + q) * 64u + lane;
    const std::uint64_t bc = b < n ? b : n - 1u;  // clamped: every load stays inside the arrays
    off = a.offsets[bc];
    len = a.lengths[bc];
  };
  fetch(0, c0_off, c0_len);
  fetch(1, c1_off, c1_len);

  // wave-uniform stream state: the next lane to issue s, the end of the current chunk A (the one
  // holding s) and of the prepared chunk after it, B (eb == ea: none); their accumulator buffers sa, sb
  std::uint32_t s = 0, ea = 0, eb = 0, sa = 0, sb = 0;
  std::uint32_t iq = 0, np = 0, quit = 0;  // next chunk to look at, chunks prepared
  auto wave_fence = [] {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  auto leave = [&] {
    if (lane == 0 && atomicExch(wg_hit, 1u) == 0u)
      __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    quit = 1u;
  };
  // prepares the next chunk with lanes as B, its lanes from eb on; false when none is left (or on quit)
  auto prepare = [&]() -> bool {
    while (iq < ns && quit == 0u) {
      const std::uint32_t q = iq++;
      const std::uint64_t b = (s0 + q) * 64u + lane;
      const bool live = b < n;
      const std::uint32_t len = live ? c0_len : 0u;
      const std::uint64_t off = c0_off;
      c0_off = c1_off;
      c0_len = c1_len;
      fetch(q + 2u, c1_off, c1_len);
      quit = __builtin_amdgcn_readfirstlane(quit | (__ballot(poll.next(seq)) != 0 ? 1u : 0u));
      if (__ballot(len > kPackMax) != 0) leave();
      if (quit != 0u) return false;
      const std::uint32_t k = (len + 63u) >> 6;
      std::uint32_t total;
      const std::uint32_t ex = dev::lane_prefix(k, &total);
      const std::uint32_t T = __builtin_amdgcn_readfirstlane(total);
      if (T == 0u) {  // every block empty: the CRCs are the seeds
        if (live) a.out[b] = inj[0];
        continue;
      }
      const std::uint32_t slot = np++ & 3u, v0 = eb + ex;  // the block's first lane in the stream
      wave_fence();  // reads of the chunk two before (descriptors, map) and of this buffer are done
      desc[(slot & 1u) * 64u + lane] = make_uint4(static_cast<std::uint32_t>(off), static_cast<std::uint32_t>(off >> 32), len, v0);
      for (std::uint32_t r = 0; __ballot(r < k) != 0; ++r)
        if (r < k) map[(v0 + r) & 2047u] = static_cast<std::uint8_t>(slot << 6 | lane);
      acc[slot * 64u + lane] = inj[len];
      accq[slot] = q;
      wave_fence();
      eb += T;
      sb = slot;
      return true;
    }
    return false;
  };

  uint4 qv[2][dev::kLaneGran];
  std::uint32_t m_o[2], m_sh[2], m_acc[2];
  std::int32_t m_lead[2];   // 8 x the bytes of the piece in front of the block
  std::uint32_t m_done[2];  // wave-uniform: 1 + the buffers of the chunks this substep completes, 3 bits each
  bool m_dead[2];           // wave-uniform: past the wave's last lane
  bool m_fast[2];           // wave-uniform: dword-aligned loads (else 16-byte granules)
  auto issue = [&](int r) {
    if (quit == 0u) {
      if (s >= ea && eb > ea) {  // A is done (the last substep may have run into B): B becomes A
        ea = eb;
        sa = sb;
      }
      if (s >= ea && prepare()) {  // none prepared (s == ea == eb): the next chunk becomes A
        ea = eb;
        sa = sb;
      }
      if (s < ea && eb == ea) prepare();  // a chunk B for the substep to run into
    }
    m_dead[r] = __builtin_amdgcn_readfirstlane(s >= ea || quit != 0u ? 1u : 0u) != 0u;
    if (m_dead[r]) return;
    const std::uint32_t e = eb - s < 64u ? eb : s + 64u;  // never past B
    const std::uint32_t v = s + lane;
    const bool live = v < e;
    const std::uint32_t mv = map[v & 2047u];
    const std::uint32_t bslot = mv >> 6, blk = mv & 63u;
    const uint4 d = desc[(bslot & 1u) * 64u + blk];
    const std::uint32_t len = live ? d.z : 0u;
    const std::uint32_t g = v - d.w;  // this lane's piece of the block
    const std::uint32_t k = (len + 63u) >> 6;
    const std::int32_t c_lane = static_cast<std::int32_t>(len) - 64 * static_cast<std::int32_t>(k - g);
    const std::uintptr_t blo = base + (static_cast<std::uint64_t>(d.y) << 32 | d.x);
    const std::uintptr_t p = static_cast<std::uintptr_t>(static_cast<std::int64_t>(blo) + c_lane);
    // Four dword-aligned 16-byte loads and one dword (as the row kernel's interior rows: one
    // v_alignbyte per dword realigns them) unless a piece in front of its block could reach into the
    // page before the block's first byte (the block starts within 16 bytes of a page): then the wave
    // takes the 16-byte granules the block touches (realigned by two selects and a v_alignbyte).
    const bool fast = __ballot(live && c_lane < 0 && (blo & 4095u) < 16u) == 0;
    m_fast[r] = fast;
    if (fast) {
      const std::uintptr_t pd = p & ~static_cast<std::uintptr_t>(3);
      const std::uint32_t o3 = static_cast<std::uint32_t>(p & 3u);
      // load i covers [pd + 16 i, + 16), never past the piece's end (at most the block's): it holds a
      // byte of the block iff pd + 16 i + 16 > blo; the dword at pd + 64 holds the piece's last o3 bytes
      const std::int32_t rel = c_lane - static_cast<std::int32_t>(o3) + 16;
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[r][i] = dev::gload16(live && rel + 16 * i > 0 ? pd + 16u * i : dmy);
      qv[r][4] = make_uint4(*reinterpret_cast<dev::g_u32*>(live && o3 != 0u ? pd + 64u : dmy), 0u, 0u, 0u);
      m_o[r] = o3;
    } else {
      const std::uintptr_t al = p & ~static_cast<std::uintptr_t>(15);
      const std::uint32_t o = static_cast<std::uint32_t>(p & 15u);
      // granule i holds a byte of the block iff al + 16 i - blo lies in (-16, len), i.e. al + 16 i - blo
      // + 15 in [0, len + 15) (32-bit arithmetic: -80 < al - blo < len); the others read `dummy`, so no
      // load leaves the 16-byte granules the block touches
      const std::int32_t rel = c_lane - static_cast<std::int32_t>(o) + 15;
#pragma unroll
      for (int i = 0; i < dev::kLaneGran; ++i) {
        const bool in = live && static_cast<std::uint32_t>(rel + 16 * i) < len + 15u;
        qv[r][i] = dev::gload16(in ? al + 16u * i : dmy);
      }
      m_o[r] = o;
    }
    m_lead[r] = live ? (c_lane < 0 ? -8 * c_lane : 0) : 512;  // bits in front of the block (512: all)
    m_sh[r] = live ? k - 1u - g : 0u;
    m_acc[r] = live ? bslot * 64u + blk : ~0u;
    // the chunks whose last lane lies in [s, e): A when e reaches its end, B too when e is its end
    const std::uint32_t done = (ea <= e ? sa + 1u : 0u) | (eb > ea && eb <= e ? (sb + 1u) << 3 : 0u);
    m_done[r] = __builtin_amdgcn_readfirstlane(done);
    s = e;
  };
  auto readout = [&](std::uint32_t slot) {
    const std::uint32_t q = __builtin_amdgcn_readfirstlane(accq[slot]);
    const std::uint64_t b = (s0 + q) * 64u + lane;
    const std::uint32_t crc = acc[slot * 64u + lane];
    if (b < n) a.out[b] = crc;
  };
  auto fold = [&](int r) {
    std::uint32_t d[16];
    if (m_fast[r]) {
      const std::uint32_t raw[17] = {qv[r][0].x, qv[r][0].y, qv[r][0].z, qv[r][0].w, qv[r][1].x, qv[r][1].y,
                                     qv[r][1].z, qv[r][1].w, qv[r][2].x, qv[r][2].y, qv[r][2].z, qv[r][2].w,
                                     qv[r][3].x, qv[r][3].y, qv[r][3].z, qv[r][3].w, qv[r][4].x};
#pragma unroll
      for (int k = 0; k < 16; ++k) d[k] = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], m_o[r]);
    } else {
      dev::lane_dwords<1>(qv[r], m_o[r], d);
    }
    const std::uint32_t lead8 = static_cast<std::uint32_t>(m_lead[r]);
    dev::Reg reg{0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k) dev::slice4(tab, reg, dev::mask_front(d[k], lead8, k), kc);
    const std::uint32_t p = reg.value();
    const std::uint32_t sh = m_sh[r];
    const std::uint32_t lb = kListLsp + (sh >> 1) * 1024u + ((sh & 1u) << 6);
    std::uint32_t l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = dev::lds_at(tab, lb + 128u * j + (((p >> (4 * j)) & 15u) << 2));
    const std::uint32_t v = dev::xor3(dev::xor3(l[0], l[1], l[2]), dev::xor3(l[3], l[4], l[5]), l[6] ^ l[7]);
    if (m_acc[r] != ~0u) __hip_atomic_fetch_xor(acc + m_acc[r], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    const std::uint32_t done = m_done[r];
    if (done != 0u) {
      wave_fence();
      if (done & 7u) readout((done & 7u) - 1u);
      if (done >> 3) readout((done >> 3) - 1u);
    }
  };
  issue(0);
  for (bool fin = false; !fin;) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      issue(k ^ 1);
      if (m_dead[k]) {
        fin = true;
        break;
      }
      fold(k);
    }
  }
}

__global__ __launch_bounds__(kListThreads) void crc_list_lanes(RowsArgs a) {
  __shared__ __attribute__((aligned(16))) std::uint8_t lds[kListLdsBytes];
  __shared__ std::uint32_t wg_words[2];  // this workgroup flagged the batch / took the packed mode
  std::uint32_t* wg_hit = &wg_words[0];
  if (threadIdx.x == 0) wg_words[0] = wg_words[1] = 0;  // (ordered before any use by the barrier below)
  std::uint32_t* tab = reinterpret_cast<std::uint32_t*>(lds);
  std::uint32_t* inj = reinterpret_cast<std::uint32_t*>(lds + kListInj);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the batch's counts as the general path's debug entry points report them when it does not run
    // (tkv_debug_irregular_*); the prepass rewrites them when it does
    std::uint32_t* c = const_cast<std::uint32_t*>(a.counts);
    c[0] = c[1] = c[2] = c[3] = 0;
    c[kCountLanes] = c[kCountPhases] = c[kCountSmall4] = c[kCountSmall8] = 0;
  }
  const std::uint32_t lane = threadIdx.x & 63u;
  const std::uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const std::uint32_t wave = blockIdx.x * kListWaves + wv;
  const std::uint64_t W = a.nwaves, n = a.nblocks;
  const std::uint64_t TS = (n + 63u) / 64u;
  const std::uint64_t s0 = wave * TS / W;
  const std::uint32_t ns = static_cast<std::uint32_t>((wave + 1) * TS / W - s0);
  std::uint32_t* flags = const_cast<std::uint32_t*>(a.gate_flags);
  const std::uint32_t seq = a.gate_seq;
  // the first step's lengths before anything else: a workgroup that meets a block over kPackMax there
  // leaves before its table fill (a batch of long blocks costs this launch little more than its dispatch)
  const std::uint64_t b00 = s0 * 64u + lane;
  const std::uint32_t len00 = ns != 0 ? a.lengths[b00 < n ? b00 : n - 1u] : 0u;
  // a wave whose first step holds a longer block starts in the packed mode (no lane-mode prologue)
  const bool long0 = __ballot(ns != 0 && b00 < n && len00 > kLaneMax) != 0;
  if (__syncthreads_or(ns != 0 && b00 < n && len00 > kPackMax ? 1 : 0) != 0) {
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  dev::fill_lds_slicing16(a.tabs, tab);
  std::uint32_t* lsp = reinterpret_cast<std::uint32_t*>(lds + kListLsp);
  for (std::uint32_t i = threadIdx.x; i < 8u * 16u * 16u; i += blockDim.x) {
    // source order (columns 48-63 of each (j, v) row: coalesced), scattered into the shift tables
    const std::uint32_t j = i >> 8, v = (i >> 4) & 15u, sh = 15u - (i & 15u);
    lsp[((sh >> 1) * 8u + j) * 32u + (v | ((sh & 1u) << 4))] = a.tabs->lane_shift[j][v][63u - sh];
  }
  for (std::uint32_t i = threadIdx.x; i <= kPackMax; i += blockDim.x) inj[i] = a.tabs->init_shift[i] ^ a.out_xor;
  __syncthreads();
  if (ns == 0) return;
  const dev::LaneConstX kc = dev::lane_const16(lane);
  std::uint8_t* ws = lds + kListWaveArea + wv * kListWaveBytes;
  std::uint8_t* win = ws + 32;  // the step's bytes from its granule start
  const std::uintptr_t base = reinterpret_cast<std::uintptr_t>(a.base);
  constexpr int R = kListRing;
  std::uint64_t m_off[R];
  std::uint32_t m_len[R];
  auto fetch = [&](std::uint32_t j, int k) {  // step j's descriptors
    const std::uint64_t b = (s0 + j) * 64u + lane;
    const std::uint64_t bc = b < n ? b : n - 1u;
    m_off[k] = a.offsets[bc];
    m_len[k] = a.lengths[bc];
  };
  uint4 d[R][kListRows];
  std::uint32_t f_rel[R], f_len[R];  // the block's byte in the window (or its offset's low word), its length
  std::uint32_t f_hi[R];             // gathered steps: the offset's high word
  bool staged[R];
  std::uint32_t quit = 0;           // wave-uniform (readfirstlane): the wave stops
  std::uint32_t sw = long0 ? 0 : ns;  // wave-uniform: the first step of the packed mode (ns: none)
  auto issue = [&](std::uint32_t j, int k) {  // step j's bytes, from its descriptors in slot k
    const std::uint64_t b = (s0 + j) * 64u + lane;
    const bool live = j < ns && b < n;
    const std::uint64_t off = m_off[k];
    const std::uint32_t len = m_len[k];
    const std::uint64_t lb = __ballot(live && len > kPackMax);
    // one store per workgroup (the first wave to meet a block over kPackMax: an LDS exchange elects it)
    if (lb != 0 && lane == 0 && atomicExch(wg_hit, 1u) == 0u)
      __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    quit = __builtin_amdgcn_readfirstlane(quit | (lb != 0 ? 1u : 0u));
    if (__ballot(live && len > kLaneMax) != 0 && j < sw) sw = j;  // the packed mode from here
    const std::uint64_t lo = dev::readlane64(off, 0);  // (lane 0 is live whenever any lane is)
    const std::uint64_t al = (base + lo) & ~static_cast<std::uint64_t>(15);
    const std::uint64_t rel = base + off - al;
    const bool fit = !live || (off >= lo && rel + len <= kListSpan);
    // (a step of the packed mode loads nothing here: a descriptor of 0 records reads no memory)
    const bool all = __ballot(!fit) == 0 && __ballot(live) != 0 && j < sw;
    const std::uint32_t hi = dev::wave_max(live ? static_cast<std::uint32_t>(rel < kListSpan ? rel + len : 0u) : 0u);
    const std::uint32_t nrec = all ? ((hi + 15u) & ~15u) : 0u;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(static_cast<std::uintptr_t>(
            static_cast<std::uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(al))) |
            static_cast<std::uint64_t>(static_cast<std::uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<std::uint32_t>(al >> 32)))) << 32)),
        0, __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
#pragma unroll
    for (int r = 0; r < kListRows; ++r) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16u * lane + 1024u * r, 0, 0);
      d[k][r] = uint4{v[0], v[1], v[2], v[3]};
    }
    staged[k] = all;
    f_rel[k] = all ? static_cast<std::uint32_t>(rel) : static_cast<std::uint32_t>(off);
    f_hi[k] = static_cast<std::uint32_t>(off >> 32);
    f_len[k] = live ? len : 0xFFFFFFFFu;
  };
  auto fold = [&](std::uint32_t j, int k) {
    const std::uint32_t len = f_len[k];
    const bool live = len != 0xFFFFFFFFu;
    const std::uint32_t L = live ? len : 0u;
    std::uint32_t crc;
    if (staged[k]) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < kListRows; ++r) *reinterpret_cast<uint4*>(win + 1024u * r + 16u * lane) = d[k][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // the payload read as dwords ending on its last byte, the z bytes in front zeroed, every lane
      // through the step's longest block with its register frozen after its own (tkv_wal_device.hip)
      const std::uint32_t nd = (L + 3u) >> 2;
      const std::uint32_t nmax = dev::wave_max(nd);
      const std::uint32_t z = 4u * nd - L;
      const std::uint32_t b0 = 32u + f_rel[k] - z;  // from the slot's start (32 bytes of slack in front)
      const std::uint32_t* w = reinterpret_cast<const std::uint32_t*>(win - 32 + (b0 & ~3u));
      const std::uint32_t sh = b0 & 3u;
      std::uint32_t lo = w[1];
      dev::Reg r{0u, 0u};
      dev::slice4(tab, r, __builtin_amdgcn_alignbyte(lo, w[0], sh) & (~0u << (8u * z)), kc);
      if (nd == 0u) r = dev::Reg{0u, 0u};
      for (std::uint32_t i = 1; i < nmax; ++i) {
        const std::uint32_t hw = w[i + 1u];
        dev::Reg t = r;
        dev::slice4(tab, t, __builtin_amdgcn_alignbyte(hw, lo, sh), kc);
        if (i < nd) r = t;
        lo = hw;
      }
      crc = r.value() ^ inj[L];  // (inj holds Shift_L(0xFFFFFFFF) ^ xorout)
    } else {
      // a step that is not one window: each lane loads its own block's granules (lane_phase's loads)
      const std::uintptr_t blk = base + (static_cast<std::uint64_t>(f_hi[k]) << 32 | f_rel[k]);
      uint4 q[dev::kLaneGran];
      dev::lane_issue<1>(blk, L, reinterpret_cast<std::uintptr_t>(a.dummy), q);
      std::uint32_t dd[1][16], nn[1] = {L}, rr[1] = {a.init_default};
      dev::lane_dwords<1>(q, static_cast<std::uint32_t>(blk & 15u), dd[0]);
      dev::lane_fold<1, false>(tab, kc, dd, nn, rr);
      crc = rr[0] ^ a.out_xor;
    }
    const std::uint64_t b = (s0 + j) * 64u + lane;
    if (live) a.out[b] = crc;
  };
  FlagPoll poll(flags, gridDim.x, lane);
  if (sw != 0) {
    // prologue: descriptors of steps 0 .. R-1, their data, then the descriptors of steps R .. 2R-1
#pragma unroll
    for (int k = 0; k < R; ++k) fetch(static_cast<std::uint32_t>(k), k);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      issue(static_cast<std::uint32_t>(k), k);
      fetch(static_cast<std::uint32_t>(k + R), k);
      __builtin_amdgcn_sched_barrier(0);  // in order: the loop's waits count the loads issued after these
    }
    // a first step that is not one window (blocks spread out, or 64-byte blocks back to back): the
    // packed mode, whose per-lane pieces take such layouts faster than per-lane granule loads
    if (!staged[0]) sw = 0;
  }
  for (std::uint32_t t = 0; t < sw && quit == 0u; t += R) {
    const bool hit = poll.next(seq);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const std::uint32_t j = t + static_cast<std::uint32_t>(k);
      if (j >= sw || quit != 0u) break;
      fold(j, k);
      issue(j + R, k);
      fetch(j + 2u * R, k);
    }
    // another workgroup met a block over kPackMax: the general path folds the batch
    quit = __builtin_amdgcn_readfirstlane(quit | (__ballot(hit) != 0 ? 1u : 0u));
  }
  if (quit != 0u || sw >= ns) return;
  // the packed mode for steps [sw, ns): its LDS area is this wave's window slot (the wave's own LDS
  // reads of the window are done: in order); one store per workgroup says it ran
  if (lane == 0 && atomicExch(&wg_words[1], 1u) == 0u)
    __hip_atomic_store(flags + kListMaxGroups + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  pack_walk(a, lds, ws, s0 + sw, ns - sw, lane, kc, poll, wg_hit);
}



}  // namespace

// ---- irregular-batch prepass -----------------------------------------------------------------------
// One exclusive scan over the blocks of the pair (small blocks, rows of large blocks), packed in a
// u64 (small count in the low word, rows in the high word), then a scatter that
//   * lists small blocks (len <= kSmallMax) in s_off/s_len/s_idx for the small-block phase,
//   * compacts large blocks into big_off/big_len/big_idx with their row offsets (row_scan) for the
//     row kernel, and records the first large block of every row-kernel wave (wave_start),
//   * leaves counts = {large blocks, small blocks, rows of large blocks}.
constexpr int kScanTile = 4096;  // blocks per scan tile (rows_tile_scan)
constexpr std::uint32_t kScanGroupsPerCu = 2;

__device__ __forceinline__ std::uint64_t scan_item(std::uint32_t len) {
  return len <= kSmallMax ? 1ull : static_cast<std::uint64_t>(rows_for_len(len)) << 32;
}

// Also records per tile whether its blocks qualify for stream mode: each at least kStreamMinLen
// bytes and ending where the next one starts.
// Stream mode's geometry: row 0 starts at the stream start rounded down to 16 bytes (offset zoff
// from base, the stream starting s0rel bytes into it) and TR rows of 4 KiB cover the stream. Only
// meaningful when the blocks lie back to back in order (the prepass checks that).
struct StreamGeom {
  std::uint64_t zoff, s0rel, rows;
};
__device__ __forceinline__ StreamGeom stream_geometry(const std::uint8_t* base, const std::uint64_t* offsets,
                                                      const std::uint32_t* lengths, std::uint32_t n) {
  const std::uint64_t off0 = offsets[0];
  const std::uint64_t s0rel = (reinterpret_cast<std::uintptr_t>(base) + off0) & 15u;
  // zoff may lie up to 15 bytes before base (a base that is not 16-byte aligned, with the stream
  // starting in its first bytes): it wraps as a u64, and base + zoff is still row 0's address, so
  // the row count is taken from the stream's own extent, never by comparing with zoff.
  const std::uint64_t zoff = off0 - s0rel;
  const std::uint64_t end = offsets[n - 1] + lengths[n - 1];
  return {zoff, s0rel, end >= off0 ? (end - off0 + s0rel + kRow - 1) / kRow : 0};
}

// Scan tiles of kScanTile blocks, looped over by at most kScanGroupsPerCu workgroups per CU, T
// threads with kScanTile / T consecutive blocks each. Batches of more than kFusedTiles tiles (over 4 M blocks: WAL-record-sized batches) take
// 512-thread tiles, which keep more tiles in flight per CU; fewer tiles keep 1024 threads (in one
// process, 1 GiB batches, profiles/r3/scan_tiles/: WAL payloads of 36 B with 8-byte gaps 1820 ->
// 1957 GB/s, back-to-back 36 B 1991 -> 2212, 64 B 2687 -> 2818, 128 B 730 -> 697 GB/s; cfg4 and
// the 64 KiB stream batch unchanged either way).
struct ScanLds {  // rows_scan_tiles_body's workspace (1024 threads)
  std::uint64_t part[1024], cpart[1024];
  std::uint32_t lpart[1024];
  std::uint32_t sph;
};
__device__ __forceinline__ void rows_scan_tiles_body(ScanLds& L, std::uint64_t* tile_sums, std::uint32_t* tile_lanes,
                                                     std::uint64_t* tile_cls, std::uint32_t ntiles, std::uint32_t n,
                                                     std::uint32_t* counts, const std::uint32_t* tile_ok,
                                                     const std::uint8_t* base, const std::uint64_t* offsets,
                                                     const std::uint32_t* lengths, std::uint64_t* sinfo);

template <unsigned kTileThreads>
__global__ __launch_bounds__(kTileThreads) void rows_tile_scan(const std::uint8_t* sbase, const std::uint64_t* offsets,
                                                              const std::uint32_t* lengths, std::uint32_t n,
                                                              std::uint64_t* scan, std::uint64_t* tile_sums,
                                                              std::uint32_t* tile_ok, std::uint32_t* row0, std::uint32_t Ws,
                                                              std::uint32_t* lscan, std::uint32_t* tile_lanes,
                                                              std::uint32_t* cscan, std::uint64_t* tile_cls,
                                                              std::uint32_t group_stream, const std::uint32_t* gate,
                                                              std::uint32_t seq, const std::uint32_t* gate_flags) {
  if (gate != nullptr) {
    // after crc_list_lanes: the general path runs only if one of its workgroups met a long block;
    // workgroup 0 publishes the verdict for the launches that follow
    bool hit = false;
    for (unsigned i = threadIdx.x; i < kListMaxGroups; i += kTileThreads) hit = hit || gate_flags[i] == seq;
    const bool open = __syncthreads_or(hit ? 1 : 0) != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *const_cast<std::uint32_t*>(gate) = open ? seq : 0u;
    if (!open) return;
  }
  constexpr unsigned kTileWaves = kTileThreads / 64;
  constexpr unsigned kTileBpt = kScanTile / kTileThreads;
  static_assert(kScanTile % kTileThreads == 0 && kTileWaves >= 1 && kTileBpt >= 4 && kTileBpt % 4 == 0,
                "tile shape");
  __shared__ std::uint64_t wsum[kTileWaves], lsum[kTileWaves];
  __shared__ std::uint32_t wok[kTileWaves];
  // stream mode's wave partition (used only if the prepass picks stream mode): row0[0..Ws], grid-stride
  for (std::uint32_t w = blockIdx.x * kTileThreads + threadIdx.x; w <= Ws; w += gridDim.x * kTileThreads) {
    const std::uint64_t TR = stream_geometry(sbase, offsets, lengths, n).rows;
    row0[w] = static_cast<std::uint32_t>(dev::stream_row0<kStreamSkew>(w, TR, Ws));
  }
  // one tile per workgroup (1024 threads), or tiles looped over by a bounded grid (512 threads, batches
  // of more than kFusedTiles tiles): the loop costs the 1024-thread shape a spill (125 VGPRs)
  auto tile_body = [&](const std::uint32_t tile) {
    const std::uint64_t base = static_cast<std::uint64_t>(tile) * kScanTile + threadIdx.x * kTileBpt;
    const unsigned lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    // Every block first counts as a small or large one (v); lane blocks, the two group classes and the
    // small blocks over kGroup8Max bytes are also counted in one packed u64 (16 bits each, lane blocks
    // lowest, then 4- and 8-lane group blocks, then the rest up to kSmallMax: a tile has at most 4096 of
    // each), so the one scan below yields all of them, and the tile's verdict on them (below) only
    // subtracts. The last two fields also place listed small blocks in their class's list (cscan).
    std::uint64_t pk[kTileBpt];
    std::uint64_t v[kTileBpt], s = 0;
    std::uint64_t ls = 0;
    // Loads at clamped indices, all issued before any is used (n >= 1 here): one round trip for the
    // lengths, one more for the offsets, which only a thread whose blocks are all long enough for stream
    // mode reads (a lane-block batch never touches them).
    std::uint32_t len[kTileBpt];
    bool ok = true;
#pragma unroll
    for (unsigned i = 0; i < kTileBpt; ++i) {
      const std::uint64_t b = base + i;
      len[i] = lengths[b < n ? b : n - 1];
    }
#pragma unroll
    for (unsigned i = 0; i < kTileBpt; ++i) {
      const bool in = base + i < n;
      len[i] = in ? len[i] : 0u;
      pk[i] = !in                    ? 0ull
              : len[i] <= kLaneMax    ? 1ull
              : len[i] <= kGroupMax   ? 1ull << 16
              : len[i] <= kGroup8Max  ? 1ull << 32
              : len[i] <= kSmallMax   ? 1ull << 48
                                      : 0ull;
      v[i] = in ? scan_item(len[i]) : 0ull;
      s += v[i];
      ls += pk[i];
      ok = ok && (!in || len[i] >= kStreamMinLen);
    }
    if (ok && base < n) {
      std::uint64_t o[kTileBpt + 1];
#pragma unroll
      for (unsigned i = 0; i <= kTileBpt; ++i) o[i] = offsets[base + i < n ? base + i : n - 1];
#pragma unroll
      for (unsigned i = 0; i < kTileBpt; ++i) ok = ok && (base + i + 1 >= n || o[i] + len[i] == o[i + 1]);
    }
    // Inclusive scans of the thread sums inside the wave (cross-lane shifts, no barriers), then the
    // wave totals through LDS: one barrier instead of the 20 of a workgroup-wide Hillis-Steele.
    std::uint64_t inc = s;
    std::uint64_t linc = ls;
#pragma unroll
    for (unsigned off = 1; off < 64; off <<= 1) {
      const std::uint64_t y = __shfl_up(inc, off, 64);
      const std::uint64_t ly = __shfl_up(linc, off, 64);
      inc += lane >= off ? y : 0ull;
      linc += lane >= off ? ly : 0ull;
    }
    const bool wave_ok = __ballot(!ok) == 0;
    if (lane == 63u) {
      wsum[wid] = inc;
      lsum[wid] = linc;
      wok[wid] = wave_ok ? 1u : 0u;
    }
    __syncthreads();
    std::uint64_t wpre = 0, tot = 0, lpre = 0, ltot = 0;
    std::uint32_t all_ok = 1;
#pragma unroll
    for (unsigned w = 0; w < kTileWaves; ++w) {
      const std::uint64_t t = wsum[w];
      const std::uint64_t lt = lsum[w];
      wpre += w < wid ? t : 0ull;
      tot += t;
      lpre += w < wid ? lt : 0ull;
      ltot += lt;
      all_ok &= wok[w];
    }
    // A tile with at least kLaneDenseTile lane blocks leaves them to the lane phase (in no list); one
    // with at most kGroupTileRows rows of large blocks leaves each group class of which it holds at
    // least that class's threshold to that class's group pass; in other tiles they are listed as small
    // blocks, so a batch with a few of them scattered about pays no phase walk over its metadata.
    const bool few_rows = (tot >> 32) <= kGroupTileRows;
    auto cls = [&](int c) { return static_cast<std::uint32_t>((ltot >> (16 * c)) & 0xFFFFu); };
    const std::uint32_t tph = (cls(0) >= kLaneDenseTile ? kTileLanes : 0u) |
                              (few_rows && cls(1) >= kGroupDenseTile ? kTileGroups : 0u) |
                              (few_rows && cls(2) >= kGroup8DenseTile ? kTileGroups8 : 0u);
    const std::uint64_t tmask = ((tph & kTileLanes) ? 0xFFFFull : 0ull) | ((tph & kTileGroups) ? 0xFFFFull << 16 : 0ull) |
                                ((tph & kTileGroups8) ? 0xFFFFull << 32 : 0ull);
    auto taken = [&](std::uint64_t x) {  // the phase blocks among packed counts x
      x &= tmask;
      return static_cast<std::uint32_t>((x & 0xFFFFu) + ((x >> 16) & 0xFFFFu) + ((x >> 32) & 0xFFFFu));
    };
    // listed blocks of kGroupMax + 1 .. kGroup8Max bytes (none when the 8-lane pass takes them) and of
    // kGroup8Max + 1 .. kSmallMax bytes among packed counts x, as the low and high half of a u32
    const std::uint64_t c8mask = (tph & kTileGroups8) ? 0ull : 0xFFFFull << 32;
    auto cls_pair = [&](std::uint64_t x) {
      return static_cast<std::uint32_t>(((x & c8mask) >> 32) | ((x >> 48) << 16));
    };
    // A tile whose bytes are mostly in small blocks (at least kStreamSmallTile blocks of at most
    // kSmallMax bytes and at most kGroupTileRows rows of larger ones) does not qualify for stream mode
    // (unless group_stream, a debug setting): the group passes and the small phase fold such blocks at
    // the rate of gapped ones, where the stream walk's rows of many block ends ran slower (back-to-back
    // 128 B: 1404 against 2351 GB/s, profiles/r3/group_phase/; 300-1000 B: 2893 against 3206,
    // profiles/r4/s5/). Tiles whose bytes are in larger blocks keep stream mode, where it wins (cfg4,
    // 64 KiB blocks, and short batches of any blocks).
    const bool small_tile = few_rows && static_cast<std::uint32_t>(tot) >= kStreamSmallTile;
    const bool stream_ok = all_ok && (group_stream != 0u || !small_tile);
    const std::uint64_t tile_n = n - static_cast<std::uint64_t>(tile) * kScanTile;  // blocks in the tile
    const bool all_taken = taken(ltot) == (tile_n < kScanTile ? tile_n : kScanTile);
    if (threadIdx.x == 0) tile_ok[tile] = (stream_ok ? kTileStream : 0u) | tph | (all_taken ? kTileAllTaken : 0u);
    std::uint64_t run = wpre + inc - s;  // exclusive, lane and group blocks counted as small
    std::uint64_t lrun = lpre + linc - ls;
    if (tph == 0 && base + kTileBpt <= n) {
      // every block of such a tile is listed: this thread's entries as whole 16-byte stores
      // (scan, lscan and cscan are 16-byte aligned scratch, base a multiple of kTileBpt >= 4)
      std::uint64_t sc[kTileBpt];
      std::uint32_t cs[kTileBpt];
#pragma unroll
      for (unsigned i = 0; i < kTileBpt; ++i) {
        sc[i] = run;
        cs[i] = cls_pair(lrun);
        run += v[i];
        lrun += pk[i];
      }
#pragma unroll
      for (unsigned i = 0; i < kTileBpt; i += 2)
        *reinterpret_cast<ulonglong2*>(scan + base + i) = make_ulonglong2(sc[i], sc[i + 1]);
#pragma unroll
      for (unsigned i = 0; i < kTileBpt; i += 4) {
        *reinterpret_cast<uint4*>(lscan + base + i) = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(cscan + base + i) = make_uint4(cs[i], cs[i + 1], cs[i + 2], cs[i + 3]);
      }
    } else {
#pragma unroll
      for (unsigned i = 0; i < kTileBpt; ++i) {
        if (base + i < n && !taken(pk[i])) {  // the scatter reads these for listed blocks only
          const std::uint32_t t = taken(lrun);
          scan[base + i] = run - t;  // (t <= the small count in run's low half: no borrow)
          lscan[base + i] = t;
          cscan[base + i] = cls_pair(lrun);
        }
        run += v[i];
        lrun += pk[i];
      }
    }
    if (threadIdx.x == kTileThreads - 1) {
      const std::uint32_t tl = taken(ltot);
      tile_sums[tile] = tot - tl;
      tile_lanes[tile] = tl;
      const std::uint32_t tc = cls_pair(ltot);
      tile_cls[tile] = (tc & 0xFFFFu) | (static_cast<std::uint64_t>(tc >> 16) << 32);
    }
  };
  if constexpr (kTileThreads == 512) {
    const std::uint32_t ntiles = static_cast<std::uint32_t>((static_cast<std::uint64_t>(n) + kScanTile - 1) / kScanTile);
    for (std::uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      tile_body(tile);
      __syncthreads();  // wsum, lsum and wok are rewritten by the next tile
    }
  } else {
    tile_body(blockIdx.x);
  }
}

// Scan of the tile sums for batches of more than kFusedTiles tiles (one workgroup), with the
// stream-mode verdict over all tiles: when every tile qualified, counts and s_info take stream mode's
// values (as stream_block does for fused batches) and rows_finish builds the block ends.
__device__ __forceinline__ StreamGeom stream_geometry(const std::uint8_t* base, const std::uint64_t* offsets,
                                                      const std::uint32_t* lengths, std::uint32_t n);
__device__ __forceinline__ void rows_scan_tiles_body(ScanLds& L, std::uint64_t* tile_sums, std::uint32_t* tile_lanes,
                                                     std::uint64_t* tile_cls, std::uint32_t ntiles, std::uint32_t n,
                                                     std::uint32_t* counts, const std::uint32_t* tile_ok,
                                                     const std::uint8_t* base, const std::uint64_t* offsets,
                                                     const std::uint32_t* lengths, std::uint64_t* sinfo) {
  std::uint64_t* part = L.part;
  std::uint64_t* cpart = L.cpart;
  std::uint32_t* lpart = L.lpart;
  std::uint32_t& sph = L.sph;
  if (threadIdx.x == 0) sph = 0;  // (the loop's first barrier orders this before the ORs below)
  std::uint64_t carry = 0, lcarry = 0, ccarry = 0;
  bool all_stream = true;
  std::uint32_t ph = 0;  // kTilePhases flags over the tiles
  for (std::uint32_t t0 = 0; t0 < ntiles; t0 += 1024) {
    const std::uint32_t i = t0 + threadIdx.x;
    all_stream = all_stream && (i >= ntiles || (tile_ok[i] & kTileStream) != 0);
    ph |= i < ntiles ? tile_ok[i] & kTilePhases : 0u;
    const std::uint64_t x = i < ntiles ? tile_sums[i] : 0ull;
    const std::uint32_t lx = i < ntiles ? tile_lanes[i] : 0u;
    const std::uint64_t cx = i < ntiles ? tile_cls[i] : 0ull;
    part[threadIdx.x] = x;
    lpart[threadIdx.x] = lx;
    cpart[threadIdx.x] = cx;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const std::uint64_t y = threadIdx.x >= static_cast<unsigned>(off) ? part[threadIdx.x - off] : 0ull;
      const std::uint32_t ly = threadIdx.x >= static_cast<unsigned>(off) ? lpart[threadIdx.x - off] : 0u;
      const std::uint64_t cy = threadIdx.x >= static_cast<unsigned>(off) ? cpart[threadIdx.x - off] : 0ull;
      __syncthreads();
      part[threadIdx.x] += y;
      lpart[threadIdx.x] += ly;
      cpart[threadIdx.x] += cy;
      __syncthreads();
    }
    if (i < ntiles) {
      tile_sums[i] = carry + part[threadIdx.x] - x;  // exclusive tile offsets
      tile_lanes[i] = static_cast<std::uint32_t>(lcarry + lpart[threadIdx.x] - lx);
      tile_cls[i] = ccarry + cpart[threadIdx.x] - cx;
    }
    const std::uint64_t tot = part[1023];
    const std::uint32_t ltot = lpart[1023];
    const std::uint64_t ctot = cpart[1023];
    __syncthreads();
    carry += tot;
    lcarry += ltot;
    ccarry += ctot;
  }
#pragma unroll
  for (unsigned m = 32; m > 0; m >>= 1) ph |= __shfl_xor(ph, m, 64);
  if ((threadIdx.x & 63u) == 0 && ph != 0) atomicOr(&sph, ph);
  const bool stream = __syncthreads_and(all_stream ? 1 : 0) != 0;
  if (threadIdx.x == 0) {
    counts[kCountPhases] = stream ? 0u : sph >> 1;
    if (stream) {
      const StreamGeom g = stream_geometry(base, offsets, lengths, n);
      counts[0] = 0;
      counts[1] = 0;
      counts[2] = static_cast<std::uint32_t>(g.rows);
      counts[3] = kModeStream;
      counts[kCountLanes] = 0;  // every block is longer than kLaneMax in stream mode
      counts[kCountSmall4] = 0;
      counts[kCountSmall8] = 0;
      sinfo[0] = g.zoff;
      sinfo[1] = g.s0rel;
      return;
    }
    const std::uint32_t ns = static_cast<std::uint32_t>(carry), nl = static_cast<std::uint32_t>(lcarry);
    counts[0] = n - ns - nl;                               // large blocks
    counts[1] = ns;                                        // small blocks
    counts[2] = static_cast<std::uint32_t>(carry >> 32);  // rows of the large blocks
    counts[3] = 0;                                         // general path
    counts[kCountLanes] = nl;                              // lane blocks
    counts[kCountSmall8] = static_cast<std::uint32_t>(ccarry);
    counts[kCountSmall4] = ns - static_cast<std::uint32_t>(ccarry) - static_cast<std::uint32_t>(ccarry >> 32);
  }
}
__global__ __launch_bounds__(1024) void rows_scan_tiles(std::uint64_t* tile_sums, std::uint32_t* tile_lanes,
                                                       std::uint64_t* tile_cls, std::uint32_t ntiles, std::uint32_t n, std::uint32_t* counts,
                                                       const std::uint32_t* tile_ok, const std::uint8_t* base,
                                                       const std::uint64_t* offsets, const std::uint32_t* lengths,
                                                       std::uint64_t* sinfo, const std::uint32_t* gate, std::uint32_t seq) {
  if (gate_closed(gate, seq)) return;
  __shared__ ScanLds L;
  rows_scan_tiles_body(L, tile_sums, tile_lanes, tile_cls, ntiles, n, counts, tile_ok, base, offsets, lengths, sinfo);
}

// Scatter of one block (rows_finish): e = its exclusive (small count, rows) pair, nlane = lane blocks
// and group blocks in front of it that those phases fold, tk = its tile's flags,
// TR = rows of all large blocks. A large block cut between row-kernel waves gets its
// result zeroed here, since the row kernel XORs every piece of it into the result (crc_rows_body,
// irregular batches). len and off are the block's length and offset (loaded by the caller).
__device__ __forceinline__ void finish_block(std::uint64_t off, std::uint32_t len, std::uint64_t b, std::uint64_t e,
                                             std::uint64_t nlane, std::uint64_t cpre, std::uint32_t n4,
                                             std::uint32_t n8, std::uint64_t TR, const PrepassOut& o,
                                             std::uint32_t W, std::uint32_t* out, std::uint32_t tk) {
  if (phase_block(len, tk)) return;  // the lane or group phase's (in a sparse tile it is small)
  const std::uint32_t nsmall = static_cast<std::uint32_t>(e);
  if (len <= kSmallMax) {
    // class lists one after the other: [0, n4) up to kGroupMax bytes, then n8 up to kGroup8Max, then the rest
    const std::uint32_t c8 = static_cast<std::uint32_t>(cpre), c16 = static_cast<std::uint32_t>(cpre >> 32);
    const std::uint32_t pos = len <= kGroupMax ? nsmall - c8 - c16 : len <= kGroup8Max ? n4 + c8 : n4 + n8 + c16;
    o.s_off[pos] = off;
    o.s_len[pos] = len;
    o.s_idx[pos] = static_cast<std::uint32_t>(b);
    return;
  }
  const std::uint32_t k = static_cast<std::uint32_t>(b - nsmall - nlane);  // compacted index
  const std::uint64_t lo = e >> 32;
  o.big_off[k] = off;
  o.big_len[k] = len;
  o.big_idx[k] = static_cast<std::uint32_t>(b);
  o.row_scan[k] = static_cast<std::uint32_t>(lo);
  const std::uint64_t hi = lo + rows_for_len(len);
  // waves whose first row g0(w) = floor(w*TR/W) lies in [lo, hi): w in [ceil(lo*W/TR), ceil(hi*W/TR))
  const std::uint64_t wlo = (lo * W + TR - 1) / TR;
  const std::uint64_t whi = (hi * W + TR - 1) / TR;
  for (std::uint64_t w = wlo; w < whi && w < W; ++w) o.wave_start[w] = k;
  // cut iff some wave starts strictly inside the block (g0 is nondecreasing in w)
  if (whi > wlo && (whi - 1) * TR / W > lo) out[b] = 0u;
}

__device__ __forceinline__ void stream_block(const std::uint8_t* base, const std::uint64_t* offsets,
                                             const std::uint32_t* lengths, std::uint32_t n, std::uint64_t b,
                                             std::uint64_t off, std::uint32_t len, std::uint32_t W,
                                             const std::uint32_t* row0, std::uint32_t* counts, std::uint64_t* ends,
                                             std::uint64_t* sinfo, std::uint32_t* wave_start);
__global__ void rows_finish(const std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                            std::uint32_t n, const std::uint64_t* scan, const std::uint64_t* tile_offs,
                            std::uint32_t* counts, const std::uint32_t* tile_ok, PrepassOut o, std::uint32_t W,
                            std::uint32_t* out, std::uint64_t* ends, std::uint64_t* sinfo, std::uint32_t Ws,
                            const std::uint32_t* row0, const std::uint32_t* gate, std::uint32_t seq) {
  if (gate_closed(gate, seq)) return;
  const bool stream = dev::sload32(counts, 3) == kModeStream;  // rows_scan_tiles found every tile back to back
  const std::uint32_t nchunks = static_cast<std::uint32_t>((static_cast<std::uint64_t>(n) + 255u) / 256u);
  for (std::uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const std::uint64_t b = c * static_cast<std::uint64_t>(256) + threadIdx.x;
    if (b >= n) continue;
    // (256-block chunks: a chunk lies in one scan tile, so its flags are one scalar load)
    const std::uint64_t t = b / kScanTile;
    const std::uint32_t tk = stream ? 0u : dev::sload32(tile_ok, static_cast<std::uint32_t>(c / (kScanTile / 256u)));
    if (tk & kTileAllTaken) continue;  // every block of the tile is the lane or a group phase's: nothing to list
    const std::uint32_t len = lengths[b];
    if (stream) {
      stream_block(base, offsets, lengths, n, b, offsets[b], len, Ws, row0, counts, ends, sinfo, o.wave_start);
      continue;
    }
    if (phase_block(len, tk)) continue;  // the lane or group phase's
    const std::uint32_t cs = o.cscan[b];
    const std::uint64_t cpre = o.tile_cls[t] + (cs & 0xFFFFu) + (static_cast<std::uint64_t>(cs >> 16) << 32);
    finish_block(offsets[b], len, b, scan[b] + tile_offs[t], o.lscan[b] + o.tile_lanes[t], cpre,
                 dev::sload32(counts, kCountSmall4), dev::sload32(counts, kCountSmall8), counts[2], o, W, out, tk);
  }
}

// rows_finish with the scan of the tile sums folded in (ntiles <= kFusedFinishTiles): every workgroup sums
// the tile sums in front of its own tile and over all tiles itself (at most 4 loads per thread), so
// no single-workgroup tile-scan launch sits between the tile scan and the scatter. Workgroup 0
// publishes counts for the row kernel.
constexpr std::uint32_t kFusedTiles = 1024;
// The fused scatter re-reads every tile sum in each of its workgroups, so its cost grows with the
// tile count: above kFusedFinishTiles tiles the one-workgroup scan (rows_scan_tiles) and the plain
// scatter measured faster (one process, profiles/r5/scatter/: 300-1000 B gapped 3116 -> 3224-3334
// GB/s, 180-400 B 2549 -> 2650, 257-512 B 2879 -> 3480; cfg4's 32 tiles keep the fused kernel).
constexpr std::uint32_t kFusedFinishTiles = 128;
// Batches of at most kFusedTiles tiles: every scatter workgroup sums the tile sums itself. (Letting
// the tile scan's last workgroup scan them measured far slower in one process: 300-1000 B gapped
// 3041 -> 1934 GB/s, cfg4 -2 %, profiles/r4/s14/, most likely from the device-scope fence each
// tile-scan workgroup needs before its ticket.) A 256-thread workgroup per 256 blocks, each re-reading
// all tile sums: one 1024-thread workgroup per scan tile with 4 blocks per thread cuts those re-reads
// by 16 but measured slower (300-1000 B gapped 3210 -> 2929 GB/s, profiles/r4/s7/): the scatter's
// latency, not the re-reads, is what the finish pays for.
constexpr std::uint32_t kFinishPer = 1;
constexpr std::uint32_t kFinishThreads = 256;
constexpr std::uint32_t kFinishGroupsPerCu = 16;  // rows_finish
// Stream mode (every tile qualified): instead of the small/large lists, every block
// gets its end E[b] in bytes from row 0 (the stream start rounded down to 16 bytes), and every
// row-kernel wave the first block ending in or after its first row; counts = {0, 0, rows, 1} and
// s_info = {row 0's offset from base, stream start within row 0}.
__device__ __forceinline__ void stream_block(const std::uint8_t* base, const std::uint64_t* offsets,
                                             const std::uint32_t* lengths, std::uint32_t n, std::uint64_t b,
                                             std::uint64_t off, std::uint32_t len, std::uint32_t W,
                                             const std::uint32_t* row0, std::uint32_t* counts, std::uint64_t* ends,
                                             std::uint64_t* sinfo, std::uint32_t* wave_start) {
  const StreamGeom g = stream_geometry(base, offsets, lengths, n);
  if (b == 0) {
    counts[0] = 0;
    counts[1] = 0;
    counts[2] = static_cast<std::uint32_t>(g.rows);
    counts[3] = kModeStream;
    counts[kCountLanes] = 0;  // every block is longer than kLaneMax in stream mode
    counts[kCountSmall4] = 0;
    counts[kCountSmall8] = 0;
    sinfo[0] = g.zoff;
    sinfo[1] = g.s0rel;
  }
  const std::uint64_t e = off + len - g.zoff;
  ends[b] = e;
  // waves whose first row lies in (row of the previous end, row of this end]
  const std::uint64_t rb1 = (e - 1) / kRow + 1;                   // row of this end, plus one
  const std::uint64_t rp1 = b == 0 ? 0 : (e - len - 1) / kRow + 1;  // same for the previous end
  for (std::uint32_t w = dev::stream_first_wave(row0, rp1, W); w < W && row0[w] < rb1; ++w)
    wave_start[w] = static_cast<std::uint32_t>(b);
}

template <unsigned T, unsigned PER>
__global__ __launch_bounds__(T) void rows_finish_fused(
    const std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths, std::uint32_t n,
    const std::uint64_t* scan, const std::uint64_t* tile_sums, const std::uint32_t* tile_ok, std::uint32_t ntiles,
    std::uint32_t* counts, PrepassOut o, std::uint32_t W, std::uint32_t* out, std::uint64_t* ends,
    std::uint64_t* sinfo, std::uint32_t Ws, const std::uint32_t* row0, const std::uint32_t* gate, std::uint32_t seq) {
  if (gate_closed(gate, seq)) return;
  static_assert(kScanTile % (T * PER) == 0 && T % 64 == 0, "a workgroup lies in one scan tile");
  constexpr std::uint32_t kWaves = T / 64;
  __shared__ std::uint64_t red[8][kWaves];
  const std::uint32_t my_tile = blockIdx.x * (T * PER) / kScanTile;
  // The workgroup's own operands are loaded first, so their latency overlaps the tile-sum reduction
  // (the scan values of a lane block were never written and are not used).
  const std::uint64_t b0 = blockIdx.x * static_cast<std::uint64_t>(T * PER) + threadIdx.x;
  std::uint32_t len[PER], lsc[PER], csc[PER];
  std::uint64_t off[PER], sc[PER];
#pragma unroll
  for (unsigned r = 0; r < PER; ++r) {
    const std::uint64_t b = b0 + r * T;
    const bool live = b < n;
    len[r] = live ? lengths[b] : 0u;
    off[r] = live ? offsets[b] : 0ull;
    sc[r] = live ? scan[b] : 0ull;
    lsc[r] = live ? o.lscan[b] : 0u;
    csc[r] = live ? o.cscan[b] : 0u;
  }
  const std::uint32_t mtk = tile_ok[my_tile];
  std::uint64_t before = 0, all = 0, bad = 0, lbefore = 0, lall = 0, cbefore = 0, call = 0;
  std::uint32_t ph = 0;  // kTilePhases flags over the tiles
  for (std::uint32_t i = threadIdx.x; i < ntiles; i += T) {
    const std::uint64_t v = tile_sums[i];
    const std::uint64_t lv = o.tile_lanes[i];
    const std::uint64_t cv = o.tile_cls[i];
    const std::uint32_t tk = tile_ok[i];
    all += v;
    before += i < my_tile ? v : 0ull;
    lall += lv;
    lbefore += i < my_tile ? lv : 0ull;
    call += cv;
    cbefore += i < my_tile ? cv : 0ull;
    bad += (tk & kTileStream) ? 0u : 1u;
    ph |= tk & kTilePhases;
  }
  // Wave sums by cross-lane exchange, then the kWaves partial sums through LDS (one barrier).
#pragma unroll
  for (unsigned m = 32; m > 0; m >>= 1) {
    before += __shfl_xor(before, m, 64);
    all += __shfl_xor(all, m, 64);
    bad += __shfl_xor(bad, m, 64);
    lbefore += __shfl_xor(lbefore, m, 64);
    lall += __shfl_xor(lall, m, 64);
    cbefore += __shfl_xor(cbefore, m, 64);
    call += __shfl_xor(call, m, 64);
    ph |= __shfl_xor(ph, m, 64);
  }
  const unsigned wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 0) {
    red[0][wid] = before;
    red[1][wid] = all;
    red[2][wid] = bad;
    red[3][wid] = lbefore;
    red[4][wid] = lall;
    red[5][wid] = ph;
    red[6][wid] = cbefore;
    red[7][wid] = call;
  }
  __syncthreads();
  std::uint64_t tile_off = 0, total = 0, nbad = 0, tile_loff = 0, ltotal = 0, aph = 0, tile_coff = 0, ctotal = 0;
#pragma unroll
  for (unsigned w = 0; w < kWaves; ++w) {
    tile_off += red[0][w];
    total += red[1][w];
    nbad += red[2][w];
    tile_loff += red[3][w];
    ltotal += red[4][w];
    aph |= red[5][w];
    tile_coff += red[6][w];
    ctotal += red[7][w];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) counts[kCountPhases] = nbad == 0 ? 0u : static_cast<std::uint32_t>(aph) >> 1;
  if (nbad == 0) {  // every block qualifies: stream mode
#pragma unroll
    for (unsigned r = 0; r < PER; ++r) {
      const std::uint64_t b = b0 + r * T;
      if (b < n) stream_block(base, offsets, lengths, n, b, off[r], len[r], Ws, row0, counts, ends, sinfo, o.wave_start);
    }
    return;
  }
  const std::uint32_t n8 = static_cast<std::uint32_t>(ctotal);
  const std::uint32_t n4 = static_cast<std::uint32_t>(total) - n8 - static_cast<std::uint32_t>(ctotal >> 32);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const std::uint32_t ns = static_cast<std::uint32_t>(total), nl = static_cast<std::uint32_t>(ltotal);
    counts[0] = n - ns - nl;                               // large blocks
    counts[1] = ns;                                        // small blocks
    counts[2] = static_cast<std::uint32_t>(total >> 32);  // rows of the large blocks
    counts[3] = 0;                                         // general path
    counts[kCountLanes] = nl;                              // lane blocks (crc_stream's lane phase)
    counts[kCountSmall4] = n4;
    counts[kCountSmall8] = n8;
  }
#pragma unroll
  for (unsigned r = 0; r < PER; ++r) {
    const std::uint64_t b = b0 + r * T;
    if (b >= n) break;
    const std::uint64_t cpre = tile_coff + (csc[r] & 0xFFFFu) + (static_cast<std::uint64_t>(csc[r] >> 16) << 32);
    finish_block(off[r], len[r], b, sc[r] + tile_off, lsc[r] + tile_loff, cpre, n4, n8, total >> 32, o, W, out, mtk);
  }
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

// Short host spans (crc32::update of one WAL record, wal.cpp:54-57, or a small group commit of a
// few records): one workgroup of kSpanThreads per span of at most kSpanMax bytes, read from mapped
// pinned memory at a 16-byte aligned position. Thread i folds dwords [i*per, (i+1)*per) from a
// zero register with slicing-by-4 lookups into one copy of the tables in LDS (bytes past the
// span's end in its last dword by Sarwate steps), moves its partial past the bytes that follow its
// segment (one GF(2) multiply by x^(8d)), and the XOR of all partials plus Shift_len(init) is the
// new raw register (crc_s(D) = Shift_|D|(s) ^ crc_0(D)). Thread 0 writes register ^ out_xor to
// out[b] (mapped host memory) and counts the span done on a device-memory counter (release at
// system scope, so the result has reached the host first); the workgroup that completes the count
// (counter value base + n - 1: the counter only grows, the host tracks base) writes `seq` to *done in
// host memory, which the host polls. One PCIe write per launch: a count kept in host memory took
// one serialized PCIe atomic per span (256 spans: 263 us). The row kernels would fill 160 KiB of LDS
// per workgroup and need a seam fix-up launch; this is one small launch. One span travels in the
// kernel arguments (desc == nullptr), more in a descriptor array in mapped memory.
constexpr unsigned kSpanThreads = 256;
constexpr std::uint32_t kSpanMax = 16u << 10;  // 16 dwords per thread at most
__device__ __forceinline__ std::uint32_t span_x8n(const DeviceTables* t, std::uint32_t d) {  // d < 2^24
  return dev::multmodp(t->rows_shift[d >> 12], t->head_shift[d & 4095u][31], t->poly);
}
__global__ __launch_bounds__(kSpanThreads) void crc_span(const std::uint8_t* stage, SpanDesc one, const SpanDesc* desc,
                                                          std::uint32_t out_xor, std::uint32_t* out, std::uint32_t* count,
                                                          std::uint32_t base, std::uint32_t* done, std::uint32_t seq,
                                                          const DeviceTables* t) {
  __shared__ std::uint32_t tb[4 * 256];
  __shared__ std::uint32_t part[kSpanThreads / 64];
  const SpanDesc sd = desc ? desc[blockIdx.x] : one;
  const std::uint32_t len = sd.len;
  const std::uint32_t nd = (len + 3u) / 4u;                           // dwords, the last may be partial
  const std::uint32_t per = (nd + kSpanThreads - 1u) / kSpanThreads;  // <= 16
  const std::uint32_t d0 = threadIdx.x * per;
  const std::uint32_t d1 = d0 + per < nd ? d0 + per : nd;
  const std::uint32_t* src = reinterpret_cast<const std::uint32_t*>(stage + sd.pos);
  std::uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = d0 + i < d1 ? src[d0 + i] : 0u;  // all loads issued before the fold
  for (std::uint32_t u = threadIdx.x; u < 1024u; u += kSpanThreads) tb[u] = t->slice[u >> 8][u & 255u];
  const std::uint32_t b1 = 4u * d1 < len ? 4u * d1 : len;  // end of this thread's bytes
  const std::uint32_t shift = span_x8n(t, len - b1);        // independent of the data: overlaps the loads
  __syncthreads();
  std::uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const std::uint32_t d = d0 + i;
    if (d < d1) {
      if (4u * d + 4u <= len) {
        const std::uint32_t x = c ^ w[i];
        c = tb[768u + (x & 255u)] ^ tb[512u + ((x >> 8) & 255u)] ^ tb[256u + ((x >> 16) & 255u)] ^ tb[x >> 24];
      } else {
        for (std::uint32_t k = 0; 4u * d + k < len; ++k) c = (c >> 8) ^ tb[(c ^ (w[i] >> (8u * k))) & 255u];
      }
    }
  }
  std::uint32_t v = d0 < d1 ? dev::multmodp(c, shift, t->poly) : 0u;
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v ^= __shfl_xor(v, m, 64);
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    std::uint32_t r = dev::multmodp(sd.init, span_x8n(t, len), t->poly);
#pragma unroll
    for (unsigned k = 0; k < kSpanThreads / 64; ++k) r ^= part[k];
    out[blockIdx.x] = r ^ out_xor;
    if (gridDim.x == 1u) {  // one span (update()): no count to keep
      __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      const std::uint32_t old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old == base + gridDim.x - 1u) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// SSTable stamp fix-up (tkv_sst_block_crcs_device): out[i] holds the CRC of image i as it lies, with
// whatever its crc32_ field holds (bytes [17, 21)). By linearity, the CRC with those bytes read as
// zero is out[i] ^ crc_0(E), E = the field bytes followed by size-21 zero bytes, and
// crc_0(E) = Shift_{size-21}(crc_0(field)). One thread per image; store != 0 writes the result into
// the field. Images shorter than kSstMinImage keep the CRC of the image as it lies.
constexpr std::uint32_t kSstCrcOffset = 17, kSstMinImage = 22;
__global__ void sst_fix(std::uint8_t* file, const std::uint64_t* offsets, const std::uint32_t* sizes,
                        std::uint32_t* out, std::uint64_t n, int store, const DeviceTables* tabs) {
  const std::uint64_t i = blockIdx.x * static_cast<std::uint64_t>(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  const std::uint32_t size = sizes[i];
  if (size < kSstMinImage) return;
  std::uint8_t* f = file + offsets[i] + kSstCrcOffset;
  std::uint32_t c = 0;  // crc_0 of the 4 field bytes (Sarwate steps, crc32.cpp:12-14 without init)
  for (int k = 0; k < 4; ++k) c = (c >> 8) ^ tabs->slice[0][(c ^ f[k]) & 0xFFu];
  const std::uint32_t z = size - (kSstCrcOffset + 4);  // zero bytes after the field
  const std::uint32_t h = z % kRow;
  std::uint32_t c2 = 0;
  for (int b = 0; b < 32; ++b)
    if (c >> b & 1u) c2 ^= tabs->head_shift[h][b];  // Shift_h(c)
  const std::uint32_t v = out[i] ^ dev::shift_rows(tabs, c2, z / kRow);
  out[i] = v;
  if (store)
    for (int k = 0; k < 4; ++k) f[k] = static_cast<std::uint8_t>(v >> (8 * k));
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
std::uint64_t prepass_tiles(std::uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t launch_rows(const RowsArgs& a, bool aligned, bool uniform, unsigned grid, hipStream_t st) {
  if (uniform) {
    if (aligned) hipLaunchKernelGGL((crc_rows<true, true>), dim3(grid), dim3(kRowsThreads), 0, st, a);
    else hipLaunchKernelGGL((crc_rows<false, true>), dim3(grid), dim3(kRowsThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((crc_rows<false, false>), dim3(grid), dim3(kRowsThreads), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_packed(const RowsArgs& a, unsigned grid, hipStream_t st) {
  if (a.len == kRow) hipLaunchKernelGGL(crc_packed<true>, dim3(grid), dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL(crc_packed<false>, dim3(grid), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

// Lanes per block of crc_packed_small: G with len = 64 G, a power of two up to 32 (0: not this
// kernel's batch. Other multiples of 16 up to 2 KiB, right-aligned in 64 G-byte slots with zeros in
// front, measured 6-10 % faster through crc_packed_small_gen, profiles/r6/small_uniform/lens.jsonl;
// between 2 and 4 KiB a slot is a whole 4 KiB row and the generic kernel measured faster,
// profiles/r2/packed_small/ab_slots.jsonl).
std::uint32_t packed_small_group(std::uint32_t len) {
  for (std::uint32_t g = 1; g <= 32u; g <<= 1)
    if (len == 64u * g) return g;
  return 0;
}

template <int G>
void launch_small_g(const RowsArgs& a, unsigned grid, hipStream_t st) {
  hipLaunchKernelGGL((crc_packed_small<G>), dim3(grid), dim3(kThreads), 0, st, a);
}

hipError_t launch_packed_small(const RowsArgs& a, unsigned grid, hipStream_t st) {
  switch (packed_small_group(a.len)) {
    case 1: launch_small_g<1>(a, grid, st); break;
    case 2: launch_small_g<2>(a, grid, st); break;
    case 4: launch_small_g<4>(a, grid, st); break;
    case 8: launch_small_g<8>(a, grid, st); break;
    case 16: launch_small_g<16>(a, grid, st); break;
    case 32: launch_small_g<32>(a, grid, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Lanes per block of crc_packed_small_gen: the smallest power of two G >= 2 with 64 G >= len, for
// 64 < len <= 2 KiB (0 otherwise).
std::uint32_t packed_small_gen_group(std::uint32_t len) {
  if (len <= kLaneMax || len > 2048u) return 0;
  std::uint32_t g = 2;
  while (64u * g < len) g <<= 1;
  return g;
}

template <int G>
void launch_small_gen_g(const RowsArgs& a, unsigned grid, hipStream_t st) {
  if (a.init_raw) hipLaunchKernelGGL((crc_packed_small_gen<G, true>), dim3(grid), dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL((crc_packed_small_gen<G, false>), dim3(grid), dim3(kThreads), 0, st, a);
}

hipError_t launch_packed_small_gen(const RowsArgs& a, unsigned grid, hipStream_t st) {
  switch (packed_small_gen_group(a.len)) {
    case 2: launch_small_gen_g<2>(a, grid, st); break;
    case 4: launch_small_gen_g<4>(a, grid, st); break;
    case 8: launch_small_gen_g<8>(a, grid, st); break;
    case 16: launch_small_gen_g<16>(a, grid, st); break;
    case 32: launch_small_gen_g<32>(a, grid, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Uniform lane-block batch (a.len <= kLaneMax): ALIGN from the base pointer and the stride.
template <int ALIGN, int NG>
void launch_lanes_shape(RowsArgs a, unsigned ncu, hipStream_t st) {
  const std::uint64_t steps = (static_cast<std::uint64_t>(a.nblocks) + 63u) / 64u;
  const std::uint64_t waves = kThreads / 64u;
  const std::uint64_t grid = std::max<std::uint64_t>(1, std::min<std::uint64_t>(ncu, (steps + waves - 1) / waves));
  a.nwaves = static_cast<std::uint32_t>(grid * waves);
  hipLaunchKernelGGL((crc_lanes_n<ALIGN, NG>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, st, a);
}

template <int ALIGN, int NF>
void launch_lanes_r_nf(RowsArgs a, unsigned ncu, hipStream_t st) {
  const std::uint64_t steps = (static_cast<std::uint64_t>(a.nblocks) + 63u) / 64u;
  const std::uint64_t waves = kThreads / 64u;
  const std::uint64_t grid = std::max<std::uint64_t>(1, std::min<std::uint64_t>(ncu, (steps + waves - 1) / waves));
  a.nwaves = static_cast<std::uint32_t>(grid * waves);
  hipLaunchKernelGGL((crc_lanes_r<ALIGN, NF>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, st, a);
}
template <int ALIGN, int NF = 1>
void launch_lanes_r(const RowsArgs& a, std::uint32_t nf, unsigned ncu, hipStream_t st) {
  if constexpr (NF < 16) {
    if (nf != NF) {
      launch_lanes_r<ALIGN, NF + 1>(a, nf, ncu, st);
      return;
    }
  }
  launch_lanes_r_nf<ALIGN, NF>(a, ncu, st);
}

// Uniform lane-block batch (a.len <= kLaneMax): ALIGN from the base pointer and the stride, the window
// (NG granules) from the length.
hipError_t launch_lanes(const RowsArgs& a, unsigned ncu, hipStream_t st) {
  if (a.len > kLaneMax) return hipErrorInvalidValue;
  const std::uintptr_t m = reinterpret_cast<std::uintptr_t>(a.base) | static_cast<std::uintptr_t>(a.stride);
  const int align = (m & 15u) == 0 ? 16 : (m & 3u) == 0 ? 4 : 1;
  // lengths that are not whole dwords, default register: right-aligned windows (crc_lanes_r_body, whose
  // window start is then never dword-aligned). In one process against crc_lanes_n
  // (profiles/r4/lanes_r/): 59 B +8.6 %, 59 B at stride 67 +5.2 %, 26 B +0.1 %; lengths of whole
  // dwords (no Sarwate tail to save) measured 3 % slower at 16 and 48 B and keep crc_lanes_n.
  const std::uint32_t nf = (a.len + 3u) / 4u, lead = 4u * nf - a.len;
  const bool lanes_r = a.init_raw == nullptr && lead != 0u;
  const std::uint32_t mis = align == 16 ? 0u : align == 4 ? 12u : 15u;  // worst start offset in a granule
  const std::uint32_t ng = std::max<std::uint32_t>(1u, (a.len + mis + 15u) / 16u);  // granules a block can touch
  // a step's bytes fit one 3 KiB LDS buffer (the last lane's block, its alignment slack and the
  // realigning read's extra dword included) and the granule path would realign: stage through LDS.
  // In one process against crc_lanes_n (profiles/r4/lanes_lds/): 33 B +2.3 %, 36 B +0.7 %, 36 B at
  // base + 3 +5.3 %, 36 B stride 44 +1.3 %; 16-byte aligned blocks (no realignment to save) and blocks
  // under 28 bytes (a step copies more than it folds) measured slower and keep crc_lanes_n.
  if (a.init_raw == nullptr && align != 16 && a.len >= 28u && a.stride <= dev::kLanesLdsMaxStride &&
      15u + 63u * a.stride + a.len + 8u <= dev::kLanesLdsBuf) {
    const std::uint64_t steps = (static_cast<std::uint64_t>(a.nblocks) + 63u) / 64u;
    const std::uint64_t waves = kThreads / 64u;
    const std::uint64_t grid = std::max<std::uint64_t>(1, std::min<std::uint64_t>(ncu, (steps + waves - 1) / waves));
    RowsArgs b = a;
    b.nwaves = static_cast<std::uint32_t>(grid * waves);
    const dim3 g(static_cast<unsigned>(grid)), t(kThreads);
    const std::uint32_t nw = (a.len + 3u) / 4u;  // words to read (the tail's included)
    const std::uint32_t kb = (15u + 63u * a.stride + a.len + 8u + 1023u) / 1024u;  // KiB a step copies
#define TKV_LANES_LDS_KB(RA, NW)                                                             \
    if (kb <= 1) hipLaunchKernelGGL((crc_lanes_lds<RA, NW, 1>), g, t, 0, st, b);             \
    else if (kb == 2) hipLaunchKernelGGL((crc_lanes_lds<RA, NW, 2>), g, t, 0, st, b);        \
    else hipLaunchKernelGGL((crc_lanes_lds<RA, NW, 3>), g, t, 0, st, b);
#define TKV_LANES_LDS(RA)                                                                    \
    if (nw <= 4) { TKV_LANES_LDS_KB(RA, 4) }                                                \
    else if (nw <= 8) { TKV_LANES_LDS_KB(RA, 8) }                                           \
    else if (nw <= 12) { TKV_LANES_LDS_KB(RA, 12) }                                         \
    else { TKV_LANES_LDS_KB(RA, 16) }
    if (align == 1) { TKV_LANES_LDS(true) } else { TKV_LANES_LDS(false) }
#undef TKV_LANES_LDS
#undef TKV_LANES_LDS_KB
    return hipGetLastError();
  }
  if (lanes_r) {
    launch_lanes_r<1>(a, nf, ncu, st);
    return hipGetLastError();
  }
#define TKV_LANES_N(A)                                           \
  switch (ng) {                                                  \
    case 1: launch_lanes_shape<A, 1>(a, ncu, st); break;         \
    case 2: launch_lanes_shape<A, 2>(a, ncu, st); break;         \
    case 3: launch_lanes_shape<A, 3>(a, ncu, st); break;         \
    case 4: launch_lanes_shape<A, 4>(a, ncu, st); break;         \
    default: launch_lanes_shape<A, 5>(a, ncu, st); break;        \
  }
  if (align == 16) { TKV_LANES_N(16) }
  else if (align == 4) { TKV_LANES_N(4) }
  else { TKV_LANES_N(1) }
#undef TKV_LANES_N
  return hipGetLastError();
}

hipError_t launch_fixup(const RowsArgs& a, hipStream_t st) {
  const unsigned grid = (2u * a.nwaves + 255u) / 256u;  // one thread per seam record
  hipLaunchKernelGGL(crc_fixup, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

// Waves of crc_list_lanes for a batch of nblocks: one workgroup per CU (at most kListMaxGroups) or
// fewer when the 64-block steps run out (tkv_debug_list_lanes_waves reports it to the tests).
std::uint32_t list_lanes_waves(std::uint64_t nblocks, unsigned ncu) {
  const std::uint64_t steps = (nblocks + 63u) / 64u;
  const std::uint64_t grid = std::max<std::uint64_t>(
      1, std::min<std::uint64_t>(std::min<std::uint64_t>(ncu, kListMaxGroups), (steps + kListWaves - 1) / kListWaves));
  return static_cast<std::uint32_t>(grid * kListWaves);
}

// One-pass lane kernel of an irregular batch (default initial register): see crc_list_lanes.
hipError_t launch_list_lanes(const RowsArgs& a, unsigned ncu, hipStream_t st) {
  RowsArgs b = a;
  b.nwaves = list_lanes_waves(a.nblocks, ncu);
  const std::uint64_t grid = b.nwaves / kListWaves;
  hipLaunchKernelGGL(crc_list_lanes, dim3(static_cast<unsigned>(grid)), dim3(kListThreads), 0, st, b);
  return hipGetLastError();
}

hipError_t launch_prepass(const std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                          std::uint32_t n, std::uint64_t* scan, std::uint64_t* tile_sums, std::uint32_t* tile_ok,
                          std::uint32_t* counts, std::uint64_t* sinfo, std::uint64_t* ends, const PrepassOut& o,
                          std::uint32_t W, std::uint32_t ncu, std::uint32_t* out, std::uint32_t* row0,
                          std::uint32_t group_stream, const std::uint32_t* gate, std::uint32_t seq,
                          const std::uint32_t* gate_flags, hipStream_t st) {
  const std::uint32_t Ws = ncu * (kStreamThreads / 64);  // crc_stream's waves
  // Grid sizes in 64-bit arithmetic: n may be close to 2^32 (the host caps it at kMaxIrregularBlocks).
  const std::uint64_t ntiles = prepass_tiles(n);
  const std::uint64_t nfused = (static_cast<std::uint64_t>(n) + kFinishThreads * kFinishPer - 1) / (kFinishThreads * kFinishPer);
  const std::uint64_t nfinish = (static_cast<std::uint64_t>(n) + 255) / 256;
  // batches of more than kFusedTiles tiles: at most kScanGroupsPerCu tile-scan workgroups per CU, each
  // looping over tiles: against one workgroup per tile, gapped 36-byte WAL payloads 2567 -> 2625 GB/s,
  // back-to-back 36 B 2933 -> 3018, the rest within noise (4 or 8 per CU measured the same or lower;
  // profiles/r5/scatter/)
  const std::uint64_t scap = std::uint64_t(ncu) * kScanGroupsPerCu;
  const unsigned gscan = static_cast<unsigned>(ntiles < scap ? ntiles : scap);
  if (ntiles <= kFusedTiles)
    hipLaunchKernelGGL(rows_tile_scan<1024>, dim3(static_cast<unsigned>(ntiles)), dim3(1024), 0, st, base, offsets,
                       lengths, n, scan, tile_sums, tile_ok, row0, Ws, o.lscan, o.tile_lanes, o.cscan, o.tile_cls,
                       group_stream, gate, seq, gate_flags);
  else
    hipLaunchKernelGGL(rows_tile_scan<512>, dim3(gscan), dim3(512), 0, st, base, offsets,
                       lengths, n, scan, tile_sums, tile_ok, row0, Ws, o.lscan, o.tile_lanes, o.cscan, o.tile_cls,
                       group_stream, gate, seq, gate_flags);
  if (ntiles <= kFusedFinishTiles) {
    hipLaunchKernelGGL((rows_finish_fused<kFinishThreads, kFinishPer>), dim3(static_cast<unsigned>(nfused)), dim3(kFinishThreads), 0, st, base,
                       offsets, lengths, n, scan, tile_sums, tile_ok, static_cast<std::uint32_t>(ntiles), counts, o,
                       W, out, ends, sinfo, Ws, row0, gate, seq);
  } else {
    hipLaunchKernelGGL(rows_scan_tiles, dim3(1), dim3(1024), 0, st, tile_sums, o.tile_lanes, o.tile_cls,
                       static_cast<std::uint32_t>(ntiles), n, counts, tile_ok, base, offsets, lengths, sinfo, gate, seq);
    // at most kFinishGroupsPerCu workgroups per CU, each looping over 256-block chunks: a batch whose
    // gate stays closed (crc_list_lanes folded it) no longer dispatches one workgroup per 256 blocks
    // (gapped 36-byte WAL payloads 2441 -> 2555 GB/s, back-to-back 36 B 2755 -> 2973;
    // profiles/r5/scatter/)
    const std::uint64_t gcap = std::uint64_t(ncu) * kFinishGroupsPerCu;
    hipLaunchKernelGGL(rows_finish, dim3(static_cast<unsigned>(nfinish < gcap ? nfinish : gcap)), dim3(256), 0, st, base, offsets, lengths,
                       n, scan, tile_sums, counts, tile_ok, o, W, out, ends, sinfo, Ws, row0, gate, seq);
  }
  return hipGetLastError();
}


// Stream-mode row walk of an irregular batch (returns at once unless the prepass chose stream mode);
// launched before crc_rows<false, false>, which finishes the block CRCs.
hipError_t launch_stream_rows(const RowsArgs& a, hipStream_t st, unsigned grid) {
  RowsArgs b = a;
  b.nwaves = grid * (kStreamThreads / 64);
  hipLaunchKernelGGL(crc_stream, dim3(grid), dim3(kStreamThreads), 0, st, b);
  return hipGetLastError();
}

hipError_t launch_span(const std::uint8_t* stage, const SpanDesc& one, const SpanDesc* desc, std::uint32_t n,
                       std::uint32_t out_xor, std::uint32_t* out, std::uint32_t* count, std::uint32_t base,
                       std::uint32_t* done, std::uint32_t seq, const DeviceTables* tabs, hipStream_t st) {
  if (n == 0 || (desc == nullptr && (n != 1 || one.len > kSpanMax || (one.pos & 15u))) ||
      (reinterpret_cast<std::uintptr_t>(stage) & 15u))
    return hipErrorInvalidValue;  // the host checks every descriptor's length and alignment
  hipLaunchKernelGGL(crc_span, dim3(n), dim3(kSpanThreads), 0, st, stage, one, desc, out_xor, out, count, base, done,
                     seq, tabs);
  return hipGetLastError();
}

hipError_t launch_sst_fix(std::uint8_t* file, const std::uint64_t* offsets, const std::uint32_t* sizes,
                          std::uint32_t* out, std::uint64_t n, int store, const DeviceTables* tabs, hipStream_t st) {
  const std::uint64_t grid = (n + 255) / 256;
  if (grid) hipLaunchKernelGGL(sst_fix, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, file, offsets, sizes, out,
                               n, store, tabs);
  return hipGetLastError();
}

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
