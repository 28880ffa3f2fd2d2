// Internal definitions shared by the CRC-32 kernels (tkv_crc32_kernels.hip) and the host runtime
// (tkv_crc32_host.cpp). Not part of the public C ABI (include/tkv_crc32.h).
#pragma once

#include <cstddef>
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define TKV_HD __host__ __device__
#else
#define TKV_HD
#endif

namespace tkv {

// CRC-32/ISO-HDLC parameters of frankie::core::crc32 (/root/reference/src/core/crc32.hpp:9-11).
constexpr std::uint32_t kPoly = 0xEDB88320u;  // reflected polynomial
constexpr std::uint32_t kInit = 0xFFFFFFFFu;  // init and xorout
// CRC-32C (Castagnoli, RFC 3720 §B.4): same reflection, init and xorout; SURVEY.md §8f rank 4.
constexpr std::uint32_t kPolyC = 0x82F63B78u;

// Checksum families the engine serves; each has its own DeviceTables on every device.
enum Algo : int { kAlgoCrc32 = 0, kAlgoCrc32c = 1, kNumAlgos = 2 };
constexpr std::uint32_t algo_poly(int algo) { return algo == kAlgoCrc32c ? kPolyC : kPoly; }

// Work decomposition of the row kernel.
constexpr int kSeg = 64;                 // contiguous bytes one lane folds per row
constexpr int kRow = 64 * kSeg;          // bytes one wave folds per row (4 KiB)
constexpr int kWavesPerWG = 16;          // packed kernel: 1024-thread workgroups, one per CU (LDS-bound)
constexpr int kThreads = 64 * kWavesPerWG;
constexpr int kRowsWavesPerWG = 12;      // generic row kernels: 768 threads (162 VGPRs at ILP 2)
constexpr int kRowsThreads = 64 * kRowsWavesPerWG;

// LDS image (160 KiB, one workgroup per CU):
//   words [0, 32768): slicing-by-4 tables T0..T3, each entry replicated 32x so lane c of every
//                     32-lane half reads bank c: byte address = pair*64K + e*256 + t*128 + c*4,
//                     table index = 2*pair + t.
//   words [32768, 40960): lane-shift nibble tables LS[j][v][lane] (j nibble, v value).
constexpr int kLdsSliceWords = 4 * 256 * 32;
constexpr int kLdsLaneWords = 8 * 16 * 64;
constexpr int kLdsWords = kLdsSliceWords + kLdsLaneWords;
constexpr std::uint32_t kLdsLaneBase = kLdsSliceWords * 4u;  // byte offset of LS in LDS

// Constant tables uploaded once per device (global memory, read by every workgroup prologue).
struct DeviceTables {
  std::uint32_t slice[4][256];          // slicing-by-4: T0 = Sarwate table, Tk[i] = Shift_1 o T(k-1)
  std::uint32_t lane_shift[8][16][64];  // LS[j][v][l] = Shift_{(63-l)*kSeg}(v << 4j)
  std::uint32_t horner[64];             // lanes 0..31: Shift_{kRow}(1 << l); lanes 32..63: 0
  std::uint32_t row_pow[64];            // x^(8*kRow*2^k) mod P (reflected), k = 0..63
  std::uint32_t head_shift[kRow + 1][32];  // [h][i] = Shift_h(1 << i): init injection at a head row
  std::uint32_t rows_shift[4096];       // [k] = x^(8*kRow*k) mod P: moves a piece's partial past k rows
  std::uint32_t inv_shift[kRow + 1];    // [d] = x^(-8d) mod P: moves a register back by d bytes (stream)
  std::uint32_t poly;                   // reflected polynomial the tables were built for
  std::uint32_t pad_[2];
  std::uint32_t init_shift[1024 + 1];   // [h] = Shift_h(0xFFFFFFFF): the init term of a group-walk block
};

// One partial result of a block that was split between waves (irregular / huge-block path).
struct Seam {
  std::uint64_t block;
  std::uint32_t partial;     // pure (init-0) CRC register of this wave's rows of the block
  std::uint32_t rows_after;  // rows of the block that follow this piece
  std::uint32_t flags;       // bit0 valid, bit1 piece contains row 0 (the block's head)
  std::uint32_t pad[3];
};
constexpr std::uint32_t kSeamValid = 1u;
constexpr std::uint32_t kSeamHasRow0 = 2u;

struct RowsArgs {
  const std::uint8_t* base;          // batch base pointer (device)
  const std::uint64_t* offsets;      // irregular: byte offset of block b from base
  const std::uint32_t* lengths;      // irregular: byte length of block b
  const std::uint32_t* row_scan;     // irregular: exclusive scan of rows(b); [nblocks] = total
  const std::uint32_t* wave_start;   // irregular: first block of wave w
  std::uint64_t stride;              // uniform: block b at base + b*stride
  std::uint32_t len;                 // uniform: every block's length
  std::uint32_t head_z;              // uniform: x^(8h) mod P, h = head-row length of every block
  const std::uint32_t* init_raw;     // nullable: per-block raw initial register
  std::uint32_t init_default;        // initial register when init_raw == nullptr (kInit)
  std::uint32_t out_xor;             // kInit: write finalize() values; 0: write raw registers
  std::uint32_t* out;                // per-block result
  Seam* seams;                       // 2 per wave
  const DeviceTables* tabs;
  const std::uint8_t* dummy;         // 256 zero bytes, target of loads outside any block
  std::uint32_t nblocks;
  std::uint32_t total_rows;          // uniform only (irregular reads row_scan[nblocks])
  std::uint32_t nwaves;
  std::uint32_t snap_blocks;         // uniform: partition by whole blocks (no seams)
  // irregular batches after the prepass split: `offsets`/`lengths` then list the
  // large blocks only (compacted), out_idx maps a compacted block to its batch index, and the small
  // blocks (len <= kSmallMax) are listed in s_off/s_len/s_idx for the small-block phase.
  const std::uint32_t* out_idx;      // nullable: result of compacted block k goes to out[out_idx[k]]
  const std::uint32_t* counts;       // device: [0] large blocks, [1] small blocks, [2] rows of large blocks
  const std::uint64_t* s_off;
  const std::uint32_t* s_len;
  const std::uint32_t* s_idx;
  // irregular batches in stream mode (counts[3] == kModeStream, chosen by the prepass: blocks back
  // to back, each at least kStreamMinLen bytes). Rows of 4 KiB cover the stream
  // from row 0 = the stream start rounded down to 16 bytes.
  const std::uint64_t* s_ends;       // E[b] = end of block b in bytes from row 0
  const std::uint64_t* s_info;       // [0] offset of row 0 from base, [1] stream start within row 0
  std::uint64_t* s_yq;               // per block: Y | Q << 32 at its end (crc_stream_body)
  std::uint32_t* s_wtot;             // per wave: crc_0 of its rows alone (crc_stream_body)
  const std::uint32_t* s_row0;       // [w] = first row of wave w, [nwaves] = rows (rows_tile_scan)
  std::uint32_t* s_wv;               // per block: the wave that met its end (crc_stream_body)
  // irregular batches: the caller's own arrays, which the lane phase walks (blocks of at most kLaneMax
  // bytes are in no prepass list; counts[kCountLanes] says how many there are)
  const std::uint64_t* l_off;
  const std::uint32_t* l_len;
  const std::uint32_t* l_tile;  // per scan tile of 4096 blocks: kTileLanes when its lane blocks are ours
  // irregular batches after crc_list_lanes (nullable): the kernels of the general path run only when
  // gate[0] == gate_seq, i.e. the one-pass kernel found a block it does not take
  const std::uint32_t* gate;
  std::uint32_t gate_seq;
  const std::uint32_t* gate_flags;  // crc_list_lanes: per workgroup, the call's number when it met such a block
};
// counts[kCountGate]: the call's sequence number when the general path must run (a block over
// kPackMax = 1 KiB): rows_tile_scan's workgroup 0 writes it from crc_list_lanes' per-workgroup flags
// (counts[kListFlags + g]; one writer per address: a single word written by every wave that met such
// a block took ~0.4 ms of same-address stores)
constexpr int kCountGate = 12;
constexpr int kListFlags = 64;
constexpr unsigned kListMaxGroups = 1024;
// counts[kPackFlags + g]: the call's sequence number when a wave of crc_list_lanes' workgroup g took its
// packed mode (blocks over kLaneMax bytes; tkv_debug_irregular_path)
constexpr int kPackFlags = kListFlags + static_cast<int>(kListMaxGroups);
constexpr int kCountWords = kPackFlags + static_cast<int>(kListMaxGroups);
__device__ __forceinline__ bool gate_closed(const std::uint32_t* gate, std::uint32_t seq) {
  return gate != nullptr && *gate != seq;
}
constexpr std::uint32_t kModeStream = 1;
// counts[] of an irregular batch: [0] large blocks, [1] small blocks, [2] rows of the large blocks,
// [3] mode, [4..7] stream-mode info (two u64), [8] lane and group blocks (len <= kGroupMax) of dense tiles
constexpr int kCountLanes = 8;
// counts[kCountPhases]: which of crc_stream's phases the general path needs (OR over the tiles'
// kTileLanes / kTileGroups / kTileGroups8, shifted down by 1): 1 = lane blocks, 2 / 4 = group blocks
// of 4- / 8-lane groups
constexpr int kCountPhases = 9;
// counts[kCountSmall4], counts[kCountSmall8]: listed small blocks of at most kGroupMax bytes (the first
// entries of s_off/s_len/s_idx) and of kGroupMax + 1 .. kGroup8Max bytes (the next ones); the rest of
// the counts[1] listed blocks (kGroup8Max + 1 .. kSmallMax bytes) follow them. The small-block phase
// folds each class with groups of 4, 8 or 16 lanes.
constexpr int kCountSmall4 = 10;
constexpr int kCountSmall8 = 11;

// Blocks of at most kLaneMax bytes are folded whole by one lane each, from their own initial register
// (DESIGN.md §4.5): uniform batches by crc_lanes, irregular ones by the lane phase in crc_stream's
// launch. The prepass lists them nowhere, and stream mode needs every block to be longer.
constexpr std::uint32_t kLaneMax = 64;
// Irregular blocks of kLaneMax + 1 .. kGroupMax bytes in dense tiles are folded by 4-lane groups (one
// block right-aligned in a 256-byte slot) in the group phase of crc_stream's launch, beside the lane
// phase; the prepass lists them nowhere either. Blocks of kGroupMax + 1 .. kGroup8Max
// bytes take 8-lane groups (512-byte slots) in a second pass of the group phase, over the tiles dense
// in them. (A 16-lane pass for 513-1024 B measured below the listed small phase, which folds those
// blocks in the same 1 KiB slots: 3292 against 3364 GB/s, profiles/r4/s1/probe_irregular.jsonl.)
constexpr std::uint32_t kGroupMax = 256;
constexpr std::uint32_t kGroup8Max = 512;
// The prepass leaves a scan tile's lane blocks to the lane phase only when the tile holds at least
// kLaneDenseTile of them (of its 4096), its 65-256-byte blocks to the 4-lane pass only when it holds
// at least kGroupDenseTile and its 257-512-byte blocks to the 8-lane pass only when nearly all its
// blocks are of that class; in other tiles they are listed as small blocks by class (4-, 8- and
// 16-lane groups in the small phase, the same slots). A pass walks the metadata of every block in its
// waves' ranges with the lanes of other classes idle, while listing costs a scatter per block: since
// the small phase folds each class at its own group size (round 4), a pass pays only in tiles almost
// all of its class. One process, 1 GiB gapped batches, against the round-4 start's 1024 / 2048
// (profiles/r4/group_policy/probe_thresholds.jsonl): 180-400 B 1832 -> 2612 GB/s, 100-700 B 2181 ->
// 2774, 200-700 B 2211 -> 2881; pure classes within noise (65-256 B 2948 / 2879, 257-512 B 3218 / 3156).
// The group phase also needs a tile with at most kGroupTileRows rows of large blocks (4 MiB): where
// large blocks carry the bytes, crc_rows folds the small blocks in the shadow of its row walk and the
// group phase's own latency chain (descriptor, data, fold: ~10 us) would only add to the batch
// (cfg4's general path: 1300 blocks of 255 bytes per tile, +1.2 % time with the group phase).
constexpr std::uint32_t kLaneDenseTile = 256;
constexpr std::uint32_t kGroupDenseTile = 3072;
// A back-to-back tile with at least this many blocks of at most kSmallMax bytes and at most
// kGroupTileRows rows of larger ones takes the general path, not stream mode (rows_tile_scan).
constexpr std::uint32_t kStreamSmallTile = 1024;
constexpr std::uint32_t kGroup8DenseTile = 3968;
constexpr std::uint64_t kGroupTileRows = 1024;
// Per-tile flags (tile_ok):
constexpr std::uint32_t kTileStream = 1u;     // the tile's blocks qualify for stream mode
constexpr std::uint32_t kTileLanes = 2u;      // the tile's lane blocks (len <= kLaneMax) are the lane phase's
constexpr std::uint32_t kTileGroups = 4u;     // its blocks of kLaneMax + 1 .. kGroupMax bytes the 4-lane pass's
constexpr std::uint32_t kTileGroups8 = 8u;    // kGroupMax + 1 .. kGroup8Max: the 8-lane pass's
constexpr std::uint32_t kTilePhases = kTileLanes | kTileGroups | kTileGroups8;
constexpr std::uint32_t kTileAllTaken = 32u;  // every block of the tile is a lane or group phase's: no scatter

// Whether block of length len in a tile with flags tk is folded by the lane or a group pass (and is
// in no prepass list).
__device__ __forceinline__ bool phase_block(std::uint32_t len, std::uint32_t tk) {
  return len <= kLaneMax     ? (tk & kTileLanes) != 0
         : len <= kGroupMax  ? (tk & kTileGroups) != 0
         : len <= kGroup8Max && (tk & kTileGroups8) != 0;
}

// One short host span for crc_span: `len` bytes at byte `pos` (16-byte aligned) of the mapped
// staging buffer, folded on from raw register `init`.
struct SpanDesc {
  std::uint32_t pos, len, init, pad;
};
constexpr std::uint32_t kStreamMinLen = kLaneMax + 1;  // at most one block end per 64-byte lane segment

// Outputs of the irregular prepass (scratch of one stream).
struct PrepassOut {
  std::uint64_t* s_off;
  std::uint32_t* s_len;
  std::uint32_t* s_idx;
  std::uint64_t* big_off;
  std::uint32_t* big_len;
  std::uint32_t* big_idx;
  std::uint32_t* row_scan;
  std::uint32_t* wave_start;
  std::uint32_t* lscan;       // per block: lane blocks in front of it (exclusive, within its tile)
  std::uint32_t* tile_lanes;  // per scan tile: its lane blocks (then their exclusive scan)
  // per block: listed blocks of kGroupMax + 1 .. kGroup8Max bytes in front of it (low half) and of
  // kGroup8Max + 1 .. kSmallMax bytes (high half), exclusive, within its tile
  std::uint32_t* cscan;
  std::uint64_t* tile_cls;    // per scan tile: the same two counts over the tile (low, high word), then scanned
};

// Blocks of at most kSmallMax bytes are listed by class (kCountSmall4) and folded by the small-block
// phase, a group of 4, 8 or 16 lanes (64 B each) per block, instead of occupying a whole 4 KiB row each.
constexpr std::uint32_t kSmallMax = 1024;

// Irregular batches carry u32 block indices (prepass scan, compacted lists, results): the host caps
// them below 2^32 with room for the prepass's tile rounding (4096 blocks per scan tile).
constexpr std::uint64_t kMaxIrregularBlocks = 0xFFFFFFFFull - 8192u;

// rows(b): wave-rows a block of n bytes occupies (every block, even n = 0, owns >= 1 row), and
// h(b): bytes of its head row (row 0), in [0, kRow].
TKV_HD inline std::uint32_t rows_for_len(std::uint32_t n) { return n == 0 ? 1u : (n - 1u) / kRow + 1u; }
TKV_HD inline std::uint32_t head_len(std::uint32_t n) { return n - (rows_for_len(n) - 1u) * kRow; }

// Host-side math shared with tests (tkv_crc32_host.cpp).
std::uint32_t multmodp(std::uint32_t a, std::uint32_t b, std::uint32_t poly = kPoly);  // a*b mod P
std::uint32_t x8nmodp(std::uint64_t nbytes, std::uint32_t poly = kPoly);              // x^(8n) mod P
std::uint32_t shift_bytes(std::uint32_t reg, std::uint64_t nbytes, std::uint32_t poly = kPoly);
void build_tables(DeviceTables* t, std::uint32_t poly = kPoly);

}  // namespace tkv
