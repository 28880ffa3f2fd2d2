// Host runtime of the MI355X CRC-32 engine: per-device contexts, the C ABI of include/tkv_crc32.h,
// the pinned-staging host pipeline, multi-GPU batch split and the WAL verify/stamp helpers.
// All checksum arithmetic runs in tkv_crc32_kernels.hip; this file only plans and launches it
// (the GF(2) helpers here build the constant tables and are exported for tests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "tkv_crc32.h"
#include "tkv_crc32_internal.h"
#include "tkv_engine.h"

namespace tkv {

// ---- launchers (tkv_crc32_kernels.hip) ---------------------------------------------------------
hipError_t launch_rows(const RowsArgs& a, bool aligned, bool uniform, unsigned grid, hipStream_t st);
hipError_t launch_fixup(const RowsArgs& a, hipStream_t st);
hipError_t launch_packed(const RowsArgs& a, unsigned grid, hipStream_t st);
std::uint32_t packed_small_group(std::uint32_t len);
hipError_t launch_packed_small(const RowsArgs& a, unsigned grid, hipStream_t st);
hipError_t launch_lanes(const RowsArgs& a, unsigned ncu, hipStream_t st);
std::uint32_t packed_small_gen_group(std::uint32_t len);
hipError_t launch_packed_small_gen(const RowsArgs& a, unsigned grid, hipStream_t st);
hipError_t launch_prepass(const std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                          std::uint32_t n, std::uint64_t* scan, std::uint64_t* tile_sums, std::uint32_t* tile_ok,
                          std::uint32_t* counts, std::uint64_t* sinfo, std::uint64_t* ends, const PrepassOut& o,
                          std::uint32_t W, std::uint32_t ncu, std::uint32_t* out, std::uint32_t* row0,
                          std::uint32_t group_stream, const std::uint32_t* gate, std::uint32_t seq,
                          const std::uint32_t* gate_flags, hipStream_t st);
hipError_t launch_stream_rows(const RowsArgs& a, hipStream_t st, unsigned grid);
hipError_t launch_list_lanes(const RowsArgs& a, unsigned ncu, hipStream_t st);
std::uint32_t list_lanes_waves(std::uint64_t nblocks, unsigned ncu);
std::uint64_t prepass_tiles(std::uint64_t n);
hipError_t launch_span(const std::uint8_t* stage, const SpanDesc& one, const SpanDesc* desc, std::uint32_t n,
                       std::uint32_t out_xor, std::uint32_t* out, std::uint32_t* count, std::uint32_t base,
                       std::uint32_t* done, std::uint32_t seq, const DeviceTables* tabs, hipStream_t st);
hipError_t launch_fill_uniform(std::uint8_t* dst, std::uint64_t stride, std::uint64_t len, std::uint64_t first,
                               std::uint64_t nblocks, std::uint64_t seed, hipStream_t st);
hipError_t launch_fill_blocks(std::uint8_t* base, const std::uint64_t* offsets, const std::uint32_t* lengths,
                              std::uint64_t first, std::uint64_t nblocks, std::uint64_t seed, hipStream_t st);

// ---- GF(2) arithmetic in the reflected representation (x^0 = 0x80000000) -------------------------
std::uint32_t multmodp(std::uint32_t a, std::uint32_t b, std::uint32_t poly) {
  std::uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ poly : (b >> 1);
  }
  return p;
}

std::uint32_t x8nmodp(std::uint64_t nbytes, std::uint32_t poly) {
  // x^(8n) = product over set bits k of n of x^(8*2^k); x^(8*2^k) by repeated squaring of x^8.
  std::uint32_t result = 0x80000000u;  // x^0
  std::uint32_t sq = 0x00800000u;      // x^8
  while (nbytes) {
    if (nbytes & 1u) result = multmodp(result, sq, poly);
    sq = multmodp(sq, sq, poly);
    nbytes >>= 1;
  }
  return result;
}

std::uint32_t shift_bytes(std::uint32_t reg, std::uint64_t nbytes, std::uint32_t poly) {
  return multmodp(x8nmodp(nbytes, poly), reg, poly);
}

void build_tables(DeviceTables* t, std::uint32_t poly) {
  // T0: the Sarwate table of crc32.hpp:16-30 (for poly = kPoly);
  // Tk[i] = T0[T(k-1)[i] & 0xFF] ^ (T(k-1)[i] >> 8).
  const auto mm = [poly](std::uint32_t a, std::uint32_t b) { return multmodp(a, b, poly); };
  const auto x8n = [poly](std::uint64_t n) { return x8nmodp(n, poly); };
  t->poly = poly;
  t->pad_[0] = t->pad_[1] = 0;
  for (std::uint32_t h = 0; h <= kSmallMax; ++h) t->init_shift[h] = mm(x8n(h), 0xFFFFFFFFu);
  for (std::uint32_t i = 0; i < 256; ++i) {
    std::uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? poly : 0u);
    t->slice[0][i] = c;
  }
  for (int k = 1; k < 4; ++k)
    for (std::uint32_t i = 0; i < 256; ++i)
      t->slice[k][i] = t->slice[0][t->slice[k - 1][i] & 0xFFu] ^ (t->slice[k - 1][i] >> 8);
  for (int l = 0; l < 64; ++l) {
    const std::uint32_t m = x8n(static_cast<std::uint64_t>(63 - l) * kSeg);
    for (int j = 0; j < 8; ++j)
      for (std::uint32_t v = 0; v < 16; ++v) t->lane_shift[j][v][l] = mm(m, v << (4 * j));
  }
  const std::uint32_t mrow = x8n(kRow);
  for (int l = 0; l < 64; ++l) t->horner[l] = l < 32 ? mm(mrow, 1u << l) : 0u;
  std::uint32_t p = mrow;
  for (int k = 0; k < 64; ++k) {
    t->row_pow[k] = p;
    p = mm(p, p);
  }
  std::uint32_t rk = 0x80000000u;  // x^(8*kRow*k), k = 0..4095
  for (int k = 0; k < 4096; ++k) {
    t->rows_shift[k] = rk;
    rk = mm(rk, mrow);
  }
  // x^(-8d), d = 0..kRow: Shift_1 (one zero byte) is an invertible linear map on the register
  // (x is a unit mod P: P has a constant term), so its inverse comes from Gaussian elimination over
  // GF(2) on the 32 columns Shift_1(1 << i); x^(-8d) = InvShift_1^d(x^0).
  {
    std::uint32_t a[32], inv[32];  // row i of the matrix: bit j = bit i of Shift_1(1 << j)
    std::uint32_t col[32];
    for (int j = 0; j < 32; ++j) col[j] = mm(x8n(1), 1u << j);
    for (int i = 0; i < 32; ++i) {
      a[i] = 0;
      for (int j = 0; j < 32; ++j) a[i] |= ((col[j] >> i) & 1u) << j;
      inv[i] = 1u << i;
    }
    for (int c = 0; c < 32; ++c) {
      int piv = c;
      while (!((a[piv] >> c) & 1u)) ++piv;  // exists: Shift_1 is invertible
      std::swap(a[c], a[piv]);
      std::swap(inv[c], inv[piv]);
      for (int r = 0; r < 32; ++r)
        if (r != c && ((a[r] >> c) & 1u)) {
          a[r] ^= a[c];
          inv[r] ^= inv[c];
        }
    }
    // inv[i] bit j = entry (i, j) of the inverse matrix: InvShift_1(v) bit i = parity(inv[i] & v)
    auto inv1 = [&](std::uint32_t v) {
      std::uint32_t r = 0;
      for (int i = 0; i < 32; ++i) r |= static_cast<std::uint32_t>(__builtin_parity(inv[i] & v)) << i;
      return r;
    };
    std::uint32_t v = 0x80000000u;
    for (int d = 0; d <= kRow; ++d) {
      t->inv_shift[d] = v;
      v = inv1(v);
    }
  }
  std::uint32_t z = 0x80000000u;  // x^(8h), h = 0..kRow
  for (int h = 0; h <= kRow; ++h) {
    for (int i = 0; i < 32; ++i) t->head_shift[h][i] = mm(z, 1u << i);
    z = mm(z, 0x00800000u);
  }
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(TKV_IO_ERROR, std::string(what) + ": " + hipGetErrorString(e));
}

#define TKV_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(e_, #call);   \
  } while (0)

// Scratch used by one in-flight batch on one stream (the prepass arrays and seam records are
// written and read by kernels of that stream only).
struct StreamScratch {
  Seam* seams = nullptr;
  std::uint32_t* wave_start = nullptr;
  std::uint32_t* counts = nullptr;
  // irregular prepass, sized for cap_blocks blocks (one allocation, carved below)
  void* blob = nullptr;
  std::uint64_t* scan = nullptr;
  std::uint64_t* tiles = nullptr;
  std::uint32_t* tile_ok = nullptr;  // per scan tile: its blocks qualify for stream mode
  PrepassOut po{};
  std::uint64_t cap_blocks = 0;
  std::uint32_t gate_seq = 0;  // irregular calls on this stream (crc_list_lanes' gate, counts[kCountGate])
  bool one_pass = false;       // the last irregular call launched crc_list_lanes
};

// Spans up to this size take update()'s latency path (mapped pinned memory, one crc_span launch,
// ~11 us per call up to 4 KiB, profiles/r2/put_latency/run*.jsonl); past ~16 KiB the kernel's
// own reads across PCIe cost more than copies through the copy engines (256 KiB: 116 us mapped vs
// 50 us copied, measured with the earlier row-kernel path). Host batches of at most kSpanBatchMax
// such spans and kSpanStage bytes in all take the same kernel (one workgroup per span).
// TKV_UPDATE_SMALL_BYTES overrides the threshold (0 disables both paths; for A/B measurements).
constexpr std::size_t kSmallSpan = std::size_t(16) << 10;  // longest span for crc_span (its kSpanMax)
constexpr std::size_t kSpanStage = std::size_t(64) << 10;  // mapped staging of the short-span paths
constexpr std::uint32_t kSpanBatchMax = 256;                // spans per launch on the small-batch path
std::size_t small_span_limit() {
  static const std::size_t v = [] {
    const char* e = std::getenv("TKV_UPDATE_SMALL_BYTES");
    return e ? std::min<std::size_t>(std::strtoull(e, nullptr, 10), kSmallSpan) : kSmallSpan;
  }();
  return v;
}

// Pinned staging of the host-memory pipeline: two slabs, two streams (one per slab).
constexpr std::size_t kSlab = std::size_t(256) << 20;  // bytes of block data per pipeline stage
struct HostPipe {
  hipStream_t st[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  std::uint8_t* h_data[2] = {nullptr, nullptr};
  std::uint8_t* d_data[2] = {nullptr, nullptr};
  std::uint64_t* h_off[2] = {nullptr, nullptr};
  std::uint32_t* h_len[2] = {nullptr, nullptr};
  std::uint32_t* h_init[2] = {nullptr, nullptr};
  std::uint32_t* h_out[2] = {nullptr, nullptr};
  std::uint64_t* d_off[2] = {nullptr, nullptr};
  std::uint32_t* d_len[2] = {nullptr, nullptr};
  std::uint32_t* d_init[2] = {nullptr, nullptr};
  std::uint32_t* d_out[2] = {nullptr, nullptr};
  std::size_t cap_blocks = 0;
  ~HostPipe() {
    for (int i = 0; i < 2; ++i) {
      if (st[i]) (void)hipStreamSynchronize(st[i]);
      if (done[i]) (void)hipEventDestroy(done[i]);
      if (st[i]) (void)hipStreamDestroy(st[i]);
      (void)hipHostFree(h_data[i]);
      (void)hipFree(d_data[i]);
      (void)hipHostFree(h_off[i]);
      (void)hipHostFree(h_len[i]);
      (void)hipHostFree(h_init[i]);
      (void)hipHostFree(h_out[i]);
      (void)hipFree(d_off[i]);
      (void)hipFree(d_len[i]);
      (void)hipFree(d_init[i]);
      (void)hipFree(d_out[i]);
    }
  }
};

int pipe_init(HostPipe& p, std::size_t max_blocks) {
  p.cap_blocks = max_blocks;
  for (int i = 0; i < 2; ++i) {
    TKV_HIP(hipStreamCreateWithFlags(&p.st[i], hipStreamNonBlocking));
    TKV_HIP(hipEventCreateWithFlags(&p.done[i], hipEventDisableTiming));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_data[i]), kSlab, hipHostMallocDefault));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_data[i]), kSlab));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_off[i]), max_blocks * 8, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_len[i]), max_blocks * 4, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_init[i]), max_blocks * 4, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_out[i]), max_blocks * 4, hipHostMallocDefault));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_off[i]), max_blocks * 8));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_len[i]), max_blocks * 4));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_init[i]), max_blocks * 4));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_out[i]), max_blocks * 4));
  }
  return TKV_OK;
}

// Host batches the device can read in place (see mapped_view): no data staging at all. Only the
// per-block metadata (offsets, lengths, initial registers, results) moves, in chunks of up to
// kMapChunk blocks on two alternating streams so a chunk's metadata is prepared while the previous
// chunk's kernels read the caller's bytes over PCIe.
constexpr std::size_t kMapChunk = std::size_t(1) << 21;
struct MapPipe {
  hipStream_t st[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  std::uint64_t* h_off[2] = {nullptr, nullptr};
  std::uint32_t* h_len[2] = {nullptr, nullptr};
  std::uint32_t* h_init[2] = {nullptr, nullptr};
  std::uint32_t* h_out[2] = {nullptr, nullptr};
  std::uint64_t* d_off[2] = {nullptr, nullptr};
  std::uint32_t* d_len[2] = {nullptr, nullptr};
  std::uint32_t* d_init[2] = {nullptr, nullptr};
  std::uint32_t* d_out[2] = {nullptr, nullptr};
  std::size_t cap = 0;
  ~MapPipe() {
    for (int i = 0; i < 2; ++i) {
      if (st[i]) (void)hipStreamSynchronize(st[i]);
      if (done[i]) (void)hipEventDestroy(done[i]);
      if (st[i]) (void)hipStreamDestroy(st[i]);
      (void)hipHostFree(h_off[i]);
      (void)hipHostFree(h_len[i]);
      (void)hipHostFree(h_init[i]);
      (void)hipHostFree(h_out[i]);
      (void)hipFree(d_off[i]);
      (void)hipFree(d_len[i]);
      (void)hipFree(d_init[i]);
      (void)hipFree(d_out[i]);
    }
  }
};

int map_pipe_init(MapPipe& p, std::size_t cap) {
  p.cap = cap;
  for (int i = 0; i < 2; ++i) {
    TKV_HIP(hipStreamCreateWithFlags(&p.st[i], hipStreamNonBlocking));
    TKV_HIP(hipEventCreateWithFlags(&p.done[i], hipEventDisableTiming));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_off[i]), cap * 8, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_len[i]), cap * 4, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_init[i]), cap * 4, hipHostMallocDefault));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&p.h_out[i]), cap * 4, hipHostMallocDefault));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_off[i]), cap * 8));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_len[i]), cap * 4));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_init[i]), cap * 4));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&p.d_out[i]), cap * 4));
  }
  return TKV_OK;
}

struct DevCtx {
  int dev = -1;
  int ncu = 0;
  std::uint32_t W = 0;  // waves of a full launch (one 16-wave workgroup per CU)
  DeviceTables* d_tabs[kNumAlgos] = {};  // per checksum family (Algo)
  std::uint8_t* d_dummy = nullptr;
  std::mutex mu;
  std::map<void*, std::unique_ptr<StreamScratch>> scratch;
  // synchronous update() staging (guarded by upd_mu)
  std::mutex upd_mu;
  hipStream_t st = nullptr;
  std::uint8_t* h_stage = nullptr;
  std::uint8_t* d_stage = nullptr;
  std::uint32_t* d_io = nullptr;
  std::uint32_t* h_io = nullptr;
  std::size_t stage_cap = 0;
  // short spans (crc_span): mapped pinned buffers the kernel reads and writes in place (no copy
  // engines): span bytes, descriptors, and results followed by the done count (coherent)
  std::uint8_t* h_small = nullptr;
  const std::uint8_t* d_small = nullptr;  // device view of h_small
  SpanDesc* h_desc = nullptr;
  const SpanDesc* d_desc = nullptr;
  std::uint32_t* h_res = nullptr;
  std::uint32_t* d_res = nullptr;         // device view of h_res
  std::uint32_t span_count = 0;           // spans counted on d_io[2] by all crc_span launches so far
  std::uint32_t span_seq = 0;             // sequence number of the last crc_span launch
  // host-memory batch pipeline, kept between calls (guarded by pipe_mu)
  std::mutex pipe_mu;
  std::unique_ptr<HostPipe> pipe;
  std::unique_ptr<MapPipe> mpipe;  // zero-copy batches (guarded by pipe_mu)
};

std::mutex g_mu;
DevCtx* g_ctx[64] = {};

int get_ctx(DevCtx** out) {
  int dev = 0;
  TKV_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return fail(TKV_INVALID_ARGUMENT, "device index out of range");
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx[dev]) {
    auto* c = new DevCtx();
    c->dev = dev;
    hipDeviceProp_t prop;
    TKV_HIP(hipGetDeviceProperties(&prop, dev));
    c->ncu = prop.multiProcessorCount;
    c->W = static_cast<std::uint32_t>(c->ncu) * kWavesPerWG;
    std::unique_ptr<DeviceTables> h(new DeviceTables);
    for (int algo = 0; algo < kNumAlgos; ++algo) {
      build_tables(h.get(), algo_poly(algo));
      TKV_HIP(hipMalloc(reinterpret_cast<void**>(&c->d_tabs[algo]), sizeof(DeviceTables)));
      TKV_HIP(hipMemcpy(c->d_tabs[algo], h.get(), sizeof(DeviceTables), hipMemcpyHostToDevice));
    }
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&c->d_dummy), 256));
    TKV_HIP(hipMemset(c->d_dummy, 0, 256));
    g_ctx[dev] = c;
  }
  *out = g_ctx[dev];
  return TKV_OK;
}

int get_scratch(DevCtx* c, void* stream, std::uint64_t nblocks, StreamScratch** out) {
  std::lock_guard<std::mutex> lk(c->mu);
  auto& slot = c->scratch[stream];
  if (!slot) {
    slot.reset(new StreamScratch());
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&slot->seams), sizeof(Seam) * 2 * c->W));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&slot->wave_start), sizeof(std::uint32_t) * c->W));
    // counts[0..3], then (u64) the stream-mode info at counts + 4
    // (crc_list_lanes' per-workgroup flags from word kListFlags on: general path; from kPackFlags:
    // packed mode taken)
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&slot->counts), sizeof(std::uint32_t) * kCountWords));
    TKV_HIP(hipMemset(slot->counts, 0, sizeof(std::uint32_t) * kCountWords));
  }
  StreamScratch* s = slot.get();
  if (nblocks > s->cap_blocks) {
    // doubling growth, clamped to the largest irregular batch (nblocks <= kMaxIrregularBlocks)
    const std::uint64_t cap = std::max<std::uint64_t>(nblocks, std::min<std::uint64_t>(2 * s->cap_blocks, kMaxIrregularBlocks));
    if (s->blob) {
      // Freed blocks may still be in use by earlier work on this stream.
      TKV_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
      TKV_HIP(hipFree(s->blob));
      s->blob = nullptr;
      s->cap_blocks = 0;
    }
    const std::uint64_t ntiles = prepass_tiles(cap) + 1;
    // 8-byte arrays first: scan, tiles, s_off, big_off, tile_cls; then the 4-byte ones
    const std::uint64_t bytes = 8 * (cap + 2 * ntiles + 2 * cap) + 4 * (7 * cap + 1) + 4 * 2 * ntiles + 32;
    TKV_HIP(hipMalloc(&s->blob, bytes));
    auto* p8 = static_cast<std::uint64_t*>(s->blob);
    s->scan = p8;
    s->tiles = p8 + cap;
    s->po.s_off = p8 + cap + ntiles;
    s->po.big_off = p8 + 2 * cap + ntiles;
    s->po.tile_cls = p8 + 3 * cap + ntiles;
    auto* p4 = reinterpret_cast<std::uint32_t*>(p8 + 3 * cap + 2 * ntiles);
    s->po.s_len = p4;
    s->po.s_idx = p4 + cap;
    s->po.big_len = p4 + 2 * cap;
    s->po.big_idx = p4 + 3 * cap;
    s->po.row_scan = p4 + 4 * cap;  // cap + 1 entries
    s->tile_ok = p4 + 5 * cap + 1;
    s->po.tile_lanes = s->tile_ok + ntiles;
    // cap entries, 16-byte aligned (rows_tile_scan stores them 16 bytes at a time)
    s->po.lscan = reinterpret_cast<std::uint32_t*>(
        (reinterpret_cast<std::uintptr_t>(s->po.tile_lanes + ntiles) + 15) & ~static_cast<std::uintptr_t>(15));
    s->po.cscan = s->po.lscan + ((cap + 3) & ~static_cast<std::uint64_t>(3));  // also 16-byte aligned
    s->cap_blocks = cap;
  }
  s->po.wave_start = s->wave_start;
  *out = s;
  return TKV_OK;
}

bool ptr_ok(const void* p) { return p != nullptr; }

RowsArgs base_args(DevCtx* c, StreamScratch* s, int algo) {
  RowsArgs a{};
  a.tabs = c->d_tabs[algo];
  a.dummy = c->d_dummy;
  a.seams = s->seams;
  a.init_default = kInit;
  a.out_xor = kInit;
  a.nwaves = c->W;
  return a;
}

// Uniform batches with len <= lane_max() take crc_lanes: kLaneMax.
long long lane_max() { return static_cast<long long>(kLaneMax); }

// Uniform-length batch (also used for single spans).
int run_uniform(DevCtx* c, int algo, const std::uint8_t* d_base, std::uint64_t stride, std::uint64_t len,
                const std::uint32_t* d_init, std::uint32_t init_default, std::uint32_t out_xor, std::uint32_t* d_out,
                std::uint64_t n, hipStream_t st) {
  if (n == 0) return TKV_OK;
  if (len > 0xFFFFFFFFull || n > 0xFFFFFFFFull) return fail(TKV_INVALID_ARGUMENT, "block length or count >= 2^32");
  const std::uint64_t R = rows_for_len(static_cast<std::uint32_t>(len));
  if (n * R > 0xFFFFFFFFull) return fail(TKV_INVALID_ARGUMENT, "batch larger than 2^32 rows (16 TiB)");
  StreamScratch* s = nullptr;
  if (int rc = get_scratch(c, st, 0, &s)) return rc;
  RowsArgs a = base_args(c, s, algo);
  a.base = d_base;
  a.stride = stride;
  a.len = static_cast<std::uint32_t>(len);
  a.head_z = x8nmodp(head_len(a.len), algo_poly(algo));
  a.init_raw = d_init;
  a.init_default = init_default;
  a.out_xor = out_xor;
  a.out = d_out;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.total_rows = static_cast<std::uint32_t>(n * R);
  const bool aligned = (reinterpret_cast<std::uintptr_t>(d_base) % 16 == 0) && (stride % 16 == 0) && (len % 16 == 0);
  const std::uint64_t packed_waves = static_cast<std::uint64_t>(c->ncu) * kWavesPerWG;
  if (aligned && n >= packed_waves && len != 0 && len % kRow == 0 && stride == len) {
    a.nwaves = static_cast<std::uint32_t>(packed_waves);
    a.snap_blocks = 1;
    TKV_HIP(launch_packed(a, static_cast<unsigned>(c->ncu), st));  // whole blocks per wave, no seams
    return TKV_OK;
  }
  // (aligned back-to-back 64-byte blocks: crc_packed_small's exact G = 1 kernel is faster, 4477 vs
  // 4108 GB/s, profiles/r3/lanes/ab_shapes.jsonl)
  const bool small_exact64 = aligned && !d_init && stride == len && len == 64;
  if (static_cast<long long>(len) <= lane_max() && !small_exact64) {
    // one lane per block: any stride, alignment and initial registers; the launch
    // sizes its own grid (and a.nwaves) by the window's workgroup shape
    TKV_HIP(launch_lanes(a, static_cast<unsigned>(c->ncu), st));
    return TKV_OK;
  }
  if (aligned && !d_init && stride == len && packed_small_group(a.len)) {
    // wave rows of 64/G blocks; as many workgroups as there are rows to give
    const std::uint64_t bpr = 64u / packed_small_group(a.len);
    a.total_rows = static_cast<std::uint32_t>((n + bpr - 1) / bpr);
    const std::uint64_t grid = std::max<std::uint64_t>(
        1, std::min<std::uint64_t>(c->ncu, (a.total_rows + kWavesPerWG - 1) / kWavesPerWG));
    a.nwaves = static_cast<std::uint32_t>(grid * kWavesPerWG);
    TKV_HIP(launch_packed_small(a, static_cast<unsigned>(grid), st));
    return TKV_OK;
  }
  if (packed_small_gen_group(a.len)) {
    // the same slots for any other length of 65 B - 2 KiB, stride, alignment or initial registers
    const std::uint64_t bpr = 64u / packed_small_gen_group(a.len);
    a.total_rows = static_cast<std::uint32_t>((n + bpr - 1) / bpr);
    const std::uint64_t grid = std::max<std::uint64_t>(
        1, std::min<std::uint64_t>(c->ncu, (a.total_rows + kWavesPerWG - 1) / kWavesPerWG));
    a.nwaves = static_cast<std::uint32_t>(grid * kWavesPerWG);
    TKV_HIP(launch_packed_small_gen(a, static_cast<unsigned>(grid), st));
    return TKV_OK;
  }
  // Launch only as many workgroups as there are rows to give them (small batches).
  std::uint64_t grid = std::min<std::uint64_t>(c->ncu, (a.total_rows + kRowsWavesPerWG - 1) / kRowsWavesPerWG);
  if (grid == 0) grid = 1;
  a.nwaves = static_cast<std::uint32_t>(grid * kRowsWavesPerWG);
  a.snap_blocks = n >= a.nwaves ? 1u : 0u;
  TKV_HIP(launch_rows(a, aligned, true, static_cast<unsigned>(grid), st));
  if (!a.snap_blocks) TKV_HIP(launch_fixup(a, st));
  return TKV_OK;
}

// Whether a back-to-back batch whose scan tiles are dense in group blocks may still take stream mode
// (tkv_debug_set_stream_groups; default 0: such tiles go to the general path, whose group phase folds
// those blocks faster than the stream walk's many-ends rows).
std::atomic<int> g_stream_groups{0};

// Whether irregular batches may take the one-pass kernels (tkv_debug_set_one_pass; default 1).
std::atomic<int> g_one_pass{1};

// Irregular batches of at least kListMinBlocks blocks with the default register start with the
// one-pass kernels. Below it the general path alone: a batch the one-pass kernels hand on pays their
// two short launches (~10 us), which cfg4's 131072 blocks of 256 B-1 MiB must not (one process,
// 32 MiB gapped batches against the round-5 threshold of 1 M blocks: 36-byte payloads (732 K blocks)
// 749 -> 1011 GB/s, 26-59 B 648 -> 945, back-to-back 64 B 871 -> 1245, the rest within 1 %;
// profiles/r6/pack/threshold.jsonl).
#ifndef TKV_LIST_MIN_SHIFT
#define TKV_LIST_MIN_SHIFT 18
#endif
constexpr std::uint64_t kListMinBlocks = std::uint64_t(1) << TKV_LIST_MIN_SHIFT;
int run_irregular(DevCtx* c, int algo, const std::uint8_t* d_base, const std::uint64_t* d_off, const std::uint32_t* d_len,
                  const std::uint32_t* d_init, std::uint32_t* d_out, std::uint64_t n, hipStream_t st) {
  if (n == 0) return TKV_OK;
  if (n > kMaxIrregularBlocks) return fail(TKV_INVALID_ARGUMENT, "irregular batch of more than 2^32 - 2^13 blocks");
  StreamScratch* s = nullptr;
  if (int rc = get_scratch(c, st, n, &s)) return rc;
  RowsArgs a = base_args(c, s, algo);
  a.base = d_base;
  a.offsets = s->po.big_off;  // the row kernel walks the compacted large blocks
  a.lengths = s->po.big_len;
  a.out_idx = s->po.big_idx;
  a.row_scan = s->po.row_scan;
  a.wave_start = s->wave_start;
  a.counts = s->counts;
  a.s_off = s->po.s_off;
  a.s_len = s->po.s_len;
  a.s_idx = s->po.s_idx;
  a.init_raw = d_init;
  // The group phase takes the default register's init term from the init_shift table, which holds
  // Shift_len(0xFFFFFFFF): an irregular batch without per-block registers must start from kInit
  // (base_args sets it; this guards a future caller that changes it).
  if (a.init_default != kInit) return fail(TKV_INVALID_ARGUMENT, "irregular batches start from 0xFFFFFFFF");
  a.out = d_out;
  a.nblocks = static_cast<std::uint32_t>(n);
  a.nwaves = static_cast<std::uint32_t>(c->ncu) * kRowsWavesPerWG;
  // stream mode (chosen by the prepass on the device) reuses the large-block list for the block ends,
  // the small-block offsets for the per-end registers and the seam records for the wave registers
  auto* sinfo = reinterpret_cast<std::uint64_t*>(s->counts + 4);
  a.s_ends = s->po.big_off;
  a.s_info = sinfo;
  a.s_yq = s->po.s_off;
  a.s_wtot = reinterpret_cast<std::uint32_t*>(s->seams);  // c->W entries, then the row table (c->W + 1)
  auto* row0 = a.s_wtot + c->W;                             // (the seam records hold 16 words per wave)
  a.s_row0 = row0;
  a.s_wv = s->po.big_idx;
  a.l_off = d_off;  // the lane phase walks the caller's own arrays
  a.l_len = d_len;
  a.l_tile = s->tile_ok;
  // Default registers, at least kListMinBlocks blocks: one pass of crc_list_lanes first, which folds
  // every block when none is longer than kPackMax = 1 KiB (lane blocks one per lane, longer ones in its
  // packed mode); the general path's launches then return at once. When it meets a longer block it flags
  // its workgroup and the general path folds the whole batch. Not under tkv_debug_set_stream_groups(1),
  // which keeps the byte-stream walk of back-to-back small blocks under test.
  s->one_pass = d_init == nullptr && n >= kListMinBlocks && g_one_pass.load(std::memory_order_relaxed) != 0 &&
                g_stream_groups.load(std::memory_order_relaxed) == 0;
  if (s->one_pass) {
    s->gate_seq = s->gate_seq + 1u == 0u ? 1u : s->gate_seq + 1u;
    a.gate = s->counts + kCountGate;
    a.gate_seq = s->gate_seq;
    a.gate_flags = s->counts + kListFlags;
    RowsArgs l = a;
    l.offsets = d_off;
    l.lengths = d_len;
    TKV_HIP(launch_list_lanes(l, static_cast<unsigned>(c->ncu), st));
  }
  TKV_HIP(launch_prepass(d_base, d_off, d_len, a.nblocks, s->scan, s->tiles, s->tile_ok, s->counts, sinfo, s->po.big_off,
                         s->po, a.nwaves, static_cast<std::uint32_t>(c->ncu), d_out, row0,
                         static_cast<std::uint32_t>(g_stream_groups.load(std::memory_order_relaxed)), a.gate, a.gate_seq,
                         a.gate_flags, st));
  // stream mode: crc_stream walks the rows and crc_rows finishes the block CRCs; general path:
  // crc_stream returns at once and crc_rows walks the rows (and combines its own seams)
  TKV_HIP(launch_stream_rows(a, st, static_cast<unsigned>(c->ncu)));
  TKV_HIP(launch_rows(a, false, false, static_cast<unsigned>(c->ncu), st));
  return TKV_OK;
}

bool is_pinned_or_device(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// ---- host-memory pipeline ---------------------------------------------------------------------------

// Copy blocks [b0, b0+cnt) into dst at the slab offsets so_[i]; large slabs use several threads.
void gather(std::uint8_t* dst, const std::uint8_t* src, const std::uint64_t* off, const std::uint32_t* len,
            std::uint64_t b0, std::size_t cnt, const std::uint64_t* so_) {
  const std::uint64_t bytes = so_[cnt - 1] + len[b0 + cnt - 1];
  const unsigned nt = bytes >= (std::uint64_t(32) << 20) ? 8u : 1u;
  auto part = [&](unsigned t) {
    for (std::size_t i = cnt * t / nt; i < cnt * (t + 1) / nt; ++i)
      std::memcpy(dst + so_[i], src + off[b0 + i], len[b0 + i]);
  };
  if (nt == 1) {
    part(0);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(part, t);
  for (auto& t : th) t.join();
}

// memcpy of one large range into pinned staging, split over host threads when it is large.
void copy_span(std::uint8_t* dst, const std::uint8_t* src, std::uint64_t n) {
  const unsigned nt = n >= (std::uint64_t(32) << 20) ? 8u : 1u;
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

// copy_span followed by its H2D copy on `st`, overlapped: the range goes into pinned staging in
// chunks of kSpanChunk, and each chunk's H2D copy is issued as soon as the host threads have
// finished it, so the copy engines start after the first chunk instead of after the whole range.
// One set of threads per call: each copies its share of every chunk in order and counts the chunk
// done. Pageable sources, in one process against one memcpy of the whole slab before its copy
// (tools/ab_host.py): SSTable images 1 GB 23.0 -> 20.6 ms, 4 GiB of 64 KiB blocks 78.4 -> 75.9 ms;
// a 430 MB WAL's payloads unchanged (~13.5 ms; bound elsewhere).
constexpr std::uint64_t kSpanChunk = std::uint64_t(32) << 20;
hipError_t copy_span_h2d(std::uint8_t* dst, const std::uint8_t* src, std::uint64_t n, std::uint8_t* d_dst,
                         hipStream_t st) {
  if (n < 2 * kSpanChunk) {
    copy_span(dst, src, n);
    return hipMemcpyAsync(d_dst, dst, n, hipMemcpyHostToDevice, st);
  }
  constexpr unsigned nt = 8;
  const std::uint64_t nc = (n + kSpanChunk - 1) / kSpanChunk;
  std::unique_ptr<std::atomic<unsigned>[]> done(new std::atomic<unsigned>[nc]);
  for (std::uint64_t c = 0; c < nc; ++c) done[c].store(0, std::memory_order_relaxed);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (std::uint64_t c = 0; c < nc; ++c) {
        const std::uint64_t c0 = c * kSpanChunk, cn = std::min(kSpanChunk, n - c0);
        const std::uint64_t a = c0 + cn * t / nt, e = c0 + cn * (t + 1) / nt;
        std::memcpy(dst + a, src + a, e - a);
        done[c].fetch_add(1, std::memory_order_release);
      }
    });
  hipError_t err = hipSuccess;
  for (std::uint64_t c = 0; c < nc; ++c) {
    while (done[c].load(std::memory_order_acquire) < nt) std::this_thread::yield();
    const std::uint64_t c0 = c * kSpanChunk, cn = std::min(kSpanChunk, n - c0);
    if (err == hipSuccess) err = hipMemcpyAsync(d_dst + c0, dst + c0, cn, hipMemcpyHostToDevice, st);
  }
  for (auto& t : th) t.join();
  return err;
}

// Device view of the caller's host range [base + lo_byte, base + hi_byte) when the device can read
// it in place: pinned host memory (hipHostMalloc, or hipHostRegister'd, mapped at the same address
// on this device) or device memory, with the whole range inside one allocation. Else nullptr.
// TKV_HOST_MAPPED=0 disables the zero-copy path (A/B measurements).
std::atomic<int> g_host_mapped{[] {
  const char* e = std::getenv("TKV_HOST_MAPPED");
  return (e && e[0] == '0') ? 0 : 1;
}()};

const std::uint8_t* mapped_view(const std::uint8_t* base, std::uint64_t lo_byte, std::uint64_t hi_byte) {
  if (!g_host_mapped.load(std::memory_order_relaxed) || hi_byte <= lo_byte) return nullptr;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, base + lo_byte) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (attr.type != hipMemoryTypeHost && attr.type != hipMemoryTypeDevice) return nullptr;
  if (attr.devicePointer != static_cast<const void*>(base + lo_byte)) return nullptr;  // same address only
  void* start = nullptr;
  std::size_t size = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<std::uint8_t*>(base + lo_byte))) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<std::uint8_t*>(base + lo_byte))) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  const auto s0 = reinterpret_cast<std::uintptr_t>(start);
  const auto b = reinterpret_cast<std::uintptr_t>(base);
  if (s0 == 0 || b + lo_byte < s0 || b + hi_byte > s0 + size) return nullptr;
  return base;
}

// Blocks [lo, hi) of a host batch whose bytes the kernels read in place through `dbase` (the
// device view of h_base): metadata chunks alternate between two streams; results come back per
// chunk. Uniform contiguous chunks take the packed kernel with no metadata at all.
int mapped_batch(DevCtx* c, int algo, const std::uint8_t* dbase, const std::uint64_t* off, const std::uint32_t* len,
                 const std::uint32_t* init, std::uint32_t* out, std::uint64_t lo, std::uint64_t hi) {
  const std::size_t want = static_cast<std::size_t>(std::min<std::uint64_t>(hi - lo, kMapChunk));
  std::lock_guard<std::mutex> plk(c->pipe_mu);
  if (!c->mpipe || c->mpipe->cap < want) {
    c->mpipe.reset();
    c->mpipe.reset(new MapPipe());
    if (int rc = map_pipe_init(*c->mpipe, std::max<std::size_t>(want, 1024))) {
      c->mpipe.reset();
      return rc;
    }
  }
  MapPipe& p = *c->mpipe;
  struct Pending {
    std::uint64_t lo = 0, cnt = 0;
    bool active = false;
  } pend[2];
  auto retire = [&](int k) -> int {
    if (!pend[k].active) return TKV_OK;
    TKV_HIP(hipEventSynchronize(p.done[k]));
    std::memcpy(out + pend[k].lo, p.h_out[k], pend[k].cnt * 4);
    pend[k].active = false;
    return TKV_OK;
  };
  int k = 0;
  for (std::uint64_t b0 = lo; b0 < hi; b0 += p.cap) {
    const std::size_t cnt = static_cast<std::size_t>(std::min<std::uint64_t>(hi - b0, p.cap));
    if (int rc = retire(k)) return rc;
    bool uniform = true;
    for (std::size_t i = 1; i < cnt && uniform; ++i)
      uniform = len[b0 + i] == len[b0] && off[b0 + i] == off[b0] + i * static_cast<std::uint64_t>(len[b0]);
    const std::uint32_t* d_init = nullptr;
    if (init) {
      std::memcpy(p.h_init[k], init + b0, cnt * 4);
      TKV_HIP(hipMemcpyAsync(p.d_init[k], p.h_init[k], cnt * 4, hipMemcpyHostToDevice, p.st[k]));
      d_init = p.d_init[k];
    }
    if (uniform) {
      if (int rc = run_uniform(c, algo, dbase + off[b0], len[b0], len[b0], d_init, kInit, kInit, p.d_out[k], cnt,
                               p.st[k]))
        return rc;
    } else {
      std::memcpy(p.h_off[k], off + b0, cnt * 8);
      std::memcpy(p.h_len[k], len + b0, cnt * 4);
      TKV_HIP(hipMemcpyAsync(p.d_off[k], p.h_off[k], cnt * 8, hipMemcpyHostToDevice, p.st[k]));
      TKV_HIP(hipMemcpyAsync(p.d_len[k], p.h_len[k], cnt * 4, hipMemcpyHostToDevice, p.st[k]));
      if (int rc = run_irregular(c, algo, dbase, p.d_off[k], p.d_len[k], d_init, p.d_out[k], cnt, p.st[k])) return rc;
    }
    TKV_HIP(hipMemcpyAsync(p.h_out[k], p.d_out[k], cnt * 4, hipMemcpyDeviceToHost, p.st[k]));
    TKV_HIP(hipEventRecord(p.done[k], p.st[k]));
    pend[k] = {b0, cnt, true};
    k ^= 1;
  }
  for (int i = 0; i < 2; ++i)
    if (int rc = retire(i)) return rc;
  return TKV_OK;
}

// Blocks in [lo, hi) of a host batch, processed slab by slab. Blocks larger than a slab are
// chained through update_device in slab-sized pieces on stream 0.
int host_batch(DevCtx* c, int algo, const std::uint8_t* h_base, const std::uint64_t* off, const std::uint32_t* len,
               const std::uint32_t* init, std::uint32_t* out, std::uint64_t lo, std::uint64_t hi) {
  if (hi <= lo) return TKV_OK;
  {
    // Zero copy when the device can read the caller's buffer in place (pinned host memory).
    std::uint64_t lo_byte = ~0ull, hi_byte = 0;
    for (std::uint64_t b = lo; b < hi; ++b)
      if (len[b]) {
        lo_byte = std::min<std::uint64_t>(lo_byte, off[b]);
        hi_byte = std::max<std::uint64_t>(hi_byte, off[b] + len[b]);
      }
    if (hi_byte > lo_byte) {
      if (const std::uint8_t* dbase = mapped_view(h_base, lo_byte, hi_byte))
        return mapped_batch(c, algo, dbase, off, len, init, out, lo, hi);
    }
  }
  // Largest number of blocks a slab can hold (all >= 1 byte... zero-length blocks count too).
  std::size_t max_blocks = 1;
  {
    std::uint64_t b = lo;
    while (b < hi) {
      std::size_t cnt = 0, bytes = 0;
      while (b < hi && len[b] <= kSlab && bytes + len[b] <= kSlab && cnt < (std::size_t(1) << 22)) {
        bytes += len[b];
        ++cnt;
        ++b;
      }
      if (cnt == 0) ++b;
      max_blocks = std::max(max_blocks, cnt);
    }
  }
  std::lock_guard<std::mutex> plk(c->pipe_mu);
  if (!c->pipe || c->pipe->cap_blocks < max_blocks) {
    c->pipe.reset();  // the old pipe's streams are idle: every call retires its slabs before returning
    c->pipe.reset(new HostPipe());
    if (int rc = pipe_init(*c->pipe, max_blocks)) {
      c->pipe.reset();
      return rc;
    }
  }
  HostPipe& p = *c->pipe;
  const bool src_pinned = is_pinned_or_device(h_base);
  struct Pending {
    std::uint64_t lo = 0, cnt = 0;
    bool active = false;
  } pend[2];
  auto retire = [&](int k) -> int {
    if (!pend[k].active) return TKV_OK;
    TKV_HIP(hipEventSynchronize(p.done[k]));
    std::memcpy(out + pend[k].lo, p.h_out[k], pend[k].cnt * 4);
    pend[k].active = false;
    return TKV_OK;
  };
  std::uint64_t b = lo;
  int k = 0;
  while (b < hi) {
    if (len[b] > kSlab) {
      // Huge block: chain raw registers through slab-sized device updates.
      for (int i = 0; i < 2; ++i)
        if (int rc = retire(i)) return rc;
      std::uint32_t raw = init ? init[b] : kInit;
      const std::uint8_t* src = h_base + off[b];
      std::uint64_t rem = len[b];
      while (rem) {
        const std::size_t m = static_cast<std::size_t>(std::min<std::uint64_t>(rem, kSlab));
        std::memcpy(p.h_data[0], src, m);
        p.h_init[0][0] = raw;
        TKV_HIP(hipMemcpyAsync(p.d_data[0], p.h_data[0], m, hipMemcpyHostToDevice, p.st[0]));
        TKV_HIP(hipMemcpyAsync(p.d_init[0], p.h_init[0], 4, hipMemcpyHostToDevice, p.st[0]));
        if (int rc = run_uniform(c, algo, p.d_data[0], m, m, p.d_init[0], kInit, 0u, p.d_out[0], 1, p.st[0])) return rc;
        TKV_HIP(hipMemcpyAsync(p.h_out[0], p.d_out[0], 4, hipMemcpyDeviceToHost, p.st[0]));
        TKV_HIP(hipStreamSynchronize(p.st[0]));
        raw = p.h_out[0][0];
        src += m;
        rem -= m;
      }
      out[b] = raw ^ kInit;
      ++b;
      continue;
    }
    // Next slab: the longest run of blocks that fits kSlab bytes.
    if (int rc = retire(k)) return rc;
    std::size_t cnt = 0, bytes = 0;
    const std::uint64_t b0 = b;
    bool contiguous = true, uniform = true, ascending = true;
    while (b < hi && len[b] <= kSlab && bytes + len[b] <= kSlab && cnt < p.cap_blocks) {
      if (cnt) {
        const bool asc = ascending && off[b] >= off[b - 1] + len[b - 1];
        // A dense ascending run (the span mode below) ends where its covering range would outgrow
        // the slab, so that it still goes over as one range: WAL payloads are 8 bytes apart, and a
        // slab filled by payload bytes alone covers more than kSlab and was gathered block by block
        // (430 MB of WAL payloads: 4.5 ms of gather before the first copy).
        const std::uint64_t sp = off[b - 1] + len[b - 1] - off[b0];
        if (asc && sp <= bytes + bytes / 4 + 4096 && off[b] + len[b] - off[b0] > kSlab) break;
        contiguous = contiguous && off[b] == off[b - 1] + len[b - 1];
        ascending = asc;
        uniform = uniform && len[b] == len[b0];
      }
      p.h_off[k][cnt] = bytes;
      p.h_len[k][cnt] = len[b];
      p.h_init[k][cnt] = init ? init[b] : kInit;
      bytes += len[b];
      ++cnt;
      ++b;
    }
    // How the slab's bytes reach the device:
    //  * span: ascending blocks whose covering range [off[b0], end of last) is at most 1/4 larger
    //    than their payload (WAL records, SSTable images: small headers between payloads) go over
    //    as that one range - straight from pinned memory, else one threaded memcpy into staging -
    //    and keep their offsets relative to it;
    //  * anything else is gathered block by block into the pinned staging slab.
    const std::uint64_t lo = off[b0], span = ascending ? off[b - 1] + len[b - 1] - lo : ~0ull;
    const bool span_mode = ascending && span <= kSlab && span <= bytes + bytes / 4 + 4096;
    if (span_mode) {
      if (!contiguous)
        for (std::size_t i = 0; i < cnt; ++i) p.h_off[k][i] = off[b0 + i] - lo;
      if (src_pinned) {
        TKV_HIP(hipMemcpyAsync(p.d_data[k], h_base + lo, span, hipMemcpyHostToDevice, p.st[k]));
      } else {
        TKV_HIP(copy_span_h2d(p.h_data[k], h_base + lo, span, p.d_data[k], p.st[k]));
      }
    } else {
      contiguous = false;
      gather(p.h_data[k], h_base, off, len, b0, cnt, p.h_off[k]);
      TKV_HIP(hipMemcpyAsync(p.d_data[k], p.h_data[k], bytes, hipMemcpyHostToDevice, p.st[k]));
    }
    uniform = uniform && (contiguous || !span_mode);  // the uniform kernels need blocks back to back
    TKV_HIP(hipMemcpyAsync(p.d_init[k], p.h_init[k], cnt * 4, hipMemcpyHostToDevice, p.st[k]));
    if (uniform) {
      // equal lengths, packed back to back in the slab: the uniform (packed) kernels, no prepass
      if (int rc = run_uniform(c, algo, p.d_data[k], len[b0], len[b0], p.d_init[k], kInit, kInit, p.d_out[k], cnt,
                               p.st[k]))
        return rc;
    } else {
      TKV_HIP(hipMemcpyAsync(p.d_off[k], p.h_off[k], cnt * 8, hipMemcpyHostToDevice, p.st[k]));
      TKV_HIP(hipMemcpyAsync(p.d_len[k], p.h_len[k], cnt * 4, hipMemcpyHostToDevice, p.st[k]));
      if (int rc = run_irregular(c, algo, p.d_data[k], p.d_off[k], p.d_len[k], p.d_init[k], p.d_out[k], cnt, p.st[k]))
        return rc;
    }
    TKV_HIP(hipMemcpyAsync(p.h_out[k], p.d_out[k], cnt * 4, hipMemcpyDeviceToHost, p.st[k]));
    TKV_HIP(hipEventRecord(p.done[k], p.st[k]));
    pend[k] = {b0, cnt, true};
    k ^= 1;
  }
  for (int i = 0; i < 2; ++i)
    if (int rc = retire(i)) return rc;
  return TKV_OK;
}

}  // namespace

// ---- entry points shared by the CRC-32 and CRC-32C C ABI ------------------------------------

int update_device_impl(int algo, uint32_t raw_state, const void* d_data, size_t len, uint32_t* d_out_raw, void* stream) {
  if (!ptr_ok(d_out_raw) || (len && !ptr_ok(d_data))) return fail(TKV_INVALID_ARGUMENT, "null pointer");
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  // One block of `len` bytes continued from raw_state; raw register out (no xorout).
  const auto* base = static_cast<const std::uint8_t*>(d_data ? d_data : c->d_dummy);
  return run_uniform(c, algo, base, len, len, nullptr, raw_state, 0u, d_out_raw, 1, static_cast<hipStream_t>(stream));
}

// One launch of crc_span over n spans already in the mapped staging (n == 1: `one`, else the mapped
// descriptors), then a poll of the mapped done word for this launch's sequence number, which the
// kernel releases after every result: polling saves ~5 us per call against sleeping in
// hipStreamSynchronize. After 100 ms without it, hipStreamSynchronize reports whatever held the
// kernel up. The span counter on the device (d_io[2]) only grows; the launch is done when it
// reaches span_count + n. Caller holds upd_mu.
int run_spans(DevCtx* c, int algo, const SpanDesc& one, std::uint32_t n, std::uint32_t out_xor, std::uint32_t* out) {
  std::uint32_t* done = c->h_res + kSpanBatchMax;
  if (++c->span_seq == 0) c->span_seq = 1;
  const std::uint32_t seq = c->span_seq, base = c->span_count;
  TKV_HIP(launch_span(c->d_small, one, n == 1 ? nullptr : c->d_desc, n, out_xor, c->d_res, c->d_io + 2, base,
                      c->d_res + kSpanBatchMax, seq, c->d_tabs[algo], c->st));
  if (n > 1) c->span_count = base + n;  // a one-span launch does not count
  const auto t0 = std::chrono::steady_clock::now();
  for (std::uint32_t i = 0; __atomic_load_n(done, __ATOMIC_ACQUIRE) != seq; ++i) {
    if ((i & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
      TKV_HIP(hipStreamSynchronize(c->st));
      if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) return fail(TKV_IO_ERROR, "span kernel did not report");
      break;
    }
  }
  for (std::uint32_t i = 0; i < n; ++i) out[i] = __atomic_load_n(c->h_res + i, __ATOMIC_RELAXED);
  return TKV_OK;
}

// The latency paths' stream and mapped buffers, created on first use. Caller holds upd_mu.
int ensure_upd(DevCtx* c) {
  if (!c->st) {
    TKV_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->h_io), 16, hipHostMallocDefault));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&c->d_io), 16));  // [0]: staged update result, [2]: span count
    TKV_HIP(hipMemset(c->d_io, 0, 16));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->h_small), kSpanStage, hipHostMallocMapped));
    TKV_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(const_cast<std::uint8_t**>(&c->d_small)), c->h_small, 0));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->h_desc), sizeof(SpanDesc) * kSpanBatchMax, hipHostMallocMapped));
    TKV_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(const_cast<SpanDesc**>(&c->d_desc)), c->h_desc, 0));
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->h_res), sizeof(std::uint32_t) * (kSpanBatchMax + 1),
                          hipHostMallocMapped | hipHostMallocCoherent));
    TKV_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_res), c->h_res, 0));
  }
  return TKV_OK;
}

// Small host batch (a WAL group commit of a few records, a few SSTable blocks) on the latency path:
// every block copied to a 16-byte aligned position of the mapped staging, one crc_span launch with
// a workgroup per block, finalize() values out. Returns 1 (nothing done) when the batch does not fit.
int span_batch(DevCtx* c, int algo, const uint8_t* h_base, const uint64_t* h_offsets, const uint32_t* h_lengths,
               const uint32_t* h_init_raw, uint32_t* h_out_final, uint64_t n) {
  if (n > kSpanBatchMax || small_span_limit() == 0) return 1;
  std::uint64_t total = 0;
  for (std::uint64_t i = 0; i < n; ++i) {
    if (h_lengths[i] > small_span_limit()) return 1;
    total += (static_cast<std::uint64_t>(h_lengths[i]) + 15u) & ~15ull;
  }
  if (total > kSpanStage) return 1;
  std::lock_guard<std::mutex> lk(c->upd_mu);
  if (int rc = ensure_upd(c)) return rc;
  std::uint32_t pos = 0;
  for (std::uint64_t i = 0; i < n; ++i) {
    const std::uint32_t len = h_lengths[i];
    if (len) std::memcpy(c->h_small + pos, h_base + h_offsets[i], len);
    c->h_desc[i] = SpanDesc{pos, len, h_init_raw ? h_init_raw[i] : kInit, 0};
    pos += (len + 15u) & ~15u;
  }
  return run_spans(c, algo, c->h_desc[0], static_cast<std::uint32_t>(n), kInit, h_out_final);
}

extern thread_local std::uint64_t g_update_calls[3];  // tkv_crc32_span.cpp

int update_impl(int algo, uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  if (!ptr_ok(out_raw) || (len && !ptr_ok(data))) return fail(TKV_INVALID_ARGUMENT, "null pointer");
  ++g_update_calls[1];
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  std::lock_guard<std::mutex> lk(c->upd_mu);
  if (int rc = ensure_upd(c)) return rc;
  if (len <= small_span_limit()) {
    // Latency path (one WAL record per call, wal.cpp:54-57): one small kernel (crc_span) reads the
    // span from mapped pinned memory and writes the register back into mapped memory - one launch
    // and one sync, no copy-engine round trips. An empty span leaves the register as it is
    // (crc32.cpp:9-16 loops zero times).
    if (len == 0) {
      *out_raw = raw_state;
      return TKV_OK;
    }
    std::memcpy(c->h_small, data, len);
    const SpanDesc one{0, static_cast<std::uint32_t>(len), raw_state, 0};
    return run_spans(c, algo, one, 1, 0u, out_raw);
  }
  const std::size_t want = std::min<std::size_t>(std::max<std::size_t>(len, 1 << 16), kSlab);
  if (want > c->stage_cap) {
    (void)hipHostFree(c->h_stage);
    (void)hipFree(c->d_stage);
    c->h_stage = nullptr;
    c->d_stage = nullptr;
    c->stage_cap = 0;
    TKV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->h_stage), want, hipHostMallocDefault));
    TKV_HIP(hipMalloc(reinterpret_cast<void**>(&c->d_stage), want));
    c->stage_cap = want;
  }
  std::uint32_t raw = raw_state;
  const auto* src = static_cast<const std::uint8_t*>(data);
  std::size_t rem = len;
  do {
    const std::size_t m = std::min(rem, c->stage_cap);
    if (m) {
      std::memcpy(c->h_stage, src, m);
      TKV_HIP(hipMemcpyAsync(c->d_stage, c->h_stage, m, hipMemcpyHostToDevice, c->st));
    }
    if (int rc = run_uniform(c, algo, c->d_stage, m, m, nullptr, raw, 0u, c->d_io, 1, c->st)) return rc;
    TKV_HIP(hipMemcpyAsync(c->h_io, c->d_io, 4, hipMemcpyDeviceToHost, c->st));
    TKV_HIP(hipStreamSynchronize(c->st));
    raw = c->h_io[0];
    src += m;
    rem -= m;
  } while (rem);
  *out_raw = raw;
  return TKV_OK;
}

int batch_device_impl(int algo, const uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                      const uint32_t* d_init_raw, uint32_t* d_out_final, uint64_t n, void* stream) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(d_base) || !ptr_ok(d_offsets) || !ptr_ok(d_lengths) || !ptr_ok(d_out_final))
    return fail(TKV_INVALID_ARGUMENT, "null pointer");
  if (n > kMaxIrregularBlocks) return fail(TKV_INVALID_ARGUMENT, "irregular batch of more than 2^32 - 2^13 blocks");
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  return run_irregular(c, algo, d_base, d_offsets, d_lengths, d_init_raw, d_out_final, n, static_cast<hipStream_t>(stream));
}

int batch_uniform_impl(int algo, const uint8_t* d_base, uint64_t stride, uint64_t len, const uint32_t* d_init_raw,
                       uint32_t* d_out_final, uint64_t n, void* stream) {
  if (n == 0) return TKV_OK;
  if ((len && !ptr_ok(d_base)) || !ptr_ok(d_out_final)) return fail(TKV_INVALID_ARGUMENT, "null pointer");
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  const auto* base = d_base ? d_base : c->d_dummy;
  return run_uniform(c, algo, base, stride, len, d_init_raw, kInit, kInit, d_out_final, n, static_cast<hipStream_t>(stream));
}

int batch_host_impl(int algo, const uint8_t* h_base, const uint64_t* h_offsets, const uint32_t* h_lengths,
                    const uint32_t* h_init_raw, uint32_t* h_out_final, uint64_t n) {
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_base) || !ptr_ok(h_offsets) || !ptr_ok(h_lengths) || !ptr_ok(h_out_final))
    return fail(TKV_INVALID_ARGUMENT, "null pointer");
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  if (int rc = span_batch(c, algo, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, n); rc != 1) return rc;
  return host_batch(c, algo, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, 0, n);
}

// Blocks of at least this many bytes that straddle a device's byte share are cut at the share
// boundary; their pieces run on different devices and combine on the host.
constexpr std::uint64_t kSplitMin = std::uint64_t(1) << 20;

// Split plan of a host batch over ndev devices. Byte-balanced contiguous split of
// the block list: device d takes the bytes [total*d/ndev, total*(d+1)/ndev) of the blocks laid end
// to end in index order. Without a cut block the plan is index ranges [cut[d], cut[d+1]) of the
// caller's arrays; with one (a block >= kSplitMin straddling a share boundary) every device gets its
// own piece list, pieces in block order, a cut block's head piece taking the block's init and the
// following pieces starting from 0.
struct MultiPlan {
  struct Work {
    std::vector<std::uint64_t> off;
    std::vector<std::uint32_t> len, init, out;
    std::vector<std::uint64_t> block;  // batch index of each piece
    std::vector<std::uint8_t> head;    // piece starts its block (takes the block's init)
  };
  bool split = false;
  std::vector<std::uint64_t> cut;
  std::vector<Work> work;  // split plans only, one per device
};

MultiPlan plan_multi(int ndev, const uint64_t* h_offsets, const uint32_t* h_lengths, const uint32_t* h_init_raw,
                     uint64_t n) {
  MultiPlan p;
  std::uint64_t total = 0;
  for (std::uint64_t i = 0; i < n; ++i) total += h_lengths[i];
  p.cut.assign(ndev + 1, n);
  p.cut[0] = 0;
  {
    std::uint64_t acc = 0, i = 0;
    for (int d = 1; d < ndev; ++d) {
      const std::uint64_t target = total * d / ndev;
      while (i < n && acc + h_lengths[i] <= target) acc += h_lengths[i++];
      p.cut[d] = i;
      // block i straddles the boundary (acc < target < acc + len): cut it if it is large
      if (i < n && acc < target && h_lengths[i] >= kSplitMin) p.split = true;
    }
  }
  if (!p.split) return p;
  p.work.resize(ndev);
  std::uint64_t pos = 0;  // byte position of block i's start in the end-to-end stream
  int d = 0;
  for (std::uint64_t i = 0; i < n; ++i) {
    const std::uint64_t len = h_lengths[i];
    std::uint64_t done = 0;
    do {
      while (d + 1 < ndev && pos + done >= total * (d + 1) / ndev && (len == 0 || done < len)) ++d;
      std::uint64_t take = len - done;
      if (len >= kSplitMin && d + 1 < ndev) {
        const std::uint64_t end = total * (d + 1) / ndev;  // this device's share ends here
        if (pos + len > end && end > pos + done) take = end - (pos + done);
      }
      MultiPlan::Work& w = p.work[d];
      w.off.push_back(h_offsets[i] + done);
      w.len.push_back(static_cast<std::uint32_t>(take));
      w.init.push_back(done == 0 ? (h_init_raw ? h_init_raw[i] : kInit) : 0u);
      w.block.push_back(i);
      w.head.push_back(done == 0);
      done += take;
    } while (done < len);
    pos += len;
  }
  for (auto& w : p.work) w.out.resize(w.off.size());
  return p;
}

// Results of a split plan: pieces arrive in block order across the devices, and a head piece's
// register continues through the following pieces of its block, r = Shift_len(r) ^ crc_0(piece)
// (tkv_crc32_combine). Only 4-byte registers are combined here; no data is read.
void combine_multi(const MultiPlan& p, uint64_t n, std::uint32_t poly, uint32_t* h_out_final) {
  std::uint64_t cur = n;
  std::uint32_t raw = 0;
  for (const auto& w : p.work) {
    for (std::size_t k = 0; k < w.off.size(); ++k) {
      const std::uint32_t r = w.out[k] ^ kInit;  // raw register of the piece
      if (w.head[k]) {
        if (cur != n) h_out_final[cur] = raw ^ kInit;
        cur = w.block[k];
        raw = r;
      } else {
        raw = shift_bytes(raw, w.len[k], poly) ^ r;
      }
    }
  }
  if (cur != n) h_out_final[cur] = raw ^ kInit;
}

// One host thread per device: hipSetDevice (tkv_set_device) binds the thread, and get_ctx then
// creates or finds that device's own context (tables, dummy buffer, streams, scratch, staging).
int batch_host_multi_impl(int algo, const int* devices, int ndev, const uint8_t* h_base, const uint64_t* h_offsets,
                          const uint32_t* h_lengths, const uint32_t* h_init_raw, uint32_t* h_out_final, uint64_t n) {
  if (ndev <= 0 || !ptr_ok(devices)) return fail(TKV_INVALID_ARGUMENT, "no devices");
  if (n == 0) return TKV_OK;
  if (!ptr_ok(h_base) || !ptr_ok(h_offsets) || !ptr_ok(h_lengths) || !ptr_ok(h_out_final))
    return fail(TKV_INVALID_ARGUMENT, "null pointer");
  MultiPlan plan = plan_multi(ndev, h_offsets, h_lengths, h_init_raw, n);
  std::vector<int> rcs(ndev, TKV_OK);
  std::vector<std::string> errs(ndev);
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; ++d) {
    th.emplace_back([&, d] {
      if (int rc = tkv_set_device(devices[d])) {
        rcs[d] = rc;
        errs[d] = g_err;
        return;
      }
      DevCtx* c = nullptr;
      rcs[d] = get_ctx(&c);
      if (rcs[d] == TKV_OK) {
        if (plan.split) {
          MultiPlan::Work& w = plan.work[d];
          if (!w.off.empty())
            rcs[d] = host_batch(c, algo, h_base, w.off.data(), w.len.data(), w.init.data(), w.out.data(), 0, w.off.size());
        } else {
          rcs[d] = host_batch(c, algo, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, plan.cut[d],
                              plan.cut[d + 1]);
        }
      }
      errs[d] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (int d = 0; d < ndev; ++d)
    if (rcs[d]) return fail(rcs[d], "device " + std::to_string(devices[d]) + ": " + errs[d]);
  if (plan.split) combine_multi(plan, n, algo_poly(algo), h_out_final);
  return TKV_OK;
}

int set_error(int code, const char* msg) { return fail(code, msg); }

const DeviceTables* device_tables(int algo) {
  DevCtx* c = nullptr;
  if (get_ctx(&c)) return nullptr;
  return c->d_tabs[algo];
}

}  // namespace tkv

using namespace tkv;

extern "C" {

int tkv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int tkv_set_device(int device) {
  int n = tkv_device_count();
  if (device < 0 || device >= n) return fail(TKV_INVALID_ARGUMENT, "no such device");
  TKV_HIP(hipSetDevice(device));
  DevCtx* c = nullptr;
  return get_ctx(&c);
}

const char* tkv_last_error(void) { return g_err.c_str(); }

int tkv_crc32_update_device(uint32_t raw_state, const void* d_data, size_t len, uint32_t* d_out_raw, void* stream) {
  return update_device_impl(kAlgoCrc32, raw_state, d_data, len, d_out_raw, stream);
}
int tkv_crc32_update(uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  return update_impl(kAlgoCrc32, raw_state, data, len, out_raw);
}
int tkv_crc32_batch_device(const uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                           const uint32_t* d_init_raw, uint32_t* d_out_final, uint64_t n, void* stream) {
  return batch_device_impl(kAlgoCrc32, d_base, d_offsets, d_lengths, d_init_raw, d_out_final, n, stream);
}
int tkv_crc32_batch_uniform_device(const uint8_t* d_base, uint64_t stride, uint64_t len, const uint32_t* d_init_raw,
                                   uint32_t* d_out_final, uint64_t n, void* stream) {
  return batch_uniform_impl(kAlgoCrc32, d_base, stride, len, d_init_raw, d_out_final, n, stream);
}
int tkv_crc32_batch_host(const uint8_t* h_base, const uint64_t* h_offsets, const uint32_t* h_lengths,
                         const uint32_t* h_init_raw, uint32_t* h_out_final, uint64_t n) {
  return batch_host_impl(kAlgoCrc32, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, n);
}
int tkv_crc32_batch_host_multi(const int* devices, int ndev, const uint8_t* h_base, const uint64_t* h_offsets,
                               const uint32_t* h_lengths, const uint32_t* h_init_raw, uint32_t* h_out_final,
                               uint64_t n) {
  return batch_host_multi_impl(kAlgoCrc32, devices, ndev, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, n);
}

uint32_t tkv_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return tkv::shift_bytes(crc1, len2, kPoly) ^ crc2;
}
uint32_t tkv_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return tkv::shift_bytes(crc1, len2, kPolyC) ^ crc2;
}

int tkv_crc32c_update(uint32_t raw_state, const void* data, size_t len, uint32_t* out_raw) {
  return update_impl(kAlgoCrc32c, raw_state, data, len, out_raw);
}
int tkv_crc32c_update_device(uint32_t raw_state, const void* d_data, size_t len, uint32_t* d_out_raw, void* stream) {
  return update_device_impl(kAlgoCrc32c, raw_state, d_data, len, d_out_raw, stream);
}
int tkv_crc32c_batch_device(const uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                            const uint32_t* d_init_raw, uint32_t* d_out_final, uint64_t n, void* stream) {
  return batch_device_impl(kAlgoCrc32c, d_base, d_offsets, d_lengths, d_init_raw, d_out_final, n, stream);
}
int tkv_crc32c_batch_uniform_device(const uint8_t* d_base, uint64_t stride, uint64_t len, const uint32_t* d_init_raw,
                                    uint32_t* d_out_final, uint64_t n, void* stream) {
  return batch_uniform_impl(kAlgoCrc32c, d_base, stride, len, d_init_raw, d_out_final, n, stream);
}
int tkv_crc32c_batch_host(const uint8_t* h_base, const uint64_t* h_offsets, const uint32_t* h_lengths,
                          const uint32_t* h_init_raw, uint32_t* h_out_final, uint64_t n) {
  return batch_host_impl(kAlgoCrc32c, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, n);
}
int tkv_crc32c_batch_host_multi(const int* devices, int ndev, const uint8_t* h_base, const uint64_t* h_offsets,
                                const uint32_t* h_lengths, const uint32_t* h_init_raw, uint32_t* h_out_final,
                                uint64_t n) {
  return batch_host_multi_impl(kAlgoCrc32c, devices, ndev, h_base, h_offsets, h_lengths, h_init_raw, h_out_final, n);
}

int tkv_fill_synthetic_uniform(uint8_t* d_dst, uint64_t stride, uint64_t len, uint64_t first_block, uint64_t nblocks,
                               uint64_t seed, void* stream) {
  if (len % 8 || stride % 8 || reinterpret_cast<std::uintptr_t>(d_dst) % 8)
    return fail(TKV_INVALID_ARGUMENT, "uniform fill needs 8-byte aligned blocks");
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  TKV_HIP(launch_fill_uniform(d_dst, stride, len, first_block, nblocks, seed, static_cast<hipStream_t>(stream)));
  return TKV_OK;
}

int tkv_fill_synthetic_blocks(uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                              uint64_t first_block, uint64_t nblocks, uint64_t seed, void* stream) {
  DevCtx* c = nullptr;
  if (int rc = get_ctx(&c)) return rc;
  TKV_HIP(launch_fill_blocks(d_base, d_offsets, d_lengths, first_block, nblocks, seed, static_cast<hipStream_t>(stream)));
  return TKV_OK;
}

size_t tkv_debug_tables(void* out, size_t cap) { return tkv_debug_tables_poly(kPoly, out, cap); }

size_t tkv_debug_tables_poly(uint32_t poly, void* out, size_t cap) {
  if (out && cap >= sizeof(DeviceTables)) build_tables(static_cast<DeviceTables*>(out), poly);
  return sizeof(DeviceTables);
}

uint32_t tkv_debug_multmodp(uint32_t a, uint32_t b) { return multmodp(a, b); }
uint32_t tkv_debug_x8nmodp(uint64_t nbytes) { return x8nmodp(nbytes); }
size_t tkv_debug_multi_plan(int ndev, const uint64_t* h_offsets, const uint32_t* h_lengths, const uint32_t* h_init_raw,
                            uint64_t n, uint64_t* out_rec, size_t cap) {
  if (ndev <= 0 || n == 0 || !h_offsets || !h_lengths) return 0;
  const MultiPlan p = plan_multi(ndev, h_offsets, h_lengths, h_init_raw, n);
  size_t k = 0;
  auto put = [&](int d, std::uint64_t b, std::uint64_t off, std::uint64_t len, std::uint64_t init, bool head) {
    if (out_rec && k < cap) {
      std::uint64_t* r = out_rec + 6 * k;
      r[0] = static_cast<std::uint64_t>(d);
      r[1] = b;
      r[2] = off;
      r[3] = len;
      r[4] = init;
      r[5] = head ? 1u : 0u;
    }
    ++k;
  };
  for (int d = 0; d < ndev; ++d) {
    if (p.split) {
      const auto& w = p.work[d];
      for (size_t j = 0; j < w.off.size(); ++j) put(d, w.block[j], w.off[j], w.len[j], w.init[j], w.head[j] != 0);
    } else {
      for (std::uint64_t b = p.cut[d]; b < p.cut[d + 1]; ++b)
        put(d, b, h_offsets[b], h_lengths[b], h_init_raw ? h_init_raw[b] : kInit, true);
    }
  }
  return k;
}

int tkv_debug_multi_combine(uint32_t poly, int ndev, const uint64_t* h_offsets, const uint32_t* h_lengths,
                            const uint32_t* h_init_raw, uint64_t n, const uint32_t* piece_final, uint32_t* h_out_final) {
  if (ndev <= 0 || n == 0 || !h_offsets || !h_lengths || !piece_final || !h_out_final) return TKV_INVALID_ARGUMENT;
  MultiPlan p = plan_multi(ndev, h_offsets, h_lengths, h_init_raw, n);
  size_t k = 0;
  if (!p.split) {
    for (std::uint64_t b = 0; b < n; ++b) h_out_final[b] = piece_final[b];
    return TKV_OK;
  }
  for (auto& w : p.work)
    for (auto& o : w.out) o = piece_final[k++];
  combine_multi(p, n, poly, h_out_final);
  return TKV_OK;
}

namespace {
int read_count_word(void* stream, int word) {
  DevCtx* c = nullptr;
  if (get_ctx(&c)) return -1;
  StreamScratch* s = nullptr;
  if (get_scratch(c, stream, 0, &s)) return -1;
  std::uint32_t v = 0;
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess ||
      hipMemcpy(&v, s->counts + word, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return static_cast<int>(v);
}
}  // namespace

int tkv_debug_irregular_mode(void* stream) { return read_count_word(stream, 3); }

int tkv_debug_irregular_phases(void* stream) { return read_count_word(stream, kCountPhases); }

int tkv_debug_irregular_path(void* stream) {
  DevCtx* c = nullptr;
  if (get_ctx(&c)) return -1;
  StreamScratch* s = nullptr;
  if (get_scratch(c, stream, 0, &s)) return -1;
  if (!s->one_pass) return 3;
  std::vector<std::uint32_t> f(2 * kListMaxGroups);
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess ||
      hipMemcpy(f.data(), s->counts + kListFlags, 4 * f.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  bool general = false, packed = false;
  for (unsigned i = 0; i < kListMaxGroups; ++i) {
    general = general || f[i] == s->gate_seq;
    packed = packed || f[kListMaxGroups + i] == s->gate_seq;
  }
  return general ? 2 : packed ? 1 : 0;
}

uint32_t tkv_debug_list_lanes_waves(uint64_t nblocks) {
  DevCtx* c = nullptr;
  if (get_ctx(&c)) return 0;
  return tkv::list_lanes_waves(nblocks, static_cast<unsigned>(c->ncu));
}

int tkv_debug_irregular_lists(void* stream, std::uint32_t out[3]) {
  const int w[3] = {1, kCountSmall4, kCountSmall8};
  for (int i = 0; i < 3; ++i) {
    const int v = read_count_word(stream, w[i]);
    if (v == -1) return -1;
    out[i] = static_cast<std::uint32_t>(v);
  }
  return 0;
}

int tkv_debug_set_host_mapped(int enable) { return tkv::g_host_mapped.exchange(enable ? 1 : 0); }

int tkv_debug_set_stream_groups(int enable) { return tkv::g_stream_groups.exchange(enable ? 1 : 0); }

int tkv_debug_set_one_pass(int enable) { return tkv::g_one_pass.exchange(enable ? 1 : 0); }

}  // extern "C"
