/*
 * tkv_crc32.h — C ABI of the MI355X CRC-32 block-checksum engine (libtkv_crc32.so).
 *
 * Drop-in boundary for tinykvpp's integrity hot path: the CRC-32/ISO-HDLC routine
 * frankie::core::crc32 (/root/reference/src/core/crc32.hpp:32-49, crc32.cpp:9-22) and the call
 * sites that stamp/verify WAL records (/root/reference/src/engine/wal.cpp:54-58, 89-96).
 * Plain C: pointers, sizes and integer status codes only. Every batch, device and host-pipeline
 * entry point computes on the HIP kernels for gfx950 and reports TKV_IO_ERROR when no GPU is usable;
 * none of them falls back to the CPU. The CPU computes only in the separately named single-span
 * entry points tkv_crc32[c]_update_host and tkv_crc32[c]_update_fallback, which the drop-in header
 * include/frankie_crc32.hpp uses to keep crc32::update's never-fail contract (crc32.cpp:9-16).
 *
 * State conventions (match crc32.hpp:37-46):
 *   "raw" register  = the value crc32::crc_ holds (init 0xFFFFFFFF, no xorout applied);
 *   "final" value   = crc32::finalize() = raw ^ 0xFFFFFFFF.
 *
 * Stream arguments are hipStream_t passed as void* (NULL = the legacy default stream).
 */
#ifndef TKV_CRC32_H
#define TKV_CRC32_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes mirror frankie::core::status_code (/root/reference/src/core/status.hpp:11-20). */
enum tkv_status {
  TKV_OK = 0,
  TKV_NOT_FOUND = 1,
  TKV_IO_ERROR = 2,          /* HIP runtime failure (no device, launch or copy error) */
  TKV_INVALID_ARGUMENT = 3,
  TKV_CORRUPTED = 4,         /* a verified checksum did not match (wal.cpp:93-96) */
  TKV_EOF = 5,
  TKV_OUT_OF_MEMORY = 6,
  TKV_BUFFER_OVERFLOW = 7
};

#define TKV_CRC32_DEFAULT_RAW 0xFFFFFFFFu /* crc32.hpp:9 kCRC32DefaultValue */
#define TKV_CRC32_POLYNOMIAL 0xEDB88320u  /* crc32.hpp:11 kCRC32Polynomial */

/* ---- library / device management -------------------------------------------------------------- */

/* Number of usable GPUs (0 when the HIP runtime finds none). */
int tkv_device_count(void);

/* Bind the calling thread to `device` and create that device's context (tables, scratch) if needed.
 * Every other entry point uses the calling thread's current device. */
int tkv_set_device(int device);

/* Human-readable text of the last error on this thread ("" if none). */
const char *tkv_last_error(void);

/* Build identity: 16 hex digits of sha256 over the library's sources and Makefile, baked in at build
 * time (tinykvpp_amd/build_id.py); tests and bench.py check it against the tree they run in. */
const char *tkv_build_id(void);

/* ---- crc32::update replacement ---------------------------------------------------------------- */

/* Continue raw register `raw_state` over `len` bytes of HOST memory; writes the new raw register.
 * Replaces crc32::update (crc32.hpp:37, crc32.cpp:9-16); finalize is raw ^ 0xFFFFFFFF
 * (crc32.cpp:19) and reset is raw = 0xFFFFFFFF (crc32.cpp:22). Synchronous (stages through the
 * GPU; the right tool for one span is the batch API). */
int tkv_crc32_update(uint32_t raw_state, const void *data, size_t len, uint32_t *out_raw);

/* Same over DEVICE memory, asynchronous on `stream`; *d_out_raw is written on the device. */
int tkv_crc32_update_device(uint32_t raw_state, const void *d_data, size_t len, uint32_t *d_out_raw,
                            void *stream);

/* Host-CPU latency path for ONE short span (slicing-by-8; no device, never fails on valid
 * arguments): the same register semantics as tkv_crc32_update. No other entry point calls it. The
 * drop-in header include/frankie_crc32.hpp routes spans of at most TKV_DROPIN_HOST_MAX bytes here
 * (default 65536, the measured host/GPU crossover of one call), which covers the reference's per-put
 * record stamp (wal.cpp:54-57): 0.011 us for 36 bytes against ~11 us for a GPU round trip
 * (INTEGRATION.md §1). */
int tkv_crc32_update_host(uint32_t raw_state, const void *data, size_t len, uint32_t *out_raw);
int tkv_crc32c_update_host(uint32_t raw_state, const void *data, size_t len, uint32_t *out_raw);

/* The drop-in header's recovery after tkv_crc32[c]_update returned `gpu_status` != TKV_OK: the same
 * span recomputed on the host (the slicing-by-8 code of tkv_crc32_update_host), so crc32::update
 * keeps the reference's never-fail contract (crc32.cpp:9-16) for spans of any size on a node without
 * a usable GPU. Prints one warning per process on stderr (with gpu_status and tkv_last_error()) and
 * counts the call in tkv_debug_update_counts_n out[2]. Fails only on null pointers. */
int tkv_crc32_update_fallback(int gpu_status, uint32_t raw_state, const void *data, size_t len, uint32_t *out_raw);
int tkv_crc32c_update_fallback(int gpu_status, uint32_t raw_state, const void *data, size_t len,
                               uint32_t *out_raw);

/* CRC of the concatenation A || B from crc1 = CRC(A), crc2 = CRC(B) (finalized values) and
 * len2 = |B| (zlib's crc32_combine): Shift_len2(crc1) ^ crc2, GF(2) arithmetic on the 4-byte
 * values only (host, no data, no device). The reference has no equivalent; it serves callers that
 * checksum the pieces of one record or file separately (the multi-device batch does this itself). */
uint32_t tkv_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* ---- batch APIs (new: the reference has only per-record calls, wal.cpp:54-57,89-92) ------------ */

/* Irregular batch in device memory: block i is [d_base + d_offsets[i], + d_lengths[i]) (any
 * alignment, any length, blocks may overlap). d_out_final[i] = finalize() of the block continued
 * from d_init_raw[i] (NULL: every block starts from 0xFFFFFFFF). Asynchronous on `stream`; d_* must
 * stay valid until the stream has completed. */
int tkv_crc32_batch_device(const uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
                           const uint32_t *d_init_raw, uint32_t *d_out_final, uint64_t n, void *stream);

/* Uniform batch in device memory: block i is [d_base + i*stride, + len). Fast path for fixed-size
 * WAL/SSTable blocks (no prepass; 16-byte aligned blocks take the aligned kernel). */
int tkv_crc32_batch_uniform_device(const uint8_t *d_base, uint64_t stride, uint64_t len,
                                   const uint32_t *d_init_raw, uint32_t *d_out_final, uint64_t n,
                                   void *stream);

/* Irregular batch in HOST memory on the current device: blocks are streamed through pinned
 * staging buffers with H2D copy / kernel / D2H copy overlapped on two streams. Synchronous.
 * h_base may be pageable or pinned: when every block lies inside one pinned allocation mapped at
 * the same address on the device (hipHostMalloc, hipHostRegister), the kernels read the blocks in
 * place over PCIe and only offsets, lengths and results are copied. */
int tkv_crc32_batch_host(const uint8_t *h_base, const uint64_t *h_offsets, const uint32_t *h_lengths,
                         const uint32_t *h_init_raw, uint32_t *h_out_final, uint64_t n);

/* Same, split across `ndev` devices by bytes (one host thread and stream pair per device, no
 * collective). A block of at least 1 MiB that straddles the boundary between two devices' byte
 * shares is cut there; its pieces run on both devices and their registers combine on the host
 * (tkv_crc32_combine), so one huge block also spreads over the devices. */
int tkv_crc32_batch_host_multi(const int *devices, int ndev, const uint8_t *h_base, const uint64_t *h_offsets,
                               const uint32_t *h_lengths, const uint32_t *h_init_raw, uint32_t *h_out_final,
                               uint64_t n);

/* ---- WAL record verification (wal_entry::decode's CRC check, wal.cpp:63-96) ------------------- */

/* Verify every record of a slurped WAL image (host memory, wal_reader::open, wal.cpp:204-240):
 * copies it to the device, walks the record_len chain and checks all CRCs there, and reports the
 * number of leading good records in *n_good and the byte offset where decoding stopped in
 * *stop_offset. Returns TKV_OK when the whole image verified (clean EOF), TKV_CORRUPTED at the
 * first record whose length or CRC is bad (wal.cpp:68-96 order: header size, length, CRC). */
int tkv_wal_verify(const uint8_t *h_wal, uint64_t size, uint64_t *n_good, uint64_t *stop_offset);

/* Same for a WAL image already in DEVICE memory (synchronous on `stream`). The record_len chain is
 * walked on the device (speculative parallel walk, exact stitching), then one CRC batch and a
 * first-corruption search; results and status as tkv_wal_verify. tkv_wal_verify itself copies the
 * host image to the device and takes this path (host-thread walk only as the exact fallback). */
int tkv_wal_verify_device(const uint8_t *d_wal, uint64_t size, uint64_t *n_good, uint64_t *stop_offset,
                          void *stream);

/* Check n records of a WAL image already in DEVICE memory whose start offsets are known - the record
 * list of a walk, or the offsets a group-commit writer kept: record i starts at
 * d_img + d_rec_off[i] (u32 offsets, images up to 4 GiB). Each record gets wal_entry::decode's checks
 * (wal.cpp:63-127): at least 26 bytes left, record_len + 8 within the image, the CRC-32 of the
 * record_len payload bytes equal to the stored CRC, key and value inside the payload. The payload
 * length comes from the record's own header, read from the same 16-byte granules as its payload: no
 * lengths array, no prepass. *d_first_bad (device memory) = the index of the first record failing a
 * check, n when every record passes. d_crc (nullable, device): the computed finalized CRC of every
 * payload (0 for a record whose length check failed). max_payload is a dispatch hint (the longest
 * record_len the caller expects: one lane reads each record in a window of 4-8 16-byte granules sized
 * for it, 36-byte payloads in 4, up to 100 bytes in 8); longer payloads are still checked exactly,
 * 64 bytes at a time. Asynchronous on `stream`. */
int tkv_wal_check_records_device(const uint8_t *d_img, uint64_t size, const uint32_t *d_rec_off, uint64_t n,
                                 uint32_t max_payload, uint32_t *d_crc, uint64_t *d_first_bad, void *stream);

/* Stamp n records in place (host memory): for record i at h_buf + h_offsets[i] of total size
 * h_sizes[i] (>= 8), write crc32 of bytes [8, size) LE at offset 4 (wal.cpp:54-58). */
int tkv_wal_stamp(uint8_t *h_buf, const uint64_t *h_offsets, const uint32_t *h_sizes, uint64_t n);

/* ---- SSTable data-block stamping (the format is defined here) ----------- */

/* The reference writes sstable_data_block_header::crc32_ = 0 (sstable_writer.cpp:138-144) and never
 * reads it (sstable_reader.cpp:61-89), so this stamp is this library's format decision, not
 * reference behaviour ("parity unpinned"). A data-block image as get_data_block builds it
 * (sstable_writer.cpp:150-168) is varint(20) | header[20] | varint(n) | body[n], padded to the size
 * the index entry records (index_entry::data_block_size_, sstable_format.hpp:117-121); the header's
 * crc32_ field (sstable_format.hpp:97) therefore sits at image byte TKV_SST_CRC_OFFSET. The stamp is
 * the CRC-32 of the whole image [0, size) with those 4 bytes read as zero, stored little-endian in
 * the field. Images must be at least TKV_SST_MIN_IMAGE bytes and shorter than 4 GiB. */
#define TKV_SST_CRC_OFFSET 17u
#define TKV_SST_MIN_IMAGE 22u

/* Stamp n data-block images in place in a host buffer (an SSTable file image being written). */
int tkv_sst_stamp_blocks(uint8_t *h_file, const uint64_t *h_offsets, const uint64_t *h_sizes, uint64_t n);

/* Verify n images of a host buffer; *n_bad = number of mismatching images, *first_bad = index of
 * the first (n when none). Returns TKV_OK or TKV_CORRUPTED (read_data_block's corrupted status,
 * sstable_reader.cpp:73-86). */
int tkv_sst_verify_blocks(const uint8_t *h_file, const uint64_t *h_offsets, const uint64_t *h_sizes, uint64_t n,
                          uint64_t *n_bad, uint64_t *first_bad);

/* Device-resident images: d_out[i] = the stamp value of image i (CRC with the field read as zero),
 * whatever the field holds now. With store != 0 the value is also written into the field (stamping
 * on the device). Asynchronous on `stream`. */
int tkv_sst_block_crcs_device(uint8_t *d_file, const uint64_t *d_offsets, const uint32_t *d_sizes, uint32_t *d_out,
                              uint64_t n, int store, void *stream);

/* ---- SSTable index image + footer stamping (format defined here; parity unpinned) ------------------
 * research/12-integrity-crash-consistency.md §5 asks for a checksum over the index image and the
 * footer, kept in the footer's existing crc32_ field (sstable_format.hpp:129-135). The reference
 * writes only 8 footer bytes (kFooterSize, sstable_format.hpp:140), and in the order
 * (index_size, index_offset) (sstable_writer.cpp get_footer) while decode_footer reads
 * (index_offset, index_size) (sstable_format.cpp:99-106). The footer here is the full 20-byte struct
 * in declaration order, little-endian:
 *     u32 index_offset | u32 index_size | u32 bloom_offset | u32 bloom_size | u32 crc32_
 * and crc32_ = CRC-32 of (index image || footer bytes [0, 16)), i.e. the index bytes as get_index
 * lays them out (sstable_writer.cpp get_index) followed by the footer's first four fields. */
#define TKV_SST_FOOTER_SIZE 20u
#define TKV_SST_FOOTER_CRC_OFFSET 16u

/* Write the crc32_ field of h_footer (20 bytes; its first 16 bytes already filled) from the index
 * image [h_index, h_index + index_size) (index_size may be 0). */
int tkv_sst_stamp_footer(const uint8_t *h_index, uint64_t index_size, uint8_t *h_footer);

/* Check the stored crc32_ of h_footer against the index image: TKV_OK or TKV_CORRUPTED. */
int tkv_sst_verify_footer(const uint8_t *h_index, uint64_t index_size, const uint8_t *h_footer);

/* ---- CRC-32C (Castagnoli) — SURVEY.md §8f rank 4 ------------------------------------------------ */

/* Same engine and kernels with the tables of the Castagnoli polynomial (reflected 0x82F63B78,
 * init/xorout 0xFFFFFFFF: iSCSI, RFC 3720 §B.4). Not reference behaviour; offered for a
 * format-versioned alternative. Arguments and conventions as for the tkv_crc32_* functions. */
#define TKV_CRC32C_POLYNOMIAL 0x82F63B78u
int tkv_crc32c_update(uint32_t raw_state, const void *data, size_t len, uint32_t *out_raw);
int tkv_crc32c_update_device(uint32_t raw_state, const void *d_data, size_t len, uint32_t *d_out_raw,
                             void *stream);
int tkv_crc32c_batch_device(const uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
                            const uint32_t *d_init_raw, uint32_t *d_out_final, uint64_t n, void *stream);
int tkv_crc32c_batch_uniform_device(const uint8_t *d_base, uint64_t stride, uint64_t len,
                                    const uint32_t *d_init_raw, uint32_t *d_out_final, uint64_t n,
                                    void *stream);
int tkv_crc32c_batch_host(const uint8_t *h_base, const uint64_t *h_offsets, const uint32_t *h_lengths,
                          const uint32_t *h_init_raw, uint32_t *h_out_final, uint64_t n);
int tkv_crc32c_batch_host_multi(const int *devices, int ndev, const uint8_t *h_base, const uint64_t *h_offsets,
                                const uint32_t *h_lengths, const uint32_t *h_init_raw, uint32_t *h_out_final,
                                uint64_t n);
uint32_t tkv_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* ---- synthetic data (SURVEY.md §8d generator; bench/test inputs) ------------------------------- */

int tkv_fill_synthetic_uniform(uint8_t *d_dst, uint64_t stride, uint64_t len, uint64_t first_block,
                               uint64_t nblocks, uint64_t seed, void *stream);
int tkv_fill_synthetic_blocks(uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
                              uint64_t first_block, uint64_t nblocks, uint64_t seed, void *stream);

/* ---- introspection for tests (no GPU needed) --------------------------------------------------- */

/* Copy the constant tables the kernels use (layout of tkv::DeviceTables) into `out`; returns the
 * byte size needed (call with out = NULL to query). */
size_t tkv_debug_tables(void *out, size_t cap);
/* Same for any reflected polynomial (TKV_CRC32_POLYNOMIAL, TKV_CRC32C_POLYNOMIAL). */
size_t tkv_debug_tables_poly(uint32_t poly, void *out, size_t cap);

/* Host GF(2) helpers the decomposition rests on: a*b mod P and x^(8n) mod P, reflected. */
uint32_t tkv_debug_multmodp(uint32_t a, uint32_t b);
/* The record chain tkv_wal_verify walks (host only, no CRC): writes up to `cap` record start offsets,
 * the offset after the last record and whether a header did not fit; returns the record count. */
size_t tkv_debug_wal_chain(const uint8_t *h_wal, uint64_t size, uint64_t *out_pos, size_t cap, uint64_t *end,
                           int *err);
uint32_t tkv_debug_x8nmodp(uint64_t nbytes);
/* The split tkv_crc32_batch_host_multi plans for `ndev` devices (host only, no device, no CRC):
 * writes up to `cap` pieces as 6 x u64 records {device, block, byte offset, length, initial raw
 * register, starts its block} in device order, pieces in block order; returns the piece count. */
size_t tkv_debug_multi_plan(int ndev, const uint64_t *h_offsets, const uint32_t *h_lengths,
                            const uint32_t *h_init_raw, uint64_t n, uint64_t *out_rec, size_t cap);
/* The host combine step of that plan: given each piece's finalized CRC (in the order
 * tkv_debug_multi_plan lists them), writes every block's finalized CRC. 4-byte GF(2) arithmetic on
 * registers only, for the reflected polynomial `poly`. */
int tkv_debug_multi_combine(uint32_t poly, int ndev, const uint64_t *h_offsets, const uint32_t *h_lengths,
                            const uint32_t *h_init_raw, uint64_t n, const uint32_t *piece_final,
                            uint32_t *h_out_final);
/* Update calls of the calling thread so far: out[0] through tkv_crc32[c]_update_host (the drop-in's
 * short-span host path), out[1] through tkv_crc32[c]_update (the GPU). (The round-3 entry point:
 * two words.) */
void tkv_debug_update_counts(uint64_t out[2]);
/* The same counters into out[0..n) (n may be smaller or larger than the count), plus out[2] = calls
 * through tkv_crc32[c]_update_fallback (host recomputes after a failed GPU update). Returns the number
 * of counters (3). */
size_t tkv_debug_update_counts_n(uint64_t *out, size_t n);
/* What the calling thread's last tkv_wal_verify / tkv_wal_verify_device did: out[0] = device
 * rounds (the sweep, then one per fix-up round), out[1] = 1 when it handed the image to the exact
 * host-thread walk (only a host image the device cannot hold), out[2] = 1 when a host image was
 * copied to the device, out[3] = 1 when the sweep needed no fix-up (0 when no device round ran). */
void tkv_debug_wal_last(uint64_t out[4]);
/* Per fix-up round of the calling thread's last device WAL verify, six words each: failing chunk
 * boundaries found, fix-up tasks launched, the longest task's range and all tasks' ranges (regions a
 * task may walk), the most regions one task walked and all regions walked. Writes up to n words;
 * returns the number available (0 when the sweep needed no fix-up). */
size_t tkv_debug_wal_rounds(uint64_t *out, size_t n);
/* Which path the last irregular batch on `stream` took: 1 = byte-stream row walk (blocks back to
 * back, each at least 64 bytes), 0 = general row walk; -1 on error. Synchronizes
 * the stream. */
int tkv_debug_irregular_mode(void *stream);
/* Which of crc_stream's general-path phases the last irregular batch on `stream` ran (0 in stream
 * mode): bit 0 the lane phase (blocks <= 64 B), bits 1 / 2 the 4- / 8-lane group passes (65-256 /
 * 257-512 B); -1 on error. Synchronizes the stream. */
int tkv_debug_irregular_phases(void *stream);
/* Which path folded the last irregular batch on `stream`: 0 = the one-pass kernel with one lane per
 * block only (crc_list_lanes: every block <= 64 B), 1 = the one-pass kernel with its packed mode in
 * at least one wave (every block <= 1 KiB), 2 = the general path after the one-pass kernel handed the
 * batch on (a block over 1 KiB), 3 = the general path alone (fewer than 256 K blocks, per-block
 * initial registers, tkv_debug_set_one_pass(0) or tkv_debug_set_stream_groups(1)); -1 on error.
 * Synchronizes the stream. */
int tkv_debug_irregular_path(void *stream);
/* Waves of the one-pass lane kernel (crc_list_lanes) for an irregular batch of nblocks on the current
 * device: wave w takes its 64-block steps [w TS / W, (w + 1) TS / W), TS = ceil(nblocks / 64). 0 when
 * no device is usable. */
uint32_t tkv_debug_list_lanes_waves(uint64_t nblocks);
/* The small-block lists of the last irregular batch on `stream` (all 0 in stream mode): out[0] =
 * blocks of at most 1 KiB the small-block phase folds (those no lane or group pass took), out[1] =
 * how many of them are at most 256 bytes (4-lane groups), out[2] = 257-512 bytes (8-lane groups; the
 * rest take 16-lane groups). Returns 0, or -1 on error. Synchronizes the stream. */
int tkv_debug_irregular_lists(void *stream, uint32_t out[3]);
/* Host batches from pinned host memory are read in place by the kernels (zero copy) unless this is
 * 0 (then they take the staged copy pipeline, as pageable memory does). Returns the previous
 * setting. Default 1; the environment variable TKV_HOST_MAPPED=0 sets 0 at load time. */
int tkv_debug_set_host_mapped(int enable);
/* Back-to-back irregular batches with a 4096-block scan tile of at least 1024 blocks of at most
 * 1 KiB and at most 1024 rows (4 MiB) of larger blocks take the general path, whose group passes and
 * small phase fold those blocks, unless this is 1: then they may take the byte-stream
 * walk as before round 4 (kept so its many-ends-per-row shapes stay under test). Returns the previous
 * setting. Default 0. */
int tkv_debug_set_stream_groups(int enable);
/* Irregular batches of at least 256 K blocks with the default register start with the one-pass
 * kernel (crc_list_lanes and its packed mode) unless this is 0: then they take the general path alone, as
 * smaller batches do (kept so the general path's large-batch shapes stay under test). Returns the
 * previous setting. Default 1. */
int tkv_debug_set_one_pass(int enable);


#ifdef __cplusplus
}
#endif

#endif /* TKV_CRC32_H */
