/*
 * oracle/crc32_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of lnikon/tinykvpp's CRC-32 (frankie::core::crc32), used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg to check and time the HIP path.
 * Nothing in tinykvpp_amd/ links or calls this file; the product fails loudly without its
 * HIP library instead of falling back here.
 *
 * Parity pinning: tests/test_oracle.py checks every function below against
 *   - the known answers of /root/reference/test/crc32_test.cpp:81-124,
 *   - the WAL records of test/wal_test.cpp (fixtures in tests/golden/),
 *   - outputs of the reference's own src/core/crc32.cpp compiled into oracle/_ref/ (when built),
 *   - Python's zlib.crc32 (an independent CRC-32/ISO-HDLC implementation).
 *
 * Algorithm (follows /root/reference/src/core/crc32.hpp:9-30 and crc32.cpp:9-22):
 *   reflected polynomial 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF,
 *   byte-at-a-time Sarwate table: crc = (crc >> 8) ^ T[(byte ^ crc) & 0xFF].
 *
 * Synthetic data generator: byte j of block b is LE byte (j % 8) of
 * splitmix64((b << 24) ^ (j >> 3) ^ (seed << 56)).  Zipf lengths for cfg4 as in §8d.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_POLY 0xEDB88320u   /* crc32.hpp:11 kCRC32Polynomial */
#define ORACLE_INIT 0xFFFFFFFFu   /* crc32.hpp:9  kCRC32DefaultValue */

static uint32_t g_table[256];
static int g_table_ready = 0;

/* crc32.hpp:16-30 generate_crc32_table(): 8 shift/xor rounds per entry. */
void oracle_table(uint32_t out[256]) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int bit = 0; bit < 8; ++bit) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
    out[i] = c;
  }
}

static void ensure_table(void) {
  if (!g_table_ready) {
    oracle_table(g_table);
    g_table_ready = 1;
  }
}

/* crc32.cpp:9-16 crc32::update — continues from raw (pre-xorout) state, no pre/post XOR. */
uint32_t oracle_update(uint32_t raw, const uint8_t *p, size_t n) {
  ensure_table();
  for (size_t i = 0; i < n; ++i) raw = (raw >> 8) ^ g_table[(p[i] ^ raw) & 0xFFu];
  return raw;
}

/* crc32{}.update(span).finalize() — crc32.hpp:48 default state, crc32.cpp:19 finalize. */
uint32_t oracle_crc32(const uint8_t *p, size_t n) { return oracle_update(ORACLE_INIT, p, n) ^ ORACLE_INIT; }

/* ---- synthetic generator ---- */
uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Bytes [off, off+n) of synthetic block b (one splitmix64 per aligned 8-byte group). */
void oracle_fill(uint64_t seed, uint64_t b, uint64_t off, uint8_t *out, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint64_t j = off + i;
    uint64_t w = oracle_splitmix64((b << 24) ^ (j >> 3) ^ (seed << 56));
    for (unsigned k = (unsigned)(j & 7); k < 8 && i < n; ++k, ++i) out[i] = (uint8_t)(w >> (8 * k));
  }
}

/* Sarwate CRC (init/xorout per crc32.hpp) of synthetic blocks [first, first+count) of length len
 * each; out[i] = finalize() value.  Generates the bytes in 64 KiB slabs. */
void oracle_crc_synthetic(uint64_t seed, uint64_t first, uint64_t count, uint64_t len, uint32_t *out) {
  uint8_t buf[65536];
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t b = first + i;
    uint32_t raw = ORACLE_INIT;
    for (uint64_t off = 0; off < len; off += sizeof(buf)) {
      size_t n = (size_t)((len - off) < sizeof(buf) ? (len - off) : sizeof(buf));
      oracle_fill(seed, b, off, buf, n);
      raw = oracle_update(raw, buf, n);
    }
    out[i] = raw ^ ORACLE_INIT;
  }
}

/* Zipf block length for cfg4: class k in [0,12], S = 256 * 2^k, P(k) ∝ 1/(k+1),
 * r = splitmix64((seed<<56) ^ (1<<55) ^ b), u = (r & 0xFFFFFFFF) / 2^32 against the CDF,
 * len = max(256, S - ((r >> 32) mod (S/2))). */
uint64_t oracle_zipf_len(uint64_t seed, uint64_t b) {
  double w[13], tot = 0.0, cdf = 0.0;
  for (int k = 0; k < 13; ++k) { w[k] = 1.0 / (double)(k + 1); tot += w[k]; }
  uint64_t r = oracle_splitmix64((seed << 56) ^ (1ull << 55) ^ b);
  double u = (double)(r & 0xFFFFFFFFull) / 4294967296.0;
  int k = 12;
  for (int i = 0; i < 13; ++i) {
    cdf += w[i] / tot;
    if (u < cdf) { k = i; break; }
  }
  uint64_t S = 256ull << k;
  uint64_t len = S - ((r >> 32) % (S / 2));
  return len < 256 ? 256 : len;
}

void oracle_zipf_lengths(uint64_t seed, uint64_t first, uint64_t count, uint64_t *out) {
  for (uint64_t i = 0; i < count; ++i) out[i] = oracle_zipf_len(seed, first + i);
}

/* CRC of synthetic blocks with per-block lengths (cfg4). */
void oracle_crc_synthetic_lens(uint64_t seed, uint64_t first, uint64_t count, const uint64_t *lens,
                               uint32_t *out) {
  for (uint64_t i = 0; i < count; ++i) oracle_crc_synthetic(seed, first + i, 1, lens[i], out + i);
}

/* Batch over caller-provided host buffers: out[i] = finalize(update(init_i, base+off[i], len[i])). */
void oracle_crc_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                      const uint32_t *init_raw, uint64_t n, uint32_t *out) {
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t s = init_raw ? init_raw[i] : ORACLE_INIT;
    out[i] = oracle_update(s, base + offsets[i], lengths[i]) ^ ORACLE_INIT;
  }
}

/* ---- CRC-32C (not in the reference) ----
 * Published algorithm: CRC-32C / Castagnoli, RFC 3720 §B.4 (iSCSI): reflected polynomial
 * 0x82F63B78, init 0xFFFFFFFF, xorout 0xFFFFFFFF, same byte-at-a-time Sarwate loop as
 * crc32.cpp:9-16 with the other table. Pinned by the RFC 3720 §B.4 vectors and the catalogue check
 * value crc32c("123456789") = 0xE3069283 in tests/test_oracle.py. */
#define ORACLE_POLY_C 0x82F63B78u
static uint32_t g_table_c[256];
static int g_table_c_ready = 0;

void oracle_table_c(uint32_t out[256]) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int bit = 0; bit < 8; ++bit) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY_C : (c >> 1);
    out[i] = c;
  }
}

uint32_t oracle_update_c(uint32_t raw, const uint8_t *p, size_t n) {
  if (!g_table_c_ready) {
    oracle_table_c(g_table_c);
    g_table_c_ready = 1;
  }
  for (size_t i = 0; i < n; ++i) raw = (raw >> 8) ^ g_table_c[(p[i] ^ raw) & 0xFFu];
  return raw;
}

uint32_t oracle_crc32c(const uint8_t *p, size_t n) { return oracle_update_c(ORACLE_INIT, p, n) ^ ORACLE_INIT; }

/* ---- SSTable data-block stamp (format of include/tkv_crc32.h; parity unpinned) ----
 * Image = varint(20) | header[20] | varint(n) | body (sstable_writer.cpp:150-168); the header's
 * crc32_ (sstable_format.hpp:97) is at image byte 17. Stamp = crc32 of the image with those 4 bytes
 * read as zero: computed here literally, by feeding zeros in their place. */
uint32_t oracle_sst_stamp(const uint8_t *img, size_t size) {
  static const uint8_t zeros[4] = {0, 0, 0, 0};
  if (size < 22) return 0;
  uint32_t raw = oracle_update(ORACLE_INIT, img, 17);
  raw = oracle_update(raw, zeros, 4);
  raw = oracle_update(raw, img + 21, size - 21);
  return raw ^ ORACLE_INIT;
}

/* ---- WAL records (wal.cpp:19-130; layout wal.hpp:21-27) ----
 * Record = u32 record_len | u32 crc32 | u8 op | u64 seq | u8 tombstone | u32 key_len | u32 value_len |
 * key | value, little-endian and packed (26-byte header); record_len = size - 8; the CRC covers
 * [8, 8 + record_len). */
#define ORACLE_WAL_META 26u /* wal.hpp kMetadataSize */

static uint32_t rd_le32(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

/* wal.cpp:54-58 (wal_entry::encode's stamp): for each record at offs[i], crc32 of its record_len bytes
 * after the 8-byte prefix, stored little-endian at offs[i] + 4. */
void oracle_wal_stamp(uint8_t *img, const uint64_t *offs, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t *r = img + offs[i];
    uint32_t c = oracle_crc32(r + 8, rd_le32(r));
    r[4] = (uint8_t)c;
    r[5] = (uint8_t)(c >> 8);
    r[6] = (uint8_t)(c >> 16);
    r[7] = (uint8_t)(c >> 24);
  }
}

/* engine::create's recovery loop (engine.cpp:31-53) over a slurped image (wal.cpp:204-240): decode
 * (wal.cpp:63-130) record after record until eof or the first failure. Checks in the reference's
 * order: eof on an empty view (:64-66); corrupted when fewer than 26 bytes remain (:68-70), when
 * record_len + 8 exceeds the view (:80-84; computed in 64 bits here, where the reference's u32 sum can
 * wrap into undefined behaviour), on a CRC mismatch (:86-93) and when key_len + value_len overrun the
 * record (:115-119). Returns 0 at a clean eof, 1 when corrupted; *n_good = records decoded, *stop =
 * the offset the view is parked on (the failing record's start, or size). */
int oracle_wal_decode(const uint8_t *img, uint64_t size, uint64_t *n_good, uint64_t *stop) {
  uint64_t p = 0, n = 0;
  int bad = 0;
  while (p < size) {
    if (size - p < ORACLE_WAL_META) { bad = 1; break; }
    const uint64_t rl = rd_le32(img + p);
    if (rl + 8u > size - p) { bad = 1; break; }
    if (oracle_crc32(img + p + 8, (size_t)rl) != rd_le32(img + p + 4)) { bad = 1; break; }
    const uint64_t kl = rd_le32(img + p + 18), vl = rd_le32(img + p + 22);
    if (ORACLE_WAL_META + kl + vl > 8u + rl) { bad = 1; break; }
    p += 8u + rl;
    ++n;
  }
  *n_good = n;
  *stop = p;
  return bad;
}

/* ---- Slicing-by-8 (NOT the reference algorithm; CPU comparison row only) ----
 * SURVEY.md §8d's optional "slicing-by-8 CPU row, clearly labelled 'not reference'": the same
 * CRC-32/ISO-HDLC eight bytes per step with tables T_k[i] = Shift_k o T (Intel's slicing-by-8).
 * bench.py times it beside the reference on the same bytes; tests/test_oracle.py checks it against
 * oracle_update. Never part of the product path. */
static uint32_t g_s8[8][256];
static int g_s8_ready = 0;

static void ensure_s8(void) {
  if (g_s8_ready) return;
  ensure_table();
  for (int i = 0; i < 256; ++i) {
    g_s8[0][i] = g_table[i];
    for (int k = 1; k < 8; ++k) g_s8[k][i] = (g_s8[k - 1][i] >> 8) ^ g_table[g_s8[k - 1][i] & 0xFFu];
  }
  g_s8_ready = 1;
}

uint32_t oracle_update_s8(uint32_t raw, const uint8_t *p, size_t n) {
  ensure_s8();
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= raw;
    raw = g_s8[7][lo & 0xFFu] ^ g_s8[6][(lo >> 8) & 0xFFu] ^ g_s8[5][(lo >> 16) & 0xFFu] ^ g_s8[4][lo >> 24] ^
          g_s8[3][hi & 0xFFu] ^ g_s8[2][(hi >> 8) & 0xFFu] ^ g_s8[1][(hi >> 16) & 0xFFu] ^ g_s8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) raw = (raw >> 8) ^ g_table[(*p++ ^ raw) & 0xFFu];
  return raw;
}

void oracle_crc_batch_s8(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                         uint32_t *out) {
  for (uint64_t i = 0; i < n; ++i) out[i] = oracle_update_s8(ORACLE_INIT, base + offsets[i], lengths[i]) ^ ORACLE_INIT;
}

/* Fast synthetic-block CRCs for the full-size checks (test side only): the §8d generator's 8-byte
 * words fed straight into the slicing-by-8 step above, no byte buffer. Same results as
 * oracle_crc_synthetic (tests/test_oracle.py checks both against each other and the golden
 * fixtures); ~10x faster, so a CPU test can checksum a whole 4 GiB rank shard. */
void oracle_crc_synthetic_s8(uint64_t seed, uint64_t first, uint64_t count, uint64_t len, uint32_t *out) {
  ensure_s8();
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t b = first + i;
    uint32_t raw = ORACLE_INIT;
    uint64_t j8 = 0;
    for (; (j8 + 1) * 8 <= len; ++j8) {
      uint64_t w = oracle_splitmix64((b << 24) ^ j8 ^ (seed << 56));
      uint32_t lo = (uint32_t)w ^ raw, hi = (uint32_t)(w >> 32);
      raw = g_s8[7][lo & 0xFFu] ^ g_s8[6][(lo >> 8) & 0xFFu] ^ g_s8[5][(lo >> 16) & 0xFFu] ^ g_s8[4][lo >> 24] ^
            g_s8[3][hi & 0xFFu] ^ g_s8[2][(hi >> 8) & 0xFFu] ^ g_s8[1][(hi >> 16) & 0xFFu] ^ g_s8[0][hi >> 24];
    }
    if (j8 * 8 < len) {
      uint64_t w = oracle_splitmix64((b << 24) ^ j8 ^ (seed << 56));
      for (uint64_t k = 0; j8 * 8 + k < len; ++k) raw = (raw >> 8) ^ g_table[((uint8_t)(w >> (8 * k)) ^ raw) & 0xFFu];
    }
    out[i] = raw ^ ORACLE_INIT;
  }
}

void oracle_crc_synthetic_lens_s8(uint64_t seed, uint64_t first, uint64_t count, const uint64_t *lens,
                                  uint32_t *out) {
  for (uint64_t i = 0; i < count; ++i) oracle_crc_synthetic_s8(seed, first + i, 1, lens[i], out + i);
}
