/* ORACLE TEST INFRASTRUCTURE -- never part of the shipped product.
 *
 * Plain-C restatement of the snappy raw format as the reference's COMPRESSING
 * filter uses it (compressing.h:8-37 -> SArray::CompressTo / UncompressFrom,
 * shared_array_inl.h:232-255).  snappy is a third-party dependency the
 * reference does not vendor (script/install_third.sh clones it at HEAD); the
 * build container has snappy 1.1.8 (/opt/conda/lib/libsnappy.so.1), which
 * oracle/_ref links and which pins this restatement (tests/test_oracle.py,
 * tests/golden/snappy.npz).  The published 1.1.8 algorithm, restated:
 *
 *   stream   = varint32(n) ++ fragment(0) ++ fragment(1) ++ ...
 *   fragment = greedy LZ77 parse of the next min(64 KiB, rest) input bytes,
 *              independent of every other fragment: a zeroed uint16 hash
 *              table of T = pow2 >= size clamped to [256, 16384] entries,
 *              hash(u32 at p) = (u32 * 0x1e35a7bd) >> (32 - log2 T), the
 *              "skip" heuristic (probe stride = skip++/32 grows by skip>>5),
 *              matches extended byte-exactly, 15-byte input margin.
 *   literal  : tag (len-1)<<2 (len <= 60) or 60+k with k LE length bytes
 *   copy     : len 4..11 & offset < 2048 -> 2 bytes (COPY_1), else 3 bytes
 *              (COPY_2); runs >= 68 are split 64 + ..., 64 < len < 68 -> 60 + rest
 *
 * Decoder validity follows snappy's SnappyDecoder/SnappyArrayWriter: varint
 * of at most 5 bytes (5th < 16), every tag complete, literals inside the input,
 * copies with 1 <= offset <= produced, never beyond the declared length, and
 * output == declared length at the end of the input.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define SNAP_BLOCK 65536u
#define SNAP_MAX_TABLE 16384u
#define SNAP_MUL 0x1e35a7bdu

static inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

static inline uint32_t hash32(uint32_t v, int shift) { return (v * SNAP_MUL) >> shift; }

static inline int log2_floor(uint32_t v) { return 31 - __builtin_clz(v); }

size_t port_snappy_max_compressed(size_t n) { return 32 + n + n / 6; }

static uint8_t* emit_literal(uint8_t* op, const uint8_t* lit, size_t len) {
  size_t n = len - 1;
  if (n < 60) {
    *op++ = (uint8_t)(n << 2);
  } else {
    int count = (log2_floor((uint32_t)n) >> 3) + 1;
    *op++ = (uint8_t)((59 + count) << 2);
    for (int i = 0; i < count; ++i) *op++ = (uint8_t)(n >> (8 * i));
  }
  memcpy(op, lit, len);
  return op + len;
}

static uint8_t* emit_copy_le64(uint8_t* op, size_t offset, size_t len) {
  if (len < 12 && offset < 2048) {
    *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
    *op++ = (uint8_t)(offset & 0xff);
  } else {
    *op++ = (uint8_t)(2 + ((len - 1) << 2));
    *op++ = (uint8_t)(offset & 0xff);
    *op++ = (uint8_t)(offset >> 8);
  }
  return op;
}

static uint8_t* emit_copy(uint8_t* op, size_t offset, size_t len) {
  while (len >= 68) {
    op = emit_copy_le64(op, offset, 64);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_le64(op, offset, 60);
    len -= 60;
  }
  return emit_copy_le64(op, offset, len);
}

static size_t match_len(const uint8_t* s1, const uint8_t* s2, const uint8_t* s2_limit) {
  size_t m = 0;
  while (s2 + m < s2_limit && s1[m] == s2[m]) ++m;
  return m;
}

uint32_t port_snappy_table_size(size_t n) {
  uint32_t t = 256;
  while (t < SNAP_MAX_TABLE && t < n) t <<= 1;
  return t;
}

/* One fragment; returns the bytes written at op. */
size_t port_snappy_fragment(const uint8_t* in, size_t n, uint8_t* out) {
  static uint16_t table[SNAP_MAX_TABLE];
  const uint32_t tsize = port_snappy_table_size(n);
  const int shift = 32 - log2_floor(tsize);
  memset(table, 0, tsize * sizeof(uint16_t));
  const uint8_t* ip = in;
  const uint8_t* ip_end = in + n;
  const uint8_t* next_emit = in;
  uint8_t* op = out;
  if (n >= 15) {
    const uint8_t* ip_limit = in + n - 15;
    uint32_t next_hash = hash32(ld32(++ip), shift);
    for (;;) {
      uint32_t skip = 32;
      const uint8_t* next_ip = ip;
      const uint8_t* cand;
      do {
        ip = next_ip;
        uint32_t h = next_hash;
        uint32_t step = skip >> 5;
        skip += step;
        next_ip = ip + step;
        if (next_ip > ip_limit) goto remainder;
        next_hash = hash32(ld32(next_ip), shift);
        cand = in + table[h];
        table[h] = (uint16_t)(ip - in);
      } while (ld32(ip) != ld32(cand));
      op = emit_literal(op, next_emit, (size_t)(ip - next_emit));
      uint32_t cand_bytes;
      uint32_t cur_bytes;
      do {
        const uint8_t* base = ip;
        size_t matched = 4 + match_len(cand + 4, ip + 4, ip_end);
        ip += matched;
        op = emit_copy(op, (size_t)(base - cand), matched);
        next_emit = ip;
        if (ip >= ip_limit) goto remainder;
        table[hash32(ld32(ip - 1), shift)] = (uint16_t)(ip - in - 1);
        cur_bytes = ld32(ip);
        uint32_t ch = hash32(cur_bytes, shift);
        cand = in + table[ch];
        cand_bytes = ld32(cand);
        table[ch] = (uint16_t)(ip - in);
      } while (cur_bytes == cand_bytes);
      next_hash = hash32(ld32(ip + 1), shift);
      ++ip;
    }
  }
remainder:
  if (next_emit < ip_end) op = emit_literal(op, next_emit, (size_t)(ip_end - next_emit));
  return (size_t)(op - out);
}

size_t port_snappy_compress(const void* src, size_t n, void* dst) {
  const uint8_t* in = (const uint8_t*)src;
  uint8_t* op = (uint8_t*)dst;
  uint32_t v = (uint32_t)n;
  while (v >= 128) {
    *op++ = (uint8_t)(v | 128);
    v >>= 7;
  }
  *op++ = (uint8_t)v;
  for (size_t pos = 0; pos < n; pos += SNAP_BLOCK) {
    size_t len = n - pos < SNAP_BLOCK ? n - pos : SNAP_BLOCK;
    op += port_snappy_fragment(in + pos, len, op);
  }
  return (size_t)(op - (uint8_t*)dst);
}

/* 0 ok (*len set), -1 malformed varint */
int port_snappy_uncompressed_length(const void* src, size_t n, size_t* len) {
  const uint8_t* p = (const uint8_t*)src;
  uint32_t v = 0;
  for (int i = 0; i < 5; ++i) {
    if ((size_t)i >= n) return -1;
    uint32_t b = p[i];
    if (i == 4 && b >= 16) return -1;
    v |= (b & 127u) << (7 * i);
    if (b < 128) {
      *len = v;
      return 0;
    }
  }
  return -1;
}

static size_t varint_bytes(const uint8_t* p) {
  size_t i = 0;
  while (p[i] & 128) ++i;
  return i + 1;
}

/* Same return codes as psref_snappy_uncompress: -1 header, -2 cap, -3 body. */
int port_snappy_uncompress(const void* src, size_t n, void* dst, size_t cap, size_t* out_len) {
  const uint8_t* ip = (const uint8_t*)src;
  size_t d;
  if (port_snappy_uncompressed_length(src, n, &d) != 0) return -1;
  *out_len = d;
  if (d > cap) return -2;
  const uint8_t* end = ip + n;
  ip += varint_bytes(ip);
  uint8_t* out = (uint8_t*)dst;
  size_t produced = 0;
  while (ip < end) {
    uint8_t c = *ip++;
    if ((c & 3) == 0) {
      size_t len = (c >> 2) + 1;
      if (len > 60) {
        size_t k = len - 60;
        if ((size_t)(end - ip) < k) return -3;
        len = 0;
        for (size_t i = 0; i < k; ++i) len |= (size_t)ip[i] << (8 * i);
        len += 1;
        ip += k;
      }
      if ((size_t)(end - ip) < len) return -3;
      if (d - produced < len) return -3;
      memcpy(out + produced, ip, len);
      produced += len;
      ip += len;
    } else {
      size_t len, off, k = (c & 3) == 1 ? 1 : (c & 3) == 2 ? 2 : 4;
      if ((size_t)(end - ip) < k) return -3;
      if ((c & 3) == 1) {
        len = 4 + ((c >> 2) & 7);
        off = ((size_t)(c >> 5) << 8) | ip[0];
      } else {
        len = (c >> 2) + 1;
        off = 0;
        for (size_t i = 0; i < k; ++i) off |= (size_t)ip[i] << (8 * i);
      }
      ip += k;
      if (off == 0 || off > produced || d - produced < len) return -3;
      for (size_t i = 0; i < len; ++i) out[produced + i] = out[produced + i - off];
      produced += len;
    }
  }
  return produced == d ? 0 : -3;
}
