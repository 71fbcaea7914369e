/*
 * lz4_oracle.c -- TEST INFRASTRUCTURE ONLY (see lz4_oracle.h).
 *
 * A plain-C restatement of the LZ4 block format and of the default LZ4
 * compressor (LZ4 1.9.x LZ4_compress_default: acceleration 1, a fresh zeroed
 * state, 16-bit position table with 4-byte hashing below 65,547 input bytes,
 * 32-bit position table with 5-byte hashing above), written from the
 * published format description and algorithm.  The reference
 * (/root/reference) registers no LZ4 handler and ships no LZ4 code
 * (flare/rpc/options.proto:74 only names COMPRESS_TYPE_LZ4), so parity is
 * pinned against the image's system liblz4 1.9.3 in tests/test_lz4.py, not
 * against the reference.
 */
#include "lz4_oracle.h"

#include <string.h>

#define MINMATCH 4
#define MFLIMIT 12
#define LASTLITERALS 5
#define MIN_LENGTH (MFLIMIT + 1)
#define HASHLOG 12
#define SKIP_TRIGGER 6
#define DISTANCE_MAX 65535
#define LIMIT_64K (65536 + MFLIMIT - 1)
#define RUN_MASK 15
#define ML_MASK 15

static uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

static uint64_t rd64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

size_t lz4o_max_compressed_length(size_t n) { return n + n / 255 + 16; }

/* position hash: 4 bytes into 13 bits (small inputs) or 5 bytes into 12 bits */
static uint32_t hash_at(const uint8_t *p, int small) {
  if (small) return (rd32(p) * 2654435761u) >> (32 - (HASHLOG + 1));
  return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - HASHLOG));
}

static uint8_t *put_length(uint8_t *op, size_t len) {
  for (; len >= 255; len -= 255) *op++ = 255;
  *op++ = (uint8_t)len;
  return op;
}

size_t lz4o_compress_block(const uint8_t *src, size_t n, uint8_t *dst) {
  if (n > LZ4O_MAX_INPUT) return 0;
  const int small = n < LIMIT_64K;
  uint16_t t16[1 << (HASHLOG + 1)];
  uint32_t t32[1 << HASHLOG];
  memset(t16, 0, sizeof t16);
  memset(t32, 0, sizeof t32);
#define GET(h) (small ? (uint32_t)t16[h] : t32[h])
#define PUT(h, v) do { if (small) t16[h] = (uint16_t)(v); else t32[h] = (uint32_t)(v); } while (0)

  uint8_t *op = dst;
  size_t anchor = 0, ip = 0;
  if (n >= MIN_LENGTH) {
    const size_t mflimit1 = n - MFLIMIT + 1; /* a match starts before this */
    const size_t matchlimit = n - LASTLITERALS;
    PUT(hash_at(src, small), 0);
    ip = 1;
    uint32_t fh = hash_at(src + ip, small);
    for (;;) {
      size_t match;
      /* find a match: probe positions with a growing step after misses */
      {
        size_t fwd = ip;
        unsigned step = 1, nb = 1u << SKIP_TRIGGER;
        for (;;) {
          const uint32_t h = fh;
          const size_t cur = fwd;
          const uint32_t mi = GET(h);
          ip = fwd;
          fwd += step;
          step = nb++ >> SKIP_TRIGGER;
          if (fwd > mflimit1) goto last_literals;
          match = mi;
          fh = hash_at(src + fwd, small);
          PUT(h, cur);
          if (!small && mi + DISTANCE_MAX < cur) continue; /* too far */
          if (rd32(src + match) == rd32(src + ip)) break;
        }
      }
      /* extend backwards over equal bytes */
      while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
        ip--;
        match--;
      }
      uint8_t *token = op++;
      {
        const size_t lit = ip - anchor;
        if (lit >= RUN_MASK) {
          *token = RUN_MASK << 4;
          op = put_length(op, lit - RUN_MASK);
        } else {
          *token = (uint8_t)(lit << 4);
        }
        memcpy(op, src + anchor, lit);
        op += lit;
      }
      for (;;) { /* a match at ip from `match` (the "next match" chain) */
        const size_t off = ip - match;
        *op++ = (uint8_t)off;
        *op++ = (uint8_t)(off >> 8);
        size_t ml = 0;
        while (ip + MINMATCH + ml < matchlimit && src[ip + MINMATCH + ml] == src[match + MINMATCH + ml]) ml++;
        ip += ml + MINMATCH;
        if (ml >= ML_MASK) {
          *token += ML_MASK;
          op = put_length(op, ml - ML_MASK);
        } else {
          *token += (uint8_t)ml;
        }
        anchor = ip;
        if (ip >= mflimit1) goto last_literals;
        PUT(hash_at(src + ip - 2, small), ip - 2);
        /* test the position right after the match */
        const uint32_t h = hash_at(src + ip, small);
        const uint32_t mi = GET(h);
        PUT(h, ip);
        if ((small || mi + DISTANCE_MAX >= ip) && rd32(src + mi) == rd32(src + ip)) {
          match = mi;
          token = op++;
          *token = 0;
          continue;
        }
        break;
      }
      fh = hash_at(src + ++ip, small);
    }
  }
last_literals: {
    const size_t last = n - anchor;
    if (last >= RUN_MASK) {
      *op++ = RUN_MASK << 4;
      op = put_length(op, last - RUN_MASK);
    } else {
      *op++ = (uint8_t)(last << 4);
    }
    memcpy(op, src + anchor, last);
    op += last;
  }
#undef GET
#undef PUT
  return (size_t)(op - dst);
}

/* A block is valid when it parses to exactly ulen bytes with every length,
 * offset and input position in range, and keeps the format's end rules as
 * LZ4_decompress_safe enforces them with the output capacity = ulen: a
 * match never writes the last LASTLITERALS bytes, and a literal run that
 * ends within MFLIMIT bytes of the output end, or leaves fewer than 8 input
 * bytes, is the last sequence and ends exactly at the input end.  Offset 0
 * is rejected (LZ4_decompress_safe copies from the write position itself). */
int lz4o_decompress_block(const uint8_t *src, size_t n, uint8_t *dst, size_t ulen) {
  size_t ip = 0, op = 0;
  for (;;) {
    if (ip >= n) return 0;
    const unsigned token = src[ip++];
    size_t lit = token >> 4;
    if (lit == RUN_MASK) {
      unsigned b;
      do {
        if (ip >= n) return 0;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - ip || lit > ulen - op) return 0;
    if (op + lit + MFLIMIT > ulen || ip + lit + 2 + 1 + LASTLITERALS > n) {
      if (ip + lit != n) return 0; /* must be the last sequence */
      memcpy(dst + op, src + ip, lit);
      return op + lit == ulen;
    }
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    const size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return 0;
    size_t ml = (token & ML_MASK) + MINMATCH;
    if ((token & ML_MASK) == ML_MASK) {
      unsigned b;
      do {
        if (ip >= n) return 0;
        b = src[ip++];
        ml += b;
      } while (b == 255 && ml <= ulen);
    }
    if (ml + LASTLITERALS > ulen - op) return 0;
    for (size_t k = 0; k < ml; ++k) dst[op + k] = dst[op + k - off];
    op += ml;
  }
}

/* the RPC body: varint32 uncompressed length, then one LZ4 block */
size_t lz4o_compress(const uint8_t *src, size_t n, uint8_t *dst) {
  if (n > LZ4O_MAX_INPUT) return 0;
  size_t h = 0;
  uint32_t v = (uint32_t)n;
  while (v >= 0x80) {
    dst[h++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  dst[h++] = (uint8_t)v;
  return h + lz4o_compress_block(src, n, dst + h);
}

int lz4o_header(const uint8_t *src, size_t n, uint32_t *ulen) {
  uint32_t r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((size_t)i >= n) return 0;
    const uint32_t c = src[i];
    r |= (c & 0x7fu) << (7 * i);
    if (c < 128) {
      if (i == 4 && c >= 16) return 0;
      *ulen = r;
      return i + 1;
    }
  }
  return 0;
}

int lz4o_decompress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, uint32_t *ulen) {
  *ulen = 0;
  const int h = lz4o_header(src, n, ulen);
  if (h == 0) return -1;
  if (*ulen > cap) return -2;
  return lz4o_decompress_block(src + h, n - (size_t)h, dst, *ulen) ? 1 : 0;
}
