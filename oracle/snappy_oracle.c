/*
 * snappy_oracle.c -- TEST INFRASTRUCTURE ONLY (see snappy_oracle.h).
 *
 * Clean-room C restatement of the reference's CPU Snappy path.  Every
 * function cites the reference file:line it restates; all paths are
 * relative to /root/reference/flare/io/snappy/.
 */
#include "snappy_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define BLOCK_LOG 16
#define BLOCK_SIZE ((size_t)1 << BLOCK_LOG)   /* kBlockSize, snappy.h:201-202 */
#define MAX_HT_BITS 14                          /* kMaxHashTableBits, snappy.h:204 */
#define MAX_HT_SIZE (1 << MAX_HT_BITS)          /* kMaxHashTableSize, snappy.h:205 */
#define INPUT_MARGIN 15                         /* kInputMarginBytes, snappy.cc:346 */

static inline uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

/* snappy.cc:55-77 */
size_t so_max_compressed_length(size_t n) { return 32 + n + n / 6; }

/* snappy-stubs-internal.h:327-357 */
int so_header_strict(const uint8_t *in, size_t n, uint32_t *ulen) {
  uint32_t r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((size_t)i >= n) return 0;
    uint32_t b = in[i];
    r |= (b & 127u) << (7 * i);
    if (i < 4 ? b < 128 : b < 16) {
      *ulen = r;
      return i + 1;
    }
  }
  return 0;
}

/* snappy.cc:692-711: shift grows by 7 per byte; `shift >= 32` rejects a 6th
 * byte; the 5th byte's bits above bit 3 fall off the uint32. */
int so_header_lenient(const uint8_t *in, size_t n, uint32_t *ulen) {
  uint32_t r = 0, shift = 0;
  size_t i = 0;
  for (;;) {
    if (shift >= 32) return 0;
    if (i >= n) return 0;
    uint32_t c = in[i++];
    r |= (c & 0x7fu) << shift;
    if (c < 128) break;
    shift += 7;
  }
  *ulen = r;
  return (int)i;
}

/* Varint::Encode32, snappy-stubs-internal.h:359-385 */
static size_t varint32(uint8_t *p, uint32_t v) {
  size_t k = 0;
  while (v >= 128) {
    p[k++] = (uint8_t)(v | 128);
    v >>= 7;
  }
  p[k++] = (uint8_t)v;
  return k;
}

/* EmitLiteral, snappy.cc:156-196 (the 16-byte fast path only changes which
 * bytes past the end get scribbled, never the stream). */
static uint8_t *emit_literal(uint8_t *op, const uint8_t *lit, uint32_t len) {
  uint32_t n = len - 1;
  if (n < 60) {
    *op++ = (uint8_t)(n << 2);
  } else {
    uint8_t *base = op++;
    int count = 0;
    while (n > 0) {
      *op++ = (uint8_t)(n & 0xff);
      n >>= 8;
      ++count;
    }
    *base = (uint8_t)((59 + count) << 2);
  }
  memcpy(op, lit, len);
  return op + len;
}

/* EmitCopyLessThan64, snappy.cc:198-214 */
static uint8_t *emit_copy_lt64(uint8_t *op, uint32_t offset, uint32_t len) {
  if (len < 12 && offset < 2048) {
    *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    *op++ = (uint8_t)(offset & 0xff);
  } else {
    *op++ = (uint8_t)(2 + ((len - 1) << 2));
    *op++ = (uint8_t)(offset & 0xff);
    *op++ = (uint8_t)(offset >> 8);
  }
  return op;
}

/* EmitCopy, snappy.cc:216-232: 64-byte chunks while len >= 68, one 60-byte
 * chunk if 64 < len < 68, then the remainder. */
static uint8_t *emit_copy(uint8_t *op, uint32_t offset, uint32_t len) {
  while (len >= 68) {
    op = emit_copy_lt64(op, offset, 64);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_lt64(op, offset, 60);
    len -= 60;
  }
  return emit_copy_lt64(op, offset, len);
}

/* FindMatchLength, snappy-internal.h:87-121: longest common prefix of s1 and
 * s2 bounded by s2_limit. */
static inline uint32_t match_len(const uint8_t *s1, const uint8_t *s2,
                                 const uint8_t *s2_limit) {
  uint32_t m = 0;
  while (s2 + m < s2_limit && s1[m] == s2[m]) ++m;
  return m;
}

static inline uint32_t hash_bytes(uint32_t bytes, int shift) {
  return (bytes * 0x1e35a7bdu) >> shift; /* HashBytes, snappy.cc:46-49 */
}

/* WorkingMemory::GetHashTable sizing, snappy.cc:247-271 */
static uint32_t table_size_for(size_t frag_len) {
  uint32_t ht = 256;
  while (ht < MAX_HT_SIZE && ht < frag_len) ht <<= 1;
  return ht;
}

/* internal::CompressFragment, snappy.cc:329-453 */
static uint8_t *compress_fragment(const uint8_t *input, size_t n, uint8_t *op,
                                  uint16_t *table, uint32_t table_size) {
  int log2 = 0;
  while ((1u << log2) < table_size) ++log2;
  const int shift = 32 - log2;
  const uint8_t *ip = input;
  const uint8_t *ip_end = input + n;
  const uint8_t *next_emit = ip;

  if (n >= INPUT_MARGIN) {
    const uint8_t *ip_limit = input + n - INPUT_MARGIN;
    uint32_t next_hash = hash_bytes(ld32(++ip), shift);
    for (;;) {
      /* Step 1: probe with the skip heuristic (:377-397). */
      uint32_t skip = 32;
      const uint8_t *next_ip = ip;
      const uint8_t *candidate;
      do {
        ip = next_ip;
        uint32_t h = next_hash;
        uint32_t step = skip++ >> 5;
        next_ip = ip + step;
        if (next_ip > ip_limit) goto emit_remainder;
        next_hash = hash_bytes(ld32(next_ip), shift);
        candidate = input + table[h];
        table[h] = (uint16_t)(ip - input);
      } while (ld32(ip) != ld32(candidate));

      /* Step 2: pending literal (:403). */
      op = emit_literal(op, next_emit, (uint32_t)(ip - next_emit));

      /* Step 3: copies while the 4 bytes after the last copy match (:416-439). */
      uint32_t cand_bytes;
      uint32_t cur_bytes;
      do {
        const uint8_t *base = ip;
        uint32_t matched = 4 + match_len(candidate + 4, ip + 4, ip_end);
        ip += matched;
        op = emit_copy(op, (uint32_t)(base - candidate), matched);
        next_emit = ip;
        if (ip >= ip_limit) goto emit_remainder;
        uint32_t prev_hash = hash_bytes(ld32(ip - 1), shift);
        table[prev_hash] = (uint16_t)(ip - input - 1);
        cur_bytes = ld32(ip);
        uint32_t cur_hash = hash_bytes(cur_bytes, shift);
        candidate = input + table[cur_hash];
        cand_bytes = ld32(candidate);
        table[cur_hash] = (uint16_t)(ip - input);
      } while (cur_bytes == cand_bytes);

      next_hash = hash_bytes(ld32(ip + 1), shift);
      ++ip;
    }
  }
emit_remainder:
  if (next_emit < ip_end)
    op = emit_literal(op, next_emit, (uint32_t)(ip_end - next_emit));
  return op;
}

/* Compress(Source*, Sink*), snappy.cc:875-954 */
size_t so_compress(const uint8_t *in, size_t n, uint8_t *out) {
  uint8_t *op = out + varint32(out, (uint32_t)n);
  uint16_t *table = NULL;
  if (n > 1024) table = (uint16_t *)malloc(sizeof(uint16_t) * MAX_HT_SIZE);
  uint16_t small_table[1024];
  size_t pos = 0;
  while (pos < n) {
    size_t frag = n - pos < BLOCK_SIZE ? n - pos : BLOCK_SIZE;
    uint32_t ts = table_size_for(frag);
    uint16_t *t = ts <= 1024 ? small_table : table;
    memset(t, 0, ts * sizeof(uint16_t));
    op = compress_fragment(in + pos, frag, op, t, ts);
    pos += frag;
  }
  free(table);
  return (size_t)(op - out);
}

/* Shared tag walk: DecompressAllTags (snappy.cc:716-787) + RefillTag
 * (:790-847) on a flat source, with the writer checks common to
 * SnappyArrayWriter (:1141-1227), SnappyScatteredWriter (:1331-1481) and
 * SnappyDecompressionValidator (:1254-1288).  `out` may be NULL
 * (validate-only).  Returns 1 iff eof && produced == expected (:858-868). */
static int walk_tags(const uint8_t *ip, const uint8_t *end, uint8_t *out,
                     uint32_t expected) {
  uint64_t op = 0;
  for (;;) {
    if (ip == end) return op == expected; /* RefillTag eof */
    uint32_t c = *ip++;
    if ((c & 3) == 0) {
      uint32_t len = (c >> 2) + 1;
      if (len >= 61) {
        uint32_t nb = len - 60; /* 1..4 length bytes (char_table :516-549) */
        if ((size_t)(end - ip) < nb) return 0; /* RefillTag: needed > avail */
        uint32_t v = 0;
        for (uint32_t k = 0; k < nb; ++k) v |= (uint32_t)ip[k] << (8 * k);
        len = v + 1; /* uint32 arithmetic: 0xffffffff + 1 wraps to 0 */
        ip += nb;
      }
      if ((uint64_t)(end - ip) < len) return 0;   /* premature end (:761) */
      if (op + len > expected) return 0;          /* writer overrun */
      if (out && len) memcpy(out + op, ip, len);
      op += len;
      ip += len;
    } else {
      uint32_t type = c & 3;
      uint32_t nb = type == 1 ? 1 : (type == 2 ? 2 : 4);
      if ((size_t)(end - ip) < nb) return 0;
      uint32_t len, offset;
      if (type == 1) {
        len = 4 + ((c >> 2) & 7);
        offset = ((c >> 5) << 8) | ip[0];
      } else {
        len = (c >> 2) + 1;
        offset = 0;
        for (uint32_t k = 0; k < nb; ++k) offset |= (uint32_t)ip[k] << (8 * k);
      }
      ip += nb;
      /* "produced <= offset - 1u" rejects offset 0 and offset > produced */
      if (offset == 0 || (uint64_t)offset > op) return 0;
      if (op + len > expected) return 0;
      if (out) {
        /* IncrementalCopy semantics (:98-103): byte order matters when
         * offset < len (pattern replication). */
        uint8_t *d = out + op;
        const uint8_t *s = d - offset;
        for (uint32_t k = 0; k < len; ++k) d[k] = s[k];
      }
      op += len;
    }
  }
}

/* Uncompress(Source*, Sink*), snappy.cc:1537-1563 */
int so_uncompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                  uint32_t *out_len) {
  uint32_t ulen = 0;
  int h = so_header_lenient(in, n, &ulen);
  *out_len = h ? ulen : 0;
  if (!h) return 0;
  if (ulen > out_cap) return -1;
  return walk_tags(in + h, in + n, out, ulen);
}

/* IsValidCompressedBuffer, snappy.cc:1290-1294 */
int so_is_valid(const uint8_t *in, size_t n) {
  uint32_t ulen = 0;
  int h = so_header_lenient(in, n, &ulen);
  if (!h) return 0;
  return walk_tags(in + h, in + n, NULL, ulen);
}

/* ---------------------------------------------------------------------------
 * Batched CPU baseline: threads own strided message indices. */
typedef struct {
  int tid, nthreads, mode;
  const uint8_t *in;
  const uint64_t *in_off;
  const uint32_t *in_len;
  uint32_t n_msgs;
  uint8_t *out;
  const uint64_t *out_off;
  const uint32_t *out_cap;
  uint32_t *out_len;
  int32_t *status;
} job_t;

static void *batch_worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (uint32_t i = (uint32_t)j->tid; i < j->n_msgs; i += (uint32_t)j->nthreads) {
    const uint8_t *src = j->in + j->in_off[i];
    uint8_t *dst = j->out + j->out_off[i];
    if (j->mode == 0) {
      j->out_len[i] = (uint32_t)so_compress(src, j->in_len[i], dst);
    } else {
      uint32_t ol = 0;
      int ok = so_uncompress(src, j->in_len[i], dst, j->out_cap[i], &ol);
      j->out_len[i] = ol;
      if (j->status) j->status[i] = ok == 1 ? 0 : (ok < 0 ? 3 : 1);
    }
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static double run_batch(job_t proto, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * n_threads);
  job_t *jobs = (job_t *)malloc(sizeof(job_t) * n_threads);
  double t0 = now_s();
  for (int t = 0; t < n_threads; ++t) {
    jobs[t] = proto;
    jobs[t].tid = t;
    jobs[t].nthreads = n_threads;
    pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
  double dt = now_s() - t0;
  free(th);
  free(jobs);
  return dt;
}

double so_compress_batch(const uint8_t *in, const uint64_t *in_off,
                         const uint32_t *in_len, uint32_t n_msgs, uint8_t *out,
                         const uint64_t *out_off, uint32_t *out_len,
                         int n_threads) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.mode = 0;
  p.in = in; p.in_off = in_off; p.in_len = in_len; p.n_msgs = n_msgs;
  p.out = out; p.out_off = out_off; p.out_len = out_len;
  return run_batch(p, n_threads);
}

double so_uncompress_batch(const uint8_t *in, const uint64_t *in_off,
                           const uint32_t *in_len, uint32_t n_msgs,
                           uint8_t *out, const uint64_t *out_off,
                           const uint32_t *out_cap, uint32_t *out_len,
                           int32_t *status, int n_threads) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.mode = 1;
  p.in = in; p.in_off = in_off; p.in_len = in_len; p.n_msgs = n_msgs;
  p.out = out; p.out_off = out_off; p.out_cap = out_cap; p.out_len = out_len;
  p.status = status;
  return run_batch(p, n_threads);
}
