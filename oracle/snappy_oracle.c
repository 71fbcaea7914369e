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
 * The tag loop once more, with the writer as a parameter: DecompressAllTags
 * (snappy.cc:716-787) over a source whose Peek hands out `frag`-byte pieces
 * of the stream (0 = one piece; the ref harness's FragmentSource), RefillTag
 * (:790-847) stitching a tag across pieces.  A literal is appended piece by
 * piece (:751-761): the writer sees one Append per piece it spans, and a
 * literal cut by the end of input appends what the input holds, then stops.
 * A copy is one AppendFromSelf. */
typedef struct {
  int (*append)(void *w, const uint8_t *p, size_t n);
  int (*append_from_self)(void *w, size_t offset, size_t len);
  /* TryFastAppend (NULL: the writer's fast path leaves nothing observable) */
  int (*try_fast)(void *w, const uint8_t *p, size_t available, size_t len);
} writer_ops_t;

static size_t piece_left(size_t pos, size_t n, size_t frag) {
  if (pos >= n) return 0;
  if (!frag) return n - pos;
  size_t end = (pos / frag + 1) * frag;
  return (end < n ? end : n) - pos;
}

/* Returns 1 iff the input ends between tags (the caller checks the length). */
static int tag_loop(const uint8_t *in, size_t n, size_t pos, size_t frag, void *w,
                    const writer_ops_t *ops) {
  for (;;) {
    if (pos == n) return 1;
    uint32_t c = in[pos];
    uint32_t extra = (c & 3) == 0 ? ((c >> 2) + 1 > 60 ? (c >> 2) + 1 - 60 : 0)
                                   : ((c & 3) == 1 ? 1 : ((c & 3) == 2 ? 2 : 4));
    if (n - pos < 1 + (size_t)extra) return 0; /* RefillTag: a cut tag */
    uint32_t v = 0;
    for (uint32_t k = 0; k < extra; ++k) v |= (uint32_t)in[pos + 1 + k] << (8 * k);
    pos += 1 + extra;
    if ((c & 3) == 0) {
      size_t len = extra ? (size_t)(uint32_t)(v + 1u) : (size_t)((c >> 2) + 1);
      /* :736: tried right after the tag byte, before any length bytes */
      if (!extra && ops->try_fast && ops->try_fast(w, in + pos, piece_left(pos, n, frag), len)) {
        pos += len;
        continue;
      }
      for (;;) {
        size_t a = piece_left(pos, n, frag);
        if (a >= len) {
          if (len && !ops->append(w, in + pos, len)) return 0;
          pos += len;
          break;
        }
        if (a == 0) return 0; /* premature end of input */
        if (!ops->append(w, in + pos, a)) return 0;
        pos += a;
        len -= a;
      }
    } else {
      uint32_t len = (c & 3) == 1 ? 4 + ((c >> 2) & 7) : (c >> 2) + 1;
      uint32_t offset = (c & 3) == 1 ? (((c >> 5) << 8) | v) : v;
      if (!ops->append_from_self(w, offset, len)) return 0;
    }
  }
}

/* SnappyScatteredWriter (snappy.cc:1331-1481): output in blocks of
 * kBlockSize (the last one cut at the header's length), SlowAppend filling
 * the current block before its bounds check (:1424-1451).  Bytes land at
 * their output positions in `out`; the ones past `cap` are counted, not
 * stored (the harness's copying sink). */
typedef struct {
  uint8_t *out;
  size_t cap, expected, full, blk_len, blk_used, hi;
} scatter_t;

static void sc_put(scatter_t *s, const uint8_t *p, size_t n) {
  size_t at = s->full + s->blk_used;
  for (size_t i = 0; i < n; ++i)
    if (at + i < s->cap) s->out[at + i] = p[i];
  s->blk_used += n;
  if (at + n > s->hi) s->hi = at + n;
}

static int sc_append(void *w, const uint8_t *p, size_t len) {
  scatter_t *s = (scatter_t *)w;
  size_t avail = s->blk_len - s->blk_used;
  while (len > avail) {
    sc_put(s, p, avail);
    s->full += s->blk_used; /* full_size_ += op_ptr_ - op_base_ */
    len -= avail;
    p += avail;
    if (s->full + len > s->expected) return 0; /* op_base_ / op_ptr_ keep the filled block */
    s->blk_len = s->expected - s->full < BLOCK_SIZE ? s->expected - s->full : BLOCK_SIZE;
    s->blk_used = 0;
    avail = s->blk_len;
  }
  sc_put(s, p, len);
  return 1;
}

static int sc_append_from_self(void *w, size_t offset, size_t len) {
  scatter_t *s = (scatter_t *)w;
  size_t cur = s->full + s->blk_used;
  if (offset - 1u >= cur || s->expected - cur < len) return 0; /* :1463-1466 */
  for (size_t i = 0; i < len; ++i) {
    size_t src = cur - offset + i;
    uint8_t c = src < s->cap ? s->out[src] : 0;
    sc_append(s, &c, 1);
  }
  return 1;
}

size_t so_uncompress_as_much(const uint8_t *in, size_t n, size_t frag, uint8_t *out,
                             size_t cap, size_t *got) {
  static const writer_ops_t ops = {sc_append, sc_append_from_self, NULL};
  uint32_t ulen = 0;
  *got = 0;
  int h = so_header_lenient(in, n, &ulen); /* InternalUncompress :858-868 */
  if (!h) return 0;
  scatter_t s = {out, cap, ulen, 0, 0, 0, 0};
  (void)tag_loop(in, n, (size_t)h, frag, &s, &ops);
  *got = s.hi;                   /* Flush(Produced()): every byte written */
  return s.full + s.blk_used;    /* Produced() */
}

/* SnappyIOVecWriter (snappy.cc:963-1120): the output limit is the header's
 * length; iovecs fill in order, a full one moves on to the next, and running
 * out of iovecs fails the call.  AppendFromSelf locates its source by
 * walking back over earlier (full) iovecs and copies through Append, whose
 * result it does not check (:1078-1086), or byte by byte inside the current
 * iovec (IncrementalCopy, :1106-1108). */
typedef struct {
  uint8_t *const *base;
  const size_t *len;
  size_t cnt, cur, written, total, limit;
} iovw_t;

static int iov_append(void *w, const uint8_t *p, size_t len) {
  iovw_t *s = (iovw_t *)w;
  if (s->total + len > s->limit) return 0;
  while (len > 0) {
    if (s->written >= s->len[s->cur]) {
      if (s->cur + 1 >= s->cnt) return 0;
      s->written = 0;
      ++s->cur;
    }
    size_t k = s->len[s->cur] - s->written;
    if (k > len) k = len;
    memmove(s->base[s->cur] + s->written, p, k);
    s->written += k;
    s->total += k;
    p += k;
    len -= k;
  }
  return 1;
}

static int iov_append_from_self(void *w, size_t offset, size_t len) {
  iovw_t *s = (iovw_t *)w;
  if (offset > s->total || offset == 0) return 0;
  if (len > s->limit - s->total) return 0;
  size_t fi = s->cur, fo = s->written;
  while (offset > 0) {
    if (fo >= offset) {
      fo -= offset;
      break;
    }
    offset -= fo;
    --fi;
    fo = s->len[fi];
  }
  while (len > 0) {
    if (fi != s->cur) {
      size_t k = s->len[fi] - fo;
      if (k > len) k = len;
      (void)iov_append(s, s->base[fi] + fo, k);
      len -= k;
      if (len > 0) {
        ++fi;
        fo = 0;
      }
    } else {
      size_t k = s->len[s->cur] - s->written;
      if (k == 0) {
        if (s->cur + 1 >= s->cnt) return 0;
        ++s->cur;
        s->written = 0;
        continue;
      }
      if (k > len) k = len;
      for (size_t i = 0; i < k; ++i) s->base[s->cur][s->written + i] = s->base[fi][fo + i];
      s->written += k;
      fo += k;
      s->total += k;
      len -= k;
    }
  }
  return 1;
}

/* :1035-1049: 16 bytes copied when the input, the output limit and the
 * current iovec all have 16 bytes of room; only `len` of them count (the
 * rest is overwritten later, or left behind when the call fails) */
static int iov_try_fast(void *w, const uint8_t *p, size_t available, size_t len) {
  iovw_t *s = (iovw_t *)w;
  if (len <= 16 && available >= 16 + 5 && s->limit - s->total >= 16 &&
      s->len[s->cur] - s->written >= 16) {
    memmove(s->base[s->cur] + s->written, p, 16);
    s->written += len;
    s->total += len;
    return 1;
  }
  return 0;
}

int so_uncompress_iovec(const uint8_t *in, size_t n, uint8_t *const *iov_base,
                        const size_t *iov_len, size_t iov_cnt) {
  static const writer_ops_t ops = {iov_append, iov_append_from_self, iov_try_fast};
  uint32_t ulen = 0;
  int h = so_header_lenient(in, n, &ulen); /* RawUncompressToIOVec :1122-1132 */
  if (!h) return 0;
  /* no iovecs and output to place: the reference reads iov[0] (undefined);
   * with ulen 0 no Append ever reaches the iovecs */
  if (iov_cnt == 0 && ulen > 0) return 0;
  iovw_t s = {iov_base, iov_len, iov_cnt, 0, 0, 0, ulen};
  return tag_loop(in, n, (size_t)h, 0, &s, &ops) && s.total == ulen;
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
