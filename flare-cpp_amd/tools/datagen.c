/*
 * datagen.c -- integer-seeded synthetic RPC-body generators.
 *
 * Portable: splitmix64 only, no <random>.  Used by bench.py and the tests to
 * build the C2/C3/CM/C5 batches identically on every host.
 *
 *   text   (C3, CM, C5): Zipf(s=1) over a 5000-word vocabulary (seed 12345),
 *                        word lengths 2+r%9, letters 'a'+r%26; separator from
 *                        p=r%100: <5 ". ", <10 ", ", <12 "\n", else " ";
 *                        body i seeded 0x7E47*1000003+i, truncated to size.
 *                        Anchor: body 0 at 64 KiB compresses to 32,380 B.
 *   random (C2):         little-endian splitmix64 words, body i seeded
 *                        0xC0FFEE*1000003+i.  Anchor: body 0 at 4 KiB
 *                        compresses to 4,101 B (80 20 f4 ff 0f ...).
 *   mixed sizes (CM):    one stream seeded 0x5EED; size_i =
 *                        floor(256/(1-u*(1-2^-12))), u=(r>>11)*2^-53, clamped
 *                        to [256, 1 MiB]; body i is random if i%4==3 else text.
 *   SnappyMessageProto (C5): {text = text body of a CM-distributed size,
 *                        numbers = (r%17) int32 values (int32)r}, serialized
 *                        in proto2 wire format (field 1 LEN, field 2 unpacked
 *                        varints; negative int32 -> 10-byte varint).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define VOCAB 5000

typedef struct { uint64_t s; } sm64;
static inline uint64_t sm_next(sm64 *r) {
  uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static char g_words[VOCAB][11];
static uint8_t g_wlen[VOCAB];
static double g_cdf[VOCAB];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_vocab(void) {
  sm64 r = {12345};
  for (int i = 0; i < VOCAB; ++i) {
    int len = 2 + (int)(sm_next(&r) % 9);
    for (int k = 0; k < len; ++k) g_words[i][k] = (char)('a' + sm_next(&r) % 26);
    g_wlen[i] = (uint8_t)len;
  }
  double tot = 0, acc = 0;
  for (int i = 0; i < VOCAB; ++i) tot += 1.0 / (i + 1);
  for (int i = 0; i < VOCAB; ++i) {
    acc += 1.0 / (i + 1);
    g_cdf[i] = acc / tot;
  }
}

static inline int zipf_pick(double u) {
  int lo = 0, hi = VOCAB - 1; /* first i with cdf[i] > u */
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (g_cdf[mid] > u) hi = mid; else lo = mid + 1;
  }
  return lo;
}

void dg_text_body(uint64_t index, uint8_t *out, size_t n) {
  pthread_once(&g_once, init_vocab);
  sm64 r = {0x7E47ull * 1000003ull + index};
  size_t pos = 0;
  while (pos < n) {
    double u = (double)(sm_next(&r) >> 11) * (1.0 / 9007199254740992.0);
    int w = zipf_pick(u);
    uint64_t p = sm_next(&r) % 100;
    const char *sep = p < 5 ? ". " : (p < 10 ? ", " : (p < 12 ? "\n" : " "));
    for (int k = 0; k < g_wlen[w] && pos < n; ++k) out[pos++] = (uint8_t)g_words[w][k];
    for (const char *s = sep; *s && pos < n; ++s) out[pos++] = (uint8_t)*s;
  }
}

void dg_random_body(uint64_t index, uint8_t *out, size_t n) {
  sm64 r = {0xC0FFEEull * 1000003ull + index};
  size_t pos = 0;
  while (pos < n) {
    uint64_t v = sm_next(&r);
    for (int k = 0; k < 8 && pos < n; ++k) out[pos++] = (uint8_t)(v >> (8 * k));
  }
}

/* CM size distribution. */
void dg_mixed_sizes(uint64_t n, uint32_t *sizes) {
  sm64 r = {0x5EED};
  for (uint64_t i = 0; i < n; ++i) {
    double u = (double)(sm_next(&r) >> 11) * (1.0 / 9007199254740992.0);
    double x = 256.0 / (1.0 - u * (1.0 - 1.0 / 4096.0));
    uint64_t s = (uint64_t)floor(x);
    if (s < 256) s = 256;
    if (s > (1u << 20)) s = 1u << 20;
    sizes[i] = (uint32_t)s;
  }
}

static size_t put_varint64(uint8_t *p, uint64_t v) {
  size_t k = 0;
  while (v >= 128) { p[k++] = (uint8_t)(v | 128); v >>= 7; }
  p[k++] = (uint8_t)v;
  return k;
}

/* C5: serialized SnappyMessageProto i; returns serialized length.  With
 * out == NULL only the length is computed.  text_len from dg_mixed_sizes. */
size_t dg_snappy_message(uint64_t index, uint32_t text_len, uint8_t *out) {
  sm64 r = {0x5A9Bull * 1000003ull + index};
  uint64_t cnt = sm_next(&r) % 17;
  uint8_t tmp[16];
  size_t n = 0;
  /* field 1, wire type 2 */
  if (out) out[n] = 0x0a;
  n += 1;
  size_t k = put_varint64(tmp, text_len);
  if (out) memcpy(out + n, tmp, k);
  n += k;
  if (out) dg_text_body(index, out + n, text_len);
  n += text_len;
  for (uint64_t j = 0; j < cnt; ++j) {
    int32_t v = (int32_t)(uint32_t)sm_next(&r);
    if (out) out[n] = 0x10; /* field 2, varint */
    n += 1;
    k = put_varint64(tmp, (uint64_t)(int64_t)v); /* sign-extended int32 */
    if (out) memcpy(out + n, tmp, k);
    n += k;
  }
  return n;
}

uint64_t dg_fnv1a64(const uint8_t *p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
  return h;
}

/* Batch fill: kind 0 = text, 1 = random, 2 = mixed (i%4==3 random),
 * 3 = SnappyMessageProto (sizes[] are text lengths; lens written to
 * out_lens).  Messages are written at out + offsets[i]. */
typedef struct {
  int kind, tid, nt;
  uint64_t first, n;
  const uint32_t *sizes;
  const uint64_t *offsets;
  uint8_t *out;
  uint32_t *out_lens;
} fill_job;

static void *fill_worker(void *a) {
  fill_job *j = (fill_job *)a;
  for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nt) {
    uint64_t gi = j->first + i;
    uint8_t *dst = j->out + j->offsets[i];
    switch (j->kind) {
      case 0: dg_text_body(gi, dst, j->sizes[i]); break;
      case 1: dg_random_body(gi, dst, j->sizes[i]); break;
      case 2:
        if (gi % 4 == 3) dg_random_body(gi, dst, j->sizes[i]);
        else dg_text_body(gi, dst, j->sizes[i]);
        break;
      default: {
        size_t l = dg_snappy_message(gi, j->sizes[i], dst);
        if (j->out_lens) j->out_lens[i] = (uint32_t)l;
      }
    }
  }
  return NULL;
}

void dg_fill_batch(int kind, uint64_t first_index, uint64_t n,
                   const uint32_t *sizes, const uint64_t *offsets, uint8_t *out,
                   uint32_t *out_lens, int n_threads) {
  pthread_once(&g_once, init_vocab);
  if (n_threads < 1) n_threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * n_threads);
  fill_job *jobs = (fill_job *)malloc(sizeof(fill_job) * n_threads);
  for (int t = 0; t < n_threads; ++t) {
    fill_job jj = {kind, t, n_threads, first_index, n, sizes, offsets, out, out_lens};
    jobs[t] = jj;
    pthread_create(&th[t], NULL, fill_worker, &jobs[t]);
  }
  for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* Per-message FNV digests of a batch (for fixtures / quick equality). */
void dg_digest_batch(const uint8_t *base, const uint64_t *offsets,
                     const uint32_t *lens, uint64_t n, uint64_t *out) {
  for (uint64_t i = 0; i < n; ++i) out[i] = dg_fnv1a64(base + offsets[i], lens[i]);
}
