// wenc_model.cc -- CPU model of the wave-per-fragment Snappy encoder
// (flare-cpp_amd/csrc/snappy_encode_wave.hip), lane arrays standing in for
// the 64 lanes of a wave.  Development tool: it pins the block/event
// restatement of internal::CompressFragment (/root/reference/flare/io/snappy/
// snappy.cc:329-453) byte-for-byte against the oracle on CPU before the HIP
// kernel mirrors it, and counts the per-block work the kernel will do.
//
//   g++ -O2 -o build/wenc_model tools/wenc_model.cc oracle/snappy_oracle.c \
//       flare-cpp_amd/tools/datagen.c -lpthread -lm && build/wenc_model
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
#include "../oracle/snappy_oracle.h"
void dg_text_body(uint64_t index, uint8_t* out, size_t n);
void dg_random_body(uint64_t index, uint8_t* out, size_t n);
size_t dg_snappy_message(uint64_t index, uint32_t text_len, uint8_t* out);
}

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

static const u32 kHashMul = 0x1e35a7bdu;
static inline u32 hashb(u32 x, int shift) { return (x * kHashMul) >> shift; }

struct Stats {
  u64 blocks = 0, events = 0, probes = 0, pred_rounds = 0, deep = 0, slow_resolve = 0, long_match = 0,
      jumps = 0, direct_inserts = 0, frags = 0, fast = 0, why[6] = {0, 0, 0, 0, 0, 0};
} st;
static int g_trace = 0;

static u8* emit_literal(u8* op, const u8* lit, u32 len) {
  u32 n = len - 1;
  if (n < 60) {
    *op++ = (u8)(n << 2);
  } else {
    u8* base = op++;
    int count = 0;
    while (n > 0) {
      *op++ = (u8)(n & 0xff);
      n >>= 8;
      ++count;
    }
    *base = (u8)((59 + count) << 2);
  }
  memcpy(op, lit, len);
  return op + len;
}
static u8* emit_copy_lt64(u8* op, u32 offset, u32 len) {
  if (len < 12 && offset < 2048) {
    *op++ = (u8)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    *op++ = (u8)(offset & 0xff);
  } else {
    *op++ = (u8)(2 + ((len - 1) << 2));
    *op++ = (u8)(offset & 0xff);
    *op++ = (u8)(offset >> 8);
  }
  return op;
}
static u8* emit_copy(u8* op, u32 offset, u32 len) {
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

// byte at fragment position p, 0 past the end (the kernel's buffer loads)
static inline u8 fb(const u8* f, u32 n, u32 p) { return p < n ? f[p] : 0; }
static inline u32 ld32z(const u8* f, u32 n, u32 p) {
  return fb(f, n, p) | (u32)fb(f, n, p + 1) << 8 | (u32)fb(f, n, p + 2) << 16 | (u32)fb(f, n, p + 3) << 24;
}

// One fragment: the block/event form.
static u8* wenc_fragment(const u8* f, u32 n, u8* op, u16* table, u32 ht) {
  st.frags++;
  int lg = 0;
  while ((1u << lg) < ht) ++lg;
  const int shift = 32 - lg;
  memset(table, 0, ht * sizeof(u16));
  u32 next_emit = 0;
  if (n >= 15) {
    const u32 lim = n - 15;
    enum { LIT, POST } mode = LIT;
    u32 p = 1, sk = 32;  // LIT: next probe and its skip counter
    u32 ip = 0;          // POST: copy end
    for (;;) {
      const u32 pos = mode == LIT ? p : ip;
      const u32 B = pos & ~63u;
      st.blocks++;
      // POST whose ip-1 lies in an earlier block: committed before the reads
      u64 I = 0;
      if (mode == POST) {
        if (ip - 1 < B) {
          table[hashb(ld32z(f, n, ip - 1), shift)] = (u16)(ip - 1);
          st.direct_inserts++;
        } else {
          I = 1ull << (ip - 1 - B);
        }
      }
      // ---- per-lane block data
      u32 X[64], h[64], T[64];
      int pred1[64], pred2[64], pred3[64];
      bool deep[64];
      for (int k = 0; k < 64; ++k) {
        X[k] = ld32z(f, n, B + k);
        h[k] = hashb(X[k], shift);
        T[k] = table[h[k]];
      }
      // pred1 by rounds: active lanes write their id into a per-hash slot
      // (highest wins), winners leave; a round-r+1 winner is the pred1 of the
      // round-r winner of its hash.  (The kernel does this in the LDS table.)
      {
        bool active[64];
        int lastwin[64];
        for (int k = 0; k < 64; ++k) { active[k] = true; pred1[k] = -1; lastwin[k] = -1; deep[k] = false; }
        for (int r = 0; r < 3; ++r) {
          bool any = false;
          for (int k = 0; k < 64; ++k) any |= active[k];
          if (!any) break;
          st.pred_rounds++;
          // slot[h] = highest active lane
          int win_of[64];
          for (int k = 0; k < 64; ++k) {
            win_of[k] = -1;
            if (!active[k]) continue;
            for (int j = 63; j >= 0; --j)
              if (active[j] && h[j] == h[k]) { win_of[k] = j; break; }
          }
          for (int k = 0; k < 64; ++k) {
            if (!active[k]) continue;
            if (win_of[k] == k) {
              if (lastwin[k] >= 0) pred1[lastwin[k]] = k;
              active[k] = false;
            } else {
              lastwin[k] = win_of[k];
            }
          }
          // losers: the round's winner of their hash is their newest candidate
          // for "the lane whose pred1 I am": kept in lastwin
        }
        // still undecided after 3 rounds (a long same-hash chain): unknown
        // pred1 (-2), and so is the pred1 of the last round's winner above it
        for (int k = 0; k < 64; ++k)
          if (active[k]) {
            deep[k] = true;
            pred1[k] = -2;
            if (lastwin[k] >= 0) pred1[lastwin[k]] = -2;
          }
      }
      for (int k = 0; k < 64; ++k) {
        pred2[k] = pred1[k] >= 0 ? pred1[pred1[k]] : pred1[k] == -2 ? -2 : -1;
        pred3[k] = pred2[k] >= 0 ? pred1[pred2[k]] : pred2[k] == -2 ? -2 : -1;
        deep[k] = pred1[k] == -2;
      }
      // check the rounds' pred1 against a direct scan (model self-check)
      for (int k = 0; k < 64; ++k) {
        if (pred1[k] == -2) continue;
        int d = -1;
        for (int j = k - 1; j >= 0; --j)
          if (h[j] == h[k]) { d = j; break; }
        if (d != pred1[k]) { fprintf(stderr, "pred1 mismatch B=%u k=%d %d %d\n", B, k, d, pred1[k]); exit(1); }
      }
      // candidate of lane k with inserted set I (position)
      auto resolve = [&](int k, u64 Iset) -> u32 {
        {  // the kernel's fast rule: pred1 if inserted, else T when the chain below is known empty
          const bool i1 = pred1[k] >= 0 && ((Iset >> pred1[k]) & 1);
          const bool i2 = pred2[k] >= 0 && ((Iset >> pred2[k]) & 1);
          const bool useT = pred1[k] == -1 || (pred1[k] >= 0 && !i1 && (pred2[k] == -1 || (pred2[k] >= 0 && !i2 && pred3[k] == -1)));
          if (!i1 && !useT) st.deep++;
        }
        const int ps[3] = {pred1[k], pred2[k], pred3[k]};
        for (int i = 0; i < 3; ++i) {
          if (ps[i] == -1) return T[k];
          if (ps[i] == -2) break;  // unknown beyond here
          if ((Iset >> ps[i]) & 1) return B + ps[i];
        }
        // chain deeper than 3 or undecided: scan (the kernel's slow path)
        st.slow_resolve++;
        for (int j = k - 1; j >= 0; --j)
          if (h[j] == h[k] && ((Iset >> j) & 1)) return B + j;
        return T[k];
      };

      bool done = false;     // emit_remainder reached
      bool leave = false;    // parse continues in a later block
      while (!done && !leave) {
        u32 q = 0, cand = 0;
        bool found = false;
        // would the kernel's fast event path (FSG_WENC_FAST) take this event?
        bool fast_ok = mode == POST;
        int why = mode == POST ? -1 : 0;  // first reason the fast path would not take it
        const u32 ip_at = ip;
        if (mode == POST) {
          const int k0 = (int)(ip - B);
          if (fast_ok && pred1[k0] != -1 && why < 0) why = 1;
          fast_ok = fast_ok && pred1[k0] == -1;
          cand = resolve(k0, I);
          I |= 1ull << k0;
          st.probes++;
          if (g_trace) printf("post %u %u\n", ip, cand);
          if (ld32z(f, n, cand) == X[k0]) {
            q = ip;
            found = true;
          } else {
            mode = LIT;
            p = ip + 1;
            sk = 32;
            if (p >= B + 64) { leave = true; break; }
          }
        }
        if (!found) {
          // literal search from p (inside this block)
          while (p < B + 64) {
            const u32 step = sk >> 5;
            if (p + step > lim) { done = true; break; }
            const int k = (int)(p - B);
            if (fast_ok && pred1[k] != -1 && why < 0) why = 2;
            if (fast_ok && !(p - ip_at <= 32 && sk < 64) && why < 0) why = 3;
            fast_ok = fast_ok && pred1[k] == -1 && p - ip_at <= 32 && sk < 64;
            cand = resolve(k, I);
            I |= 1ull << k;
            st.probes++;
            if (g_trace) printf("probe %u %u\n", p, cand);
            const u32 cur = p;
            p += step;
            ++sk;
            if (ld32z(f, n, cand) == X[k]) {
              q = cur;
              found = true;
              break;
            }
          }
          if (done) break;
          if (!found) { leave = true; break; }
          // literal [next_emit, q)
          op = emit_literal(op, f + next_emit, q - next_emit);
        }
        st.events++;
        // copy at q from cand
        u32 m = 4;
        while (q + m < n && f[cand + m] == f[q + m]) ++m;
        if (m > 20) st.long_match++;
        if (fast_ok && (m < 20 || q + 20 >= n)) st.fast++;
        else st.why[why >= 0 ? why : 4]++;
        if (g_trace) printf("copy %u %u %u\n", q, cand, m);
        op = emit_copy(op, q - cand, m);
        ip = q + m;
        next_emit = ip;
        if (ip >= lim) { done = true; break; }
        mode = POST;
        if (ip - 1 < B + 64) I |= 1ull << (ip - 1 - B);
        if (ip >= B + 64) {
          if (((ip) & ~63u) > B + 64) st.jumps++;
          leave = true;
        }
      }
      // ---- commit the block's inserts in position order
      for (int k = 0; k < 64; ++k)
        if ((I >> k) & 1) table[h[k]] = (u16)(B + k);
      if (done) break;
    }
  }
  if (next_emit < n) op = emit_literal(op, f + next_emit, n - next_emit);
  return op;
}

static size_t wenc_compress(const u8* in, size_t n, u8* out) {
  u32 v = (u32)n;
  u8* op = out;
  while (v >= 128) { *op++ = (u8)(v | 128); v >>= 7; }
  *op++ = (u8)v;
  static u16 table[1 << 14];
  size_t pos = 0;
  while (pos < n) {
    const u32 frag = n - pos < 65536 ? (u32)(n - pos) : 65536u;
    u32 ht = 256;
    while (ht < (1u << 14) && ht < frag) ht <<= 1;
    op = wenc_fragment(in + pos, frag, op, table, ht);
    pos += frag;
  }
  return (size_t)(op - out);
}

static u64 rng_s = 88172645463325252ull;
static u64 rnd() {
  rng_s ^= rng_s << 13;
  rng_s ^= rng_s >> 7;
  rng_s ^= rng_s << 17;
  return rng_s;
}

static int check(const std::vector<u8>& x, const char* what) {
  std::vector<u8> a(so_max_compressed_length(x.size()) + 64), b(a.size());
  const size_t la = so_compress(x.data(), x.size(), a.data());
  const size_t lb = wenc_compress(x.data(), x.size(), b.data());
  if (la != lb || memcmp(a.data(), b.data(), la)) {
    fprintf(stderr, "MISMATCH %s n=%zu (oracle %zu, model %zu)\n", what, x.size(), la, lb);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  int bad = 0, cases = 0;
  if (argc > 2) {  // trace one input: wenc_model t <bytes as decimal list>
    g_trace = 1;
    std::vector<u8> x;
    for (int i = 2; i < argc; ++i) x.push_back((u8)atoi(argv[i]));
    std::vector<u8> b(so_max_compressed_length(x.size()) + 64);
    wenc_compress(x.data(), x.size(), b.data());
    return 0;
  }
  const int reps = argc > 1 ? atoi(argv[1]) : 1;
  for (int r = 0; r < reps; ++r) {
    // random alphabets, 0..140 KB (as tests/test_gpu_parity.py)
    for (int t = 0; t < 400; ++t) {
      const u32 c = rnd() % 3;
      const u32 nn = c == 0 ? rnd() % 100 : c == 1 ? rnd() % 5000 : rnd() % 140000;
      const u32 alpha[5] = {2, 3, 8, 40, 256};
      const u32 a = alpha[rnd() % 5];
      std::vector<u8> x(nn);
      for (auto& v : x) v = (u8)(rnd() % a);
      bad += check(x, "random");
      ++cases;
    }
    // runs and periodic data
    for (u32 per = 1; per <= 70; per += 3) {
      std::vector<u8> x(20000 + per * 37);
      for (size_t i = 0; i < x.size(); ++i) x[i] = (u8)((i % per) * 7 + 1);
      bad += check(x, "periodic");
      ++cases;
    }
    // text (the C3 generator) at several sizes, and SnappyMessageProto bodies
    for (u32 t = 0; t < 64; ++t) {
      const u32 nn = t < 32 ? 65536 : (u32)(rnd() % 200000);
      std::vector<u8> x(nn);
      dg_text_body(1000 * r + t, x.data(), nn);
      bad += check(x, "text");
      ++cases;
    }
    for (u32 t = 0; t < 200; ++t) {
      std::vector<u8> x(70000 + 64);
      const size_t nn = dg_snappy_message(7000 * r + t, (u32)(rnd() % 60000), x.data());
      x.resize(nn);
      bad += check(x, "proto");
      ++cases;
    }
    // text with random runs inside
    for (u32 t = 0; t < 20; ++t) {
      std::vector<u8> x(40000);
      dg_text_body(500 + t, x.data(), x.size());
      const u32 at = rnd() % 30000, len = rnd() % 9000;
      for (u32 i = 0; i < len && at + i < x.size(); ++i) x[at + i] = (u8)rnd();
      bad += check(x, "text+random");
      ++cases;
    }
  }
  printf("%d cases, %d mismatches\n", cases, bad);
  printf("frags %llu blocks %llu (%.1f/frag) events %llu (%.2f/block) probes %llu (%.2f/block) pred_rounds %.2f/block "
         "deep %llu slow_resolve %llu long_match %llu jumps %llu direct_inserts %llu\n",
         (unsigned long long)st.frags, (unsigned long long)st.blocks, (double)st.blocks / st.frags,
         (unsigned long long)st.events, (double)st.events / st.blocks, (unsigned long long)st.probes,
         (double)st.probes / st.blocks, (double)st.pred_rounds / st.blocks, (unsigned long long)st.deep,
         (unsigned long long)st.slow_resolve, (unsigned long long)st.long_match, (unsigned long long)st.jumps,
         (unsigned long long)st.direct_inserts);
  // C3-only statistics
  st = Stats();
  for (u32 t = 0; t < 256; ++t) {
    std::vector<u8> x(65536), o(so_max_compressed_length(65536) + 64);
    dg_text_body(t * 257, x.data(), x.size());
    wenc_compress(x.data(), x.size(), o.data());
  }
  printf("C3 fast-path events %.1f%%; others per block: not post %.3f, pred at ip %.3f, pred in search %.3f, "
         "search past 32 %.3f, long match %.3f\n", 100.0 * st.fast / st.events, (double)st.why[0] / st.blocks,
         (double)st.why[1] / st.blocks, (double)st.why[2] / st.blocks, (double)st.why[3] / st.blocks,
         (double)st.why[4] / st.blocks);
  {
    Stats c3 = st;
    st = Stats();
    for (u32 t = 0; t < 300; ++t) {
      std::vector<u8> x(70000 + 64), o(so_max_compressed_length(70064) + 64);
      const size_t nn = dg_snappy_message(t * 31, 16384 + (u32)(rnd() % 48000), x.data());
      wenc_compress(x.data(), nn, o.data());
    }
    printf("proto 16-64K: events %.2f/block probes %.2f/block pred_rounds %.2f/block slow %llu fast-path events %.1f%%\n",
           (double)st.events / st.blocks, (double)st.probes / st.blocks, (double)st.pred_rounds / st.blocks,
           (unsigned long long)st.slow_resolve, 100.0 * st.fast / st.events);
    st = c3;
  }
  printf("C3: blocks %.1f/frag events %.2f/block probes %.2f/block pred_rounds %.2f/block slow %llu kernel-slow %llu long %llu "
         "jumps %llu\n",
         (double)st.blocks / st.frags, (double)st.events / st.blocks, (double)st.probes / st.blocks,
         (double)st.pred_rounds / st.blocks, (unsigned long long)st.slow_resolve, (unsigned long long)st.deep,
         (unsigned long long)st.long_match, (unsigned long long)st.jumps);
  return bad != 0;
}
