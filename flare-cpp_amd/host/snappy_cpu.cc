// snappy_cpu.cc -- see snappy_cpu.h.
#include "snappy_cpu.h"

#include <algorithm>
#include <cstring>
#include <memory>

namespace flare::snappy::cpu {

namespace {

constexpr size_t kFragment = 1u << 16;        // snappy.h kBlockSize
constexpr uint32_t kMaxTable = 1u << 14;      // snappy.h kMaxHashTableSize
constexpr size_t kInputMargin = 15;           // snappy.cc:346

inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint64_t load64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

// snappy.cc:46-53: multiplicative hash of 4 little-endian bytes.
inline uint32_t hash4(uint32_t bytes, int shift) { return (bytes * 0x1e35a7bdu) >> shift; }

// snappy-internal.h:87-121: bytes equal between s1 and s2, s2 < s2_end.
inline size_t match_length(const uint8_t* s1, const uint8_t* s2, const uint8_t* s2_end) {
  size_t m = 0;
  while (s2 + m + 8 <= s2_end) {
    const uint64_t x = load64(s1 + m) ^ load64(s2 + m);
    if (x) return m + ((size_t)__builtin_ctzll(x) >> 3);
    m += 8;
  }
  while (s2 + m < s2_end && s1[m] == s2[m]) ++m;
  return m;
}

// snappy.cc:156-196 (length n = len - 1 in 1..4 trailing bytes above 59).
// Literals of <= 16 bytes copy 16 (the reference's fast path, :172-180): the
// input has >= 15 bytes after any literal the main loop emits, and the output
// buffer's MaxCompressedLength slack covers the over-write.
inline uint8_t* emit_literal(uint8_t* op, const uint8_t* lit, size_t len, bool fast) {
  uint32_t n = (uint32_t)(len - 1);
  if (fast && len <= 16) {
    *op++ = (uint8_t)(n << 2);
    memcpy(op, lit, 16);
    return op + len;
  }
  if (n < 60) {
    *op++ = (uint8_t)(n << 2);
  } else {
    uint8_t* tag = op++;
    int count = 0;
    while (n > 0) {
      *op++ = (uint8_t)n;
      n >>= 8;
      ++count;
    }
    *tag = (uint8_t)((59 + count) << 2);
  }
  memcpy(op, lit, len);
  return op + len;
}

// snappy.cc:198-214: one copy of 4..64 bytes, COPY_1 when it fits.
inline uint8_t* emit_copy_lt64(uint8_t* op, size_t offset, size_t len) {
  if (len < 12 && offset < 2048) {
    *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    *op++ = (uint8_t)offset;
  } else {
    *op++ = (uint8_t)(2 + ((len - 1) << 2));
    *op++ = (uint8_t)offset;
    *op++ = (uint8_t)(offset >> 8);
  }
  return op;
}

// snappy.cc:216-232: 64-byte copies while >= 68 remain, a 60 if 65..67 remain.
inline uint8_t* emit_copy(uint8_t* op, size_t offset, size_t len) {
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

// internal::CompressFragment, snappy.cc:329-453.  `table` has `entries`
// (a power of two, 256..16384) zeroed u16 slots.
uint8_t* compress_fragment(const uint8_t* in, size_t n, uint8_t* op, uint16_t* table, uint32_t entries) {
  const int shift = 32 - __builtin_ctz(entries);
  const uint8_t* ip = in;
  const uint8_t* const base = in;
  const uint8_t* const ip_end = in + n;
  const uint8_t* next_emit = in;
  if (n >= kInputMargin) {
    const uint8_t* const ip_limit = in + n - kInputMargin;
    uint32_t next_hash = hash4(load32(++ip), shift);
    for (;;) {
      // probe with the skip heuristic (:372-397): the step grows by one
      // every 32 misses
      uint32_t skip = 32;
      const uint8_t* next_ip = ip;
      const uint8_t* cand;
      do {
        ip = next_ip;
        const uint32_t h = next_hash;
        next_ip = ip + (skip++ >> 5);
        if (next_ip > ip_limit) goto emit_remainder;
        next_hash = hash4(load32(next_ip), shift);
        cand = base + table[h];
        table[h] = (uint16_t)(ip - base);
      } while (load32(ip) != load32(cand));
      op = emit_literal(op, next_emit, (size_t)(ip - next_emit), true);
      // copies while the position after each one matches again (:404-444)
      uint32_t cand_bytes;
      uint64_t eight;
      do {
        const uint8_t* const start = ip;
        const size_t matched = 4 + match_length(cand + 4, ip + 4, ip_end);
        ip += matched;
        op = emit_copy(op, (size_t)(start - cand), matched);
        next_emit = ip;
        if (ip >= ip_limit) goto emit_remainder;
        eight = load64(ip - 1);
        table[hash4((uint32_t)eight, shift)] = (uint16_t)(ip - base - 1);
        const uint32_t cur = hash4((uint32_t)(eight >> 8), shift);
        cand = base + table[cur];
        cand_bytes = load32(cand);
        table[cur] = (uint16_t)(ip - base);
      } while ((uint32_t)(eight >> 8) == cand_bytes);
      next_hash = hash4((uint32_t)(eight >> 16), shift);
      ++ip;
    }
  }
emit_remainder:
  if (next_emit < ip_end) op = emit_literal(op, next_emit, (size_t)(ip_end - next_emit), false);
  return op;
}

// Extra bytes after a tag byte: a literal's 1..4 length bytes (lengths
// 61..64), a copy's 1, 2 or 4 offset bytes (char_table, snappy.cc:516-549).
inline size_t tag_extra(uint8_t c) {
  if ((c & 3) == 0) return (c >> 2) >= 60 ? (size_t)((c >> 2) - 59) : 0;
  return (c & 3) == 3 ? 4 : (c & 3);
}

inline uint32_t load_le(const uint8_t* p, size_t k) {
  uint32_t v = 0;
  for (size_t i = 0; i < k; ++i) v |= (uint32_t)p[i] << (8 * i);
  return v;
}

// Copy of len bytes from op - off to op; `room` = writable bytes from op
// (>= len).  With >= len + 16 of room it over-copies in 8-byte steps like
// IncrementalCopyFastPath (snappy.cc:140-152): an offset below 8 first
// widens the pattern to 8 bytes.
inline void copy_back(uint8_t* d, size_t off, size_t len, size_t room) {
  const uint8_t* s = d - off;
  if (room >= len + 16) {
    if (off >= 8) {
      for (size_t i = 0; i < len; i += 8) memcpy(d + i, s + i, 8);
      return;
    }
    if (off >= len) {
      memcpy(d, s, 8);
      if (len > 8) memcpy(d + 8, s + 8, 8);
      return;
    }
  }
  if (off >= len) {
    memcpy(d, s, len);
  } else {
    for (size_t i = 0; i < len; ++i) d[i] = s[i];  // IncrementalCopy :98-103
  }
}

template <bool kWrite>
bool decode_tags(const uint8_t* ip, const uint8_t* end, uint8_t* out, uint32_t expected, size_t out_cap,
                 size_t* produced) {
  size_t op = 0;
  bool ok = false;
  for (;;) {
    if (ip == end) {  // RefillTag's eof: input ends between tags (:795-801)
      ok = op == expected;
      break;
    }
    const uint8_t c = *ip;
    const size_t extra = tag_extra(c);
    if ((size_t)(end - ip) < extra + 1) break;  // a tag cut by the end (:818-826)
    ++ip;
    if ((c & 3) == 0) {
      uint32_t len32 = (c >> 2) + 1u;
      if (len32 >= 61) len32 = load_le(ip, extra) + 1u;  // uint32: 0xffffffff + 1 == 0
      ip += extra;
      const size_t len = len32;
      if (kWrite && len <= 16 && (size_t)(end - ip) >= 16 && op + 16 <= out_cap && len <= expected - op) {
        memcpy(out + op, ip, 16);  // TryFastAppend (:1386-1398)
        op += len;
        ip += len;
        continue;
      }
      // the writer takes what the input holds and the header allows (:744-761,
      // SlowAppend :1424-1451); any shortfall fails the stream
      const size_t take = std::min({len, (size_t)(end - ip), (size_t)expected - op});
      if (kWrite) memcpy(out + op, ip, take);
      op += take;
      if (take < len) break;
      ip += len;
    } else {
      size_t len, off;
      if ((c & 3) == 1) {
        len = 4 + ((c >> 2) & 7);
        off = ((size_t)(c >> 5) << 8) | ip[0];
      } else {
        len = (c >> 2) + 1u;
        off = load_le(ip, extra);
      }
      ip += extra;
      // offset 0 or beyond the output so far; no room left (:1200-1210,
      // :1410-1413, :1463-1466): all-or-nothing
      if (off - 1u >= op || (size_t)expected - op < len) break;
      if (kWrite) copy_back(out + op, off, len, out_cap - op);
      op += len;
    }
  }
  if (produced) *produced = op;
  return ok;
}

// Byte source over fragments (Source::Peek/Skip).
struct FragReader {
  const uint8_t* const* frag;
  const size_t* len;
  size_t n, k = 0, pos = 0;
  size_t avail() const { return k < n ? len[k] - pos : 0; }
  const uint8_t* ptr() const { return frag[k] + pos; }
  void settle() {  // skip empty / used-up fragments
    while (k < n && pos == len[k]) {
      ++k;
      pos = 0;
    }
  }
  bool get(uint8_t* c) {
    settle();
    if (k == n) return false;
    *c = frag[k][pos++];
    return true;
  }
};

// SnappyScatteredWriter (snappy.cc:1331-1481) with the positions of its
// blocks; bytes land at their absolute output positions.
struct ScatterModel {
  std::vector<uint8_t>* out;
  size_t expected;
  size_t full = 0;      // full_size_
  size_t blk_len = 0;   // op_limit_ - op_base_ (0: no block yet)
  size_t blk_used = 0;  // op_ptr_ - op_base_
  size_t size() const { return full + blk_used; }
  void put(const uint8_t* ip, size_t n) {
    const size_t at = full + blk_used;
    if (out->size() < at + n) out->resize(at + n);
    memcpy(out->data() + at, ip, n);
    blk_used += n;
  }
  bool append(const uint8_t* ip, size_t len) {
    size_t avail = blk_len - blk_used;
    if (len <= avail) {
      put(ip, len);
      return true;
    }
    while (len > avail) {  // SlowAppend
      put(ip, avail);
      full += blk_used;  // full_size_ += op_ptr_ - op_base_
      len -= avail;
      ip += avail;
      if (full + len > expected) return false;  // op_base_/op_ptr_ keep the filled block
      blk_len = std::min<size_t>(kFragment, expected - full);
      blk_used = 0;
      avail = blk_len;
    }
    put(ip, len);
    return true;
  }
  bool append_from_self(size_t offset, size_t len) {
    const size_t cur = size();
    if (offset - 1u >= cur || expected - cur < len) return false;
    for (size_t i = 0; i < len; ++i) {
      const uint8_t c = (*out)[cur - offset + i];
      append(&c, 1);
    }
    return true;
  }
};

}  // namespace

size_t UncompressAsMuchAsPossible(const uint8_t* const* frag, const size_t* frag_len, size_t n_frag,
                                  std::vector<uint8_t>* out) {
  out->clear();
  FragReader r{frag, frag_len, n_frag};
  uint32_t expected = 0;
  {  // ReadUncompressedLength (snappy.cc:692-711)
    uint32_t shift = 0;
    for (;;) {
      uint8_t c;
      if (shift >= 32 || !r.get(&c)) return 0;
      expected |= (uint32_t)(c & 0x7f) << shift;
      if (c < 128) break;
      shift += 7;
    }
  }
  ScatterModel w{out, expected};
  for (;;) {
    // a whole tag (byte + extra bytes) from one or more fragments (RefillTag)
    uint8_t c;
    if (!r.get(&c)) break;  // eof between tags
    const size_t extra = tag_extra(c);
    uint8_t e[4] = {0, 0, 0, 0};
    bool whole = true;
    for (size_t i = 0; i < extra && whole; ++i) whole = r.get(&e[i]);
    if (!whole) break;
    if ((c & 3) == 0) {
      uint32_t len32 = (c >> 2) + 1u;
      if (len32 >= 61) len32 = load_le(e, extra) + 1u;
      size_t len = len32;
      bool ok = true;
      for (;;) {  // the literal, fragment by fragment (:751-761)
        r.settle();
        const size_t a = r.avail();
        if (a >= len) {
          if (len) {
            ok = w.append(r.ptr(), len);
            r.pos += len;
          }
          break;
        }
        if (a == 0 || !w.append(r.ptr(), a)) {  // premature end of input, or no room
          ok = false;
          break;
        }
        len -= a;
        r.pos += a;
      }
      if (!ok) break;
    } else {
      size_t len, off;
      if ((c & 3) == 1) {
        len = 4 + ((c >> 2) & 7);
        off = ((size_t)(c >> 5) << 8) | e[0];
      } else {
        len = (c >> 2) + 1u;
        off = load_le(e, extra);
      }
      if (!w.append_from_self(off, len)) break;
    }
  }
  // the sink got every byte written (Flush(Produced()) stops at the blocks
  // allocated); the count is Produced() itself
  return w.size();
}

size_t ReadHeader(const uint8_t* in, size_t n, uint32_t* len, bool strict) {
  uint32_t r = 0;
  for (size_t i = 0; i < 5; ++i) {
    if (i >= n) return 0;
    const uint8_t c = in[i];
    r |= (uint32_t)(c & 0x7f) << (7 * i);  // i == 4: bits above 31 fall off
    if (c < 128) {
      if (strict && i == 4 && c >= 16) return 0;
      *len = r;
      return i + 1;
    }
  }
  return 0;
}

size_t Compress(const uint8_t* in, size_t n, uint8_t* out) {
  uint8_t* op = out;
  uint32_t v = (uint32_t)n;  // Varint::Encode32 (snappy-stubs-internal.h:359-385)
  while (v >= 128) {
    *op++ = (uint8_t)(v | 128);
    v >>= 7;
  }
  *op++ = (uint8_t)v;
  // the hash table per call, as WorkingMemory (snappy.cc:247-271): on the
  // stack up to 4096 entries, else on the heap (no thread_local: TLS access
  // from this library measured 2x slower once the HIP runtime is up)
  uint16_t small[4096];
  std::unique_ptr<uint16_t[]> big;
  uint16_t* table = small;
  if (n > 4096) {
    big.reset(new uint16_t[kMaxTable]);
    table = big.get();
  }
  for (size_t pos = 0; pos < n; pos += kFragment) {
    const size_t frag = std::min(kFragment, n - pos);
    uint32_t entries = 256;  // WorkingMemory::GetHashTable (:247-271)
    while (entries < kMaxTable && entries < frag) entries <<= 1;
    memset(table, 0, entries * sizeof(uint16_t));
    op = compress_fragment(in + pos, frag, op, table, entries);
  }
  return (size_t)(op - out);
}

bool Decode(const uint8_t* in, size_t n, size_t hdr, uint8_t* out, uint32_t expected, size_t* produced,
            size_t out_cap) {
  return decode_tags<true>(in + hdr, in + n, out, expected, out_cap > expected ? out_cap : expected, produced);
}

bool Uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, bool strict) {
  uint32_t ulen = 0;
  const size_t h = ReadHeader(in, n, &ulen, strict);
  if (h == 0 || ulen > out_cap) return false;
  return decode_tags<true>(in + h, in + n, out, ulen, out_cap, nullptr);
}

bool IsValid(const uint8_t* in, size_t n) {
  uint32_t ulen = 0;
  const size_t h = ReadHeader(in, n, &ulen, false);
  return h != 0 && decode_tags<false>(in + h, in + n, nullptr, ulen, 0, nullptr);
}

}  // namespace flare::snappy::cpu
