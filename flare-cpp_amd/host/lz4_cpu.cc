// lz4_cpu.cc -- host LZ4 block codec (see lz4_cpu.h).
#include "lz4_cpu.h"

#include <cstring>
#include <vector>

namespace flare::lz4::cpu {

namespace {

constexpr size_t kMinMatch = 4, kMfLimit = 12, kLastLiterals = 5;
constexpr size_t kSmallLimit = 65536 + kMfLimit - 1;  // 16-bit positions below
constexpr size_t kDistanceMax = 65535;

inline uint32_t Load32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t Load64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

// Position table of one block: 8,192 x u16 (small inputs, 4-byte hash) or
// 4,096 x u32 (5-byte hash), zeroed -- the state of a fresh LZ4 stream.
class Table {
 public:
  explicit Table(bool small) : small_(small) { std::memset(slots_, 0, sizeof slots_); }
  uint32_t Hash(const uint8_t* p) const {
    return small_ ? (Load32(p) * 2654435761u) >> 19
                  : static_cast<uint32_t>(((Load64(p) << 24) * 889523592379ull) >> 52);
  }
  uint32_t Get(uint32_t h) const {
    return small_ ? reinterpret_cast<const uint16_t*>(slots_)[h] : slots_[h];
  }
  void Set(uint32_t h, size_t pos) {
    if (small_) reinterpret_cast<uint16_t*>(slots_)[h] = static_cast<uint16_t>(pos);
    else slots_[h] = static_cast<uint32_t>(pos);
  }
  // a candidate the format can reach (16-bit positions are always in range)
  bool Reachable(size_t cand, size_t pos) const { return small_ || cand + kDistanceMax >= pos; }

 private:
  bool small_;
  uint32_t slots_[4096];
};

uint8_t* PutRun(uint8_t* op, size_t len) {  // 255-continued length bytes
  while (len >= 255) {
    *op++ = 255;
    len -= 255;
  }
  *op++ = static_cast<uint8_t>(len);
  return op;
}

size_t CommonLength(const uint8_t* a, const uint8_t* b, const uint8_t* limit) {
  size_t c = 0;
  while (a + c + 8 <= limit) {
    const uint64_t x = Load64(a + c) ^ Load64(b + c);
    if (x) return c + (__builtin_ctzll(x) >> 3);
    c += 8;
  }
  while (a + c < limit && a[c] == b[c]) ++c;
  return c;
}

// Literal run [from, from + len) behind a token whose high nibble it sets.
uint8_t* EmitLiterals(uint8_t* token, const uint8_t* from, size_t len) {
  uint8_t* op = token + 1;
  if (len >= 15) {
    *token = 15 << 4;
    op = PutRun(op, len - 15);
  } else {
    *token = static_cast<uint8_t>(len << 4);
  }
  std::memcpy(op, from, len);
  return op + len;
}

}  // namespace

size_t CompressBlock(const uint8_t* in, size_t n, uint8_t* out) {
  uint8_t* op = out;
  size_t anchor = 0;
  if (n > kMfLimit) {
    Table t(n < kSmallLimit);
    const size_t match_end = n - kMfLimit + 1;  // matches start below this
    const uint8_t* const count_limit = in + n - kLastLiterals;
    t.Set(t.Hash(in), 0);
    size_t pos = 1;
    uint32_t next_hash = t.Hash(in + pos);
    for (;;) {
      size_t cand = 0;
      bool found = false;
      // probe forward; after every 64 misses the step grows by one
      for (size_t probe = pos, step = 1, misses = 64;;) {
        const uint32_t h = next_hash;
        const size_t here = probe;
        const uint32_t c = t.Get(h);
        pos = probe;
        probe += step;
        step = misses++ >> 6;
        if (probe > match_end) break;
        next_hash = t.Hash(in + probe);
        t.Set(h, here);
        if (!t.Reachable(c, here)) continue;
        if (Load32(in + c) == Load32(in + pos)) {
          cand = c;
          found = true;
          break;
        }
      }
      if (!found) break;
      while (pos > anchor && cand > 0 && in[pos - 1] == in[cand - 1]) {
        --pos;
        --cand;
      }
      uint8_t* token = op;
      op = EmitLiterals(token, in + anchor, pos - anchor);
      bool done = false;
      for (;;) {
        const size_t off = pos - cand;
        op[0] = static_cast<uint8_t>(off);
        op[1] = static_cast<uint8_t>(off >> 8);
        op += 2;
        const size_t extra = CommonLength(in + pos + kMinMatch, in + cand + kMinMatch, count_limit);
        pos += kMinMatch + extra;
        if (extra >= 15) {
          *token += 15;
          op = PutRun(op, extra - 15);
        } else {
          *token += static_cast<uint8_t>(extra);
        }
        anchor = pos;
        if (pos >= match_end) {
          done = true;
          break;
        }
        t.Set(t.Hash(in + pos - 2), pos - 2);
        const uint32_t h = t.Hash(in + pos);
        const uint32_t c = t.Get(h);
        t.Set(h, pos);
        if (!t.Reachable(c, pos) || Load32(in + c) != Load32(in + pos)) break;
        cand = c;  // another match right away: a token with no literals
        token = op++;
        *token = 0;
      }
      if (done) break;
      next_hash = t.Hash(in + ++pos);
    }
  }
  return static_cast<size_t>(EmitLiterals(op, in + anchor, n - anchor) - out);
}

bool DecompressBlock(const uint8_t* in, size_t n, uint8_t* out, size_t ulen) {
  size_t ip = 0, op = 0;
  auto run = [&](size_t& len, size_t bound) {  // 255-continued length bytes
    for (;;) {
      if (ip >= n) return false;
      const unsigned b = in[ip++];
      len += b;
      if (b != 255 || len > bound) return true;
    }
  };
  for (;;) {
    if (ip >= n) return false;
    const unsigned token = in[ip++];
    size_t lit = token >> 4;
    if (lit == 15 && !run(lit, n)) return false;
    if (lit > n - ip || lit > ulen - op) return false;
    if (op + lit + kMfLimit > ulen || ip + lit + 3 + kLastLiterals > n) {
      // the last sequence: literals only, ending the input and the output
      if (ip + lit != n) return false;
      std::memcpy(out + op, in + ip, lit);
      return op + lit == ulen;
    }
    std::memcpy(out + op, in + ip, lit);
    ip += lit;
    op += lit;
    const size_t off = in[ip] | (static_cast<size_t>(in[ip + 1]) << 8);
    ip += 2;
    if (off == 0 || off > op) return false;
    size_t len = (token & 15) + kMinMatch;
    if ((token & 15) == 15 && !run(len, ulen)) return false;
    if (len + kLastLiterals > ulen - op) return false;
    uint8_t* d = out + op;
    if (off >= len) {
      std::memcpy(d, d - off, len);
    } else {
      const uint8_t* from = d - off;  // overlapping: byte by byte, in order
      for (size_t k = 0; k < len; ++k) d[k] = from[k];
    }
    op += len;
  }
}

size_t ReadHeader(const uint8_t* in, size_t n, uint32_t* ulen) {
  uint32_t v = 0;
  for (size_t i = 0; i < 5 && i < n; ++i) {
    v |= static_cast<uint32_t>(in[i] & 0x7f) << (7 * i);
    if (in[i] < 128) {
      if (i == 4 && in[i] >= 16) return 0;
      *ulen = v;
      return i + 1;
    }
  }
  return 0;
}

size_t Compress(const uint8_t* in, size_t n, uint8_t* out) {
  if (n > kMaxInput) return 0;
  size_t h = 0;
  for (uint32_t v = static_cast<uint32_t>(n);; v >>= 7) {
    out[h++] = static_cast<uint8_t>(v < 128 ? v : (v | 0x80));
    if (v < 128) break;
  }
  return h + CompressBlock(in, n, out + h);
}

}  // namespace flare::lz4::cpu
