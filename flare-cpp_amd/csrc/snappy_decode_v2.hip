// snappy_decode_v2.hip -- latency-tolerant batched Snappy decode for gfx950.
//
// One LANE per message (64 messages per wave), like decode_lane_kernel, but
// restructured so a lane pays ONE memory round trip per batch of up to
// kPieces output pieces instead of several dependent round trips per tag:
//
//   1. the next 32 input bytes sit in registers (two 16-byte chunks loaded at
//      the end of the previous batch), so tag headers are parsed with VALU
//      byte selects, never with dependent loads;
//   2. each tag is cut into <=16-byte pieces; a batch parses up to kPieces
//      pieces and issues one 16-byte load per piece (literal bytes from the
//      input, copy bytes from this message's already-written output);
//   3. one wait, then one 16-byte store per piece.
//
// A copy whose source overlaps output still pending in the current batch
// (offset too small) closes the batch early; the next batch's loads are
// issued after this batch's stores in program order, which the hardware
// keeps ordered for one lane's same-address accesses.  Copies with
// offset < 16 (pattern replication, snappy.cc:98-152) are expanded in
// registers from the `offset` pattern bytes.  All reference checks
// (snappy.cc:716-868, writer checks :1141-1481) are applied per tag exactly
// as in decode_lane_kernel; statuses are identical.
#include "snappy_device.h"

namespace fsg {

constexpr int kPieces = 12;
constexpr u32 kWinBytes = 64;  // register window of input bytes

__device__ __forceinline__ u32 mux8(const u32 (&w)[8], u32 d) {
  // d in [0, 8): binary tree of selects (keeps the window in registers)
  u32 a0 = (d & 1) ? w[1] : w[0];
  u32 a1 = (d & 1) ? w[3] : w[2];
  u32 a2 = (d & 1) ? w[5] : w[4];
  u32 a3 = (d & 1) ? w[7] : w[6];
  u32 b0 = (d & 2) ? a1 : a0;
  u32 b1 = (d & 2) ? a3 : a2;
  return (d & 4) ? b1 : b0;
}

// Register-resident select: v_cndmask trees written as masks so the compiler
// cannot turn the window into a dynamically indexed (scratch) array.
__device__ __forceinline__ u32 pick(u32 m, u32 a, u32 b) { return (b & m) | (a & ~m); }
__device__ __forceinline__ u32 mux16(const u32 (&w)[16], u32 d) {
  const u32 m0 = 0u - (d & 1), m1 = 0u - ((d >> 1) & 1), m2 = 0u - ((d >> 2) & 1),
            m3 = 0u - ((d >> 3) & 1);
  u32 a[8], b[4], c[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = pick(m0, w[2 * i], w[2 * i + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i) b[i] = pick(m1, a[2 * i], a[2 * i + 1]);
#pragma unroll
  for (int i = 0; i < 2; ++i) c[i] = pick(m2, b[2 * i], b[2 * i + 1]);
  return pick(m3, c[0], c[1]);
}

__device__ __forceinline__ u32 alignbyte(u32 hi, u32 lo, u32 s) {
  return __builtin_amdgcn_alignbyte(hi, lo, s);  // (hi:lo) >> (8*s), low 32 bits
}

// 16-byte load that never touches bytes at or beyond `limit` (exclusive,
// absolute): plain unaligned load when safe, else aligned chunks + funnel.
__device__ __forceinline__ u32x4 load16_guarded(const u8* p, const u8* limit) {
  u32x4 v;
  if (p + 16 <= limit) {
    __builtin_memcpy(&v, p, 16);
    return v;
  }
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const u8* c0 = reinterpret_cast<const u8*>(a & ~uintptr_t(15));
  const u32 sh = (u32)(a & 15);
  u32x4 x = *reinterpret_cast<const u32x4*>(c0);  // contains p: safe
  u32x4 y = {0, 0, 0, 0};
  if (c0 + 16 < limit) y = *reinterpret_cast<const u32x4*>(c0 + 16);
  u32 t[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  const u32 d = sh >> 2, b = sh & 3;
  u32 r0 = alignbyte(mux8(t, d + 1), mux8(t, d), b);
  u32 r1 = alignbyte(mux8(t, d + 2), mux8(t, d + 1), b);
  u32 r2 = alignbyte(mux8(t, d + 3), mux8(t, d + 2), b);
  u32 r3 = alignbyte(d + 4 < 8 ? mux8(t, d + 4) : 0u, mux8(t, d + 3), b);
  v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3;
  return v;
}

// Store the first n (1..16) bytes of v at p exactly.
__device__ __forceinline__ void store_exact(u8* p, u32x4 v, u32 n) {
  if (n == 16) { __builtin_memcpy(p, &v, 16); return; }
  u64 lo = (u64)v[0] | ((u64)v[1] << 32);
  u64 hi = (u64)v[2] | ((u64)v[3] << 32);
  if (n & 8) { stu64(p, lo); p += 8; lo = hi; }
  if (n & 4) { stu32(p, (u32)lo); p += 4; lo >>= 32; }
  if (n & 2) { u16 s = (u16)lo; __builtin_memcpy(p, &s, 2); p += 2; lo >>= 16; }
  if (n & 1) { *p = (u8)lo; }
}

__device__ __forceinline__ int parse_header_v2(const u8* ip, u32 n, bool strict, u32* ulen) {
  u32 r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((u32)i >= n) return 0;
    u32 c = ip[i];
    r |= (c & 0x7fu) << (7 * i);
    if (c < 128) {
      if (strict && i == 4 && c >= 16) return 0;
      *ulen = r;
      return i + 1;
    }
  }
  return 0;
}

// Byte k of a little-endian 16-byte register block.
__device__ __forceinline__ u32 byte_of(u32x4 v, u32 k) {
  u32 d = k >> 2;
  u32 w = d == 0 ? v[0] : d == 1 ? v[1] : d == 2 ? v[2] : v[3];
  return (w >> (8 * (k & 3))) & 0xffu;
}

__global__ __launch_bounds__(64) void decode_batch_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_cap,
    u32* __restrict__ out_len, i32* __restrict__ status_out, u32 flags) {
  const u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool strict = flags & 2u;
  i32 status = -1;  // -1 = running
  const u8* ib = nullptr;
  u8* ob = nullptr;
  u32 n_in = 0, expected = 0, ip = 0, op = 0;
  if (m < n_msgs) {
    ib = in + in_off[m];
    n_in = in_len[m];
    u32 ulen = 0;
    int h = parse_header_v2(ib, n_in, strict, &ulen);
    if (h == 0) {
      status = kBadHeader;
      out_len[m] = 0;
    } else {
      out_len[m] = ulen;
      if (ulen > out_cap[m]) status = kSlotTooSmall;
      expected = ulen;
      ip = (u32)h;
      ob = out + out_off[m];
    }
  } else {
    status = kOk;  // idle lane
  }
  const u8* in_end = ib + n_in;
  u8* const out_end = ob + expected;

  // current tag being cut into pieces
  u32 rem = 0;      // bytes of the current tag still to emit
  u32 src = 0;      // literal: input offset; copy: output offset
  bool lit = false;

  // 64-byte input window (registers), aligned to 16 bytes.  The window for
  // the next batch is loaded in the same round trip as this batch's pieces.
  u32 win[16];
  const u8* wptr = nullptr;
#define LOAD_WINDOW()                                                           \
  do {                                                                          \
    const u8* p_ = ib + ip;                                                     \
    wptr = reinterpret_cast<const u8*>(reinterpret_cast<uintptr_t>(p_) & ~uintptr_t(15)); \
    _Pragma("unroll") for (int c_ = 0; c_ < 4; ++c_) {                          \
      u32x4 a_ = {0, 0, 0, 0};                                                  \
      if (wptr + 16 * c_ < in_end) a_ = *reinterpret_cast<const u32x4*>(wptr + 16 * c_); \
      win[4 * c_ + 0] = a_[0]; win[4 * c_ + 1] = a_[1];                         \
      win[4 * c_ + 2] = a_[2]; win[4 * c_ + 3] = a_[3];                         \
    }                                                                           \
  } while (0)
  if (status < 0) LOAD_WINDOW();

  while (__any(status < 0)) {
    // ---------------- parse phase: up to kPieces pieces ----------------
    const u32 batch_start = op;
    bool closed = status >= 0;
    bool slow = false;  // a copy with offset < 16 is next
    u32 slow_off = 0;
    u32x4 data[kPieces];
    u32 dst[kPieces];
    u32 cnt[kPieces];
#pragma unroll
    for (int j = 0; j < kPieces; ++j) {
      cnt[j] = 0;
      dst[j] = 0;
      data[j] = u32x4{0, 0, 0, 0};
      if (!closed && rem == 0) {
        // need a new tag header
        if (ip == n_in) {
          status = (op == expected) ? kOk : kCorrupt;  // eof (RefillTag)
          closed = true;
        } else {
          const u32 o = (u32)((ib + ip) - wptr);
          if (o > kWinBytes - 5) {
            closed = true;  // header may run past the register window
          } else {
            const u32 d = o >> 2, bsh = o & 3;
            const u32 lo = mux16(win, d), hi = mux16(win, d + 1);
            const u32 t0 = alignbyte(hi, lo, bsh);          // bytes o..o+3
            const u32 b4 = (hi >> (8 * bsh)) & 0xffu;        // byte o+4
            const u32 c = t0 & 0xffu;
            const u32 avail = n_in - ip - 1;                 // bytes after the tag byte
            const u32 space = expected - op;
            if ((c & 3) == 0) {
              u32 len = (c >> 2) + 1;
              u32 hl = 1;
              if (len >= 61) {
                const u32 nb = len - 60;
                if (avail < nb) { status = kCorrupt; closed = true; }
                else {
                  const u64 ext = ((u64)b4 << 24) | (t0 >> 8);  // bytes o+1..o+4
                  const u32 v = (u32)(ext & (nb == 4 ? 0xffffffffull : ((1ull << (8 * nb)) - 1)));
                  len = v + 1;  // uint32 wrap (snappy.cc:747-748)
                  hl = 1 + nb;
                }
              }
              if (!closed) {
                if (avail - (hl - 1) < len || space < len) { status = kCorrupt; closed = true; }
                else {
                  lit = true;
                  src = ip + hl;
                  rem = len;
                  ip += hl + len;
                }
              }
            } else {
              const u32 type = c & 3;
              const u32 nb = type == 1 ? 1u : (type == 2 ? 2u : 4u);
              u32 len, off;
              if (type == 1) {
                len = 4 + ((c >> 2) & 7);
                off = ((c >> 5) << 8) | ((t0 >> 8) & 0xffu);
              } else if (type == 2) {
                len = (c >> 2) + 1;
                off = (t0 >> 8) & 0xffffu;
              } else {
                len = (c >> 2) + 1;
                off = (t0 >> 8) | (b4 << 24);
              }
              if (avail < nb) { status = kCorrupt; closed = true; }
              else if (off - 1u >= op || space < len) { status = kCorrupt; closed = true; }
              else if (off < 16) {
                // pattern copy: handled after this batch is flushed
                if (op == batch_start) {
                  slow = true;
                  slow_off = off;
                  ip += 1 + nb;
                  lit = false;
                  rem = len;
                  src = op - off;
                }
                closed = true;
              } else {
                lit = false;
                src = op - off;
                rem = len;
                ip += 1 + nb;
              }
            }
          }
        }
      }
      if (!closed && rem > 0) {
        const u32 n = rem < 16 ? rem : 16;
        if (!lit && src + n > batch_start) {
          closed = true;  // source still pending in this batch
        } else {
          const u8* sp = lit ? ib + src : ob + src;
          const u8* lim = lit ? in_end : out_end;
          data[j] = load16_guarded(sp, lim);
          dst[j] = op;
          cnt[j] = n;
          src += n;
          op += n;
          rem -= n;
        }
      }
    }
    // next batch's window: issued with this batch's piece loads (one round trip)
    if (status < 0 && !slow) LOAD_WINDOW();
    // ---------------- store phase ----------------
#pragma unroll
    for (int j = 0; j < kPieces; ++j) {
      if (cnt[j]) {
        u8* dp = ob + dst[j];
        if (dp + 16 <= out_end) __builtin_memcpy(dp, &data[j], 16);
        else store_exact(dp, data[j], cnt[j]);
      }
    }
    // ---------------- pattern copy (offset < 16) ----------------
    if (slow) {
      // pattern = the `slow_off` bytes before op (all final: flushed above)
      u32x4 pat = load16_guarded(ob + src, out_end);  // bytes src .. src+15, first slow_off valid
      u32 kk = 0;  // pattern phase: output byte i of the tag = pattern[i mod off]
      while (rem > 0) {
        const u32 n = rem < 16 ? rem : 16;
        u32 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          u32 acc = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc |= byte_of(pat, kk) << (8 * r);
            kk = (kk + 1 == slow_off) ? 0u : kk + 1;
          }
          w[q] = acc;
        }
        u32x4 v = {w[0], w[1], w[2], w[3]};
        u8* dp = ob + op;
        if (dp + 16 <= out_end) __builtin_memcpy(dp, &v, 16);
        else store_exact(dp, v, n);
        op += n;
        rem -= n;
      }
    }
    // the pattern copy consumed no window bytes beyond ip; reload after it
    if (status < 0 && slow) LOAD_WINDOW();
  }
  if (m < n_msgs) status_out[m] = status;
}

hipError_t launch_decode_v2(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  decode_batch_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(
      in, in_off, in_len, n_msgs, out, out_off, out_cap, out_len, status, flags);
  return hipGetLastError();
}

}  // namespace fsg
