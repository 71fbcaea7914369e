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
  // keep pointer provenance (global address space): no integer round trip
  const u32 sh = (u32)(reinterpret_cast<uintptr_t>(p) & 15);
  const u8* c0 = p - sh;
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

// Address of a 16-byte load that covers [p, p + n) (p + n <= limit) and
// never touches memory outside [align16(start), limit) -- i.e. only bytes of
// the region or of the aligned 16-byte chunk holding its first byte.
// Returns the address; *sh = p - address (0..15; 0 whenever p + 16 <= limit).
// Branch-free, so every piece issues exactly one load and no wait is needed
// until the batch's store phase.
__device__ __forceinline__ const u8* safe16(const u8* p, const u8* start, const u8* limit, u32* sh) {
  const u8* lo = start - (reinterpret_cast<uintptr_t>(start) & 15);
  const u8* tail = limit - 16;
  const u8* a = (p + 16 <= limit) ? p : (tail > lo ? tail : lo);
  *sh = (u32)(p - a);
  return a;
}

// v >> (8 * sh) as a 16-byte little-endian value (sh in 0..15).
__device__ __forceinline__ u32x4 shr_bytes(u32x4 v, u32 sh) {
  u32 t[8] = {v[0], v[1], v[2], v[3], 0u, 0u, 0u, 0u};
  const u32 d = sh >> 2, b = sh & 3;
  u32x4 r;
  r[0] = alignbyte(mux8(t, d + 1), mux8(t, d), b);
  r[1] = alignbyte(mux8(t, d + 2), mux8(t, d + 1), b);
  r[2] = alignbyte(d + 3 < 8 ? mux8(t, d + 3) : 0u, mux8(t, d + 2), b);
  r[3] = alignbyte(d + 4 < 8 ? mux8(t, d + 4) : 0u, mux8(t, d + 3), b);
  return r;
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
    u32* __restrict__ out_len, i32* __restrict__ status_out, u32 flags,
    u32* __restrict__ work_counter) {
  // Persistent mode (work_counter != null): a bounded number of lanes pull
  // message indices from a device counter, so the number of messages in
  // flight -- and with it each lane's share of L2/MALL for its
  // back-reference window -- is a launch parameter.  Otherwise one lane per
  // message.
  const bool strict = flags & 2u;
  u32 m = n_msgs;
  i32 status = kOk;  // >= 0: idle / finished, -1: running
  const u8* ib = nullptr;
  u8* ob = nullptr;
  u32 n_in = 0, expected = 0, ip = 0, op = 0;
  const u8* in_end = nullptr;
  u8* out_end = nullptr;
  bool exhausted = false;  // no more messages for this lane

#define ACQUIRE_MESSAGE()                                                     \
  do {                                                                        \
    if (work_counter) m = atomicAdd(work_counter, 1u);                        \
    else m = exhausted ? n_msgs : blockIdx.x * blockDim.x + threadIdx.x;      \
    if (m >= n_msgs) { exhausted = true; status = kOk; break; }               \
    ib = in + in_off[m];                                                      \
    n_in = in_len[m];                                                         \
    in_end = ib + n_in;                                                       \
    op = 0;                                                                   \
    u32 ulen_ = 0;                                                            \
    const int h_ = parse_header_v2(ib, n_in, strict, &ulen_);                 \
    status = -1;                                                              \
    if (h_ == 0) { status = kBadHeader; out_len[m] = 0; expected = 0; }       \
    else {                                                                    \
      out_len[m] = ulen_;                                                     \
      if (ulen_ > out_cap[m]) status = kSlotTooSmall;                         \
      expected = ulen_;                                                       \
      ip = (u32)h_;                                                           \
      ob = out + out_off[m];                                                  \
      out_end = ob + expected;                                                \
    }                                                                         \
  } while (0)

  // current tag being cut into pieces
  u32 rem = 0;      // bytes of the current tag still to emit
  u32 src = 0;      // literal: input offset; copy: output offset
  bool lit = false;

  // 64-byte input window (registers), aligned to 16 bytes.  The window for
  // the next batch is loaded in the same round trip as this batch's pieces.
  u32 win[16];
  const u8* wptr = nullptr;
  u32 wip = 0;  // input offset of window byte 0 (mod 2^32)
#define LOAD_WINDOW()                                                           \
  do {                                                                          \
    const u8* p_ = ib + ip;                                                     \
    wptr = p_ - (reinterpret_cast<uintptr_t>(p_) & 15);                         \
    wip = ip - (u32)(reinterpret_cast<uintptr_t>(p_) & 15);                     \
    /* chunks past the input repeat the last chunk: safe to read, and the   \
       parser never uses bytes beyond n_in (avail checks) */                   \
    const u8* last_ = (in_end - 1) - (reinterpret_cast<uintptr_t>(in_end - 1) & 15); \
    _Pragma("unroll") for (int c_ = 0; c_ < 4; ++c_) {                          \
      const u8* q_ = wptr + 16 * c_;                                            \
      u32x4 a_ = *reinterpret_cast<const u32x4*>(q_ <= last_ ? q_ : last_);     \
      win[4 * c_ + 0] = a_[0]; win[4 * c_ + 1] = a_[1];                         \
      win[4 * c_ + 2] = a_[2]; win[4 * c_ + 3] = a_[3];                         \
    }                                                                           \
  } while (0)
  // first message (finished-at-init messages publish their status and pull again)
  for (;;) {
    ACQUIRE_MESSAGE();
    if (exhausted || status < 0) break;
    status_out[m] = status;
    if (!work_counter) { exhausted = true; break; }
  }
  if (status < 0) LOAD_WINDOW();
  else for (int i_ = 0; i_ < 16; ++i_) win[i_] = 0;

  // `w` is the parser's copy of the window.  It is only ever written by
  // opaque moves taken right after a wait, so the compiler never has a
  // pending load on it inside the divergent parse (where it would otherwise
  // re-wait vmcnt(0) at every piece and serialise the batch's loads).
  u32 w[16];
#define TAKE_WINDOW() \
  _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_) asm volatile("v_mov_b32 %0, %1" : "=v"(w[i_]) : "v"(win[i_]))
  TAKE_WINDOW();

  while (__any(status < 0)) {
    // ---------------- parse phase: up to kPieces pieces ----------------
    const u32 batch_start = op;
    bool closed = status >= 0;
    bool slow = false;  // a copy with offset < 16 is next
    u32 slow_off = 0;
    u32x4 data[kPieces];
    u32 dst[kPieces];
    u32 cnt[kPieces];
    u32 shf[kPieces];  // byte shift of each piece inside its 16-byte load
    // Straight-line piece steps: every decision is a select, so the wave runs
    // one instruction stream with no exec-mask branching; only the piece's
    // single 16-byte load is predicated.
#pragma unroll
    for (int j = 0; j < kPieces; ++j) {
      // ---- tag header at ip (evaluated always, committed only if needed)
      const bool need = !closed && rem == 0;
      const bool eof = need && ip == n_in;                   // RefillTag eof
      const u32 o = ip - wip;
      const bool inwin = o <= kWinBytes - 5;
      const u32 oc = inwin ? o : 0u;
      const u32 d = oc >> 2, bsh = oc & 3;
      const u32 lo = mux16(w, d), hi = mux16(w, d + 1);
      const u32 t0 = alignbyte(hi, lo, bsh);                 // bytes o..o+3
      const u32 b4 = (hi >> (8 * bsh)) & 0xffu;               // byte o+4
      const u32 c = t0 & 0xffu;
      const u32 type = c & 3;
      const bool is_lit = type == 0;
      const u32 l0 = (c >> 2) + 1;                            // LITERAL / COPY_2 / COPY_4 length
      const bool longlit = is_lit && l0 >= 61;                // 1..4 length bytes (:744-750)
      const u32 nbl = longlit ? l0 - 60 : 0u;
      const u32 ext = (b4 << 24) | (t0 >> 8);                 // bytes o+1..o+4, little endian
      const u32 msk = nbl >= 4 ? 0xffffffffu : ((1u << (8 * nbl)) - 1u);
      const u32 litlen = longlit ? (ext & msk) + 1u : l0;     // uint32 wrap: 0xffffffff+1 == 0
      const u32 nb = is_lit ? nbl : (type == 1 ? 1u : (type == 2 ? 2u : 4u));
      const u32 clen = type == 1 ? 4 + ((c >> 2) & 7) : l0;
      const u32 coff = type == 1 ? (((c >> 5) << 8) | ((t0 >> 8) & 0xffu))
                                 : (type == 2 ? ((t0 >> 8) & 0xffffu) : ext);
      const u32 len = is_lit ? litlen : clen;
      const u32 avail = n_in - ip - 1;                        // bytes after the tag byte
      const u32 space = expected - op;
      const bool bad = avail < nb ||                          // tag runs past the input
                       (is_lit ? (avail - nb < len || space < len)    // premature end / overrun
                               : (coff - 1u >= op || space < len));   // offset 0 or > produced
      const bool small = !is_lit && coff < 16;                // pattern copy
      const bool hdr = need && !eof && inwin;
      const bool corrupt = hdr && bad;
      const bool defer_small = hdr && !bad && small && op != batch_start;
      const bool take = hdr && !bad && !defer_small;
      status = eof ? (op == expected ? kOk : kCorrupt) : (corrupt ? kCorrupt : status);
      closed = closed || eof || corrupt || (need && !eof && !inwin) || defer_small || (take && small);
      slow_off = (take && small) ? coff : slow_off;
      slow = slow || (take && small);
      src = take ? (is_lit ? ip + 1 + nb : op - coff) : src;
      rem = take ? len : rem;
      lit = take ? is_lit : lit;
      ip = take ? ip + 1 + nb + (is_lit ? len : 0u) : ip;
      // ---- one <=16-byte piece of the current tag
      const u32 n = rem < 16 ? rem : 16u;
      const bool have = !closed && rem > 0;
      const bool hazard = have && !lit && src + n > batch_start;  // source pending in this batch
      closed = closed || hazard;
      const bool emit = have && !hazard;
      // load address: region base + clamped offset, never outside the region
      // (or the aligned 16-byte chunk holding its first byte)
      const u8* base = lit ? ib : ob;
      const u32 rlen = lit ? n_in : expected;
      const int lo_off = -(int)(reinterpret_cast<uintptr_t>(base) & 15);
      const int tail = (int)rlen - 16;
      const int a_off = (src + 16 <= rlen) ? (int)src : (tail > lo_off ? tail : lo_off);
      if (emit) __builtin_memcpy(&data[j], base + a_off, 16);  // the only load of this piece
      shf[j] = emit ? (u32)((int)src - a_off) : 0u;
      dst[j] = op;
      cnt[j] = emit ? n : 0u;
      src += emit ? n : 0u;
      op += emit ? n : 0u;
      rem -= emit ? n : 0u;
    }
    // next batch's window: issued with this batch's piece loads, so the one
    // wait below covers both (one round trip per batch)
    if (status < 0) LOAD_WINDOW();
    // ---------------- store phase ----------------
    // One wait for every piece load, here: pass the data through opaque moves
    // before the first store.  (If a piece's registers were first touched
    // after an earlier store was issued, the compiler -- unable to count the
    // divergently issued loads -- would wait vmcnt(0) and drain that store.)
    // Each piece is then stored from its own registers.
    u32x4 pd[kPieces];
#pragma unroll
    for (int j = 0; j < kPieces; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("v_mov_b32 %0, %1" : "=v"(pd[j][q]) : "v"(data[j][q]));
    }
    TAKE_WINDOW();
    // Rare fix-ups as wave-uniform branches: a piece at a region end was
    // loaded from a clamped address (shift != 0).
    {
      bool any_shift = false;
#pragma unroll
      for (int j = 0; j < kPieces; ++j) any_shift = any_shift || shf[j] != 0;
      if (__any(any_shift)) {
#pragma unroll
        for (int j = 0; j < kPieces; ++j)
          if (shf[j]) pd[j] = shr_bytes(pd[j], shf[j]);
      }
    }
    // 16-byte stores (they may scribble past the piece inside the slot; the
    // next piece's store, later in program order, rewrites those bytes)...
#pragma unroll
    for (int j = 0; j < kPieces; ++j) {
      if (cnt[j] && dst[j] + 16 <= expected) __builtin_memcpy(ob + dst[j], &pd[j], 16);
    }
    // ...then the exact-length pieces, which can only be the batch's last ones
    // (their slot has < 16 bytes left).
    {
      bool any_tail = false;
#pragma unroll
      for (int j = 0; j < kPieces; ++j) any_tail = any_tail || (cnt[j] && dst[j] + 16 > expected);
      if (__any(any_tail)) {
#pragma unroll
        for (int j = 0; j < kPieces; ++j)
          if (cnt[j] && dst[j] + 16 > expected) store_exact(ob + dst[j], pd[j], cnt[j]);
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
    // publish finished messages and (persistent mode) pull the next ones
    if (!exhausted && status >= 0) {
      for (;;) {
        status_out[m] = status;
        if (!work_counter) { exhausted = true; break; }
        ACQUIRE_MESSAGE();
        if (exhausted || status < 0) break;
      }
      rem = 0;
      if (status < 0) {
        LOAD_WINDOW();
        TAKE_WINDOW();  // once per message
      }
    }
  }
#undef TAKE_WINDOW
#undef ACQUIRE_MESSAGE
}

// lanes == 0 or no counter: one lane per message.
hipError_t launch_decode_v2(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, u32* counter, u32 lanes, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  if (counter && lanes && lanes < n_msgs) {
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(u32), stream);
    if (e != hipSuccess) return e;
    decode_batch_kernel<<<(lanes + 63) / 64, 64, 0, stream>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_cap, out_len, status, flags, counter);
  } else {
    decode_batch_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_cap, out_len, status, flags, nullptr);
  }
  return hipGetLastError();
}

}  // namespace fsg
