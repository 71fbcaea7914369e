// snappy_pieces.h -- 16-byte piece helpers shared by the gfx950 decoders.
//
// A "piece" is at most 16 bytes of one tag's output: one unaligned 16-byte
// load (input bytes for a literal, earlier output for a copy) and an exact
// store of the piece's length.  Copies with offset < 16 (the overlapping
// IncrementalCopy case, /root/reference/flare/io/snappy/snappy.cc:98-152) are
// cut into pieces whose length is a multiple of the offset, so every piece
// stores the same 16-byte expansion of the `off`-byte pattern.
#pragma once

#include "snappy_device.h"

namespace fsg {

__device__ __forceinline__ u32 alignbyte(u32 hi, u32 lo, u32 s) {
  return __builtin_amdgcn_alignbyte(hi, lo, s);  // (hi:lo) >> (8*s), low 32 bits
}

__device__ __forceinline__ u32 mux8(const u32 (&w)[8], u32 d) {
  const u32 a0 = (d & 1) ? w[1] : w[0];
  const u32 a1 = (d & 1) ? w[3] : w[2];
  const u32 a2 = (d & 1) ? w[5] : w[4];
  const u32 a3 = (d & 1) ? w[7] : w[6];
  const u32 b0 = (d & 2) ? a1 : a0;
  const u32 b1 = (d & 2) ? a3 : a2;
  return (d & 4) ? b1 : b0;
}

// v >> (8 * sh) as a 16-byte little-endian value (sh in 0..15).
__device__ __forceinline__ u32x4 shr_bytes(u32x4 v, u32 sh) {
  const u32 t[8] = {v[0], v[1], v[2], v[3], 0u, 0u, 0u, 0u};
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
  const u64 hi = (u64)v[2] | ((u64)v[3] << 32);
  if (n & 8) { stu64(p, lo); p += 8; lo = hi; }
  if (n & 4) { stu32(p, (u32)lo); p += 4; lo >>= 32; }
  if (n & 2) { const u16 s = (u16)lo; __builtin_memcpy(p, &s, 2); p += 2; lo >>= 16; }
  if (n & 1) { *p = (u8)lo; }
}

// 16 bytes at base[off ..] where only base[lo_off .. limit) may be touched
// (lo_off = -(base & 15): the aligned block holding base[0] is always mapped).
// Near the end the load moves back and the bytes are shifted down.
__device__ __forceinline__ int clamped_origin(u32 off, u32 limit, u32 bal) {
  const int tail = (int)limit - 16, lo = -(int)bal;
  return (off + 16 <= limit) ? (int)off : (tail > lo ? tail : lo);
}

// v_perm selector for output byte t of a pattern of period `off`, expanded to
// 16 bytes (see expand_pattern).
__device__ __forceinline__ u32 pat_sel_byte(u32 off, u32 t) {
  if (off <= 8) return t % off;                          // (p1:p0)
  if (t < 8) return t;                                   // (p1:p0), t < off
  if (t < 12) return t < off ? 4 + (t - 8) : t - off;    // (p2:p0)
  if (t < off) return 4 + (t - 12);                      // (p3:p0)
  return t - off;  // (p1:p0) if off <= 12, else (p3:p0) low bytes
}

// Fills a 16-entry selector table (one u32x4 per period 1..15) from the 64
// lanes of a wave: lane l writes dword (l & 3) of entry l >> 2.
__device__ __forceinline__ void init_pattern_table(u32x4* sel_tab, u32 lane) {
  const u32 off = lane >> 2, q = lane & 3;
  u32 s = 0;
  if (off > 0)
    for (u32 r = 0; r < 4; ++r) s |= pat_sel_byte(off, 4 * q + r) << (8 * r);
  reinterpret_cast<u32*>(sel_tab)[lane] = s;
}

// X[t] = P[t mod off], t < 16, for a pattern P of period off (1..15) whose
// first `off` bytes are valid.
__device__ __forceinline__ u32x4 expand_pattern(u32x4 p, u32 off, const u32x4* sel_tab) {
  const u32x4 s = sel_tab[off];
  u32x4 x;
  x[0] = __builtin_amdgcn_perm(p[1], p[0], s[0]);
  x[1] = __builtin_amdgcn_perm(p[1], p[0], s[1]);
  x[2] = __builtin_amdgcn_perm(off <= 8 ? p[1] : p[2], p[0], s[2]);
  x[3] = __builtin_amdgcn_perm(off <= 12 ? p[1] : p[3], p[0], s[3]);
  return x;
}

// (16 / off) * off - 1 for off = 1..15, as nibbles: the piece length (minus
// one) of a pattern copy.
__host__ __device__ constexpr u64 pat_step_nibbles() {
  u64 k = 0;
  for (u32 off = 1; off < 16; ++off) k |= (u64)((16 / off) * off - 1) << (4 * off);
  return k;
}
constexpr u64 kPatStep = pat_step_nibbles();
__device__ __forceinline__ u32 pat_step(u32 off) { return (u32)((kPatStep >> (4 * off)) & 15u) + 1u; }

// Varint32 header: ReadUncompressedLength (snappy.cc:692-711) when !strict,
// Parse32WithLimit (snappy-stubs-internal.h:327-357) when strict.  Returns the
// header length, 0 if invalid.
__device__ __forceinline__ int parse_varint_header(const u8* ip, u32 n, bool strict, u32* ulen) {
  u32 r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((u32)i >= n) return 0;
    const u32 c = ip[i];
    r |= (c & 0x7fu) << (7 * i);  // i == 4: bits above 31 fall off
    if (c < 128) {
      if (strict && i == 4 && c >= 16) return 0;
      *ulen = r;
      return i + 1;
    }
  }
  return 0;
}

}  // namespace fsg
