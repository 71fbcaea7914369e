// wave_util.h -- wave-level helpers shared by the gfx950 two-pass decoders
// (Snappy: snappy_decode_v4.hip; LZ4: lz4_decode2.hip): DPP scans, buffer
// loads of a message's bytes, LDS ordering, the OR store into a zeroed
// output window.
#pragma once

#include "snappy_pieces.h"

namespace fsg {
namespace {

__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
  const u32 lane = __lane_id();
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    const u32 t = __shfl_up(v, d, 64);
    v += lane >= d ? t : 0u;
  }
  return v;
}

__device__ __forceinline__ u32 readlane(u32 v, u32 l) {
  return (u32)__builtin_amdgcn_readlane((int)v, (int)l);
}

// Orders one wave's LDS accesses across lanes.  A wave's LDS instructions
// execute in issue order, so a read issued after another lane's write sees
// it: only the compiler must keep program order (the accesses share one
// array, so they may alias and are not reordered), and no s_waitcnt is
// needed -- the wave barrier just pins the schedule.
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_wave_barrier(); }

// 16 bytes of a message buffer at `off`, never touching bytes outside
// [-(bal), limit) (see clamped_origin).
[[maybe_unused]] __device__ __forceinline__ u32x4 load16_clamped(const u8* base, u32 off, u32 limit, u32 bal) {
  const int a = clamped_origin(off, limit, bal);
  u32x4 v;
  __builtin_memcpy(&v, base + a, 16);
  const u32 sh = (u32)((int)off - a);
  return sh ? shr_bytes(v, sh) : v;
}

// A message's compressed bytes as a buffer: base = the 16-byte-aligned block
// holding its first byte, num_records = its last byte's dword end.  A raw
// buffer load returns 0 for every dword that reaches past num_records and
// touches no memory there (per dword, measured on gfx950:
// tools/probes/buffer_oob_probe.hip), so loads at dword-aligned offsets need
// no clamping: every dword holding a message byte lies inside the aligned
// block structure the message occupies.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t msg_rsrc(const u8* abase, u32 bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(abase), (short)0,
                                           (int)((bytes + 3) & ~3u), 0x00020000);
}

// 16 bytes at buffer offset P (any alignment): one 16-byte and one 4-byte
// load at the dword below P, then a byte shift (bytes past the end read 0).
__device__ __forceinline__ u32x4 rsrc_load16(__amdgpu_buffer_rsrc_t r, u32 P) {
  const u32 a = P & ~3u, s = P & 3u;
  const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
  const u32 d4 = __builtin_amdgcn_raw_buffer_load_b32(r, a + 16, 0, 0);
  return u32x4{__builtin_amdgcn_alignbyte(d[1], d[0], s), __builtin_amdgcn_alignbyte(d[2], d[1], s),
               __builtin_amdgcn_alignbyte(d[3], d[2], s), __builtin_amdgcn_alignbyte(d4, d[3], s)};
}

// The same in two steps, so that several loads are in flight before the
// first shift waits for its data: raw_load16 issues the loads, shifted16
// applies the byte shift.
struct Raw16 {
  u32x4 d;
  u32 d4, s;
};
__device__ __forceinline__ Raw16 raw_load16(__amdgpu_buffer_rsrc_t r, u32 P) {
  const u32 a = P & ~3u;
  return Raw16{__builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0),
               __builtin_amdgcn_raw_buffer_load_b32(r, a + 16, 0, 0), P & 3u};
}
__device__ __forceinline__ u32x4 shifted16(const Raw16& x) {
  return u32x4{__builtin_amdgcn_alignbyte(x.d[1], x.d[0], x.s), __builtin_amdgcn_alignbyte(x.d[2], x.d[1], x.s),
               __builtin_amdgcn_alignbyte(x.d[3], x.d[2], x.s), __builtin_amdgcn_alignbyte(x.d4, x.d[3], x.s)};
}

// The 5 tag bytes at buffer offset P: bytes P..P+3 in .x, byte P+4 in the low
// byte of .y (one 8-byte load at the dword below P).
__device__ __forceinline__ u32x2 rsrc_tag5(__amdgpu_buffer_rsrc_t r, u32 P) {
  const u32 a = P & ~3u, s = P & 3u;
  const u32x2 d = __builtin_amdgcn_raw_buffer_load_b64(r, a, 0, 0);
  return u32x2{__builtin_amdgcn_alignbyte(d[1], d[0], s), d[1] >> (8 * s)};
}

// Waits for every outstanding memory operation of the wave.  The asm
// statement clobbers memory, so the compiler keeps later loads after it
// (the bare s_waitcnt builtin is not a memory barrier to the optimizer).
__device__ __forceinline__ void wait_all_memory() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }

// Inclusive prefix sum over the 64 lanes with DPP row shifts and row
// broadcasts (gfx9 wave64): 7 VALU steps, no LDS round trip.
__device__ __forceinline__ u32 dpp_incl_scan(u32 v) {
  u32 r = v;
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xf, 0xf, true);   // row_shr:3
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)r, 0x114, 0xf, 0xe, false);  // row_shr:4, banks 1-3
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)r, 0x118, 0xf, 0xc, false);  // row_shr:8, banks 2-3
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)r, 0x142, 0xa, 0xf, false);  // row_bcast:15
  r += (u32)__builtin_amdgcn_update_dpp(0, (int)r, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return r;
}

__device__ __forceinline__ u32x4 lds_read16(const u8* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}

// OR n (1..16) bytes of v into the window at byte offset w, whose bytes
// there are zero: five aligned ds_or_b32 whatever w and n, so the LDS time
// is fixed per instruction instead of per misaligned lane, and no size
// branches.  Bytes past n are masked to zero (mtab[n]: the byte mask of n
// bytes, a 17-entry LDS table), so nothing lands past w + n; the shift by
// w & 3 bytes is one v_perm per output dword (selector byte j = 4 + j - b
// picks byte j - b of the pair (v[k], v[k-1])).  10 VALU, where computing
// the masks and shifts inline took ~40.
__device__ __forceinline__ void or_store(u8* sb, u32 w, u32x4 v, u32 n, const u32x4* mtab) {
  const u32x4 mk = mtab[n];
  v[0] &= mk[0];
  v[1] &= mk[1];
  v[2] &= mk[2];
  v[3] &= mk[3];
  // bytes 4-b .. 7-b: the 8-byte sequence 01..08 from byte 3-b = (~w) & 3
  const u32 sel = __builtin_amdgcn_alignbyte(0x08070605u, 0x04030201u, ~w);
  const u32 o0 = __builtin_amdgcn_perm(v[0], 0u, sel);
  const u32 o1 = __builtin_amdgcn_perm(v[1], v[0], sel);
  const u32 o2 = __builtin_amdgcn_perm(v[2], v[1], sel);
  const u32 o3 = __builtin_amdgcn_perm(v[3], v[2], sel);
  const u32 o4 = __builtin_amdgcn_perm(0u, v[3], sel);
  u32* d = reinterpret_cast<u32*>(sb) + (w >> 2);
  __hip_atomic_fetch_or(d + 0, o0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or(d + 1, o1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or(d + 2, o2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or(d + 3, o3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_or(d + 4, o4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// mtab[n] (n = 0..16): 0xff in the first n bytes.  68 threads fill it.
__device__ __forceinline__ void init_mask_table(u32x4* mtab, u32 t) {
  if (t < 68) {
    const u32 n = t >> 2, q = t & 3;
    const u32 have = n > 4 * q ? n - 4 * q : 0u;
    reinterpret_cast<u32*>(mtab)[t] = have >= 4 ? 0xffffffffu : (have ? 0xffffffffu >> (32 - 8 * have) : 0u);
  }
}

}  // namespace
}  // namespace fsg
