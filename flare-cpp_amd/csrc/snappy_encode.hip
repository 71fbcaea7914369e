// snappy_encode.hip -- batched Snappy encode for gfx950.
//
// encode_wave_kernel: one WAVE (64-thread workgroup) per message.  The
// message is compressed fragment by fragment (64 KiB, snappy.cc:887-948)
// into its own output slot, byte-identical to the reference's
// internal::CompressFragment (snappy.cc:329-453):
//   * the hash table (htsize x u16, htsize chosen per fragment exactly as
//     WorkingMemory::GetHashTable, snappy.cc:247-271) lives in LDS and is
//     zeroed per fragment (zero entries act as "position 0", :391);
//   * the greedy probe loop with the skip heuristic is evaluated W probes at
//     a time: lane k owns probe k, computes its position from a wave prefix
//     sum of the skip steps, hashes it, reads the table, and resolves
//     intra-window hash collisions (a later probe must see the position an
//     earlier probe of the same window stored, :391-395) by lane shuffles;
//     the first matching lane (ballot) ends the stretch and exactly the
//     probes before it commit their table writes (last writer per hash wins);
//   * FindMatchLength (snappy-internal.h:87-121) compares 64 bytes per step,
//     one per lane, the first mismatch found by ballot;
//   * literals are copied by all lanes 16 bytes at a time.
#include "snappy_device.h"

namespace fsg {

constexpr int kProbeWindow = 16;  // probes evaluated per wave step: one DPP row

// Lane l of a 16-lane row gets v from lane l - D (ROW_SHR) or l + D (ROW_SHL)
// of the same row, `old` where that lane is outside the row: one VALU
// instruction, where a shuffle is an LDS round trip.
#define FSG_ROW_SHR(old, v, D) ((u32)__builtin_amdgcn_update_dpp((int)(old), (int)(v), 0x110 + (D), 0xf, 0xf, false))
#define FSG_ROW_SHL(old, v, D) ((u32)__builtin_amdgcn_update_dpp((int)(old), (int)(v), 0x100 + (D), 0xf, 0xf, false))
#define FSG_REP15(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

__device__ __forceinline__ u32 wave_bcast(u32 v, int src_lane) {
  return (u32)__builtin_amdgcn_readlane((int)v, src_lane);
}

// EmitLiteral (snappy.cc:156-196), whole wave.  Returns new op.
__device__ u64 emit_literal_wave(u8* dst, u64 op, const u8* lit, u32 len) {
  const int lane = lane_id();
  u32 n = len - 1;
  u32 hl;
  if (n < 60) {
    if (lane == 0) dst[op] = (u8)(n << 2);
    hl = 1;
  } else {
    u32 count = n < (1u << 8) ? 1 : n < (1u << 16) ? 2 : n < (1u << 24) ? 3 : 4;
    if (lane == 0) dst[op] = (u8)((59 + count) << 2);
    if (lane >= 1 && (u32)lane <= count) dst[op + lane] = (u8)(n >> (8 * (lane - 1)));
    hl = 1 + count;
  }
  u8* d = dst + op + hl;
  u32 k = (u32)lane * 16;
  for (; k + 16 <= len; k += kWave * 16) copy16(d + k, lit + k);
  // tail: fewer than 16 * 64 bytes may remain unaligned to the 16-byte grid
  u32 done = (len / 16) * 16;
  for (u32 t = done + lane; t < len; t += kWave) d[t] = lit[t];
  return op + hl + len;
}

// EmitCopyLessThan64 (snappy.cc:198-214) by one lane.
__device__ __forceinline__ u64 emit_copy_lt64(u8* dst, u64 op, u32 offset, u32 len) {
  if (len < 12 && offset < 2048) {
    dst[op] = (u8)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    dst[op + 1] = (u8)(offset & 0xff);
    return op + 2;
  }
  dst[op] = (u8)(2 + ((len - 1) << 2));
  dst[op + 1] = (u8)(offset & 0xff);
  dst[op + 2] = (u8)(offset >> 8);
  return op + 3;
}

// EmitCopy (snappy.cc:216-232): length of the emitted bytes, written by lane 0.
__device__ u64 emit_copy_wave(u8* dst, u64 op, u32 offset, u32 len) {
  u64 o = op;
  u32 l = len;
  // Compute the byte count uniformly; lane 0 writes.
  u64 nbytes = 0;
  {
    u32 ll = l;
    while (ll >= 68) { nbytes += (offset < 2048 && 64 < 12) ? 2 : 3; ll -= 64; }
    if (ll > 64) { nbytes += 3; ll -= 60; }
    nbytes += (ll < 12 && offset < 2048) ? 2 : 3;
  }
  if (lane_id() == 0) {
    while (l >= 68) { o = emit_copy_lt64(dst, o, offset, 64); l -= 64; }
    if (l > 64) { o = emit_copy_lt64(dst, o, offset, 60); l -= 60; }
    emit_copy_lt64(dst, o, offset, l);
  }
  return op + nbytes;
}

// FindMatchLength(s1, s2, s2_limit) with the whole wave.
__device__ u32 match_length_wave(const u8* s1, const u8* s2, const u8* s2_limit) {
  const int lane = lane_id();
  u32 m = 0;
  const u32 lim = (u32)(s2_limit - s2);
  for (;;) {
    u32 idx = m + (u32)lane;
    bool eq = idx < lim && s1[idx] == s2[idx];
    u64 neq = __ballot(!eq);
    if (neq) return m + (u32)(__ffsll((unsigned long long)neq) - 1);
    m += kWave;
  }
}

// internal::CompressFragment (snappy.cc:329-453), one wave.
__device__ u64 compress_fragment_wave(const u8* input, u32 n, u8* dst, u64 op,
                                      u16* table, int shift) {
  const int lane = lane_id();
  u32 next_emit = 0;
  if (n >= kInputMarginBytes) {
    const u32 ip_limit = n - kInputMarginBytes;
    u32 ip = 1;
    for (;;) {
      // ---- Step 1: probe stretch (snappy.cc:377-397), W probes per step.
      u32 skip = 32;
      u32 cand_pos = 0;
      bool found = false;
      for (;;) {
        // lane k: p_k = ip + sum_{j<k} ((skip + j) >> 5)
        u32 step = (skip + (u32)lane) >> 5;
        u32 incl = step;
        incl += FSG_ROW_SHR(0u, incl, 1);
        incl += FSG_ROW_SHR(0u, incl, 2);
        incl += FSG_ROW_SHR(0u, incl, 4);
        incl += FSG_ROW_SHR(0u, incl, 8);
        u32 p = ip + incl - step;
        u32 p_next = p + step;
        // probe k runs iff the following position is still <= ip_limit (:387)
        bool exec = lane < kProbeWindow && p_next <= ip_limit;
        u32 bytes = exec ? ldu32(input + p) : 0u;
        u32 h = hash_bytes(bytes, shift);
        u32 old = exec ? (u32)table[h] : 0u;
        // latest earlier probe in this window with the same hash (a probe
        // that does not run carries a key no hash equals)
        const u32 hx = exec ? h : (0x40000000u | (u32)lane);
        int prev = -1;
#define FSG_COLL(D) { const u32 hd = FSG_ROW_SHR(0x7fffffffu, hx, D); if (prev < 0 && hd == hx) prev = lane - (D); }
        FSG_REP15(FSG_COLL)
#undef FSG_COLL
        u32 pp = __shfl(p, prev < 0 ? lane : prev, kWave);
        u32 cand = prev >= 0 ? pp : old;
        bool match = exec && ldu32(input + cand) == bytes;
        u64 mm = __ballot(match);
        u64 em = __ballot(exec);
        int last;  // last probe that commits its table write
        if (mm) last = __ffsll((unsigned long long)mm) - 1;
        else last = em ? 63 - __clzll((long long)em) : -1;
        // commit table[h_k] = p_k for k <= last, last writer per hash wins
        bool later = false;
#define FSG_LATER(D) { const u32 hd = FSG_ROW_SHL(0x7fffffffu, hx, D); if (lane + (D) <= last && hd == hx) later = true; }
        FSG_REP15(FSG_LATER)
#undef FSG_LATER
        if (exec && lane <= last && !later) table[h] = (u16)p;
        if (mm) {
          ip = wave_bcast(p, last);
          cand_pos = wave_bcast(cand, last);
          found = true;
          break;
        }
        if (em != ((1ull << kProbeWindow) - 1)) break;  // hit ip_limit
        ip = wave_bcast(p_next, kProbeWindow - 1);
        skip += kProbeWindow;
      }
      if (!found) goto emit_remainder;

      // ---- Step 2: pending literal (:403).
      op = emit_literal_wave(dst, op, input + next_emit, ip - next_emit);

      // ---- Step 3: copies while the next 4 bytes match again (:416-439).
      for (;;) {
        u32 base = ip;
        u32 matched = 4 + match_length_wave(input + cand_pos + 4, input + ip + 4,
                                            input + n);
        ip += matched;
        op = emit_copy_wave(dst, op, base - cand_pos, matched);
        next_emit = ip;
        if (ip >= ip_limit) goto emit_remainder;
        u32 prev_bytes = ldu32(input + ip - 1);
        u32 cur_bytes = ldu32(input + ip);
        u32 ph = hash_bytes(prev_bytes, shift);
        u32 ch = hash_bytes(cur_bytes, shift);
        // LDS ops of one wave execute in order: the read below sees this write
        // (hash(ip-1) == hash(ip) must yield candidate ip-1, :434-436).
        if (lane == 0) table[ph] = (u16)(ip - 1);
        u32 c = (u32)table[ch];
        cand_pos = c;
        u32 cb = ldu32(input + c);
        if (lane == 0) table[ch] = (u16)ip;
        if (cb != cur_bytes) break;
      }
      ++ip;  // next stretch starts at ip + 1 (:441-442)
    }
  }
emit_remainder:
  if (next_emit < n) op = emit_literal_wave(dst, op, input + next_emit, n - next_emit);
  return op;
}

__global__ __launch_bounds__(64) void encode_wave_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, u32* __restrict__ out_len,
    i32* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) u16 table[];
  const u32 m = blockIdx.x;
  if (m >= n_msgs) return;
  const int lane = lane_id();
  const u8* src = in + in_off[m];
  const u32 n = in_len[m];
  u8* dst = out + out_off[m];
  // varint32 header (snappy.cc:877-881)
  const int hl = varint32_len(n);
  if (lane < hl) {
    u32 b = (n >> (7 * lane)) & 0x7f;
    if (lane + 1 < hl) b |= 0x80;
    dst[lane] = (u8)b;
  }
  u64 op = (u64)hl;
  for (u32 pos = 0; pos < n; pos += kBlockSize) {
    const u32 frag = min(n - pos, kBlockSize);
    const u32 ht = table_size_for(frag);
    const int shift = 32 - (31 - __clz((int)ht));
    u32* t32 = reinterpret_cast<u32*>(table);
    __syncthreads();
    for (u32 i = (u32)lane; i < ht / 2; i += kWave) t32[i] = 0u;
    __syncthreads();
    op = compress_fragment_wave(src + pos, frag, dst, op, table, shift);
  }
  if (lane == 0) {
    out_len[m] = (u32)op;
    status[m] = kOk;
  }
}

hipError_t launch_encode(const u8* in, const u64* in_off, const u32* in_len,
                         u32 n_msgs, u32 max_in_len, u8* out, const u64* out_off,
                         u32* out_len, i32* status, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  u32 cap = max_in_len == 0 || max_in_len > kBlockSize ? kBlockSize : max_in_len;
  size_t lds = (size_t)table_size_for(cap) * sizeof(u16);
  encode_wave_kernel<<<n_msgs, 64, lds, stream>>>(in, in_off, in_len, n_msgs,
                                                  out, out_off, out_len, status);
  return hipGetLastError();
}

}  // namespace fsg
