// snappy_encode_v2.hip -- lane-per-message batched Snappy encode for gfx950.
//
// The reference's greedy parse (internal::CompressFragment,
// /root/reference/flare/io/snappy/snappy.cc:329-453) is a strictly sequential
// chain per 64 KiB fragment: every probe reads and rewrites the hash table
// the next probe depends on.  A 64 KiB fragment needs a 32 KiB table, so LDS
// (160 KiB/CU) could hold only 5 fragments per CU; instead every LANE owns one
// message at a time and keeps its table (htsize x u16, zeroed per fragment
// exactly as WorkingMemory::GetHashTable, snappy.cc:247-271) in a private
// slice of a global workspace.  That gives 64 concurrent chains per wave and
// tens of thousands per GPU, which is what hides the per-probe memory
// latency.  Lanes pull message indices from a device-wide counter, so a few
// large messages do not serialise a wave.
//
// Output bytes are identical to snappy::Compress(Source*, Sink*)
// (snappy.cc:875-954): varint32 length, then one CompressFragment per
// 64 KiB fragment, concatenated into the message's slot.  Emit helpers
// follow EmitLiteral/EmitCopy (snappy.cc:156-232) including the reference's
// 16-byte literal fast path, which only scribbles inside the slot's
// MaxCompressedLength headroom.
#include "snappy_device.h"

namespace fsg {

__device__ __forceinline__ u8* emit_literal_lane(u8* op, const u8* lit, u32 len, bool fast) {
  const u32 n = len - 1;
  if (n < 60) {
    *op++ = (u8)(n << 2);
    if (fast && len <= 16) {  // snappy.cc:175-179
      copy16(op, lit);
      return op + len;
    }
  } else {
    u8* base = op++;
    u32 count = 0;
    u32 v = n;
    while (v > 0) {
      *op++ = (u8)(v & 0xff);
      v >>= 8;
      ++count;
    }
    *base = (u8)((59 + count) << 2);
  }
  u32 k = 0;
  for (; k + 16 <= len; k += 16) copy16(op + k, lit + k);
  for (; k < len; ++k) op[k] = lit[k];
  return op + len;
}

__device__ __forceinline__ u8* emit_copy_lt64_lane(u8* op, u32 offset, u32 len) {
  if (len < 12 && offset < 2048) {
    op[0] = (u8)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
    op[1] = (u8)(offset & 0xff);
    return op + 2;
  }
  op[0] = (u8)(2 + ((len - 1) << 2));
  op[1] = (u8)(offset & 0xff);
  op[2] = (u8)(offset >> 8);
  return op + 3;
}

__device__ __forceinline__ u8* emit_copy_lane(u8* op, u32 offset, u32 len) {
  while (len >= 68) {
    op = emit_copy_lt64_lane(op, offset, 64);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_lt64_lane(op, offset, 60);
    len -= 60;
  }
  return emit_copy_lt64_lane(op, offset, len);
}

// FindMatchLength (snappy-internal.h:87-121): 8 bytes at a time.
__device__ __forceinline__ u32 match_length_lane(const u8* s1, const u8* s2, const u8* s2_limit) {
  u32 m = 0;
  while (s2 + m + 8 <= s2_limit) {
    const u64 x = ldu64(s2 + m) ^ ldu64(s1 + m);
    if (x) return m + (u32)(__builtin_ctzll(x) >> 3);
    m += 8;
  }
  while (s2 + m < s2_limit && s1[m] == s2[m]) ++m;
  return m;
}

// internal::CompressFragment on one lane; table has `ht` zeroed entries.
__device__ u8* compress_fragment_lane(const u8* input, u32 n, u8* op, u16* table, int shift) {
  const u8* ip = input;
  const u8* ip_end = input + n;
  const u8* next_emit = ip;
  if (n >= kInputMarginBytes) {
    const u8* ip_limit = input + n - kInputMarginBytes;
    u32 next_hash = hash_bytes(ldu32(++ip), shift);
    for (;;) {
      u32 skip = 32;
      const u8* next_ip = ip;
      const u8* candidate;
      do {
        ip = next_ip;
        const u32 h = next_hash;
        const u32 step = skip++ >> 5;
        next_ip = ip + step;
        if (next_ip > ip_limit) goto emit_remainder;
        next_hash = hash_bytes(ldu32(next_ip), shift);
        candidate = input + table[h];
        table[h] = (u16)(ip - input);
      } while (ldu32(ip) != ldu32(candidate));

      op = emit_literal_lane(op, next_emit, (u32)(ip - next_emit), true);

      u32 cur_bytes, cand_bytes;
      do {
        const u8* base = ip;
        const u32 matched = 4 + match_length_lane(candidate + 4, ip + 4, ip_end);
        ip += matched;
        op = emit_copy_lane(op, (u32)(base - candidate), matched);
        next_emit = ip;
        if (ip >= ip_limit) goto emit_remainder;
        const u64 w = ldu64(ip - 1);
        const u32 ph = hash_bytes((u32)w, shift);
        table[ph] = (u16)(ip - input - 1);
        cur_bytes = (u32)(w >> 8);
        const u32 ch = hash_bytes(cur_bytes, shift);
        candidate = input + table[ch];
        cand_bytes = ldu32(candidate);
        table[ch] = (u16)(ip - input);
      } while (cur_bytes == cand_bytes);

      next_hash = hash_bytes(ldu32(ip + 1), shift);
      ++ip;
    }
  }
emit_remainder:
  if (next_emit < ip_end) op = emit_literal_lane(op, next_emit, (u32)(ip_end - next_emit), false);
  return op;
}

__global__ __launch_bounds__(256) void encode_lane_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, u32* __restrict__ out_len,
    i32* __restrict__ status, u16* __restrict__ tables, u32 table_entries,
    u32* __restrict__ work_counter) {
  const u32 slot = blockIdx.x * blockDim.x + threadIdx.x;
  u16* table = tables + (u64)slot * table_entries;
  for (;;) {
    const u32 m = atomicAdd(work_counter, 1u);
    if (m >= n_msgs) break;
    const u8* src = in + in_off[m];
    const u32 n = in_len[m];
    u8* dst = out + out_off[m];
    // varint32 header (snappy.cc:877-881)
    u8* op = dst;
    {
      u32 v = n;
      while (v >= 128) { *op++ = (u8)(v | 128); v >>= 7; }
      *op++ = (u8)v;
    }
    for (u32 pos = 0; pos < n; pos += kBlockSize) {
      const u32 frag = min(n - pos, kBlockSize);
      const u32 ht = table_size_for(frag);
      const int shift = 32 - (31 - __clz((int)ht));
      u32x4* t4 = reinterpret_cast<u32x4*>(table);
      const u32x4 z = {0, 0, 0, 0};
      for (u32 i = 0; i < ht / 8; ++i) t4[i] = z;
      op = compress_fragment_lane(src + pos, frag, op, table, shift);
    }
    out_len[m] = (u32)(op - dst);
    status[m] = kOk;
  }
}

// Workspace layout: [counter: 256 B][tables: slots x entries x u16]
size_t encode_v2_workspace_bytes(u32 n_msgs, u32 max_in_len, u32* slots_out) {
  u32 cap = max_in_len == 0 || max_in_len > kBlockSize ? kBlockSize : max_in_len;
  const u32 entries = table_size_for(cap);
  // enough lanes to fill the chip several times over: 256 CUs x 16 waves x 64
  u32 slots = n_msgs < 262144u ? n_msgs : 262144u;
  slots = (slots + 255) / 256 * 256;
  if (slots == 0) slots = 256;
  if (slots_out) *slots_out = slots;
  return 256 + (size_t)slots * entries * sizeof(u16);
}

hipError_t launch_encode_v2(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u32 max_in_len, u8* out, const u64* out_off,
                            u32* out_len, i32* status, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  u32 slots = 0;
  const size_t need = encode_v2_workspace_bytes(n_msgs, max_in_len, &slots);
  if (ws == nullptr || ws_bytes < need) return hipErrorInvalidValue;
  u32 cap = max_in_len == 0 || max_in_len > kBlockSize ? kBlockSize : max_in_len;
  const u32 entries = table_size_for(cap);
  u32* counter = reinterpret_cast<u32*>(ws);
  u16* tables = reinterpret_cast<u16*>(reinterpret_cast<u8*>(ws) + 256);
  hipError_t e = hipMemsetAsync(counter, 0, 256, stream);
  if (e != hipSuccess) return e;
  encode_lane_kernel<<<slots / 256, 256, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off,
                                                      out_len, status, tables, entries, counter);
  return hipGetLastError();
}

}  // namespace fsg
