// lz4.hip -- batched LZ4 block codec for gfx950 (SURVEY.md section 8(f) row
// 4: COMPRESS_TYPE_LZ4 = 4, flare/rpc/options.proto:74, for which the
// reference registers no handler).  A second codec on the same batch layout
// as the Snappy path: packed inputs, per-message offsets/lengths, 16-byte
// aligned output slots, a status word per message.
//
// RPC body: varint32 of the uncompressed length (Snappy's header form), then
// one LZ4 block.  The encoder is the default LZ4 block compressor (LZ4 1.9.x
// LZ4_compress_default: acceleration 1, a fresh zeroed state; below 65,547
// input bytes 8,192 16-bit positions hashed from 4 bytes, above 4,096 32-bit
// positions hashed from 5 bytes, offsets <= 65,535), so a block is byte-equal
// to liblz4's; oracle/lz4_oracle.c restates it on the CPU and
// tests/test_lz4.py pins that against the system liblz4 1.9.3.
//
// One lane per message for both directions: LZ4 has no per-tag length table
// to index ahead (a sequence's length is in its token and extension bytes),
// so the decode walk is serial per message like Snappy's; the encoder is a
// serial greedy chain.  Position tables live in the workspace (16 KiB per
// message), zeroed by the launch.
#include "snappy_device.h"

namespace fsg {

namespace {

// The block codec is __host__ __device__ so tools/lz4_host_check.hip can run
// it on the CPU (under AddressSanitizer) against the oracle.
#define LZ4_HD __host__ __device__ __forceinline__

LZ4_HD u32 ld32(const u8* p) {
  u32 v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
LZ4_HD u64 ld64(const u8* p) {
  u64 v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
LZ4_HD void cp16(u8* d, const u8* s) {
  u32x4 v;
  __builtin_memcpy(&v, s, 16);
  __builtin_memcpy(d, &v, 16);
}

constexpr u32 kLz4MinMatch = 4;
constexpr u32 kLz4MfLimit = 12;
constexpr u32 kLz4LastLiterals = 5;
constexpr u32 kLz4HashLog = 12;
constexpr u32 kLz4SkipTrigger = 6;
constexpr u32 kLz4DistanceMax = 65535;
constexpr u32 kLz4Limit64K = 65536 + kLz4MfLimit - 1;
constexpr u32 kLz4MaxInput = 0x7E000000u;  // LZ4_MAX_INPUT_SIZE
constexpr u32 kLz4TableBytes = 16384;       // either table: 8,192 x u16 or 4,096 x u32
#ifndef FSG_LZ4_BATCH
#define FSG_LZ4_BATCH 6
#endif
constexpr u32 kLz4Batch = FSG_LZ4_BATCH;    // match-search probes loaded together

LZ4_HD u32 lz4_hash(const u8* p, bool small) {
  if (small) return (ld32(p) * 2654435761u) >> (32 - (kLz4HashLog + 1));
  return (u32)(((ld64(p) << 24) * 889523592379ull) >> (64 - kLz4HashLog));
}

// n bytes from s to d, 16 at a time then singly (never past d + n)
LZ4_HD void copy_exact(u8* d, const u8* s, u32 n) {
  u32 k = 0;
  for (; k + 16 <= n; k += 16) cp16(d + k, s + k);
  for (; k < n; ++k) d[k] = s[k];
}

LZ4_HD u8* put_length(u8* op, u32 len) {
  for (; len >= 255; len -= 255) *op++ = 255;
  *op++ = (u8)len;
  return op;
}

// count of equal bytes at a[i], b[i] with a + i < limit (LZ4_count)
LZ4_HD u32 match_count(const u8* a, const u8* b, const u8* limit) {
  u32 c = 0;
  while (a + c + 8 <= limit) {
    const u64 x = ld64(a + c) ^ ld64(b + c);
    if (x) return c + ((u32)__builtin_ctzll(x) >> 3);
    c += 8;
  }
  while (a + c < limit && a[c] == b[c]) ++c;
  return c;
}

// One block (the oracle's lz4o_compress_block); returns bytes written.
__host__ __device__ u32 lz4_compress_block(const u8* src, u32 n, u8* dst, u8* table) {
  const bool small = n < kLz4Limit64K;
  u16* t16 = reinterpret_cast<u16*>(table);
  u32* t32 = reinterpret_cast<u32*>(table);
  auto get = [&](u32 h) -> u32 { return small ? (u32)t16[h] : t32[h]; };
  auto put = [&](u32 h, u32 v) {
    if (small) t16[h] = (u16)v;
    else t32[h] = v;
  };
  u8* op = dst;
  u32 anchor = 0;
  if (n >= kLz4MfLimit + 1) {
    const u32 mflimit1 = n - kLz4MfLimit + 1;  // a match starts before this
    const u8* matchlimit = src + n - kLz4LastLiterals;
    put(lz4_hash(src, small), 0);
    u32 ip = 1;
    u32 fh = lz4_hash(src + ip, small);
    for (;;) {
      u32 match;
      // find a match: probe with a step that grows after every 64 misses.
      // kLz4Batch probes at a time: their positions, hashes, table entries and
      // candidate words are loaded together (one round trip each instead of
      // one per probe), then the probes run in order exactly as the
      // reference's loop -- a probe's table read sees the writes of the
      // earlier probes of the batch, taken from the batch itself -- and the
      // first match ends the batch (the later probes write nothing).
      {
        u32 fwd = ip, step = 1, nb = 1u << kLz4SkipTrigger;
        u32 h = fh;
        for (;;) {
          u32 cur[kLz4Batch], hs[kLz4Batch], mi[kLz4Batch], cw[kLz4Batch], iw[kLz4Batch];
          bool ok[kLz4Batch];
          u32 f = fwd, st = step, b = nb, hh = h;
#pragma unroll
          for (u32 k = 0; k < kLz4Batch; ++k) {
            const bool live = k == 0 || ok[k - 1];  // cur[k] <= mflimit1: its bytes are in the block
            cur[k] = f;
            hs[k] = hh;
            f += st;
            st = b++ >> kLz4SkipTrigger;
            ok[k] = live && f <= mflimit1;
            hh = ok[k] ? lz4_hash(src + f, small) : 0u;
            iw[k] = live ? ld32(src + cur[k]) : 0u;
          }
#pragma unroll
          for (u32 k = 0; k < kLz4Batch; ++k) mi[k] = get(hs[k]);
#pragma unroll
          for (u32 k = 1; k < kLz4Batch; ++k)
#pragma unroll
            for (u32 j = 0; j < k; ++j) mi[k] = hs[j] == hs[k] ? cur[j] : mi[k];
#pragma unroll
          for (u32 k = 0; k < kLz4Batch; ++k) cw[k] = ok[k] ? ld32(src + mi[k]) : 0u;  // (an invalid probe's
                                                                                      // position may lie past n)
          bool found = false;
#pragma unroll
          for (u32 k = 0; k < kLz4Batch; ++k) {
            ip = cur[k];
            if (!ok[k]) goto last_literals;
            match = mi[k];
            put(hs[k], cur[k]);
            if (!small && mi[k] + kLz4DistanceMax < cur[k]) continue;  // too far
            if (cw[k] == iw[k]) {
              found = true;
              break;
            }
          }
          if (found) break;
          fwd = f;
          step = st;
          nb = b;
          h = hh;
        }
      }
      while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {  // extend backwards
        --ip;
        --match;
      }
      u8* token = op++;
      {
        const u32 lit = ip - anchor;
        if (lit >= 15) {
          *token = 15 << 4;
          op = put_length(op, lit - 15);
        } else {
          *token = (u8)(lit << 4);
        }
        copy_exact(op, src + anchor, lit);
        op += lit;
      }
      for (;;) {  // a match at ip from `match`, then possibly another at once
        const u32 off = ip - match;
        op[0] = (u8)off;
        op[1] = (u8)(off >> 8);
        op += 2;
        const u32 ml = match_count(src + ip + kLz4MinMatch, src + match + kLz4MinMatch, matchlimit);
        ip += ml + kLz4MinMatch;
        if (ml >= 15) {
          *token += 15;
          op = put_length(op, ml - 15);
        } else {
          *token += (u8)ml;
        }
        anchor = ip;
        if (ip >= mflimit1) goto last_literals;
        put(lz4_hash(src + ip - 2, small), ip - 2);
        const u32 h = lz4_hash(src + ip, small), mi = get(h);
        put(h, ip);
        if ((small || mi + kLz4DistanceMax >= ip) && ld32(src + mi) == ld32(src + ip)) {
          match = mi;
          token = op++;
          *token = 0;
          continue;
        }
        break;
      }
      fh = lz4_hash(src + ++ip, small);
    }
  }
last_literals : {
  const u32 last = n - anchor;
  if (last >= 15) {
    *op++ = 15 << 4;
    op = put_length(op, last - 15);
  } else {
    *op++ = (u8)(last << 4);
  }
  copy_exact(op, src + anchor, last);
  op += last;
}
  return (u32)(op - dst);
}

// One block to exactly ulen bytes (the oracle's lz4o_decompress_block):
// true when valid.
__host__ __device__ bool lz4_decompress_block(const u8* src, u32 n, u8* dst, u32 ulen) {
  u32 ip = 0, op = 0;
  for (;;) {
    if (ip >= n) return false;
    const u32 token = src[ip++];
    u32 lit = token >> 4;
    if (lit == 15) {
      u32 b;
      do {
        if (ip >= n) return false;
        b = src[ip++];
        lit += b;
      } while (b == 255 && lit <= n);
    }
    if (lit > n - ip || lit > ulen - op) return false;
    if ((u64)op + lit + kLz4MfLimit > ulen || (u64)ip + lit + 2 + 1 + kLz4LastLiterals > n) {
      if (ip + lit != n) return false;  // must be the last sequence
      copy_exact(dst + op, src + ip, lit);
      return op + lit == ulen;
    }
    copy_exact(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    const u32 off = (u32)src[ip] | ((u32)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return false;
    u32 ml = (token & 15) + kLz4MinMatch;
    if ((token & 15) == 15) {
      u32 b;
      do {
        if (ip >= n) return false;
        b = src[ip++];
        ml += b;
      } while (b == 255 && ml <= ulen);
    }
    if ((u64)ml + kLz4LastLiterals > ulen - op) return false;
    u8* d = dst + op;
    if (off >= 16) {
      copy_exact(d, d - off, ml);  // each 16-byte step reads bytes already written
    } else {
      const u8* from = d - off;  // overlapping: byte by byte, in order
      for (u32 k = 0; k < ml; ++k) d[k] = from[k];
    }
    op += ml;
  }
}

__global__ __launch_bounds__(64) void lz4_encode_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                                      const u32* __restrict__ in_len, u32 n_msgs, u8* out,
                                                      const u64* __restrict__ out_off, u32* __restrict__ out_len,
                                                      i32* __restrict__ status, u8* tables) {
  const u32 m = blockIdx.x * 64 + threadIdx.x;
  if (m >= n_msgs) return;
  const u32 n = in_len[m];
  u8* ob = out + out_off[m];
  if (n > kLz4MaxInput) {
    out_len[m] = 0;
    status[m] = kCorrupt;
    return;
  }
  u32 h = 0, v = n;
  while (v >= 0x80) {
    ob[h++] = (u8)(v | 0x80);
    v >>= 7;
  }
  ob[h++] = (u8)v;
  out_len[m] = h + lz4_compress_block(in + in_off[m], n, ob + h, tables + (u64)m * kLz4TableBytes);
  status[m] = kOk;
}

__global__ __launch_bounds__(64) void lz4_decode_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                                      const u32* __restrict__ in_len, u32 n_msgs, u8* out,
                                                      const u64* __restrict__ out_off,
                                                      const u32* __restrict__ out_cap, u32* __restrict__ out_len,
                                                      i32* __restrict__ status, bool fallback_only) {
  const u32 m = blockIdx.x * 64 + threadIdx.x;
  if (m >= n_msgs) return;
  // (fallback_only: the messages lz4_decode2.hip's index pass could not
  // index, status kNeedFallback)
  if (fallback_only && status[m] != kNeedFallback) return;
  const u8* ib = in + in_off[m];
  const u32 n = in_len[m];
  // header: the strict varint32 form of the oracle (lz4o_header)
  u32 ulen = 0, h = 0;
  bool hok = false;
  for (u32 i = 0; i < 5 && i < n; ++i) {
    const u32 c = ib[i];
    ulen |= (c & 0x7fu) << (7 * i);
    if (c < 128) {
      hok = !(i == 4 && c >= 16);
      h = i + 1;
      break;
    }
  }
  if (!hok) {
    out_len[m] = 0;
    status[m] = kBadHeader;
    return;
  }
  out_len[m] = ulen;
  if (ulen > out_cap[m]) {
    status[m] = kSlotTooSmall;
    return;
  }
  status[m] = lz4_decompress_block(ib + h, n - h, out + out_off[m], ulen) ? kOk : kCorrupt;
}

}  // namespace

size_t lz4_compress_workspace_bytes(u32 n_msgs) { return (size_t)n_msgs * kLz4TableBytes; }

hipError_t launch_lz4_encode(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                             const u64* out_off, u32* out_len, i32* status, void* ws, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(ws, 0, lz4_compress_workspace_bytes(n_msgs), stream);
  if (e != hipSuccess) return e;
  lz4_encode_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off, out_len,
                                                           status, static_cast<u8*>(ws));
  return hipGetLastError();
}

hipError_t launch_lz4_decode(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                             const u64* out_off, const u32* out_cap, u32* out_len, i32* status,
                             hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  lz4_decode_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off, out_cap,
                                                           out_len, status, false);
  return hipGetLastError();
}

hipError_t launch_lz4_decode_fallback(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                                      const u64* out_off, const u32* out_cap, u32* out_len, i32* status,
                                      hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  lz4_decode_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off, out_cap,
                                                           out_len, status, true);
  return hipGetLastError();
}

}  // namespace fsg
