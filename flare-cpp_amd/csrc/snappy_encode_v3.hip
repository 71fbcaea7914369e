// snappy_encode_v3.hip -- lane-per-message Snappy encode with batched
// speculative probes, for gfx950.
//
// Same unit of work and table placement as encode_lane_kernel (v2): every
// lane owns a message and a u16 hash table in the workspace, zeroed per
// fragment (WorkingMemory::GetHashTable, snappy.cc:247-271).  v2 restates
// internal::CompressFragment (snappy.cc:329-453) literally, paying two
// dependent global round trips per probe (table entry, then candidate bytes)
// plus one per 8 bytes of match extension.  v3 keeps the exact greedy parse
// but resolves it K probes at a time:
//
//   * The probe positions of a batch are known in advance: after a copy the
//     sequence is [ip (after inserting ip-1), ip+1, ip+2, ...], inside a
//     literal run it is the skip-heuristic sequence p += skip++ >> 5.  Only
//     the first matching probe ends the batch.
//   * Round trip 1 loads the K table entries.  A probe that hashes to the
//     same slot as an earlier probe of the batch (or the ip-1 insertion)
//     takes that earlier position as its candidate -- exactly what the
//     sequential table read-then-write would have returned.
//   * Round trip 2 loads 16 candidate bytes per probe and the input window
//     for the next batch.  The first probe whose 4 bytes match wins; its match
//     length is read from the same 16 bytes (99% of C3 matches are <= 16 B);
//     longer matches extend 16 bytes per load.
//   * Table writes of the probes up to the winner are then committed in
//     program order (later writes of a slot win, as in the reference).
//
// Input bytes for hashing, for the winner's comparison and for short
// literals come from an 80-byte per-lane window in LDS ([dword][lane]
// layout), loaded with the candidates one batch ahead.  (Round 6 measured
// the window in registers, read by a barrel shift, so that the kernel needs
// no LDS beside a five-table encode_wave_kernel workgroup: C3 even, C5
// 18.8 -> 21.1 ms)
//
// Output bytes equal snappy::Compress(Source*, Sink*) (snappy.cc:875-954);
// EmitLiteral / EmitCopy follow snappy.cc:156-232.
#include "options.h"
#include "snappy_device.h"

#include <cstdlib>
#include <mutex>

namespace fsg {

namespace {

#ifndef FSG_V3_PROBES
#define FSG_V3_PROBES 3
#endif
constexpr int kKFlat = FSG_V3_PROBES;  // probes per batch
#ifndef FSG_V3_POST_PROBES
#define FSG_V3_POST_PROBES 1
#endif
constexpr int kPostFlat = FSG_V3_POST_PROBES;  // probes per batch right after a copy
// Batches with split messages (> 64 KiB) end in a few long fragment chains
// running alone, bound by each chain's round trips: more probes per batch
// there (C5 56.1 -> 52.9 ms; on C3, where every lane stays busy, the extra
// probes' traffic costs 108 -> 118 ms).
#ifndef FSG_V3_PROBES_SPLIT
#define FSG_V3_PROBES_SPLIT 4
#endif
#ifndef FSG_V3_POST_PROBES_SPLIT
#define FSG_V3_POST_PROBES_SPLIT 2
#endif
constexpr u32 kWinChunks = 5;      // 80-byte input window
// Table entries carry a 16-bit fingerprint of the 4 bytes at the stored
// position (high half; the position is the low half).  A probe whose
// fingerprint differs from its candidate's cannot match, so it skips the
// candidate load: about half of the probes fail, and their candidate lines
// were a quarter of the fetched bytes.  A fingerprint hit is confirmed by
// the loaded bytes as before, so the parse is unchanged (FSG_V3_FP=0: the
// reference's u16 position-only entries).
#ifndef FSG_V3_FP
#define FSG_V3_FP 1
#endif
constexpr bool kFp = FSG_V3_FP;
#if FSG_V3_FP
typedef u32 tent;
#else
typedef u16 tent;
#endif
__device__ __forceinline__ u32 fp_of(u32 x) { return (x * 0x9E3779B1u) & 0xffff0000u; }
__device__ __forceinline__ tent tab_entry(u32 pos, u32 x) { return (tent)(kFp ? pos | fp_of(x) : pos); }
constexpr u32 kWinDw = kWinChunks * 4;

__device__ u32x4 g_enc_dummy[2];

__device__ __forceinline__ u32 abyte(u32 hi, u32 lo, u32 s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

// Tag bytes of one EmitCopyLessThan64 (snappy.cc:198-214): packed little
// endian in the low bytes of the result; *nb = 2 or 3.
__device__ __forceinline__ u32 copy_tag_lt64(u32 offset, u32 len, u32* nb) {
  if (len < 12 && offset < 2048) {
    *nb = 2;
    return (1u + ((len - 4) << 2) + ((offset >> 8) << 5)) | ((offset & 0xffu) << 8);
  }
  *nb = 3;
  return (2u + ((len - 1) << 2)) | ((offset & 0xffffu) << 8);
}

// EmitCopy (snappy.cc:216-232).  Stores 4 bytes per tag (the spare bytes are
// overwritten by later output or lie in the slot's headroom).
__device__ __forceinline__ u8* emit_copy_v3(u8* op, u32 offset, u32 len) {
  u32 nb;
  while (len >= 68) {
    stu32(op, copy_tag_lt64(offset, 64, &nb));
    op += nb;
    len -= 64;
  }
  if (len > 64) {
    stu32(op, copy_tag_lt64(offset, 60, &nb));
    op += nb;
    len -= 60;
  }
  stu32(op, copy_tag_lt64(offset, len, &nb));
  return op + nb;
}

// Literal tag (snappy.cc:156-196); returns the tag length.
__device__ __forceinline__ u32 literal_tag(u32 len, u64* tag) {
  const u32 n = len - 1;
  if (n < 60) { *tag = n << 2; return 1; }
  const u32 count = n < (1u << 8) ? 1 : n < (1u << 16) ? 2 : n < (1u << 24) ? 3 : 4;
  *tag = (u64)((59 + count) << 2) | ((u64)n << 8);
  return 1 + count;
}

// Literal of `len` bytes copied from global memory (16 bytes at a time; the
// last store may spill into bytes later output overwrites, or the headroom).
__device__ __forceinline__ u8* emit_literal_global(u8* op, const u8* lit, u32 len) {
  u64 tag;
  const u32 tl = literal_tag(len, &tag);
  stu64(op, tag);
  op += tl;
  u32 k = 0;
  for (; k + 64 <= len; k += 64) {
    u32x4 a, b, c, d;
    __builtin_memcpy(&a, lit + k, 16);
    __builtin_memcpy(&b, lit + k + 16, 16);
    __builtin_memcpy(&c, lit + k + 32, 16);
    __builtin_memcpy(&d, lit + k + 48, 16);
    __builtin_memcpy(op + k, &a, 16);
    __builtin_memcpy(op + k + 16, &b, 16);
    __builtin_memcpy(op + k + 32, &c, 16);
    __builtin_memcpy(op + k + 48, &d, 16);
  }
  for (; k + 16 <= len; k += 16) copy16(op + k, lit + k);
  for (; k < len; ++k) op[k] = lit[k];
  return op + len;
}

}  // namespace

// Work items.  Messages of more than one 64 KiB fragment are split into one
// item per fragment (fragments compress independently: fresh table, offsets
// inside the fragment, snappy.cc:875-954), listed by encode_plan_kernel and
// handed out first; fragment k is staged in region k of the message's slot
// (R = slot / fragments bytes each) and encode_gather_kernel packs the regions.
// Then every single-fragment message is one item.  A fragment whose output
// would not fit its region (only possible for near-incompressible data close
// to MaxCompressedLength) marks its message kNeedFallback; the fallback pass
// (FSG_ENC_FALLBACK) re-encodes those messages whole, one lane each.
constexpr u32 kEncFallback = 1u;

template <int kK, int kPostProbes>
__global__ __launch_bounds__(64) void encode_pipe_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, u32* __restrict__ out_len,
    i32* __restrict__ status, tent* __restrict__ tables, u32 table_entries,
    u32* __restrict__ ctr, const u32* __restrict__ items, u32* __restrict__ sizes, u32 mode,
    u32 region_cap, u32 wave_min, u32 wave_share, u64 wave_all_bytes) {
  __shared__ u32 win[(kWinDw + 1) * kWave];
  const u32 lane = threadIdx.x;
  const u32 slot = blockIdx.x * blockDim.x + lane;
  tent* table = tables + (u64)slot * table_entries;
  auto wrd = [&](u32 d) -> u32 { return win[d * kWave + lane]; };
  const bool fallback = mode & kEncFallback;
  // wave_min != 0: the long list holds the split messages' fragments and the
  // messages of [wave_min, 64 KiB] bytes; encode_wave_kernel takes its first
  // `quota` units, the lanes the rest
  const u32 n_items = (fallback || !items) ? 0u : ctr[1];
  const u32 quota = (fallback || !items || !wave_min) ? 0u : wave_quota(ctr, wave_share, wave_all_bytes);
  const u32 lane_units = n_items - quota;

  for (;;) {
    const u32 w = atomicAdd(&ctr[fallback ? 4 : 0], 1u);
    u32 m, f_first, f_end;     // message, fragment range [f_first, f_end) in bytes
    bool staged = false;       // a fragment of a split message
    const u32 unit = quota + w;
    if (w < lane_units) {
      m = items[2 * unit];
      const u32 f = items[2 * unit + 1];
      staged = f != kWholeUnit;
      f_first = staged ? f << kBlockLog : 0u;
    } else {
      m = w - lane_units;
      if (m >= n_msgs) break;
      if (fallback ? status[m] != kNeedFallback
                   : ((items && in_len[m] > kBlockSize) ||
                      (wave_min && in_len[m] >= wave_min && in_len[m] <= kBlockSize)))
        continue;
      f_first = 0;
    }
    const u8* mb = in + in_off[m];
    const u32 total = in_len[m];
    f_end = staged ? min(total, f_first + kBlockSize) : total;
    u8* const dst = out + out_off[m];
    const u32 hdr = (u32)varint32_len(total);
    u8* op = dst;
    u8* op_lim = nullptr;      // staged: last byte a tag may start at (spill room kept)
    u8* region = dst;
    if (staged) {
      const u32 nfr = (total + kBlockSize - 1) >> kBlockLog;
      u32 R = ((u32)max_compressed_length(total) - hdr) / nfr & ~15u;
      if (region_cap && region_cap < R) R = region_cap;
      region = dst + hdr + (u64)(f_first >> kBlockLog) * R;
      op = region;
      op_lim = region + R - 32;
    }
    if (!staged || f_first == 0) {
      u8* h = dst;
      u32 v = total;
      while (v >= 128) { *h++ = (u8)(v | 128); v >>= 7; }
      *h++ = (u8)v;
      if (!staged) op = h;
    }
    bool ovf = false;
    // room for `bytes` more output (+16 spill) in a staged region
    auto room = [&](u32 bytes) -> bool { return !op_lim || op + bytes + 16 <= op_lim; };
    const u32 al = (u32)(reinterpret_cast<uintptr_t>(mb) & 15);
    const u8* abase = mb - al;
    const u32 last_chunk = total ? (al + total - 1) >> 4 : 0u;

    for (u32 fpos = f_first; fpos < f_end && !ovf; fpos += kBlockSize) {
      const u32 n = min(total - fpos, kBlockSize);
      const u8* fb = mb + fpos;
      const u32 ht = table_size_for(n);
      const int shift = 32 - (31 - __clz((int)ht));
      // zeroed table (snappy.cc:247-271): every entry is position 0
      auto fill_table = [&](u32 x0) {
        const u32 e = kFp ? (u32)tab_entry(0, x0) : 0u;
        u32x4* t4 = reinterpret_cast<u32x4*>(table);
        const u32x4 z = {e, e, e, e};
        for (u32 i = 0; i < ht * (u32)sizeof(tent) / 16; ++i) t4[i] = z;
      };
      if (!kFp) fill_table(0);
      if (n < kInputMarginBytes) {  // snappy.cc:346-347,446-450
        if (!room(n + 5)) { ovf = true; break; }
        op = emit_literal_global(op, fb, n);
        continue;
      }
      const u32 lim = n - kInputMarginBytes;

      // ---- input window: chunks [wc, wc + 5) of the message (aligned base)
      int wbase = 0;  // fragment position of window byte 0
      auto window_chunks = [&](u32 pos, u32x4 (&g)[kWinChunks]) -> u32 {
        const u32 c = (al + fpos + pos) >> 4;
#pragma unroll
        for (u32 i = 0; i < kWinChunks; ++i) {
          const u32 k = c + i <= last_chunk ? c + i : last_chunk;
          __builtin_memcpy(&g[i], abase + 16 * k, 16);
        }
        return c;
      };
      auto window_store = [&](u32 c, const u32x4 (&g)[kWinChunks]) {
#pragma unroll
        for (u32 i = 0; i < kWinChunks; ++i)
#pragma unroll
          for (u32 q = 0; q < 4; ++q) win[(4 * i + q) * kWave + lane] = g[i][q];
        wbase = (int)(16 * c) - (int)(al + fpos);
      };
      auto rd32 = [&](u32 pos) -> u32 {
        const u32 o = (u32)((int)pos - wbase);
        return abyte(wrd((o >> 2) + 1), wrd(o >> 2), o & 3);
      };
      // 16 bytes at window offset o (o + 20 <= 80)
      auto rd128 = [&](u32 o) -> u32x4 {
        u32x4 v;
#pragma unroll
        for (u32 q = 0; q < 4; ++q) v[q] = abyte(wrd((o >> 2) + q + 1), wrd((o >> 2) + q), o & 3);
        return v;
      };
      auto in_win = [&](u32 pos, u32 len) -> bool {
        const int o = (int)pos - wbase;
        return o >= 0 && o + (int)len <= (int)(16 * kWinChunks);
      };
      {
        u32x4 g0[kWinChunks];
        const u32 c = window_chunks(0, g0);
        window_store(c, g0);
      }
      if (kFp) fill_table(rd32(0));

      u32 ip = 1, next_emit = 0, skip = 32;
      bool post = false;
      for (;;) {
        // ---- probe positions of this batch (SK[k]: skip counter at probe k)
        u32 P[kK], SK[kK];
        bool live[kK];
        bool stop = false;  // a scan probe failed its bound: emit_remainder
        u32 s = post ? ip + 1 : ip, sk = post ? 32u : skip;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < kK; ++k) {
          SK[k] = sk;
          if (k == 0 && post) {
            P[k] = ip;
            live[k] = true;
            continue;
          }
          const u32 step = sk >> 5;
          const bool bound = s + step <= lim;  // next_ip > ip_limit -> remainder
          // after a copy the next copy usually starts at ip: fewer probes
          // (a capped probe is simply left for the next batch)
          const bool capped = post && k >= kPostProbes;
          stop = stop || (ok && !capped && !bound);
          ok = ok && bound && !capped;
          P[k] = s;
          live[k] = ok;
          if (ok) { s += step; ++sk; }
        }
        // window: pre-insertion, hash bytes of every live probe
        const u32 lo_need = post ? ip - 1 : P[0];
        u32 hi_need = P[0] + 4;
#pragma unroll
        for (int k = 0; k < kK; ++k) hi_need = live[k] ? P[k] + 4 : hi_need;
        if (!in_win(lo_need, hi_need - lo_need)) {
          u32x4 g0[kWinChunks];
          const u32 c = window_chunks(lo_need, g0);
          window_store(c, g0);
        }
        // probes past the (reloaded) window wait for the next batch, which
        // resumes the scan at the first of them
        int defer_k = -1;
#pragma unroll
        for (int k = kK - 1; k >= 0; --k)
          if (live[k] && !in_win(P[k], 4)) defer_k = k;
#pragma unroll
        for (int k = 0; k < kK; ++k) live[k] = live[k] && (defer_k < 0 || k < defer_k);
        if (defer_k >= 0) {
          stop = false;
#pragma unroll
          for (int k = 0; k < kK; ++k)
            if (k == defer_k) { s = P[k]; sk = SK[k]; }
        }
        u32 X[kK], H[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k) {
          X[k] = live[k] ? rd32(P[k]) : 0u;
          H[k] = hash_bytes(X[k], shift);
        }
        const u32 xpre = post ? rd32(ip - 1) : 0u;
        const u32 hpre = post ? hash_bytes(xpre, shift) : 0u;
        // ---- round trip 1: table entries
        u32 T[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k) T[k] = table[live[k] ? H[k] : 0u];
        // candidates: the sequential read-then-write order, resolved in
        // registers; need[k]: the candidate may match, its bytes are loaded
        u32 C[kK];
        bool need[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k) {
          u32 c = T[k] & 0xffffu;
          bool mb = !kFp || (T[k] & 0xffff0000u) == fp_of(X[k]);
          if (post && hpre == H[k]) { c = ip - 1; mb = xpre == X[k]; }
#pragma unroll
          for (int j = 0; j < k; ++j)
            if (live[j] && H[j] == H[k]) { c = P[j]; mb = X[j] == X[k]; }
          C[k] = c;
          need[k] = live[k] && mb;
        }
        // ---- round trip 2: candidate bytes + next window
        u32x4 CB[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k) {
          const u8* a = need[k] ? fb + C[k] : reinterpret_cast<const u8*>(g_enc_dummy);
          __builtin_memcpy(&CB[k], a, 16);
        }
        // refresh the window from lo_need only once half of it is consumed:
        // reloading all 80 bytes every batch (text advances ~7 bytes per
        // batch) cost 5 scattered 16-byte loads per lane per batch
        const bool pref = (int)lo_need - wbase >= 32;
        u32x4 gn[kWinChunks];
        u32 nc = 0;
        if (pref) nc = window_chunks(lo_need, gn);
        // winner
        int win_k = -1;
#pragma unroll
        for (int k = kK - 1; k >= 0; --k)
          if (need[k] && CB[k][0] == X[k]) win_k = k;
        // commit table writes (program order)
        if (post) table[hpre] = tab_entry(ip - 1, xpre);
#pragma unroll
        for (int k = 0; k < kK; ++k)
          if (live[k] && (win_k < 0 || k <= win_k)) table[H[k]] = tab_entry(P[k], X[k]);

        if (win_k >= 0) {
          u32 p = P[0], cand = C[0];
          u32x4 cb = CB[0];
#pragma unroll
          for (int k = 1; k < kK; ++k)
            if (win_k == k) { p = P[k]; cand = C[k]; cb = CB[k]; }
          // literal [next_emit, p)
          if (!room(p - next_emit + 5 + 3 * ((n - p + 63) >> 6) + 3)) { ovf = true; break; }
          if (p > next_emit) {
            const u32 len = p - next_emit;
            if (len <= 16 && in_win(next_emit, 20)) {
              u64 tag;
              const u32 tl = literal_tag(len, &tag);
              *op = (u8)tag;
              const u32x4 v = rd128((u32)((int)next_emit - wbase));
              __builtin_memcpy(op + tl, &v, 16);
              op += tl + len;
            } else {
              op = emit_literal_global(op, fb + next_emit, len);
            }
          }
          // match length: FindMatchLength(cand + 4, p + 4, fragment end)
          u32 mlen;
          {
            u32x4 pb;
            if (in_win(p, 20)) {
              pb = rd128((u32)((int)p - wbase));
            } else if (fpos + p + 16 <= total) {
              __builtin_memcpy(&pb, fb + p, 16);
            } else {  // last bytes of the message: load [p-1, p+15) and shift
              u32x4 t;
              __builtin_memcpy(&t, fb + p - 1, 16);
              pb[0] = abyte(t[1], t[0], 1);
              pb[1] = abyte(t[2], t[1], 1);
              pb[2] = abyte(t[3], t[2], 1);
              pb[3] = t[3] >> 8;  // byte p+15 is past the message: clamped below
            }
            const u64 x0 = ((u64)(pb[1] ^ cb[1]) << 32) | (pb[0] ^ cb[0]);
            const u64 x1 = ((u64)(pb[3] ^ cb[3]) << 32) | (pb[2] ^ cb[2]);
            mlen = x0 ? (u32)(__builtin_ctzll(x0) >> 3) : x1 ? 8 + (u32)(__builtin_ctzll(x1) >> 3) : 16u;
            if (mlen == 16) {
              while (p + mlen + 16 <= n) {
                u32x4 a, b;
                __builtin_memcpy(&a, fb + cand + mlen, 16);
                __builtin_memcpy(&b, fb + p + mlen, 16);
                const u64 y0 = ((u64)(a[1] ^ b[1]) << 32) | (a[0] ^ b[0]);
                const u64 y1 = ((u64)(a[3] ^ b[3]) << 32) | (a[2] ^ b[2]);
                if (y0 | y1) {
                  mlen += y0 ? (u32)(__builtin_ctzll(y0) >> 3) : 8 + (u32)(__builtin_ctzll(y1) >> 3);
                  goto matched;
                }
                mlen += 16;
              }
              while (p + mlen < n && fb[cand + mlen] == fb[p + mlen]) ++mlen;
            }
          matched:
            mlen = min(mlen, n - p);
          }
          op = emit_copy_v3(op, p - cand, mlen);
          ip = p + mlen;
          next_emit = ip;
          post = true;
          if (pref) window_store(nc, gn);
          if (ip >= lim) break;  // emit_remainder
        } else {
          if (pref) window_store(nc, gn);
          if (stop) break;       // emit_remainder
          ip = s;
          skip = sk;
          post = false;
        }
      }
      if (!ovf && next_emit < n) {
        if (!room(n - next_emit + 5)) { ovf = true; break; }
        op = emit_literal_global(op, fb + next_emit, n - next_emit);
      }
    }
    if (staged) {
      sizes[unit] = ovf ? 0xffffffffu : (u32)(op - region);
    } else {
      out_len[m] = (u32)(op - dst);
      status[m] = kOk;
    }
  }
}

// Lists the fragments of every message longer than one fragment (one item
// each) and the messages themselves; ctr[1] = items, ctr[2] = split messages.
// With long_min != 0 (the wave encoder is on) the messages of [long_min,
// 64 KiB] bytes are listed too, one whole-message unit each (fragment field
// kWholeUnit), and the bytes of all listed units are summed (ctr[6..7]) for
// the wave / lane split (wave_quota).
__global__ void encode_plan_kernel(const u32* __restrict__ in_len, u32 n_msgs,
                                   u32* __restrict__ ctr, u32* __restrict__ items,
                                   u32* __restrict__ frag_base, u32* __restrict__ big_list, u32 long_min) {
  const u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs) return;
  const u32 len = in_len[m];
  if (len > kBlockSize) {
    const u32 nfr = (len + kBlockSize - 1) >> kBlockLog;
    const u32 base = atomicAdd(&ctr[1], nfr);
    frag_base[m] = base;
    big_list[atomicAdd(&ctr[2], 1u)] = m;
    for (u32 k = 0; k < nfr; ++k) {
      items[2 * (base + k)] = m;
      items[2 * (base + k) + 1] = k;
    }
  } else if (long_min && len >= long_min) {
    const u32 u = atomicAdd(&ctr[1], 1u);
    items[2 * u] = m;
    items[2 * u + 1] = kWholeUnit;
  } else {
    return;
  }
  if (long_min) atomicAdd(reinterpret_cast<unsigned long long*>(ctr + 6), (unsigned long long)len);
}

// One wave per split message (grid-stride over the list): moves fragments 1..
// down behind fragment 0
// (ascending, 4 KiB batches; destinations never pass their sources) and
// writes the message's length and status.
__global__ __launch_bounds__(256) void encode_gather_kernel(
    const u32* __restrict__ in_len, u8* out, const u64* __restrict__ out_off,
    u32* __restrict__ out_len, i32* __restrict__ status, u32* __restrict__ ctr,
    const u32* __restrict__ frag_base, const u32* __restrict__ big_list,
    const u32* __restrict__ sizes, u32 region_cap) {
  const u32 lane = threadIdx.x & 63;
  const u32 n_big = ctr[2];
  const u32 wave0 = (u32)__builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const u32 n_waves = (gridDim.x * blockDim.x) >> 6;
  for (u32 idx = wave0; idx < n_big; idx += n_waves) {
    const u32 m = big_list[idx];
    const u32 total = in_len[m];
    const u32 nfr = (total + kBlockSize - 1) >> kBlockLog;
    const u32 hdr = (u32)varint32_len(total);
    u32 R = ((u32)max_compressed_length(total) - hdr) / nfr & ~15u;
    if (region_cap && region_cap < R) R = region_cap;
    const u32* sz = sizes + frag_base[m];
    bool bad = false;
    for (u32 k = lane; k < nfr; k += 64) bad = bad || sz[k] == 0xffffffffu;
    if (__any(bad)) {
      if (lane == 0) status[m] = kNeedFallback;
      continue;
    }
    u8* const dst = out + out_off[m];
    u32 pos = hdr + sz[0];
    for (u32 k = 1; k < nfr; ++k) {
      const u8* src = dst + hdr + (u64)k * R;
      u8* d = dst + pos;
      const u32 len = sz[k];
      for (u32 c0 = 0; c0 < len; c0 += 4096) {
        u32x4 x[4];
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 c = c0 + 1024 * r + 16 * lane;
          if (c < len) __builtin_memcpy(&x[r], src + c, 16);
        }
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 c = c0 + 1024 * r + 16 * lane;
          if (c < len) {
            if (c + 16 <= len) {
              __builtin_memcpy(d + c, &x[r], 16);
            } else {
              u8 b[16];
              __builtin_memcpy(b, &x[r], 16);
              for (u32 q = 0; q < len - c; ++q) d[c + q] = b[q];
            }
          }
        }
      }
      pos += len;
    }
    if (lane == 0) {
      out_len[m] = pos;
      status[m] = kOk;
    }
  }
}

// Per-lane hash tables for the lane-per-message encoder: [counter: 256 B]
// [tables: slots x entries x sizeof(tent)] (tent = u32 with FSG_V3_FP, the
// default: position + fingerprint, twice the u16 footprint), entries per WorkingMemory::GetHashTable
// (snappy.cc:247-271) for the largest fragment of the batch.
size_t encode_tables_workspace_bytes(u32 n_msgs, u32 max_in_len, u32* slots_out) {
  u32 cap = max_in_len == 0 || max_in_len > kBlockSize ? kBlockSize : max_in_len;
  const u32 entries = table_size_for(cap);
  // enough lanes to fill the chip several times over: 256 CUs x 16 waves x 64
  u32 slots = n_msgs < 262144u ? n_msgs : 262144u;
  slots = (slots + 255) / 256 * 256;
  if (slots == 0) slots = 256;
  if (slots_out) *slots_out = slots;
  return 256 + (size_t)slots * entries * sizeof(tent);
}

// Plan region: units (2 x u32 each: message, fragment or kWholeUnit), per-unit
// sizes, per-message first unit, split-message list.  Present when a message
// may be split (max_in_len > 64 KiB) or may be long enough for the wave
// encoder (>= kWaveMinBound).  (max_in_len 0 = unknown: no plan, every
// message encoded whole by one lane.)
constexpr u32 kWaveMinBound = 4096;  // smallest wave_min the plan region is sized for
constexpr u32 kSmallBatchEnc = 64;   // batches of at most this many messages: every message on the wave encoder
// Batches of short bodies only (at most this many bytes each): every message
// on the wave encoder too.  Their tables are small (8 KiB for 4 KiB bodies),
// so many waves fit per CU, and nothing else in the batch needs the LDS:
// 131,072 x 4 KiB text 19.1 -> 8.6 ms, 65,536 x 8 KiB 18.5 -> 11.4 ms
// against the lanes.
#ifndef FSG_ENC_ALL_WAVE_MAX
#define FSG_ENC_ALL_WAVE_MAX 8192
#endif
constexpr u32 kAllWaveMax = FSG_ENC_ALL_WAVE_MAX;
__host__ __device__ inline bool all_on_wave(u32 n_msgs, u32 max_in_len) {
  return max_in_len >= kInputMarginBytes && (n_msgs <= kSmallBatchEnc || max_in_len <= kAllWaveMax);
}
size_t encode_plan_bytes(u32 n_msgs, u32 max_in_len) {
  if (max_in_len < kWaveMinBound && !all_on_wave(n_msgs, max_in_len)) return 0;
  u64 per_msg = ((u64)max_in_len + kBlockSize - 1) >> kBlockLog;
  if (per_msg < 1) per_msg = 1;
  const u64 max_items = (u64)n_msgs * per_msg;
  return (size_t)(max_items * 12 + (u64)n_msgs * 8 + 256);
}

__global__ void encode_wave_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                   const u32* __restrict__ in_len, u32 n_msgs, u8* out,
                                   const u64* __restrict__ out_off, u32* __restrict__ out_len,
                                   i32* __restrict__ status, u32* __restrict__ ctr, const u32* __restrict__ items,
                                   u32* __restrict__ sizes, u32 region_cap, u32 share_permille, u64 all_bytes,
                                   u32 tab_stride);

// Per-device side stream for the wave encoder (created on first use; nullptr:
// the wave encoder runs on the caller's stream before the lanes).
namespace {
struct EncSide {
  hipStream_t stream = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  std::mutex mu;
};
EncSide* enc_side() {
  constexpr int kMaxDevices = 64;
  static EncSide g[kMaxDevices];
  static std::once_flag once[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  EncSide* s = &g[dev];
  std::call_once(once[dev], [s] {
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->join, hipEventDisableTiming) != hipSuccess)
      s->stream = nullptr;
  });
  return s->stream ? s : nullptr;
}
}  // namespace

hipError_t launch_encode_v3(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u32 max_in_len, u8* out, const u64* out_off,
                            u32* out_len, i32* status, void* ws, size_t ws_bytes,
                            u32 slots, u32 entries, size_t tables_bytes, u32 region_cap,
                            hipStream_t stream, u32 wave_min) {
  if (n_msgs == 0) return hipSuccess;
  u32* ctr = reinterpret_cast<u32*>(ws);
  tent* tables = reinterpret_cast<tent*>(reinterpret_cast<u8*>(ws) + 256);
  hipError_t e = hipMemsetAsync(ctr, 0, 256, stream);
  if (e != hipSuccess) return e;
  const size_t plan = encode_plan_bytes(n_msgs, max_in_len);
  u32 *items = nullptr, *sizes = nullptr, *frag_base = nullptr, *big_list = nullptr;
  const bool can_split = max_in_len > kBlockSize;
  if (wave_min && wave_min < kWaveMinBound) wave_min = kWaveMinBound;
  // A batch of at most one wave of messages (the host runtime's one-caller
  // batches: the wave encoder's latency for one message is a fraction of one
  // lane's, 4 KiB text ~0.2 ms against 1.1 ms in the C1 echo trace), or of
  // short bodies only (kAllWaveMax): every message on the wave encoder
  if (wave_min && all_on_wave(n_msgs, max_in_len)) wave_min = kInputMarginBytes;
  if (max_in_len < wave_min) wave_min = 0;  // nothing long enough (or no bound known)
  if (plan && ws_bytes >= tables_bytes + plan && (can_split || wave_min)) {
    const u64 max_items = (plan - 256 - (u64)n_msgs * 8) / 12;
    u8* p = reinterpret_cast<u8*>(ws) + tables_bytes;
    items = reinterpret_cast<u32*>(p);
    sizes = items + 2 * max_items;
    frag_base = sizes + max_items;
    big_list = frag_base + n_msgs;
    encode_plan_kernel<<<(n_msgs + 255) / 256, 256, 0, stream>>>(in_len, n_msgs, ctr, items, frag_base, big_list,
                                                                 wave_min);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else {
    wave_min = 0;
  }
  // Lanes in flight beside the wave encoder (decided here, once it is known
  // to run): 3/4 of the messages, at most 131,072.  The lanes' waves share
  // the SIMDs with the wave encoder's waves, whose serial chains set the
  // batch's time, and fewer lanes keep their tables and recent input
  // cache-resident, each encoding more messages.  Measured (A/B, one box): C5
  // 27.0 -> 18.8 ms (131,072 of 262,144; 98,304: 20.8, 196,608: 22.4), C3
  // 92.3 -> 85.4 ms (49,152 of 65,536; 32,768: 85.3).  Option encode_lanes
  // (a cap applied by the caller) replaces this rule.
  if (wave_min && n_msgs > 64 && opt(kOptEncodeLanes) == 0) {
    u32 beside = (u32)(((u64)n_msgs * 3 / 4 + 255) / 256 * 256);
    if (beside > 131072u) beside = 131072u;
    if (beside < slots) slots = beside;
  }
  // (options encode_wave_share / encode_wave_all_mb: the tests force the lane
  // share with encode_wave_all_mb 0).  The wave encoder's share of the long
  // units' bytes above the all-on-wave bound, in permille: C3, A/B on one box
  // (profiles/r6/enc/ab_c3_share_sweep*.log), 400 86.3-86.9 ms, 425 80.8-81.0,
  // 450 80.4-80.6, 475 80.2-80.3, 500 82.4-82.6, 550 89.6-90.1.
  const i64 share_opt = opt(kOptEncodeWaveShare), all_opt = opt(kOptEncodeWaveAllMb);
  const u32 kShare = share_opt >= 0 && share_opt <= 1000 ? (u32)share_opt : 475u;  // permille
  const u64 kAllBytes = (all_opt >= 0 && all_opt < (1 << 24) ? (u64)all_opt : 640ull) << 20;
  auto pipe = max_in_len > kBlockSize || max_in_len == 0
                  ? encode_pipe_kernel<FSG_V3_PROBES_SPLIT, FSG_V3_POST_PROBES_SPLIT>
                  : encode_pipe_kernel<kKFlat, kPostFlat>;
  // The wave encoder's share of the long units (hash table in LDS, one wave
  // per fragment: snappy_encode_wave.hip) runs on a side stream beside the
  // lanes, one wave per table's worth of LDS.
  EncSide* side = wave_min ? enc_side() : nullptr;
  std::unique_lock<std::mutex> lk;
  if (wave_min) {
    const u32 cap = max_in_len > kBlockSize ? kBlockSize : max_in_len;
    const u32 ht = table_size_for(cap), lds = ht * 2;
    // Workgroups of wg waves, one table each in the workgroup's LDS.  LDS is
    // allocated per workgroup in 1,280-byte granules out of 163,840 per CU
    // (profiles/r5/wenc/lds_resident_probe.txt: one-wave workgroups of
    // 31,744 B fit five per CU, of 32,256 B four), so five 32 KiB tables fit
    // only as one five-wave workgroup.
    constexpr u32 kCuLds = 160u * 1024u, kLdsGranule = 1280u;
    // Waves per workgroup (option encode_wave_wg, 1..5; default 1).  Five
    // 32 KiB tables fit per CU only as one five-wave workgroup, which takes
    // the CU's whole LDS: C3 with every unit on the wave encoder 159 -> 132
    // ms, but beside the lanes (whose 80-byte LDS windows then find no room)
    // C3 gained <= 1% and C5 lost 12% with the lanes' windows moved to
    // registers, and batches of short bodies alone lost 33-60% (DESIGN.md
    // section 5, round 6).
    const i64 wg_opt = opt(kOptEncodeWaveWg);
    u32 wg = wg_opt >= 1 && wg_opt <= (i64)kWaveEncMaxWaves ? (u32)wg_opt : 1u;
    while (wg > 1 && wg * lds > kCuLds) --wg;
    const u32 alloc = (wg * lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule;
    u32 per_cu = (kCuLds / alloc) * wg;
    if (per_cu > 32) per_cu = 32;  // waves per CU
    const i64 pc_opt = opt(kOptEncodeWavePerCu);
    if (pc_opt > 0 && (u64)pc_opt < per_cu) per_cu = (u32)pc_opt;
    u32 waves = 256u * (per_cu ? per_cu : 1u);
    // A batch has at most n_msgs x fragments units; the waves past them find
    // no unit but are still dispatched (one 4 KiB body: 5,120 waves of 8 KiB
    // tables, ~60 us in front of the lanes' launch).
    {
      const u64 units = (u64)n_msgs * (((u64)max_in_len + kBlockSize - 1) >> kBlockLog);
      if (units && units < waves) waves = (u32)units;
    }
    hipStream_t wstream = stream;
    if (side) {
      lk = std::unique_lock<std::mutex>(side->mu);
      if ((e = hipEventRecord(side->fork, stream)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(side->stream, side->fork, 0)) != hipSuccess) return e;
      wstream = side->stream;
    }
    if (wg > waves) wg = waves;
    encode_wave_kernel<<<(waves + wg - 1) / wg, 64 * wg, wg * lds, wstream>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_len, status, ctr, items, sizes, region_cap, kShare, kAllBytes, ht);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (side && (e = hipEventRecord(side->join, side->stream)) != hipSuccess) return e;
  }
  pipe<<<slots / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off, out_len, status, tables, entries,
                                      ctr, items, sizes, 0u, region_cap, wave_min, kShare, kAllBytes);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (side && (e = hipStreamWaitEvent(stream, side->join, 0)) != hipSuccess) return e;
  if (lk.owns_lock()) lk.unlock();
  if (items && can_split) {
    encode_gather_kernel<<<1024, 256, 0, stream>>>(in_len, out, out_off, out_len, status, ctr,
                                                   frag_base, big_list, sizes, region_cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    pipe<<<slots / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off, out_len, status,
                                        tables, entries, ctr, nullptr, nullptr, kEncFallback, 0u, 0u, 0u, 0ull);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace fsg
