// snappy_decode_v3.hip -- software-pipelined lane-per-message Snappy decode
// for gfx950.
//
// Same unit of work as decode_batch_kernel (v2): one LANE per message, tags cut
// into <=16-byte pieces, batches of pieces with one 16-byte load and one
// 16-byte store each.  The difference is how a lane spends the memory round
// trip.  With one lane per message a C3 launch (65,536 x 64 KiB) has a single
// wave per SIMD, so v2 sat parked on `s_waitcnt` for ~40% of its cycles
// (rocprofv3 SQ_WAIT_ANY, profiles/r1).  v3 overlaps the two halves of the work:
//
//   iteration t:  A  issue the piece loads of batch t-1   (records from t-1)
//                 B  parse batch t into piece records      (VALU, overlaps A)
//                 G  issue input-ring prefetch loads
//                 C  wait for A; store batch t-1
//
// Batch t's loads are issued in iteration t+1, after batch t-1's stores in
// program order, so the only hazard is the one v2 already handles: a copy whose
// source overlaps output still pending in its own batch closes the batch.
//
// Tag headers are read from a per-lane ring of input bytes in LDS (16 x
// 16-byte chunks, [dword][lane] layout: conflict-free ds_read2_b32), refilled
// two iterations ahead of the parse, instead of a 16:1 register mux.  Copies
// with offset < 16 (pattern replication, IncrementalCopy snappy.cc:98-152) are
// cut into pieces whose length is a multiple of the offset, so every piece is
// the same 16-byte expansion of the pattern, built with four v_perm_b32 from a
// selector table in LDS.
//
// Reference checks and statuses are exactly those of decode_lane_kernel
// (DecompressAllTags snappy.cc:716-787, writer checks :1141-1481,
// result :858-868).
#include "snappy_pieces.h"

namespace fsg {

namespace {

#ifndef FSG_V3_PIECES
#define FSG_V3_PIECES 16
#endif
#ifndef FSG_V3_LOOKBACK
#define FSG_V3_LOOKBACK 8
#endif
constexpr int kP3 = FSG_V3_PIECES;      // pieces per batch
constexpr int kLook = FSG_V3_LOOKBACK;  // earlier pieces searched to re-source a hazard
constexpr u32 kRingChunks = 16;  // 16-byte chunks per lane ring (256 B)
constexpr u32 kRingDwords = kRingChunks * 4;
constexpr u32 kAhead = 4;        // chunks fetched per iteration

// piece record meta word
constexpr u32 kKindLit = 0, kKindCopy = 1, kKindPat = 2;
__device__ __forceinline__ u32 m_cnt(u32 m) { return m & 31u; }
__device__ __forceinline__ u32 m_kind(u32 m) { return (m >> 5) & 3u; }
__device__ __forceinline__ u32 m_shf(u32 m) { return (m >> 7) & 15u; }
__device__ __forceinline__ bool m_exact(u32 m) { return (m >> 11) & 1u; }
__device__ __forceinline__ u32 m_off(u32 m) { return (m >> 12) & 15u; }

__device__ u32x4 g_dummy16[1];  // target of the loads of empty pieces

}  // namespace

__global__ __launch_bounds__(64) void decode_pipe_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_cap,
    u32* __restrict__ out_len, i32* __restrict__ status_out, u32 flags) {
  // [dword][lane]; dword 64 = copy of dword 0; dwords 65..68 absorb the
  // writes of unused prefetch chunks (the writes are unconditional so every
  // prefetch register is consumed on every path: no pending load crosses the
  // loop back edge, where the compiler would drain vmcnt)
  __shared__ u32 ring[(kRingDwords + 5) * kWave];
  __shared__ u32x4 sel_tab[16];

  const u32 lane = threadIdx.x;
  init_pattern_table(sel_tab, lane);
  __syncthreads();

  const bool strict = flags & 2u;
  const u32 m = blockIdx.x * blockDim.x + lane;
  // FSG_INTERNAL_FALLBACK_ONLY: decode only the messages the two-pass decoder
  // (v4) left to this kernel (status kNeedFallback), leave the rest alone.
  const bool fallback_only = flags & kFlagFallbackOnly;
  const bool valid_msg = m < n_msgs && (!fallback_only || status_out[m] == kNeedFallback);

  // ---- message setup (header, slot check)
  i32 status = kOk;  // < 0: parsing
  const u8* ib = in;
  u8* ob = out;
  u32 n_in = 0, expected = 0, ip = 0;
  if (valid_msg) {
    ib = in + in_off[m];
    n_in = in_len[m];
    u32 ulen = 0;
    const int h = parse_varint_header(ib, n_in, strict, &ulen);
    if (h == 0) { status = kBadHeader; out_len[m] = 0; }
    else {
      out_len[m] = ulen;
      expected = ulen;
      ip = (u32)h;
      ob = out + out_off[m];
      status = ulen > out_cap[m] ? kSlotTooSmall : -1;
    }
  }
  const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
  const u32 obal = (u32)(reinterpret_cast<uintptr_t>(ob) & 15);
  const u8* abase = ib - ibal;                       // 16-byte aligned input base
  const u32 last_chunk = n_in ? (ibal + n_in - 1) >> 4 : 0u;

  // ---- input ring: chunk k of the message lives in ring slot k & 15
  u32 wend = 0;  // chunks [.., wend) written to the ring
  u32 iend = 0;  // chunks [.., iend) issued
  auto ring_write = [&](u32 k, u32x4 v, bool live) {
    const u32 d = live ? (k & (kRingChunks - 1)) * 4 : kRingDwords + 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) ring[(d + i) * kWave + lane] = v[i];
    ring[(d == 0 ? kRingDwords : kRingDwords + 1) * kWave + lane] = v[0];
  };
  if (status < 0) {  // prefill synchronously: 4 chunks
    u32x4 c0[kAhead];
#pragma unroll
    for (u32 c = 0; c < kAhead; ++c) {
      const u32 k = c <= last_chunk ? c : last_chunk;
      c0[c] = *reinterpret_cast<const u32x4*>(abase + 16 * k);
    }
#pragma unroll
    for (u32 c = 0; c < kAhead; ++c)
      ring_write(c, c0[c], c <= last_chunk);
    wend = iend = (last_chunk + 1 < kAhead) ? last_chunk + 1 : kAhead;
  }

  // ---- parse state
  u32 op = 0;        // parser's output position
  u32 rem = 0;       // bytes of the current tag still to cut
  u32 src = 0;       // literal: input offset; copy: output offset; pattern: pattern start
  u32 kind = 0;      // current tag kind
  u32 pstep = 16;    // piece length of the current tag
  u32 poff = 0;      // pattern period

  // ---- executor state
  u32 eop = 0;       // executor's output position (= op one batch behind)

  // piece records: batch being parsed (cur) and batch being executed (prev)
  u32 rx_prev[kP3], rm_prev[kP3];
#pragma unroll
  for (int j = 0; j < kP3; ++j) { rx_prev[j] = 0; rm_prev[j] = 0; }

  // ring prefetch registers: loaded at the end of iteration t (after its
  // stores, so the loop head never waits on a store), written to the ring in
  // iteration t+1 after its parse, used by the parse of iteration t+2
  u32x4 g[kAhead];
#pragma unroll
  for (u32 c = 0; c < kAhead; ++c) g[c] = u32x4{0, 0, 0, 0};
  u32 gk_w = 0, gn_w = 0;  // chunks held by g

  bool more = true;
  auto iteration = [&]() {
    // ---------- A: loads of the previous batch's pieces
    u32x4 data[kP3];
#pragma unroll
    for (int j = 0; j < kP3; ++j) {
      const u32 mm = rm_prev[j];
      const u8* base = m_kind(mm) == kKindLit ? ib : ob;
      const u8* a = m_cnt(mm) ? base + (int)rx_prev[j] : reinterpret_cast<const u8*>(g_dummy16);
      __builtin_memcpy(&data[j], a, 16);
    }

    // ---------- B: parse this batch
    u32 rx[kP3], rm[kP3], pdst[kP3];
    const u32 batch_start = op;
    bool closed = status >= 0;
#pragma unroll
    for (int j = 0; j < kP3; ++j) {
      const bool need = !closed && rem == 0;
      const bool eof = need && ip == n_in;  // RefillTag eof
      const u32 P = ip + ibal;
      const bool inwin = (P + 5 <= 16 * wend) || wend > last_chunk;
      const u32 dw = (P >> 2) & (kRingDwords - 1), bsh = P & 3;
      const u32 lo = ring[dw * kWave + lane], hi = ring[(dw + 1) * kWave + lane];
      const u32 t0 = alignbyte(hi, lo, bsh);       // bytes ip..ip+3
      const u32 b4 = (hi >> (8 * bsh)) & 0xffu;      // byte ip+4
      const u32 c = t0 & 0xffu;
      const u32 type = c & 3;
      const bool is_lit = type == 0;
      const u32 l0 = (c >> 2) + 1;
      const bool longlit = is_lit && l0 >= 61;       // 1..4 length bytes (:744-750)
      const u32 nbl = longlit ? l0 - 60 : 0u;
      const u32 ext = (b4 << 24) | (t0 >> 8);        // bytes ip+1..ip+4
      const u32 msk = nbl >= 4 ? 0xffffffffu : ((1u << (8 * nbl)) - 1u);
      const u32 litlen = longlit ? (ext & msk) + 1u : l0;  // uint32 wrap: 0xffffffff+1 == 0
      const u32 nb = is_lit ? nbl : (type == 1 ? 1u : (type == 2 ? 2u : 4u));
      const u32 clen = type == 1 ? 4 + ((c >> 2) & 7) : l0;
      const u32 coff = type == 1 ? (((c >> 5) << 8) | ((t0 >> 8) & 0xffu))
                                 : (type == 2 ? ((t0 >> 8) & 0xffffu) : ext);
      const u32 len = is_lit ? litlen : clen;
      const u32 avail = n_in - ip - 1;
      const u32 space = expected - op;
      const bool bad = avail < nb ||
                       (is_lit ? (avail - nb < len || space < len)
                               : (coff - 1u >= op || space < len));
      const bool small = !is_lit && coff < 16;
      const bool hdr = need && !eof && inwin;
      const bool corrupt = hdr && bad;
      // a pattern copy reads the `off` bytes before it: only at a batch start
      const bool defer_small = hdr && !bad && small && op != batch_start;
      const bool take = hdr && !bad && !defer_small;
      status = eof ? (op == expected ? kOk : kCorrupt) : (corrupt ? kCorrupt : status);
      closed = closed || eof || corrupt || (need && !eof && !inwin) || defer_small;
      const u32 tkind = is_lit ? kKindLit : (small ? kKindPat : kKindCopy);
      kind = take ? tkind : kind;
      poff = take ? (small ? coff : 0u) : poff;
      pstep = take ? (small ? pat_step(coff) : 16u) : pstep;
      src = take ? (is_lit ? ip + 1 + nb : op - coff) : src;
      rem = take ? len : rem;
      ip = take ? ip + 1 + nb + (is_lit ? len : 0u) : ip;
      // ---- one piece of the current tag
      const u32 n = rem < pstep ? rem : pstep;
      const bool have = !closed && rem > 0;
      // A copy whose source is output still pending in this batch is
      // re-sourced to where those bytes come from -- the literal's input
      // bytes or the (already final) source of an earlier copy piece -- if
      // one of the last kLook pieces covers it; otherwise the batch closes.
      const bool pend = have && kind == kKindCopy && src + n > batch_start;
      u32 fdst = 0, fm = 0, fx = 0;
#pragma unroll
      for (int k = (j > kLook ? j - kLook : 0); k < j; ++k) {
        const bool cv = (rm[k] != 0) & (pdst[k] <= src);
        fdst = cv ? pdst[k] : fdst;
        fm = cv ? rm[k] : fm;
        fx = cv ? rx[k] : fx;
      }
      const u32 fkind = m_kind(fm);
      const bool fwd = pend & (fm != 0) & (src >= batch_start) & (src + n <= fdst + m_cnt(fm)) &
                       (fkind != kKindPat);
      const bool hazard = pend & !fwd;
      closed = closed || hazard;
      const bool emit = have && !hazard;
      const u32 fsrc = fx + m_shf(fm) + (src - fdst);
      const u32 ekind = fwd ? fkind : kind;
      const u32 esrc = fwd ? fsrc : src;
      const bool lit = ekind == kKindLit;
      const u32 rlen = lit ? n_in : expected;
      const int lo_off = -(int)(lit ? ibal : obal);
      const int tail = (int)rlen - 16;
      const int a_off = (esrc + 16 <= rlen) ? (int)esrc : (tail > lo_off ? tail : lo_off);
      rx[j] = (u32)a_off;
      pdst[j] = op;
      rm[j] = emit ? (n | (ekind << 5) | ((u32)((int)esrc - a_off) << 7) |
                      ((op + 16 > expected ? 1u : 0u) << 11) | (poff << 12))
                   : 0u;
      src += (emit && kind != kKindPat) ? n : 0u;
      op += emit ? n : 0u;
      rem -= emit ? n : 0u;
    }

    // ---------- C: wait for A, write the prefetched chunks, store batch t-1
#pragma unroll
    for (u32 c = 0; c < kAhead; ++c) ring_write(gk_w + c, g[c], c < gn_w);
    wend = gn_w ? gk_w + gn_w : wend;

    bool any_shift = false, any_pat = false, any_exact = false;
#pragma unroll
    for (int j = 0; j < kP3; ++j) {
      any_shift = any_shift || m_shf(rm_prev[j]) != 0;
      any_pat = any_pat || m_kind(rm_prev[j]) == kKindPat;
      any_exact = any_exact || m_exact(rm_prev[j]);
    }
    if (__any(any_shift)) {
#pragma unroll
      for (int j = 0; j < kP3; ++j)
        if (m_shf(rm_prev[j])) data[j] = shr_bytes(data[j], m_shf(rm_prev[j]));
    }
    if (__any(any_pat)) {
#pragma unroll
      for (int j = 0; j < kP3; ++j)
        if (m_kind(rm_prev[j]) == kKindPat && m_cnt(rm_prev[j]))
          data[j] = expand_pattern(data[j], m_off(rm_prev[j]), sel_tab);
    }
    u32 dsts[kP3];
#pragma unroll
    for (int j = 0; j < kP3; ++j) {
      const u32 mm = rm_prev[j];
      dsts[j] = eop;
      if (m_cnt(mm) && !m_exact(mm)) __builtin_memcpy(ob + eop, &data[j], 16);
      eop += m_cnt(mm);
    }
    if (__any(any_exact)) {
#pragma unroll
      for (int j = 0; j < kP3; ++j) {
        const u32 mm = rm_prev[j];
        if (m_cnt(mm) && m_exact(mm)) store_exact(ob + dsts[j], data[j], m_cnt(mm));
      }
    }

    // ---------- G: ring prefetch from the parse position
    {
      const u32 P = ip + ibal;
      const u32 pc = P >> 4;
      const u32 base = pc >= iend ? pc : iend;  // a long literal jumped past the ring: restart
      u32 cnt = 0;
#pragma unroll
      for (u32 c = 0; c < kAhead; ++c) {
        const u32 k = base + c;
        const bool ok = status < 0 && k <= last_chunk && k <= pc + (kRingChunks - 1);
        cnt += ok ? 1u : 0u;
        const u32 kk = k <= last_chunk ? k : last_chunk;
        g[c] = *reinterpret_cast<const u32x4*>(n_in ? abase + 16 * kk
                                                    : reinterpret_cast<const u8*>(g_dummy16));
      }
      iend = cnt ? base + cnt : iend;
      gk_w = base;
      gn_w = cnt;
    }

    bool had = false;
#pragma unroll
    for (int j = 0; j < kP3; ++j) {
      had = had || rm[j] != 0;
      rx_prev[j] = rx[j];
      rm_prev[j] = rm[j];
    }
    more = __any(status < 0 || had);
  };

  __builtin_amdgcn_s_waitcnt(0);  // drain the prologue's loads once, outside the loop
  while (more) iteration();
  if (valid_msg) status_out[m] = status;
}

hipError_t launch_decode_v3(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  decode_pipe_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off,
                                                           out_cap, out_len, status, flags);
  return hipGetLastError();
}

}  // namespace fsg
