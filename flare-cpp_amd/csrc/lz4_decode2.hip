// lz4_decode2.hip -- two-pass LZ4 block decode for gfx950 (SURVEY.md section
// 8(f) row 4: COMPRESS_TYPE_LZ4, /root/reference/flare/rpc/options.proto:74),
// on the machinery of the Snappy decoder (snappy_decode_v4.hip): a
// lane-per-message index pass that validates every block and marks its
// sequence boundaries in a bitmap, then a wave-per-message execution pass.
//
// Body = varint32 uncompressed length + one LZ4 block (lz4.hip).  A block is a
// chain of sequences: token (literal-length nibble, match-length nibble),
// literal-length extension bytes, the literals, a 2-byte offset, match-length
// extension bytes; the last sequence stops after its literals.  Rules:
// oracle/lz4_oracle.c lz4o_decompress_block (pinned to liblz4 1.9.3 by
// tests/test_lz4.py).
//
//   pass 1, lz4_index_kernel (one LANE per message): the oracle's walk without
//     touching output -- every check of lz4o_decompress_block, so the message's
//     final status comes from here -- and a bitmap over the block bytes with
//     TWO bits per sequence: its token and its offset field.  Tokens and
//     offsets alternate, so bit 2i is token i and bit 2i+1 its offset.  Input
//     through a per-lane LDS ring of 16-byte chunks (loads one iteration ahead
//     of the parse), bits through a per-lane LDS ring of 128-byte groups.
//     Blocks over big_min bytes are listed instead and indexed by
//     lz4_index_big_kernel, a wave per block (pointer doubling over 64-byte
//     windows, as the Snappy pass 1b).
//
//   pass 2, lz4_exec_kernel (one WAVE per message): takes up to 64 sequences
//     per group, one per lane.  From the three positions T (token), O (offset
//     field) and T' (next token) a lane needs only the token byte and the two
//     offset bytes, both prefetched one group ahead:
//       literal length  D = O - T - 1 (token + extension bytes + literals):
//                       D <= 14: lit = D; else the extension is 255.. b with
//                       D + 240 = 256 * n_ext + b, so lit = D - ((D + 240) >> 8)
//       match length    E = T' - O - 2 extension bytes: E = 0: (token & 15) + 4,
//                       E = 1: 19 + the byte at O + 2, E >= 2: long (a whole-wave
//                       sequence, which reads the byte at T' - 1)
//     The lane's output (literal, then match) gets its position from a prefix
//     sum; literals and far match chunks are written in round A, near match
//     chunks in rounds B in dependency order, in an LDS output window flushed
//     to the slot (as the Snappy pass 2).  A sequence with more than 64
//     literal or match bytes runs alone, by the whole wave, straight to the
//     slot.
//
// Messages whose bitmap does not fit the workspace get kNeedFallback and are
// decoded by lz4.hip's lane-per-message kernel.
#include <cstdlib>
#include <mutex>

#include "options.h"
#include "wave_util.h"

namespace fsg {

hipError_t launch_lz4_decode_fallback(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                                      const u64* out_off, const u32* out_cap, u32* out_len, i32* status,
                                      hipStream_t stream);

namespace {

// ---- pass 1 geometry
constexpr u32 kL4RingChunks = 16;  // per-lane input ring: 16 chunks of 16 bytes
constexpr u32 kL4RingDwords = 4 * kL4RingChunks;
#ifndef FSG_L4_TWO_PER_STEP
#define FSG_L4_TWO_PER_STEP 1
#endif
#ifndef FSG_L4_AHEAD
#define FSG_L4_AHEAD 8
#endif
// 12 steps of up to two sequences per iteration: C3 LZ4 index 2.97 ms (24
// single-sequence steps) -> 2.43 (10: 2.41, 8: 2.45, 16: 2.88, 24: 4.19 --
// the parse outruns the ring's loads; 12 with 10 chunks ahead: 2.47).
#ifndef FSG_L4_STEPS
#define FSG_L4_STEPS 12
#endif
constexpr u32 kL4Ahead = FSG_L4_AHEAD;  // chunks loaded per iteration
constexpr int kL4Steps = FSG_L4_STEPS;  // half-steps (token or offset field) per iteration
constexpr u32 kL4BitGroups = 4;    // per-lane ring of 128-byte bit groups (4 words each)
constexpr u32 kL4BitWords = 4 * kL4BitGroups;
constexpr i32 kL4Parsing = -1;

// ---- pass 2 geometry
constexpr u32 kL4Waves = 4;                   // waves per block
// The ring is refilled while it holds fewer than kL4RefillBelow positions; a
// fill adds <= 512 bits = <= 342 positions (two per three bytes).  With 1,024
// positions and a refill below 260, the next group's prefetch (issued at the
// end of this one) always finds its positions in the ring; measured slower
// on C3 than 512 / 130 all the same (6.66 vs 6.37 ms, A/B on one box, the
// larger ring costing a wave per SIMD), as were four round-A chunks per pass
// (6.95 vs 6.37: 84 VGPRs) and a 2,560-byte window (6.85).
#ifndef FSG_L4_RING
#define FSG_L4_RING 512
#endif
#ifndef FSG_L4_ITEMS
#define FSG_L4_ITEMS 2
#endif
constexpr u32 kL4Ring = FSG_L4_RING;          // bitmap positions per wave
constexpr u32 kL4FillWords = 16;
constexpr u32 kL4RefillBelow = kL4Ring >= 1024 ? 2 * (2 * 64 + 1) + 2 : 2 * 64 + 2;
static_assert(kL4RefillBelow + 342 <= kL4Ring, "a fill fits the ring");
constexpr u32 kL4ItemsPerPass = FSG_L4_ITEMS;  // round-A chunks per lane per round trip
#ifndef FSG_L4_WINDOW
#define FSG_L4_WINDOW 3072
#endif
constexpr u32 kL4Window = FSG_L4_WINDOW;      // LDS output window per wave
constexpr u32 kL4Keep = 1024;                 // history kept when it slides
constexpr u32 kL4GroupBytes = 1024;           // output bytes per group
constexpr u32 kL4Long = 64;                   // longer literal or match: whole-wave sequence
constexpr u32 kL4StageMax = (kL4Window + 32) / 2 - 16;  // period staged in LDS (long overlapping match)
static_assert(kL4Keep + kL4GroupBytes + 48 <= kL4Window, "a group fits the window after a slide");

// Diagnostic build only (-DFSG_STAMPS): per-phase cycle totals of
// lz4_exec_kernel summed over waves (slots 0-5), groups (6) and rounds-B
// iterations (7); read back with fsg_debug_l4stamps (tools/stamps.py lz4).
#ifdef FSG_STAMPS
__device__ unsigned long long g_l4_stamps[8];
#define L4STAMP(k)                                    \
  do {                                                \
    const u64 t_ = __builtin_amdgcn_s_memtime();      \
    st_[k] += t_ - t_last_;                           \
    t_last_ = t_;                                     \
  } while (0)
#define L4COUNT(k) (st_[k] += 1)
#else
#define L4STAMP(k) do { } while (0)
#define L4COUNT(k) do { } while (0)
#endif

// Far chunks: earlier output of this wave, read through the slot's buffer
// with an sc1 load (served by L2; the CU's L1 may hold a line filled before
// the bytes were stored -- see snappy_decode_v4.hip, far_load).
__device__ __forceinline__ u32x4 far16(__amdgpu_buffer_rsrc_t r, u32 off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}

// ===========================================================================
// Pass 1: validate + index, one lane per message.
//
// One step per sequence: the lane reads the 20 ring bytes from the dword
// holding its token (5 LDS dwords, one round trip).  When the sequence's
// offset field and match-length byte lie within them (literals of <= 12
// bytes: ~97% of text sequences) the whole sequence is checked and consumed
// in that step; a longer literal leaves the lane at its offset field
// (half = 1) for the next step, which the ring serves from wherever the
// literal ends.  The step is straight-line code with selects: every lane
// runs the same instructions whichever half it is in.  A 255 extension byte
// (a literal of >= 270 or a match of >= 274 bytes) stalls the lane until the
// end of the iteration, where its run of 255s is read from global memory.
__device__ __forceinline__ u32 mux4(u32 d0, u32 d1, u32 d2, u32 d3, u32 i) {
  const u32 a = (i & 1) ? d1 : d0;
  const u32 b = (i & 1) ? d3 : d2;
  return (i & 2) ? b : a;
}

__global__ __launch_bounds__(64) void lz4_index_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u32 n_msgs,
    const u32* __restrict__ out_cap, u32* __restrict__ out_len, i32* __restrict__ status_out,
    u32* __restrict__ bm_counter, u32* __restrict__ bm_base_out, u32* __restrict__ hdr_out,
    u32* __restrict__ bitmap, u64 bm_capacity_words, u32* __restrict__ big_list, u32 big_min) {
  // [dword][lane]; rows kL4RingDwords.. +3 repeat rows 0..3 (a 5-dword read
  // at the ring's end wraps)
  __shared__ u32 ring[(kL4RingDwords + 4) * kWave];
  __shared__ u32 bmr[kL4BitWords * kWave];
  const u32 lane = threadIdx.x;
  const u32 m = blockIdx.x * kWave + lane;
  const bool valid = m < n_msgs;
  const u8* ib = valid ? in + in_off[m] : in;
  const u32 n_in = valid ? in_len[m] : 0u;

  // header (lz4o_header: strict varint32) and slot (lz4o_decompress)
  i32 st = kOk;
  u32 ulen = 0, h = 0;
  if (valid) {
    h = (u32)parse_varint_header(ib, n_in, true, &ulen);
    if (h == 0) {
      st = kBadHeader;
      out_len[m] = 0;
    } else {
      out_len[m] = ulen;
      st = ulen > out_cap[m] ? kSlotTooSmall : kL4Parsing;
    }
  }
  const u8* bb = ib + h;
  const u32 n = st < 0 ? n_in - h : 0u;  // block bytes

  // bitmap: round_up(ceil(n / 32), 4) words, one bump allocation per wave
  const u32 words = st < 0 ? (((n + 31) >> 5) + 3) & ~3u : 0u;
  const u32 incl = wave_incl_scan(words);
  const u32 total = readlane(incl, 63);
  u32 base0 = 0;
  if (lane == 0 && total) base0 = atomicAdd(bm_counter, total);
  base0 = readlane(base0, 0);
  const u32 bmb = base0 + incl - words;
  if (st < 0 && (u64)bmb + words > bm_capacity_words) st = kNeedFallback;
  if (valid) {
    bm_base_out[m] = bmb;
    hdr_out[m] = h;
  }
  // blocks of more than big_min bytes: walked by lz4_index_big_kernel, a wave
  // per message (a lane takes ~60 ms per MB; bm_counter[1] counts the list)
  if (st < 0 && n > big_min) {
    st = kNeedBigIndex;
    big_list[atomicAdd(&bm_counter[1], 1u)] = m;
  }
  u32* bm = bitmap + bmb;

  const u32 bal = (u32)(reinterpret_cast<uintptr_t>(bb) & 15);
  const u8* abase = bb - bal;
  const u32 last_chunk = n ? (bal + n - 1) >> 4 : 0u;
#define L4_CHUNK(k) (*reinterpret_cast<const u32x4*>(abase + 16 * ((k) <= last_chunk ? (k) : last_chunk)))
#define L4_RING_WRITE(k, v)                                                             \
  do {                                                                                  \
    const u32 d_ = ((k) & (kL4RingChunks - 1)) * 4;                                     \
    _Pragma("unroll") for (u32 i_ = 0; i_ < 4; ++i_) ring[(d_ + i_) * kWave + lane] = (v)[i_]; \
    if (d_ == 0) {                                                                      \
      _Pragma("unroll") for (u32 i_ = 0; i_ < 4; ++i_) ring[(kL4RingDwords + i_) * kWave + lane] = (v)[i_]; \
    }                                                                                   \
  } while (0)

  u32 wend = 0, iend = 0;  // chunks landed in the ring end at wend; loads issued end at iend
  if (st < 0 && n) {
    u32x4 c0[4];
#pragma unroll
    for (u32 c = 0; c < 4; ++c) c0[c] = L4_CHUNK(c);
#pragma unroll
    for (u32 c = 0; c < 4; ++c)
      if (c <= last_chunk) L4_RING_WRITE(c, c0[c]);
    wend = iend = last_chunk + 1 < 4 ? last_chunk + 1 : 4u;
  }
#pragma unroll
  for (u32 q = 0; q < kL4BitWords; ++q) bmr[q * kWave + lane] = 0;
  u32 fg = 0;  // lowest bit group not yet stored
  const u32 ngroups = words >> 2;

  // walk state: pos = the next token (half 0) or offset field (half 1)
  u32 pos = 0, op = 0, nib = 0;
  bool half = false, stall = false;
  u32x4 g[kL4Ahead];
#pragma unroll
  for (u32 c = 0; c < kL4Ahead; ++c) g[c] = u32x4{0, 0, 0, 0};
  u32 gk = 0, gn = 0;
  __builtin_amdgcn_s_waitcnt(0);

  while (__any(st < 0)) {
    // a step at pos reads 20 ring bytes: pos + bal + 20 <= 16 * wend, or
    // anywhere once the ring reached the block's last chunk (bytes past the
    // block are never used: every used byte is checked against n)
    u32 lim = 0;
    if (st < 0) lim = wend > last_chunk ? 0xffffffffu : (16 * wend >= bal + 20 ? 16 * wend - bal - 20 : 0u);
#pragma unroll
    for (int j = 0; j < kL4Steps; ++j) {
      const bool look = st < 0 && !stall && (pos <= lim || (!half && pos >= n));
      const u32 P = pos + bal;
      const u32 dw = (P >> 2) & (kL4RingDwords - 1), s = P & 3;
      const u32 D0 = ring[dw * kWave + lane], D1 = ring[(dw + 1) * kWave + lane];
      const u32 D2 = ring[(dw + 2) * kWave + lane], D3 = ring[(dw + 3) * kWave + lane];
      const u32 D4 = ring[(dw + 4) * kWave + lane];
      const u32 x0 = alignbyte(D1, D0, s);
      // the token at pos (lz4o_decompress_block :168-184)
      const u32 tok = x0 & 0xffu, l0 = tok >> 4, b1 = (x0 >> 8) & 0xffu;
      const bool lx = l0 == 15;
      const u32 lit = l0 + (lx ? b1 : 0u);
      const u32 ipl = pos + 1 + (lx ? 1u : 0u);
      const bool slow0 = lx && b1 == 255;
      // (bitwise, not short-circuit: no branch in the unrolled walk; when
      // pos >= n the wrapped differences are never the deciding term)
      const u32 room = (n - ipl) < (ulen - op) ? (n - ipl) : (ulen - op);
      const bool tfail = (pos >= n) | (lx & (pos + 1 >= n)) | (!slow0 & (lit > room));
      // (u32: op <= ulen always; ipl <= n unless tfail)
      const bool last = lit + 12 > ulen - op || lit + 8 > n - ipl;
      const bool last_ok = ipl + lit == n && op + lit == ulen;
      const u32 rel = ipl + lit - pos;  // offset field - pos
      const bool fused = s + rel <= 15;
      // the offset field and match length (:188-202): at pos (half 1) or
      // right after the literal (a fused step); q + 8 <= n there
      const u32 k = half ? s : s + rel;  // <= 15 whenever used
      const u32 kd = k >> 2;
      const u32 w = alignbyte(mux4(D1, D2, D3, D4, kd), mux4(D0, D1, D2, D3, kd), k & 3);
      const u32 off = w & 0xffffu, b2 = (w >> 16) & 0xffu;
      const u32 nv = half ? nib : (tok & 15);
      const u32 opb = half ? op : op + lit;
      const u32 qpos = half ? pos : pos + rel;
      const bool mx = nv == 15;
      const u32 ml = nv + 4 + (mx ? b2 : 0u);
      const bool slow1 = mx && b2 == 255;
      const bool mfail = off == 0 || off > opb || (!slow1 && ml + 5 > ulen - opb);  // (opb <= ulen unless tfail)
      // outcomes
      const bool tstage = look && !half;
      const bool t_ok = tstage && !tfail && !slow0;  // token accepted: its bit
      const bool mstage = look && (half || (t_ok && !last && fused));
      const bool m_ok = mstage && !mfail && !slow1;   // match accepted: the offset field's bit
      const bool m_stall = mstage && !mfail && slow1;
      atomicOr(&bmr[((pos >> 5) & (kL4BitWords - 1)) * kWave + lane], t_ok ? 1u << (pos & 31) : 0u);
      atomicOr(&bmr[((qpos >> 5) & (kL4BitWords - 1)) * kWave + lane], m_ok ? 1u << (qpos & 31) : 0u);
      i32 nst = st;
      nst = (tstage && tfail) || (mstage && mfail) ? kCorrupt : nst;
      nst = t_ok && last ? (last_ok ? kOk : kCorrupt) : nst;
      st = nst;
      stall = stall || (tstage && !tfail && slow0) || m_stall;
      const bool to_half1 = (t_ok && !last && !fused) || m_stall;
      const u32 pos0 = pos;
      pos = m_ok ? qpos + 2 + (mx ? 1u : 0u) : (to_half1 ? qpos : pos);
      op = m_ok ? opb + ml : (to_half1 ? opb : op);
      nib = to_half1 ? nv : nib;
      half = m_ok ? false : (to_half1 ? true : half);
#if FSG_L4_TWO_PER_STEP
      // ---- the next sequence in the same step, when its token and offset
      // field lie in the 20 bytes read (offsets <= 15 from the first dword)
      // and it is a plain one: a literal of <= 14 bytes, no 255 match byte,
      // not the last sequence, every check passing.  Otherwise the next step
      // takes it the general way (and reports what failed).  pos < n - 4
      // here: the sequence before was not the last (q + 8 <= n).
      {
        const u32 k2 = s + (pos - pos0);
        const u32 w2 = alignbyte(mux4(D1, D2, D3, D4, k2 >> 2), mux4(D0, D1, D2, D3, k2 >> 2), k2 & 3);
        const u32 tok2 = w2 & 0xffu, l2 = tok2 >> 4;
        const u32 k3 = k2 + 1 + l2;
        const u32 w3 = alignbyte(mux4(D1, D2, D3, D4, k3 >> 2), mux4(D0, D1, D2, D3, k3 >> 2), k3 & 3);
        const u32 off2 = w3 & 0xffffu, bb2 = (w3 >> 16) & 0xffu;
        const u32 nib2 = tok2 & 15;
        const bool mx2 = nib2 == 15;
        const u32 ml2 = nib2 + 4 + (mx2 ? bb2 : 0u);
        const u32 opb2 = op + l2;
        // (not last: lit + 12 <= ulen - op and lit + 8 <= n - (pos + 1), which
        // also keep the literal inside the input and the output)
        const bool ok2 = m_ok & (k3 <= 15) & (l2 < 15) & !(mx2 & (bb2 == 255)) &
                         (l2 + 12 <= ulen - op) & (l2 + 8 <= n - pos - 1) & (off2 != 0) & (off2 <= opb2) &
                         (ml2 + 5 <= ulen - opb2);
        const u32 q2 = pos + 1 + l2;
        atomicOr(&bmr[((pos >> 5) & (kL4BitWords - 1)) * kWave + lane], ok2 ? 1u << (pos & 31) : 0u);
        atomicOr(&bmr[((q2 >> 5) & (kL4BitWords - 1)) * kWave + lane], ok2 ? 1u << (q2 & 31) : 0u);
        pos = ok2 ? q2 + 2 + (mx2 ? 1u : 0u) : pos;
        op = ok2 ? opb2 + ml2 : op;
      }
#endif
    }
    // ---------- stalled lanes: extension runs of 255s, from global memory
    if (stall && st < 0) {
      stall = false;
      if (!half) {  // a literal length: 15 + 255 + ... from pos + 2
        u32 p = pos + 2, lit = 15 + 255, b = 255;
        bool bad = false;
        do {
          if (p >= n) {
            bad = true;
            break;
          }
          b = bb[p++];
          lit += b;
        } while (b == 255 && lit <= n);  // (lit > n fails the next check either way)
        if (bad || lit > n - p || lit > ulen - op) {
          st = kCorrupt;
        } else {
          atomicOr(&bmr[((pos >> 5) & (kL4BitWords - 1)) * kWave + lane], 1u << (pos & 31));
          if ((u64)op + lit + 12 > ulen || (u64)p + lit + 8 > n) {  // the last sequence
            st = (p + lit == n && op + lit == ulen) ? kOk : kCorrupt;
          } else {
            op += lit;
            nib = bb[pos] & 15;
            pos = p + lit;
            half = true;
          }
        }
      } else {  // a match length: 19 + 255 + ... from pos + 3 (offset checked)
        u32 p = pos + 3, ml = 15 + 4 + 255, b = 255;
        bool bad = false;
        do {
          if (p >= n) {
            bad = true;
            break;
          }
          b = bb[p++];
          ml += b;
        } while (b == 255 && ml <= ulen);
        if (bad || (u64)ml + 5 > ulen - op) {
          st = kCorrupt;
        } else {
          atomicOr(&bmr[((pos >> 5) & (kL4BitWords - 1)) * kWave + lane], 1u << (pos & 31));
          op += ml;
          pos = p;
          half = false;
        }
      }
    }

    // ---------- store the bit groups the walk has left (every group of an
    // OK message is stored, zero groups included: the bitmap is not zeroed)
    if (st < 0 || st == kOk) {
      const u32 cur = st < 0 ? pos >> 7 : ngroups;
#pragma unroll
      for (u32 kk = 0; kk < kL4BitGroups; ++kk) {
        const u32 gi = fg + kk;
        if (gi < cur) {
          const u32 sl = (gi & (kL4BitGroups - 1)) * 4;
          u32x4 v;
#pragma unroll
          for (u32 q = 0; q < 4; ++q) v[q] = bmr[(sl + q) * kWave + lane];
          *reinterpret_cast<u32x4*>(bm + 4 * gi) = v;
#pragma unroll
          for (u32 q = 0; q < 4; ++q) bmr[(sl + q) * kWave + lane] = 0;
        }
      }
      for (u32 gi = fg + kL4BitGroups; gi < cur; ++gi) *reinterpret_cast<u32x4*>(bm + 4 * gi) = u32x4{0, 0, 0, 0};
      fg = cur > fg ? cur : fg;
    }

    // ---------- land last iteration's chunks, load the next ones
#pragma unroll
    for (u32 c = 0; c < kL4Ahead; ++c)
      if (c < gn) L4_RING_WRITE(gk + c, g[c]);
    wend = gn ? gk + gn : wend;
    gn = 0;
    if (st < 0) {
      const u32 pc = (pos + bal) >> 4;
      const u32 base = pc >= iend ? pc : iend;  // a long literal jumped past the ring: restart there
      if (pc >= iend) wend = pc;                // (nothing at or above pc is landed)
#pragma unroll
      for (u32 c = 0; c < kL4Ahead; ++c) {
        const u32 kc = base + c;
        gn += (kc <= last_chunk && kc <= pc + (kL4RingChunks - 1)) ? 1u : 0u;
        g[c] = L4_CHUNK(kc);
      }
      gk = base;
      iend = base + gn > iend ? base + gn : iend;
    }
  }
#undef L4_CHUNK
#undef L4_RING_WRITE
  if (valid) status_out[m] = st;
}

// ===========================================================================
// Pass 1, large blocks: one WAVE per listed message.  The lane walk reads its
// input through a 256-byte per-lane ring loaded 128 bytes per iteration, and a
// lone lane takes ~60 ms per MB.  Here the wave stages the block into an 8 KiB
// LDS ring, 4 KiB (64 lanes x 64 bytes) at a time, and indexes it 64 bytes
// per step, as the Snappy pass 1b (snappy_decode_v4.hip, index_big_message):
// every lane decodes the sequence that would start at its byte (literal
// length, offset field, match length, successor, the checks that need no walk
// state), the real sequence starts in the window -- the chain from the
// current position -- come from pointer doubling over the successors, their
// output positions from a prefix sum, and the position-dependent checks of
// lz4o_decompress_block run on all of them at once.  A sequence the window
// cannot decode (a 255 extension byte, an offset field more than 20 bytes on)
// is taken by a wave-uniform serial step.  Bits: the block's bitmap words are
// zeroed first, then ORed in.
constexpr u32 kBigRing = 8192;
constexpr u32 kBigRingDw = kBigRing / 4;
constexpr u32 kBigHalf = kBigRing / 2;
constexpr u32 kBigWaves = 4;

__device__ __forceinline__ u32 rfl(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }

// 4 bytes at byte k (0..20) of the 24 bytes X01 | X23 << 64 | X45 << 128
__device__ __forceinline__ u32 window4(u64 X01, u64 X23, u64 X45, u32 k) {
  const u64 lo = k < 8 ? X01 : (k < 16 ? X23 : X45);
  const u64 hi = k < 8 ? X23 : X45;
  const u32 sh = 8 * (k & 7);
  return sh ? (u32)((lo >> sh) | (hi << (64 - sh))) : (u32)lo;
}

__device__ i32 lz4_walk_big(u32 m, const u8* __restrict__ in, const u64* __restrict__ in_off,
                            const u32* __restrict__ in_len, const u32* __restrict__ out_len,
                            const u32* __restrict__ bm_base, const u32* __restrict__ hdr, u32* __restrict__ bitmap,
                            u32* ring, u32 lane) {
  const u32 h = rfl(hdr[m]);
  const u32 ulen = rfl(out_len[m]);
  const u32 n = rfl(in_len[m]) - h;  // > big_min > 0
  const u8* bb = in + in_off[m] + h;
  u32* bm = bitmap + rfl(bm_base[m]);
  const u32 words = (((n + 31) >> 5) + 3) & ~3u;
  for (u32 z = 4 * lane; z < words; z += 256) *reinterpret_cast<u32x4*>(bm + z) = u32x4{0, 0, 0, 0};
  wait_all_memory();  // the zeros land before the ORs
  const u32 bal = (u32)(reinterpret_cast<uintptr_t>(bb) & 15);
  const u8* abase = bb - bal;
  const u32 last_chunk = (bal + n - 1) >> 4;
  const __amdgpu_buffer_rsrc_t rs = msg_rsrc(abase, bal + n);
  // 4 bytes at block position p from global memory (bytes past the block read 0)
  auto g4 = [&](u32 p) -> u32 {
    const u32 P = p + bal;
    const u32 lo = rfl(__builtin_amdgcn_raw_buffer_load_b32(rs, P & ~3u, 0, 0));
    const u32 hi = rfl(__builtin_amdgcn_raw_buffer_load_b32(rs, (P & ~3u) + 4, 0, 0));
    return (u32)((((u64)hi << 32) | lo) >> (8 * (P & 3)));
  };
  // ring slots of chunks [c0, c0 + nch) (16-byte chunks from abase)
  auto stage = [&](u32 c0, u32 nch) {
    wave_lds_fence();
    for (u32 r = 0; r < nch; r += 64) {
      const u32 k = c0 + r + lane;
      const u32 kk = k <= last_chunk ? k : last_chunk;
      const u32x4 v = *reinterpret_cast<const u32x4*>(abase + 16 * kk);
      *reinterpret_cast<u32x4*>(ring + ((4 * k) & (kBigRingDw - 1))) = v;
    }
    wave_lds_fence();
    if (lane < 8) ring[kBigRingDw + lane] = ring[lane];  // reads that wrap the ring's end
    wave_lds_fence();
  };
  u32 sb = 0;  // the ring holds input offsets [sb, sb + kBigRing) from abase
  stage(0, kBigRing / 16);
  // the ring holds [P, P + 88) after this (P < sb + kBigHalf)
  auto keep = [&](u32 P) {
    if (P >= sb + kBigHalf) {  // slide by a half, or restage after a jump
      const u32 nsb = P & ~(kBigHalf - 1);
      if (nsb == sb + kBigHalf)
        stage((sb + kBigRing) >> 4, kBigHalf / 16);
      else
        stage(nsb >> 4, kBigRing / 16);
      sb = nsb;
    }
  };
  // 24 bytes at input offset P from the ring
  auto read24 = [&](u32 P, u64& X01, u64& X23, u64& X45) {
    const u32 dw = (P >> 2) & (kBigRingDw - 1), s = 8 * (P & 3);
    u32 d[7];
#pragma unroll
    for (u32 i = 0; i < 7; ++i) d[i] = ring[dw + i];
    u32 x[6];
#pragma unroll
    for (u32 i = 0; i < 6; ++i) x[i] = (u32)((((u64)d[i + 1] << 32) | d[i]) >> s);
    X01 = ((u64)x[1] << 32) | x[0];
    X23 = ((u64)x[3] << 32) | x[2];
    X45 = ((u64)x[5] << 32) | x[4];
  };
  auto set_bit = [&](u32 p) {
    if (lane == 0) __hip_atomic_fetch_or(bm + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  u32 pos = 0, op = 0;
  i32 status = -1;
  // One sequence at pos, wave-uniform (the lane walk's rules in order,
  // lz4o_decompress_block :168-202): returns with pos / op advanced, or
  // status set.
  auto serial = [&]() {
    keep(pos + bal);
    u64 X01, X23, X45;
    read24(pos + bal, X01, X23, X45);
    const u32 x0 = rfl((u32)X01);
    const u32 tok = x0 & 0xffu;
    u32 lit = tok >> 4, ip = pos + 1;
    if (lit == 15) {
      if (ip >= n) {
        status = kCorrupt;
        return;
      }
      u32 b = (x0 >> 8) & 0xffu;
      lit += b;
      ++ip;
      while (b == 255 && lit <= n) {
        if (ip >= n) {
          status = kCorrupt;
          return;
        }
        b = g4(ip) & 0xffu;
        ++ip;
        lit += b;
      }
    }
    if (lit > n - ip || lit > ulen - op) {
      status = kCorrupt;
      return;
    }
    set_bit(pos);
    if ((u64)op + lit + 12 > ulen || (u64)ip + lit + 8 > n) {  // the last sequence
      status = (ip + lit == n && op + lit == ulen) ? kOk : kCorrupt;
      return;
    }
    const u32 q = ip + lit;  // q + 8 <= n
    op += lit;
    const u32 k = q - pos;
    const u32 w = k <= 20 ? rfl(window4(X01, X23, X45, k)) : g4(q);
    const u32 off = w & 0xffffu;
    if (off == 0 || off > op) {
      status = kCorrupt;
      return;
    }
    set_bit(q);
    const u32 nib = tok & 15;
    u32 ml = nib + 4;
    ip = q + 2;
    if (nib == 15) {
      u32 b = (w >> 16) & 0xffu;
      ml += b;
      ++ip;
      while (b == 255 && ml <= ulen) {
        if (ip >= n) {
          status = kCorrupt;
          return;
        }
        b = g4(ip) & 0xffu;
        ++ip;
        ml += b;
      }
    }
    if ((u64)ml + 5 > ulen - op) {
      status = kCorrupt;
      return;
    }
    op += ml;
    pos = ip;
  };

  while (status < 0) {
    pos = rfl(pos);
    op = rfl(op);
    sb = rfl(sb);
    if (pos >= n) {
      status = kCorrupt;
      break;
    }
    const u32 wb = pos & ~31u;
    keep(wb + bal);
    // ---------- every lane decodes the sequence that would start at p
    const u32 p = wb + lane;
    u64 X01, X23, X45;
    read24(p + bal, X01, X23, X45);
    const u32 x0 = (u32)X01;
    const u32 tok = x0 & 0xffu, l0 = tok >> 4, b1 = (x0 >> 8) & 0xffu;
    const bool lx = l0 == 15;
    const bool slow_t = lx && b1 == 255;  // a run of 255s: the serial step
    const u32 lit = l0 + (lx ? b1 : 0u);
    const u32 ipl = p + 1 + (lx ? 1u : 0u);
    const bool bad_tok = (p >= n) | (lx & (p + 1 >= n));
    // (ipl <= n unless bad_tok; u32 differences only read when !bad_tok)
    const bool bad_lit = !slow_t && lit > n - ipl;
    const bool last_static = !slow_t && lit + 8 > n - ipl;
    const u32 k = 1 + (lx ? 1u : 0u) + lit;  // offset field - p
    const u32 w = window4(X01, X23, X45, k <= 20 ? k : 0u);
    const u32 off = w & 0xffffu, nib = tok & 15, b2 = (w >> 16) & 0xffu;
    const bool mx = nib == 15;
    const u32 ml = nib + 4 + (mx ? b2 : 0u);
    const bool complex = slow_t || (!last_static && (k > 20 || (mx && b2 == 255)));
    const u32 succ = p + k + 2 + (mx ? 1u : 0u);
    const bool stop = bad_tok || bad_lit || last_static || complex || succ >= wb + 64;
    // ---------- the chain from pos by pointer doubling (J: successor lane,
    // 64 = none in this window; M: the lanes within 2^r steps).  A sequence
    // is >= 3 bytes, so <= 22 start in 64 bytes: 5 rounds.
    u32 J = stop ? 64u : succ - wb;
    u64 M = 1ull << lane;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const u32 src = J < 64 ? J : lane;
      const u64 Mj = ((u64)(u32)__shfl((int)(u32)(M >> 32), (int)src, 64) << 32) |
                     (u32)__shfl((int)(u32)M, (int)src, 64);
      const u32 Jj = (u32)__shfl((int)J, (int)src, 64);
      if (J < 64) {
        M |= Mj;
        J = Jj;
      }
    }
    const u32 first = pos - wb;
    const u64 S = ((u64)readlane((u32)(M >> 32), first) << 32) | readlane((u32)M, first);
    const bool in_s = (S >> lane) & 1ull;
    // ---------- output positions and the position-dependent checks
    // (a chain lane that is not an event below has its lit + ml exact)
    const u32 len = in_s && !(bad_tok || bad_lit || last_static || complex) ? lit + ml : 0u;
    const u32 incl = dpp_incl_scan(len);
    const u32 opk = op + incl - len;
    const bool e_bad = in_s && (bad_tok || bad_lit || (!slow_t && lit > ulen - opk));
    const bool e_last = in_s && !e_bad && !slow_t && (last_static || (u64)opk + lit + 12 > ulen);
    const bool e_cx = in_s && !e_bad && !e_last && complex;
    const bool e_mbad = in_s && !e_bad && !e_last && !complex &&
                        (off == 0 || off > opk + lit || (u64)ml + 5 > ulen - opk - lit);
    const u64 Ev = __ballot(e_bad || e_last || e_cx || e_mbad);
    const u32 E = Ev ? (u32)__builtin_ctzll(Ev) : 64u;
    // bits: the chain below the event (and the token of a last sequence)
    if (in_s && (lane < E || (lane == E && e_last)))
      __hip_atomic_fetch_or(bm + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (in_s && lane < E) {
      const u32 q = p + k;
      __hip_atomic_fetch_or(bm + (q >> 5), 1u << (q & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (E < 64) {
      const u32 kind = readlane(e_bad || e_mbad ? 1u : (e_last ? ((ipl + lit == n && opk + lit == ulen) ? 2u : 1u) : 3u),
                                E);
      if (kind == 1) {
        status = kCorrupt;
        break;
      }
      if (kind == 2) {
        status = kOk;
        break;
      }
      pos = wb + E;  // a sequence for the serial step
      op = readlane(opk, E);
      serial();
      continue;
    }
    const u32 L = 63u - (u32)__builtin_clzll(S);
    pos = readlane(succ, L);
    op = readlane(opk + len, L);
  }
  return status;
}

__global__ __launch_bounds__(kBigWaves * 64) void lz4_index_big_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len,
    const u32* __restrict__ out_len, i32* __restrict__ status_out, u32* __restrict__ counter,
    const u32* __restrict__ big_list, const u32* __restrict__ bm_base, const u32* __restrict__ hdr,
    u32* __restrict__ bitmap) {
  __shared__ u32 ring_s[kBigWaves][kBigRingDw + 8];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 count = counter[1];
  if (count == 0) return;
  for (;;) {  // lane 0 adds 1; its result is the index
    const u32 got = atomicAdd(&counter[2], lane == 0 ? 1u : 0u);
    const u32 idx = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (idx >= count) break;
    const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)big_list[idx]);
    const i32 st = lz4_walk_big(m, in, in_off, in_len, out_len, bm_base, hdr, bitmap, ring_s[wv], lane);
    if (lane == 0) status_out[m] = st;
  }
}

// ===========================================================================
// Pass 2: execute, one wave per message.
__device__ __forceinline__ void lz4_exec_message(
    u32 m, const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len, const u32* __restrict__ bm_base,
    const u32* __restrict__ hdr, const u32* __restrict__ bitmap, u32* ring, u8* sb, const u32x4* sel_tab,
    const u32x4* mtab, u32 lane) {
  const u32 h = hdr[m];
  const u32 n = in_len[m] - h;
  const u32 expected = out_len[m];
  const u32* bm = bitmap + bm_base[m];
  const u8* bb = in + in_off[m] + h;
  u8* ob = out + out_off[m];
  const u32 bbal = (u32)(reinterpret_cast<uintptr_t>(bb) & 15);
  const u32 obal = (u32)(reinterpret_cast<uintptr_t>(ob) & 15);
  const __amdgpu_buffer_rsrc_t irsrc = msg_rsrc(bb - bbal, bbal + n);
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(ob - obal, (short)0, (int)(expected + obal), 0x00020000);
  const u32 nwords = (n + 31) >> 5;
  constexpr u32 M = kL4Ring - 1;

  u32 head = 0, tail = 0, scan = 0, op = 0;
  int sbase = -(int)obal;  // output position of sb[0] (window blocks = the slot's 16-byte blocks)
  u32 flushed = 0;         // output [0, flushed) is in the slot
  auto zero_from = [&](u32 from) {
    const u32 i = from + 16 * lane;
    if (i < kL4Window + 32) *reinterpret_cast<u32x4*>(sb + i) = u32x4{0, 0, 0, 0};
  };
  zero_from(0);
  u32 zero_end = 1024;
  wave_lds_fence();
  auto fill_word = [&](u32 sc) -> u32 {
    const u32 wi = sc + (lane >> 2);
    return (lane < 4 * kL4FillWords && wi < nwords) ? bm[wi] : 0u;
  };
  u32 bmw = fill_word(scan);
#ifdef FSG_STAMPS
  u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 t_last_ = __builtin_amdgcn_s_memtime();
#endif
  // prefetched per lane for the group at pf_head: 20 bytes from the dword
  // below the token, 8 from the dword below the offset field
  u32 pf_head = 0xffffffffu, pf_tail = 0;  // (entries at or above pf_tail were not in the ring yet)
  u32x4 pd = u32x4{0, 0, 0, 0};
  u32 pd4 = 0;
  u32x2 po = u32x2{0, 0};
  auto prefetch = [&](u32 t, u32 o) {
    const u32 a = (t + bbal) & ~3u;
    pd = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
    pd4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
    po = __builtin_amdgcn_raw_buffer_load_b64(irsrc, (o + bbal) & ~3u, 0, 0);
  };
  auto flush_to = [&](u32 fe) {
    if (fe <= flushed) return;
    const int b0 = (int)(((flushed + obal) & ~15u)) - (int)obal;
    for (int blk = b0 + 16 * (int)lane; blk < (int)fe; blk += 1024) {
      const u32 lo = blk < (int)flushed ? flushed : (u32)blk;
      const u32 hi = blk + 16 < (int)fe ? (u32)(blk + 16) : fe;
      if (hi - lo == 16) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(sb + (blk - sbase));
        __builtin_memcpy(ob + blk, &v, 16);
      } else {
        store_exact(ob + lo, lds_read16(sb + ((int)lo - sbase)), hi - lo);
      }
    }
    flushed = fe;
  };

  // one fill: kL4FillWords bitmap words (prefetched in bmw) into the ring
  auto fill = [&]() {
    u32 bits = (bmw >> (8 * (lane & 3))) & 0xffu;
    const u32 bitbase = (scan + (lane >> 2)) * 32 + 8 * (lane & 3);
    const u32 cnt = __builtin_popcount(bits);
    const u32 inc = dpp_incl_scan(cnt);
    u32 slot = tail + inc - cnt;
    while (bits) {
      ring[slot & M] = bitbase + __builtin_ctz(bits);
      ++slot;
      bits &= bits - 1;
    }
    tail += readlane(inc, 63);
    scan += kL4FillWords;
    bmw = fill_word(scan);
    wave_lds_fence();
  };

  for (;;) {
    // ---------- refill the position ring (a group needs 2 * 64 + 1 entries)
    if (tail - head < kL4RefillBelow && scan < nwords) {
      fill();
      L4STAMP(0);
      continue;
    }
    const u32 avail = tail - head;
    if (avail == 0 || op >= expected) break;
    const bool done = scan >= nwords;
    // done: the 2k - 1 entries left are k sequences, the last without offset
    const u32 kseq = done ? ((avail + 1) >> 1 < 64 ? (avail + 1) >> 1 : 64u) : ((avail - 1) >> 1 < 64 ? (avail - 1) >> 1 : 64u);
    const bool valid = lane < kseq;
    const bool is_last = done && 2 * lane + 1 >= avail;
    const u32 T = ring[(head + 2 * lane) & M];
    const u32 O = is_last ? n : ring[(head + 2 * lane + 1) & M];
    const u32 Tn = ring[(head + 2 * lane + 2) & M];
    if (pf_head != head || pf_tail < head + 2 * kseq) prefetch(T, O);

    // ---------- decode one sequence per lane (checked by pass 1)
    const u32 s = (T + bbal) & 3u;
    const u32 tok = alignbyte(pd[1], pd[0], s) & 0xffu;
    // bytes T+1 .. T+16 (a short literal's bytes)
    const bool q3 = s == 3;
    const u32 w0 = q3 ? pd[1] : pd[0], w1 = q3 ? pd[2] : pd[1], w2 = q3 ? pd[3] : pd[2];
    const u32 w3 = q3 ? pd4 : pd[3];
    const u32 b = (s + 1) & 3u;
    const u32x4 xr = u32x4{alignbyte(w1, w0, b), alignbyte(w2, w1, b), alignbyte(w3, w2, b), alignbyte(pd4, w3, b)};
    const u32 D = O - T - 1;
    const u32 lit = D <= 14 ? D : D - ((D + 240) >> 8);
    const u32 lsrc = O - lit;
    const u32 ow = alignbyte(po[1], po[0], (O + bbal) & 3u);  // bytes O .. O+3
    const u32 off = ow & 0xffffu;
    const u32 E = Tn - O - 2;
    const u32 ml = is_last ? 0u : (E == 0 ? (tok & 15) + 4 : 19 + ((ow >> 16) & 0xffu));
    const bool lng = valid && (lit > kL4Long || ml > kL4Long || (!is_last && E >= 2));
    const u64 bigm = __ballot(lng);
    L4STAMP(1);

    if (bigm & 1ull) {
      // ---------- a long sequence: the whole wave, straight to the slot
      const u32 L = readlane(lit, 0), S = readlane(lsrc, 0);
      const bool last0 = readlane(is_last ? 1u : 0u, 0) != 0;
      const u32 OFF = readlane(off, 0), E0 = readlane(E, 0), Tn0 = readlane(Tn, 0);
      u32 ML = last0 ? 0u : readlane(ml, 0);
      if (!last0 && E0 >= 2) {  // 19 + 255 (E - 1) + the last extension byte
        const u32 P = Tn0 - 1 + bbal;
        const u32 x = __builtin_amdgcn_raw_buffer_load_b32(irsrc, P & ~3u, 0, 0);
        ML = 19 + 255 * (E0 - 1) + ((x >> (8 * (P & 3))) & 0xffu);
      }
      flush_to(op);
      for (u32 k0 = 0; k0 < L; k0 += 4096) {  // literal: 4 KiB per step, loads first
        Raw16 x[4];
#pragma unroll
        for (u32 r = 0; r < 4; ++r) x[r] = raw_load16(irsrc, S + k0 + 1024 * r + lane * 16 + bbal);
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 k = k0 + 1024 * r + lane * 16;
          if (k < L) store_exact(ob + op + k, shifted16(x[r]), L - k < 16 ? L - k : 16u);
        }
      }
      op += L;
      if (ML) {
        wait_all_memory();  // every byte below op is in the slot (L2)
        const u32 d = op, src = op - OFF;
        if (OFF >= ML) {  // no overlap: a straight copy
          for (u32 k0 = 0; k0 < ML; k0 += 4096) {
            u32x4 x[4];
#pragma unroll
            for (u32 r = 0; r < 4; ++r) x[r] = far16(orsrc, src + k0 + 1024 * r + lane * 16 + obal);
#pragma unroll
            for (u32 r = 0; r < 4; ++r) {
              const u32 k = k0 + 1024 * r + lane * 16;
              if (k < ML) store_exact(ob + d + k, x[r], ML - k < 16 ? ML - k : 16u);
            }
          }
        } else if (OFF < 16) {  // period < 16: every piece is the same expanded pattern
          const u32x4 P = expand_pattern(far16(orsrc, src + obal), OFF, sel_tab);
          const u32 stp = pat_step(OFF);
          for (u32 k = lane * stp; k < ML; k += 64 * stp) store_exact(ob + d + k, P, ML - k < stp ? ML - k : stp);
        } else if (OFF <= kL4StageMax) {
          // period OFF staged twice in the window (free until the restart
          // below): chunk j reads its 16 bytes at phase 16 j mod OFF
          for (u32 i = 16 * lane; i < OFF; i += 1024) {
            const u32x4 x = far16(orsrc, src + i + obal);
            const u32 c = OFF - i < 16 ? OFF - i : 16u;
            store_exact(sb + i, x, c);
            store_exact(sb + OFF + i, x, c);
          }
          wave_lds_fence();
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the staged bytes are in LDS
          u32 ph = (16 * lane) % OFF;
          const u32 inc = 1024 % OFF;
          for (u32 k = 16 * lane; k < ML; k += 1024) {
            store_exact(ob + d + k, lds_read16(sb + ph), ML - k < 16 ? ML - k : 16u);
            ph += inc;
            ph = ph >= OFF ? ph - OFF : ph;
          }
        } else {
          // a long period: steps of at most OFF bytes, each reading only
          // bytes the earlier steps stored
          const u32 step = (OFF & ~15u) < 4096 ? (OFF & ~15u) : 4096u;
          for (u32 k0 = 0; k0 < ML; k0 += step) {
            const u32 e = k0 + step < ML ? k0 + step : ML;
            for (u32 k = k0 + 16 * lane; k < e; k += 1024)
              store_exact(ob + d + k, far16(orsrc, src + k + obal), e - k < 16 ? e - k : 16u);
            wait_all_memory();
          }
        }
        op += ML;
      }
      // restart the window one block before the block holding op; its head
      // (the bytes [sbase, op)) comes back from the slot
      wait_all_memory();
      sbase = (int)((op + obal) & ~15u) - (int)obal - 16;
      zero_from(0);
      zero_end = 1024;
      wave_lds_fence();
      if (lane < 2) {
        const int lo = sbase + 16 * (int)lane;
        if (lo >= 0 && (u32)lo < op) {
          const u32 c = op - (u32)lo < 16 ? op - (u32)lo : 16u;
          store_exact(sb + 16 * lane, far16(orsrc, (u32)lo + obal), c);
        }
      }
      wave_lds_fence();
      flushed = op;
      head += last0 ? 1u : 2u;
      pf_head = 0xffffffffu;
      // the sequence's bytes hold no other positions: resume the bitmap scan
      // at the next token's word
      if (head == tail && !last0) {
        const u32 nw = Tn0 >> 5;
        if (nw > scan) {
          scan = nw;
          bmw = fill_word(scan);
        }
      }
      L4STAMP(2);
      continue;
    }
    const u32 take = bigm ? (u32)__builtin_ctzll(bigm) : kseq;
    const bool v = lane < take;

    // ---------- output positions: <= kL4GroupBytes per group
    const u32 len = v ? lit + ml : 0u;
    const u32 incl = dpp_incl_scan(len);
    const u32 t_op = op + incl - len;
    const bool fits = v && incl <= kL4GroupBytes;
    const u32 k_seq = (u32)__builtin_popcountll(__ballot(fits));
    const u32 tot = readlane(incl, k_seq - 1);
    const bool group_last = readlane(is_last ? 1u : 0u, k_seq - 1) != 0;

    // ---------- slide the window if this group would overrun it
    if (op + tot - sbase > kL4Window) {
      const int nsb = (int)(((op - kL4Keep + obal) & ~15u)) - (int)obal;
      // far chunks may read up to 15 bytes at and above the new base
      if ((int)flushed < nsb + 16) flush_to((u32)((int)((op + obal) & ~15u) - (int)obal));
      wait_all_memory();
      const u32 shift = (u32)(nsb - sbase), keep = (u32)((int)op - nsb);
      for (u32 k = 0; k < keep; k += 1024) {
        const u32 i = k + 16 * lane;
        u32x4 x = u32x4{0, 0, 0, 0};
        if (i < keep) x = *reinterpret_cast<const u32x4*>(sb + shift + i);
        wave_lds_fence();
        if (i < keep) *reinterpret_cast<u32x4*>(sb + i) = x;
        wave_lds_fence();
      }
      sbase = nsb;
      zero_end = (keep + 15) & ~15u;
    }
    // ---------- prefetch the next group; the ring is refilled first when
    // the next group would find it short (a fill writes slots below nh only:
    // tail - nh < kL4RefillBelow and a fill adds <= 342), so the prefetch
    // covers all of that group's positions (else the group reloads them
    // itself, one exposed round trip)
    {
      const u32 nh = head + 2 * k_seq;
      if (tail - nh < kL4RefillBelow && scan < nwords) fill();
      const u32 nT = ring[(nh + 2 * lane) & M];
      const u32 nO = ring[(nh + 2 * lane + 1) & M];
      prefetch(nT, nO);
      pf_head = nh;
      pf_tail = tail;
    }
    while (op + tot + 20 - sbase > zero_end) {
      zero_from(zero_end);
      zero_end += 1024;
    }
    wave_lds_fence();
    L4STAMP(3);

    // ---------- round A: literals (registers for <= 14 bytes, else the
    // input) and the match's leading chunks whose source starts below the
    // window base (the slot)
    const u32 mo = t_op + lit - off;  // match source
    const bool pat = off < 16 && off < ml;
    const u32 nch = (ml + 15) >> 4;
    const u32 below = (u32)(sbase - (int)mo);
    const u32 kfar = (int)below > 0 ? ((below - 1) >> 4) + 1 : 0u;
    const u32 kc = (!fits || is_last || pat) ? 0u : (kfar < nch ? kfar : nch);
    // a literal of <= 14 bytes comes from the prefetched token bytes; a
    // longer one in 16-byte chunks from the input
    const bool regl = fits && lit > 0 && lit <= 14;
    const u32 nlm = (fits && lit > 14) ? (lit + 15) >> 4 : 0u;
    const u32 wa = (u32)((int)t_op - sbase);
    const u32 wm = wa + lit;
    // load items: input literal chunks [0, nlm), then far chunks [0, kc); two
    // per round trip
    const u32 nit = nlm + kc;
    // the previous groups' completed blocks, 1 KiB at a time
    auto flush_group = [&]() {
      const int fe = (int)((op + obal) & ~15u) - (int)obal;
      if (fe >= (int)flushed + 1024) flush_to((u32)fe);
    };
    if (!__ballot(nit > 0)) {
      flush_group();
      if (regl) or_store(sb, wa, xr, lit, mtab);
    }
    for (u32 i0 = 0; __ballot(i0 < nit); i0 += kL4ItemsPerPass) {
      u32x4 xs[kL4ItemsPerPass];
      u32 ys[kL4ItemsPerPass];
#pragma unroll
      for (u32 r = 0; r < kL4ItemsPerPass; ++r) {
        xs[r] = u32x4{0, 0, 0, 0};
        ys[r] = 0;
      }
#pragma unroll
      for (u32 r = 0; r < kL4ItemsPerPass; ++r) {
        const u32 it = i0 + r;
        if (it < nlm) {
          const u32 a = (lsrc + 16 * it + bbal) & ~3u;
          xs[r] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
          ys[r] = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
        } else if (it < nit) {
          xs[r] = far16(orsrc, mo + 16 * (it - nlm) + obal);
        }
      }
      if (i0 == 0) {  // while the loads are in flight
        flush_group();
        if (regl) or_store(sb, wa, xr, lit, mtab);
      }
#pragma unroll
      for (u32 r = 0; r < kL4ItemsPerPass; ++r) {
        const u32 it = i0 + r;
        if (it < nlm) {
          const u32 sh = (lsrc + 16 * it + bbal) & 3u;
          const u32x4 x = u32x4{alignbyte(xs[r][1], xs[r][0], sh), alignbyte(xs[r][2], xs[r][1], sh),
                                alignbyte(xs[r][3], xs[r][2], sh), alignbyte(ys[r], xs[r][3], sh)};
          const u32 rr = lit - 16 * it;
          or_store(sb, wa + 16 * it, x, rr < 16 ? rr : 16u, mtab);
        } else if (it < nit) {
          const u32 k = it - nlm;
          const u32 rr = ml - 16 * k;
          or_store(sb, wm + 16 * k, xs[r], rr < 16 ? rr : 16u, mtab);
        }
      }
    }
    wave_lds_fence();
    L4STAMP(4);

    // ---------- rounds B: the near match chunks in dependency order (as the
    // Snappy pass 2: a chunk runs once its source ends at or below the first
    // unfinished chunk; read-modify-write merges exactly n bytes).  C3 text
    // takes 6.5 rounds per group.  Also letting a chunk run once no other
    // pending lane's output overlaps its source (the overlapping lanes found
    // by two binary searches over the lanes' output bounds, ds_bpermute)
    // cut that only to 5.2 -- the dependencies are real chains -- and was
    // slower (exec 5.57 -> 6.30 ms, A/B on one box).
    u32 rem = (fits && !is_last && kc < nch) ? ml - 16 * kc : 0u;
    u32 cw = wm + 16 * kc;
    u32 sw = (u32)((int)mo - sbase) + 16 * kc;
    const u32 stp = pat ? pat_step(off) : 16u;
    u32 nb = rem < stp ? rem : stp;
    bool pf = pat;
    u32 ne = rem ? (pf ? cw : sw + nb) : 0xffffffffu;
    u64 pend = __ballot(rem > 0);
    while (pend) {
      const u32 W = readlane(cw, (u32)__builtin_ctzll(pend));
      if (ne <= W) {
        u32x4 x = lds_read16(sb + sw);
        if (pf) x = expand_pattern(x, off, sel_tab);
        const u32x4 o = lds_read16(sb + cw);
        const u32x4 mk = mtab[nb];
        u32x4 y;
        y[0] = (x[0] & mk[0]) | (o[0] & ~mk[0]);
        y[1] = (x[1] & mk[1]) | (o[1] & ~mk[1]);
        y[2] = (x[2] & mk[2]) | (o[2] & ~mk[2]);
        y[3] = (x[3] & mk[3]) | (o[3] & ~mk[3]);
        __builtin_memcpy(sb + cw, &y, 16);
        rem -= nb;
        cw += nb;
        sw = pat ? cw - stp : sw + nb;
        pf = false;
        nb = rem < stp ? rem : stp;
        ne = rem ? sw + nb : 0xffffffffu;
      }
      wave_lds_fence();
      pend = __ballot(rem > 0);
      L4COUNT(7);
    }
    op += tot;
    head += group_last ? 2 * k_seq - 1 : 2 * k_seq;
    L4STAMP(5);
    L4COUNT(6);
  }
  flush_to(expected);
#ifdef FSG_STAMPS
  if (lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&g_l4_stamps[k], (unsigned long long)st_[k]);
#endif
}

// 7 waves per SIMD (72 VGPRs): exec 5.79 -> 5.49 ms against 6 (A/B, one
// box); 8 (64 VGPRs, 18 spilled, 2,816-byte window) 7.6 ms.
#ifndef FSG_L4_EXEC_WAVES
#define FSG_L4_EXEC_WAVES 7
#endif
__global__ __launch_bounds__(kL4Waves * 64) __attribute__((amdgpu_waves_per_eu(FSG_L4_EXEC_WAVES, FSG_L4_EXEC_WAVES))) void lz4_exec_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u32 n_msgs,
    u8* out, const u64* __restrict__ out_off, const u32* __restrict__ out_len, const i32* __restrict__ status,
    const u32* __restrict__ bm_base, const u32* __restrict__ hdr, const u32* __restrict__ bitmap) {
  __shared__ __attribute__((aligned(16))) u8 wl_s[kL4Waves][4 * kL4Ring + kL4Window + 32];
  __shared__ u32x4 sel_tab[16];
  __shared__ u32x4 mask_tab[17];
  if (threadIdx.x < 64) init_pattern_table(sel_tab, threadIdx.x);
  init_mask_table(mask_tab, threadIdx.x);
  __syncthreads();
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 m = blockIdx.x * kL4Waves + wv;
  if (m >= n_msgs || status[m] != kOk || out_len[m] == 0) return;
  lz4_exec_message(m, in, in_off, in_len, out, out_off, out_len, bm_base, hdr, bitmap,
                   reinterpret_cast<u32*>(wl_s[wv]), wl_s[wv] + 4 * kL4Ring, sel_tab, mask_tab, lane);
}

}  // namespace

#ifdef FSG_STAMPS
extern "C" int fsg_debug_l4stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l4_stamps), sizeof(g_l4_stamps));
  if (reset) {
    unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_l4_stamps), z, sizeof(z));
  }
  return e == hipSuccess ? 0 : -1;
}
#endif

// Workspace: [0, 256) counters (0 bitmap words allocated, 1 large blocks
// listed, 2 large blocks taken) | bm_base[n] | hdr[n] | big_list[n] | bitmap
// words (round_up(ceil(block / 32), 4) per message <= total / 32 + 4 n).
constexpr u64 kL4Head = 256;
__host__ u64 l4_list_bytes(u32 n) { return ((u64)n * 4 + 255) & ~(u64)255; }
size_t lz4_decode_workspace_bytes(u32 n_msgs, u64 total_in_bytes) {
  return kL4Head + 3 * l4_list_bytes(n_msgs) + 4 * (total_in_bytes / 32 + 4 * (u64)n_msgs + 4);
}
// blocks above this many bytes take the wave walk (FSG_L4_BIG_MIN, read per
// call: the tests lower it)
constexpr u32 kL4BigMin = 65536;
constexpr u32 kL4SmallBatch = 256;
constexpr u32 kL4BigMinSmall = 2048;

// Per-device event that orders the execution pass behind the index pass in
// the two-stream form (created on first use; nullptr: one stream).
namespace {
struct L4Two {
  hipEvent_t pass1 = nullptr;
  std::mutex mu;
};
L4Two* l4_two() {
  constexpr int kMaxDevices = 64;
  static L4Two g[kMaxDevices];
  static std::once_flag once[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  L4Two* t = &g[dev];
  std::call_once(once[dev], [t] {
    if (hipEventCreateWithFlags(&t->pass1, hipEventDisableTiming) != hipSuccess) t->pass1 = nullptr;
  });
  return t->pass1 ? t : nullptr;
}
}  // namespace

hipError_t launch_lz4_decode2(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                              const u64* out_off, const u32* out_cap, u32* out_len, i32* status, void* ws,
                              size_t ws_bytes, hipStream_t stream, hipStream_t pass1_stream) {
  if (n_msgs == 0) return hipSuccess;
  const u64 fixed = kL4Head + 3 * l4_list_bytes(n_msgs);
  if (ws_bytes < fixed) return hipErrorInvalidValue;
  // Two-stream form (as launch_decode_v4's): the index pass on pass1_stream,
  // the execution and fallback passes on `stream` behind an event, so a
  // caller's next batch walks while this one executes
  L4Two* two = pass1_stream && pass1_stream != stream ? l4_two() : nullptr;
  hipStream_t s1 = two ? pass1_stream : stream;
  hipError_t e = hipSuccess;
  if (pass1_stream && pass1_stream != stream && !two) {  // no event: order stream behind pass1_stream
    hipEvent_t ev = nullptr;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, pass1_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev, 0);
    if (ev) (void)hipEventDestroy(ev);
    if (e != hipSuccess) return e;
  }
  u8* w = static_cast<u8*>(ws);
  u32* counter = reinterpret_cast<u32*>(w);
  u32* bm_base = reinterpret_cast<u32*>(w + kL4Head);
  u32* hdr = reinterpret_cast<u32*>(w + kL4Head + l4_list_bytes(n_msgs));
  u32* big_list = reinterpret_cast<u32*>(w + kL4Head + 2 * l4_list_bytes(n_msgs));
  u32* bitmap = reinterpret_cast<u32*>(w + fixed);
  // a batch of at most kL4SmallBatch messages has the chip to itself: a
  // wave per block is quicker than one lane per block from a few KiB on
  // (option lz4_big_min overrides, -1 = this rule)
  const i64 bm_opt = opt(kOptLz4BigMin);
  const u32 big_min = bm_opt >= 0 && bm_opt <= 0xffffffffll ? (u32)bm_opt
                                                            : (n_msgs <= kL4SmallBatch ? kL4BigMinSmall : kL4BigMin);
  const u64 cap_words = (ws_bytes - fixed) / 16 * 4;  // whole 16-byte groups
  e = hipMemsetAsync(counter, 0, kL4Head, s1);
  if (e != hipSuccess) return e;
  lz4_index_kernel<<<(n_msgs + 63) / 64, 64, 0, s1>>>(in, in_off, in_len, n_msgs, out_cap, out_len, status,
                                                      counter, bm_base, hdr, bitmap, cap_words, big_list, big_min);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // (a grid of 256 blocks: with no listed block each wave reads the count and leaves)
  lz4_index_big_kernel<<<256, kBigWaves * 64, 0, s1>>>(in, in_off, in_len, out_len, status, counter, big_list,
                                                       bm_base, hdr, bitmap);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (two) {
    std::lock_guard<std::mutex> lk(two->mu);
    if ((e = hipEventRecord(two->pass1, s1)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(stream, two->pass1, 0)) != hipSuccess) return e;
  }
  lz4_exec_kernel<<<(n_msgs + kL4Waves - 1) / kL4Waves, kL4Waves * 64, 0, stream>>>(
      in, in_off, in_len, n_msgs, out, out_off, out_len, status, bm_base, hdr, bitmap);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_lz4_decode_fallback(in, in_off, in_len, n_msgs, out, out_off, out_cap, out_len, status, stream);
}

}  // namespace fsg
