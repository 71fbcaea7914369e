// snappy_decode_v4.hip -- two-pass Snappy decode for gfx950: a lane-per-message
// index pass, then a wave-per-message execution pass.
//
// Why two passes.  The lane-per-message decoders (v1-v3) give a 65,536 x
// 64 KiB batch exactly one wave per SIMD, and every piece load/store of a wave
// instruction touches 64 unrelated cache lines.  The only serial part of Snappy
// decode is finding the tag boundaries (each tag's length is in its first
// bytes); everything else -- output offsets (a prefix sum), literal bytes and
// most copy sources -- is data-parallel.  So:
//
//   pass 1, index_kernel (one LANE per message): the reference's tag walk
//     (SnappyDecompressor::DecompressAllTags, /root/reference/flare/io/snappy/
//     snappy.cc:716-787, with the writer checks of :1141-1227 / :1331-1481)
//     without touching output.  It produces the per-message status (pass 2
//     adds the copy-offset check, :1200/:1410/:1466, where every tag's output
//     position is already known) and a tag-start bitmap over the compressed
//     bytes (bit p = a tag starts at compressed offset p), 1/8 of the input
//     size.  Pure VALU + LDS ring
//     reads; each lane reads its own input once.
//
//   pass 2, exec_kernel (one WAVE per message, only status-OK messages):
//     walks the bitmap, takes up to 64 tags per group (one per lane), decodes
//     them, prefix-sums their output lengths, cuts them into <= 16-byte pieces
//     (one piece per lane) and executes the pieces in dependency rounds: a
//     piece runs once every byte it reads precedes the first unfinished piece
//     of the group.  Literal pieces and copies from before the group run in
//     round 1; text needs ~5 rounds per 64-tag group.  The 64 lanes of a
//     piece instruction touch a few neighbouring lines of one message, so the
//     loads/stores coalesce, and 4 waves per workgroup / up to 8 per SIMD hide
//     the latency.  Literals longer than 64 bytes are copied by the whole wave,
//     1 KiB per instruction.
//
// Rounds rely on the in-order processing of one wave's vector memory
// instructions: a round's loads are issued after the previous round's stores
// (same wave), so they observe them, exactly as v3's batches do.
//
// A message whose bitmap does not fit the workspace gets status kNeedFallback
// in pass 1 and is decoded serially by one lane in pass 3 (fallback_kernel).
#include "options.h"
#include "snappy_lane_decode.h"
#include "snappy_pieces.h"
#include "wave_util.h"

#include <atomic>
#include <mutex>

namespace fsg {

namespace {

// ---- pass 1 geometry (per-lane LDS ring of input chunks, as v3)
// tags per iteration of the lane walk: 32 for single-stream batches (C3
// 7.37 -> 7.33 ms), 24 for the planned large-batch walk (CM +1.8% at 32)
constexpr int kIdxTagsOne = 32, kIdxTagsPlanned = 24;
// Input bounds of the lane walk checked once per iteration instead of per
// tag (see the walk): ~5 fewer VALU per tag step.
// Pass 1b walks two 64-byte windows per step (see index_big_message).
// Pass 1b's priority on the forked path's non-huge set (A/B knob; 0 = none).
// The one-stream lane walk stores its bitmap four groups at a time (see
// index_kernel).
// The tag-start bitmap is written whole by the index passes instead of
// zeroed by the launch (see the lane walk's group stores).
// Rounds B with pattern chunks outside the common path (see exec5_message).
constexpr u32 kRingChunks = 16;              // 16-byte chunks per lane (256 B)
constexpr u32 kAhead = 7;                    // chunks prefetched per iteration
// Waves per pass-1 workgroup.  One: most resident waves for large batches
// (CM 15.1 ms vs 17.9 with four).  Four (82 KB of LDS: one workgroup per CU,
// one wave per SIMD) pins the placement and makes the pass insensitive to the
// launches before it (launch-order effect); C3 the same
// either way (7.81 vs 7.84 ms).
#ifndef FSG_IDX_WAVES
#define FSG_IDX_WAVES 1
#endif
constexpr u32 kIdxWaves = FSG_IDX_WAVES;
static_assert(kIdxWaves == 1 || kIdxWaves == 2 || kIdxWaves == 4, "tag table init");
// The one-stream lane walk of batches of short bodies (mean compressed size
// < 16 KiB, e.g. C2) runs four waves per workgroup so its bitmap allocation
// takes one device-scope atomic per workgroup instead of one per wave: C2
// 0.1354 -> 0.1276 ms; with long walks (C3) the one-wave blocks stay ahead
// (6.02 vs 6.06 ms).
#ifndef FSG_IDX_WAVES_SERIAL
#define FSG_IDX_WAVES_SERIAL 4
#endif
constexpr u32 kIdxWavesSerial = FSG_IDX_WAVES_SERIAL;
static_assert(kIdxWavesSerial == 1 || kIdxWavesSerial == 2 || kIdxWavesSerial == 4, "tag table init");

// ---- pass 1b (index_big_message, run by exec_kernel's large-message waves) geometry
constexpr u32 kBigIndexMin = 8 * 1024;       // large: compressed size above
constexpr u32 kBigIndexMax = 48 * 1024;      // clamp(4 x the batch mean, min, max)
#ifndef FSG_HUGE_KB
#define FSG_HUGE_KB 256
#endif
constexpr u32 kHugeIndexBytes = FSG_HUGE_KB * 1024;  // large ones handed out first (forked: chunked walk)
constexpr u32 kBigStageChunks = 5 * 64;      // 16-byte chunks staged per wave
constexpr u32 kBigStageBytes = 16 * kBigStageChunks;

// ---- pass 2 geometry
constexpr u32 kWavesPerBlock = 4;
#ifndef FSG_TAG_RING
#define FSG_TAG_RING 512
#endif
constexpr u32 kTagRing = FSG_TAG_RING;       // tag positions per wave (LDS)
constexpr u32 kFillWords = kTagRing / 32;    // bitmap words per fill (<= kTagRing / 2 tags)
constexpr u32 kMaxPieces = 64;
// bm_base[m] with this bit set: the message is one literal starting at the
// low bits (set by pass 1; bitmap bases stay below 2^31 words)
constexpr u32 kSingleLiteral = 0x80000000u;

__device__ u32x4 g_dummy_chunk[1];

// Diagnostic build only (-DFSG_STAMPS): per-phase cycle totals of exec_kernel,
// summed over waves, read back with fsg_debug_stamps.
#ifdef FSG_STAMPS
__device__ unsigned long long g_stamps[24];  // 0-7 exec5_message phases; 8-15 exec5_packed phases, 16 its set-up, 17-20 counts
#define STAMP(k) do { const u64 t_ = __builtin_amdgcn_s_memtime(); st_[k] += t_ - t_last_; t_last_ = t_; } while (0)
#else
#define STAMP(k) do { } while (0)
#endif


// ceil(len / step) for a pattern copy: len <= 64 and step >= 9 (pat_step of
// offsets 1..15), so the answer is 1..8 -- counted instead of divided.
__device__ __forceinline__ u32 pattern_pieces(u32 len, u32 step) {
  u32 pc = 1;
#pragma unroll
  for (u32 k = 1; k < 8; ++k) pc += len > k * step ? 1u : 0u;
  return pc;
}

}  // namespace

// ===========================================================================
// Pass 1: index + validate.  One lane per message.
// Bump allocation of `total` (this wave's sum) from *counter with one atomic
// per workgroup: every thread of the block calls it; blk is LDS scratch of
// (waves + 1) words.  Returns the wave's base.  A device-scope atomic on one
// address is serialised across the chip: one per wave cost the 1M-message
// plan pass ~0.25 ms.
__device__ __forceinline__ u32 block_bump(u32 total, u32* counter, u32* blk) {
  const u32 wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) blk[wv] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 t = 0;
    for (u32 w = 0; w < nw; ++w) {
      const u32 x = blk[w];
      blk[w] = t;
      t += x;
    }
    blk[nw] = t ? atomicAdd(counter, t) : 0u;
  }
  __syncthreads();
  const u32 r = blk[nw] + blk[wv];
  __syncthreads();
  return r;
}

// ===========================================================================
// Per-lane start of pass 1 (one message per lane, the whole wave calling):
// header (ReadUncompressedLength / Parse32WithLimit), slot check, the
// message's bitmap words (bump-allocated per wave), and the large-message
// list.  Returns the status (< 0: the lane walk follows) and sets the
// header length, expected length and bitmap base.
__device__ __forceinline__ i32 index_prologue(
    const u8* ib, u32 n_in, bool valid_msg, u32 m, u32 lane, u32 n_msgs, u32 flags,
    const u32* __restrict__ out_cap, u32* __restrict__ out_len, u32* __restrict__ bm_counter,
    u32* __restrict__ bm_base_out, u32* __restrict__ bitmap, u64 bm_capacity_words,
    u32* __restrict__ big_count, u32* __restrict__ big_list, u32 big_threshold, u32* ip,
    u32* expected, u32* bm_base_ret, u32* blk = nullptr) {
  const bool strict = flags & 2u;
  const bool validate = flags & 1u;
  i32 status = kOk;  // < 0: parsing
  if (valid_msg) {
    u32 ulen = 0;
    const int h = parse_varint_header(ib, n_in, strict, &ulen);
    if (h == 0) {
      status = kBadHeader;
      out_len[m] = 0;
    } else {
      out_len[m] = ulen;
      *expected = ulen;
      *ip = (u32)h;
      status = (!validate && ulen > out_cap[m]) ? kSlotTooSmall : -1;
    }
  }

  // ---- bitmap allocation: round_up(ceil(n_in / 32), 4) words, bump-allocated
  // per wave (order is irrelevant; bases stay 16-byte aligned)
  u32 bm_base = 0;
  if (bitmap) {
    const u32 words = status < 0 ? (((n_in + 31) >> 5) + 3) & ~3u : 0u;
    const u32 incl = wave_incl_scan(words);
    const u32 total = readlane(incl, 63);
    u32 base0 = 0;
    if (blk) {
      base0 = block_bump(total, bm_counter, blk);
    } else {
      if (lane == 0 && total) base0 = atomicAdd(bm_counter, total);
      base0 = readlane(base0, 0);
    }
    bm_base = base0 + incl - words;
    if (status < 0 && (u64)bm_base + words > bm_capacity_words) status = kNeedFallback;
    if (valid_msg) bm_base_out[m] = bm_base;
  }
  *bm_base_ret = bm_base;

  // ---- large messages go to index_big_message (a whole wave per message);
  // one lane would walk them serially for tens of milliseconds
  if (big_list) {
    // the largest ones (> kHugeIndexBytes) are listed from the end of the
    // list so both large-message passes hand them out first
    const bool big = status < 0 && n_in > big_threshold;
    const bool huge = big && n_in > kHugeIndexBytes;
    const u64 bb = __ballot(big && !huge), bh = __ballot(huge);
    const u64 below = (1ull << lane) - 1;
    if (bb) {
      u32 base1 = 0;
      if (lane == 0) base1 = atomicAdd(big_count, (u32)__builtin_popcountll(bb));
      base1 = readlane(base1, 0);
      if (big && !huge) big_list[base1 + (u32)__builtin_popcountll(bb & below)] = m;
    }
    if (bh) {
      u32 base2 = 0;
      if (lane == 0) base2 = atomicAdd(big_count + 8, (u32)__builtin_popcountll(bh));
      base2 = readlane(base2, 0);
      if (huge) big_list[n_msgs - 1 - (base2 + (u32)__builtin_popcountll(bh & below))] = m;
    }
    if (big) status = kNeedBigIndex;
  }
  return status;
}

// Size classes of the planned lane walk (see index_plan_kernel).
constexpr u32 kWalkClasses = 16;
__device__ __forceinline__ u32 walk_class(u32 n_in) {
  const u32 lg = 31u - (u32)__builtin_clz(n_in | 1u);
  return kWalkClasses - 1 - (lg < kWalkClasses - 1 ? lg : kWalkClasses - 1);
}

// Pass 1 plan (batches whose large messages are indexed on a side stream):
// the prologue alone, so pass 1b can start on the listed large messages while
// the lane walk (index_kernel<true>) runs; lanes left for the walk get
// kNeedLaneWalk.
constexpr u32 kPlanThreads = 1024;
__global__ __launch_bounds__(kPlanThreads) void index_plan_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, const u32* __restrict__ out_cap,
    u32* __restrict__ out_len, i32* __restrict__ status_out, u32 flags,
    u32* __restrict__ bm_counter, u32* __restrict__ bm_base_out,
    u32* __restrict__ bitmap, u64 bm_capacity_words, u32* __restrict__ big_count,
    u32* __restrict__ big_list, u32 big_threshold, u32* __restrict__ walk_rank,
    u32* __restrict__ walk_hist) {
  __shared__ u32 blk[kPlanThreads / 64 + 1];
  __shared__ u32 hist[kWalkClasses], hbase[kWalkClasses];
  const u32 lane = threadIdx.x & 63;
  const u32 m = blockIdx.x * kPlanThreads + threadIdx.x;
  const bool valid_msg = m < n_msgs;
  const u8* ib = valid_msg ? in + in_off[m] : in;
  const u32 n_in = valid_msg ? in_len[m] : 0u;
  u32 ip = 0, expected = 0, bm_base = 0;
  if (threadIdx.x < kWalkClasses) hist[threadIdx.x] = 0;
  __syncthreads();
  const i32 st = index_prologue(ib, n_in, valid_msg, m, lane, n_msgs, flags, out_cap, out_len,
                                bm_counter, bm_base_out, bitmap, bm_capacity_words, big_count,
                                big_list, big_threshold, &ip, &expected, &bm_base, blk);
  if (valid_msg) status_out[m] = st < 0 ? kNeedLaneWalk : st;
  if (!walk_rank) return;
  // Size classes for the lane walk (a wave's walk lasts as long as its
  // longest message): class = 15 - floor(log2(compressed size)), so the
  // largest come first; rank within the class from a per-class counter.
  const bool walk = valid_msg && st < 0;
  const u32 cls = walk_class(n_in);
  u32 mine = 0, below_mask_cnt = 0;
#pragma unroll
  for (u32 c = 0; c < kWalkClasses; ++c) {
    const u64 b = __ballot(walk && cls == c);
    const u32 cnt = (u32)__builtin_popcountll(b);
    if (lane == c) mine = cnt;
    if (cls == c) below_mask_cnt = (u32)__builtin_popcountll(b & ((1ull << lane) - 1));
  }
  // per-class ranks: this wave's base inside the block (LDS atomics), then
  // one global atomic per class per block
  u32 base = 0;
  if (lane < kWalkClasses && mine) base = atomicAdd(&hist[lane], mine);
  __syncthreads();
  if (threadIdx.x < kWalkClasses) {
    const u32 h = hist[threadIdx.x];
    hbase[threadIdx.x] = h ? atomicAdd(&walk_hist[threadIdx.x], h) : 0u;
  }
  __syncthreads();
  base = (u32)__shfl((int)base, (int)(cls & (kWalkClasses - 1)), 64);
  if (walk) walk_rank[m] = hbase[cls & (kWalkClasses - 1)] + base + below_mask_cnt;
}

// Class offsets of the size-ordered lane walk (one block): exclusive prefix
// of the per-class counts, and the number of messages to walk.
__global__ __launch_bounds__(64) void walk_offsets_kernel(u32* __restrict__ walk_hist) {
  const u32 lane = threadIdx.x;
  const u32 v = lane < kWalkClasses ? walk_hist[lane] : 0u;
  const u32 inc = wave_incl_scan(v);
  if (lane < kWalkClasses) walk_hist[kWalkClasses + lane] = inc - v;
  if (lane == 63) walk_hist[2 * kWalkClasses] = inc;
}

// Lane-walk order: perm[offset(class) + rank] = m for every message to walk.
__global__ __launch_bounds__(256) void walk_scatter_kernel(
    const u32* __restrict__ in_len, u32 n_msgs, const i32* __restrict__ status,
    const u32* __restrict__ walk_rank, const u32* __restrict__ walk_hist, u32* __restrict__ perm) {
  const u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs || status[m] != kNeedLaneWalk) return;
  perm[walk_hist[kWalkClasses + walk_class(in_len[m])] + walk_rank[m]] = m;
}

// kPlanned: index_plan_kernel ran first (statuses, bitmap bases and the
// large-message list are in place; only kNeedLaneWalk messages are walked).
template <bool kPlanned, bool kLean = false, u32 kW = kIdxWaves>
__global__ __launch_bounds__(64 * kW)
__attribute__((amdgpu_waves_per_eu(kLean ? 6 : 1))) void index_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, const u32* __restrict__ out_cap,
    u32* __restrict__ out_len, i32* __restrict__ status_out, u32 flags,
    u32* __restrict__ bm_counter, u32* __restrict__ bm_base_out,
    u32* __restrict__ bitmap, u64 bm_capacity_words, u32* __restrict__ big_count,
    u32* __restrict__ big_list, u32 big_threshold, const u32* __restrict__ walk_perm,
    const u32* __restrict__ walk_hist, u32 walk_part = 0, u32 split_class = 0) {
  // Lean geometry (the two-stream form, whose walk runs beside the previous
  // batch's execution pass in the CU resources that pass leaves free: <= 80
  // VGPRs, 12.3 KB of LDS): an 8-chunk input ring, 16 tags per iteration, 4
  // chunks prefetched, 2 bit groups (an iteration's tags lie within the 128
  // bytes the ring holds, so within 2 groups of 128 input bytes).
  constexpr int kIdxTags = kLean ? 16 : (kPlanned ? kIdxTagsPlanned : kIdxTagsOne);
  constexpr u32 kRC = kLean ? 8 : kRingChunks, kRD = kRC * 4, kAH = kLean ? 4 : kAhead;
  // Bit groups (4 words each) per lane.  The one-stream walk (C2, C3) stores
  // its groups four at a time (kSuper: 64 bytes of bitmap, 512 input bytes,
  // as four back-to-back 16-byte stores of one lane), so the L2 merges them
  // into whole lines: stored one at a time, ~18 us apart, a lane's groups
  // left the XCD's L2 between stores and every 16-byte store cost a line
  // write (0.90 GB written for C3's 0.27 GB bitmap).  Its ring
  // then holds 8 groups: the groups since the last stored super-group (<= 3)
  // plus the <= 3 an iteration spans.
  constexpr bool kSuper = !kPlanned && !kLean;
  constexpr u32 kBG = kLean ? 2 : (kSuper ? 8 : 4), kBW = 4 * kBG;
  // per wave, [dword][lane]; dword 64 = copy of dword 0; 65..68 absorb
  // unused prefetches
  // The lean form takes its LDS dynamically (idx_lean_lds_bytes(), given at
  // launch): with a compile-time size the compiler sizes the VGPR allocation
  // for the occupancy that LDS alone would allow (97 registers reserved for
  // 52 used), too many to fit beside the execution pass's waves.
  extern __shared__ u32 idx_dyn_lds[];
  __shared__ u32 ring_s[kLean ? 1 : kW][kLean ? 1 : (kRD + 5) * kWave];
  __shared__ u32 tagtab_s[kLean ? 1 : 256];
  __shared__ u32 bmr_s[kLean ? 1 : kW][kLean ? 1 : kBW * kWave];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  u32* const ring = kLean ? idx_dyn_lds + wv * (kRD + 5) * kWave : ring_s[wv];
  u32* const tagtab = kLean ? idx_dyn_lds + kW * (kRD + 5) * kWave : tagtab_s;
  u32* const bmr = kLean ? idx_dyn_lds + kW * (kRD + 5) * kWave + 256 + wv * kBW * kWave : bmr_s[wv];

  const u32 lane = threadIdx.x & 63;
  // Tag table (the role of char_table, snappy.cc:516-549): per tag byte c,
  // bits 0-4 the right shift of 0xffffffff that masks the nb extra bytes
  // ((32 - 8 nb) & 31: a shift uses the low 5 bits of its operand), 5 long
  // literal, 8-15 advance without a long literal's length, 16-23 length
  // (short literal / copies).
#pragma unroll
  for (u32 q = 0; q < 4 / kW; ++q) {
    const u32 c = threadIdx.x * (4 / kW) + q, type = c & 3, l0 = (c >> 2) + 1;
    u32 nb, len, lit = 0, ll = 0;
    if (type == 0) {
      lit = 1;
      nb = l0 > 60 ? l0 - 60 : 0;
      ll = nb ? 1 : 0;
      len = nb ? 0 : l0;
    } else if (type == 1) {
      nb = 1;
      len = 4 + ((c >> 2) & 7);
    } else {
      nb = type == 2 ? 2 : 4;
      len = l0;
    }
    const u32 adv = 1 + nb + (lit && !ll ? len : 0);
    tagtab[c] = ((32 - 8 * nb) & 31) | (ll << 5) | (adv << 8) | (len << 16);
  }
  __syncthreads();
  // planned with a walk order: lane g walks message walk_perm[g], the
  // messages grouped by size class so a wave's lanes finish together
  const u32 gid = blockIdx.x * blockDim.x + threadIdx.x;
  // (walk_part 1 / 2: only the walk order's positions below / from the
  // first one of class split_class -- the larger / the smaller bodies)
  const bool ordered = kPlanned && walk_perm;
  const u32 n_walk = ordered ? walk_hist[2 * kWalkClasses] : n_msgs;
  // (split_class bits 8-15, when set: the first class another pass takes --
  // positions from its first one are not walked here; no pass sets it now)
  const u32 tcls = split_class >> 8;
  const u32 split = walk_part ? walk_hist[kWalkClasses + (split_class & 0xffu)] : 0u;
  const u32 t_hi = tcls ? walk_hist[kWalkClasses + tcls] : n_walk;
  const u32 w_lo = walk_part == 2 ? split : 0u, w_hi = walk_part == 1 ? split : t_hi;
  const bool valid_msg = ordered ? gid < w_hi - w_lo : gid < n_walk;
  const u32 m = ordered ? (valid_msg ? walk_perm[w_lo + gid] : 0u) : gid;

  const u8* ib = valid_msg ? in + in_off[m] : in;
  const u32 n_in = valid_msg ? in_len[m] : 0u;
  u32 expected = 0, ip = 0, bm_base = 0;
  i32 status = kOk;
  if (!kPlanned) {
    __shared__ u32 blk_s[kW + 1];
    status = index_prologue(ib, n_in, valid_msg, m, lane, n_msgs, flags, out_cap, out_len,
                            bm_counter, bm_base_out, bitmap, bm_capacity_words, big_count, big_list,
                            big_threshold, &ip, &expected, &bm_base, kW > 1 ? blk_s : nullptr);
  } else if (valid_msg && status_out[m] == kNeedLaneWalk) {
    u32 ulen = 0;
    ip = (u32)parse_varint_header(ib, n_in, flags & 2u, &ulen);  // valid: checked by the plan
    expected = ulen;
    bm_base = bitmap ? bm_base_out[m] : 0u;
    status = -1;
  }
  const bool walked = status < 0;  // (planned: the other lanes' statuses stand)
  u32* bm = bitmap ? bitmap + bm_base : nullptr;

  const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
  const u8* abase = ib - ibal;
  const u32 last_chunk = n_in ? (ibal + n_in - 1) >> 4 : 0u;

  u32 wend = 0, iend = 0;
  auto ring_write = [&](u32 k, u32x4 v, bool live) {
    const u32 d = live ? (k & (kRC - 1)) * 4 : kRD + 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) ring[(d + i) * kWave + lane] = v[i];
    ring[(d == 0 ? kRD : kRD + 1) * kWave + lane] = v[0];
  };
  // Single-literal message (random bodies: the encoder emits one literal when
  // it finds no match): its first tag is a literal whose bytes end the input.
  // Decided here from the first chunks, once per message; pass 2 copies such
  // a message without walking the bitmap (bm_base = kSingleLiteral | source).
  u32 single_src = 0;
  if (status < 0) {
    u32x4 c0[4];
#pragma unroll
    for (u32 c = 0; c < 4; ++c) {
      const u32 k = c <= last_chunk ? c : last_chunk;
      c0[c] = *reinterpret_cast<const u32x4*>(abase + 16 * k);
    }
#pragma unroll
    for (u32 c = 0; c < 4; ++c) ring_write(c, c0[c], c <= last_chunk);
    wend = iend = (last_chunk + 1 < 4) ? last_chunk + 1 : 4;
    // tag byte at ip (header <= 5 bytes) and its <= 4 length bytes lie in the
    // first 32 bytes of the aligned chunks (ibal + 9 < 32)
    const u32 P = ip + ibal;
    const u32 w[8] = {c0[0][0], c0[0][1], c0[0][2], c0[0][3], c0[1][0], c0[1][1], c0[1][2], c0[1][3]};
    const u32 d = P >> 2;
    const u32 w0 = mux8(w, d), w1 = mux8(w, d + 1), w2 = d + 2 < 8 ? mux8(w, d + 2) : 0u;
    const u32 t0 = alignbyte(w1, w0, P & 3);
    const u32 ext = alignbyte(alignbyte(w2, w1, P & 3), t0, 1);
    const u32 c = t0 & 0xffu;
    const u32 l0 = (c >> 2) + 1;
    const u32 nbl = l0 > 60 ? l0 - 60 : 0u;
    const u32 val = ext & (0xffffffffu >> ((32 - 8 * nbl) & 31));
    const u32 len = nbl ? val + 1u : l0;
    const u64 end = (u64)ip + 1 + nbl + len;
    if ((c & 3) == 0 && end == n_in && ip < n_in && len == expected) single_src = ip + 1 + nbl;
  }

  u32 op = 0;
  // Tag-start bits go to a per-lane LDS ring of 4 groups of 128 input bytes
  // (group g in slot g & 3, [word][lane]) by a fire-and-forget ds_or; a group
  // is stored to the bitmap (if it holds bits) once the walk has left it.  One
  // iteration covers at most 3 groups (the input ring spans 256 bytes, and a
  // long literal that leaves it ends the lane's iteration).
#pragma unroll
  for (u32 q = 0; q < kBW; ++q) bmr[q * kWave + lane] = 0;
  u32 fg = 0;  // lowest group that may still hold unstored bits

  u32x4 g[kAH];
#pragma unroll
  for (u32 c = 0; c < kAH; ++c) g[c] = u32x4{0, 0, 0, 0};
  u32 gk_w = 0, gn_w = 0;

  __builtin_amdgcn_s_waitcnt(0);
  bool more = __any(status < 0);
  while (more) {
    // ---------- parse up to kIdxTags tags from the ring
    // a tag at ip is parsed this iteration iff ip < lim: still parsing, before
    // the end of input, and its 5 bytes are in the ring
    u32 lim = 0;
    if (status < 0) {
      const u32 ring_end = 16 * wend >= 4 + ibal ? 16 * wend - 4 - ibal : 0u;
      lim = (wend > last_chunk || ring_end > n_in) ? n_in : ring_end;
    }
    // Software-pipelined: tag j+1's ring read is issued (in program order)
    // before tag j's checks and its ds_or, so the LDS latency overlaps them;
    // the compiler does not move LDS reads above the atomic.
    auto ring_read = [&](u32 at, u32& lo, u32& hi) {
      const u32 P = at + ibal;
      const u32 dw = (P >> 2) & (kRD - 1);
      lo = ring[dw * kWave + lane];
      hi = ring[(dw + 1) * kWave + lane];
    };
    u32 lo, hi;
    ring_read(ip, lo, hi);
    const u32 op_it = op;
    u32 lmax = 0;  // the largest long-literal length looked at this iteration
#pragma unroll
    for (int j = 0; j < kIdxTags; ++j) {
      const u32 bsh = (ip + ibal) & 3;
      const u32 t0 = alignbyte(hi, lo, bsh);          // bytes ip..ip+3
      const u32 ext = alignbyte(hi >> (8 * bsh), t0, 1);  // bytes ip+1..ip+4
      // tag decode through the tag table (DecompressAllTags :716-787): the
      // 0..4 bytes after the tag byte are a literal's length or a copy's
      // offset, masked to their count nb; selects, no exec-mask branches.
      const u32 c = t0 & 0xffu;
      const u32 e = tagtab[c];
      const u32 val = ext & (0xffffffffu >> (e & 31u));
      // a long literal's length (uint32 wrap: 0xffffffff+1 == 0, as the
      // reference's uint32 sum), else the table's (0 for long literals); masks,
      // not a select, so the compiler keeps the unrolled walk branch-free
      const u32 llmask = 0u - ((e >> 5) & 1u);
      const u32 lpart = (val + 1u) & llmask;
      const u32 len = lpart + ((e >> 16) & 0xffu);
      // The walk advances over every tag below lim whether or not it passed
      // its checks, so the checks stay off the ip -> ip dependency chain.
      // After the first failing tag the status is final (kCorrupt): what the
      // walk reads from there on only sets bits in the LDS ring, which are
      // never stored for a corrupt message, and ring indices are masked.
      const bool look = ip < lim;
      const u32 adv = (e >> 8) & 0xffu;  // tag byte + extra bytes (+ a short literal's bytes)
      const u32 step = adv + lpart;
      const u32 ip_next = look ? ip + step : ip;
      if (j + 1 < kIdxTags) ring_read(ip_next, lo, hi);
      // Bounds are checked once per iteration (below), not per tag: a tag
      // whose bytes run past the input leaves ip_next > n_in (no u32 wrap
      // while lpart <= n_in, since ip <= n_in < 2^31 and adv <= 65), after
      // which no later tag of the iteration is looked at (ip >= lim); a
      // larger lpart (a huge or wrapping 4-byte literal length) shows in lmax.
      // The bit and length of such a tag land only in state that a corrupt
      // message never stores.
      lmax = look && lpart > lmax ? lpart : lmax;
      atomicOr(&bmr[((ip >> 5) & (kBW - 1)) * kWave + lane], look ? 1u << (ip & 31) : 0u);
      op += look ? len : 0u;
      ip = ip_next;
    }
    if (status < 0 && (ip > n_in || lmax > n_in)) status = kCorrupt;
    // writer space (:1166, :1400), checked once per iteration: op only grows,
    // and one iteration cannot wrap it (accepted literals fit the input)
    if (status < 0 && (op > expected || op < op_it)) status = kCorrupt;
    // end of input between tags (RefillTag eof): the result, snappy.cc:858-868
    if (status < 0 && ip == n_in) status = op == expected ? kOk : kCorrupt;

    // ---------- store the bit groups the walk has left
    // The bitmap is not zeroed by the launch: every group of a message the
    // execution pass will read is stored here, zero groups included (a
    // single-literal message's bitmap is never read), and the groups a long
    // literal jumps over are stored as zeros; at the end the walk's
    // remaining groups up to the allocation (ceil(n_in / 128)).
    if (bm && !single_src) {
      const u32 ngroups = (((n_in + 31) >> 5) + 3) >> 2;
      const u32 cur0 = status < 0 ? ip >> 7 : (status == kOk ? ngroups : 0u);
      // super-group stores: while walking, only the whole super-groups below
      // the current one; once the walk is over, everything up to the end
      const u32 cur = kSuper && status < 0 ? cur0 & ~3u : cur0;
      if constexpr (kSuper) {
        // fg is a multiple of 4 until the walk ends: the super-group at fg
        // is one half of the 8-slot ring; past fg + 4 only after a long
        // literal (or at the end)
        auto super_store = [&](u32 g0) {
          const u32 sl = (g0 & 4u) * 4;
          u32x4 v[4];
#pragma unroll
          for (u32 q = 0; q < 16; ++q) v[q >> 2][q & 3] = bmr[(sl + q) * kWave + lane];
#pragma unroll
          for (u32 k = 0; k < 4; ++k)
            if (g0 + k < cur) *reinterpret_cast<u32x4*>(bm + 4 * (g0 + k)) = v[k];
#pragma unroll
          for (u32 q = 0; q < 16; ++q) bmr[(sl + q) * kWave + lane] = 0;
        };
        if (cur > fg) {
          super_store(fg);
          if (cur > fg + 4) {
            super_store(fg + 4);
            for (u32 gi = fg + 8; gi < cur; ++gi) *reinterpret_cast<u32x4*>(bm + 4 * gi) = u32x4{0, 0, 0, 0};
          }
          fg = cur;
        }
      } else {
#pragma unroll
        for (u32 k = 0; k < kBG; ++k) {
          const u32 gi = fg + k;
          if (gi < cur) {
            const u32 sl = (gi & (kBG - 1)) * 4;
            u32x4 v;
#pragma unroll
            for (u32 q = 0; q < 4; ++q) v[q] = bmr[(sl + q) * kWave + lane];
            *reinterpret_cast<u32x4*>(bm + 4 * gi) = v;
#pragma unroll
            for (u32 q = 0; q < 4; ++q) bmr[(sl + q) * kWave + lane] = 0;
          }
        }
        for (u32 gi = fg + kBG; gi < cur; ++gi) *reinterpret_cast<u32x4*>(bm + 4 * gi) = u32x4{0, 0, 0, 0};
        fg = cur > fg ? cur : fg;
      }
    }

    // ---------- land the chunks loaded last iteration
#pragma unroll
    for (u32 c = 0; c < kAH; ++c) ring_write(gk_w + c, g[c], c < gn_w);
    wend = gn_w ? gk_w + gn_w : wend;

    // ---------- prefetch from the parse position
    {
      const u32 P = ip + ibal;
      const u32 pc = P >> 4;
      const u32 base = pc >= iend ? pc : iend;  // a long literal jumped past the ring: restart
      u32 cnt = 0;
#pragma unroll
      for (u32 c = 0; c < kAH; ++c) {
        const u32 k = base + c;
        const bool ok = status < 0 && k <= last_chunk && k <= pc + (kRC - 1);
        cnt += ok ? 1u : 0u;
        const u32 kk = k <= last_chunk ? k : last_chunk;
        g[c] = *reinterpret_cast<const u32x4*>(n_in ? abase + 16 * kk
                                                    : reinterpret_cast<const u8*>(g_dummy_chunk));
      }
      iend = cnt ? base + cnt : iend;
      gk_w = base;
      gn_w = cnt;
    }
    more = __any(status < 0);
  }
  const bool mine = valid_msg && (!kPlanned || walked);
  if (mine) status_out[m] = status;
  if (mine && bitmap && status == kOk && single_src) bm_base_out[m] = kSingleLiteral | single_src;
}

// ===========================================================================
// Pass 1b: index + validate one LARGE message per wave (compressed size >
// the launch's big_threshold, listed by pass 1).  One lane walking 100K+ tags serially
// is the tail of a mixed batch; here the walk advances a 64-byte window
// [wb, wb+64) at a time: every lane decodes the tag that WOULD start at
// wb + lane (length, advance, offset, local validity -- the same branch-free
// decode and checks as pass 1), the real tag starts in the window (the chain
// from the current position) are found by pointer doubling over the lanes'
// successor pointers (5 rounds of shuffles), their output positions by a
// prefix sum, and the position-dependent checks run on all of them at once.
// Input is staged into LDS 5 KiB at a time.
// ===========================================================================
// Indexes message m (listed by pass 1) with the calling wave: writes its
// bitmap bits and returns its final status.  `st` is the wave's LDS stage
// (kBigStageBytes + 16 bytes).
__device__ __forceinline__ i32 index_big_message(
    u32 m, const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, const u32* __restrict__ out_len, bool strict,
    const u32* __restrict__ bm_base, u32* __restrict__ bitmap, u32* st, u32 lane, u8* ob,
    bool& seg) {
  const u8* ib = in + in_off[m];
  const u32 n_in = in_len[m];
  const u32 expected = out_len[m];
  u32 ulen = 0;
  u32 ip = (u32)parse_varint_header(ib, n_in, strict, &ulen);  // pass 1 accepted it
  u32 op = 0;
  i32 status = -1;
  u32* bm = bitmap + bm_base[m];
  {  // the launch does not zero the bitmap: this message's words first
    const u32 words = (((n_in + 31) >> 5) + 3) & ~3u;
    for (u32 wd = 4 * lane; wd < words; wd += 256) *reinterpret_cast<u32x4*>(bm + wd) = u32x4{0, 0, 0, 0};
  }
  const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
  const u8* abase = ib - ibal;
  const u32 last_chunk = (ibal + n_in - 1) >> 4;
  int spos = -1;  // message position of stage byte 0 (-1: nothing staged)
  u32 send = 0;   // positions [spos, send) are valid in the stage

  // Two 64-byte windows per step, A = [wb, wb + 64) and B = [wb + 64,
  // wb + 128), each lane decoding one candidate tag in each: the pointer
  // doubling does not depend on where the chain enters a window, so both
  // windows' doublings run interleaved (one latency chain of shuffles per
  // 128 bytes instead of per 64), and B's chain is read at A's exit.
  while (status < 0) {
    if (ip >= n_in) {  // end of input between tags (snappy.cc:858-868)
      status = (ip == n_in && op == expected) ? kOk : kCorrupt;
      break;
    }
    const u32 wb = ip & ~31u;
    // ---------- stage input covering [wb, wb + 128 + 8)
    if (spos < 0 || wb < (u32)spos || wb + 136 > send) {
      const u32 c0 = (wb + ibal) >> 4;
      u32x4 x[kBigStageChunks / 64];
#pragma unroll
      for (u32 r = 0; r < kBigStageChunks / 64; ++r) {
        u32 k = c0 + r * 64 + lane;
        k = k <= last_chunk ? k : last_chunk;
        x[r] = *reinterpret_cast<const u32x4*>(abase + 16 * k);
      }
      wave_lds_fence();  // previous window's stage reads are done
#pragma unroll
      for (u32 r = 0; r < kBigStageChunks / 64; ++r)
        *reinterpret_cast<u32x4*>(st + 4 * (r * 64 + lane)) = x[r];
      wave_lds_fence();
      spos = (int)(16 * c0) - (int)ibal;
      send = (u32)spos + kBigStageBytes - 8;
    }
    // ---------- every lane decodes the tag that would start at wb + lane
    // (A) and at wb + 64 + lane (B): length, offset, next position, local
    // validity (tag and literal bytes present), successor lane in the window
    struct Cand {
      u32 len, coff, nxt, J;
      bool lit, bad_local;
    };
    auto decode = [&](u32 p) {
      const u32 s = p - (u32)spos;
      const u32 dw = s >> 2, bsh = s & 3;
      const u32 lo = st[dw], hi = st[dw + 1];
      const u32 t0 = alignbyte(hi, lo, bsh);
      const u32 b4 = (hi >> (8 * bsh)) & 0xffu;
      const u32 c = t0 & 0xffu;
      const u32 type = c & 3;
      Cand d;
      d.lit = type == 0;
      const u32 l0 = (c >> 2) + 1;
      const bool longlit = d.lit & (l0 >= 61);
      const u32 nb = d.lit ? (longlit ? l0 - 60 : 0u) : (1u << (type - 1));
      const u32 ext = (b4 << 24) | (t0 >> 8);
      const u32 val = nb >= 4 ? ext : ext & ((1u << (8 * nb)) - 1u);
      d.len = d.lit ? (longlit ? val + 1u : l0) : (type == 1 ? 4 + ((c >> 2) & 7) : l0);
      d.coff = type == 1 ? (((c >> 5) << 8) | val) : val;
      const u32 avail = n_in - p - 1;
      d.bad_local = (p >= n_in) | (avail < nb) | (d.lit & (avail - nb < d.len));
      const u32 adv = 1 + nb + (d.lit ? d.len : 0u);
      d.nxt = p + adv;
      d.J = (d.bad_local || adv >= 64 - lane || d.nxt >= n_in) ? 64u : lane + adv;
      return d;
    };
    const u32 pA = wb + lane, pB = wb + 64 + lane;
    const Cand A = decode(pA), B = decode(pB);
    // ---------- pointer doubling in both windows (see the one-window form)
    u64 MA = 1ull << lane, MB = 1ull << lane;
    u32 JA = A.J, JB = B.J;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const u32 sA = JA < 64 ? JA : lane, sB = JB < 64 ? JB : lane;
      const u64 MAj = ((u64)(u32)__shfl((int)(u32)(MA >> 32), (int)sA, 64) << 32) |
                      (u32)__shfl((int)(u32)MA, (int)sA, 64);
      const u64 MBj = ((u64)(u32)__shfl((int)(u32)(MB >> 32), (int)sB, 64) << 32) |
                      (u32)__shfl((int)(u32)MB, (int)sB, 64);
      const u32 JAj = (u32)__shfl((int)JA, (int)sA, 64);
      const u32 JBj = (u32)__shfl((int)JB, (int)sB, 64);
      if (JA < 64) {
        MA |= MAj;
        JA = JAj;
      }
      if (JB < 64) {
        MB |= MBj;
        JB = JBj;
      }
    }
    const u32 firstA = ip - wb;
    const u64 SA = ((u64)readlane((u32)(MA >> 32), firstA) << 32) | readlane((u32)MA, firstA);
    const u32 lastA = 63u - (u32)__builtin_clzll(SA);
    const u32 ipA = readlane(A.nxt, lastA);  // where the chain leaves A
    // B is entered when A's last tag is good and ends inside B
    const bool enterB = ipA >= wb + 64 && ipA < wb + 128 && ipA < n_in;
    const u32 firstB = enterB ? ipA - wb - 64 : 0u;
    const u64 SB = enterB ? ((u64)readlane((u32)(MB >> 32), firstB) << 32) | readlane((u32)MB, firstB) : 0ull;
    const bool inA = (SA >> lane) & 1ull, inB = (SB >> lane) & 1ull;
    // output positions: A's chain from op, then B's
    const u32 lvA = inA ? A.len : 0u;
    const u32 incA = dpp_incl_scan(lvA);
    const u32 t_opA = op + incA - lvA;
    const u32 opA = op + readlane(incA, 63);
    const u32 lvB = inB ? B.len : 0u;
    const u32 incB = dpp_incl_scan(lvB);
    const u32 t_opB = opA + incB - lvB;
    // writer space and copy offset checks (:761, :1166, :1200, :1410, :1466)
    const bool badA = inA && (A.bad_local || expected - t_opA < A.len || (!A.lit && A.coff - 1u >= t_opA));
    const bool badB = inB && (B.bad_local || expected - t_opB < B.len || (!B.lit && B.coff - 1u >= t_opB));
    if (__any(badA || badB)) {
      status = kCorrupt;
      break;
    }
    // 64 KiB output segments (see the one-window form)
    if (seg) {
      const bool spanA = inA && A.len > 0 && ((t_opA ^ (t_opA + A.len - 1)) >> 16) != 0;
      const bool spanB = inB && B.len > 0 && ((t_opB ^ (t_opB + B.len - 1)) >> 16) != 0;
      const bool xA = inA && !A.lit && t_opA - A.coff < (t_opA & ~0xffffu);
      const bool xB = inB && !B.lit && t_opB - B.coff < (t_opB & ~0xffffu);
      if (__any(spanA || spanB || xA || xB)) seg = false;
      if (seg && inA && t_opA != 0 && (t_opA & 0xffffu) == 0 && t_opA + 4 <= expected)
        __builtin_memcpy(ob + t_opA, &pA, 4);
      if (seg && inB && t_opB != 0 && (t_opB & 0xffffu) == 0 && t_opB + 4 <= expected)
        __builtin_memcpy(ob + t_opB, &pB, 4);
    }
    if (SB) {
      const u32 lastB = 63u - (u32)__builtin_clzll(SB);
      ip = readlane(B.nxt, lastB);
      op = opA + readlane(incB, 63);
    } else {
      ip = ipA;
      op = opA;
    }
    const u64 Sw = lane < 2 ? SA : SB;
    const u32 wbits = (lane & 1) == 0 ? (u32)Sw : (u32)(Sw >> 32);
    if (lane < 4 && wbits) bm[(wb >> 5) + lane] = wbits;
  }
  return status;
}

// Pass 1b launch: one wave per listed large message (taken from a counter,
// huge ones first).  Each finished message goes to pass 2's work lists: its
// 64 KiB segments (seg_list: m | k << 32 | last << 63) when the stream
// allows them, else the whole message (whole_list).
__global__ __launch_bounds__(4 * 64) void index_big_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, const u32* __restrict__ out_len, u32 flags,
    i32* __restrict__ status_out, const u32* __restrict__ bm_base,
    u32* __restrict__ bitmap, const u32* __restrict__ big_count,
    const u32* __restrict__ big_list, u32* __restrict__ big_next, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, u64* __restrict__ seg_list, u32* __restrict__ seg_count,
    u32* __restrict__ whole_list, u32* __restrict__ whole_count, u32 mode) {
  __shared__ u32 stage_s[4][kBigStageBytes / 4 + 4];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const bool strict = flags & 2u;
  // mode 0: every listed message, the huge ones (> kHugeIndexBytes) first;
  // 1: the huge ones only; 2: the others only (the forked path walks the two
  // sets on two streams, so the others' execution starts without waiting for
  // the longest walks)
  const u32 n_huge = mode == 2 ? 0u : big_count[8];
  const u32 count = (mode == 1 ? 0u : big_count[0]) + n_huge;
  if (count == 0) return;  // uniform batches: no atomics on the shared counter
  for (;;) {  // all-lane atomic: lane 0 adds 1, lane 0's result is the index
    const u32 got = atomicAdd(big_next, lane == 0 ? 1u : 0u);
    const u32 idx = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (idx >= count) break;
    const u32 m = idx < n_huge ? big_list[n_msgs - 1 - idx] : big_list[idx - n_huge];
    bool seg = true;
    const i32 st = index_big_message(m, in, in_off, in_len, out_len, strict, bm_base, bitmap,
                                     stage_s[wv], lane, out + out_off[m], seg);
    if (lane == 0) status_out[m] = st;
    if (st != kOk) continue;
    const u32 expected = out_len[m];
    u32 nseg = 0;  // > 1: run as segments
    if (seg && expected > 65536u) {
      nseg = (expected + 65535u) >> 16;
      if (expected - ((nseg - 1) << 16) < 4) --nseg;  // the tail joins the previous segment
    }
    bool whole = nseg < 2;
    if (!whole) {
      u32 b = 0;
      if (lane == 0) b = atomicAdd(seg_count, nseg);
      b = readlane(b, 0);
      for (u32 k = lane; k < nseg; k += 64) {
        const u64 e = b + k < n_msgs
            ? ((u64)m | ((u64)k << 32) | ((u64)(k == nseg - 1) << 63))
            : 0xffffffffull;  // past the list: dropped, the message runs whole
        if (b + k < n_msgs) seg_list[b + k] = e;
      }
      if (b + nseg > n_msgs) {
        // partly listed: the listed entries become holes
        for (u32 k = lane; b + k < n_msgs && k < nseg; k += 64) seg_list[b + k] = 0xffffffffull;
        whole = true;
      }
    }
    if (whole) {
      u32 b = 0;
      if (lane == 0) b = atomicAdd(whole_count, 1u);
      b = readlane(b, 0);
      if (lane == 0) whole_list[b] = m;
    }
  }
}

// ===========================================================================
// Pass 1b, chunked (the huge messages of the forked path): one wave walking a
// ~520 KB body serially was CM's longest chain (5.6 ms).  The body's
// compressed bytes are cut into kChunkBytes chunks, walked in parallel:
//
//   spec   one wave per chunk walks from the chunk's first byte AS IF a tag
//          started there (chunk 0: from the header's end, exact) and writes
//          that chain's tag-start bits for the chunk, its exit (the first chain
//          position past the chunk), the output length of its tags and whether
//          it reached a tag that cannot be decoded.
//   fixup  one wave per message, chunk by chunk: the true chain enters chunk k
//          at chunk k-1's true exit; it is followed (pointer doubling, a window
//          at a time) until it reaches a tag start of the speculative chain --
//          from there both chains are one chain, so chunk k's speculative bits,
//          exit and length hold (text meets within ~10 bytes).
//          The bits before the meeting point are rewritten, the chunk's true
//          output length corrected, and the chunks' output bases summed.  A
//          chunk the true chain crosses without meeting is rewritten whole.
//   check  one wave per chunk, with the true bits and base: the writer checks
//          (snappy.cc:1166, :1200, :1400, :1410, :1466) and the 64 KiB segment
//          rules of index_big_message.
//   final  one wave per message: status and pass 2's work lists.
// ===========================================================================
constexpr u32 kChunkBytes = 32 * 1024;  // a multiple of 512: chunks own whole bitmap words
struct ChunkRec {
  u32 m, k, exit, bad, len, base, flags, nchunks;
};
constexpr u32 kChunkBad = 1, kChunkNoSeg = 2;

namespace {
// The candidate tag at message position p (stage st holds positions
// [spos, spos + kBigStageBytes)): pass 1b's branch-free decode.
struct Cand2 {
  u32 len, coff, nxt, J;
  bool lit, bad_local;
};
__device__ __forceinline__ Cand2 decode_cand(const u32* st, int spos, u32 p, u32 n_in, u32 lane) {
  const u32 s = p - (u32)spos;
  const u32 dw = s >> 2, bsh = s & 3;
  const u32 lo = st[dw], hi = st[dw + 1];
  const u32 t0 = alignbyte(hi, lo, bsh);
  const u32 b4 = (hi >> (8 * bsh)) & 0xffu;
  const u32 c = t0 & 0xffu;
  const u32 type = c & 3;
  Cand2 d;
  d.lit = type == 0;
  const u32 l0 = (c >> 2) + 1;
  const bool longlit = d.lit & (l0 >= 61);
  const u32 nb = d.lit ? (longlit ? l0 - 60 : 0u) : (1u << (type - 1));
  const u32 ext = (b4 << 24) | (t0 >> 8);
  const u32 val = nb >= 4 ? ext : ext & ((1u << (8 * nb)) - 1u);
  d.len = d.lit ? (longlit ? val + 1u : l0) : (type == 1 ? 4 + ((c >> 2) & 7) : l0);
  d.coff = type == 1 ? (((c >> 5) << 8) | val) : val;
  const u32 avail = n_in - p - 1;
  d.bad_local = (p >= n_in) | (avail < nb) | (d.lit & (avail - nb < d.len));
  const u32 adv = 1 + nb + (d.lit ? d.len : 0u);
  d.nxt = p + adv;
  d.J = (d.bad_local || adv >= 64 - lane || d.nxt >= n_in) ? 64u : lane + adv;
  return d;
}

// Stage input covering [wb, wb + 72) for the window at wb (kept across calls).
struct Stage {
  int spos = -1;
  u32 send = 0;
};
__device__ __forceinline__ void stage_for(Stage& sg, u32* st, const u8* abase, u32 ibal, u32 last_chunk, u32 wb,
                                          u32 lane) {
  if (sg.spos >= 0 && wb >= (u32)sg.spos && wb + 72 <= sg.send) return;
  const u32 c0 = (wb + ibal) >> 4;
  u32x4 x[kBigStageChunks / 64];
#pragma unroll
  for (u32 r = 0; r < kBigStageChunks / 64; ++r) {
    u32 k = c0 + r * 64 + lane;
    k = k <= last_chunk ? k : last_chunk;
    x[r] = *reinterpret_cast<const u32x4*>(abase + 16 * k);
  }
  wave_lds_fence();
#pragma unroll
  for (u32 r = 0; r < kBigStageChunks / 64; ++r) *reinterpret_cast<u32x4*>(st + 4 * (r * 64 + lane)) = x[r];
  wave_lds_fence();
  sg.spos = (int)(16 * c0) - (int)ibal;
  sg.send = (u32)sg.spos + kBigStageBytes - 8;
}

// The chain from position `first` inside the window at wb (pointer doubling
// over the lanes' successors, as index_big_message): bit j = a tag starts at
// wb + j on that chain.
__device__ __forceinline__ u64 window_chain(const Cand2& d, u32 first, u32 lane) {
  u32 J = d.J;
  u64 M = 1ull << lane;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const u32 src = J < 64 ? J : lane;
    const u64 Mj = ((u64)(u32)__shfl((int)(u32)(M >> 32), (int)src, 64) << 32) | (u32)__shfl((int)(u32)M, (int)src, 64);
    const u32 Jj = (u32)__shfl((int)J, (int)src, 64);
    if (J < 64) {
      M |= Mj;
      J = Jj;
    }
  }
  return ((u64)readlane((u32)(M >> 32), first) << 32) | readlane((u32)M, first);
}

__device__ __forceinline__ u64 bm_window(const u32* bm, u32 wb) {
  return ((u64)bm[(wb >> 5) + 1] << 32) | bm[wb >> 5];
}
// positions [lo, hi) of the window at wb as a mask
__device__ __forceinline__ u64 range_mask(u32 wb, u32 lo, u32 hi) {
  const u32 a = lo > wb ? lo - wb : 0u, b = hi > wb ? (hi - wb < 64 ? hi - wb : 64u) : 0u;
  if (a >= b) return 0ull;
  const u64 up = b >= 64 ? ~0ull : ((1ull << b) - 1);
  return up & ~((1ull << a) - 1);
}
}  // namespace

// The chunk records of the huge messages (set 1 of the forked path): one
// thread per huge message (listed from the end of big_list).
__global__ void chunk_list_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                  const u32* __restrict__ in_len, const u32* __restrict__ big_count,
                                  const u32* __restrict__ big_list, u32 n_msgs, u32 flags,
                                  u32* __restrict__ chunk_count, ChunkRec* __restrict__ recs,
                                  u32* __restrict__ first_rec, u32 max_recs) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 n_huge = big_count[8];
  if (i >= n_huge) return;
  const u32 m = big_list[n_msgs - 1 - i];
  const u32 n_in = in_len[m];
  const u32 K = (n_in + kChunkBytes - 1) / kChunkBytes;
  const u32 b = atomicAdd(chunk_count, K);
  first_rec[i] = b + K <= max_recs ? b : 0xffffffffu;
  if (b + K > max_recs) return;
  for (u32 k = 0; k < K; ++k) {
    ChunkRec r{};
    r.m = m;
    r.k = k;
    r.nchunks = K;
    recs[b + k] = r;
  }
  (void)in;
  (void)in_off;
  (void)flags;
}

// spec: one wave per chunk record (work counter).
__global__ __launch_bounds__(4 * 64) void chunk_spec_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u32 flags,
    const u32* __restrict__ bm_base, u32* __restrict__ bitmap, const u32* __restrict__ chunk_count,
    ChunkRec* __restrict__ recs, u32* __restrict__ next, u32 max_recs) {
  __shared__ u32 stage_s[4][kBigStageBytes / 4 + 4];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 cnt = *chunk_count < max_recs ? *chunk_count : max_recs;
  u32* st = stage_s[wv];
  for (;;) {
    const u32 got = atomicAdd(next, lane == 0 ? 1u : 0u);
    const u32 idx = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (idx >= cnt) break;
    const ChunkRec r = recs[idx];
    const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)r.m);
    const u8* ib = in + in_off[m];
    const u32 n_in = in_len[m];
    const u32 cs = r.k * kChunkBytes;
    const u32 ce = cs + kChunkBytes < n_in ? cs + kChunkBytes : n_in;
    u32* bm = bitmap + bm_base[m];
    // this chunk's bitmap words (the last chunk: up to the allocation's end)
    {
      const u32 w0 = cs >> 5;
      const u32 w1 = ce == n_in ? ((((n_in + 31) >> 5) + 3) & ~3u) : ce >> 5;
      for (u32 wd = w0 + lane; wd < w1; wd += 64) bm[wd] = 0u;
    }
    u32 ip = cs;
    if (r.k == 0) {
      u32 ulen = 0;
      ip = (u32)parse_varint_header(ib, n_in, flags & 2u, &ulen);
    }
    const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
    const u8* abase = ib - ibal;
    const u32 last_chunk = (ibal + n_in - 1) >> 4;
    Stage sg;
    u32 op = 0, bad = 0;
    wave_lds_fence();
    for (u32 guard = 0; guard < kChunkBytes + 64; ++guard) {
      if (ip >= ce || ip >= n_in) break;
      const u32 wb = ip & ~31u;
      stage_for(sg, st, abase, ibal, last_chunk, wb, lane);
      const Cand2 d = decode_cand(st, sg.spos, wb + lane, n_in, lane);
      const u64 S = window_chain(d, ip - wb, lane);
      const u64 Sin = S & range_mask(wb, cs, ce);
      const bool in_s = (Sin >> lane) & 1ull;
      if (__any(in_s && d.bad_local)) {
        bad = 1;
        // the chain stops at its first undecodable tag
        const u64 B = __ballot(in_s && d.bad_local);
        ip = wb + (u32)__builtin_ctzll(B);
        const u64 keep = Sin & ((1ull << (ip - wb)) | ((1ull << (ip - wb)) - 1));
        if (lane < 2) {
          const u32 wbits = lane == 0 ? (u32)keep : (u32)(keep >> 32);
          if (wbits) atomicOr(bm + (wb >> 5) + lane, wbits);
        }
        break;
      }
      const u32 lv = in_s ? d.len : 0u;
      op += readlane(dpp_incl_scan(lv), 63);
      if (lane < 2) {
        const u32 wbits = lane == 0 ? (u32)Sin : (u32)(Sin >> 32);
        if (wbits) atomicOr(bm + (wb >> 5) + lane, wbits);
      }
      // the exit is the chain's first position past the chunk, which may lie
      // in this window (a window straddles ce)
      const u64 Sx = S & range_mask(wb, ce, 0xffffffffu);
      if (Sx) {
        ip = wb + (u32)__builtin_ctzll(Sx);
        break;
      }
      const u32 last = 63u - (u32)__builtin_clzll(S);
      ip = readlane(d.nxt, last);
    }
    if (lane == 0) {
      recs[idx].exit = ip;
      recs[idx].bad = bad;
      recs[idx].len = op;
    }
  }
}

// fixup: one wave per huge message, chunk by chunk (see above).  mstat[i]:
// 1 = the message's chain is sound end to end (its chunks' checks follow).
__global__ __launch_bounds__(4 * 64) void chunk_fixup_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len,
    const u32* __restrict__ out_len, const u32* __restrict__ bm_base, u32* __restrict__ bitmap,
    const u32* __restrict__ big_count, ChunkRec* __restrict__ recs, const u32* __restrict__ first_rec,
    u32* __restrict__ mstat, u32* __restrict__ next) {
  __shared__ u32 stage_s[4][kBigStageBytes / 4 + 4];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 n_huge = big_count[8];
  u32* st = stage_s[wv];
  for (;;) {
    const u32 got = atomicAdd(next, lane == 0 ? 1u : 0u);
    const u32 i = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (i >= n_huge) break;
    const u32 b = first_rec[i];
    if (b == 0xffffffffu) continue;  // (records did not fit: cannot happen with the sized workspace)
    const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)recs[b].m);
    const u32 K = recs[b].nchunks;
    const u8* ib = in + in_off[m];
    const u32 n_in = in_len[m];
    const u32 expected = out_len[m];
    u32* bm = bitmap + bm_base[m];
    const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
    const u8* abase = ib - ibal;
    const u32 last_chunk = (ibal + n_in - 1) >> 4;
    Stage sg;
    bool ok = recs[b].bad == 0;
    u32 e = recs[b].exit, run = recs[b].len;
    if (lane == 0) recs[b].base = 0;
    // the lengths of the tags in `mask` of the window at wb (all lanes)
    auto mask_len = [&](u32 wb, u64 mask, const Cand2& d) -> u32 {
      const bool in_m = (mask >> lane) & 1ull;
      return readlane(dpp_incl_scan(in_m ? d.len : 0u), 63);
    };
    for (u32 k = 1; k < K && ok; ++k) {
      const u32 cs = k * kChunkBytes;
      const u32 ce = cs + kChunkBytes < n_in ? cs + kChunkBytes : n_in;
      const ChunkRec R = recs[b + k];
      if (lane == 0) recs[b + k].base = run;
      const u32 w0 = cs >> 5;
      const u32 w1 = ce == n_in ? ((((n_in + 31) >> 5) + 3) & ~3u) : ce >> 5;
      if (e >= ce) {  // a literal spans the chunk: no tag starts in it
        wave_lds_fence();
        for (u32 wd = w0 + lane; wd < w1; wd += 64) bm[wd] = 0u;
        if (lane == 0) recs[b + k].len = 0;
        continue;
      }
      // ---- the true chain from e until it meets a speculative tag start
      u32 pos = e, true_len = 0, meet = 0xffffffffu;
      for (u32 guard = 0; guard < kChunkBytes; ++guard) {
        if (pos >= ce) break;
        const u32 wb = pos & ~31u;
        stage_for(sg, st, abase, ibal, last_chunk, wb, lane);
        const Cand2 d = decode_cand(st, sg.spos, wb + lane, n_in, lane);
        const u64 S = window_chain(d, pos - wb, lane);
        const u64 Sin = S & range_mask(wb, cs, ce);
        const u64 SP = bm_window(bm, wb) & range_mask(wb, cs, ce);
        const u64 common = Sin & SP;
        u64 T = Sin;
        if (common) {
          meet = wb + (u32)__builtin_ctzll(common);
          T = Sin & ((1ull << (meet - wb)) - 1);
        }
        if (__any(((T >> lane) & 1ull) && d.bad_local)) {
          ok = false;
          break;
        }
        true_len += mask_len(wb, T, d);
        if (meet != 0xffffffffu) break;
        const u64 Sx = S & range_mask(wb, ce, 0xffffffffu);  // (the exit, as in spec)
        if (Sx) {
          pos = wb + (u32)__builtin_ctzll(Sx);
          break;
        }
        const u32 last = 63u - (u32)__builtin_clzll(S);
        pos = readlane(d.nxt, last);
      }
      if (!ok) break;
      u32 spec_before = 0;
      if (meet != 0xffffffffu) {
        // the speculative tags in [cs, meet): their output length
        for (u32 wb = cs; wb < meet; wb += 64) {
          const u64 SP = bm_window(bm, wb) & range_mask(wb, cs, meet);
          if (!SP) continue;
          stage_for(sg, st, abase, ibal, last_chunk, wb, lane);
          const Cand2 d = decode_cand(st, sg.spos, wb + lane, n_in, lane);
          spec_before += mask_len(wb, SP, d);
        }
        if (R.bad) ok = false;  // the true chain runs into the speculative chain's bad tag
      }
      // ---- rewrite the bits before the meeting point (the whole chunk if
      // none): clear them, then walk the true chain from e again, setting its
      const u32 upto = meet != 0xffffffffu ? meet : ce;
      wave_lds_fence();
      for (u32 wd = w0 + lane; wd < ((upto + 31) >> 5); wd += 64) {
        const u32 lo = wd << 5;
        const u32 keepm = upto >= lo + 32 ? 0u : (0xffffffffu << (upto - lo));  // bits from the meet on stay
        // (atomics, performed in L2: a plain load of the OR below could hit an
        // L1 line filled before this store)
        atomicAnd(bm + wd, keepm);
      }
      if (meet == 0xffffffffu && ce == n_in)
        for (u32 wd = ((ce + 31) >> 5) + lane; wd < w1; wd += 64) bm[wd] = 0u;
      wave_lds_fence();
      {
        u32 p2 = e;
        for (u32 guard = 0; guard < kChunkBytes && p2 < upto; ++guard) {
          const u32 wb = p2 & ~31u;
          stage_for(sg, st, abase, ibal, last_chunk, wb, lane);
          const Cand2 d = decode_cand(st, sg.spos, wb + lane, n_in, lane);
          const u64 S = window_chain(d, p2 - wb, lane);
          const u64 T = S & range_mask(wb, cs, upto);
          if (lane < 2) {
            const u32 wbits = lane == 0 ? (u32)T : (u32)(T >> 32);
            if (wbits) atomicOr(bm + (wb >> 5) + lane, wbits);
          }
          const u32 last = 63u - (u32)__builtin_clzll(S);
          p2 = readlane(d.nxt, last);
        }
      }
      const u32 new_len = meet != 0xffffffffu ? true_len + R.len - spec_before : true_len;
      if (lane == 0) recs[b + k].len = new_len;
      run += new_len;
      e = meet != 0xffffffffu ? R.exit : pos;
    }
    if (ok) ok = e == n_in && run == expected;
    if (lane == 0) mstat[i] = ok ? 1u : 0u;
  }
}

// check: one wave per chunk record, with the true bits and the chunk's base.
__global__ __launch_bounds__(4 * 64) void chunk_check_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len,
    const u32* __restrict__ out_len, const u32* __restrict__ bm_base, const u32* __restrict__ bitmap,
    const u32* __restrict__ chunk_count, ChunkRec* __restrict__ recs, u8* out, const u64* __restrict__ out_off,
    u32* __restrict__ next, u32 max_recs) {
  __shared__ u32 stage_s[4][kBigStageBytes / 4 + 4];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 cnt = *chunk_count < max_recs ? *chunk_count : max_recs;
  u32* st = stage_s[wv];
  for (;;) {
    const u32 got = atomicAdd(next, lane == 0 ? 1u : 0u);
    const u32 idx = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (idx >= cnt) break;
    const ChunkRec R = recs[idx];
    const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)R.m);
    const u8* ib = in + in_off[m];
    u8* ob = out + out_off[m];
    const u32 n_in = in_len[m];
    const u32 expected = out_len[m];
    const u32* bm = bitmap + bm_base[m];
    const u32 cs = R.k * kChunkBytes;
    const u32 ce = cs + kChunkBytes < n_in ? cs + kChunkBytes : n_in;
    const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
    const u8* abase = ib - ibal;
    const u32 last_chunk = (ibal + n_in - 1) >> 4;
    Stage sg;
    u32 op = (u32)__builtin_amdgcn_readfirstlane((int)R.base), flags = 0;
    for (u32 wb = cs; wb < ce; wb += 64) {
      const u64 S = bm_window(bm, wb) & range_mask(wb, cs, ce);
      if (!S) continue;
      stage_for(sg, st, abase, ibal, last_chunk, wb, lane);
      const u32 p = wb + lane;
      const Cand2 d = decode_cand(st, sg.spos, p, n_in, lane);
      const bool in_s = (S >> lane) & 1ull;
      const u32 lv = in_s ? d.len : 0u;
      const u32 incl = dpp_incl_scan(lv);
      const u32 t_op = op + incl - lv;
      // writer space and copy offset checks (:761, :1166, :1200, :1410, :1466)
      if (__any(in_s && (d.bad_local || expected - t_op < d.len || (!d.lit && d.coff - 1u >= t_op)))) flags |= kChunkBad;
      // 64 KiB output segments (index_big_message's rules)
      const bool span = in_s && d.len > 0 && ((t_op ^ (t_op + d.len - 1)) >> 16) != 0;
      const bool xcopy = in_s && !d.lit && t_op - d.coff < (t_op & ~0xffffu);
      if (__any(span || xcopy)) flags |= kChunkNoSeg;
      if (!(flags & kChunkNoSeg) && in_s && t_op != 0 && (t_op & 0xffffu) == 0 && t_op + 4 <= expected)
        __builtin_memcpy(ob + t_op, &p, 4);
      op += readlane(incl, 63);
    }
    if (lane == 0) recs[idx].flags = flags;
  }
}

// After pass 1b: a message's status and its place in pass 2's work lists
// (its 64 KiB segments when the stream allows them, else the whole message).
__device__ __forceinline__ void list_big_message(u32 m, i32 st, bool seg, u32 lane, const u32* __restrict__ out_len,
                                                 i32* __restrict__ status_out, u32 n_msgs,
                                                 u64* __restrict__ seg_list, u32* __restrict__ seg_count,
                                                 u32* __restrict__ whole_list, u32* __restrict__ whole_count) {
  if (lane == 0) status_out[m] = st;
  if (st != kOk) return;
  const u32 expected = out_len[m];
  u32 nseg = 0;  // > 1: run as segments
  if (seg && expected > 65536u) {
    nseg = (expected + 65535u) >> 16;
    if (expected - ((nseg - 1) << 16) < 4) --nseg;  // the tail joins the previous segment
  }
  bool whole = nseg < 2;
  if (!whole) {
    u32 b = 0;
    if (lane == 0) b = atomicAdd(seg_count, nseg);
    b = readlane(b, 0);
    for (u32 k = lane; k < nseg; k += 64) {
      const u64 e = b + k < n_msgs ? ((u64)m | ((u64)k << 32) | ((u64)(k == nseg - 1) << 63)) : 0xffffffffull;
      if (b + k < n_msgs) seg_list[b + k] = e;
    }
    if (b + nseg > n_msgs) {
      for (u32 k = lane; b + k < n_msgs && k < nseg; k += 64) seg_list[b + k] = 0xffffffffull;
      whole = true;
    }
  }
  if (whole) {
    u32 b = 0;
    if (lane == 0) b = atomicAdd(whole_count, 1u);
    b = readlane(b, 0);
    if (lane == 0) whole_list[b] = m;
  }
}

// final: one wave per huge message (a message whose records did not fit is
// walked here serially, as index_big_kernel would).
__global__ __launch_bounds__(4 * 64) void chunk_final_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u32 flags,
    const u32* __restrict__ bm_base, u32* __restrict__ bitmap, u8* out, const u64* __restrict__ out_off,
    const u32* __restrict__ big_list, const u32* __restrict__ out_len, i32* __restrict__ status_out,
    const u32* __restrict__ big_count, const ChunkRec* __restrict__ recs, const u32* __restrict__ first_rec,
    const u32* __restrict__ mstat, u32 n_msgs, u64* __restrict__ seg_list, u32* __restrict__ seg_count,
    u32* __restrict__ whole_list, u32* __restrict__ whole_count, u32* __restrict__ next) {
  __shared__ u32 stage_s[4][kBigStageBytes / 4 + 4];
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  const u32 n_huge = big_count[8];
  for (;;) {
    const u32 got = atomicAdd(next, lane == 0 ? 1u : 0u);
    const u32 i = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (i >= n_huge) break;
    const u32 b = first_rec[i];
    if (b == 0xffffffffu) {
      const u32 m = big_list[n_msgs - 1 - i];
      bool seg = true;
      const i32 st = index_big_message(m, in, in_off, in_len, out_len, flags & 2u, bm_base, bitmap, stage_s[wv],
                                       lane, out + out_off[m], seg);
      list_big_message(m, st, seg, lane, out_len, status_out, n_msgs, seg_list, seg_count, whole_list, whole_count);
      continue;
    }
    const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)recs[b].m);
    const u32 K = recs[b].nchunks;
    u32 fl = 0;
    for (u32 k = lane; k < K; k += 64) fl |= recs[b + k].flags;
    const bool bad = __any(fl & kChunkBad), noseg = __any(fl & kChunkNoSeg);
    const bool ok = mstat[i] != 0 && !bad;
    list_big_message(m, ok ? kOk : kCorrupt, !noseg, lane, out_len, status_out, n_msgs, seg_list, seg_count,
                     whole_list, whole_count);
  }
}

// ===========================================================================
// Pass 2: execute.  One wave per status-OK message.
//
// Output is assembled in a per-wave LDS window `sb` (kWindow bytes) holding
// output positions [sbase, sbase + kWindow); sbase is kept congruent to the
// slot's address modulo 16 so window offsets and global addresses share
// 16-byte alignment.  Per group of <= 64 pieces:
//   round A   literal pieces (input bytes) and far copies (source before the
//             window, already stored) load from global memory -- one round
//             trip, all independent -- and land in the window;
//   rounds B  near copies (source inside the window) resolve in LDS in
//             dependency rounds, OR-ing their bytes into the zeroed window
//             ahead of the write front (five aligned ds_or_b32 per piece);
//   flush     completed 16-byte blocks go to global memory, 1 KiB per wave
//             instruction.
// The window slides (keeping >= 2 KiB of history) when a group would overrun
// it.  Literals longer than 64 bytes bypass it: the wave copies them
// global-to-global, 1 KiB per instruction.
// ===========================================================================
namespace {
// A/B knobs of the execution pass
// The software-pipelined execution pass (exec6_message; A/B variant).
// Window and kept history: 3 KiB / 1 KiB at 7 waves per SIMD (C3 6.35 ->
// 6.20 ms against 4 KiB / 2 KiB at 6 waves, A/B on one box; 4 KiB / 1 KiB
// at 6 waves 6.33, a 256-entry tag ring 7.04).
#ifndef FSG_WINDOW
#define FSG_WINDOW 3072
#define FSG_KEEP 1024
#endif
constexpr u32 kWindow = FSG_WINDOW;  // LDS output window per wave
constexpr u32 kKeep = FSG_KEEP;      // history kept when the window slides
// After a slide op - sbase <= keep + 15; a group adds <= 16 * kMaxPieces
// bytes and an OR store writes up to 20 bytes past a piece's start, all of
// which must stay inside the window's kWindow + 32 bytes.
constexpr u32 kMaxKeep = (kWindow - 16 * 64 - 48) & ~15u;
static_assert(kKeep <= kMaxKeep, "kept history leaves room for one group");


}  // namespace

// A far copy's 16 source bytes: output this wave stored in an earlier group,
// read from the slot with an sc1 load, which is served by L2 and bypasses
// this CU's L1 (MI355X_MICROARCH.md, visibility table).  Why that matters:
// an L1 line can be filled while part of it is still unwritten -- a far load
// just after a long literal's window restart, or the neighbouring message's
// slot sharing a 128-byte line -- and the vector L1 is not specified to pick
// up later stores.  Ordering in L2: a wave's vector memory operations return
// in issue order, loads and stores alike, and every far source was flushed
// at least one group before it is read, behind that group's waited tag loads
// ("far copies").  src + 16 <= op <= the slot length
// (far sources end >= 16 bytes below the window base, which is <= op - 16), so
// the range check never clips a needed byte.
__device__ __forceinline__ u32x4 far_load(__amdgpu_buffer_rsrc_t r, u32 off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}

// One message, executed by the calling wave (see the pass-2 comment above).
__device__ __forceinline__ void exec_message(
    u32 m, const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u8* out, const u64* __restrict__ out_off,
    const u32* __restrict__ out_len, i32* __restrict__ status, const u32* __restrict__ bm_base,
    const u32* __restrict__ bitmap, u32* ring, u8* pmap, u8* sb, const u32x4* sel_tab,
    const u32x4* mtab, u32 lane, i32 st, u32 ip0, u32 op0, u32 op1, bool prio, u32 keep_hist) {
  // One message (ip0 = op0 = 0, op1 = its length), or one segment of a large
  // one: output [op0, op1) from the tags starting at input offset ip0, whose
  // copies stay inside the segment (checked by the index walk).
  // every per-message scalar is loaded up front (one round trip, not a chain)
  const u32 bmb = bm_base[m];
  const u32 n_in = in_len[m];
  const u32 expected = out_len[m];
  const u8* ib = in + in_off[m];
  u8* ob = out + out_off[m];
  if (st != kOk) return;
  const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
  const u32 obal = (u32)(reinterpret_cast<uintptr_t>(ob) & 15);
  // the message's input as a buffer: tag and literal loads need no clamping
  const __amdgpu_buffer_rsrc_t irsrc = msg_rsrc(ib - ibal, ibal + n_in);
  // the message's slot as a buffer: far copies load through it past L1
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(ob - obal, (short)0, (int)(expected + obal), 0x00020000);

  if ((bmb & kSingleLiteral) && op1 == expected && op0 == 0) {
    // one literal (checked by pass 1): a straight copy, 4 KiB per step with
    // all loads first
    const u32 S = bmb & ~kSingleLiteral;
    for (u32 k0 = 0; k0 < expected; k0 += 4096) {
      u32x4 x[4];
#pragma unroll
      for (u32 r = 0; r < 4; ++r) {
        const u32 k = k0 + 1024 * r + lane * 16;
        x[r] = k < expected ? rsrc_load16(irsrc, S + k + ibal) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (u32 r = 0; r < 4; ++r) {
        const u32 k = k0 + 1024 * r + lane * 16;
        if (k < expected) store_exact(ob + k, x[r], expected - k < 16 ? expected - k : 16u);
      }
    }
    return;
  }
  const u32* bm = bitmap + bmb;
  const u32 nwords = (n_in + 31) >> 5;

#ifdef FSG_STAMPS
  u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 t_last_ = __builtin_amdgcn_s_memtime();
#endif
  u32 head = 0, tail = 0, scan = ip0 >> 5, op = op0;
  int sbase = (int)((op0 + obal) & ~15u) - (int)obal;  // output position of sb[0]
  u32 flushed = op0;  // output [op0, flushed) is in global memory
  // window bytes from the write front up to zero_end are zero, so rounds B
  // can OR their pieces in (or_store)
  auto zero_from = [&](u32 from) {  // 1 KiB of zeros at a 16-aligned offset
    const u32 i = from + 16 * lane;
    if (i < kWindow + 32) *reinterpret_cast<u32x4*>(sb + i) = u32x4{0, 0, 0, 0};
  };
  zero_from(0);
  u32 zero_end = 1024;
  wave_lds_fence();
  // next fill, prefetched: lane l holds word scan + l / 4 and takes its byte l % 4
  auto fill_word = [&](u32 sc) -> u32 {
    const u32 wi = sc + (lane >> 2);
    return (lane < 4 * kFillWords && wi < nwords) ? bm[wi] : 0u;
  };
  u32 bmw = fill_word(scan);
  u32 pf_head = 0xffffffffu, pf_cnt = 0;  // tag bytes prefetched for ring [pf_head, +pf_cnt)
  u32x2 tv = u32x2{0, 0};

  // Store window bytes [flushed, fe) to the slot: one 16-byte block per lane,
  // whole aligned blocks with one store, partial edge blocks exactly.
  auto flush_to = [&](u32 fe) {
    if (fe <= flushed) return;
    const int b0 = (int)(((flushed + obal) & ~15u)) - (int)obal;  // block start <= flushed
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

  for (;;) {
    // ---------- refill the tag ring from the bitmap (keeps >= 64 tags ahead)
    if (tail - head < 2 * kMaxPieces && scan < nwords) {
      if (prio) __builtin_amdgcn_s_setprio(1);  // the fill's bitmap load: same rule (C3 -1.5%)
      u32 bits = (bmw >> (8 * (lane & 3))) & 0xffu;  // 8 bits per lane
      const u32 bitbase = (scan + (lane >> 2)) * 32 + 8 * (lane & 3);
      // a segment's walk starts at ip0: earlier tag starts are not its own
      if (bitbase < ip0) bits &= bitbase + 8 <= ip0 ? 0u : (0xffu << (ip0 - bitbase)) & 0xffu;
      const u32 cnt = __builtin_popcount(bits);
      const u32 incl = dpp_incl_scan(cnt);
      u32 slot = tail + incl - cnt;
      while (bits) {
        ring[slot & (kTagRing - 1)] = bitbase + __builtin_ctz(bits);
        ++slot;
        bits &= bits - 1;
      }
      tail += readlane(incl, 63);
      scan += kFillWords;
      bmw = fill_word(scan);
      wave_lds_fence();
      STAMP(0);
      continue;
    }
    const u32 avail = tail - head;
    if (avail == 0 || op >= op1) break;
    const u32 take0 = avail < 64 ? avail : 64u;
    const bool valid = lane < take0;
    const u32 pos = valid ? ring[(head + lane) & (kTagRing - 1)] : 0u;
    if (pf_head != head || pf_cnt < take0)
      tv = valid ? rsrc_tag5(irsrc, pos + ibal) : u32x2{0, 0};

    // ---------- decode one tag per lane (checked by pass 1)
    // A wave on its way to the group's global loads (round A; and the bitmap
    // load of a fill) runs at raised priority until it has issued them, so the
    // SIMD's issue slots go to the waves that will put memory requests in
    // flight (A/B on one box: C3 7.53 -> 7.37 ms, C2 neutral; CM +2%, so
    // only for the single-stream batches: `prio`; lowering it only for
    // rounds B instead measured the same).
    if (prio) __builtin_amdgcn_s_setprio(1);
    const u32 t0 = tv[0], t1 = tv[1];
    const u32 c = t0 & 0xffu;
    const u32 type = c & 3;
    const bool is_lit = type == 0;
    const u32 l0 = (c >> 2) + 1;
    const bool longlit = is_lit && l0 >= 61;
    const u32 nbl = longlit ? l0 - 60 : 0u;
    const u32 ext = (t0 >> 8) | (t1 << 24);
    const u32 msk = nbl >= 4 ? 0xffffffffu : ((1u << (8 * nbl)) - 1u);
    const u32 litlen = longlit ? (ext & msk) + 1u : l0;
    const u32 nb = is_lit ? nbl : (type == 1 ? 1u : (type == 2 ? 2u : 4u));
    const u32 clen = type == 1 ? 4 + ((c >> 2) & 7) : l0;
    const u32 coff = type == 1 ? (((c >> 5) << 8) | ((t0 >> 8) & 0xffu))
                               : (type == 2 ? ((t0 >> 8) & 0xffffu) : ext);
    const u32 len = is_lit ? litlen : clen;
    const u32 lsrc = pos + 1 + nb;

    const u64 bigm = __ballot(valid && is_lit && len > 64);
    STAMP(1);
    if (bigm & 1ull) {
      // ---------- long literal: written straight to the slot by the whole
      // wave; the window restarts behind it
      const u32 L = readlane(len, 0), S = readlane(lsrc, 0);
      if ((u64)op + L > op1) {  // writer overrun
        if (lane == 0) status[m] = kCorrupt;
        return;
      }
      flush_to(op);
      // 4 KiB per step: all loads first, so their latencies overlap
      for (u32 k0 = 0; k0 < L; k0 += 4096) {
        u32x4 x[4];
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 k = k0 + 1024 * r + lane * 16;
          x[r] = k < L ? rsrc_load16(irsrc, S + k + ibal) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 k = k0 + 1024 * r + lane * 16;
          if (k < L) store_exact(ob + op + k, x[r], L - k < 16 ? L - k : 16u);
        }
      }
      op += L;
      flushed = op;
      // The window restarts one block before the block holding op, so that
      // >= 16 flushed bytes precede it (a copy reading before the window
      // then reads only stored bytes); its head comes from the literal's tail.
      sbase = (int)((op + obal) & ~15u) - (int)obal - 16;
      zero_from(0);
      zero_end = 1024;
      wave_lds_fence();
      if (lane < 2) {
        const u32 lo = (u32)sbase + 16 * lane;
        if (lo < op) {
          const u32 cnt = op - lo < 16 ? op - lo : 16u;
          store_exact(sb + 16 * lane, rsrc_load16(irsrc, S + L - (op - lo) + ibal), cnt);
        }
      }
      wave_lds_fence();
      head += 1;
      pf_head = 0xffffffffu;
      // the literal's bytes hold no tag starts: resume the bitmap scan at the
      // word of the next tag instead of scanning the zero words in between
      if (head == tail) {
        const u32 nw = (S + L) >> 5;
        if (nw > scan) {
          scan = nw;
          bmw = fill_word(scan);
        }
      }
      STAMP(7);
      continue;
    }
    const u32 take = bigm ? (u32)__builtin_ctzll(bigm) : take0;
    const bool v = lane < take;

    // ---------- pieces: <= 16 bytes each, one per lane
    const bool pat = !is_lit && coff < 16;
    const u32 step = pat ? pat_step(coff) : 16u;
    const u32 pc = v ? (pat ? pattern_pieces(len, step) : (len + 15) >> 4) : 0u;
    const u32 lv = v ? len : 0u;
    const u32 incl = dpp_incl_scan(pc | (lv << 16));
    const u32 incl_pc = incl & 0xffffu, excl_pc = incl_pc - pc;
    const u32 t_op = op + (incl >> 16) - lv;
    const bool fits = v && incl_pc <= kMaxPieces && t_op < op1;
    const u32 k_tags = (u32)__builtin_popcountll(__ballot(fits));
    const u32 tot_pc = readlane(incl_pc, k_tags - 1);
    const u32 tot_len = readlane(incl >> 16, k_tags - 1);
    // copy offset 0 or past the bytes produced so far: the reference's
    // writer check (snappy.cc:1200, :1410, :1466); the message is corrupt
    // and the writer's space check (:1166, :1400) against the header length
    if (__any(fits && ((u64)t_op + len > op1 || (!is_lit && (coff == 0 || coff > t_op - op0))))) {
      if (lane == 0) status[m] = kCorrupt;
      return;
    }

    STAMP(2);
    // ---------- slide the window if this group would overrun it
    if (op + tot_len - sbase > kWindow) {
      const int nsb = (int)(((op - keep_hist + obal) & ~15u)) - (int)obal;
      // a far piece (source below the new base) may read up to 15 bytes at
      // and above the base, so those must be stored too
      if ((int)flushed < nsb + 16) flush_to((u32)((int)((op + obal) & ~15u) - (int)obal));
      // From this group on, far loads read bytes below the new base + 16:
      // stored by this flush or by earlier groups' flushes, which may still
      // be in flight (no waited load was issued after the last of them, the
      // ordering argument of DESIGN.md §4).  Wait until they are
      // acknowledged by L2, where the far loads (sc1) are served.  Once per
      // slide (~every 3 KiB of output).
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
      zero_end = (keep + 15) & ~15u;  // the copied blocks end in zeros past op
    }
    // ---------- prefetch the next group's tag bytes (lands during this group; issued after a
    // slide's store wait, which then waits only for older operations)
    {
      const u32 nh = head + k_tags;
      const u32 na = tail - nh;
      const u32 ncnt = na < 64 ? na : 64u;
      if (lane < ncnt) {
        const u32 npos = ring[(nh + lane) & (kTagRing - 1)];
        tv = rsrc_tag5(irsrc, npos + ibal);
      }
      pf_head = nh;
      pf_cnt = ncnt;
    }

    while (op + tot_len + 20 - sbase > zero_end) {  // the group's OR stores land in zeros
      zero_from(zero_end);
      zero_end += 1024;
    }
    wave_lds_fence();

    if (fits)
      for (u32 p = 0; p < pc; ++p) pmap[excl_pc + p] = (u8)lane;
    wave_lds_fence();
    const bool has = lane < tot_pc;
    const u32 t = has ? pmap[lane] : 0u;
    const u32 kind = is_lit ? 0u : (pat ? 2u : 1u);
    const u32 A = t_op;
    const u32 B = len | (excl_pc << 8) | (kind << 16) | ((pat ? coff : 0u) << 20);
    const u32 C = is_lit ? lsrc : t_op - coff;
    const u32 At = __shfl(A, t, 64), Bt = __shfl(B, t, 64), Ct = __shfl(C, t, 64);
    const u32 lenT = Bt & 0xffu, exT = (Bt >> 8) & 0xffu, kT = (Bt >> 16) & 3u, offT = Bt >> 20;
    const u32 stepT = kT == 2 ? pat_step(offT) : 16u;
    const u32 qs = (lane - exT) * stepT;
    const u32 dst = At + qs;
    const u32 n = lenT - qs < stepT ? lenT - qs : stepT;
    const u32 src = kT == 2 ? Ct : Ct + qs;
    const u32 need_end = kT == 0 ? 0u : (kT == 2 ? At : src + n);
    u8* const wdst = sb + ((int)dst - sbase);

    STAMP(3);
    // ---------- round A: literal pieces and far copies, from global memory
    const bool global_src = has && (kT == 0 || (int)src < sbase);
    u32x4 xa = u32x4{0, 0, 0, 0};
    if (global_src)
      xa = kT == 0 ? rsrc_load16(irsrc, src + ibal) : far_load(orsrc, src + obal);
    if (prio) __builtin_amdgcn_s_setprio(0);
    // the previous group's completed blocks are flushed while these loads are
    // in flight (far sources lie before the window: flushed long ago)
    {
      const int fe = (int)((op + obal) & ~15u) - (int)obal;
      // once a wave instruction's worth (1 KiB) is complete: every lane
      // stores a full block.  A slide first flushes what it would drop, so
      // far sources (below the window base) are always in global memory.
      if (fe >= (int)flushed + 1024) flush_to((u32)fe);
    }
    if (global_src) {
      if (kT == 2) xa = expand_pattern(xa, offT, sel_tab);
      store_exact(wdst, xa, n);  // (or_store here measured 4% slower)
    }
    wave_lds_fence();

    STAMP(4);
    // ---------- rounds B: near copies, in LDS, in dependency order.  The
    // pending set lives in a scalar mask: per round one find-first, one
    // readlane and one ballot (C3 7.95 -> 7.87 ms against a per-lane done
    // flag re-balloted each round).  The pattern expansion keeps its branch:
    // running it for every piece measured 2.8% slower.
    u64 pend = __ballot(has && !global_src);
    while (pend) {
      const u32 wm = readlane(dst, (u32)__builtin_ctzll(pend));
      const bool ready = ((pend >> lane) & 1ull) && need_end <= wm;
      if (ready) {
        u32x4 x = lds_read16(sb + ((int)src - sbase));
        if (kT == 2) x = expand_pattern(x, offT, sel_tab);
        or_store(sb, (u32)((int)dst - sbase), x, n, mtab);
      }
      wave_lds_fence();
      pend &= ~__ballot(ready);
    }
    op += tot_len;
    head += k_tags;

    STAMP(5);
  }
  if (op != op1) {  // the stream ended early (snappy.cc:858-868)
    if (lane == 0) status[m] = kCorrupt;
    return;
  }
  flush_to(op1);
#ifdef FSG_STAMPS
  if (lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&g_stamps[k], (unsigned long long)st_[k]);
#endif
}

// ===========================================================================
// Pass 2, v5 (default): one TAG per lane.
//
// Same walk as v4 (tag ring from the bitmap, LDS output window, far copies
// from the slot, flush, slide, long literals), with the per-group work cut
// down to what a tag needs:
//   - the next group's tag bytes are prefetched as 20 bytes per lane (one
//     16-byte and one 4-byte buffer load at the dword below the tag: no
//     clamping, bytes past the message read 0), so a short literal's bytes
//     (<= 16 of them follow the tag byte) are already in registers -- a
//     literal tag needs no load of its own;
//   - the tag is decoded through a 256-entry table in LDS (char_table,
//     snappy.cc:516-549);
//   - no piece map: a lane executes its own tag as <= 4 chunks of 16 bytes.
//     Round A writes every chunk whose source is in registers or global
//     memory (literals, far copies); rounds B run the near chunks in
//     dependency order (a chunk runs once its source ends at or below the
//     first unfinished chunk of the group).  A copy with offset < 16 that
//     overlaps itself writes pat_step(off)-byte chunks of its expanded
//     pattern; each later chunk copies the previous one.
// ===========================================================================
namespace {
constexpr u32 kGroupBytes = 1024;  // output bytes per group (as v4: 64 pieces x 16)

// Per tag byte c: bits 0-4 the right shift of 0xffffffff that masks the nb
// extra bytes ((32 - 8 nb) & 31), bit 5 long literal (length = extra + 1),
// bit 6 literal, bits 8-14 length (short literal, copies), bits 16-18 nb,
// bits 20-30 COPY_1's offset bits 8-10 (snappy.cc:744-781).
__device__ __forceinline__ u32 exec_tag_entry(u32 c) {
  const u32 type = c & 3, l0 = (c >> 2) + 1;
  u32 nb, len, lit = 0, ll = 0, hi = 0;
  if (type == 0) {
    lit = 1;
    nb = l0 > 60 ? l0 - 60 : 0;
    ll = nb ? 1 : 0;
    len = nb ? 0 : l0;
  } else if (type == 1) {
    nb = 1;
    len = 4 + ((c >> 2) & 7);
    hi = (c >> 5) << 8;
  } else {
    nb = type == 2 ? 2 : 4;
    len = l0;
  }
  return ((32 - 8 * nb) & 31) | (ll << 5) | (lit << 6) | (len << 8) | (nb << 16) | (hi << 20);
}
}  // namespace

__device__ __forceinline__ void exec5_message(
    u32 m, const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u8* out, const u64* __restrict__ out_off,
    const u32* __restrict__ out_len, i32* __restrict__ status, const u32* __restrict__ bm_base,
    const u32* __restrict__ bitmap, u32* ring, const u32* tagtab, u8* sb, const u32x4* sel_tab,
    const u32x4* mtab, u32 lane, i32 st, u32 ip0, u32 op0, u32 op1, bool prio, u32 keep_hist) {
  const u32 bmb = bm_base[m];
  const u32 n_in = in_len[m];
  const u32 expected = out_len[m];
  const u8* ib = in + in_off[m];
  u8* ob = out + out_off[m];
  if (st != kOk) return;
  const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
  const u32 obal = (u32)(reinterpret_cast<uintptr_t>(ob) & 15);
  const __amdgpu_buffer_rsrc_t irsrc = msg_rsrc(ib - ibal, ibal + n_in);
  // the slot as a buffer: far copies load through it past L1 (see far_load)
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(ob - obal, (short)0, (int)(expected + obal), 0x00020000);

  if ((bmb & kSingleLiteral) && op1 == expected && op0 == 0) {
    const u32 S = bmb & ~kSingleLiteral;
    for (u32 k0 = 0; k0 < expected; k0 += 4096) {
      Raw16 x[4];
#pragma unroll
      for (u32 r = 0; r < 4; ++r) x[r] = raw_load16(irsrc, S + k0 + 1024 * r + lane * 16 + ibal);
#pragma unroll
      for (u32 r = 0; r < 4; ++r) {
        const u32 k = k0 + 1024 * r + lane * 16;
        if (k < expected) store_exact(ob + k, shifted16(x[r]), expected - k < 16 ? expected - k : 16u);
      }
    }
    return;
  }
  const u32* bm = bitmap + bmb;
  const u32 nwords = (n_in + 31) >> 5;
#ifdef FSG_STAMPS
  u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 t_last_ = __builtin_amdgcn_s_memtime();
#endif

  u32 head = 0, tail = 0, scan = ip0 >> 5, op = op0;
  int sbase = (int)((op0 + obal) & ~15u) - (int)obal;  // output position of sb[0]
  u32 flushed = op0;                                    // output [op0, flushed) is in global memory
  auto zero_from = [&](u32 from) {  // 1 KiB of zeros at a 16-aligned offset
    const u32 i = from + 16 * lane;
    if (i < kWindow + 32) *reinterpret_cast<u32x4*>(sb + i) = u32x4{0, 0, 0, 0};
  };
  zero_from(0);
  u32 zero_end = 1024;
  wave_lds_fence();
  auto fill_word = [&](u32 sc) -> u32 {
    const u32 wi = sc + (lane >> 2);
    return (lane < 4 * kFillWords && wi < nwords) ? bm[wi] : 0u;
  };
  u32 bmw = fill_word(scan);
  // the next group's tag bytes: 20 bytes from the dword below the tag
  u32 pf_head = 0xffffffffu, pf_cnt = 0;
  u32 pf_pos = 0;  // the ring positions the prefetch used
  u32x4 pd = u32x4{0, 0, 0, 0};
  u32 pd4 = 0;
  auto prefetch = [&](u32 p) {
    const u32 a = (p + ibal) & ~3u;
    pd = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
    pd4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
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

  for (;;) {
    // ---------- refill the tag ring from the bitmap (as v4)
    if (tail - head < 2 * kMaxPieces && scan < nwords) {
      if (prio) __builtin_amdgcn_s_setprio(1);
      u32 bits = (bmw >> (8 * (lane & 3))) & 0xffu;
      const u32 bitbase = (scan + (lane >> 2)) * 32 + 8 * (lane & 3);
      if (bitbase < ip0) bits &= bitbase + 8 <= ip0 ? 0u : (0xffu << (ip0 - bitbase)) & 0xffu;
      const u32 cnt = __builtin_popcount(bits);
      const u32 incl = dpp_incl_scan(cnt);
      u32 slot = tail + incl - cnt;
      while (bits) {
        ring[slot & (kTagRing - 1)] = bitbase + __builtin_ctz(bits);
        ++slot;
        bits &= bits - 1;
      }
      tail += readlane(incl, 63);
      scan += kFillWords;
      bmw = fill_word(scan);
      wave_lds_fence();
      STAMP(0);
      continue;
    }
    const u32 avail = tail - head;
    if (avail == 0 || op >= op1) break;
    const u32 take0 = avail < 64 ? avail : 64u;
    const bool valid = lane < take0;
    // every lane reads the ring and prefetches: a lane past the valid tags
    // reads a stale position, whose buffer loads return message bytes or 0
    const u32 pos = ring[(head + lane) & (kTagRing - 1)];
    if (pf_head != head || pf_cnt < take0) prefetch(pos);
    if (prio) __builtin_amdgcn_s_setprio(1);

    // ---------- decode one tag per lane (checked by pass 1)
    const u32 s = (pos + ibal) & 3u;
    const u32 c = __builtin_amdgcn_alignbyte(pd[1], pd[0], s) & 0xffu;
    const u32 e = tagtab[c];
    // bytes pos+1 .. pos+16 (a short literal's bytes; a copy's offset bytes)
    const bool q = s == 3;
    const u32 w0 = q ? pd[1] : pd[0], w1 = q ? pd[2] : pd[1], w2 = q ? pd[3] : pd[2];
    const u32 w3 = q ? pd4 : pd[3];
    const u32 b = (s + 1) & 3u;
    const u32x4 xr = u32x4{__builtin_amdgcn_alignbyte(w1, w0, b), __builtin_amdgcn_alignbyte(w2, w1, b),
                           __builtin_amdgcn_alignbyte(w3, w2, b), __builtin_amdgcn_alignbyte(pd4, w3, b)};
    const u32 val = xr[0] & (0xffffffffu >> (e & 31u));
    const bool is_lit = e & 64u;
    const u32 len = (e & 32u) ? val + 1u : (e >> 8) & 0x7fu;
    const u32 off = val + (e >> 20);
    const u32 nb = (e >> 16) & 7u;
    const u32 lsrc = pos + 1 + nb;

    const u64 bigm = __ballot(valid && is_lit && len > 64);
    STAMP(1);
    if (bigm & 1ull) {
      // ---------- long literal: written straight to the slot by the whole
      // wave; the window restarts behind it (as v4)
      const u32 L = readlane(len, 0), S = readlane(lsrc, 0);
      if ((u64)op + L > op1) {
        if (lane == 0) status[m] = kCorrupt;
        return;
      }
      flush_to(op);
      for (u32 k0 = 0; k0 < L; k0 += 4096) {
        Raw16 x[4];
#pragma unroll
        for (u32 r = 0; r < 4; ++r) x[r] = raw_load16(irsrc, S + k0 + 1024 * r + lane * 16 + ibal);
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 k = k0 + 1024 * r + lane * 16;
          if (k < L) store_exact(ob + op + k, shifted16(x[r]), L - k < 16 ? L - k : 16u);
        }
      }
      op += L;
      flushed = op;
      sbase = (int)((op + obal) & ~15u) - (int)obal - 16;
      zero_from(0);
      zero_end = 1024;
      wave_lds_fence();
      if (lane < 2) {
        const u32 lo = (u32)sbase + 16 * lane;
        if (lo < op) {
          const u32 cnt = op - lo < 16 ? op - lo : 16u;
          store_exact(sb + 16 * lane, rsrc_load16(irsrc, S + L - (op - lo) + ibal), cnt);
        }
      }
      wave_lds_fence();
      head += 1;
      pf_head = 0xffffffffu;
      if (head == tail) {
        const u32 nw = (S + L) >> 5;
        if (nw > scan) {
          scan = nw;
          bmw = fill_word(scan);
        }
      }
      STAMP(7);
      continue;
    }
    const u32 take = bigm ? (u32)__builtin_ctzll(bigm) : take0;
    const bool v = lane < take;

    // ---------- output positions: <= kGroupBytes per group
    const u32 lv = v ? len : 0u;
    const u32 incl = dpp_incl_scan(lv);
    const u32 t_op = op + incl - lv;
    const bool fits = v && incl <= kGroupBytes && t_op < op1;
    const u32 k_tags = (u32)__builtin_popcountll(__ballot(fits));
    const u32 tot_len = readlane(incl, k_tags - 1);
    // the writer's checks (snappy.cc:1166, :1200, :1400, :1410, :1466)
    if (__any(fits && (len > op1 - t_op || (!is_lit && (off == 0 || off > t_op - op0))))) {
      if (lane == 0) status[m] = kCorrupt;
      return;
    }

    // ---------- slide the window if this group would overrun it (as v4)
    if (op + tot_len - sbase > kWindow) {
      const int nsb = (int)(((op - keep_hist + obal) & ~15u)) - (int)obal;
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
    // ---------- prefetch the next group's tag bytes; zero the window ahead
    auto prefetch_next_and_zero = [&]() {
      {
        const u32 nh = head + k_tags;
        const u32 na = tail - nh;
        const u32 ncnt = na < 64 ? na : 64u;
        pf_pos = ring[(nh + lane) & (kTagRing - 1)];
        prefetch(pf_pos);
        pf_head = nh;
        pf_cnt = ncnt;
      }
      while (op + tot_len + 20 - sbase > zero_end) {
        zero_from(zero_end);
        zero_end += 1024;
      }
      wave_lds_fence();
    };

    STAMP(2);
    // ---------- chunks: a literal's all come in round A (registers for
    // chunk 0 of a short literal, else the input); a copy's leading chunks
    // whose 16-byte source starts below the window base come from the slot
    // (far: stored at least one group ago); the rest run in rounds B
    const u32 src = is_lit ? lsrc : t_op - off;
    const u32 nch = (len + 15) >> 4;
    const bool pat = !is_lit && off < 16 && off < len;
    // leading chunks done in round A: all of a literal's; a copy's whose
    // 16-byte source starts below the window base (far: from the slot), then
    // those whose source ends at or below the group's first output byte op
    // (near-ready: final window bytes, read from LDS) -- none for a pattern.
    // A near-ready chunk would run in the first round B anyway; in round A it
    // is one OR store among the group's, not a read-modify-write of its own.
    const u32 below = (u32)(sbase - (int)src);  // > 0 as int: far
    const u32 kfar = (int)below > 0 ? ((below - 1) >> 4) + 1 : 0u;
    // chunk k's source ends at src + min(16 (k + 1), len): <= op for the
    // first (op - src) / 16 chunks, or all of them when src + len <= op
    const u32 kready = src + len <= op ? nch : (src < op ? (op - src) >> 4 : 0u);
    const u32 klead = kfar > kready ? kfar : kready;
    const u32 kc = pat ? 0u : (klead < nch ? klead : nch);
    const u32 kf = fits ? (is_lit ? nch : kc) : 0u;
    const bool reg0 = is_lit && nb == 0;
    // Loads only here: the data is first used after the flush below, so all
    // of a lane's chunk loads are in flight together.  A literal chunk is a
    // 16- and a 4-byte load at the dword below it, shifted later by sh; a far
    // chunk one unaligned 16-byte load (shift 0).
    const u32 sh = is_lit ? (src + ibal) & 3u : 0u;
    auto gload = [&](u32 k, u32x4& d, u32& d4) {
      if (is_lit) {
        const u32 a = (src + 16 * k + ibal) & ~3u;
        d = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
        d4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
      } else if (k >= kfar) {  // near-ready: final bytes below op in the window
        d = lds_read16(sb + ((int)(src + 16 * k) - sbase));
      } else {
        d = far_load(orsrc, src + 16 * k + obal);
      }
    };
    auto shf = [&](const u32x4& d, u32 d4, u32 t) {
      return u32x4{__builtin_amdgcn_alignbyte(d[1], d[0], t), __builtin_amdgcn_alignbyte(d[2], d[1], t),
                   __builtin_amdgcn_alignbyte(d[3], d[2], t), __builtin_amdgcn_alignbyte(d4, d[3], t)};
    };
    u32x4 a0 = xr, a1 = u32x4{0, 0, 0, 0};
    u32 a0e = 0, a1e = 0;
    if (kf > 0 && !reg0) gload(0, a0, a0e);
    const u64 m1 = __ballot(kf > 1);
    if (m1 && kf > 1) gload(1, a1, a1e);
    // (the round-A loads go out before the next group's ring read and tag
    // prefetch and the window zeroing: their latency is the group's longest
    // wait; the near-ready LDS reads above read bytes below op, which the
    // zeroing (from zero_end >= op) does not touch)
    prefetch_next_and_zero();
    if (prio) __builtin_amdgcn_s_setprio(0);
    STAMP(3);
    {  // the previous groups' completed blocks, while the loads are in flight
      const int fe = (int)((op + obal) & ~15u) - (int)obal;
      if (fe >= (int)flushed + 1024) flush_to((u32)fe);
    }
    STAMP(4);
    const u32 wa = (u32)((int)t_op - sbase);
    if (kf > 0) or_store(sb, wa, shf(a0, a0e, reg0 ? 0u : sh), len < 16 ? len : 16u, mtab);
    if (m1) {
      if (kf > 1) or_store(sb, wa + 16, shf(a1, a1e, sh), len - 16 < 16 ? len - 16 : 16u, mtab);
      // chunks 2-3 (literals and far copies of 33..64 bytes: rare) reuse the
      // registers, one more round trip
      if (__ballot(kf > 2)) {
        if (kf > 2) gload(2, a0, a0e);
        if (kf > 3) gload(3, a1, a1e);
        if (kf > 2) or_store(sb, wa + 32, shf(a0, a0e, sh), len - 32 < 16 ? len - 32 : 16u, mtab);
        if (kf > 3) or_store(sb, wa + 48, shf(a1, a1e, sh), len - 48, mtab);
      }
    }
    wave_lds_fence();

    STAMP(5);
    // ---------- rounds B: near chunks, in LDS, in dependency order.  Per
    // lane: the current chunk's window offsets (cw destination, sw source),
    // its length n and the end of the bytes it needs, ne (~0: lane done).
    // A chunk runs once ne <= the first unfinished chunk's destination; it is
    // written read-modify-write: 16 window bytes are read and written back
    // with the chunk's n bytes merged in (v_bfi with the n-byte mask), so the
    // write is exact whatever n.  Within one write instruction overlapping
    // lanes land highest-lane-last (tools/probes/lds_overlap_probe.hip), and
    // a lane's 16-byte span only reaches later chunks, whose bytes it writes
    // back unchanged unless their own (higher) lane writes them.
    u32 rem = (fits && kf < nch) ? len - 16 * kf : 0u;
    u32 cw = (u32)((int)t_op - sbase) + 16 * kf;
    u32 sw = (u32)((int)src - sbase) + 16 * kf;
    const u32 stp = pat ? pat_step(off) : 16u;
    u32 n = rem < stp ? rem : stp;
    bool pf = pat;
    u32 ne = rem ? (pf ? cw : sw + n) : 0xffffffffu;
    u64 pend = __ballot(rem > 0);
    // Most groups (~90% on text) hold no pattern copy: their rounds run a
    // loop with no per-lane pattern state (the general loop below costs ~6
    // more instructions per round).
    if (!__ballot(pat && rem > 0)) {
      while (pend) {
        const u32 W = readlane(cw, (u32)__builtin_ctzll(pend));
        if (ne <= W) {
          const u32x4 x = lds_read16(sb + sw);
          const u32x4 o = lds_read16(sb + cw);
          const u32x4 mk = mtab[n];
          u32x4 y;
          y[0] = (x[0] & mk[0]) | (o[0] & ~mk[0]);
          y[1] = (x[1] & mk[1]) | (o[1] & ~mk[1]);
          y[2] = (x[2] & mk[2]) | (o[2] & ~mk[2]);
          y[3] = (x[3] & mk[3]) | (o[3] & ~mk[3]);
          __builtin_memcpy(sb + cw, &y, 16);
          rem -= n;
          cw += n;
          sw += n;
          n = rem < 16u ? rem : 16u;
          ne = rem ? sw + n : 0xffffffffu;
        }
        wave_lds_fence();
        pend = __ballot(rem > 0);
      }
    }
    while (pend) {
      const u32 W = readlane(cw, (u32)__builtin_ctzll(pend));
      if (ne <= W) {
        u32x4 x = lds_read16(sb + sw);
        if (pf) x = expand_pattern(x, off, sel_tab);
        const u32x4 o = lds_read16(sb + cw);
        const u32x4 mk = mtab[n];
        u32x4 y;
        y[0] = (x[0] & mk[0]) | (o[0] & ~mk[0]);
        y[1] = (x[1] & mk[1]) | (o[1] & ~mk[1]);
        y[2] = (x[2] & mk[2]) | (o[2] & ~mk[2]);
        y[3] = (x[3] & mk[3]) | (o[3] & ~mk[3]);
        __builtin_memcpy(sb + cw, &y, 16);
        rem -= n;
        cw += n;
        sw = pat ? cw - stp : sw + n;
        pf = false;
        n = rem < stp ? rem : stp;
        ne = rem ? sw + n : 0xffffffffu;
      }
      wave_lds_fence();
      pend = __ballot(rem > 0);
    }
    op += tot_len;
    head += k_tags;
    STAMP(6);
  }
  if (op != op1) {  // the stream ended early (snappy.cc:858-868)
    if (lane == 0) status[m] = kCorrupt;
    return;
  }
  flush_to(op1);
#ifdef FSG_STAMPS
  if (lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&g_stamps[k], (unsigned long long)st_[k]);
#endif
}

// ===========================================================================
// Pass 2, packed (the forked path's short bodies, walk part 2): several
// bodies per wave, their tags in ONE stream of 64-tag groups.
//
// Run one wave per body, a short body spends most of its time in set-up and
// dependent round trips (its sizes, then its bitmap words, then its tag
// bytes, then its literal bytes) and in half-empty groups (CM: 1.0M bodies
// under 4 KiB compressed, ~64 tags each).  Here a wave takes a batch of up to
// 64 bodies of the walk order, one per lane, so their sizes load in one round
// trip, and lays their outputs end to end in one VIRTUAL output space: body j
// at V_j, congruent to its slot address modulo 16, so no 16-byte block holds
// two bodies.  The tag ring is filled from the bodies' bitmaps one after
// another; an entry carries its body (j << 24 | position, kFirstTag on a
// body's first tag, whose output length then includes the gap up to V_j).
// From there the walk is exec5_message's on virtual positions: a tag's input
// and slot offsets come from its body's lane by ds_bpermute, far copies load
// through one buffer over the output, and the window flush writes each
// body's blocks to its own slot.
// Pass 1 left every body here kOk with tag lengths summing to its length, so
// a body's first tag lands at V_j exactly.  The check pass 2 adds (copy
// offsets, snappy.cc:1200/:1410/:1466) marks a body kCorrupt and drops the bad
// tag; no other body is touched.  Single-literal bodies are copied by the wave
// first.  A batch whose offsets do not fit 32 bits hands its bodies to pass 3
// (kNeedFallback).
// ===========================================================================
#ifndef FSG_PACK_GUARD_STATUS
#define FSG_PACK_GUARD_STATUS kNeedFallback
#endif
namespace {
constexpr u32 kFirstTag = 1u << 23;
constexpr u32 kMidLit = 896;  // literals up to this length run inside a packed group (56 chunks)
__device__ __forceinline__ u32 lane_bperm(u32 v, u32 src) {
  return (u32)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ u32 wave_max(u32 v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 o = (u32)__shfl_xor((int)v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
}  // namespace

__device__ __forceinline__ void exec5_packed(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len, i32* __restrict__ status,
    const u32* __restrict__ bm_base, const u32* __restrict__ bitmap, const u32* __restrict__ perm, u32 first,
    u32 count, u32* ring, const u32* tagtab, u8* sb, const u32x4* sel_tab, const u32x4* mtab, u32 lane,
    u32 keep_hist) {
#ifdef FSG_STAMPS
  u64 st_[16] = {};
  u64 t_last_ = __builtin_amdgcn_s_memtime();
#define PCOUNT(k) (st_[k] += 1)
#else
#define PCOUNT(k) do { } while (0)
#endif
  // ---------- the batch: one body per lane
  const bool have = lane < count;
  const u32 m = have ? perm[first + lane] : 0u;
  const i32 st = have ? status[m] : kCorrupt;
  const u32 bmb_m = have ? bm_base[m] : 0u;
  const u32 n_in = have ? in_len[m] : 0u;
  const u32 E_m = have ? out_len[m] : 0u;
  const u64 io = have ? in_off[m] : 0ull;
  const u64 oo = have ? out_off[m] : 0ull;
  const u32 ial = (u32)(reinterpret_cast<uintptr_t>(in) & 15), oal = (u32)(reinterpret_cast<uintptr_t>(out) & 15);
  const bool ok = have && st == kOk;
  // offsets from the 16-aligned buffer bases must fit 32 bits (with slack for
  // the 20-byte tag loads past a body's end)
  const bool wide = io + ial + n_in + 64 >= (1ull << 32) || oo + oal + E_m + 64 >= (1ull << 32);
  if (__ballot(ok && wide)) {
    if (ok) status[m] = kNeedFallback;
    return;
  }
  const u32 ioff_m = (u32)io + ial, ooff = (u32)oo + oal;
  const u8* const inb = in - ial;
  u8* const outb = out - oal;
  // one buffer over the batch's input and one over its slots, to the furthest
  // body's last dword (the range check is per dword: a dword reaching past
  // num_records reads 0 whole)
  const u32 in_lim = (wave_max(ok ? ioff_m + n_in : 0u) + 3) & ~3u;
  const u32 out_lim = (wave_max(ok ? ooff + E_m : 0u) + 3) & ~3u;
  const __amdgpu_buffer_rsrc_t irsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(inb), (short)0, (int)in_lim, 0x00020000);
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(outb, (short)0, (int)out_lim, 0x00020000);

  // ---------- single-literal bodies: copied by the wave
  const bool single = ok && (bmb_m & kSingleLiteral) && E_m > 0;
  for (u64 S1 = __ballot(single); S1; S1 &= S1 - 1) {
    const u32 j = (u32)__builtin_ctzll(S1);
    const u32 src = readlane(ioff_m, j) + (readlane(bmb_m, j) & ~kSingleLiteral);
    const u32 dst = readlane(ooff, j), L = readlane(E_m, j);
    PCOUNT(13);
    for (u32 k0 = 0; k0 < L; k0 += 4096) {
      Raw16 x[4];
#pragma unroll
      for (u32 r = 0; r < 4; ++r) x[r] = raw_load16(irsrc, src + k0 + 1024 * r + lane * 16);
#pragma unroll
      for (u32 r = 0; r < 4; ++r) {
        const u32 k = k0 + 1024 * r + lane * 16;
        if (k < L) store_exact(outb + (dst + k), shifted16(x[r]), L - k < 16 ? L - k : 16u);
      }
    }
  }

  // ---------- the other bodies, compacted to lanes 0 .. np-1 in walk order
  // (ds_permute: lane i sends its body to lane rank(i)), then laid out
  const bool pk = ok && !(bmb_m & kSingleLiteral) && E_m > 0;
  const u64 P = __ballot(pk);
  if (!P) {
#ifdef FSG_STAMPS
    STAMP(8);
    if (lane == 0)
      for (int k = 0; k < 16; ++k) atomicAdd(&g_stamps[8 + k], (unsigned long long)st_[k]);
#endif
    return;
  }
  const u32 np = (u32)__builtin_popcountll(P);
  const u32 rank = (u32)__builtin_popcountll(P & ((1ull << lane) - 1));
  const u32 to = pk ? rank : np + lane - rank;  // a permutation of the lanes
  auto compact = [&](u32 x) -> u32 { return (u32)__builtin_amdgcn_ds_permute((int)(to << 2), (int)x); };
  const u32 ioff = compact(ioff_m), bmb = compact(bmb_m), bm_id = compact(m);
  const u32 c_ooff = compact(ooff), c_E = compact(E_m), c_nin = compact(n_in);
  const bool body = lane < np;
  const u32 sz = body ? ((c_ooff & 15u) + c_E + 15u) & ~15u : 0u;
  const u32 V = dpp_incl_scan(sz) - sz + (c_ooff & 15u);  // body start
  const u32 VE = V + c_E;                                 // body end
  // (ds_bpermute reads 0 from a lane outside EXEC: every lane permutes, the
  // select comes after)
  const u32 ve_prev = lane_bperm(VE, lane - 1);
  const u32 gap = lane ? V - ve_prev : 0u;  // < 32: up to the body's start
  const u32 oadj = c_ooff - V;             // slot offset = virtual position + oadj
  // the bodies' bitmaps as one run of words: body j's at [Wb_j, Wb_j + nw_j)
  const u32 nw = body ? (c_nin + 31) >> 5 : 0u;
  const u32 w_incl = dpp_incl_scan(nw);
  const u32 Wtot = readlane(w_incl, 63);
  const u32 misc = gap | ((w_incl - nw) << 5);  // gap, Wb
  PCOUNT(11);
  STAMP(8);

  u32 head = 0, tail = 0;
  u32 op = readlane(V, 0);
  const u32 op_end = readlane(VE, np - 1);
  int sbase = (int)(op & ~15u);  // virtual position of sb[0]
  u32 flushed = op;              // virtual [.., flushed) is in the slots
  u32 fl_j = 0;                  // the first body the flush may still write
  auto zero_from = [&](u32 from) {  // 1 KiB of zeros at a 16-aligned offset
    const u32 i = from + 16 * lane;
    if (i < kWindow + 32) *reinterpret_cast<u32x4*>(sb + i) = u32x4{0, 0, 0, 0};
  };
  zero_from(0);
  u32 zero_end = 1024;
  wave_lds_fence();
  // The ring fill reads kFillWords words of the run at vw, across bodies: the
  // lane's word w = vw + lane / 4 belongs to body fbody (the body holding vw,
  // fcur, or one starting inside the window).  Its load is issued one fill
  // ahead (bmw, with fst = the lane's body | its word index in the body << 8).
  u32 vw = 0, fcur = 0;
  u32 bmw = 0, fst = 0;
  auto fill_load = [&]() {
    const u32 w = vw + (lane >> 2);
    u32 j = fcur, mine = fcur;
    for (;;) {  // bodies starting inside the window (uniform)
      const u32 jn = j + 1;
      if (jn >= np) break;
      const u32 wbn = readlane(misc, jn) >> 5;
      if (wbn >= vw + kFillWords) break;
      mine = w >= wbn ? jn : mine;
      j = jn;
    }
    const u32 wb = lane_bperm(misc, mine) >> 5, bb = lane_bperm(bmb, mine);
    fst = mine | ((w - wb) << 8);
    bmw = w < Wtot ? bitmap[bb + (w - wb)] : 0u;
    // the body holding the next window's first word
    fcur = j + 1 < np && (readlane(misc, j + 1) >> 5) == vw + kFillWords ? j + 1 : j;
  };
  fill_load();
  u32 pf_head = 0xffffffffu, pf_cnt = 0;
  u32x4 pd = u32x4{0, 0, 0, 0};
  u32 pd4 = 0;
  auto prefetch = [&](u32 p, u32 iof) {
    const u32 a = (p + iof) & ~3u;
    pd = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
    pd4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
  };
  // the window's completed bytes [flushed, fe) to their bodies' slots
  auto flush_to = [&](u32 fe) {
    if (fe <= flushed) return;
    u32 j = fl_j;
    while (j < np) {
      const u32 bV = readlane(V, j), bE = readlane(VE, j), bo = readlane(oadj, j);
      if (bE > flushed) {
        const u32 lo_b = flushed > bV ? flushed : bV, hi_b = fe < bE ? fe : bE;
        for (u32 blk = (lo_b & ~15u) + 16 * lane; blk < hi_b; blk += 1024) {
          const u32 lo = blk < lo_b ? lo_b : blk;
          const u32 hi = blk + 16 < hi_b ? blk + 16 : hi_b;
          if (hi - lo == 16) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(sb + ((int)blk - sbase));
            __builtin_memcpy(outb + (blk + bo), &v, 16);
          } else {
            store_exact(outb + (lo + bo), lds_read16(sb + ((int)lo - sbase)), hi - lo);
          }
        }
        if (bE > fe) break;  // the body goes on past fe
      }
      ++j;
    }
    fl_j = j;
    flushed = fe;
  };

  // every iteration fills, takes a long literal or takes >= 1 tag (>= 2
  // input bytes): more iterations than input bytes mean a broken invariant,
  // and the batch's bodies then go to pass 3 (serial, exact)
  const u32 guard_max = wave_max(pk ? n_in : 0u) * 64 + 1024;
  u32 guard = 0;
  for (;;) {
    if (++guard > guard_max) {
      if (pk) status[m] = FSG_PACK_GUARD_STATUS;
      return;
    }
    // ---------- refill the tag ring from the bodies' bitmaps, in order
    if (tail - head < 2 * kMaxPieces && vw < Wtot) {
      u32 bits = (bmw >> (8 * (lane & 3))) & 0xffu;
      const u32 bitbase = (fst >> 8) * 32 + 8 * (lane & 3);
      const u32 cnt = __builtin_popcount(bits);
      const u32 incl = dpp_incl_scan(cnt);
      u32 slot = tail + incl - cnt;
      const u32 hi_bits = (fst & 0xffu) << 24;
      // a body's first tag: the lowest bit of its first word's first byte
      // (the header is at most 5 bytes)
      u32 first = bitbase == 0 ? kFirstTag : 0u;
      while (bits) {
        ring[slot & (kTagRing - 1)] = hi_bits | (bitbase + __builtin_ctz(bits)) | first;
        first = 0;
        ++slot;
        bits &= bits - 1;
      }
      tail += readlane(incl, 63);
      vw += kFillWords;
      fill_load();
      wave_lds_fence();
      STAMP(0);
      continue;
    }
    const u32 avail = tail - head;
    if (avail == 0) break;
    const u32 take0 = avail < 64 ? avail : 64u;
    const bool valid = lane < take0;
    const u32 ent = ring[(head + lane) & (kTagRing - 1)];
    const u32 tj = ent >> 24, pos = ent & (kFirstTag - 1);
    const u32 t_ioff = lane_bperm(ioff, tj);
    if (pf_head != head || pf_cnt < take0) prefetch(pos, t_ioff);

    // ---------- decode one tag per lane (checked by pass 1)
    const u32 s = (pos + t_ioff) & 3u;
    const u32 c = __builtin_amdgcn_alignbyte(pd[1], pd[0], s) & 0xffu;
    const u32 e = tagtab[c];
    const bool q = s == 3;
    const u32 w0 = q ? pd[1] : pd[0], w1 = q ? pd[2] : pd[1], w2 = q ? pd[3] : pd[2];
    const u32 w3 = q ? pd4 : pd[3];
    const u32 b = (s + 1) & 3u;
    const u32x4 xr = u32x4{__builtin_amdgcn_alignbyte(w1, w0, b), __builtin_amdgcn_alignbyte(w2, w1, b),
                           __builtin_amdgcn_alignbyte(w3, w2, b), __builtin_amdgcn_alignbyte(pd4, w3, b)};
    const u32 val = xr[0] & (0xffffffffu >> (e & 31u));
    const bool is_lit = e & 64u;
    const u32 len = (e & 32u) ? val + 1u : (e >> 8) & 0x7fu;
    const u32 off = val + (e >> 20);
    const u32 nb = (e >> 16) & 7u;
    const u32 lsrc = pos + 1 + nb;  // body-relative

    // literals over kMidLit bytes go straight to the slot (below); shorter
    // ones over 64 bytes run inside the group, copied by the whole wave
    const u64 bigm = __ballot(valid && is_lit && len > kMidLit);
    STAMP(1);
    if (bigm & 1ull) {
      // ---------- long literal: straight to the slot by the whole wave; the
      // window restarts behind it (pass 1 checked its length)
      const u32 L = readlane(len, 0), S = readlane(lsrc, 0), j0 = readlane(tj, 0);
      if (readlane(ent, 0) & kFirstTag) op += readlane(misc, j0) & 31u;
      const u32 iof = readlane(ioff, j0), oad = readlane(oadj, j0);
      flush_to(op);
      for (u32 k0 = 0; k0 < L; k0 += 4096) {
        Raw16 x[4];
#pragma unroll
        for (u32 r = 0; r < 4; ++r) x[r] = raw_load16(irsrc, iof + S + k0 + 1024 * r + lane * 16);
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
          const u32 k = k0 + 1024 * r + lane * 16;
          if (k < L) store_exact(outb + (op + k + oad), shifted16(x[r]), L - k < 16 ? L - k : 16u);
        }
      }
      op += L;
      flushed = op;
      sbase = (int)(op & ~15u) - 16;
      zero_from(0);
      zero_end = 1024;
      wave_lds_fence();
      if (lane < 2) {
        const u32 lo = (u32)sbase + 16 * lane;
        if (lo < op) {
          const u32 cnt = op - lo < 16 ? op - lo : 16u;
          store_exact(sb + 16 * lane, rsrc_load16(irsrc, iof + S + L - (op - lo)), cnt);
        }
      }
      wave_lds_fence();
      head += 1;
      pf_head = 0xffffffffu;
      if (head == tail) {  // the bitmap words under the literal hold no tag
        const u32 wl = (readlane(misc, j0) >> 5) + ((S + L) >> 5);
        if (wl > vw) {
          vw = wl;
          fcur = j0;
          fill_load();
        }
      }
      STAMP(7);
      PCOUNT(10);
      continue;
    }
    const u32 take = bigm ? (u32)__builtin_ctzll(bigm) : take0;
    const bool v = lane < take;

    // ---------- output positions (a body's first tag carries the gap to its
    // start): <= kGroupBytes per group
    const u32 t_misc = lane_bperm(misc, tj);
    const u32 g = (ent & kFirstTag) ? t_misc & 31u : 0u;
    const u32 lv = v ? len + g : 0u;
    const u32 incl = dpp_incl_scan(lv);
    const u32 t_op = op + incl - lv + g;
    const bool fits = v && incl <= kGroupBytes && t_op < op_end;
    const u32 k_tags = (u32)__builtin_popcountll(__ballot(fits));
    const u32 tot_len = readlane(incl, k_tags - 1);
    // the writer's checks (snappy.cc:1166, :1200, :1400, :1410, :1466) against
    // the tag's body; a failing tag marks its body and writes nothing
    const u32 t_V = lane_bperm(V, tj), t_VE = lane_bperm(VE, tj);
    const bool bad = fits && (len > t_VE - t_op || (!is_lit && (off == 0 || off > t_op - t_V)));
    const u32 t_m = lane_bperm(bm_id, tj);
    if (__ballot(bad)) {
      if (bad) status[t_m] = kCorrupt;
    }
    const bool run = fits && !bad;
    const bool mid = run && is_lit && len > 64;  // a literal of 65..kMidLit bytes

    // ---------- slide the window if this group would overrun it
    if (op + tot_len - sbase > kWindow) {
      const int nsb = (int)((op - keep_hist) & ~15u);
      if ((int)flushed < nsb + 16) flush_to(op & ~15u);
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
    auto prefetch_next_and_zero = [&]() {
      {
        const u32 nh = head + k_tags;
        const u32 na = tail - nh;
        const u32 ncnt = na < 64 ? na : 64u;
        const u32 nent = ring[(nh + lane) & (kTagRing - 1)];
        prefetch(nent & (kFirstTag - 1), lane_bperm(ioff, nent >> 24));
        pf_head = nh;
        pf_cnt = ncnt;
      }
      while (op + tot_len + 20 - sbase > zero_end) {
        zero_from(zero_end);
        zero_end += 1024;
      }
      wave_lds_fence();
    };

    STAMP(2);
    // ---------- chunks (as exec5_message; far sources through the slots' buffer)
    const u32 src = is_lit ? lsrc : t_op - off;
    const u32 nch = (len + 15) >> 4;
    const bool pat = !is_lit && off < 16 && off < len;
    const u32 below = (u32)(sbase - (int)src);  // > 0 as int: far
    const u32 kfar = (int)below > 0 ? ((below - 1) >> 4) + 1 : 0u;
    const u32 kready = src + len <= op ? nch : (src < op ? (op - src) >> 4 : 0u);
    const u32 klead = kfar > kready ? kfar : kready;
    const u32 kc = pat ? 0u : (klead < nch ? klead : nch);
    const u32 kf = run && !mid ? (is_lit ? nch : kc) : 0u;
    const bool reg0 = is_lit && nb == 0;
    const u32 t_oadj = lane_bperm(oadj, tj);
    const u32 sh = is_lit ? (src + t_ioff) & 3u : 0u;
    auto gload = [&](u32 k, u32x4& d, u32& d4) {
      if (is_lit) {
        const u32 a = (src + 16 * k + t_ioff) & ~3u;
        d = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
        d4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
      } else if (k >= kfar) {
        d = lds_read16(sb + ((int)(src + 16 * k) - sbase));
      } else {
        d = far_load(orsrc, src + 16 * k + t_oadj);
      }
    };
    auto shf = [&](const u32x4& d, u32 d4, u32 t) {
      return u32x4{__builtin_amdgcn_alignbyte(d[1], d[0], t), __builtin_amdgcn_alignbyte(d[2], d[1], t),
                   __builtin_amdgcn_alignbyte(d[3], d[2], t), __builtin_amdgcn_alignbyte(d4, d[3], t)};
    };
    u32x4 a0 = xr, a1 = u32x4{0, 0, 0, 0};
    u32 a0e = 0, a1e = 0;
    if (kf > 0 && !reg0) gload(0, a0, a0e);
    const u64 m1 = __ballot(kf > 1);
    if (m1 && kf > 1) gload(1, a1, a1e);
    // the group's first literal over 64 bytes: chunk i by lane i, loaded with
    // the other round-A loads
    const u64 ML = __ballot(mid);
    u32x4 md = u32x4{0, 0, 0, 0};
    u32 md4 = 0, mcnt = 0, mw = 0, msh = 0;
    auto mid_load = [&](u32 L0) {
      const u32 ms = readlane(lsrc, L0) + readlane(t_ioff, L0);
      const u32 ml = readlane(len, L0);
      const u32 k = 16 * lane;
      msh = ms & 3u;
      mcnt = 0;
      if (k < ml) {
        const u32 a = (ms + k) & ~3u;
        md = __builtin_amdgcn_raw_buffer_load_b128(irsrc, a, 0, 0);
        md4 = __builtin_amdgcn_raw_buffer_load_b32(irsrc, a + 16, 0, 0);
        mcnt = ml - k < 16 ? ml - k : 16u;
        mw = (u32)((int)readlane(t_op, L0) - sbase) + k;
      }
    };
    if (ML) mid_load((u32)__builtin_ctzll(ML));
    prefetch_next_and_zero();
    STAMP(3);
    {
      const u32 fe = op & ~15u;
      if (fe >= flushed + 1024) flush_to(fe);
    }
    STAMP(4);
    const u32 wa = (u32)((int)t_op - sbase);
    if (kf > 0) or_store(sb, wa, shf(a0, a0e, reg0 ? 0u : sh), len < 16 ? len : 16u, mtab);
    if (m1) {
      if (kf > 1) or_store(sb, wa + 16, shf(a1, a1e, sh), len - 16 < 16 ? len - 16 : 16u, mtab);
      if (__ballot(kf > 2)) {
        if (kf > 2) gload(2, a0, a0e);
        if (kf > 3) gload(3, a1, a1e);
        if (kf > 2) or_store(sb, wa + 32, shf(a0, a0e, sh), len - 32 < 16 ? len - 32 : 16u, mtab);
        if (kf > 3) or_store(sb, wa + 48, shf(a1, a1e, sh), len - 48, mtab);
      }
    }
    if (ML) {
      if (mcnt) or_store(sb, mw, shf(md, md4, msh), mcnt, mtab);
      for (u64 rest = ML & (ML - 1); rest; rest &= rest - 1) {  // more of them (rare)
        mid_load((u32)__builtin_ctzll(rest));
        if (mcnt) or_store(sb, mw, shf(md, md4, msh), mcnt, mtab);
      }
    }
    wave_lds_fence();

    STAMP(5);
    // ---------- rounds B (as exec5_message)
    u32 rem = (run && !mid && kf < nch) ? len - 16 * kf : 0u;
    u32 cw = (u32)((int)t_op - sbase) + 16 * kf;
    u32 sw = (u32)((int)src - sbase) + 16 * kf;
    const u32 stp = pat ? pat_step(off) : 16u;
    u32 n = rem < stp ? rem : stp;
    bool pf = pat;
    u32 ne = rem ? (pf ? cw : sw + n) : 0xffffffffu;
    u64 pend = __ballot(rem > 0);
    if (!__ballot(pat && rem > 0)) {
      while (pend) {
        const u32 W = readlane(cw, (u32)__builtin_ctzll(pend));
        if (ne <= W) {
          const u32x4 x = lds_read16(sb + sw);
          const u32x4 o = lds_read16(sb + cw);
          const u32x4 mk = mtab[n];
          u32x4 y;
          y[0] = (x[0] & mk[0]) | (o[0] & ~mk[0]);
          y[1] = (x[1] & mk[1]) | (o[1] & ~mk[1]);
          y[2] = (x[2] & mk[2]) | (o[2] & ~mk[2]);
          y[3] = (x[3] & mk[3]) | (o[3] & ~mk[3]);
          __builtin_memcpy(sb + cw, &y, 16);
          rem -= n;
          cw += n;
          sw += n;
          n = rem < 16u ? rem : 16u;
          ne = rem ? sw + n : 0xffffffffu;
        }
        wave_lds_fence();
        pend = __ballot(rem > 0);
      }
    }
    while (pend) {
      const u32 W = readlane(cw, (u32)__builtin_ctzll(pend));
      if (ne <= W) {
        u32x4 x = lds_read16(sb + sw);
        if (pf) x = expand_pattern(x, off, sel_tab);
        const u32x4 o = lds_read16(sb + cw);
        const u32x4 mk = mtab[n];
        u32x4 y;
        y[0] = (x[0] & mk[0]) | (o[0] & ~mk[0]);
        y[1] = (x[1] & mk[1]) | (o[1] & ~mk[1]);
        y[2] = (x[2] & mk[2]) | (o[2] & ~mk[2]);
        y[3] = (x[3] & mk[3]) | (o[3] & ~mk[3]);
        __builtin_memcpy(sb + cw, &y, 16);
        rem -= n;
        cw += n;
        sw = pat ? cw - stp : sw + n;
        pf = false;
        n = rem < stp ? rem : stp;
        ne = rem ? sw + n : 0xffffffffu;
      }
      wave_lds_fence();
      pend = __ballot(rem > 0);
    }
    op += tot_len;
    head += k_tags;
    STAMP(6);
    PCOUNT(9);
  }
  flush_to(op);
#ifdef FSG_STAMPS
  STAMP(4);
  if (lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd(&g_stamps[8 + k], (unsigned long long)st_[k]);
#endif
  (void)op_end;
}


// 7 waves per SIMD by default (FSG_EXEC_WAVES; 72 VGPRs, 22.2 KB of LDS per
// block with the 3 KiB window: C3 6.35 -> 6.20 ms against 6 waves with a
// 4 KiB window, A/B on one box; 8 waves spill and were slower).
// The v4 variant (exec_kernel<4>) shares the setting and was not re-measured
// at 7.
// The first kBigBlocks blocks take the large messages listed by pass 1 from a
// device counter (blocks dispatch in order, so the longest messages start
// first); every other block runs the wave-per-message mapping and skips them.
// (A fully persistent grid was measured slower on uniform batches.)
#ifndef FSG_EXEC_WAVES
#define FSG_EXEC_WAVES 7
#endif
template <int V>
__global__ __launch_bounds__(kWavesPerBlock * 64) __attribute__((amdgpu_waves_per_eu(FSG_EXEC_WAVES, FSG_EXEC_WAVES))) void exec_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len,
    i32* __restrict__ status, const u32* __restrict__ bm_base,
    u32* __restrict__ bitmap, const u32* __restrict__ seg_list,
    const u32* __restrict__ seg_count, const u32* __restrict__ whole_list,
    const u32* __restrict__ whole_count, u32* __restrict__ exec_next, u32 big_blocks,
    u32 big_threshold, u32 prio, u32 keep_hist, u32 small_stride, const u32* __restrict__ walk_perm = nullptr,
    const u32* __restrict__ walk_hist = nullptr, u32 walk_part = 0, u32 split_class = 0) {
  // per wave: the tag ring, then the output window
  __shared__ __attribute__((aligned(16))) u8 wl_s[kWavesPerBlock][4 * kTagRing + kWindow + 32];
  __shared__ __attribute__((aligned(16))) u8 pmap_s[kWavesPerBlock][V == 5 ? 1 : kMaxPieces];
  __shared__ u32x4 sel_tab[16];
  __shared__ u32 tagtab[V == 5 ? 256 : 1];
  __shared__ u32x4 mask_tab[17];
  static_assert(kWavesPerBlock * 64 == 256, "one tag table entry per thread");

  if (threadIdx.x < 64) init_pattern_table(sel_tab, threadIdx.x);
  if constexpr (V == 5) tagtab[threadIdx.x] = exec_tag_entry(threadIdx.x);
  init_mask_table(mask_tab, threadIdx.x);
  __syncthreads();
  // one message (or segment) with the pass-2 variant V
  auto run = [&](u32 m, u32* ring, u8* pmap, u8* sb, u32 lane, i32 st, u32 ip0, u32 op0, u32 op1) {
    if constexpr (V == 5)
      exec5_message(m, in, in_off, in_len, out, out_off, out_len, status, bm_base, bitmap, ring, tagtab,
                    sb, sel_tab, mask_tab, lane, st, ip0, op0, op1, prio != 0, keep_hist);
    else
      exec_message(m, in, in_off, in_len, out, out_off, out_len, status, bm_base, bitmap, ring, pmap,
                   sb, sel_tab, mask_tab, lane, st, ip0, op0, op1, prio != 0, keep_hist);
  };

  // wave index made visibly uniform: the message's sizes, pointers and the
  // walk state (head, tail, op, window base) then live in SGPRs and branches
  // on them are scalar
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  u32* ring = reinterpret_cast<u32*>(wl_s[wv]);
  u8* pmap = pmap_s[wv];
  u8* sb = wl_s[wv] + 4 * kTagRing;

  if (blockIdx.x >= big_blocks) {
    // one message per wave; or, with small_stride (blocks), every
    // small_stride-th group of kWavesPerBlock messages: a wave runs many
    // small messages, paying its launch and the block's table set-up once
    // (the forked path's batches of mostly small bodies)
    const u32 m0 = (blockIdx.x - big_blocks) * kWavesPerBlock + wv;
    const u32 step = small_stride ? small_stride * kWavesPerBlock : 0xffffffffu;
    if (walk_perm) {
      // the messages in walk order (forked path): positions [lo, hi) of
      // walk_perm -- part 1 / 2 the larger / smaller bodies, 3 all of them
      const u32 n_walk = walk_hist[2 * kWalkClasses];
      // (split_class bits 8-15: the first class another pass takes, whose
      // positions on are not executed here; no pass sets it now)
      const u32 tcls = split_class >> 8;
      const u32 split = walk_hist[kWalkClasses + (split_class & 0xffu)];
      const u32 t_hi = tcls ? walk_hist[kWalkClasses + tcls] : n_walk;
      const u32 lo = walk_part == 2 ? split : 0u, hi = walk_part == 1 ? split : t_hi;
      for (u32 i = m0; i < hi - lo; i = i + step < i ? 0xffffffffu : i + step) {
        const u32 m = walk_perm[lo + i];
        run(m, ring, pmap, sb, lane, status[m], 0u, 0u, out_len[m]);
      }
      return;
    }
    for (u32 m = m0; m < n_msgs; m = m + step < m ? 0xffffffffu : m + step)
      if (in_len[m] <= big_threshold) run(m, ring, pmap, sb, lane, status[m], 0u, 0u, out_len[m]);
    return;
  }
  // large messages, listed by pass 1b: whole ones first (the longest start
  // first), then 64 KiB segments of the others
  const u32 n_whole = *whole_count;
  const u32 n_seg_raw = *seg_count;
  const u32 n_seg = n_seg_raw < n_msgs ? n_seg_raw : n_msgs;
  const u32 total = n_whole + n_seg;
  if (total == 0) return;
  const u64* segs = reinterpret_cast<const u64*>(seg_list);
  for (;;) {  // all-lane atomic: lane 0 adds 1, lane 0's result is the index
    const u32 got = atomicAdd(exec_next, lane == 0 ? 1u : 0u);
    const u32 idx = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (idx >= total) break;
    if (idx < n_whole) {
      const u32 m = whole_list[idx];
      run(m, ring, pmap, sb, lane, status[m], 0u, 0u, out_len[m]);
      continue;
    }
    const u64 e = segs[idx - n_whole];
    const u32 m = (u32)e;
    if (m == 0xffffffffu) continue;  // a hole (the message runs whole)
    const u32 k = (u32)(e >> 32) & 0x7fffffffu;
    const u32 expected = out_len[m];
    const u32 op0 = k << 16;
    const u32 op1 = (e >> 63) ? expected : op0 + 65536u;
    u32 ip0 = 0;  // segment k > 0 starts at the input offset pass 1b left in its slot
    if (k) __builtin_memcpy(&ip0, out + out_off[m] + op0, 4);
    run(m, ring, pmap, sb, lane, status[m], ip0, op0, op1);
  }
}

// The packed execution pass (exec5_packed) over walk part 2 (the bodies of
// size class >= split_class): batches of `batch` consecutive walk positions
// from a work counter.
#ifndef FSG_PACK_WAVES
#define FSG_PACK_WAVES 6
#endif
__global__ __launch_bounds__(kWavesPerBlock * 64) __attribute__((amdgpu_waves_per_eu(FSG_PACK_WAVES, FSG_PACK_WAVES))) void exec_packed_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len, i32* __restrict__ status,
    const u32* __restrict__ bm_base, const u32* __restrict__ bitmap, const u32* __restrict__ walk_perm,
    const u32* __restrict__ walk_hist, u32 split_class, u32* __restrict__ batch_next, u32 batch, u32 keep_hist) {
  __shared__ __attribute__((aligned(16))) u8 wl_s[kWavesPerBlock][4 * kTagRing + kWindow + 32];
  __shared__ u32x4 sel_tab[16];
  __shared__ u32 tagtab[256];
  __shared__ u32x4 mask_tab[17];
  static_assert(kWavesPerBlock * 64 == 256, "one tag table entry per thread");
  if (threadIdx.x < 64) init_pattern_table(sel_tab, threadIdx.x);
  tagtab[threadIdx.x] = exec_tag_entry(threadIdx.x);
  init_mask_table(mask_tab, threadIdx.x);
  __syncthreads();
  const u32 wv = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const u32 lane = threadIdx.x & 63;
  u32* ring = reinterpret_cast<u32*>(wl_s[wv]);
  u8* sb = wl_s[wv] + 4 * kTagRing;
  const u32 n_walk = walk_hist[2 * kWalkClasses];
  const u32 tcls = split_class >> 8;
  const u32 lo = walk_hist[kWalkClasses + (split_class & 0xffu)];
  const u32 hi = tcls ? walk_hist[kWalkClasses + tcls] : n_walk;
  const u32 n = hi > lo ? hi - lo : 0u;
  for (;;) {
    const u32 got = atomicAdd(batch_next, lane == 0 ? 1u : 0u);
    const u32 bi = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if ((u64)bi * batch >= n) break;
    const u32 first = bi * batch;
    const u32 cnt = n - first < batch ? n - first : batch;
    exec5_packed(in, in_off, in_len, out, out_off, out_len, status, bm_base, bitmap, walk_perm, lo + first, cnt,
                 ring, tagtab, sb, sel_tab, mask_tab, lane, keep_hist);
  }
}

#ifdef FSG_STAMPS
extern "C" int fsg_debug_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
  if (reset) {
    unsigned long long z[24] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  return e == hipSuccess ? 0 : -1;
}
#endif

// Pass 3: the messages whose bitmap did not fit the workspace (status
// kNeedFallback, header and slot already checked by pass 1), one lane each,
// with the reference's serial tag loop.  A lean grid-sized launch: no LDS, a
// status load per lane.  (Measured: a grid-sized launch here keeps the next
// call's passes at full speed on C3, a one-block launch or none does not --
// DESIGN.md section 5; the former v3 fallback launch cost 14 us more on C2.)
__global__ __launch_bounds__(64) void fallback_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len,
    u32 n_msgs, u8* out, const u64* __restrict__ out_off, const u32* __restrict__ out_len,
    i32* __restrict__ status, u32 flags) {
  const u32 m = blockIdx.x * 64 + threadIdx.x;
  if (m >= n_msgs || status[m] != kNeedFallback) return;
  const u8* ib = in + in_off[m];
  const u32 n_in = in_len[m];
  u32 ulen = 0;
  const int h = parse_varint_header(ib, n_in, flags & 2u, &ulen);
  status[m] = decode_one(ib + h, ib + n_in, out + out_off[m], out_len[m], true);
}

// Workspace layout (bytes from the start; every counter a u32, zeroed by the
// launch's one fill together with the lists):
//   [0, 256)  counters, at the kWs* offsets below
//   then kListBases arrays of base_bytes = round_up(4 n, 256) bytes each:
//     0 bm_base[n] | 1 big_list[n] | 2-3 seg_list[n] (u64) | 4 whole_list[n] |
//     5 walk_rank[n] | 6 walk_perm[n] | 7 walk_hist (16 classes + count) |
//     8-9 seg_list2[n] (u64) | 10 whole_list2[n]
//   then the tag-start bitmap words.
// Set 0 = every large message (one stream) or the non-huge ones (forked);
// set 1 = the huge ones (forked, second side stream).
constexpr u32 kWsBmCounter = 0;        // bitmap bump allocator
constexpr u32 kWsSet1BigNext = 16;     // set 1: pass-1b work counter
constexpr u32 kWsSet1SegCount = 32;    // set 1: segment count
constexpr u32 kWsSet1WholeCount = 48;  // set 1: whole-message count
constexpr u32 kWsBigCount = 64;        // large-message count (huge count at +32: big_count + 8)
constexpr u32 kWsHugeCount = kWsBigCount + 32;
constexpr u32 kWsSet0BigNext = 128;
constexpr u32 kWsSet0SegCount = 160;
constexpr u32 kWsSet0ExecNext = 192;   // pass-2 queue head
constexpr u32 kWsSet0WholeCount = 224;
constexpr u32 kWsSet1ExecNext = 240;
constexpr u32 kWsChunkCount = 80;      // chunked pass 1b: records listed
constexpr u32 kWsChunkSpecNext = 84;   //   work counters of its passes
constexpr u32 kWsChunkFixNext = 88;
constexpr u32 kWsChunkCheckNext = 92;
constexpr u32 kWsChunkFinalNext = 100;
constexpr u32 kWsPackNext = 104;      // packed execution: batch counter
constexpr u32 kWsCounterBytes = 256;
// the counters are distinct u32 slots inside the 256-byte header
constexpr u32 kWsOffsets[] = {kWsBmCounter, kWsSet1BigNext, kWsSet1SegCount, kWsSet1WholeCount, kWsBigCount,
                              kWsHugeCount, kWsSet0BigNext, kWsSet0SegCount, kWsSet0ExecNext, kWsSet0WholeCount,
                              kWsSet1ExecNext, kWsChunkCount, kWsChunkSpecNext, kWsChunkFixNext,
                              kWsChunkCheckNext, kWsChunkFinalNext, kWsPackNext};
constexpr bool ws_offsets_ok() {
  for (u32 i = 0; i < sizeof(kWsOffsets) / sizeof(kWsOffsets[0]); ++i) {
    if (kWsOffsets[i] % 4 || kWsOffsets[i] + 4 > kWsCounterBytes) return false;
    for (u32 j = 0; j < i; ++j)
      if (kWsOffsets[i] < kWsOffsets[j] + 4 && kWsOffsets[j] < kWsOffsets[i] + 4) return false;
  }
  return true;
}
static_assert(ws_offsets_ok(), "workspace counters overlap or leave the header");
constexpr u64 kListBases = 11;  // u32 arrays of n entries before the bitmap
// The chunked pass 1b's records live at the workspace's end: 1/64 of it
// (>= 40 bytes per 20 KiB of input: one 32-byte record per 32 KiB chunk plus
// two words per huge message).
constexpr u64 kChunkRegionDiv = 64;
size_t decode_v4_workspace_bytes(u32 n_msgs, u64 total_in_bytes) {
  const u64 base_bytes = (4ull * n_msgs + 255) & ~255ull;
  const u64 words = total_in_bytes / 32 + 4ull * n_msgs + 64;
  const u64 base = 256 + kListBases * base_bytes + 4 * words;
  return (size_t)(base + base / (kChunkRegionDiv - 1) + 512);
}

// Per-device side stream and fork/join events for launch_decode_v4 (created
// on first use; the mutex orders each call's record/wait pairs when several
// host threads decode at once).  nullptr when they cannot be created: the
// passes then run in one stream.
struct SideStream {
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // the huge messages' pass 1b + execution (nullptr: not created)
  hipEvent_t join2 = nullptr;
  hipStream_t stream3 = nullptr;  // the larger small bodies' walk + execution (split walk)
  hipEvent_t join3 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  hipEvent_t pass1 = nullptr;  // two-stream calls: pass 1 done (fsg_decompress_batch_2s)
  std::mutex mu;
};
static SideStream* side_stream() {
  constexpr int kMaxDevices = 64;
  static SideStream g_side[kMaxDevices];
  static std::once_flag g_once[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  SideStream* s = &g_side[dev];
  std::call_once(g_once[dev], [s] {
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->pass1, hipEventDisableTiming) != hipSuccess)
      s->stream = nullptr;
    // optional second side stream (the huge messages of a forked batch)
    if (s->stream && (hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking) != hipSuccess ||
                      hipEventCreateWithFlags(&s->join2, hipEventDisableTiming) != hipSuccess))
      s->stream2 = nullptr;
    if (s->stream && (hipStreamCreateWithFlags(&s->stream3, hipStreamNonBlocking) != hipSuccess ||
                      hipEventCreateWithFlags(&s->join3, hipEventDisableTiming) != hipSuccess))
      s->stream3 = nullptr;
  });
  return s->stream ? s : nullptr;
}

// Dynamic LDS of the lean lane walk: per wave an 8-chunk input ring (+5
// dwords) and 2 bit groups, [dword][lane]; the 256-entry tag table.
constexpr size_t idx_lean_lds_bytes() { return 4 * (kIdxWaves * (8 * 4 + 5 + 8) * kWave + 256); }

hipError_t launch_decode_v4(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, void* ws, size_t ws_bytes, hipStream_t stream,
                            int exec_variant, hipStream_t pass1_stream) {
  if (n_msgs == 0) return hipSuccess;
  // Two-stream form: pass 1 (fill, lane walk, pass 1b) on pass1_stream, pass 2
  // (exec, fallback) on `stream` behind an event, so a caller's next batch
  // (its own workspace and outputs) can walk while this one executes.
  SideStream* two = nullptr;
  if (pass1_stream && pass1_stream != stream) {
    two = side_stream();
    if (!two) {
      // No per-device event set: order `stream` behind whatever the caller
      // queued on pass1_stream with a temporary event and run every pass on
      // `stream` (as capi.hip's single-pass path does).
      hipEvent_t ev = nullptr;
      hipError_t e0 = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (e0 == hipSuccess) e0 = hipEventRecord(ev, pass1_stream);
      if (e0 == hipSuccess) e0 = hipStreamWaitEvent(stream, ev, 0);
      if (ev) (void)hipEventDestroy(ev);
      if (e0 != hipSuccess) return e0;
      pass1_stream = nullptr;
    }
  }
  hipStream_t const caller_stream = stream;
  // planned lane walk in size-class order (FSG_WALK_ORDER=0 disables)
  // (options: csrc/options.h, set with fsg_set_option; never the environment here)
  const bool kSplitHuge = opt(kOptSplitHuge) != 0;  // 0: one side stream
  const bool kWalkOrder = opt(kOptWalkOrder) != 0;
  // Two-stream form: the lean lane walk (FSG_LEAN_WALK=0: the standard one).
  // Measured (C3, stream of two alternating batches, one box): lean 6.13 ms
  // per batch, standard 6.57, serial 6.15; an execution pass made persistent
  // at 5 or 6 blocks per CU to leave wave slots for the walk: 6.38 / 7.25
  // (the dispatcher does not spread a persistent grid evenly); the execution
  // pass held to six blocks per CU by padding its LDS, with a two-wave lean
  // walk in the space left: 6.32 vs serial 6.11 (the walk's instructions
  // compete with an execution pass already at the issue limit).
  const bool kLeanWalk = opt(kOptLeanWalk) != 0;
  if (two) stream = pass1_stream;  // every pass-1 launch below goes there
  // pass 2: one tag per lane (5) or <= 16-byte pieces per lane (4)
  auto* const ek = exec_variant == 4 ? &exec_kernel<4> : &exec_kernel<5>;
  u8* w = static_cast<u8*>(ws);
  const u64 base_bytes = (4ull * n_msgs + 255) & ~255ull;
  // the fixed part, the chunk-record region and a bitmap of at least the
  // per-message minimum (decode_v4_workspace_bytes with no input): below it
  // the region arithmetic below would underflow
  if (ws_bytes < decode_v4_workspace_bytes(n_msgs, 0)) return hipErrorInvalidValue;
  u32* counter = reinterpret_cast<u32*>(w + kWsBmCounter);
  u32* big_count = reinterpret_cast<u32*>(w + kWsBigCount);
  u32* bm_base = reinterpret_cast<u32*>(w + 256);
  u32* big_list = reinterpret_cast<u32*>(w + 256 + base_bytes);
  u64* seg_list = reinterpret_cast<u64*>(w + 256 + 2 * base_bytes);
  u32* whole_list = reinterpret_cast<u32*>(w + 256 + 4 * base_bytes);
  // the planned lane walk's order: ranks, the permutation, class counts and
  // offsets (+ the walk count)
  u32* walk_rank = reinterpret_cast<u32*>(w + 256 + 5 * base_bytes);
  u32* walk_perm = reinterpret_cast<u32*>(w + 256 + 6 * base_bytes);
  u32* walk_hist = reinterpret_cast<u32*>(w + 256 + 7 * base_bytes);
  // the huge messages' pass-2 work lists (forked path, second side stream)
  u64* seg_list2 = reinterpret_cast<u64*>(w + 256 + 8 * base_bytes);
  u32* whole_list2 = reinterpret_cast<u32*>(w + 256 + 10 * base_bytes);
  u32* bitmap = reinterpret_cast<u32*>(w + 256 + kListBases * base_bytes);
  // chunk records (chunked pass 1b) at the end, the bitmap before them
  // (256-byte aligned whatever ws_bytes: the passes load its records with
  // scalar loads, which ignore the low address bits)
  const u64 chunk_bytes = (ws_bytes / kChunkRegionDiv) & ~255ull;
  const u64 chunk_off = (ws_bytes - chunk_bytes) & ~255ull;
  u8* const chunk_region = w + chunk_off;
  u64 cap_words = (chunk_off - 256 - kListBases * base_bytes) / 4;
  if (cap_words >= kSingleLiteral) cap_words = kSingleLiteral - 1;  // bases < 2^31 words
  // zero the counters and the bitmap (pass 1 writes only groups holding
  // tags) with one fill from the counters to the end of the bitmap: the
  // lists between them are 20 B per message (A/B: C2 0.159 -> 0.157 ms, C3
  // and CM neutral; a zeroing kernel in place of the runtime fill makes the
  // next index pass place its one-wave workgroups unevenly: C3 +0.27 ms)
  // counters and lists only: the passes that write the bitmap store every
  // word the execution pass reads (C3: an 80 us fill of 267 MB saved)
  hipError_t e = hipMemsetAsync(w, 0, 256 + kListBases * base_bytes, stream);
  if (e != hipSuccess) return e;
  // Large-message threshold: 4x the batch's mean compressed size (estimated
  // from the workspace, which callers size from the packed input), clamped
  // to [8, 48] KiB.  The lane pass's time is its longest message; uniform
  // batches (C2, C3) send nothing to the wave pass.
  const u64 est_total_in = cap_words > 4ull * n_msgs + 64 ? (cap_words - 4ull * n_msgs - 64) * 32 : 0;
  u64 thr = 4 * est_total_in / n_msgs;
  thr = thr < kBigIndexMin ? kBigIndexMin : (thr > kBigIndexMax ? kBigIndexMax : thr);
  // A batch of at most one wave of messages (the host runtime's one-caller
  // batches): the lane walk would be one lane per message, its latency the
  // longest message's tag chain (~160 us for a 4 KiB text body), where pass
  // 1b walks each message with a whole wave (a few us).  Every message goes
  // to pass 1b (option small_batch sets the bound; 0 disables).
  const i64 kSmallBatch = opt(kOptSmallBatch);
  if ((i64)n_msgs <= kSmallBatch) thr = 0;
  const u32 big_threshold = (u32)thr;
  const u32 idx_blocks = (n_msgs + 64 * kIdxWaves - 1) / (64 * kIdxWaves);
  // Order of the forked path's small-message execution.  The split point:
  // bodies of size class >= kSplitClass (compressed size < 2^(16 -
  // kSplitClass) bytes; option split_class) vs the larger ones.
  // Option split_walk (A/B): 0 the execution in message order
  // after one walk; 1 the walk and execution split on two streams (above);
  // 2 one walk, then the execution in walk order (size classes, largest
  // first); 3 (default) one walk, then the smaller bodies' execution, then
  // the larger ones'.  CM, A/B on one box, two rounds, with the chunked
  // huge-body walk: 0 6.74 / 6.72, 1 (unchunked) 7.54 / 7.45 -- the third
  // stream shares a hardware queue with the huge bodies' stream and waits
  // behind it --, 2 6.55 / 6.45, 3 6.45 / 6.44 ms.  In message order a
  // wave's run of bodies mixes sizes and the launch waits for the waves that
  // drew the larger ones (execution 4.66 ms; in walk order 3.91).
  const u32 split_mode = (u32)opt(kOptSplitWalk);
  const bool split_walk = split_mode == 1;
  const u32 kSplitClass = (u32)opt(kOptSplitClass) % kWalkClasses;
  auto launch_index = [&](bool planned, hipStream_t st = nullptr, u32 part = 0) -> hipError_t {
    if (planned)
      index_kernel<true><<<idx_blocks, 64 * kIdxWaves, 0, st ? st : stream>>>(
          in, in_off, in_len, n_msgs, out_cap, out_len, status, flags, counter, bm_base, bitmap,
          cap_words, big_count, big_list, big_threshold, kWalkOrder ? walk_perm : nullptr, walk_hist, part,
          kSplitClass);
    else if (two && kLeanWalk)
      index_kernel<false, true><<<idx_blocks, 64 * kIdxWaves, idx_lean_lds_bytes(), stream>>>(
          in, in_off, in_len, n_msgs, out_cap, out_len, status, flags, counter, bm_base, bitmap,
          cap_words, big_count, big_list, big_threshold, nullptr, nullptr);
    else if (est_total_in < 16384ull * n_msgs)
      index_kernel<false, false, kIdxWavesSerial><<<(n_msgs + 64 * kIdxWavesSerial - 1) / (64 * kIdxWavesSerial),
                                                    64 * kIdxWavesSerial, 0, stream>>>(
          in, in_off, in_len, n_msgs, out_cap, out_len, status, flags, counter, bm_base, bitmap,
          cap_words, big_count, big_list, big_threshold, nullptr, nullptr);
    else
      index_kernel<false><<<idx_blocks, 64 * kIdxWaves, 0, stream>>>(
          in, in_off, in_len, n_msgs, out_cap, out_len, status, flags, counter, bm_base, bitmap,
          cap_words, big_count, big_list, big_threshold, nullptr, nullptr);
    return hipGetLastError();
  };
  // Pass 1b and the large-message exec blocks run on a side stream, after a
  // plan pass (headers, bitmap bases, the large-message list) and beside the
  // lane walk and the one-wave-per-message exec launch: pass 1b is bound by
  // the serial window walk of the few largest bodies and leaves most CUs
  // idle, which the small messages' passes fill.  Both streams join before
  // the fallback pass.
  // Only for batches of > 128K messages (the mixed-size ones): a fork and
  // join cost ~10 us (C2 0.159 -> 0.169 ms), and uniform batches send nothing
  // to pass 1b (CM 14.4 -> 12.1 ms).  Option decode_fork 0/1 forces (A/B).
  const u32 small_blocks = (n_msgs + kWavesPerBlock - 1) / kWavesPerBlock;
  // A/B knob; at least one block: the large-message lists are only drained there
  const i64 big_opt = opt(kOptExecBigBlocks);
  const u32 kBigBlocks = big_opt >= 1 && big_opt <= (1 << 20) ? (u32)big_opt : 512u;
  const u32 kPrio = opt(kOptExecPrio) != 0 ? 1u : 0u;  // A/B knob: 0 disables the priority raise
  // history kept when an exec window slides (option exec_keep: the tests
  // shrink it to exercise the slide's flush rule; 512..kMaxKeep bytes, a
  // multiple of 16; anything else is the default)
  u32 keep_hist = kKeep;
  {
    const i64 v = opt(kOptExecKeep);
    if (v >= 512 && v <= (i64)kMaxKeep && v % 16 == 0) keep_hist = (u32)v;
  }
  const i64 fork_opt = opt(kOptDecodeFork);
  const bool fork = !two && (fork_opt >= 0 ? fork_opt != 0 : n_msgs > 131072u);
  const u32 big_blocks = small_blocks < kBigBlocks ? small_blocks : kBigBlocks;
  // pass 1b: large messages, one wave each (an empty list costs one short
  // launch); they land in pass 2's work lists.  set 0: every large message
  // (one stream) or the non-huge ones (forked); set 1: the huge ones (forked,
  // second side stream), with their own counters and lists.
  struct BigSet {
    u32 *big_next, *seg_count, *whole_count, *exec_next;
    u64* seg_list;
    u32* whole_list;
  };
  const BigSet set0{reinterpret_cast<u32*>(w + kWsSet0BigNext), reinterpret_cast<u32*>(w + kWsSet0SegCount),
                    reinterpret_cast<u32*>(w + kWsSet0WholeCount), reinterpret_cast<u32*>(w + kWsSet0ExecNext),
                    seg_list, whole_list};
  const BigSet set1{reinterpret_cast<u32*>(w + kWsSet1BigNext), reinterpret_cast<u32*>(w + kWsSet1SegCount),
                    reinterpret_cast<u32*>(w + kWsSet1WholeCount), reinterpret_cast<u32*>(w + kWsSet1ExecNext),
                    seg_list2, whole_list2};
  auto launch_index_big_set = [&](hipStream_t st, const BigSet& b, u32 mode) -> hipError_t {
    const u32 q = (n_msgs + 3) / 4;
    const u32 blocks = q < 1024u ? q : 1024u;
    index_big_kernel<<<blocks, 256, 0, st>>>(
        in, in_off, in_len, out_len, flags, status, bm_base, bitmap, big_count, big_list,
        b.big_next, n_msgs, out, out_off, b.seg_list, b.seg_count, b.whole_list, b.whole_count, mode);
    return hipGetLastError();
  };
  auto launch_index_big = [&](hipStream_t st) -> hipError_t { return launch_index_big_set(st, set0, 0u); };
  // The forked path's large-message launches: CM 9.9 -> 8.85 ms with 1,792
  // blocks against 512 when they ran alone after the lane walk; 1,024 since
  // the small bodies' execution (walk order, 3,584 blocks) runs beside them:
  // CM 6.32-6.37 -> 6.20-6.25 ms for the two grid sizes together (A/B on one
  // box, four rounds).
  const i64 bbf_opt = opt(kOptExecBigBlocksFork);  // A/B knob, separate from the one-stream launch's
  const u32 kBigBlocksFork = bbf_opt >= 1 && bbf_opt <= (1 << 20) ? (u32)bbf_opt : 1024u;
  auto launch_big = [&](hipStream_t st, const BigSet& b, u32 mode) -> hipError_t {
    hipError_t e2 = launch_index_big_set(st, b, mode);
    if (e2 != hipSuccess) return e2;
    // the large-message blocks only (exit after one atomic when the lists
    // are empty)
    const u32 fork_big_blocks = small_blocks < kBigBlocksFork ? small_blocks : kBigBlocksFork;
    ek<<<fork_big_blocks, kWavesPerBlock * 64, 0, st>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_len, status, bm_base, bitmap,
        reinterpret_cast<const u32*>(b.seg_list), b.seg_count, b.whole_list, b.whole_count, b.exec_next,
        fork_big_blocks, big_threshold, 0u, keep_hist, 0u, nullptr, nullptr, 0u, 0u);
    return hipGetLastError();
  };
  // The huge messages' pass 1b, chunked (chunk_*_kernel): when the record
  // region holds a batch of this workspace's size (option chunked_huge 0:
  // one wave per message).  On by default since the small bodies' execution runs
  // in walk order (FSG_SPLIT_WALK 3): CM 6.77-6.81 -> 6.44 ms, where the
  // chunked walk alone had measured slower (the huge bodies were then off
  // the critical path).
  const bool kChunked = opt(kOptChunkedHuge) != 0;  // (the tests run both forms)
  // record region: 8 B per possible huge message (its first record, its
  // chain verdict), then the chunk records -- sized for the batch's bound on
  // huge messages (est_total_in / kHugeIndexBytes), the records after them
  const u64 max_huge_need = est_total_in / kHugeIndexBytes + 1;
  const u64 max_huge = 8 * max_huge_need < chunk_bytes ? max_huge_need : chunk_bytes / 320;
  const u64 max_recs = max_huge ? (chunk_bytes - 8 * max_huge) / sizeof(ChunkRec) : 0;
  u32* const first_rec = reinterpret_cast<u32*>(chunk_region);
  u32* const mstat = first_rec + max_huge;
  ChunkRec* const recs = reinterpret_cast<ChunkRec*>(chunk_region + 8 * max_huge);
  const bool chunked = kChunked && max_huge >= est_total_in / kHugeIndexBytes + 1 &&
                       max_recs >= est_total_in / kChunkBytes + est_total_in / kHugeIndexBytes + 2;
  auto launch_big_chunked = [&](hipStream_t st, const BigSet& b) -> hipError_t {
    u32* const cctr = reinterpret_cast<u32*>(w + kWsChunkCount);
    const u32 lb = (u32)((max_huge + 255) / 256);
    chunk_list_kernel<<<lb ? lb : 1u, 256, 0, st>>>(in, in_off, in_len, big_count, big_list, n_msgs, flags, cctr,
                                                     recs, first_rec, (u32)max_recs);
    const u32 wb = (u32)(max_recs / 4 + 1 < 1024 ? max_recs / 4 + 1 : 1024);
    chunk_spec_kernel<<<wb, 256, 0, st>>>(in, in_off, in_len, flags, bm_base, bitmap, cctr, recs,
                                          reinterpret_cast<u32*>(w + kWsChunkSpecNext), (u32)max_recs);
    const u32 hb = (u32)(max_huge / 4 + 1 < 256 ? max_huge / 4 + 1 : 256);
    chunk_fixup_kernel<<<hb, 256, 0, st>>>(in, in_off, in_len, out_len, bm_base, bitmap, big_count, recs, first_rec,
                                           mstat, reinterpret_cast<u32*>(w + kWsChunkFixNext));
    chunk_check_kernel<<<wb, 256, 0, st>>>(in, in_off, in_len, out_len, bm_base, bitmap, cctr, recs, out, out_off,
                                           reinterpret_cast<u32*>(w + kWsChunkCheckNext), (u32)max_recs);
    chunk_final_kernel<<<hb, 256, 0, st>>>(in, in_off, in_len, flags, bm_base, bitmap, out, out_off, big_list,
                                           out_len, status, big_count, recs, first_rec, mstat, n_msgs, b.seg_list,
                                           b.seg_count, b.whole_list, b.whole_count,
                                           reinterpret_cast<u32*>(w + kWsChunkFinalNext));
    hipError_t e2 = hipGetLastError();
    if (e2 != hipSuccess) return e2;
    const u32 fork_big_blocks = small_blocks < kBigBlocksFork ? small_blocks : kBigBlocksFork;
    ek<<<fork_big_blocks, kWavesPerBlock * 64, 0, st>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_len, status, bm_base, bitmap,
        reinterpret_cast<const u32*>(b.seg_list), b.seg_count, b.whole_list, b.whole_count, b.exec_next,
        fork_big_blocks, big_threshold, 0u, keep_hist, 0u, nullptr, nullptr, 0u, 0u);
    return hipGetLastError();
  };
  // The forked path's small-message launches: a grid of kSmallPersist blocks,
  // each wave looping over messages; CM 7.31 -> 7.02 ms against one wave per
  // message (A/B on one box, two passes; 1,024 blocks: 7.11, 3,584: 7.03);
  // 3,584 (two rounds of blocks at 7 waves per SIMD) since the execution
  // runs in walk order (see kBigBlocksFork).  Option small_persist (blocks:
  // the tests shrink it; 0 = one wave per message).
  const i64 sp_opt = opt(kOptSmallPersist);
  const u32 kSmallPersist = sp_opt >= 0 && sp_opt <= (1 << 20) ? (u32)sp_opt : 3584u;
  auto launch_small = [&](hipStream_t st, u32 part) -> hipError_t {
    // one wave per message; large ones are skipped (big_blocks = 0: no block
    // takes the large-message role).  part 1 / 2: the messages of that part
    // of the split walk, in walk order.
    const u32 grid = kSmallPersist && kSmallPersist < small_blocks ? kSmallPersist : small_blocks;
    ek<<<grid, kWavesPerBlock * 64, 0, st>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_len, status, bm_base, bitmap,
        reinterpret_cast<const u32*>(seg_list), set0.seg_count, whole_list, set0.whole_count, set0.exec_next,
        0u, big_threshold, 0u, keep_hist, grid < small_blocks ? grid : 0u, part ? walk_perm : nullptr,
        part ? walk_hist : nullptr, part, kSplitClass);
    return hipGetLastError();
  };
  // The short bodies of walk part 2 packed several to a wave (exec5_packed):
  // option exec_pack = bodies per batch (1..64, default 32; 0 = one wave per
  // body, the small-message grid above).  Grid: the small-message grid's
  // size.  Measured on CM (A/B on one box):
  // 5.85-5.92 ms against 6.11-6.19 with one wave per body, once literals of
  // 65..896 bytes ran inside the group (6.60-6.63 while each was a
  // wave-wide copy with a window restart).
  const i64 pack_opt = opt(kOptExecPack);
  const u32 kPackBatch = pack_opt >= 1 && pack_opt <= 64 ? (u32)pack_opt : 0u;
  auto launch_packed = [&](hipStream_t st) -> hipError_t {
    const u32 grid = kSmallPersist && kSmallPersist < small_blocks ? kSmallPersist : small_blocks;
    exec_packed_kernel<<<grid, kWavesPerBlock * 64, 0, st>>>(
        in, in_off, in_len, out, out_off, out_len, status, bm_base, bitmap, walk_perm, walk_hist, kSplitClass,
        reinterpret_cast<u32*>(w + kWsPackNext), kPackBatch, keep_hist);
    return hipGetLastError();
  };
  SideStream* side = fork ? side_stream() : nullptr;
  if (side) {
    // the plan pass lists the large messages; pass 1b starts on them while
    // the lane walk runs
    index_plan_kernel<<<(n_msgs + kPlanThreads - 1) / kPlanThreads, kPlanThreads, 0, stream>>>(
        in, in_off, in_len, n_msgs, out_cap, out_len, status, flags, counter, bm_base, bitmap,
        cap_words, big_count, big_list, big_threshold, kWalkOrder ? walk_rank : nullptr, walk_hist);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (kWalkOrder) {
      walk_offsets_kernel<<<1, 64, 0, stream>>>(walk_hist);
      walk_scatter_kernel<<<(n_msgs + 255) / 256, 256, 0, stream>>>(in_len, n_msgs, status, walk_rank,
                                                                  walk_hist, walk_perm);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // The huge messages (> kHugeIndexBytes compressed) are walked and
    // executed on a second side stream, so the other large messages'
    // execution starts when their own (shorter) walks end instead of after
    // the longest walk: CM 7.6 -> see DESIGN.md section 5.
    std::lock_guard<std::mutex> lk(side->mu);
    if ((e = hipEventRecord(side->fork, stream)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(side->stream, side->fork, 0)) != hipSuccess) return e;
    const bool split = kSplitHuge && side->stream2;
    if (split) {
      if ((e = hipStreamWaitEvent(side->stream2, side->fork, 0)) != hipSuccess) return e;
      if ((e = chunked ? launch_big_chunked(side->stream2, set1) : launch_big(side->stream2, set1, 1u)) != hipSuccess)
        return e;
      if ((e = hipEventRecord(side->join2, side->stream2)) != hipSuccess) return e;
    }
    if ((e = launch_big(side->stream, set0, split ? 2u : 0u)) != hipSuccess) return e;
    if ((e = hipEventRecord(side->join, side->stream)) != hipSuccess) return e;
    const bool three = split_walk && kWalkOrder && side->stream3;
    if (three) {
      // the larger small bodies: walk and execution on the third stream
      if ((e = hipStreamWaitEvent(side->stream3, side->fork, 0)) != hipSuccess) return e;
      if ((e = launch_index(true, side->stream3, 1u)) != hipSuccess) return e;
      if ((e = launch_small(side->stream3, 1u)) != hipSuccess) return e;
      if ((e = hipEventRecord(side->join3, side->stream3)) != hipSuccess) return e;
      if ((e = launch_index(true, stream, 2u)) != hipSuccess) return e;
      if ((e = launch_small(stream, 2u)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(stream, side->join3, 0)) != hipSuccess) return e;
    } else {
      if ((e = launch_index(true)) != hipSuccess) return e;
      if (kWalkOrder && split_mode == 2) {
        if ((e = launch_small(stream, 3u)) != hipSuccess) return e;
      } else if (kWalkOrder && split_mode == 3) {
        if ((e = kPackBatch ? launch_packed(stream) : launch_small(stream, 2u)) != hipSuccess) return e;
        if ((e = launch_small(stream, 1u)) != hipSuccess) return e;
      } else {
        if ((e = launch_small(stream, 0u)) != hipSuccess) return e;
      }
    }
    if ((e = hipStreamWaitEvent(stream, side->join, 0)) != hipSuccess) return e;
    if (split && (e = hipStreamWaitEvent(stream, side->join2, 0)) != hipSuccess) return e;
  } else {
    // one stream: pass 1, pass 1b, then one exec launch whose first blocks
    // take the large messages (dispatched first) and the rest one message
    // per wave
    if ((e = launch_index(false)) != hipSuccess) return e;
    if ((e = launch_index_big(stream)) != hipSuccess) return e;
    if (two) {
      std::lock_guard<std::mutex> lk(two->mu);
      if ((e = hipEventRecord(two->pass1, stream)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(caller_stream, two->pass1, 0)) != hipSuccess) return e;
      stream = caller_stream;
    }
    ek<<<big_blocks + small_blocks, kWavesPerBlock * 64, 0, stream>>>(
        in, in_off, in_len, n_msgs, out, out_off, out_len, status, bm_base, bitmap,
        reinterpret_cast<const u32*>(seg_list), set0.seg_count, whole_list, set0.whole_count, set0.exec_next,
        big_blocks, big_threshold, kPrio, keep_hist, 0u, nullptr, nullptr, 0u, 0u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  fallback_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, out, out_off,
                                                         out_len, status, flags);
  return hipGetLastError();
}

}  // namespace fsg
