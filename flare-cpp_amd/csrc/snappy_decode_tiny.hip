// snappy_decode_tiny.hip -- one LANE per tiny message, tag walk and execution
// fused, the message's whole output in LDS.
//
// Why.  The forked path's small bodies pay a fixed cost per message in the
// two-pass decoder: a lane walk writes the bitmap, then a whole wave reads it
// back, fills a tag ring, prefetches tag bytes, zeroes a window and flushes --
// ~1,600 wave instructions and four dependent memory round trips for a body
// that holds one or two 64-tag groups (CM: 595K bodies of < 512 compressed
// bytes, avg ~380 B of output).  A body that small fits a lane:
// its output (<= kTinyOut bytes) lives in the lane's LDS, its input streams
// through a 256-byte LDS ring, and the lane runs the reference's tag loop
// (SnappyDecompressor::DecompressAllTags, /root/reference/flare/io/snappy/
// snappy.cc:716-787, with the writer checks of SnappyArrayWriter :1331-1481)
// with every copy inside LDS, then stores the body with 16-byte stores.
//
// Output bytes and statuses equal the two-pass decoder's (and so the
// reference's): the same checks as index_kernel's walk (tag and literal bytes
// present, 4-byte literal lengths as the reference's uint32 sum) and as
// exec5_message (copy offset 0 or past the output written, writer overrun),
// and the stream must end exactly at the header length (:858-868).
//
// Copies go forward in 16-byte steps and may write up to 15 bytes past their
// end (the reference's fast paths do the same, snappy.cc:98-152): later tags
// overwrite them, and only [0, length) is stored.  A copy with offset < 16
// repeats one 16-byte expansion of its pattern (pat_step bytes per step).
//
// Used by the forked path (batches of > 128K messages) for the walk classes
// >= kTinyClass (compressed size < 512 B), which then neither the lane walk nor
// the execution pass touch.  A body of more than kTinyOut output bytes in
// those classes (possible only for ratios above 1.5) gets kNeedFallback: the
// final pass decodes it serially (fallback_kernel).
//
// MEASURED SLOWER, off by default (option tiny_pass):
// CM 6.2 -> 7.5 ms (per-lane contiguous LDS) / 8.0 ms (this dword-interleaved
// form).  The pass took 2.5 / 4.7 ms for the 595K bodies the lane walk and
// execution pass handle in ~2.3 ms: its LDS allows two waves per CU, each
// lane's tag loop is a chain of dependent LDS round trips with divergent
// literal / copy / pattern paths, and while it runs the side streams' passes
// find no LDS.  Kept, tested (test_tiny_body_pass, the "1t1" fuzz mode), as
// the measured alternative.
#include "snappy_lane_decode.h"
#include "snappy_pieces.h"
#include "wave_util.h"

namespace fsg {

namespace {
constexpr u32 kTinyOut = 768;            // output bytes a lane holds
constexpr u32 kTinyOutDw = 200;          // dwords of output per lane (+ the over-write tail, <= 19 B)
constexpr u32 kTinyRingDw = 64;          // dwords of input ring per lane (256 B, 16 chunks)
constexpr u32 kTinyRingChunks = kTinyRingDw / 4;
constexpr u32 kTinySync = 8;             // tag steps between the wave's ring landings
static_assert(kTinyOutDw * 4 >= kTinyOut + 20, "over-write tail");

// The tag table of exec5_message (exec_tag_entry, snappy_decode_v4.hip): per
// tag byte c, bits 0-4 the right shift of 0xffffffff masking the nb extra
// bytes, bit 5 long literal, bit 6 literal, bits 8-14 length (short literal,
// copies), bits 16-18 nb, bits 20-30 COPY_1's offset bits 8-10
// (snappy.cc:744-781).
__device__ __forceinline__ u32 tiny_tag_entry(u32 c) {
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

// The lane's LDS is dword-interleaved ([dword][lane]: dword d of lane l at
// d * 64 + l), so a wave's dword accesses at per-lane offsets never share a
// bank; a 16-byte read at any byte offset is five dword reads and a byte
// shift, a 16-byte write five dword writes (the first merged with the bytes
// below it) -- against one LDS cycle per lane for an unaligned 16-byte read
// and two for a write in a per-lane contiguous layout ("LDS
// access costs").  One wave per block; two blocks fill a CU's LDS.
__global__ __launch_bounds__(64) void tiny_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len, i32* __restrict__ status,
    const u32* __restrict__ walk_perm, const u32* __restrict__ walk_hist, u32 walk_classes, u32 tiny_class) {
  __shared__ u32 outs[kTinyOutDw * 64];
  __shared__ u32 rings[kTinyRingDw * 64];
  __shared__ u32 tagtab[256];
  __shared__ u32x4 sel_tab[16];
  const u32 lane = threadIdx.x;
#pragma unroll
  for (u32 q = 0; q < 4; ++q) tagtab[4 * lane + q] = tiny_tag_entry(4 * lane + q);
  init_pattern_table(sel_tab, lane);
  __syncthreads();
  u32* const ol = outs + lane;   // dword d at ol[64 d]
  u32* const rl = rings + lane;  // dword d at rl[64 (d & 63)]

  // 16 bytes at byte b of the output (o) or the ring (r)
  auto read16 = [&](bool ring, u32 b) -> u32x4 {
    const u32 d = b >> 2, sh = b & 3;
    u32 w[5];
#pragma unroll
    for (u32 q = 0; q < 5; ++q) w[q] = ring ? rl[64 * ((d + q) & (kTinyRingDw - 1))] : ol[64 * (d + q)];
    return u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], sh), __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                 __builtin_amdgcn_alignbyte(w[3], w[2], sh), __builtin_amdgcn_alignbyte(w[4], w[3], sh)};
  };
  // x to output bytes [o, o + 16); the bytes of the first dword below o are
  // kept, up to 3 bytes past o + 16 are overwritten (later tags rewrite them)
  auto write16 = [&](u32 o, u32x4 x) {
    const u32 d = o >> 2, sh = o & 3;
    if (sh == 0) {
#pragma unroll
      for (u32 q = 0; q < 4; ++q) ol[64 * (d + q)] = x[q];
    } else {
      const u32 old = ol[64 * d];
      const u32 keep = 0xffffffffu >> (32 - 8 * sh);
      const u32 r = 4 - sh;
      ol[64 * d] = (old & keep) | (x[0] << (8 * sh));
      ol[64 * (d + 1)] = __builtin_amdgcn_alignbyte(x[1], x[0], r);
      ol[64 * (d + 2)] = __builtin_amdgcn_alignbyte(x[2], x[1], r);
      ol[64 * (d + 3)] = __builtin_amdgcn_alignbyte(x[3], x[2], r);
      ol[64 * (d + 4)] = x[3] >> (8 * r);
    }
  };

  const u32 lo = walk_hist[walk_classes + tiny_class];
  const u32 hi = walk_hist[2 * walk_classes];
  const u32 n = hi > lo ? hi - lo : 0u;
  const u32 stride = gridDim.x * 64;
  // rounds: lane l of block b takes positions b*64 + l + k*stride; the walk
  // order sorts by size class, so a round's 64 bodies are of similar size
  for (u32 base = blockIdx.x * 64; base < n; base += stride) {
    const u32 i = base + lane;
    const bool have = i < n;
    const u32 m = have ? walk_perm[lo + i] : 0u;
    bool act = have && status[m] == kNeedLaneWalk;
    const u32 n_in = have ? in_len[m] : 0u;
    const u32 ulen = have ? out_len[m] : 0u;  // the header's length (plan pass)
    const u8* ib = in + (have ? in_off[m] : 0ull);
    const u32 ibal = (u32)(reinterpret_cast<uintptr_t>(ib) & 15);
    const __amdgpu_buffer_rsrc_t irsrc = msg_rsrc(ib - ibal, act ? ibal + n_in : 0u);
    if (act && ulen > kTinyOut) {  // does not fit the lane's LDS: the serial pass
      status[m] = kNeedFallback;
      act = false;
    }
    // the ring's 16 chunks, landed now, and the next 8 in flight (chunks
    // past the body read 0)
    u32x4 g[kTinyRingChunks];
#pragma unroll
    for (u32 k = 0; k < kTinyRingChunks; ++k) g[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * k, 0, 0);
    u32x4 h[8];
#pragma unroll
    for (u32 k = 0; k < 8; ++k) h[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * (kTinyRingChunks + k), 0, 0);
#pragma unroll
    for (u32 k = 0; k < kTinyRingChunks; ++k)
#pragma unroll
      for (u32 q = 0; q < 4; ++q) rl[64 * (4 * k + q)] = g[k][q];
    u32 wend = kTinyRingChunks;  // chunks [wend - 16, wend) are in the ring, [wend, wend + 8) in h
    // header length (checked by the plan pass: <= 5 bytes, < 0x80 ends it)
    u32 ip = 0;
    {
      const u32x4 hr = read16(true, ibal);
      const u64 hb = (u64)hr[0] | ((u64)hr[1] << 32);
      u32 k = 0;
      while (k < 4 && ((hb >> (8 * k)) & 0x80u)) ++k;
      ip = k + 1;
    }
    u32 op = 0;
    i32 st = kOk;
    u32 lrem = 0;  // bytes of a literal still to copy (longer than the ring holds)
    // Landings are wave-wide, every kTinySync tag steps: a lane whose next
    // bytes are not in the ring idles until then, so no lane's wait for its
    // input stalls the others (a wave's loads and stores share one counter:
    // any wait inside the loop would wait for every load issued before it).
    // The chunks landed were requested one landing earlier; the output and
    // the statuses are stored after the round, when every lane is done.
    for (u32 it = 0; __any(act); ++it) {
      if ((it & (kTinySync - 1)) == kTinySync - 1) {
        // land h where its 8 slots hold consumed chunks only (those below
        // the chunk of the next byte the lane reads), then request the next 8
        const u32 pc = (ip + ibal) >> 4;
        if (act && wend + 8 <= pc + kTinyRingChunks) {
#pragma unroll
          for (u32 k = 0; k < 8; ++k)
#pragma unroll
            for (u32 q = 0; q < 4; ++q) rl[64 * ((4 * (wend + k) + q) & (kTinyRingDw - 1))] = h[k][q];
          wend += 8;
#pragma unroll
          for (u32 k = 0; k < 8; ++k) h[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * (wend + k), 0, 0);
        }
      }
      if (act) {
        const u32 P = ip + ibal;
        const u32 have_end = 16 * wend;  // ring bytes end (aligned-buffer offset)
        // this step's piece source (ring / output), its length and the
        // number of 16-byte (or pattern-step) pieces
        bool from_ring = true, pattern = false;
        u32 src = 0, cnt = 0, stp = 16, off = 0;
        if (lrem) {
          // ---- more of a long literal, as far as the ring holds it
          const u32 avail = have_end - P;
          cnt = lrem < avail ? lrem : (avail & ~15u);
          src = P;
          lrem -= cnt;
          ip += cnt;
        } else if (ip == n_in) {  // end of input between tags (:858-868), empty bodies included
          st = op == ulen ? kOk : kCorrupt;
          act = false;
        } else if (P + 5 <= have_end || ibal + n_in <= have_end) {
          // ---- one tag (bounds and the writer's checks as the two-pass decoder)
          const u32 d = P >> 2, bs = P & 3;
          const u32 w0 = rl[64 * (d & (kTinyRingDw - 1))], w1 = rl[64 * ((d + 1) & (kTinyRingDw - 1))];
          const u32 t0 = __builtin_amdgcn_alignbyte(w1, w0, bs);
          const u32 ext = __builtin_amdgcn_alignbyte(w1 >> (8 * bs), t0, 1);
          const u32 e = tagtab[t0 & 0xffu];
          const u32 val = ext & (0xffffffffu >> (e & 31u));
          const bool is_lit = e & 64u;
          const u32 nb = (e >> 16) & 7u;
          const u32 llmask = 0u - ((e >> 5) & 1u);
          const u32 lpart = (val + 1u) & llmask;
          const u32 tlen = (e >> 8) & 0x7fu;
          const u32 len = lpart + tlen;
          const u32 adv = 1 + nb + (is_lit ? tlen : 0u);
          const u32 step = adv + lpart;
          if (step > n_in - ip || step < adv) {  // runs past the input (or wraps)
            st = kCorrupt;
            act = false;
          } else if (len > ulen - op) {  // writer overrun (:1166, :1400)
            st = kCorrupt;
            act = false;
          } else if (is_lit) {
            // the tag, then as many whole 16-byte pieces of the literal as
            // the ring holds (all of it when it ends there): the rest later
            const u32 S = P + 1 + nb;
            const u32 avail = have_end - S;
            cnt = len <= avail ? len : (avail & ~15u);
            src = S;
            ip += 1 + nb + cnt;
            lrem = len - cnt;
          } else {
            off = val + (e >> 20);
            if (off == 0 || off > op) {  // (:1200, :1410, :1466)
              st = kCorrupt;
              act = false;
            } else {
              from_ring = false;
              src = op - off;
              cnt = len;
              pattern = off < 16;
              stp = pattern ? pat_step(off) : 16u;
              ip += step;
            }
          }
        }
        // ---- the pieces: cnt bytes from src to op (a pattern: one 16-byte
        // expansion, stp bytes per piece)
        u32x4 x = u32x4{0, 0, 0, 0};
        for (u32 k = 0; k < cnt; k += stp) {
          if (k == 0 || !pattern) {
            x = read16(from_ring, src + k);
            if (pattern) x = expand_pattern(x, off, sel_tab);
          }
          write16(op + k, x);
        }
        op += cnt;
      }
      wave_lds_fence();
    }
    // ---- the round's bodies and statuses
    if (have && status[m] == kNeedLaneWalk) {
      status[m] = st;
      if (st == kOk) {
        u8* ob = out + out_off[m];
        for (u32 k = 0; k < ulen; k += 16) {
          const u32x4 v = u32x4{ol[64 * (k / 4)], ol[64 * (k / 4 + 1)], ol[64 * (k / 4 + 2)], ol[64 * (k / 4 + 3)]};
          store_exact(ob + k, v, ulen - k < 16 ? ulen - k : 16u);
        }
      }
    }
    wave_lds_fence();
  }
}

// Grid: two one-wave blocks per CU (68.5 KB of LDS each).
hipError_t launch_tiny(const u8* in, const u64* in_off, const u32* in_len, u8* out, const u64* out_off,
                       const u32* out_len, i32* status, const u32* walk_perm, const u32* walk_hist,
                       u32 walk_classes, u32 tiny_class, u32 blocks, hipStream_t stream) {
  tiny_kernel<<<blocks, 64, 0, stream>>>(in, in_off, in_len, out, out_off, out_len, status, walk_perm, walk_hist,
                                         walk_classes, tiny_class);
  return hipGetLastError();
}

}  // namespace fsg
