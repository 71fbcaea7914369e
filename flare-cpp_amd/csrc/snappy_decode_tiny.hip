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
#include "snappy_lane_decode.h"
#include "snappy_pieces.h"
#include "wave_util.h"

namespace fsg {

namespace {
constexpr u32 kTinyOut = 768;                       // output bytes a lane holds
constexpr u32 kTinyOutCap = kTinyOut + 16;          // + the over-copy tail
constexpr u32 kTinyRingChunks = 16;                 // 16-byte input chunks in the ring
constexpr u32 kTinyRing = 16 * kTinyRingChunks;     // 256 B
constexpr u32 kTinyLane = kTinyOutCap + kTinyRing + 16;  // + a mirror of slot 0: 1,056 B
constexpr u32 kTinyLongLit = 64;                    // longer literals come from global memory

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

__device__ __forceinline__ u32x4 lds16(const u8* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void sts16(u8* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }
}  // namespace

// One wave per block; kTinyBlocksPerCU blocks fill a CU's LDS.
__global__ __launch_bounds__(64) void tiny_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_len, i32* __restrict__ status,
    const u32* __restrict__ walk_perm, const u32* __restrict__ walk_hist, u32 walk_classes, u32 tiny_class) {
  __shared__ __attribute__((aligned(16))) u8 lds[64 * kTinyLane];
  __shared__ u32 tagtab[256];
  __shared__ u32x4 sel_tab[16];
  const u32 lane = threadIdx.x;
#pragma unroll
  for (u32 q = 0; q < 4; ++q) tagtab[4 * lane + q] = tiny_tag_entry(4 * lane + q);
  init_pattern_table(sel_tab, lane);
  __syncthreads();
  u8* const ol = lds + lane * kTinyLane;  // output [0, kTinyOutCap)
  u8* const rg = ol + kTinyOutCap;        // ring [0, 256) + mirror of [0, 16) at 256

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
    // the ring's first 16 chunks, landed now, and the next 8 in flight
    // (chunks past the body read 0)
    u32x4 g[kTinyRingChunks];
#pragma unroll
    for (u32 k = 0; k < kTinyRingChunks; ++k) g[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * k, 0, 0);
    u32x4 h[8];
#pragma unroll
    for (u32 k = 0; k < 8; ++k) h[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * (kTinyRingChunks + k), 0, 0);
#pragma unroll
    for (u32 k = 0; k < kTinyRingChunks; ++k) sts16(rg + 16 * k, g[k]);
    sts16(rg + kTinyRing, g[0]);
    u32 wend = kTinyRingChunks;  // chunks [wend - 16, wend) are in the ring, [wend, wend + 8) in h
    // header length (checked by the plan pass: <= 5 bytes, < 0x80 ends it)
    u32 ip = 0;
    {
      const u32x4 hv = lds16(rg + ibal);
      const u64 hb = (u64)hv[0] | ((u64)hv[1] << 32);
      u32 k = 0;
      while (k < 4 && ((hb >> (8 * k)) & 0x80u)) ++k;
      ip = k + 1;
    }
    u32 op = 0;
    i32 st = kOk;
    while (__any(act)) {
      if (act) {
        // ---- one tag (bounds and the writer's checks as the two-pass decoder)
        const u32 P = ip + ibal;
        // The tag's <= 5 bytes (and a short literal's bytes) must be in the
        // ring, else the prefetched chunks land and the tag runs next time.
        // A landing never overwrites an unread chunk: a tag spans at most 66
        // bytes (6 chunks), so it needs a chunk >= wend only when wend <= pc + 5,
        // and the 8 chunks landed (< pc + 16) take the slots of chunks < pc.
        auto land = [&]() {
#pragma unroll
          for (u32 k = 0; k < 8; ++k) {
            const u32 sl = (wend + k) & (kTinyRingChunks - 1);
            sts16(rg + 16 * sl, h[k]);
            if (sl == 0) sts16(rg + kTinyRing, h[k]);
          }
          wend += 8;
#pragma unroll
          for (u32 k = 0; k < 8; ++k) h[k] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, 16 * (wend + k), 0, 0);
        };
        if (ip == n_in) {  // end of input between tags (:858-868), empty bodies included
          st = op == ulen ? kOk : kCorrupt;
          act = false;
        } else if (((P + 4) >> 4) >= wend) {
          land();
        } else {
          const u32x4 tv = lds16(rg + (P & (kTinyRing - 1)));
          const u32 c = tv[0] & 0xffu;
          const u32 e = tagtab[c];
          const u32 ext = __builtin_amdgcn_alignbyte(tv[1], tv[0], 1);
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
          } else if (is_lit && len <= kTinyLongLit && ((P + step - 1) >> 4) >= wend) {
            land();
          } else if (len > ulen - op) {  // writer overrun (:1166, :1400)
            st = kCorrupt;
            act = false;
          } else if (is_lit) {
            const u32 S = P + 1 + nb;  // the literal's bytes, aligned-buffer offset
            if (len <= kTinyLongLit) {
              for (u32 k = 0; k < len; k += 16) sts16(ol + op + k, lds16(rg + ((S + k) & (kTinyRing - 1))));
            } else {
              for (u32 k = 0; k < len; k += 16) sts16(ol + op + k, rsrc_load16(irsrc, S + k));
            }
            op += len;
            ip += step;
          } else {
            const u32 off = val + (e >> 20);
            if (off == 0 || off > op) {  // (:1200, :1410, :1466)
              st = kCorrupt;
              act = false;
            } else {
              const u8* src = ol + op - off;
              if (off >= 16) {
                for (u32 k = 0; k < len; k += 16) sts16(ol + op + k, lds16(src + k));
              } else {
                const u32x4 x = expand_pattern(lds16(src), off, sel_tab);
                const u32 stp = pat_step(off);
                for (u32 k = 0; k < len; k += stp) sts16(ol + op + k, x);
              }
              op += len;
              ip += step;
            }
          }
        }
        if (act && ip == n_in) {  // (the same test, one iteration sooner)
          st = op == ulen ? kOk : kCorrupt;
          act = false;
        }
        if (!act) {  // this lane's body is done: its status, and its bytes
          status[m] = st;
          if (st == kOk) {
            u8* ob = out + out_off[m];
            for (u32 k = 0; k < ulen; k += 16) store_exact(ob + k, lds16(ol + k), ulen - k < 16 ? ulen - k : 16u);
          }
        }
      }
      wave_lds_fence();
    }
  }
}

// Grid: two one-wave blocks per CU (kTinyLane x 64 + tables = 68.9 KB each).
hipError_t launch_tiny(const u8* in, const u64* in_off, const u32* in_len, u8* out, const u64* out_off,
                       const u32* out_len, i32* status, const u32* walk_perm, const u32* walk_hist,
                       u32 walk_classes, u32 tiny_class, u32 blocks, hipStream_t stream) {
  tiny_kernel<<<blocks, 64, 0, stream>>>(in, in_off, in_len, out, out_off, out_len, status, walk_perm, walk_hist,
                                         walk_classes, tiny_class);
  return hipGetLastError();
}

}  // namespace fsg
