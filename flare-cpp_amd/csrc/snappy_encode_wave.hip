// snappy_encode_wave.hip -- one wave per 64 KiB fragment, hash table in LDS.
//
// internal::CompressFragment (/root/reference/flare/io/snappy/snappy.cc:
// 329-453) is a serial greedy parse: every probe reads the table slot of its
// 4-byte hash and overwrites it with its own position, and the parse decides
// which positions are probed.  This kernel runs that parse exactly, with the
// fragment's table (WorkingMemory::GetHashTable, snappy.cc:247-271: htsize
// u16 entries, zeroed) in the wave's LDS, and does the per-position work 64
// positions at a time:
//
//   block  the 64 positions q = B + lane.  Each lane loads the 20 input bytes
//          at q, hashes the first 4, reads its table slot T (the table as of
//          the block's start), loads the 20 bytes at T (issued one block
//          ahead: see "speculation"), and finds its in-block predecessors with
//          the same hash (pred rounds, below).  From these it knows, for any
//          set I of positions inserted so far in the block, its candidate --
//          the newest inserted same-hash position below it, else T -- whether
//          the candidate's 4 bytes match, and the match length.
//   events the parse itself, wave-uniform: a literal search from p with the
//          skip heuristic (snappy.cc:377-397) is one ballot over the block's
//          probe positions (all positions probed before a lane are inserted
//          before it), the first matching lane wins, the copy and the probe
//          after it (snappy.cc:416-439) update I.  Text has ~6 copies per
//          64-position block.
//   commit the block's inserted positions are written to the table in
//          position order (one ds_write_b16 under the inserted mask: the
//          highest lane wins a shared slot, as the newest write does).
//
// Pred rounds: every lane writes its position into its table slot (highest
// lane wins), reads it back; the winners leave, the losers repeat; a lane
// that wins round r+1 is the predecessor of the winner of round r with its
// hash.  Three rounds at most: chains longer than that are resolved by a
// serial scan when a probe needs them.  The commit restores every slot first.
//
// Speculation: the next block's table reads and candidate loads are issued
// before this block's events (hiding the load latency behind them); at the
// next block's start the table is read again, and a lane whose slot changed
// (this block inserted into it) takes the new candidate's bytes from this
// block's lanes (ds_bpermute) -- a position this block inserted.
//
// CPU model of the same algorithm, checked byte-for-byte against the oracle:
// tools/wenc_model.cc.  Output bytes equal snappy::Compress (snappy.cc:
// 875-954); EmitLiteral / EmitCopy follow snappy.cc:156-232.
#include "snappy_device.h"

namespace fsg {

namespace {

constexpr u32 kPredNone = 0xff, kPredUnknown = 0xfe;

// Diagnostic build only (-DFSG_STAMPS): per-phase cycle totals of the wave
// encoder, summed over waves (fsg_debug_wstamps).
#ifdef FSG_STAMPS
__device__ unsigned long long g_wstamps[16];  // 0-7 cycles per phase, 8-11 counts, 12-13 cycles
#define STAMP(k) do { const u64 t_ = __builtin_amdgcn_s_memtime(); st_[k] += t_ - t_last_; t_last_ = t_; } while (0)
#define WCOUNT(k) (st_[k] += 1)
#else
#define STAMP(k) do { } while (0)
#define WCOUNT(k) do { } while (0)
#endif

__device__ __forceinline__ u32 rl(u32 v, u32 l) { return (u32)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ u32 bperm(u32 v, u32 src) { return (u32)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v); }
__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_wave_barrier(); }
__device__ __forceinline__ u32 ab(u32 hi, u32 lo, u32 s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

struct W5 {
  u32 w[5];
};

// 20 bytes at buffer offset P: one 16- and one 8-byte load at the dword below,
// issued now, shifted by shifted20() when used (bytes past the buffer read 0).
struct Raw20 {
  u32x4 d;
  u32x2 e;
  u32 s;
};
__device__ __forceinline__ Raw20 raw20(__amdgpu_buffer_rsrc_t r, u32 P) {
  const u32 a = P & ~3u;
  return Raw20{__builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0), __builtin_amdgcn_raw_buffer_load_b64(r, a + 16, 0, 0),
               P & 3u};
}
__device__ __forceinline__ W5 shifted20(const Raw20& x) {
  W5 o;
  o.w[0] = ab(x.d[1], x.d[0], x.s);
  o.w[1] = ab(x.d[2], x.d[1], x.s);
  o.w[2] = ab(x.d[3], x.d[2], x.s);
  o.w[3] = ab(x.e[0], x.d[3], x.s);
  o.w[4] = ab(x.e[1], x.e[0], x.s);
  return o;
}

// number of equal leading bytes of a and b (0..20)
__device__ __forceinline__ u32 eq_prefix20(const W5& a, const W5& b) {
  u32 n = 20;
#pragma unroll
  for (int i = 4; i >= 0; --i) {
    const u32 x = a.w[i] ^ b.w[i];
    n = x ? 4 * i + ((u32)__builtin_ctz(x) >> 3) : n;
  }
  return n;
}

// Inclusive prefix sum over the 64 lanes (DPP row shifts and broadcasts).
__device__ __forceinline__ u32 incl_scan64(u32 v) {
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

// EmitCopyLessThan64 (snappy.cc:198-214) as packed bytes; *nb = 2 or 3.
__device__ __forceinline__ u32 copy_tag(u32 offset, u32 len, u32* nb) {
  if (len < 12 && offset < 2048) {
    *nb = 2;
    return (1u + ((len - 4) << 2) + ((offset >> 8) << 5)) | ((offset & 0xffu) << 8);
  }
  *nb = 3;
  return (2u + ((len - 1) << 2)) | ((offset & 0xffffu) << 8);
}

}  // namespace

// One fragment, encoded by the calling wave.  fr: buffer descriptor of the
// fragment's message (offset fal + position = the byte's offset); fb: the
// fragment's first byte.  Output from obase; returns the end, or nullptr if a
// staged region (op_lim != nullptr) would overflow.
//
// Output bytes are stored straight to the slot; a block's commit-time output
// is held in registers and stored at the start of the NEXT block, after that
// block's input waits (see held0): the waits then never cover young stores (a
// wave's loads and stores share one counter, so a wait for a load issued
// before a burst of stores would wait for the stores too).  The table is the
// wave's only LDS.
__device__ u8* wave_fragment(__amdgpu_buffer_rsrc_t fr, u32 fal, const u8* fb, u32 n, u8* obase, u8* op_lim,
                             u16* table, u32 ht, u32 lane) {
  const int shift = 32 - (31 - __builtin_clz(ht));
#ifdef FSG_STAMPS
  u64 st_[16] = {};
  u64 t_last_ = __builtin_amdgcn_s_memtime();
#endif
  // zeroed table (snappy.cc:247-271)
  for (u32 i = 8 * lane; i < ht; i += 512) *reinterpret_cast<u32x4*>(table + i) = u32x4{0, 0, 0, 0};
  lds_fence();
  const u32 cap = op_lim ? (u32)(op_lim - obase) : 0xffffffffu;
  u32 opos = 0;
  auto room = [&](u32 bytes) -> bool { return cap == 0xffffffffu || opos + bytes + 16 <= cap; };
  // nb (1..5) tag bytes, one lane per byte
  auto put_tag = [&](u64 tag, u32 nb) {
    if (lane < nb) obase[opos + lane] = (u8)(tag >> (8 * (lane & 7)));
    opos += nb;
  };
  // literal [s, e): tag, then the bytes from the lanes holding them (this
  // block's xw0c or the previous block's xw0p), else a global copy
  auto emit_literal = [&](u32 s, u32 e, u32 B, u32 xw0c, bool prev_ok, u32 xw0p) {
    const u32 len = e - s;
    const u32 nm1 = len - 1;
    if (nm1 < 60) {
      put_tag(nm1 << 2, 1);
    } else {
      const u32 cnt = nm1 < (1u << 8) ? 1 : nm1 < (1u << 16) ? 2 : nm1 < (1u << 24) ? 3 : 4;
      put_tag((u64)((59 + cnt) << 2) | ((u64)nm1 << 8), 1 + cnt);
    }
    if (s >= B || (prev_ok && s + 64 >= B)) {
      const u32 qc = B + lane;
      if (qc >= s && qc < e) obase[opos + qc - s] = (u8)xw0c;
      if (prev_ok) {
        const u32 qp = B - 64 + lane;
        if (qp >= s && qp < e) obase[opos + qp - s] = (u8)xw0p;
      }
      opos += len;
    } else {
      u8* d = obase + opos;
      for (u32 k0 = 0; k0 < len; k0 += 1024) {  // 1 KiB per step, 16 bytes per lane
        const u32 k = k0 + 16 * lane;
        if (k < len) {
          const u32 c = len - k < 16 ? len - k : 16u;
          if (c == 16) {
            u32x4 v;
            __builtin_memcpy(&v, fb + s + k, 16);
            __builtin_memcpy(d + k, &v, 16);
          } else {
            for (u32 i = 0; i < c; ++i) d[k + i] = fb[s + k + i];
          }
        }
      }
      opos += len;
    }
  };
  // EmitCopy (snappy.cc:216-232): 64-byte pieces while len >= 68 (written
  // straight to global memory, one 3-byte tag per lane), one 60-byte piece if
  // 64 < len < 68, then the rest
  auto emit_copy = [&](u32 offset, u32 len) {
    u32 nb;
    if (len >= 68) {
      const u32 n64 = (len - 68) / 64 + 1;
      const u32 t = copy_tag(offset, 64, &nb);  // 3 bytes
      for (u32 i0 = 0; i0 < n64; i0 += 64) {
        const u32 i = i0 + lane;
        if (i < n64) {
          u8* d = obase + opos + 3 * i;
          d[0] = (u8)t;
          d[1] = (u8)(t >> 8);
          d[2] = (u8)(t >> 16);
        }
      }
      opos += 3 * n64;
      len -= 64 * n64;
    }
    if (len > 64) {
      put_tag(copy_tag(offset, 60, &nb), 3);
      len -= 60;
    }
    const u32 t = copy_tag(offset, len, &nb);
    put_tag(t, nb);
  };

  // ---- deferred emission: the block's common events (a literal whose bytes
  // are in this block's or the previous block's registers, a copy of <= 64
  // bytes) are recorded one per lane -- in the lane of the event's first
  // parse position (the post-copy probe, or the search start), so events sit
  // in increasing lanes, EvM marking them: q | literal length << 16,
  // candidate | match length << 16 (fast events: the lane's precomputed
  // fEQL / fECM, FastEv) -- and written together: sizes, a prefix sum over
  // the lanes, then one output byte per lane.  Other events flush the
  // recorded ones first and take the paths above.
  u32 EQL = 0, ECM = 0, fEQL = 0, fECM = 0;
  u64 EvM = 0, FastEv = 0;
  // A block's commit-time output (<= 128 bytes: one byte per lane in two
  // registers) is held until the next block has waited for its input and
  // issued its loads, then stored by two unconditional buffer stores (lanes
  // past the count store out of range, which the buffer drops).  Stored at
  // once, it would sit in the wave's one memory counter ahead of the next
  // block's input loads, and the wait for those loads would wait for the
  // stores too.
  u32 held0 = 0, held1 = 0, held_n = 0, held_at = 0;
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      obase, (short)0, (int)(cap != 0xffffffffu ? cap : (u32)max_compressed_length(n)), 0x00020000);
  auto store_held = [&]() {
    const u32 o0 = lane < held_n ? held_at + lane : 0x80000000u;
    const u32 o1 = lane + 64 < held_n ? held_at + 64 + lane : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b8((u8)held0, orsrc, (int)o0, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((u8)held1, orsrc, (int)o1, 0, 0);
    held_n = 0;
  };
  auto emit_pending = [&](u32 B, u32 xw0c, u32 xw0p, bool hold = false) -> bool {
    if (!EvM) return true;
    const bool fe = (FastEv >> lane) & 1ull;
    const u32 eql = fe ? fEQL : EQL, ecm = fe ? fECM : ECM;
    const u32 q = eql & 0xffffu, L = eql >> 16, cand = ecm & 0xffffu, ml = ecm >> 16;
    const bool ve = (EvM >> lane) & 1ull;
    const u32 nm1 = L - 1;
    const u32 tl = L == 0 ? 0u : (nm1 < 60 ? 1u : 2u);  // L <= 128 here
    const u32 lt = nm1 < 60 ? nm1 << 2 : (240u | (nm1 << 8));
    u32 cnb;
    const u32 ct = copy_tag(q - cand, ml, &cnb);
    const u32 sz = ve ? tl + L + cnb : 0u;
    const u32 incl = incl_scan64(sz);
    const u32 excl = incl - sz;
    const u32 total = rl(incl, 63);
    if (!room(total)) return false;
    // per event: output offset, literal tag length, literal length, literal
    // start relative to B - 64 (0..127)
    const u32 A = excl | (tl << 12) | (L << 14) | ((q - L - (B - 64)) << 22);
    for (u32 j0 = 0; j0 < total; j0 += 64) {
      const u32 j = j0 + lane;
      u32 e = (u32)__builtin_ctzll(EvM);
      for (u64 mm = EvM & (EvM - 1); mm; mm &= mm - 1) {
        const u32 k = (u32)__builtin_ctzll(mm);
        e = j >= rl(excl, k) ? k : e;
      }
      const u32 a = bperm(A, e), ltv = bperm(lt, e), ctv = bperm(ct, e);
      const u32 r = j - (a & 0xfffu), tle = (a >> 12) & 3u, le = (a >> 14) & 0xffu, xs = a >> 22;
      const u32 x = xs + (r - tle);  // literal byte's position relative to B - 64
      const u32 bp = bperm(xw0p, x & 63), bc = bperm(xw0c, x & 63);
      u32 byte;
      if (r < tle) byte = ltv >> (8 * r);
      else if (r < tle + le) byte = x < 64 ? bp : bc;
      else byte = ctv >> (8 * ((r - tle - le) & 3));
      if (hold && total <= 128) {
        if (j0 == 0) held0 = byte;
        else held1 = byte;
        continue;
      }
      if (j < total) obase[opos + j] = (u8)byte;
    }
    if (hold && total <= 128) {
      held_n = total;
      held_at = opos;
    }
    opos += total;
    EvM = 0;
    FastEv = 0;
    return true;
  };

  u32 next_emit = 0;
  if (n >= kInputMarginBytes) {
    const u32 lim = n - kInputMarginBytes;
    bool post = false;
    u32 p = 1, sk = 32, ip = 0;
    // pipeline state: input of blocks B and B+64, the speculative slot and
    // candidate bytes of the next block, the previous block's input
    u32 curB = 0xffffffffu;  // base of the block whose input is in xw
    W5 xw{}, xw1{}, xwp{};
    Raw20 xr2{};  // input of block curB + 128, in flight
    u32 Tn = 0;
    Raw20 cbn{};
    bool spec = false, prev_ok = false;
    u32 guard = 0;
    for (;;) {
      if (++guard > n / 16 + 64) break;  // cannot happen: every block advances the parse
      const u32 pos = post ? ip : p;
      const u32 B = pos & ~63u;
      // ---- input of this block (and the next one, one block ahead)
      if (curB != 0xffffffffu && B == curB + 64) {
        xwp = xw;
        xw = xw1;
        xw1 = shifted20(xr2);  // issued a block ago
        prev_ok = true;
      } else {
        const Raw20 r0 = raw20(fr, fal + B + lane), r1 = raw20(fr, fal + B + 64 + lane);
        xw = shifted20(r0);
        xw1 = shifted20(r1);
        spec = false;
        prev_ok = false;
      }
      xr2 = raw20(fr, fal + B + 128 + lane);
      curB = B;
      STAMP(0);
      // a copy ending at this block's first position: its ip-1 insert was
      // committed by the previous block if that block was processed
      u64 I = 0;
      if (post) {
        if (ip - 1 < B) {
          if (!prev_ok) {  // ip-1 in a block a long copy jumped: insert it here
            const u32 x = (u32)fb[ip - 1] | (u32)fb[ip] << 8 | (u32)fb[ip + 1] << 16 | (u32)fb[ip + 2] << 24;
            if (lane == 0) table[(x * kHashMul) >> shift] = (u16)(ip - 1);
            lds_fence();
          }
        } else {
          I = 1ull << (ip - 1 - B);
        }
      }
      // ---- table slots and candidate bytes
      const u32 X = xw.w[0];
      const u32 h = (X * kHashMul) >> shift;
      const u32 h1 = (xw1.w[0] * kHashMul) >> shift;
      // (the LDS reads of this block's slots, the next block's speculative
      // slots and the first pred round go out together: one wait)
      const u32 T = table[h];
      const u32 Tn_next = table[h1];
      lds_fence();
      table[h] = (u16)(B + lane);
      lds_fence();
      const u32 rb0 = table[h];
      lds_fence();
      W5 cb;
      {
        // the speculative loads are right unless the previous block changed the slot
        const bool fix = !spec || T != Tn;
        const bool inprev = prev_ok && T + 64 >= B && T < B;
        const u32 src = inprev ? T - (B - 64) : lane;
        W5 pb;
#pragma unroll
        for (int i = 0; i < 5; ++i) pb.w[i] = bperm(xwp.w[i], src);
        const bool need_load = fix && !inprev;
        const W5 sp = spec ? shifted20(cbn) : W5{};
#pragma unroll
        for (int i = 0; i < 5; ++i) cb.w[i] = !fix ? sp.w[i] : pb.w[i];
        // (the load and its wait stay inside the branch: a wait after the
        // join would be counted for the branch-taken path and, on the
        // common path, wait for the input loads issued just before)
        if (__ballot(need_load)) {
          const Raw20 rr = raw20(fr, fal + (need_load ? T : 0u));
          const W5 ld = shifted20(rr);
#pragma unroll
          for (int i = 0; i < 5; ++i) cb.w[i] = need_load ? ld.w[i] : cb.w[i];
        }
      }
      // ---- the next block's slots and candidate loads, speculative: read
      // before this block's pred rounds and commit, so a slot that differs at
      // the next block's start was written by this block's commit (a position
      // of this block: its bytes come from these lanes by ds_bpermute)
      Tn = Tn_next;
      cbn = raw20(fr, fal + Tn);
      spec = true;
      store_held();  // the previous block's output (see held0)
      STAMP(1);
      // ---- pred rounds (the table slots are restored by the commit)
      // Every active lane writes its position into its slot (highest lane
      // wins) and reads it back; the winners leave and listen one more
      // round: what they read then is the winner of that round among their
      // hash's remaining lanes -- the nearest lane below them with their
      // hash, their predecessor -- or their own position if none remain.
      // After a fourth round the lanes still in it are unknown (a chain of
      // five or more; resolved by a scan when probed).  Round 1 went out
      // with the slot reads above.
      u32 p1 = kPredNone;
      {
        bool active = true, listen = false;
        u32 rb = rb0;
        for (int r = 0; r < 4; ++r) {
          if (r > 0) {
            if (!__ballot(active)) break;
            if (active) table[h] = (u16)(B + lane);
            lds_fence();
            rb = (active || listen) ? (u32)table[h] : 0u;
            lds_fence();
          }
          if (listen) p1 = rb != B + lane ? rb - B : (u32)kPredNone;
          if (r == 3) {
            if (active) p1 = kPredUnknown;
            break;
          }
          const bool win = active && rb == B + lane;
          listen = win;
          active = active && !win;
        }
      }
      // (ds_bpermute reads 0 from a lane outside EXEC, so every permute runs
      // on all lanes and the selects come after)
      const u32 t2 = bperm(p1, p1 & 63);
      const u32 p2 = p1 < 64 ? t2 : p1;
      const u32 X1 = bperm(X, p1 & 63);
      W5 w1;
#pragma unroll
      for (int i = 0; i < 5; ++i) w1.w[i] = bperm(xw.w[i], p1 & 63);
      const u32 ml1 = eq_prefix20(xw, w1);
      const bool mT = X == cb.w[0];
      const u32 mlT = eq_prefix20(xw, cb);
      // packed candidates: position | match length << 16 | 4-byte match << 31
      const u32 packT = T | (mlT << 16) | ((u32)mT << 31);
      const u32 packP = (B + (p1 & 63)) | (ml1 << 16) | ((u32)(X == X1) << 31);
      // Lane classes for the event loop, as 64-bit masks: a lane without an
      // in-block predecessor (most) always takes T, so the search is scalar
      // work on these masks; only lanes with a predecessor below the first
      // T-match are looked at one by one.
      const u64 HasP = __ballot(p1 < 64), Unk = __ballot(p1 == kPredUnknown);
      const u64 MTb = __ballot(mT);
      const u64 Deep = __ballot(p1 < 64 && p2 != kPredNone);  // a second predecessor below
      const u64 Stat = ~(HasP | Unk);
      STAMP(2);
      // exact candidate of lane k by a scan of the lanes below it
      auto scan = [&](u32 k, u64 Ims) -> u32 {
        const u32 hk = rl(h, k), xk = rl(X, k);
        u32 j = 64;
        WCOUNT(10);
        for (int i = (int)k - 1; i >= 0; --i) {
          WCOUNT(11);
          if (((Ims >> i) & 1ull) && rl(h, (u32)i) == hk) { j = (u32)i; break; }
        }
        if (j == 64) return rl(packT, k);
        W5 a, b;
#pragma unroll
        for (int i = 0; i < 5; ++i) { a.w[i] = rl(xw.w[i], k); b.w[i] = rl(xw.w[i], j); }
        return (B + j) | (eq_prefix20(a, b) << 16) | ((u32)(rl(X, j) == xk) << 31);
      };
      // packed candidate of a lane with a predecessor (or unknown chain), for
      // the inserted set Ims below it
      auto resolve_p = [&](u32 j, u64 Ims) -> u32 {
        if ((Unk >> j) & 1ull) return scan(j, Ims);
        const u32 pj = rl(p1, j);
        if ((Ims >> pj) & 1ull) return rl(packP, j);
        if (!((Deep >> j) & 1ull)) return rl(packT, j);
        return scan(j, Ims);
      };

      // ---- fast events, precomputed per lane k: the event a post-copy
      // arrival at B + k makes under the fast rules (snappy.cc:428-438 and
      // the stride-1 probes of :377-397): the probe at B + k by a lane with
      // no in-block predecessor; if it misses, the probes B+k+1 .. B+k+c
      // (skip 32..63) up to their first T-match, no predecessor lane among
      // those before it; a match shorter than the 20 compared bytes.  Kept:
      // the next parse position, the inserted lanes, the event record, and
      // FastM, the lanes whose arrival the rules decide.
      u32 fsucc, filo, fihi;
      u64 FastM;
      {
        const u64 SM = Stat & MTb, NS = ~Stat;
        const u32 k = lane;
        const u32 c = 63 - k < 32 ? 63 - k : 32u;
        const u64 S = k < 63 ? ((1ull << c) - 1) << (k + 1) : 0ull;
        const u64 Mst = S & SM;
        const u32 ks = (u32)__builtin_ctzll(Mst | 0x8000000000000000ull);
        const u64 below = (1ull << ks) - 1;
        const bool hit = packT >> 31;
        const bool miss_ok = Mst != 0 && (S & NS & below) == 0 && (int)lim - (int)(B + k) - 1 >= (int)c;
        const u32 pks = bperm(packT, ks);
        const u32 fpk = hit ? packT : pks;
        const u32 fq = hit ? B + k : B + ks;
        u32 fml = (fpk >> 16) & 31u;
        const bool lng = fml >= 20 && fq + 20 < n;
        fml = fml < n - fq ? fml : n - fq;
        // (plus the insert of the next arrival's ip - 1, snappy.cc:432-434,
        // when it lies in the block; after the input limit it is never read)
        const u32 im1 = fq + fml - 1 - B;
        const u64 Iadd = (1ull << k) | (hit ? 0ull : S & ((below << 1) | 1ull)) | (im1 < 64 ? 1ull << im1 : 0ull);
        fsucc = fq + fml;
        filo = (u32)Iadd;
        fihi = (u32)(Iadd >> 32);
        fEQL = fq | ((fq - (B + k)) << 16);
        fECM = (fpk & 0xffffu) | (fml << 16);
        FastM = __ballot(((Stat >> k) & 1ull) && (hit || miss_ok) && !lng);
      }
      STAMP(12);
      bool done = false, leave = false;
      for (u32 ev = 0; !done && !leave && ev < 200; ++ev) {
        // ---- fast events (see the per-lane precomputation above): a walk
        // over the lanes' successors while the arrival lane's event is fast,
        // up to the first arrival past the block or the input limit
        if (post && ((FastM >> (ip - B)) & 1ull)) {
          const u32 stop = lim < B + 64 ? lim : B + 64;
          u32 k0 = ip - B, nip;
          u64 evs = 0, iadd = 0;
          for (;;) {
            nip = rl(fsucc, k0);
            iadd |= ((u64)rl(fihi, k0) << 32) | (u64)rl(filo, k0);
            evs |= 1ull << k0;
            if (nip >= stop) break;
            k0 = nip - B;
            if (!((FastM >> k0) & 1ull)) break;
          }
          I |= iadd;
          EvM |= evs;
          FastEv |= evs;
          ev += (u32)__builtin_popcountll(evs);
          ip = nip;
          next_emit = ip;
          done = ip >= lim;
          leave = !done && ip >= B + 64;
          STAMP(13);
        }
        if (done || leave || ev >= 200) break;
        u32 q = 0, pk = 0;
        bool found = false;
        const u32 key = (post ? ip : p) - B;  // the event's lane (see EvM)
        if (post) {
          // the probe right after a copy (snappy.cc:428-438), lane k0
          const u32 k0 = ip - B;
          pk = ((Stat >> k0) & 1ull) ? rl(packT, k0) : resolve_p(k0, I);
          I |= 1ull << k0;
          if (pk >> 31) {
            q = ip;
            found = true;
          } else {
            post = false;
            p = ip + 1;
            sk = 32;
          }
          STAMP(3);
        }
        if (!found) {
          if (p >= B + 64) { leave = true; break; }
          // the literal search (snappy.cc:377-397) inside this block: the
          // step-1 probes first, then (no match among them) the later ones
          const u32 a = p - B;
          u32 c = 64 - a;
          bool rem = false;
          if (sk < 64 && 64 - sk < c) c = 64 - sk;
          {
            const u32 room_l = lim >= p ? lim - p : 0u;
            if (sk >= 64) c = 0;
            if (room_l < c) { c = room_l; rem = true; }
          }
          u64 S = (c >= 64 ? ~0ull : ((1ull << c) - 1)) << a;
          u32 pp = p + c, s = sk + c;
          u32 ks = 64;
          for (int pass = 0; pass < 2; ++pass) {
            // lanes that always take T: a mask test
            const u64 Mst = S & Stat & MTb;
            ks = Mst ? (u32)__builtin_ctzll(Mst) : 64u;
            if (ks < 64) pk = rl(packT, ks);
            // lanes with a predecessor below it, in order
            u64 D = S & ~Stat & (ks < 64 ? ((1ull << ks) - 1) : ~0ull);
            while (D) {
              const u32 j = (u32)__builtin_ctzll(D);
              const u32 pj = resolve_p(j, I | (S & ((1ull << j) - 1)));
              if (pj >> 31) {
                ks = j;
                pk = pj;
                break;
              }
              D &= D - 1;
            }
            if (ks < 64 || rem || pp >= B + 64 || pass == 1) break;
            // no match among the step-1 probes: the rest of the block
            while (pp < B + 64) {
              const u32 step = s >> 5;
              if (pp + step > lim) { rem = true; break; }
              S |= 1ull << (pp - B);
              pp += step;
              ++s;
            }
          }
          if (ks == 64) {
            // no match left in this block: every probe inserted
            I |= S;
            if (rem) { done = true; break; }
            p = pp;
            sk = s;
            leave = true;
            break;
          }
          I |= S & (ks == 63 ? ~0ull : ((2ull << ks) - 1));
          q = B + ks;
          STAMP(3);
        }
        // literal [next_emit, q) (snappy.cc:403; empty after a copy)
        // ---- copy at q (FindMatchLength, snappy-internal.h:87-121)
        const u32 cand = pk & 0xffffu;
        u32 mlen = (pk >> 16) & 31u;
        if (mlen >= 20 && q + 20 < n) {
          // past the 20 compared bytes: 256 bytes per step, 4 per lane,
          // through the descriptor (two aligned dwords per 4 bytes)
          auto ld4 = [&](u32 P) -> u32 {
            const u32 a4 = (fal + P) & ~3u;
            const u32x2 d = __builtin_amdgcn_raw_buffer_load_b64(fr, a4, 0, 0);
            return ab(d[1], d[0], (fal + P) & 3u);
          };
          u32 m = 20;
          for (;;) {
            const u32 o = m + 4 * lane;
            const bool inr = q + o < n;
            const u32 x = ld4(inr ? cand + o : 0u) ^ ld4(inr ? q + o : 0u);
            u32 eqb = x ? ((u32)__builtin_ctz(x) >> 3) : 4u;
            const u32 left = inr ? n - (q + o) : 0u;
            if (eqb > left) eqb = left;
            const u64 stop = __ballot(eqb < 4);
            if (stop) {
              const u32 l = (u32)__builtin_ctzll(stop);
              m += 4 * l + rl(eqb, l);
              break;
            }
            m += 256;
          }
          mlen = m;
          STAMP(7);
        }
        if (mlen > n - q) mlen = n - q;
        {
          const u32 L = q - next_emit;
          const bool lit_regs = L == 0 || next_emit >= B || (prev_ok && next_emit + 64 >= B);
          if (lit_regs && mlen <= 64) {
            const bool mine = lane == key;
            EQL = mine ? q | (L << 16) : EQL;
            ECM = mine ? cand | (mlen << 16) : ECM;
            EvM |= 1ull << key;
          } else {
            if (!emit_pending(B, X, xwp.w[0])) return nullptr;
            if (L) {
              if (!room(L + 5)) return nullptr;
              emit_literal(next_emit, q, B, X, prev_ok, xwp.w[0]);
            }
            if (!room(3 * (mlen / 60 + 2))) return nullptr;
            emit_copy(q - cand, mlen);
          }
        }
        WCOUNT(9);
        ip = q + mlen;
        next_emit = ip;
        if (ip >= lim) { done = true; break; }
        post = true;
        if (ip - 1 < B + 64) I |= 1ull << (ip - 1 - B);
        if (ip >= B + 64) leave = true;
        STAMP(4);
      }
      STAMP(3);
      // ---- commit: restore the slots the pred rounds overwrote, then the
      // inserted positions (highest lane wins a shared slot)
      table[h] = (u16)T;
      lds_fence();
      if ((I >> lane) & 1ull) table[h] = (u16)(B + lane);
      lds_fence();
      if (!emit_pending(B, X, xwp.w[0], true)) return nullptr;
      STAMP(5);
      WCOUNT(8);
      if (done) break;
      // the next block's speculation holds only for block B + 64
      const u32 npos = post ? ip : p;
      if ((npos & ~63u) != B + 64) spec = false;
    }
  }
  store_held();  // the last block's output
  if (next_emit < n) {
    if (!room(n - next_emit + 5)) return nullptr;
    // remainder (snappy.cc:446-450): bytes from global memory
    emit_literal(next_emit, n, 0xffffffffu, 0u, false, 0u);
  }
  STAMP(6);
#ifdef FSG_STAMPS
  if (lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd(&g_wstamps[k], (unsigned long long)st_[k]);
#endif
  return obase + opos;
}

#ifdef FSG_STAMPS
extern "C" int fsg_debug_wstamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wstamps), sizeof(g_wstamps));
  if (reset) {
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wstamps), z, sizeof(z));
  }
  return e == hipSuccess ? 0 : -1;
}
#endif

// The wave encoder's units: the first `quota` units of encode_plan_kernel's
// long list (every fragment of a split message, every message of [wave_min,
// 64 KiB] bytes; wave_quota), from one work counter (ctr[5]).  Output
// placement as encode_pipe_kernel: a split message's fragment k goes to
// region k of its slot (sizes[] = its length, or ~0 on overflow), a whole
// message to its slot behind the varint header.
//
// A workgroup holds blockDim.x / 64 waves, each with its own table of
// tab_stride entries in the workgroup's LDS (wave w: entries [w tab_stride,
// (w + 1) tab_stride)); the waves share nothing else.  Five waves of 32 KiB
// tables fill the CU's 160 KiB as ONE allocation: five one-wave workgroups of
// 32 KiB do not fit (profiles/r5/wenc/lds_resident_probe.txt: four resident),
// and a single workgroup may declare all 163,840 bytes (MI355X_MICROARCH.md,
// occupancy).
__global__ __launch_bounds__(64 * kWaveEncMaxWaves) void encode_wave_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off, const u32* __restrict__ in_len, u32 n_msgs,
    u8* out, const u64* __restrict__ out_off, u32* __restrict__ out_len, i32* __restrict__ status,
    u32* __restrict__ ctr, const u32* __restrict__ items, u32* __restrict__ sizes, u32 region_cap,
    u32 share_permille, u64 all_bytes, u32 tab_stride) {
  extern __shared__ __attribute__((aligned(16))) u16 wtab_all[];
  const u32 lane = threadIdx.x & 63;
  u16* const wtab = wtab_all + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * tab_stride;
  const u32 quota = (u32)__builtin_amdgcn_readfirstlane((int)wave_quota(ctr, share_permille, all_bytes));
  (void)n_msgs;
  for (;;) {
    const u32 got = atomicAdd(&ctr[5], lane == 0 ? 1u : 0u);
    const u32 w = (u32)__builtin_amdgcn_readfirstlane((int)got);
    if (w >= quota) break;
    u32 m = items[2 * w];
    const u32 f = items[2 * w + 1];
    const bool staged = f != kWholeUnit;
    const u32 f_first = staged ? f << kBlockLog : 0u;
    m = (u32)__builtin_amdgcn_readfirstlane((int)m);
    const u8* mb = in + in_off[m];
    const u32 total = in_len[m];
    const u32 n = staged ? (total - f_first < kBlockSize ? total - f_first : kBlockSize) : total;
    u8* const dst = out + out_off[m];
    const u32 hdr = (u32)varint32_len(total);
    u8* op = dst;
    u8* op_lim = nullptr;
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
      if (lane == 0) {
        u8* hp = dst;
        u32 v = total;
        while (v >= 128) { *hp++ = (u8)(v | 128); v >>= 7; }
        *hp = (u8)v;
      }
      if (!staged) op = dst + hdr;
    }
    const u8* fb = mb + f_first;
    const u32 fal = (u32)(reinterpret_cast<uintptr_t>(fb) & 3);
    const __amdgpu_buffer_rsrc_t fr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u8*>(fb - fal), (short)0, (int)((fal + n + 3) & ~3u), 0x00020000);
    const u32 ht = table_size_for(n);
    u8* end = wave_fragment(fr, fal, fb, n, op, op_lim, wtab, ht, lane);
    if (lane == 0) {
      if (staged) {
        sizes[w] = end ? (u32)(end - region) : 0xffffffffu;
      } else {
        out_len[m] = (u32)(end - dst);
        status[m] = kOk;
      }
    }
  }
}


}  // namespace fsg
