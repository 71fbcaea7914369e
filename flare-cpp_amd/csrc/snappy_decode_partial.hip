// snappy_decode_partial.hip -- the reference's other two decode entry points,
// batched on gfx950 beside Uncompress (paths under /root/reference/flare/io/
// snappy/):
//
//   * UncompressAsMuchAsPossible(Source*, Sink*), snappy.cc:1530-1535: the
//     tag loop through SnappyScatteredWriter (:1331-1481), returning
//     Produced() and handing the sink what was written, also when the
//     stream stops early.
//   * RawUncompressToIOVec(const char*, size_t, const iovec*, size_t),
//     snappy.cc:1122-1132 with SnappyIOVecWriter (:963-1120).
//
// Both start from the batch decoder (fsg_decompress_batch, lenient header):
// a stream it accepts has been written whole, byte-identical to the
// reference's output.
//
//   as much as possible: an accepted stream produced exactly its header
//     length.  Every other message -- the reference stops inside it -- is
//     re-run by partial_kernel, one lane per message, through a model of the
//     scattered writer: 64 KiB blocks (the last cut at the header length),
//     SlowAppend filling the current block before its bounds check (so a
//     literal that overruns the header length leaves the block's part of
//     it, and Produced() counts that block twice, :1424-1451), copies all or
//     nothing, a literal cut by the end of input appended up to there.  The
//     source is cut into `frag`-byte pieces, as the reference's Peek hands
//     them out (a literal is appended piece by piece, which changes where a
//     failing append stops); 0 = one piece.  Corrupt streams are the rare
//     path: one lane walks each, moving literals and copies 16 bytes at a
//     time where the bytes allow it (copies whose source lies 16 or more
//     bytes back, inside the current 64 KiB block), else byte by byte -- a
//     rejected message of L output bytes costs O(L / 16) to O(L) serial
//     steps of one lane.
//   iovec: the decoder writes the caller's staging slot; iov_scatter_kernel,
//     one wave per accepted message, copies it into the message's iovecs in
//     order.  When they hold fewer bytes than the header length the
//     reference fills every iovec with the output's prefix before its
//     `false` (Append and AppendFromSelf copy what fits, then find no next
//     iovec, :1005-1032, :1089-1099), so the kernel copies that prefix and
//     reports FSG_IOV_TOO_SMALL.  A stream the decoder rejected is re-run by
//     iov_model_kernel, one lane per message, through a model of
//     SnappyIOVecWriter writing the iovecs in place, so they end as the
//     reference leaves them: the decoded prefix, a literal cut by the end of
//     input appended up to there, and the 16-byte spill of the last
//     TryFastAppend (:1035-1049) where no later tag overwrote it.  The lane
//     walks byte by byte: a rejected message of L output bytes costs O(L)
//     serial byte operations on one lane (a 64 KiB body ~3 ms).
#include "snappy_device.h"

namespace fsg {

constexpr i32 kIovTooSmall = 4;  // FSG_IOV_TOO_SMALL

namespace {

// SnappyScatteredWriter's state for one message; bytes land at their output
// positions in the slot [o, o + cap).
struct Scatter {
  u8* o;
  u64 cap, expected, full, blk_len, blk_used, hi;
  bool overflow;  // a byte fell past the slot: the result is not representable

  __device__ void put(const u8* p, u64 n) {
    const u64 at = full + blk_used;
    if (at + n > cap) {
      overflow = true;
    } else {
      u64 i = 0;
      for (; i + 16 <= n; i += 16) copy16(o + at + i, p + i);  // 16 bytes at a time
      for (; i < n; ++i) o[at + i] = p[i];
    }
    blk_used += n;
    if (at + n > hi) hi = at + n;
  }
  // Append (:1380-1391) / SlowAppend (:1424-1451)
  __device__ bool append(const u8* p, u64 len) {
    u64 avail = blk_len - blk_used;
    while (len > avail) {
      put(p, avail);
      full += blk_used;  // full_size_ += op_ptr_ - op_base_
      len -= avail;
      p += avail;
      if (full + len > expected) return false;  // op_base_ / op_ptr_ keep the filled block
      blk_len = expected - full < kBlockSize ? expected - full : kBlockSize;
      blk_used = 0;
      avail = blk_len;
    }
    put(p, len);
    return true;
  }
  // AppendFromSelf (:1409-1421) / SlowAppendFromSelf (:1455-1477): checked
  // once, then byte by byte through Append (which cannot fail any more)
  __device__ bool append_from_self(u64 offset, u64 len) {
    const u64 cur = full + blk_used;
    if (offset - 1u >= cur || expected - cur < len) return false;
    u64 i = 0;
    // inside the current block, with the source 16 or more bytes back, a
    // 16-byte chunk reads only bytes already written: whole chunks
    if (offset >= 16 && blk_used + len <= blk_len && cur + len <= cap) {
      for (; i + 16 <= len; i += 16) copy16(o + cur + i, o + cur - offset + i);
      blk_used += i;
      if (cur + i > hi) hi = cur + i;
    }
    for (; i < len && !overflow; ++i) {
      const u8 c = o[cur - offset + i];
      append(&c, 1);
    }
    return true;
  }
};

// bytes left in the source piece holding position pos (Source::Peek)
__device__ __forceinline__ u64 piece_left(u64 pos, u64 n, u64 frag) {
  if (pos >= n) return 0;
  if (!frag) return n - pos;
  const u64 end = (pos / frag + 1) * frag;
  return (end < n ? end : n) - pos;
}

}  // namespace

// One lane per message.  On entry status[] / got[] hold the batch decoder's
// verdict and header length; accepted messages only copy got to produced.
__global__ __launch_bounds__(64) void partial_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                                     const u32* __restrict__ in_len, u32 n_msgs, u32 frag,
                                                     u8* __restrict__ out, const u64* __restrict__ out_off,
                                                     const u32* __restrict__ out_cap, u32* __restrict__ got,
                                                     u64* __restrict__ produced, i32* __restrict__ status) {
  const u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs) return;
  if (status[m] == kOk) {
    produced[m] = got[m];
    return;
  }
  const u8* ip = in + in_off[m];
  const u64 n = in_len[m];
  // ReadUncompressedLength (:692-711): a 6th byte or the end of input fails
  u32 expected = 0, shift = 0;
  u64 pos = 0;
  for (;;) {
    if (shift >= 32 || pos >= n) {
      produced[m] = 0;
      got[m] = 0;
      status[m] = kBadHeader;
      return;
    }
    const u32 c = ip[pos++];
    expected |= (c & 0x7fu) << shift;
    if (c < 128) break;
    shift += 7;
  }
  Scatter w{out + out_off[m], out_cap[m], expected, 0, 0, 0, 0, false};
  bool eof = false;
  for (;;) {  // DecompressAllTags (:716-787), RefillTag (:790-847)
    if (pos == n) {
      eof = true;
      break;
    }
    const u32 c = ip[pos];
    const u32 type = c & 3;
    const u32 l0 = (c >> 2) + 1;
    const u32 extra = type == 0 ? (l0 > 60 ? l0 - 60 : 0u) : (type == 1 ? 1u : (type == 2 ? 2u : 4u));
    if (n - pos < 1 + (u64)extra) break;  // a tag cut by the end of input
    u32 v = 0;
    for (u32 k = 0; k < extra; ++k) v |= (u32)ip[pos + 1 + k] << (8 * k);
    pos += 1 + extra;
    if (type == 0) {
      u64 len = extra ? (u64)(u32)(v + 1u) : (u64)l0;  // uint32: 0xffffffff + 1 == 0
      bool ok = true;
      for (;;) {  // the literal, piece by piece (:751-761)
        const u64 a = piece_left(pos, n, frag);
        if (a >= len) {
          if (len) ok = w.append(ip + pos, len);
          pos += len;
          break;
        }
        if (a == 0 || !w.append(ip + pos, a)) {  // premature end of input, or no room
          ok = false;
          break;
        }
        pos += a;
        len -= a;
      }
      if (!ok) break;
    } else {
      const u64 len = type == 1 ? 4 + ((c >> 2) & 7) : l0;
      const u64 offset = type == 1 ? (((u64)(c >> 5) << 8) | v) : (u64)v;
      if (!w.append_from_self(offset, len)) break;
    }
    if (w.overflow) break;
  }
  if (w.overflow) {
    status[m] = kSlotTooSmall;
    got[m] = 0;
    produced[m] = 0;
    return;
  }
  got[m] = (u32)w.hi;                                // Flush(Produced()): every byte written
  produced[m] = w.full + w.blk_used;                 // Produced()
  status[m] = eof && w.full + w.blk_used == expected ? kOk : kCorrupt;
}

// One wave per message: an accepted stream's staged output into its iovecs
// [iov_first[m], iov_first[m + 1]) in order (SnappyIOVecWriter fills them
// one after another, :1005-1032), when they hold the header length.
__global__ __launch_bounds__(256) void iov_scatter_kernel(const u8* __restrict__ stage,
                                                          const u64* __restrict__ stage_off,
                                                          const u32* __restrict__ out_len, u32 n_msgs,
                                                          const u64* __restrict__ iov_base,
                                                          const u64* __restrict__ iov_len,
                                                          const u32* __restrict__ iov_first,
                                                          i32* __restrict__ status) {
  const u32 lane = threadIdx.x & 63;
  const u32 m = (u32)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
  if (m >= n_msgs || status[m] != kOk) return;
  u64 ulen = out_len[m];
  const u32 j0 = iov_first[m], j1 = iov_first[m + 1];
  u64 room = 0;
  for (u32 j = j0 + lane; j < j1; j += 64) room += iov_len[j];
  for (int s = 32; s > 0; s >>= 1) room += __shfl_xor(room, s, 64);
  if (room < ulen) {
    // the reference's `false` after filling every iovec with the prefix
    if (lane == 0) status[m] = kIovTooSmall;
    ulen = room;
  }
  const u8* src = stage + stage_off[m];
  u64 pos = 0;
  for (u32 j = j0; j < j1 && pos < ulen; ++j) {
    const u64 len = iov_len[j];
    const u64 take = len < ulen - pos ? len : ulen - pos;
    u8* dst = reinterpret_cast<u8*>(iov_base[j]);
    const u8* s = src + pos;
    u64 k = 16 * (u64)lane;
    for (; k + 16 <= take; k += 16 * 64) copy16(dst + k, s + k);
    for (; k < take; ++k) dst[k] = s[k];  // the tail: < 16 bytes, one lane
    pos += take;
  }
}

namespace {
// SnappyIOVecWriter (snappy.cc:963-1120) over the message's iovecs
// [j0, j0 + cnt): bytes land in place.
struct IovWriter {
  const u64* base;
  const u64* len;
  u32 cnt, cur;
  u64 written, total, limit;

  __device__ u8* at(u32 j, u64 off) const { return reinterpret_cast<u8*>(base[j]) + off; }
  // Append (:1005-1032)
  __device__ bool append(const u8* p, u64 n) {
    if (total + n > limit) return false;
    while (n > 0) {
      if (written >= len[cur]) {
        if (cur + 1 >= cnt) return false;
        written = 0;
        ++cur;
      }
      u64 k = len[cur] - written;
      if (k > n) k = n;
      u8* d = at(cur, written);
      for (u64 i = 0; i < k; ++i) d[i] = p[i];
      written += k;
      total += k;
      p += k;
      n -= k;
    }
    return true;
  }
  // TryFastAppend (:1035-1049): 16 bytes copied, len of them counted
  __device__ bool try_fast(const u8* p, u64 available, u64 n) {
    if (n <= 16 && available >= 16 + 5 && limit - total >= 16 && len[cur] - written >= 16) {
      u8* d = at(cur, written);
      for (u32 i = 0; i < 16; ++i) d[i] = p[i];
      written += n;
      total += n;
      return true;
    }
    return false;
  }
  // AppendFromSelf (:1051-1117): the source found by walking back over the
  // earlier iovecs; pieces from them through Append (result unchecked), the
  // rest byte by byte inside the current iovec (IncrementalCopy)
  __device__ bool append_from_self(u64 offset, u64 n) {
    if (offset > total || offset == 0) return false;
    if (n > limit - total) return false;
    u32 fi = cur;
    u64 fo = written;
    while (offset > 0) {
      if (fo >= offset) {
        fo -= offset;
        break;
      }
      offset -= fo;
      --fi;
      fo = len[fi];
    }
    while (n > 0) {
      if (fi != cur) {
        u64 k = len[fi] - fo;
        if (k > n) k = n;
        (void)append(at(fi, fo), k);
        n -= k;
        if (n > 0) {
          ++fi;
          fo = 0;
        }
      } else {
        u64 k = len[cur] - written;
        if (k == 0) {
          if (cur + 1 >= cnt) return false;
          ++cur;
          written = 0;
          continue;
        }
        if (k > n) k = n;
        u8* d = at(cur, written);
        const u8* s = at(fi, fo);
        for (u64 i = 0; i < k; ++i) d[i] = s[i];
        written += k;
        fo += k;
        total += k;
        n -= k;
      }
    }
    return true;
  }
};
}  // namespace

// One lane per message the batch decoder rejected (kCorrupt): the tag loop
// (DecompressAllTags :716-787 over a flat source, RefillTag :790-847) through
// IovWriter, so the iovecs end as RawUncompressToIOVec leaves them.  The
// verdict stays the decoder's.
__global__ __launch_bounds__(64) void iov_model_kernel(const u8* __restrict__ in, const u64* __restrict__ in_off,
                                                       const u32* __restrict__ in_len, u32 n_msgs,
                                                       const u64* __restrict__ iov_base,
                                                       const u64* __restrict__ iov_len,
                                                       const u32* __restrict__ iov_first,
                                                       const i32* __restrict__ status) {
  const u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs || status[m] != kCorrupt) return;
  const u8* ip = in + in_off[m];
  const u64 n = in_len[m];
  // ReadUncompressedLength (:692-711): the decoder accepted the header
  u32 expected = 0, shift = 0;
  u64 pos = 0;
  for (;;) {
    if (shift >= 32 || pos >= n) return;
    const u32 c = ip[pos++];
    expected |= (c & 0x7fu) << shift;
    if (c < 128) break;
    shift += 7;
  }
  const u32 j0 = iov_first[m], cnt = iov_first[m + 1] - j0;
  if (cnt == 0) return;  // no iovec to write (with output to place the reference reads iov[0])
  IovWriter w{iov_base + j0, iov_len + j0, cnt, 0, 0, 0, expected};
  for (;;) {
    if (pos == n) return;
    const u32 c = ip[pos];
    const u32 type = c & 3;
    const u32 l0 = (c >> 2) + 1;
    const u32 extra = type == 0 ? (l0 > 60 ? l0 - 60 : 0u) : (type == 1 ? 1u : (type == 2 ? 2u : 4u));
    if (n - pos < 1 + (u64)extra) return;  // a tag cut by the end of input
    u32 v = 0;
    for (u32 k = 0; k < extra; ++k) v |= (u32)ip[pos + 1 + k] << (8 * k);
    pos += 1 + extra;
    if (type == 0) {
      u64 len = extra ? (u64)(u32)(v + 1u) : (u64)l0;
      if (!extra && w.try_fast(ip + pos, n - pos, len)) {  // :736, before any length bytes
        pos += len;
        continue;
      }
      const u64 a = n - pos;
      if (a < len) {  // premature end of input: the bytes there are appended first
        if (a) (void)w.append(ip + pos, a);
        return;
      }
      if (len && !w.append(ip + pos, len)) return;
      pos += len;
    } else {
      const u64 len = type == 1 ? 4 + ((c >> 2) & 7) : l0;
      const u64 offset = type == 1 ? (((u64)(c >> 5) << 8) | v) : (u64)v;
      if (!w.append_from_self(offset, len)) return;
    }
  }
}

hipError_t launch_decode_partial(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u32 frag,
                                 u8* out, const u64* out_off, const u32* out_cap, u32* got, u64* produced,
                                 i32* status, hipStream_t stream) {
  if (!n_msgs) return hipSuccess;
  partial_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, frag, out, out_off,
                                                         out_cap, got, produced, status);
  return hipGetLastError();
}

hipError_t launch_iov_scatter(const u8* in, const u64* in_off, const u32* in_len, const u8* stage,
                              const u64* stage_off, const u32* out_len, u32 n_msgs, const u64* iov_base,
                              const u64* iov_len, const u32* iov_first, i32* status, hipStream_t stream) {
  if (!n_msgs) return hipSuccess;
  iov_scatter_kernel<<<(n_msgs + 3) / 4, 256, 0, stream>>>(stage, stage_off, out_len, n_msgs, iov_base, iov_len,
                                                          iov_first, status);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  iov_model_kernel<<<(n_msgs + 63) / 64, 64, 0, stream>>>(in, in_off, in_len, n_msgs, iov_base, iov_len, iov_first,
                                                         status);
  return hipGetLastError();
}

}  // namespace fsg
