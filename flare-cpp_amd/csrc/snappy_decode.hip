// snappy_decode.hip -- batched Snappy decode for gfx950.
//
// decode_lane_kernel: one LANE per message.  Each lane runs the reference's
// tag loop (SnappyDecompressor::DecompressAllTags,
// /root/reference/flare/io/snappy/snappy.cc:716-787) on a flat compressed
// body with the writer checks of the reference's writers (SnappyArrayWriter
// :1141-1227 / SnappyScatteredWriter :1331-1481 / validator :1254-1288): every
// status is identical to the reference's bool, every output byte identical.
// A wave therefore walks 64 independent messages at once; every load/store
// is a per-lane 8/16-byte unaligned access into that lane's own slot, so no
// lane ever reads or writes another lane's bytes and no cross-lane ordering
// is needed.  Writes never pass the slot's expected length (the reference's
// 16-byte over-writes are only taken when the space-left checks allow).
#include "snappy_lane_decode.h"

namespace fsg {

// ReadUncompressedLength (snappy.cc:692-711) or Parse32WithLimit
// (snappy-stubs-internal.h:327-357).  Returns header length, 0 if invalid.
__device__ __forceinline__ int parse_header(const u8* ip, u32 n, bool strict,
                                            u32* ulen) {
  u32 r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((u32)i >= n) return 0;
    u32 c = ip[i];
    r |= (c & 0x7fu) << (7 * i);  // i == 4: bits above 31 fall off
    if (c < 128) {
      if (strict && i == 4 && c >= 16) return 0;
      *ulen = r;
      return i + 1;
    }
  }
  return 0;  // a 6th byte would be needed: shift >= 32
}

__global__ __launch_bounds__(256) void decode_lane_kernel(
    const u8* __restrict__ in, const u64* __restrict__ in_off,
    const u32* __restrict__ in_len, u32 n_msgs, u8* out,
    const u64* __restrict__ out_off, const u32* __restrict__ out_cap,
    u32* __restrict__ out_len, i32* __restrict__ status, u32 flags) {
  u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs) return;
  const bool validate_only = flags & 1u;
  const bool strict = flags & 2u;
  const u8* ip = in + in_off[m];
  u32 n = in_len[m];
  u32 ulen = 0;
  int h = parse_header(ip, n, strict, &ulen);
  if (h == 0) {
    out_len[m] = 0;
    status[m] = kBadHeader;
    return;
  }
  out_len[m] = ulen;
  if (!validate_only && ulen > out_cap[m]) {
    status[m] = kSlotTooSmall;
    return;
  }
  u8* op = validate_only ? nullptr : out + out_off[m];
  status[m] = decode_one(ip + h, ip + n, op, ulen, !validate_only);
}

__global__ void header_kernel(const u8* __restrict__ in,
                              const u64* __restrict__ in_off,
                              const u32* __restrict__ in_len, u32 n_msgs,
                              u32* __restrict__ ulen_out, int lenient) {
  u32 m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_msgs) return;
  u32 ulen = 0;
  int h = parse_header(in + in_off[m], in_len[m], !lenient, &ulen);
  ulen_out[m] = h ? ulen : 0xffffffffu;
}

hipError_t launch_decode(const u8* in, const u64* in_off, const u32* in_len,
                         u32 n_msgs, u8* out, const u64* out_off,
                         const u32* out_cap, u32* out_len, i32* status,
                         u32 flags, hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  const u32 tpb = 64;
  decode_lane_kernel<<<(n_msgs + tpb - 1) / tpb, tpb, 0, stream>>>(
      in, in_off, in_len, n_msgs, out, out_off, out_cap, out_len, status, flags);
  return hipGetLastError();
}

hipError_t launch_headers(const u8* in, const u64* in_off, const u32* in_len,
                          u32 n_msgs, u32* ulen, int lenient,
                          hipStream_t stream) {
  if (n_msgs == 0) return hipSuccess;
  header_kernel<<<(n_msgs + 255) / 256, 256, 0, stream>>>(in, in_off, in_len,
                                                          n_msgs, ulen, lenient);
  return hipGetLastError();
}

}  // namespace fsg
