// snappy_lane_decode.h -- the reference's tag loop for one message on one
// lane (/root/reference/flare/io/snappy/snappy.cc:716-787 with the writer
// checks of :1141-1227 / :1331-1481).  Used by the lane-per-message kernel
// (snappy_decode.hip) and by the two-pass decoder's fallback pass for the
// messages whose tag bitmap did not fit the workspace (snappy_decode_v4.hip).
#pragma once

#include "snappy_device.h"

namespace fsg {

// One message.  Returns a status word.  `op_base` may be null when
// validate-only.
__device__ inline i32 decode_one(const u8* ip, const u8* ip_end, u8* op_base,
                          u32 expected, bool write) {
  u32 op = 0;
  for (;;) {
    if (ip == ip_end) return op == expected ? kOk : kCorrupt;  // RefillTag eof
    u32 c = *ip++;
    u32 avail = (u32)(ip_end - ip);
    u32 space = expected - op;
    if ((c & 3) == 0) {
      u32 len = (c >> 2) + 1;
      // TryFastAppend fast path (snappy.cc:1392-1405): 16-byte copy when the
      // input and output both have 16 bytes of room.
      if (len <= 16 && avail >= 16 && space >= 16) {
        if (write) copy16(op_base + op, ip);
        op += len;
        ip += len;
        continue;
      }
      if (len >= 61) {  // long literal, 1..4 length bytes (:744-750)
        u32 nb = len - 60;
        if (avail < nb) return kCorrupt;  // RefillTag cannot stitch the tag
        u32 v = 0;
        for (u32 k = 0; k < nb; ++k) v |= (u32)ip[k] << (8 * k);
        len = v + 1;  // uint32 wrap: 0xffffffff + 1 == 0 (a no-op literal)
        ip += nb;
        avail -= nb;
      }
      if (avail < len) return kCorrupt;  // premature end of input (:761)
      if (space < len) return kCorrupt;  // writer overrun
      if (write) {
        u8* d = op_base + op;
        u32 k = 0;
        for (; k + 16 <= len; k += 16) copy16(d + k, ip + k);
        for (; k < len; ++k) d[k] = ip[k];
      }
      op += len;
      ip += len;
    } else {
      u32 type = c & 3;
      u32 nb = type == 1 ? 1u : (type == 2 ? 2u : 4u);
      if (avail < nb) return kCorrupt;
      u32 len, offset;
      if (type == 1) {  // COPY_1_BYTE_OFFSET: len 4..11, 11-bit offset
        len = 4 + ((c >> 2) & 7);
        offset = ((c >> 5) << 8) | ip[0];
      } else if (type == 2) {  // COPY_2_BYTE_OFFSET
        len = (c >> 2) + 1;
        offset = (u32)ip[0] | ((u32)ip[1] << 8);
      } else {  // COPY_4_BYTE_OFFSET
        len = (c >> 2) + 1;
        offset = (u32)ip[0] | ((u32)ip[1] << 8) | ((u32)ip[2] << 16) |
                 ((u32)ip[3] << 24);
      }
      ip += nb;
      // "produced <= offset - 1u" (:1200): offset 0 or beyond produced.
      if (offset - 1u >= op) return kCorrupt;
      if (space < len) return kCorrupt;
      if (write) {
        u8* d = op_base + op;
        const u8* s = d - offset;
        if (offset >= 8 && space >= len + 8) {
          // Non-overlapping 8-byte steps; may scribble < 8 bytes past len
          // inside the slot, rewritten by later tags.
          for (u32 k = 0; k < len; k += 8) stu64(d + k, ldu64(s + k));
        } else if (space >= len + 10) {
          // IncrementalCopyFastPath (:140-152): widen the pattern until the
          // distance is >= 8, then 8-byte steps (<= 10 bytes of over-write).
          u8* dd = d;
          const u8* ss = s;
          int rem = (int)len;
          while (dd - ss < 8) {
            stu64(dd, ldu64(ss));
            rem -= (int)(dd - ss);
            dd += dd - ss;
          }
          while (rem > 0) {
            stu64(dd, ldu64(ss));
            ss += 8;
            dd += 8;
            rem -= 8;
          }
        } else {
          for (u32 k = 0; k < len; ++k) d[k] = s[k];  // IncrementalCopy (:98-103)
        }
      }
      op += len;
    }
  }
}

}  // namespace fsg
