// snappy_cpu.h -- the host-side Snappy codec of the drop-in: what the
// CompressHandler runs where a GPU job cannot pay off or cannot run (bodies
// below the size threshold, nodes without a usable GPU, a HIP error on the
// device path).  Bytes and verdicts are the reference's
// (/root/reference/flare/io/snappy/snappy.cc, vendored Snappy 1.1.3):
//
//   Compress                 snappy.cc:875-954 (64 KiB fragments, varint
//                            header) + CompressFragment :329-453 (greedy
//                            LZ77, hash table per WorkingMemory::GetHashTable
//                            :247-271, EmitLiteral :156-196, EmitCopy
//                            :198-232, FindMatchLength snappy-internal.h:87-121)
//   Decode / DecodePartial   DecompressAllTags :716-787 with the writers'
//                            checks (SnappyArrayWriter :1141-1227,
//                            SnappyScatteredWriter :1331-1481); DecodePartial
//                            also returns what the scattered writer would
//                            have flushed on failure (UncompressAsMuchAsPossible
//                            :1530-1535, InternalUncompress :858-868)
//
// This is product code, independent of the test oracle under oracle/.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace flare::snappy::cpu {

// snappy.cc:55-77: 32 + n + n/6.
inline size_t MaxCompressedLength(size_t n) { return 32 + n + n / 6; }

// Varint32 header.  strict: Parse32WithLimit (a 5th byte >= 16 is an error,
// snappy-stubs-internal.h:327-357); lenient: ReadUncompressedLength (the 5th
// byte's high bits fall off, snappy.cc:692-711).  Returns the header length,
// 0 if there is none.
size_t ReadHeader(const uint8_t* in, size_t n, uint32_t* len, bool strict);

// Compresses n bytes into `out` (at least MaxCompressedLength(n) bytes);
// returns the compressed length.  Never fails.
size_t Compress(const uint8_t* in, size_t n, uint8_t* out);

// Decodes the tags after a header of `hdr` bytes into out[0, expected).
// Returns true iff the reference accepts the stream.  *produced (optional)
// receives the bytes the reference's scattered writer holds when it stops:
// every completed tag, plus the part of a literal that fit the input and the
// header length (copies are all-or-nothing).  `out` needs `expected` bytes;
// `out_cap` > expected lets the fast paths over-write up to 16 bytes past
// the produced bytes (never past out_cap).
bool Decode(const uint8_t* in, size_t n, size_t hdr, uint8_t* out, uint32_t expected,
            size_t* produced = nullptr, size_t out_cap = 0);

// Header (lenient unless `strict`) + Decode.  `out` needs the header length.
bool Uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, bool strict);

// UncompressAsMuchAsPossible(Source*, Sink*) (snappy.cc:1530-1535) over an
// input cut into fragments (what Source::Peek hands out: cord_buf blocks).
// Models SnappyScatteredWriter exactly (64 KiB blocks capped at the header
// length, SlowAppend filling the current block before its bounds check,
// :1424-1451), so `out` (resized) receives the bytes the reference's sink
// would, and the return value is the reference's: Produced(), which counts
// the block just completed twice when SlowAppend fails (full_size_ already
// holds it while op_base_ still points at it).  A bad header returns 0.
size_t UncompressAsMuchAsPossible(const uint8_t* const* frag, const size_t* frag_len, size_t n_frag,
                                  std::vector<uint8_t>* out);

// The decoder's verdict without keeping output (IsValidCompressedBuffer,
// snappy.cc:1254-1299): a validator that only counts.
bool IsValid(const uint8_t* in, size_t n);

}  // namespace flare::snappy::cpu
