// lz4_cpu.h -- the host-side LZ4 codec of the drop-in (COMPRESS_TYPE_LZ4,
// /root/reference/flare/rpc/options.proto:74, for which the reference
// registers no handler).  Body = varint32 uncompressed length + one LZ4
// block (include/flare_lz4_gpu.h).  Blocks are those of LZ4 1.9.x
// LZ4_compress_default (acceleration 1; 8,192 16-bit positions hashed from 4
// bytes below 65,547 input bytes, 4,096 32-bit positions hashed from 5 bytes
// above), so they equal the GPU kernels' (csrc/lz4.hip) and liblz4's.
// Product code, independent of oracle/lz4_oracle.c.
#pragma once

#include <cstddef>
#include <cstdint>

namespace flare::lz4::cpu {

constexpr size_t kMaxInput = 0x7E000000;  // LZ4_MAX_INPUT_SIZE

// LZ4_compressBound, and the body bound (5 header bytes more).
inline size_t BlockBound(size_t n) { return n + n / 255 + 16; }
inline size_t MaxCompressedLength(size_t n) { return 5 + BlockBound(n); }

// The most a valid block of n bytes can decode to: every byte of a length
// extension adds at most 255 output bytes, a token with its 2-byte offset at
// most 34.  A body whose header claims more is rejected before anything is
// allocated for it.
inline bool PlausibleLength(uint64_t ulen, size_t block_bytes) {
  return ulen <= 255ull * block_bytes + 64;
}

// One block of n <= kMaxInput bytes into out (BlockBound(n) bytes); returns
// its length.
size_t CompressBlock(const uint8_t* in, size_t n, uint8_t* out);

// One block of n bytes to exactly ulen bytes; false when the block is
// invalid (include/flare_lz4_gpu.h states the rules).
bool DecompressBlock(const uint8_t* in, size_t n, uint8_t* out, size_t ulen);

// Body = header + block.  Compress returns the body length (0 above
// kMaxInput); ReadHeader returns the header length or 0.
size_t Compress(const uint8_t* in, size_t n, uint8_t* out);
size_t ReadHeader(const uint8_t* in, size_t n, uint32_t* ulen);

}  // namespace flare::lz4::cpu
