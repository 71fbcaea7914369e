/*
 * flare_lz4_gpu.h -- batched LZ4 block codec on MI355X (gfx950), in
 * libflare_snappy_gpu.so next to the Snappy calls (include/flare_snappy_gpu.h:
 * same batch layout, same status words, same fsg_init / fsg_last_error).
 *
 * Reference interface: none to replace.  The reference names
 * COMPRESS_TYPE_LZ4 = 4 (flare/rpc/options.proto:74) but registers no
 * handler for it (flare/rpc/compress.cc:26-103 holds only what
 * RegisterCompressHandler is given; flare/rpc/global.cc:372-376 registers
 * Snappy/gzip/zlib).  These calls and host/lz4_compress.cc are the handler a
 * maintainer would register at that slot.
 *
 * RPC body (our definition): varint32 of the uncompressed length, then one
 * LZ4 block.  Blocks are byte-equal to LZ4 1.9.x LZ4_compress_default; the
 * decoder accepts exactly the blocks LZ4_decompress_safe(dst capacity =
 * uncompressed length) accepts, except a match of offset 0 (rejected here).
 */
#ifndef FLARE_LZ4_GPU_H_
#define FLARE_LZ4_GPU_H_

#include <stddef.h>
#include <stdint.h>

#include "flare_snappy_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Output slot size of one body: 5 (header) + LZ4_compressBound(n). */
size_t fsg_lz4_max_compressed_length(size_t n);

/* Device workspace for fsg_lz4_compress_batch: 16 KiB of position table
 * per message. */
size_t fsg_lz4_compress_workspace_bytes(uint32_t n_msgs);

/* Batched compress: message i is d_in[d_in_off[i] .. +d_in_len[i]); its body
 * is written to d_out[d_out_off[i] ..] (slot of
 * fsg_lz4_max_compressed_length(d_in_len[i]) bytes, slots disjoint);
 * d_out_len[i] = body length, d_status[i] FSG_OK (FSG_CORRUPT above
 * 0x7E000000 input bytes, LZ4_MAX_INPUT_SIZE). */
int fsg_lz4_compress_batch(const uint8_t *d_in, const uint64_t *d_in_off,
                           const uint32_t *d_in_len, uint32_t n_msgs,
                           uint8_t *d_out, const uint64_t *d_out_off,
                           uint32_t *d_out_len, int32_t *d_status,
                           void *d_workspace, size_t workspace_bytes,
                           void *stream);

/* Batched decompress: bodies in, d_out[d_out_off[i] ..] with capacity
 * d_out_cap[i]; d_out_len[i] = the header's length; d_status[i]: FSG_OK,
 * FSG_CORRUPT, FSG_BAD_HEADER (varint32, at most 5 bytes), or
 * FSG_SLOT_TOO_SMALL. */
int fsg_lz4_decompress_batch(const uint8_t *d_in, const uint64_t *d_in_off,
                             const uint32_t *d_in_len, uint32_t n_msgs,
                             uint8_t *d_out, const uint64_t *d_out_off,
                             const uint32_t *d_out_cap, uint32_t *d_out_len,
                             int32_t *d_status, void *stream);

/* Device workspace for fsg_lz4_decompress_batch_ws: counters, two u32 per
 * message and the sequence bitmap (one bit per block byte). */
size_t fsg_lz4_decompress_workspace_bytes(uint32_t n_msgs, uint64_t total_in_bytes);

/* fsg_lz4_decompress_batch (same arguments, statuses and bytes) on the
 * two-pass decoder: a lane-per-message index pass (validation + sequence
 * bitmap; blocks over 64 KiB, or over 2 KiB in batches of <= 256 messages,
 * indexed by a wave each), then a wave-per-message execution pass.  Messages whose bitmap
 * does not fit the workspace, or every message when d_workspace is NULL or
 * smaller than fsg_lz4_decompress_workspace_bytes(n_msgs, 0), run the
 * one-pass kernel. */
int fsg_lz4_decompress_batch_ws(const uint8_t *d_in, const uint64_t *d_in_off,
                                const uint32_t *d_in_len, uint32_t n_msgs,
                                uint8_t *d_out, const uint64_t *d_out_off,
                                const uint32_t *d_out_cap, uint32_t *d_out_len,
                                int32_t *d_status, void *d_workspace,
                                size_t workspace_bytes, void *stream);

/* fsg_lz4_decompress_batch_ws in two streams: the index pass (validation +
 * sequence bitmap) on `pass1_stream`, the execution and fallback passes on
 * `stream` behind an event, so that batch k+1's index pass (latency-bound,
 * one lane per message) runs beside batch k's execution (issue-bound) when
 * the two batches have their own workspace, output, d_out_len and d_status
 * buffers.  The inputs must be ready on `pass1_stream`; calls sharing any of
 * those buffers must be ordered by the caller.  Results are valid once
 * `stream` is synchronised.  Same statuses and bytes as
 * fsg_lz4_decompress_batch.  (Snappy's counterpart: fsg_decompress_batch_2s.) */
int fsg_lz4_decompress_batch_2s(const uint8_t *d_in, const uint64_t *d_in_off,
                                const uint32_t *d_in_len, uint32_t n_msgs,
                                uint8_t *d_out, const uint64_t *d_out_off,
                                const uint32_t *d_out_cap, uint32_t *d_out_len,
                                int32_t *d_status, void *d_workspace,
                                size_t workspace_bytes, void *stream,
                                void *pass1_stream);

#ifdef __cplusplus
}
#endif
#endif /* FLARE_LZ4_GPU_H_ */
