/*
 * flare_snappy_gpu.h -- C ABI of the MI355X (gfx950) batched Snappy codec.
 *
 * This is the drop-in boundary underneath flare's CompressType plugin
 * surface.  Each entry point replaces one piece of the reference's CPU path
 * (paths relative to /root/reference):
 *
 *   fsg_max_compressed_length      flare/io/snappy/snappy.cc:55-77
 *                                  (snappy::MaxCompressedLength)
 *   fsg_get_uncompressed_length    snappy.cc:235-244 (strict,
 *                                  GetUncompressedLength(const char*,...))
 *                                  and snappy.cc:692-711 / 870-873 (lenient,
 *                                  GetUncompressedLength(Source*,...))
 *   fsg_compress_batch             snappy.cc:875-954 (snappy::Compress(Source*,
 *                                  Sink*)) as called per message by
 *                                  flare/rpc/policy/snappy_compress.cc:28-38,51-55
 *   fsg_decompress_batch           snappy.cc:1537-1563 (snappy::Uncompress(
 *                                  Source*, Sink*)) as called by
 *                                  snappy_compress.cc:40-49,57-61; with
 *                                  FSG_FLAG_VALIDATE_ONLY it is
 *                                  IsValidCompressed (snappy.cc:1290-1299);
 *                                  with FSG_FLAG_STRICT_HEADER it is the flat
 *                                  Uncompress(const char*, size_t, string*)
 *                                  (snappy.cc:1239-1251).
 *   fsg_decompress_batch_partial   snappy.cc:1530-1535
 *                                  (snappy::UncompressAsMuchAsPossible(
 *                                  Source*, Sink*), SnappyScatteredWriter
 *                                  :1331-1481)
 *   fsg_decompress_batch_iovec     snappy.cc:1122-1132
 *                                  (snappy::RawUncompressToIOVec(const char*,
 *                                  size_t, const iovec*, size_t),
 *                                  SnappyIOVecWriter :963-1120)
 *
 * Conventions: plain C, no exceptions, no torch types.  All buffers passed
 * to *_batch functions are DEVICE pointers (hipMalloc'd or device-mapped
 * pinned host memory); `stream` is a hipStream_t (NULL = default stream).
 * The calls are asynchronous on `stream`: results are valid after the
 * stream is synchronised.  Every function is thread-safe; no global state
 * is mutated after fsg_init.
 *
 * Per-message status words (int32):
 *   FSG_OK              the reference returns true and the output bytes are
 *                       byte-identical to the reference's.
 *   FSG_CORRUPT         the reference returns false (bad offset, overrun,
 *                       premature end, trailing tags, truncated tag).
 *   FSG_BAD_HEADER      the reference returns false while reading the
 *                       varint uncompressed-length header.
 *   FSG_SLOT_TOO_SMALL  caller sizing error: the header's uncompressed length
 *                       exceeds the output slot (not a reference verdict;
 *                       size slots with fsg_get_uncompressed_length).
 *   FSG_IOV_TOO_SMALL   (fsg_decompress_batch_iovec) the stream is valid but
 *                       its iovecs hold fewer bytes than the header's length:
 *                       the reference returns false.
 * On any status other than FSG_OK the content of the output slot is
 * unspecified (the reference's partial output on failure depends on the
 * source fragmentation, snappy.cc:866, and every caller discards it).
 */
#ifndef FLARE_SNAPPY_GPU_H_
#define FLARE_SNAPPY_GPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSG_OK 0
#define FSG_CORRUPT 1
#define FSG_BAD_HEADER 2
#define FSG_SLOT_TOO_SMALL 3
#define FSG_IOV_TOO_SMALL 4

/* Return codes of the host-side calls. */
#define FSG_SUCCESS 0
#define FSG_ERR_INVALID_ARG -1
#define FSG_ERR_HIP -2
#define FSG_ERR_NO_DEVICE -3

/* decompress flags */
#define FSG_FLAG_VALIDATE_ONLY 1u /* IsValidCompressed: no output written   */
#define FSG_FLAG_STRICT_HEADER 2u /* Parse32WithLimit header (flat API)     */

/* Library version string, e.g. "flare-snappy-gpu 0.1 gfx950". */
const char *fsg_version(void);

/* Binds the calling host thread to `device` and caches its properties.
 * Idempotent.  Returns FSG_SUCCESS or a negative error. */
int fsg_init(int device);

/* Last HIP error text seen by this library on the calling thread. */
const char *fsg_last_error(void);

/* Kernel variants for A/B measurement and tests: 0 = automatic choice,
 * 1 = first-generation kernels (decode: one lane per message, tag by tag;
 * encode: one wave per message with the hash table in LDS), 3 = third
 * generation (decode: software-pipelined batched pieces, one lane per
 * message; encode: lane per message with batched speculative probes and the
 * tables in the workspace, the default encoder), 4 = decode only: the
 * two-pass decoder (lane-per-message index pass writing a tag-start bitmap,
 * then one wave per message executing <= 16-byte pieces in dependency rounds
 * through an LDS output window), the default decoder whenever the workspace
 * holds its bitmap, 5 = decode only: the same two passes with one TAG per
 * lane in the execution pass (registers hold a short literal's bytes from the
 * tag prefetch; no piece map), the default since round 3.  (Generation 2 was
 * retired; 2 is rejected.)  Every
 * variant produces identical bytes and statuses.  Process-wide; not for use
 * while other threads launch batches. */
int fsg_select_kernels(int decode_variant, int encode_variant);

/* Test knob: caps the staging region of each fragment of a message longer
 * than 64 KiB (bytes; 0 = the slot split evenly, the default).  A fragment
 * whose output does not fit its region sends its message through the
 * whole-message fallback pass; small caps exercise that path.  Bytes are
 * unaffected.  Process-wide. */
int fsg_set_split_region_cap(uint32_t bytes);

/* Process-wide tuning and test options (no counterpart in the reference,
 * whose codec has no launch choices).  Each starts from its FSG_<NAME>
 * environment variable, read once when the library is loaded; the launch
 * paths read only this table, never the environment.  Names (values are
 * integers; -1 = the library's automatic rule where one exists):
 *   decode_fork (-1 | 0 | 1), split_walk (0..3), split_class, exec_keep
 *   (bytes of history at a window slide, 512..2000, multiple of 16),
 *   chunked_huge, small_persist, small_batch, split_huge, walk_order,
 *   lean_walk, exec_big_blocks, exec_prio, exec_big_blocks_fork, exec_pack,
 *   encode_wave_min, encode_wave_share, encode_wave_all_mb,
 *   encode_lanes, encode_wave_per_cu, encode_wave_wg, lz4_big_min.
 * Every value produces the same bytes and statuses.  Set between batches, not
 * while other threads launch.  FSG_ERR_INVALID_ARG for an unknown name.
 * fsg_default_option returns the built-in default (before the environment). */
int fsg_set_option(const char *name, int64_t value);
int fsg_get_option(const char *name, int64_t *value);
int fsg_default_option(const char *name, int64_t *value);

/* 32 + n + n/6 (snappy.cc:55-77). */
size_t fsg_max_compressed_length(size_t n);

/* Gather: copies n byte ranges (d_src[i], d_len[i]) to d_dst + d_dst_off[i]
 * on the device.  The sources may be pinned HOST memory (hipHostMalloc'd,
 * device-mapped): the kernel reads them over PCIe, which is how the host
 * runtime moves cord_buf blocks from the pinned blockmem_allocate hook
 * (flare/io/cord_buf.cc:159-166) into a packed batch without a staging
 * memcpy (the reference walks backing blocks, cord_buf.cc:1469-1475).
 * d_src / d_len / d_dst_off are device arrays. */
int fsg_gather_blocks(const uint64_t *d_src, const uint32_t *d_len, const uint64_t *d_dst_off,
                      uint32_t n, uint8_t *d_dst, void *stream);

/* Host-side header parse.  lenient != 0: ReadUncompressedLength rules
 * (5th byte's high bits dropped); lenient == 0: Parse32WithLimit rules.
 * Returns the header byte count (1..5), or 0 if the header is invalid. */
int fsg_get_uncompressed_length(const void *compressed, size_t n,
                                uint32_t *ulen, int lenient);

/* Device header pass: for each message writes its (lenient or strict)
 * uncompressed length into d_ulen (0xFFFFFFFF if the header is invalid).
 * Lets a caller size output slots without a host round trip per message. */
int fsg_uncompressed_lengths_batch(const uint8_t *d_in, const uint64_t *d_in_off,
                                   const uint32_t *d_in_len, uint32_t n_msgs,
                                   uint32_t *d_ulen, int lenient, void *stream);

/* Device workspace for fsg_compress_batch: per-lane hash tables (one
 * htsize-entry table per concurrently encoding lane, htsize per
 * WorkingMemory::GetHashTable, snappy.cc:247-271; 4-byte entries, a position
 * and its fingerprint, so twice the reference's u16 table: up to 16 GiB at
 * the 262,144-lane cap with 64 KiB fragments) plus a work counter.
 * max_in_len bounds every message length of the batch (0 = any).  Passing a
 * smaller or NULL workspace selects the LDS-table wave-per-message encoder. */
size_t fsg_compress_workspace_bytes(uint32_t n_msgs, uint32_t max_in_len);
/* Device workspace for fsg_decompress_batch.  total_in_bytes = the size of
 * the packed input (an upper bound of the sum of d_in_len): the two-pass
 * decoder keeps a tag-start bitmap of 1 bit per input byte there.  With
 * total_in_bytes = 0 (or a NULL / smaller workspace) the single-pass decoder
 * runs; a workspace sized for less input than the batch holds still decodes
 * every message correctly (the overflow falls back to the single-pass
 * kernel).  The workspace is scratch: its content between calls is
 * irrelevant. */
size_t fsg_decompress_workspace_bytes(uint32_t n_msgs, uint64_t total_in_bytes);

/* Batched compress.  Message i is d_in[d_in_off[i] .. +d_in_len[i]); its
 * compressed stream (varint header + 64 KiB fragments, byte-identical to
 * snappy::Compress) is written to d_out[d_out_off[i] ..]; each slot must
 * hold fsg_max_compressed_length(d_in_len[i]) bytes and slots must not
 * overlap.  d_out_len[i] receives the compressed length, d_status[i] FSG_OK.
 * max_in_len: an upper bound of every d_in_len[i] (sizes the LDS hash
 * table; pass 0 for "up to 64 KiB-fragment tables"). */
int fsg_compress_batch(const uint8_t *d_in, const uint64_t *d_in_off,
                       const uint32_t *d_in_len, uint32_t n_msgs,
                       uint32_t max_in_len, uint8_t *d_out,
                       const uint64_t *d_out_off, uint32_t *d_out_len,
                       int32_t *d_status, void *d_workspace,
                       size_t workspace_bytes, void *stream);

/* Batched decompress.  Message i's compressed bytes are
 * d_in[d_in_off[i] .. +d_in_len[i]); output goes to d_out[d_out_off[i] ..]
 * with capacity d_out_cap[i] (slots must not overlap).  d_out_len[i]
 * receives the header's uncompressed length, d_status[i] a FSG_* status.
 * flags: FSG_FLAG_VALIDATE_ONLY (d_out may be NULL), FSG_FLAG_STRICT_HEADER. */
int fsg_decompress_batch(const uint8_t *d_in, const uint64_t *d_in_off,
                         const uint32_t *d_in_len, uint32_t n_msgs,
                         uint8_t *d_out, const uint64_t *d_out_off,
                         const uint32_t *d_out_cap, uint32_t *d_out_len,
                         int32_t *d_status, uint32_t flags, void *d_workspace,
                         size_t workspace_bytes, void *stream);

/* fsg_decompress_batch with its two passes on two streams: pass 1 (header
 * checks, the tag walk, the tag-start bitmap) runs on `pass1_stream`, pass 2
 * (execution) on `stream` after pass 1 (an event).  Same bytes and statuses.
 * A caller decoding a stream of batches alternates two sets of
 * workspace / output / d_out_len / d_status buffers, so batch k+1's pass 1
 * runs beside batch k's pass 2 (the tag walk is latency-bound, the execution
 * issue-bound).  The inputs must be ready on `pass1_stream`; calls that share
 * any of those buffers must be ordered by the caller (pass 1 writes the
 * workspace, d_out_len, d_status and, for messages cut into 64 KiB segments,
 * 4 bytes of d_out).  Results are valid once `stream` is synchronised.
 * Meant for uniform batches: this form never forks the large-message passes
 * onto the side streams (fsg_decompress_batch does for batches of more than
 * 128K messages), so a mixed batch with very large bodies (CM-like) runs its
 * large-message walk before the execution pass and is faster through
 * fsg_decompress_batch.  When the library cannot create its per-device
 * events, `stream` waits on `pass1_stream` and every pass runs on `stream`. */
int fsg_decompress_batch_2s(const uint8_t *d_in, const uint64_t *d_in_off,
                            const uint32_t *d_in_len, uint32_t n_msgs,
                            uint8_t *d_out, const uint64_t *d_out_off,
                            const uint32_t *d_out_cap, uint32_t *d_out_len,
                            int32_t *d_status, uint32_t flags, void *d_workspace,
                            size_t workspace_bytes, void *stream, void *pass1_stream);

/* Batched UncompressAsMuchAsPossible (snappy.cc:1530-1535) over each
 * message's stream cut into `frag`-byte source pieces, as Source::Peek hands
 * them out (0 = one piece, a ByteArraySource; flare's cord_buf blocks carry
 * 8160 bytes).  d_out slots as for fsg_decompress_batch, sized for the
 * header's length.  Per message: d_produced[i] = the reference's return value
 * (SnappyScatteredWriter::Produced(), which counts the 64 KiB block a failing
 * SlowAppend just filled twice); d_got[i] = the bytes its sink receives, which
 * are d_out[d_out_off[i] .. + d_got[i]), byte-identical to the reference's.
 * d_status[i]: FSG_OK (the whole stream decoded), FSG_CORRUPT (it stopped
 * early), FSG_BAD_HEADER (produced 0), or FSG_SLOT_TOO_SMALL (the reference
 * would write past the slot; d_got / d_produced 0).  Workspace as for
 * fsg_decompress_batch.  Streams the batch decoder accepts cost what a
 * decompress costs; the others are walked serially, one lane each: a
 * rejected message of L output bytes costs O(L / 16) serial 16-byte steps
 * (literals, copies reaching 16+ bytes back) up to O(L) byte steps (short-
 * offset copies, block edges) -- a 64 KiB body ~0.2-3 ms on its lane. */
int fsg_decompress_batch_partial(const uint8_t *d_in, const uint64_t *d_in_off,
                                 const uint32_t *d_in_len, uint32_t n_msgs, uint32_t frag,
                                 uint8_t *d_out, const uint64_t *d_out_off,
                                 const uint32_t *d_out_cap, uint32_t *d_got,
                                 uint64_t *d_produced, int32_t *d_status, void *d_workspace,
                                 size_t workspace_bytes, void *stream);

/* Batched RawUncompressToIOVec (snappy.cc:1122-1132).  Message i's iovecs
 * are entries [d_iov_first[i], d_iov_first[i + 1]) of d_iov_base (device
 * addresses) / d_iov_len; d_iov_first has n_msgs + 1 entries.  The stream is
 * decoded into the caller's staging slot (d_stage / d_stage_off / d_stage_cap,
 * sized for the header's length, as fsg_decompress_batch's output) and then
 * copied into the iovecs in order, filling each before the next, as
 * SnappyIOVecWriter does.  d_out_len[i] = the header's length.  d_status[i]:
 * FSG_OK (the reference's true; the iovecs hold its bytes, bytes past the
 * length untouched), FSG_CORRUPT / FSG_BAD_HEADER / FSG_IOV_TOO_SMALL (its
 * false; the iovecs hold what the reference leaves in place: the output's
 * prefix filling every iovec for FSG_IOV_TOO_SMALL, the decoded prefix, a
 * literal cut by the end of input and the last fast append's 16-byte spill
 * for FSG_CORRUPT -- a rejected stream is re-walked serially by one lane,
 * O(output bytes); nothing for FSG_BAD_HEADER), or FSG_SLOT_TOO_SMALL
 * (staging sizing error; the iovecs are untouched). */
int fsg_decompress_batch_iovec(const uint8_t *d_in, const uint64_t *d_in_off,
                               const uint32_t *d_in_len, uint32_t n_msgs,
                               const uint64_t *d_iov_base, const uint64_t *d_iov_len,
                               const uint32_t *d_iov_first, uint8_t *d_stage,
                               const uint64_t *d_stage_off, const uint32_t *d_stage_cap,
                               uint32_t *d_out_len, int32_t *d_status, void *d_workspace,
                               size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FLARE_SNAPPY_GPU_H_ */
