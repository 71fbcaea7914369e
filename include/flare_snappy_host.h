/* flare_snappy_host.h -- C ABI of the host side of the drop-in
 * (libflare_rpc_snappy.so): the CompressHandler runtime's policy and device
 * controls, the flat Snappy API as the handler runs it, and the host codec
 * the handler falls back to.  Plain pointers and sizes; every function is
 * thread-safe.  Bytes and verdicts are the reference's
 * (/root/reference/flare/io/snappy/snappy.cc, vendored Snappy 1.1.3).
 *
 * The device batch ABI itself is include/flare_snappy_gpu.h. */
#ifndef FLARE_SNAPPY_HOST_H_
#define FLARE_SNAPPY_HOST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- runtime control (init / teardown with a device mask) */

/* Starts the GPU runtime on the devices in `device_mask` (bit d = HIP device
 * d; 0 = FLARE_SNAPPY_GPU_DEVICES or device 0).  Concurrent handler calls are
 * spread over the devices.  Returns the number of devices started (0: none
 * usable -- every call then runs on the host codec).  Idempotent per mask;
 * called implicitly by the first handler call. */
int fsh_init_devices(uint64_t device_mask);

/* Drains in-flight batches and releases every device resource.  Later
 * handler calls run on the host codec until fsh_init_devices runs again. */
void fsh_shutdown(void);

/* Bodies below `bytes` (default 16384, FLARE_SNAPPY_GPU_MIN_BYTES) are coded
 * on the host: one small body cannot amortise a device round trip.  0 sends
 * every body to the GPU (the GPU tests do this). */
void fsh_set_gpu_min_bytes(size_t bytes);

/* Counters since start: [0] device batches, [1] messages coded on the GPU,
 * [2] messages coded on the host, [3] messages moved to the host after a
 * device error, [4] corrupt-input verdicts, [5] outputs adopted zero-copy.
 * Writes min(n, 6) values. */
void fsh_stats(uint64_t* out, size_t n);

/* Park hooks for followers waiting on a coalesced device batch (the
 * flare::fiber_latch role, /root/reference/flare/fiber/fiber_latch.h:10-28).
 * create() returns a latch, wait() parks until signal(), destroy() frees it.
 * All four null restores the default (a condition variable). */
typedef struct fsh_park_hooks {
  void* (*create)(void);
  void (*wait)(void* latch);
  void (*signal)(void* latch);
  void (*destroy)(void* latch);
} fsh_park_hooks;
void fsh_set_park_hooks(const fsh_park_hooks* hooks);

/* Installs the pinned block allocator as cord_buf's blockmem_allocate /
 * blockmem_deallocate (/root/reference/flare/io/cord_buf.cc:159-166), so
 * handler inputs reach the device without a staging copy.  Returns 0 on
 * success. */
int fsh_use_pinned_blocks(void);

/* ---- flat API through the handler runtime (snappy.h:62-190) */

/* snappy.cc:1313-1322; never fails.  `out` holds fsh_max_compressed_length(n). */
size_t fsh_compress(const char* in, size_t n, char* out);
/* snappy.cc:1229-1237 (lenient header); `out` holds the header length. */
int fsh_raw_uncompress(const char* in, size_t n, char* out);
/* snappy.cc:235-244 (strict header). */
int fsh_get_uncompressed_length(const char* in, size_t n, size_t* result);
/* snappy.cc:1290-1294. */
int fsh_is_valid_compressed_buffer(const char* in, size_t n);
/* snappy.cc:55-77. */
size_t fsh_max_compressed_length(size_t n);

/* ---- the host codec (host/snappy_cpu.h), for bindings and tests */
size_t fsh_cpu_compress(const uint8_t* in, size_t n, uint8_t* out);
int fsh_cpu_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int strict);
int fsh_cpu_is_valid(const uint8_t* in, size_t n);
/* UncompressAsMuchAsPossible (snappy.cc:1530-1535) over `in` cut into
 * `frag`-byte fragments (0 = one fragment): returns the reference's result;
 * *got = bytes written to out (<= cap). */
size_t fsh_cpu_uncompress_as_much(const uint8_t* in, size_t n, size_t frag, uint8_t* out,
                                  size_t cap, size_t* got);

/* ---- LZ4 (host/lz4_cpu.h; COMPRESS_TYPE_LZ4, options.proto:74, has no
 * reference handler): body = varint32 length + one LZ4 block. */
/* body bound: 5 + LZ4_compressBound(n) */
size_t fsh_lz4_max_compressed_length(size_t n);
/* body of n bytes into out; its length (0 above 0x7E000000 bytes) */
size_t fsh_cpu_lz4_compress(const uint8_t* in, size_t n, uint8_t* out);
/* body to out (cap bytes): 1 ok, 0 corrupt, -1 bad header, -2 above cap;
 * *ulen = the header's length when it parses */
int fsh_cpu_lz4_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, uint32_t* ulen);
/* registers the LZ4 CompressHandler (host/lz4_compress.h); 0 on success */
int fsh_register_lz4(void);

#ifdef __cplusplus
}
#endif

#endif /* FLARE_SNAPPY_HOST_H_ */
