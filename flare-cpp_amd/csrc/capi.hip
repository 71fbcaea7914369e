// capi.hip -- extern "C" boundary of libflare_snappy_gpu.so.
// Declarations and the reference interface each call replaces:
// include/flare_snappy_gpu.h.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/flare_lz4_gpu.h"
#include "../../include/flare_snappy_gpu.h"
#include "options.h"
#include "snappy_device.h"

namespace fsg {
hipError_t launch_decode(const u8* in, const u64* in_off, const u32* in_len,
                         u32 n_msgs, u8* out, const u64* out_off,
                         const u32* out_cap, u32* out_len, i32* status,
                         u32 flags, hipStream_t stream);
hipError_t launch_decode_v3(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, hipStream_t stream);
size_t decode_v4_workspace_bytes(u32 n_msgs, u64 total_in_bytes);
hipError_t launch_decode_v4(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u8* out, const u64* out_off,
                            const u32* out_cap, u32* out_len, i32* status,
                            u32 flags, void* ws, size_t ws_bytes, hipStream_t stream,
                            int exec_variant, hipStream_t pass1_stream);
hipError_t launch_headers(const u8* in, const u64* in_off, const u32* in_len,
                          u32 n_msgs, u32* ulen, int lenient, hipStream_t stream);
size_t encode_tables_workspace_bytes(u32 n_msgs, u32 max_in_len, u32* slots_out);
size_t encode_plan_bytes(u32 n_msgs, u32 max_in_len);
hipError_t launch_encode_v3(const u8* in, const u64* in_off, const u32* in_len,
                            u32 n_msgs, u32 max_in_len, u8* out, const u64* out_off,
                            u32* out_len, i32* status, void* ws, size_t ws_bytes,
                            u32 slots, u32 entries, size_t tables_bytes, u32 region_cap,
                            hipStream_t stream, u32 wave_min);
hipError_t launch_encode(const u8* in, const u64* in_off, const u32* in_len,
                         u32 n_msgs, u32 max_in_len, u8* out, const u64* out_off,
                         u32* out_len, i32* status, hipStream_t stream);
hipError_t launch_gather_blocks(const u64* src, const u32* len, const u64* dst_off, u32 n, u8* dst,
                                hipStream_t stream);
hipError_t launch_decode_partial(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u32 frag,
                                 u8* out, const u64* out_off, const u32* out_cap, u32* got, u64* produced,
                                 i32* status, hipStream_t stream);
hipError_t launch_iov_scatter(const u8* in, const u64* in_off, const u32* in_len, const u8* stage,
                              const u64* stage_off, const u32* out_len, u32 n_msgs, const u64* iov_base,
                              const u64* iov_len, const u32* iov_first, i32* status, hipStream_t stream);
size_t lz4_compress_workspace_bytes(u32 n_msgs);
hipError_t launch_lz4_encode(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                             const u64* out_off, u32* out_len, i32* status, void* ws, hipStream_t stream);
hipError_t launch_lz4_decode(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                             const u64* out_off, const u32* out_cap, u32* out_len, i32* status,
                             hipStream_t stream);
size_t lz4_decode_workspace_bytes(u32 n_msgs, u64 total_in_bytes);
hipError_t launch_lz4_decode2(const u8* in, const u64* in_off, const u32* in_len, u32 n_msgs, u8* out,
                              const u64* out_off, const u32* out_cap, u32* out_len, i32* status, void* ws,
                              size_t ws_bytes, hipStream_t stream, hipStream_t pass1_stream);
}  // namespace fsg

namespace {
thread_local char g_err[256] = "";

int env_int(const char* name) {
  const char* e = getenv(name);
  return e ? atoi(e) : 0;
}

// ---- the option table (csrc/options.h): name, environment variable, default
struct OptDesc {
  const char* name;
  const char* env;
  int64_t dflt;
};
constexpr OptDesc kOptDesc[fsg::kOptCount] = {
    {"decode_fork", "FSG_DECODE_FORK", -1},
    {"split_walk", "FSG_SPLIT_WALK", 3},
    {"split_class", "FSG_SPLIT_CLASS", 4},
    {"exec_keep", "FSG_EXEC_KEEP", -1},
    {"chunked_huge", "FSG_CHUNKED_HUGE", 1},
    {"small_persist", "FSG_SMALL_PERSIST", 3584},
    {"small_batch", "FSG_SMALL_BATCH", 64},
    {"split_huge", "FSG_SPLIT_HUGE", 1},
    {"walk_order", "FSG_WALK_ORDER", 1},
    {"lean_walk", "FSG_LEAN_WALK", 1},
    {"exec_big_blocks", "FSG_EXEC_BIG_BLOCKS", 512},
    {"exec_prio", "FSG_EXEC_PRIO", 1},
    {"exec_big_blocks_fork", "FSG_EXEC_BIG_BLOCKS_FORK", 1024},
    {"exec_pack", "FSG_EXEC_PACK", 32},
    {"encode_wave_min", "FSG_ENCODE_WAVE_MIN", 16384},
    {"encode_wave_share", "FSG_ENCODE_WAVE_SHARE", 475},
    {"encode_wave_all_mb", "FSG_ENCODE_WAVE_ALL_MB", 640},
    {"encode_lanes", "FSG_ENCODE_LANES", 0},
    {"encode_wave_per_cu", "FSG_ENCODE_WAVE_PER_CU", 0},
    {"encode_wave_wg", "FSG_ENCODE_WAVE_WG", 1},
    {"lz4_big_min", "FSG_L4_BIG_MIN", -1},
};
std::atomic<int64_t> g_opt[fsg::kOptCount];
// the environment, once, when the library is loaded
[[maybe_unused]] const bool g_opt_init = [] {
  for (int i = 0; i < fsg::kOptCount; ++i) {
    const char* e = getenv(kOptDesc[i].env);
    g_opt[i].store(e && *e ? strtoll(e, nullptr, 10) : kOptDesc[i].dflt);
  }
  return true;
}();
int find_opt(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < fsg::kOptCount; ++i)
    if (strcmp(name, kOptDesc[i].name) == 0) return i;
  return -1;
}
// Kernel variants (0 = automatic).  Initialised from FSG_DECODE_KERNEL /
// FSG_ENCODE_KERNEL, changeable with fsg_select_kernels for A/B runs.
std::atomic<int> g_decode_variant{env_int("FSG_DECODE_KERNEL")};
std::atomic<int> g_encode_variant{env_int("FSG_ENCODE_KERNEL")};
// Messages of at least this many bytes (and every fragment of a message over
// 64 KiB) form the long list, whose units the wave encoder (hash table in
// LDS, one wave per fragment) and the lane encoder share (wave_quota); the
// shorter messages go to the lane encoder.  Option encode_wave_min
// (FSG_ENCODE_WAVE_MIN; 0 = lane encoder only).  Measured on MI355X (A/B, one box): C3
// compress 108.0 -> 98.4 ms, C5 54.9 -> 39.1 ms.
fsg::u32 encode_wave_min() {
  const int64_t v = fsg::opt(fsg::kOptEncodeWaveMin);
  return v >= 0 ? (fsg::u32)v : 16384u;
}
// Test knob: cap the staging region of a split message's fragments (bytes;
// 0 = slot / fragments).  Small caps force the whole-message fallback pass.
std::atomic<unsigned> g_region_cap{(unsigned)env_int("FSG_TEST_REGION_CAP")};

int record(hipError_t e, const char* where) {
  if (e == hipSuccess) return FSG_SUCCESS;
  snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
  return FSG_ERR_HIP;
}
}  // namespace

int64_t fsg::opt(fsg::Opt o) { return g_opt[o].load(std::memory_order_relaxed); }

extern "C" {

int fsg_set_option(const char* name, int64_t value) {
  const int i = find_opt(name);
  if (i < 0) return FSG_ERR_INVALID_ARG;
  g_opt[i].store(value, std::memory_order_relaxed);
  return FSG_SUCCESS;
}

int fsg_get_option(const char* name, int64_t* value) {
  const int i = find_opt(name);
  if (i < 0 || !value) return FSG_ERR_INVALID_ARG;
  *value = g_opt[i].load(std::memory_order_relaxed);
  return FSG_SUCCESS;
}

int fsg_default_option(const char* name, int64_t* value) {
  const int i = find_opt(name);
  if (i < 0 || !value) return FSG_ERR_INVALID_ARG;
  *value = kOptDesc[i].dflt;
  return FSG_SUCCESS;
}

const char* fsg_version(void) { return "flare-snappy-gpu 0.1 gfx950"; }

const char* fsg_last_error(void) { return g_err; }

int fsg_set_split_region_cap(uint32_t bytes) {
  g_region_cap.store(bytes);
  return FSG_SUCCESS;
}

int fsg_select_kernels(int decode_variant, int encode_variant) {
  // generation 2 (persistent-lane decode, literal lane encode) was retired:
  // superseded by 3/4 on every workload
  if (decode_variant < 0 || decode_variant > 5 || decode_variant == 2 || encode_variant < 0 ||
      encode_variant > 3 || encode_variant == 2)
    return FSG_ERR_INVALID_ARG;
  g_decode_variant.store(decode_variant);
  g_encode_variant.store(encode_variant);
  return FSG_SUCCESS;
}

int fsg_init(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    snprintf(g_err, sizeof(g_err), "fsg_init: no HIP device (%s)",
             hipGetErrorString(e));
    return FSG_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= n) return FSG_ERR_INVALID_ARG;
  return record(hipSetDevice(device), "hipSetDevice");
}

size_t fsg_max_compressed_length(size_t n) { return 32 + n + n / 6; }

int fsg_gather_blocks(const uint64_t* d_src, const uint32_t* d_len, const uint64_t* d_dst_off,
                      uint32_t n, uint8_t* d_dst, void* stream) {
  if (n && (!d_src || !d_len || !d_dst_off || !d_dst)) return FSG_ERR_INVALID_ARG;
  return record(fsg::launch_gather_blocks(d_src, d_len, d_dst_off, n, d_dst, (hipStream_t)stream),
                "fsg_gather_blocks");
}

int fsg_get_uncompressed_length(const void* compressed, size_t n,
                                uint32_t* ulen, int lenient) {
  const uint8_t* p = static_cast<const uint8_t*>(compressed);
  uint32_t r = 0;
  for (int i = 0; i < 5; ++i) {
    if ((size_t)i >= n) return 0;
    uint32_t c = p[i];
    r |= (c & 0x7fu) << (7 * i);
    if (c < 128) {
      if (!lenient && i == 4 && c >= 16) return 0;  // Parse32WithLimit
      *ulen = r;
      return i + 1;
    }
  }
  return 0;
}

int fsg_uncompressed_lengths_batch(const uint8_t* d_in, const uint64_t* d_in_off,
                                   const uint32_t* d_in_len, uint32_t n_msgs,
                                   uint32_t* d_ulen, int lenient, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_ulen))
    return FSG_ERR_INVALID_ARG;
  return record(fsg::launch_headers(d_in, d_in_off, d_in_len, n_msgs, d_ulen,
                                    lenient, (hipStream_t)stream),
                "fsg_uncompressed_lengths_batch");
}

size_t fsg_compress_workspace_bytes(uint32_t n_msgs, uint32_t max_in_len) {
  // per-lane hash tables, then the fragment plan for messages > 64 KiB
  return fsg::encode_tables_workspace_bytes(n_msgs, max_in_len, nullptr) +
         fsg::encode_plan_bytes(n_msgs, max_in_len);
}
size_t fsg_decompress_workspace_bytes(uint32_t n_msgs, uint64_t total_in_bytes) {
  // total_in_bytes = 0: no size known, only the single-pass decoders run.
  return total_in_bytes ? fsg::decode_v4_workspace_bytes(n_msgs, total_in_bytes) : 256;
}

int fsg_compress_batch(const uint8_t* d_in, const uint64_t* d_in_off,
                       const uint32_t* d_in_len, uint32_t n_msgs,
                       uint32_t max_in_len, uint8_t* d_out,
                       const uint64_t* d_out_off, uint32_t* d_out_len,
                       int32_t* d_status, void* d_workspace,
                       size_t workspace_bytes, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off ||
                 !d_out_len || !d_status))
    return FSG_ERR_INVALID_ARG;
  // The lane-per-message encoder with global-memory tables when the
  // workspace allows it (v3: batched speculative probes, the default);
  // otherwise the wave-per-message LDS-table encoder (v1).
  const int forced = g_encode_variant.load(std::memory_order_relaxed);
  fsg::u32 slots = 0;
  const size_t need = fsg::encode_tables_workspace_bytes(n_msgs, max_in_len, &slots);
  if ((forced == 0 || forced == 3) && d_workspace && workspace_bytes >= need) {
    const fsg::u32 cap = max_in_len == 0 || max_in_len > fsg::kBlockSize ? fsg::kBlockSize : max_in_len;
    // Lanes in flight: option encode_lanes caps them; otherwise
    // launch_encode_v3 caps them beside the wave encoder once it knows the
    // wave encoder runs.
    const unsigned lanes_cap = (unsigned)fsg::opt(fsg::kOptEncodeLanes);
    if (lanes_cap && lanes_cap < slots) slots = (lanes_cap + 63) / 64 * 64;
    return record(fsg::launch_encode_v3(d_in, d_in_off, d_in_len, n_msgs, max_in_len, d_out,
                                        d_out_off, d_out_len, d_status, d_workspace,
                                        workspace_bytes, slots, fsg::table_size_for(cap), need,
                                        g_region_cap.load(std::memory_order_relaxed),
                                        (hipStream_t)stream, encode_wave_min()),
                  "fsg_compress_batch");
  }
  return record(fsg::launch_encode(d_in, d_in_off, d_in_len, n_msgs, max_in_len,
                                   d_out, d_out_off, d_out_len, d_status,
                                   (hipStream_t)stream),
                "fsg_compress_batch");
}

namespace {
int decompress_impl(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                    uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                    const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status,
                    uint32_t flags, void* d_workspace, size_t workspace_bytes, void* stream,
                    void* pass1_stream);
}  // namespace

int fsg_decompress_batch(const uint8_t* d_in, const uint64_t* d_in_off,
                         const uint32_t* d_in_len, uint32_t n_msgs,
                         uint8_t* d_out, const uint64_t* d_out_off,
                         const uint32_t* d_out_cap, uint32_t* d_out_len,
                         int32_t* d_status, uint32_t flags, void* d_workspace,
                         size_t workspace_bytes, void* stream) {
  return decompress_impl(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                         d_status, flags, d_workspace, workspace_bytes, stream, nullptr);
}

int fsg_decompress_batch_2s(const uint8_t* d_in, const uint64_t* d_in_off,
                            const uint32_t* d_in_len, uint32_t n_msgs,
                            uint8_t* d_out, const uint64_t* d_out_off,
                            const uint32_t* d_out_cap, uint32_t* d_out_len,
                            int32_t* d_status, uint32_t flags, void* d_workspace,
                            size_t workspace_bytes, void* stream, void* pass1_stream) {
  return decompress_impl(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                         d_status, flags, d_workspace, workspace_bytes, stream, pass1_stream);
}

}  // extern "C"

namespace {
int decompress_impl(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                    uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                    const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status,
                    uint32_t flags, void* d_workspace, size_t workspace_bytes, void* stream,
                    void* pass1_stream) {
  const bool validate = flags & FSG_FLAG_VALIDATE_ONLY;
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out_len || !d_status ||
                 (!validate && (!d_out || !d_out_off || !d_out_cap))))
    return FSG_ERR_INVALID_ARG;
  // Kernel choice: the two-pass decoder (v4: lane-per-message index pass +
  // wave-per-message execution) when the workspace holds its tag bitmap;
  // otherwise the software-pipelined lane-per-message decoder (v3); v1 walks
  // tags without touching output for validate-only.  FSG_DECODE_KERNEL or
  // fsg_select_kernels force a variant (A/B runs).
  const int forced = g_decode_variant.load(std::memory_order_relaxed);
  const bool v4_fits = d_workspace && workspace_bytes >= fsg::decode_v4_workspace_bytes(n_msgs, 0);
  const bool two_pass = !validate && forced != 1 && forced != 3 && v4_fits;
  if (!two_pass && pass1_stream && pass1_stream != stream) {
    // single-pass kernels run on `stream` alone: order it after pass1_stream,
    // where the caller made the inputs ready
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, (hipStream_t)pass1_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)stream, ev, 0);
    if (ev) (void)hipEventDestroy(ev);
    if (e != hipSuccess) return record(e, "fsg_decompress_batch_2s");
  }
  if (validate || forced == 1)
    return record(fsg::launch_decode(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off,
                                     d_out_cap, d_out_len, d_status, flags,
                                     (hipStream_t)stream),
                  "fsg_decompress_batch");
  if (two_pass) {
    // (messages whose bitmap does not fit the workspace are finished by the
    // two-pass launches' serial fallback pass).  Execution pass: one tag per
    // lane (5, the default) or <= 16-byte pieces per lane (4).
    return record(fsg::launch_decode_v4(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off,
                                        d_out_cap, d_out_len, d_status, flags, d_workspace,
                                        workspace_bytes, (hipStream_t)stream, forced == 4 ? 4 : 5,
                                        (hipStream_t)pass1_stream),
                  "fsg_decompress_batch");
  }
  return record(fsg::launch_decode_v3(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off,
                                      d_out_cap, d_out_len, d_status, flags, (hipStream_t)stream),
                "fsg_decompress_batch");
}
}  // namespace

extern "C" {

int fsg_decompress_batch_partial(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                                 uint32_t n_msgs, uint32_t frag, uint8_t* d_out, const uint64_t* d_out_off,
                                 const uint32_t* d_out_cap, uint32_t* d_got, uint64_t* d_produced,
                                 int32_t* d_status, void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_got ||
                 !d_produced || !d_status))
    return FSG_ERR_INVALID_ARG;
  // the batch decoder (lenient header, as the Source path reads it), then the
  // streams it rejected through the scattered-writer model
  const int r = decompress_impl(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_got, d_status,
                                0u, d_workspace, workspace_bytes, stream, nullptr);
  if (r != FSG_SUCCESS) return r;
  return record(fsg::launch_decode_partial(d_in, d_in_off, d_in_len, n_msgs, frag, d_out, d_out_off, d_out_cap,
                                           d_got, d_produced, d_status, (hipStream_t)stream),
                "fsg_decompress_batch_partial");
}

int fsg_decompress_batch_iovec(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                               uint32_t n_msgs, const uint64_t* d_iov_base, const uint64_t* d_iov_len,
                               const uint32_t* d_iov_first, uint8_t* d_stage, const uint64_t* d_stage_off,
                               const uint32_t* d_stage_cap, uint32_t* d_out_len, int32_t* d_status,
                               void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_iov_base || !d_iov_len || !d_iov_first || !d_stage ||
                 !d_stage_off || !d_stage_cap || !d_out_len || !d_status))
    return FSG_ERR_INVALID_ARG;
  const int r = decompress_impl(d_in, d_in_off, d_in_len, n_msgs, d_stage, d_stage_off, d_stage_cap, d_out_len,
                                d_status, 0u, d_workspace, workspace_bytes, stream, nullptr);
  if (r != FSG_SUCCESS) return r;
  return record(fsg::launch_iov_scatter(d_in, d_in_off, d_in_len, d_stage, d_stage_off, d_out_len, n_msgs,
                                        d_iov_base, d_iov_len, d_iov_first, d_status, (hipStream_t)stream),
                "fsg_decompress_batch_iovec");
}

// ---- LZ4 (include/flare_lz4_gpu.h)
size_t fsg_lz4_max_compressed_length(size_t n) { return 5 + n + n / 255 + 16; }

size_t fsg_lz4_compress_workspace_bytes(uint32_t n_msgs) { return fsg::lz4_compress_workspace_bytes(n_msgs); }

int fsg_lz4_compress_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                           uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off, uint32_t* d_out_len,
                           int32_t* d_status, void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len || !d_status ||
                 !d_workspace || workspace_bytes < fsg::lz4_compress_workspace_bytes(n_msgs)))
    return FSG_ERR_INVALID_ARG;
  return record(fsg::launch_lz4_encode(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_len, d_status,
                                       d_workspace, (hipStream_t)stream),
                "fsg_lz4_compress_batch");
}

int fsg_lz4_decompress_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                             uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                             const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status))
    return FSG_ERR_INVALID_ARG;
  return record(fsg::launch_lz4_decode(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                       d_status, (hipStream_t)stream),
                "fsg_lz4_decompress_batch");
}

size_t fsg_lz4_decompress_workspace_bytes(uint32_t n_msgs, uint64_t total_in_bytes) {
  return fsg::lz4_decode_workspace_bytes(n_msgs, total_in_bytes);
}

int fsg_lz4_decompress_batch_ws(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                                uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                                const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status,
                                void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status))
    return FSG_ERR_INVALID_ARG;
  // no usable workspace: the one-pass lane kernel (same results)
  if (!d_workspace || workspace_bytes < fsg::lz4_decode_workspace_bytes(n_msgs, 0))
    return fsg_lz4_decompress_batch(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                    d_status, stream);
  return record(fsg::launch_lz4_decode2(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, d_workspace, workspace_bytes, (hipStream_t)stream, nullptr),
                "fsg_lz4_decompress_batch_ws");
}

int fsg_lz4_decompress_batch_2s(const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                                uint32_t n_msgs, uint8_t* d_out, const uint64_t* d_out_off,
                                const uint32_t* d_out_cap, uint32_t* d_out_len, int32_t* d_status,
                                void* d_workspace, size_t workspace_bytes, void* stream, void* pass1_stream) {
  if (n_msgs && (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status))
    return FSG_ERR_INVALID_ARG;
  if (!d_workspace || workspace_bytes < fsg::lz4_decode_workspace_bytes(n_msgs, 0)) {
    // the one-pass kernel on `stream`, ordered behind pass1_stream's work
    if (pass1_stream && pass1_stream != stream) {
      hipEvent_t ev = nullptr;
      hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventRecord(ev, (hipStream_t)pass1_stream);
      if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)stream, ev, 0);
      if (ev) (void)hipEventDestroy(ev);
      if (e != hipSuccess) return record(e, "fsg_lz4_decompress_batch_2s");
    }
    return fsg_lz4_decompress_batch(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                    d_status, stream);
  }
  return record(fsg::launch_lz4_decode2(d_in, d_in_off, d_in_len, n_msgs, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, d_workspace, workspace_bytes, (hipStream_t)stream,
                                        (hipStream_t)pass1_stream),
                "fsg_lz4_decompress_batch_2s");
}

}  // extern "C"
