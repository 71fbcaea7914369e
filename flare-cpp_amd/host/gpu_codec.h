// gpu_codec.h -- the process-wide Snappy runtime behind the snappy
// CompressHandler.
//
// The reference's handlers are plain function pointers with no context,
// called concurrently from fibers and user threads
// (/root/reference/flare/rpc/compress.h:28-39; callers in SURVEY.md §8(b)),
// so the runtime is a process singleton.  Per call it picks:
//   * the host codec (host/snappy_cpu.h) for bodies below a size threshold
//     (one small body cannot amortise a device round trip), on nodes with no
//     usable GPU, and for every message of a device batch that hit a HIP
//     error -- so, like the reference, compression never fails;
//   * otherwise a device batch: concurrent single-message calls are
//     coalesced.  The first caller to find a device idle becomes that
//     device's leader and runs every queued request as one batch
//       gather (cord_buf blocks -> device; pinned blocks are read by the GPU
//       itself, others staged through pinned memory) -> H2D ->
//       fsg_{compress,decompress}_batch -> D2H into a pinned output slab ->
//       scatter (outputs adopted zero-copy with append_user_data, small ones
//       copied)
//     and keeps leading while requests keep arriving; followers park on a
//     latch (park hooks: a flare::fiber_latch, flare/fiber/fiber_latch.h:
//     10-28, when the host framework installs one; a condition variable by
//     default).  Devices come from a mask (InitDevices / FLARE_SNAPPY_GPU_DEVICES).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "cord_buf.h"

namespace flare::gpu {

struct CodecStats {
  uint64_t batches = 0;       // device batches run
  uint64_t messages = 0;      // messages coded on a GPU
  uint64_t bytes_in = 0;      // input bytes of those
  uint64_t bytes_out = 0;     // output bytes of those
  uint64_t max_batch = 0;     // largest device batch
  uint64_t failures = 0;      // corrupt-input verdicts (the reference's false)
  uint64_t cpu_messages = 0;  // messages coded on the host
  uint64_t fallbacks = 0;     // messages moved to the host after a device error
  uint64_t adopted = 0;       // outputs adopted zero-copy from pinned slabs
};

// Park hooks (see fsh_park_hooks in include/flare_snappy_host.h).
struct ParkHooks {
  void* (*create)() = nullptr;
  void (*wait)(void*) = nullptr;
  void (*signal)(void*) = nullptr;
  void (*destroy)(void*) = nullptr;
};

class SnappyGpuCodec {
 public:
  // The process singleton.  Devices start lazily on first use (mask from
  // FLARE_SNAPPY_GPU_DEVICES: a bit mask like 0xff or a list like "0,1";
  // default device 0, or FLARE_SNAPPY_GPU_DEVICE).
  static SnappyGpuCodec& Instance();

  // Starts the devices in `mask` (0: the environment's choice) after
  // draining and releasing the current ones.  Returns the devices started.
  int InitDevices(uint64_t mask);
  // Drains and releases every device; calls then run on the host codec.
  void Shutdown();

  bool available();                 // at least one device started
  std::string error();              // why none did
  int device_count();

  // Bodies below `bytes` are coded on the host (default 16384,
  // FLARE_SNAPPY_GPU_MIN_BYTES; 0 = every body to the GPU).
  void SetMinGpuBytes(size_t bytes);
  size_t min_gpu_bytes() const;
  void SetParkHooks(const ParkHooks& hooks);

  // Single-message entry points.  Output is APPENDED to *out, like the
  // reference's Sink.  Return the reference's verdict; Compress always
  // succeeds.
  bool Compress(const cord_buf& in, cord_buf* out);
  bool Uncompress(const cord_buf& in, cord_buf* out);
  // IsValidCompressedBuffer (snappy.cc:1290-1294): the device's validate-only
  // pass, no output.
  bool IsValid(const cord_buf& in);

  // Explicit batch entry points: one device batch per device (the batch is
  // split by bytes across devices), caller's order; ok[i] = each verdict.
  bool CompressBatch(const std::vector<const cord_buf*>& in, const std::vector<cord_buf*>& out,
                     std::vector<bool>* ok);
  bool UncompressBatch(const std::vector<const cord_buf*>& in, const std::vector<cord_buf*>& out,
                       std::vector<bool>* ok);

  CodecStats stats() const;

  SnappyGpuCodec(const SnappyGpuCodec&) = delete;
  SnappyGpuCodec& operator=(const SnappyGpuCodec&) = delete;

  struct Impl;  // opaque runtime state (gpu_codec.cc)

 private:
  SnappyGpuCodec();
  ~SnappyGpuCodec();
  Impl* impl_;
};

// Host codec over cord_bufs (the runtime's fallback; also used directly by
// the flat API for small inputs).  Same verdicts as the reference.
bool CpuCompress(const cord_buf& in, cord_buf* out);
bool CpuUncompress(const cord_buf& in, cord_buf* out);

// Test hook: the next n device batches fail as a HIP error would (their
// messages then run on the host codec).
void InjectDeviceErrorsForTesting(int n);

// Pinned host memory (pinned.cc).
// Installs the pinned block allocator as cord_buf's blockmem hooks
// (cord_buf.cc:159-166).  0 on success.
int UsePinnedBlocks();
// True if [p, p + n) lies in one pinned allocation of this runtime.
bool IsPinned(const void* p, size_t n);

}  // namespace flare::gpu
