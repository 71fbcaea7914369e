// gpu_codec.h -- process-wide GPU Snappy runtime behind the snappy
// CompressHandler.
//
// The reference's handlers are plain function pointers with no context,
// called concurrently from fibers and user threads
// (/root/reference/flare/rpc/compress.h:28-39; callers in SURVEY.md §8(b)),
// so GPU state is a process singleton.  Concurrent single-message calls are
// coalesced into one device batch: the first caller to find no batch in flight
// becomes the leader, takes every queued request, and runs
//   gather (cord_buf backing blocks -> pinned staging) -> hipMemcpyAsync H2D
//   -> fsg_{compress,decompress}_batch -> D2H -> scatter (append to cord_buf)
// while followers park on a condition variable (the fiber_latch role,
// flare/fiber/fiber_latch.h:10-28) until their result is published.
// There is no CPU fallback: without a usable GPU every call returns false.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "cord_buf.h"

namespace flare::gpu {

struct CodecStats {
  uint64_t batches = 0;
  uint64_t messages = 0;
  uint64_t bytes_in = 0;
  uint64_t bytes_out = 0;
  uint64_t max_batch = 0;
  uint64_t failures = 0;
};

class SnappyGpuCodec {
 public:
  // The process singleton (device from FLARE_SNAPPY_GPU_DEVICE, default 0).
  static SnappyGpuCodec& Instance();

  bool available() const { return ok_; }
  const std::string& error() const { return err_; }

  // Single-message entry points (batched across concurrent callers).
  // Output is APPENDED to *out, like the reference's Sink.  Return the
  // reference's verdict (compress always succeeds when the GPU works).
  bool Compress(const cord_buf& in, cord_buf* out);
  bool Uncompress(const cord_buf& in, cord_buf* out);

  // Explicit batch entry points (one device batch, caller's order).
  // ok[i] receives each message's verdict.
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
  bool ok_ = false;
  std::string err_;
};

}  // namespace flare::gpu
