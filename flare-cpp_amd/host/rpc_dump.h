// rpc_dump.h -- the rpc_dump capture format: sampled
// requests written to files as baidu_std-style frames
//   "PRPC" | body_size (BE32) | meta_size (BE32) | RpcDumpMeta | request
// where `request` is the request payload exactly as received (still
// compressed per RpcDumpMeta.compress_type, attachment at its tail).
// Follows /root/reference/flare/rpc/rpc_dump.h:47-95 and rpc_dump.cc:
//   file layout :41-45, flags :47-58, RpcDumpContext::Dump :149-228,
//   Serialize :230-251, SampleIterator::Next :264-317, Pop :319-357.
// Sampling (CollectorSpeedLimit) and gflags reloading are not restated: the
// writer dumps every sample it is given.
//
// ReplayAsBaiduStd and DecompressSamples are what rpc_replay does with a dump
// (/root/reference/tools/rpc_replay/rpc_replay.cc:142-169): rebuild request
// frames from samples, or -- the GPU path -- decompress every sampled SNAPPY
// request of a dump in one device batch.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "baidu_rpc_meta.h"
#include "cord_buf.h"

namespace flare::rpc {

struct SampledRequest {
  cord_buf request;
  RpcDumpMeta meta;
};

// rpc_dump.cc:230-251 -- appends one frame to `buf`.
bool SerializeSample(cord_buf* buf, const SampledRequest& sample);

// Writes samples under `dir` as <dir>/requests.yyyymmdd_hhmmss_uuuuuu files
// of at most `max_requests_in_one_file` samples, keeping at most `max_files`
// files (oldest removed first).  Buffered data is written when a file fills,
// when 1 MiB is pending, when 2 s passed since the last write, or on Flush().
class RpcDumpWriter {
 public:
  explicit RpcDumpWriter(std::string dir, int max_requests_in_one_file = 1000,
                         int max_files = 32);
  ~RpcDumpWriter();
  bool Dump(const SampledRequest& sample);
  bool Flush();
  const std::vector<std::string>& files() const { return filenames_; }

 private:
  bool Write();
  std::string dir_;
  int max_requests_in_one_file_;
  int max_files_;
  int cur_req_count_ = 0;
  int cur_fd_ = -1;
  int64_t sched_write_time_us_;
  int64_t last_file_time_us_ = 0;
  std::vector<std::string> filenames_;
  cord_buf unwritten_;
};

// Iterates the samples of every regular file under `dir` (file names in
// sorted order -- the timestamped names sort chronologically; the reference
// uses directory order).  A file whose content is malformed is abandoned at
// the first bad frame and iteration moves on to the next file.
class SampleIterator {
 public:
  explicit SampleIterator(const std::string& dir);
  ~SampleIterator();
  // nullptr at the end.
  std::unique_ptr<SampledRequest> Next();
  // Parse one sample from the front of `buf`.  nullptr with
  // *format_error == false: not enough data yet.
  static std::unique_ptr<SampledRequest> Pop(cord_buf& buf, bool* format_error);

 private:
  std::vector<std::string> files_;
  size_t next_file_ = 0;
  int cur_fd_ = -1;
  cord_buf cur_buf_;
};

// rpc_replay.cc:162-169 + PackRpcRequest's replay branch
// (baidu_rpc_protocol.cc:643-647): the baidu_std request frame that replays
// `sample` (service/method/compress type from the dump meta, attachment split
// by attachment_size).
void ReplayAsBaiduStd(const SampledRequest& sample, uint64_t correlation_id, cord_buf* frame);

// Decompress the message part (request minus attachment) of every sample:
// SNAPPY ones in one device batch, NONE ones copied.  ok[i] false on a
// corrupt body, attachment_size larger than the request, or another codec.
size_t DecompressSamples(const std::vector<const SampledRequest*>& samples,
                         std::vector<cord_buf>* bodies, std::vector<bool>* ok);

}  // namespace flare::rpc
