// rpc_dump.cc -- see rpc_dump.h.
#include "rpc_dump.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "baidu_rpc_protocol.h"
#include "compress.h"
#include "gpu_codec.h"

namespace flare::rpc {

namespace {
constexpr size_t kUnwrittenBufSize = 1024 * 1024;  // rpc_dump.cc:64
constexpr int64_t kFlushTimeoutUs = 2000000;       // rpc_dump.cc:65
constexpr size_t kReadChunk = 524288;              // rpc_dump.cc:281

int64_t now_us() {
  timeval tv;
  gettimeofday(&tv, nullptr);
  return (int64_t)tv.tv_sec * 1000000 + tv.tv_usec;
}

bool mkdirs(const std::string& dir) {
  if (dir.empty()) return false;
  std::string cur;
  size_t pos = 0;
  while (pos != std::string::npos) {
    pos = dir.find('/', pos + 1);
    cur = dir.substr(0, pos);
    if (cur.empty()) continue;
    if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
  }
  struct stat st;
  return stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

uint32_t get_be32(const char* p) {
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  return ((uint32_t)u[0] << 24) | ((uint32_t)u[1] << 16) | ((uint32_t)u[2] << 8) | u[3];
}
}  // namespace

bool SerializeSample(cord_buf* buf, const SampledRequest& sample) {
  const std::string meta = sample.meta.SerializeAsString();
  char header[12];
  policy::PackRpcHeader(header, (uint32_t)meta.size(), (uint32_t)sample.request.size());
  buf->append(header, sizeof(header));
  buf->append(meta);
  buf->append(sample.request);
  return true;
}

// ------------------------------------------------------------ RpcDumpWriter
RpcDumpWriter::RpcDumpWriter(std::string dir, int max_requests_in_one_file, int max_files)
    : dir_(std::move(dir)),
      max_requests_in_one_file_(max_requests_in_one_file > 0 ? max_requests_in_one_file : 1),
      max_files_(max_files > 0 ? max_files : 1),
      sched_write_time_us_(now_us() + kFlushTimeoutUs) {}

RpcDumpWriter::~RpcDumpWriter() {
  Flush();
  if (cur_fd_ >= 0) close(cur_fd_);
}

bool RpcDumpWriter::Dump(const SampledRequest& sample) {
  if (!SerializeSample(&unwritten_, sample)) return false;
  ++cur_req_count_;
  if (cur_req_count_ >= max_requests_in_one_file_ || unwritten_.size() >= kUnwrittenBufSize ||
      now_us() >= sched_write_time_us_)
    return Write();
  return true;
}

bool RpcDumpWriter::Flush() { return unwritten_.empty() ? true : Write(); }

bool RpcDumpWriter::Write() {
  if (cur_fd_ < 0) {
    if (!mkdirs(dir_)) {
      fprintf(stderr, "[ERROR] Fail to create directory=`%s'\n", dir_.c_str());
      return false;
    }
    while ((int)filenames_.size() >= max_files_ && !filenames_.empty()) {  // :181-184
      unlink(filenames_.front().c_str());
      filenames_.erase(filenames_.begin());
    }
    int64_t t = now_us();
    if (t <= last_file_time_us_) t = last_file_time_us_ + 1;  // monotonic postfix
    const time_t rawtime = (time_t)(t / 1000000);
    struct tm tmv;
    localtime_r(&rawtime, &tmv);
    char ts[64];
    strftime(ts, sizeof(ts), "%Y%m%d_%H%M%S", &tmv);
    char name[96];
    snprintf(name, sizeof(name), "/requests.%s_%06u", ts, (unsigned)(t - (int64_t)rawtime * 1000000));
    const std::string path = dir_ + name;
    cur_fd_ = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0666);
    if (cur_fd_ < 0) {
      fprintf(stderr, "[ERROR] Fail to open %s\n", path.c_str());
      return false;
    }
    last_file_time_us_ = t;
    filenames_.push_back(path);
  }
  bool fail = false;
  for (size_t i = 0; i < unwritten_.backing_block_num() && !fail; ++i) {
    std::string_view b = unwritten_.backing_block(i);
    while (!b.empty()) {
      const ssize_t w = write(cur_fd_, b.data(), b.size());
      if (w < 0) {
        if (errno == EINTR || errno == EAGAIN) continue;
        fail = true;
        break;
      }
      b.remove_prefix((size_t)w);
    }
  }
  unwritten_.clear();
  sched_write_time_us_ = now_us() + kFlushTimeoutUs;
  if (fail || cur_req_count_ >= max_requests_in_one_file_) {
    close(cur_fd_);
    cur_fd_ = -1;
    cur_req_count_ = 0;
  }
  return !fail;
}

// ----------------------------------------------------------- SampleIterator
SampleIterator::SampleIterator(const std::string& dir) {
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      const std::string path = dir + "/" + e->d_name;
      struct stat st;
      if (stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) files_.push_back(path);
    }
    closedir(d);
  }
  std::sort(files_.begin(), files_.end());
}

SampleIterator::~SampleIterator() {
  if (cur_fd_ >= 0) close(cur_fd_);
}

std::unique_ptr<SampledRequest> SampleIterator::Next() {
  for (;;) {
    if (!cur_buf_.empty()) {
      bool error = false;
      std::unique_ptr<SampledRequest> r = Pop(cur_buf_, &error);
      if (r) return r;
      if (error) {  // abandon this file
        cur_buf_.clear();
        if (cur_fd_ >= 0) close(cur_fd_);
        cur_fd_ = -1;
      }
    }
    if (cur_fd_ >= 0) {
      std::string chunk(kReadChunk, '\0');
      const ssize_t nr = read(cur_fd_, &chunk[0], chunk.size());
      if (nr < 0 && (errno == EAGAIN || errno == EINTR)) continue;
      if (nr > 0) {
        cur_buf_.append(chunk.data(), (size_t)nr);
        continue;
      }
      // EOF or error: a partial trailing sample is dropped
      cur_buf_.clear();
      close(cur_fd_);
      cur_fd_ = -1;
    }
    if (next_file_ >= files_.size()) return nullptr;
    cur_fd_ = open(files_[next_file_++].c_str(), O_RDONLY);
  }
}

std::unique_ptr<SampledRequest> SampleIterator::Pop(cord_buf& buf, bool* format_error) {
  char header[12];
  if (buf.copy_to(header, sizeof(header)) < sizeof(header)) return nullptr;
  if (memcmp(header, "PRPC", 4) != 0) {
    fprintf(stderr, "[ERROR] Unmatched magic string\n");
    *format_error = true;
    return nullptr;
  }
  const uint32_t body_size = get_be32(header + 4);
  const uint32_t meta_size = get_be32(header + 8);
  if (body_size > FLAGS_max_body_size) {
    fprintf(stderr, "[ERROR] Too big body=%u\n", body_size);
    *format_error = true;
    return nullptr;
  }
  if (buf.length() < sizeof(header) + (size_t)body_size) return nullptr;
  if (meta_size > body_size) {
    fprintf(stderr, "[ERROR] meta_size=%u is bigger than body_size=%u\n", meta_size, body_size);
    *format_error = true;
    return nullptr;
  }
  buf.pop_front(sizeof(header));
  cord_buf meta_buf;
  buf.cutn(&meta_buf, meta_size);
  std::unique_ptr<SampledRequest> req(new SampledRequest);
  if (!req->meta.Parse(meta_buf.to_string())) {
    fprintf(stderr, "[ERROR] Fail to parse RpcDumpMeta\n");
    *format_error = true;
    return nullptr;
  }
  buf.cutn(&req->request, body_size - meta_size);
  return req;
}

// ------------------------------------------------------------------- replay
void ReplayAsBaiduStd(const SampledRequest& sample, uint64_t correlation_id, cord_buf* frame) {
  Controller cntl;
  cntl.set_request_compress_type((CompressType)sample.meta.compress_type());
  cord_buf body(sample.request);
  cord_buf serialized;
  if (sample.meta.attachment_size() > 0) {
    body.cutn(&serialized, body.size() - (size_t)sample.meta.attachment_size());
    cntl.request_attachment().swap(body);
  } else {
    serialized.swap(body);
  }
  policy::PackRpcRequest(frame, correlation_id, sample.meta.service_name(),
                         sample.meta.method_name(), &cntl, serialized);
}

size_t DecompressSamples(const std::vector<const SampledRequest*>& samples,
                         std::vector<cord_buf>* bodies, std::vector<bool>* ok) {
  const size_t n = samples.size();
  bodies->assign(n, cord_buf());
  ok->assign(n, false);
  std::vector<cord_buf> compressed;
  std::vector<size_t> owner;
  for (size_t i = 0; i < n; ++i) {
    const SampledRequest& s = *samples[i];
    const int att = s.meta.attachment_size();
    if (att < 0 || (size_t)att > s.request.size()) continue;
    cord_buf body(s.request), msg;
    body.cutn(&msg, body.size() - (size_t)att);
    if (s.meta.compress_type() == COMPRESS_TYPE_NONE) {
      (*bodies)[i].swap(msg);
      (*ok)[i] = true;
    } else if (s.meta.compress_type() == COMPRESS_TYPE_SNAPPY) {
      compressed.emplace_back(std::move(msg));
      owner.push_back(i);
    }
  }
  if (!compressed.empty()) {
    std::vector<const cord_buf*> in(compressed.size());
    std::vector<cord_buf*> out(compressed.size());
    for (size_t k = 0; k < compressed.size(); ++k) {
      in[k] = &compressed[k];
      out[k] = &(*bodies)[owner[k]];
    }
    std::vector<bool> r;
    gpu::SnappyGpuCodec::Instance().UncompressBatch(in, out, &r);
    for (size_t k = 0; k < compressed.size(); ++k) {
      (*ok)[owner[k]] = k < r.size() && r[k];
      if (!(*ok)[owner[k]]) (*bodies)[owner[k]].clear();
    }
  }
  size_t good = 0;
  for (size_t i = 0; i < n; ++i) good += (*ok)[i] ? 1 : 0;
  return good;
}

}  // namespace flare::rpc
