// gpu_codec.cc -- see gpu_codec.h.
#include "gpu_codec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/flare_snappy_gpu.h"

namespace flare::gpu {

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {  // pinned host memory, so hipMemcpyAsync is a true DMA
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return false;
    cap = want;
    return true;
  }
  ~HostBuf() {
    if (p) (void)hipHostFree(p);
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct Request {
  const cord_buf* in;
  cord_buf* out;
  bool compress;
  bool ok = false;
  bool done = false;
};

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Host threads for gather / scatter of large chunks (the copies into and out
// of pinned staging are CPU memcpy; one core moves ~10 GB/s).
unsigned host_threads() {
  static const unsigned t = [] {
    if (const char* e = getenv("FLARE_SNAPPY_GPU_HOST_THREADS")) return (unsigned)std::max(1, atoi(e));
    const unsigned hw = std::thread::hardware_concurrency();
    return std::min(16u, std::max(1u, hw));
  }();
  return t;
}

// fn(i) for i in [a, b), split over host threads when `bytes` is large.
template <class F>
void parallel_for(uint32_t a, uint32_t b, size_t bytes, F&& fn) {
  const unsigned nt = bytes < (8u << 20) ? 1u : std::min<unsigned>(host_threads(), b - a);
  if (nt <= 1) {
    for (uint32_t i = a; i < b; ++i) fn(i);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (unsigned t = 0; t < nt; ++t) {
    const uint32_t lo = a + (uint32_t)((uint64_t)(b - a) * t / nt);
    const uint32_t hi = a + (uint32_t)((uint64_t)(b - a) * (t + 1) / nt);
    th.emplace_back([lo, hi, &fn] {
      for (uint32_t i = lo; i < hi; ++i) fn(i);
    });
  }
  for (auto& x : th) x.join();
}

}  // namespace

// A large batch is cut into chunks of consecutive messages (>= kChunkBytes of
// input each, at most kSlots in flight): chunk k's gather into pinned staging
// runs on the CPU while chunk k-1's H2D / kernels / D2H run on the GPU, and
// chunks on different streams overlap their copies with each other's kernels.
constexpr int kSlots = 3;

struct SnappyGpuCodec::Impl {
  int device = 0;
  hipStream_t streams[kSlots] = {};
  // Decode is copy-bound end to end and pipelines well in 256 MiB chunks;
  // encode is latency-bound on the GPU and needs every message of the batch
  // in one launch, so it is not chunked.  FLARE_SNAPPY_GPU_CHUNK_BYTES
  // overrides both (tests force many small chunks).
  size_t chunk_bytes = 256ull << 20;
  size_t chunk_bytes_compress = ~size_t(0);

  std::mutex mu;
  std::condition_variable cv;
  std::deque<Request*> queue;
  bool busy = false;

  DevBuf d_in, d_meta, d_out, d_ws[kSlots];
  HostBuf h_in, h_meta, h_out;
  CodecStats stats;

  // Runs one device batch for `reqs` (all compress or all decompress).
  void run(const std::vector<Request*>& reqs, bool compress);
};

SnappyGpuCodec& SnappyGpuCodec::Instance() {
  static SnappyGpuCodec* inst = new SnappyGpuCodec();  // never destroyed: handlers may run at exit
  return *inst;
}

SnappyGpuCodec::SnappyGpuCodec() : impl_(new Impl) {
  const char* dev = getenv("FLARE_SNAPPY_GPU_DEVICE");
  impl_->device = dev ? atoi(dev) : 0;
  if (fsg_init(impl_->device) != FSG_SUCCESS) {
    err_ = std::string("fsg_init failed: ") + fsg_last_error();
    return;
  }
  for (auto& st : impl_->streams) {
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
      err_ = "hipStreamCreate failed";
      return;
    }
  }
  if (const char* cb = getenv("FLARE_SNAPPY_GPU_CHUNK_BYTES")) {
    impl_->chunk_bytes = std::max<size_t>(1, strtoull(cb, nullptr, 10));
    impl_->chunk_bytes_compress = impl_->chunk_bytes;
  }
  ok_ = true;
}

SnappyGpuCodec::~SnappyGpuCodec() {
  for (auto& st : impl_->streams)
    if (st) (void)hipStreamDestroy(st);
  delete impl_;
}

CodecStats SnappyGpuCodec::stats() const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  return impl_->stats;
}

void SnappyGpuCodec::Impl::run(const std::vector<Request*>& reqs, bool compress) {
  const uint32_t n = (uint32_t)reqs.size();
  if (n == 0) return;
  if (hipSetDevice(device) != hipSuccess) return;
  // ---- sizes and layout
  std::vector<uint32_t> ulen(n, 0);
  std::vector<uint8_t> skip(n, 0);
  size_t total_in = 0, total_out = 0;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const size_t len = reqs[i]->in->size();
    // beyond the format's uint32 lengths, or (compress) a worst-case output
    // the u32 slot sizes cannot describe
    if (len > 0xffffffffu || (compress && fsg_max_compressed_length(len) > 0xffffffffu)) {
      skip[i] = 1;
      continue;
    }
    total_in += align16(len);
    if (compress) {
      total_out += align16(fsg_max_compressed_length(len));
      max_len = std::max<uint32_t>(max_len, (uint32_t)len);
    } else {
      uint8_t hdr[5];
      const size_t k = reqs[i]->in->copy_to(hdr, sizeof(hdr));
      uint32_t u = 0;
      if (fsg_get_uncompressed_length(hdr, k, &u, /*lenient=*/1) == 0) {
        skip[i] = 1;  // header unreadable: the reference returns false
        continue;
      }
      // A valid stream expands at most 64/3x (a 3-byte COPY_2 of length 64):
      // anything larger cannot decode, and the reference returns false.
      if ((uint64_t)u > 22ull * len + 64) {
        skip[i] = 1;
        continue;
      }
      ulen[i] = u;
      total_out += align16(u);
    }
  }
  // metadata: in_off u64, in_len u32, out_off u64, out_cap u32, out_len u32, status i32
  const size_t meta_bytes = (size_t)n * (8 + 4 + 8 + 4 + 4 + 4);
  if (!h_in.reserve(total_in + 16) || !h_meta.reserve(meta_bytes) || !h_out.reserve(total_out + 16) ||
      !d_in.reserve(total_in + 16) || !d_meta.reserve(meta_bytes) || !d_out.reserve(total_out + 16)) {
    return;  // every request stays !ok
  }
  uint8_t* m = h_meta.as<uint8_t>();
  auto* in_off = reinterpret_cast<uint64_t*>(m);
  auto* out_off = reinterpret_cast<uint64_t*>(m + 8ull * n);
  auto* in_len = reinterpret_cast<uint32_t*>(m + 16ull * n);
  auto* out_cap = reinterpret_cast<uint32_t*>(m + 20ull * n);
  auto* out_len = reinterpret_cast<uint32_t*>(m + 24ull * n);
  auto* status = reinterpret_cast<int32_t*>(m + 28ull * n);
  uint8_t* dm = d_meta.as<uint8_t>();
  auto* d_in_off = reinterpret_cast<uint64_t*>(dm);
  auto* d_out_off = reinterpret_cast<uint64_t*>(dm + 8ull * n);
  auto* d_in_len = reinterpret_cast<uint32_t*>(dm + 16ull * n);
  auto* d_out_cap = reinterpret_cast<uint32_t*>(dm + 20ull * n);
  auto* d_out_len = reinterpret_cast<uint32_t*>(dm + 24ull * n);
  auto* d_status = reinterpret_cast<int32_t*>(dm + 28ull * n);
  uint8_t* hin = h_in.as<uint8_t>();
  const uint8_t* hout = h_out.as<uint8_t>();

  // ---- layout (offsets only; the copies happen per chunk)
  size_t pos_in = 0, pos_out = 0;
  for (uint32_t i = 0; i < n; ++i) {
    in_off[i] = pos_in;
    out_off[i] = pos_out;
    if (skip[i]) {
      in_len[i] = 0;
      out_cap[i] = 0;
      continue;
    }
    const size_t w = reqs[i]->in->size();
    in_len[i] = (uint32_t)w;
    pos_in += align16(w);
    const size_t cap = compress ? fsg_max_compressed_length(w) : ulen[i];
    out_cap[i] = (uint32_t)cap;
    pos_out += align16(cap);
  }
  // ---- chunks: [first, end) message ranges of >= chunk_bytes input
  std::vector<uint32_t> cut{0};
  const size_t cbytes = compress ? chunk_bytes_compress : chunk_bytes;
  for (uint32_t i = 0; i < n; ++i)
    if (i + 1 < n && in_off[i + 1] - in_off[cut.back()] >= cbytes) cut.push_back(i + 1);
  cut.push_back(n);
  const size_t n_chunks = cut.size() - 1;

  bool failed = false;
  std::vector<int> pending(kSlots, -1);  // chunk in flight on each stream
  uint64_t bytes_out = 0;
  auto finish = [&](int slot) {  // wait for a slot's chunk, scatter its results
    const int k = pending[slot];
    if (k < 0) return;
    pending[slot] = -1;
    if (hipStreamSynchronize(streams[slot]) != hipSuccess) {
      fprintf(stderr, "[flare-snappy-gpu] stream error\n");
      failed = true;
      return;
    }
    // ---- scatter: append results to the callers' cord_bufs.  Serial: the
    // appends allocate fresh blocks, and page faults from many threads at once
    // measured 3x slower than one thread.
    for (uint32_t i = cut[k]; i < cut[k + 1]; ++i) {
      Request* r = reqs[i];
      if (skip[i] || status[i] != FSG_OK) {
        r->ok = false;
        continue;
      }
      r->out->append(hout + out_off[i], out_len[i]);
      r->ok = true;
      bytes_out += out_len[i];
    }
  };
  for (size_t k = 0; k < n_chunks && !failed; ++k) {
    const int slot = (int)(k % kSlots);
    finish(slot);  // its previous chunk (staging regions are disjoint, streams are not)
    if (failed) break;
    const uint32_t a = cut[k], b = cut[k + 1], cn = b - a;
    // ---- gather: cord_buf backing blocks -> pinned staging (cord_buf.cc:1469-1475)
    const size_t ia = in_off[a], ib = b < n ? in_off[b] : pos_in;
    parallel_for(a, b, ib - ia, [&](uint32_t i) {
      if (skip[i]) return;
      const cord_buf& in = *reqs[i]->in;
      size_t w = 0;
      for (size_t blk = 0; blk < in.backing_block_num(); ++blk) {
        std::string_view v = in.backing_block(blk);
        memcpy(hin + in_off[i] + w, v.data(), v.size());
        w += v.size();
      }
    });
    hipStream_t st = streams[slot];
    const size_t oa = out_off[a], ob = b < n ? out_off[b] : pos_out;
    bool ok = true;
    ok = ok && (ib == ia || hipMemcpyAsync(d_in.as<uint8_t>() + ia, hin + ia, ib - ia,
                                           hipMemcpyHostToDevice, st) == hipSuccess);
    // this chunk's offsets, lengths and caps (four column slices)
    ok = ok && hipMemcpyAsync(d_in_off + a, in_off + a, 8ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(d_out_off + a, out_off + a, 8ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(d_in_len + a, in_len + a, 4ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(d_out_cap + a, out_cap + a, 4ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
    if (!ok) {
      fprintf(stderr, "[flare-snappy-gpu] H2D copy failed\n");
      failed = true;
      break;
    }
    int rc;
    if (compress) {
      uint32_t cmax = 0;
      for (uint32_t i = a; i < b; ++i) cmax = std::max(cmax, in_len[i]);
      const size_t ws = fsg_compress_workspace_bytes(cn, cmax);
      void* wsp = d_ws[slot].reserve(ws) ? d_ws[slot].p : nullptr;  // no workspace -> LDS-table kernel
      rc = fsg_compress_batch(d_in.as<uint8_t>(), d_in_off + a, d_in_len + a, cn, cmax,
                              d_out.as<uint8_t>(), d_out_off + a, d_out_len + a, d_status + a, wsp,
                              wsp ? ws : 0, st);
    } else {
      // two-pass decoder workspace (tag bitmap); without it the single-pass kernel runs
      const size_t ws = fsg_decompress_workspace_bytes(cn, ib - ia);
      void* wsp = d_ws[slot].reserve(ws) ? d_ws[slot].p : nullptr;
      rc = fsg_decompress_batch(d_in.as<uint8_t>(), d_in_off + a, d_in_len + a, cn, d_out.as<uint8_t>(),
                                d_out_off + a, d_out_cap + a, d_out_len + a, d_status + a, 0, wsp,
                                wsp ? ws : 0, st);
    }
    if (rc != FSG_SUCCESS) {
      fprintf(stderr, "[flare-snappy-gpu] batch launch failed: %s\n", fsg_last_error());
      failed = true;
      break;
    }
    ok = hipMemcpyAsync(out_len + a, d_out_len + a, 4ull * cn, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(status + a, d_status + a, 4ull * cn, hipMemcpyDeviceToHost, st) == hipSuccess &&
         (ob == oa || hipMemcpyAsync(h_out.as<uint8_t>() + oa, d_out.as<uint8_t>() + oa, ob - oa,
                                     hipMemcpyDeviceToHost, st) == hipSuccess);
    if (!ok) {
      fprintf(stderr, "[flare-snappy-gpu] D2H copy failed\n");
      failed = true;
      break;
    }
    pending[slot] = (int)k;
  }
  for (int s2 = 0; s2 < kSlots; ++s2) {  // drain (results of a failed batch stay !ok)
    if (failed) {
      if (pending[s2] >= 0) (void)hipStreamSynchronize(streams[s2]);
      pending[s2] = -1;
    } else {
      finish(s2);
    }
  }
  if (failed) return;  // requests of unfinished chunks stay !ok
  std::lock_guard<std::mutex> lk(mu);
  stats.batches += 1;
  stats.messages += n;
  stats.bytes_in += pos_in;
  stats.bytes_out += bytes_out;
  stats.max_batch = std::max<uint64_t>(stats.max_batch, n);
}

namespace {
// Leader/follower coalescing: whoever finds the runtime idle drains the queue.
bool submit(SnappyGpuCodec::Impl* impl, Request* r);
}  // namespace

bool SnappyGpuCodec::Compress(const cord_buf& in, cord_buf* out) {
  if (!ok_) return false;
  Request r{&in, out, true};
  return submit(impl_, &r);
}

bool SnappyGpuCodec::Uncompress(const cord_buf& in, cord_buf* out) {
  if (!ok_) return false;
  Request r{&in, out, false};
  return submit(impl_, &r);
}

namespace {
bool submit(SnappyGpuCodec::Impl* impl, Request* r) {
  std::unique_lock<std::mutex> lk(impl->mu);
  impl->queue.push_back(r);
  while (!r->done) {
    if (!impl->busy) {
      impl->busy = true;
      std::vector<Request*> comp, decomp;
      for (Request* q : impl->queue) (q->compress ? comp : decomp).push_back(q);
      impl->queue.clear();
      lk.unlock();
      impl->run(comp, true);
      impl->run(decomp, false);
      lk.lock();
      for (Request* q : comp) {
        if (!q->ok) impl->stats.failures += 1;
        q->done = true;
      }
      for (Request* q : decomp) {
        if (!q->ok) impl->stats.failures += 1;
        q->done = true;
      }
      impl->busy = false;
      impl->cv.notify_all();
    } else {
      impl->cv.wait(lk);
    }
  }
  return r->ok;
}
}  // namespace

static bool run_explicit(SnappyGpuCodec::Impl* impl, bool ok, const std::vector<const cord_buf*>& in,
                         const std::vector<cord_buf*>& out, std::vector<bool>* res, bool compress) {
  if (in.size() != out.size()) return false;
  res->assign(in.size(), false);
  if (!ok) return false;
  std::vector<Request> rs(in.size());
  std::vector<Request*> ps(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    rs[i] = Request{in[i], out[i], compress};
    ps[i] = &rs[i];
  }
  {
    // serialise with the coalescing path: wait until idle, then run
    std::unique_lock<std::mutex> lk(impl->mu);
    impl->cv.wait(lk, [&] { return !impl->busy; });
    impl->busy = true;
  }
  impl->run(ps, compress);
  {
    std::lock_guard<std::mutex> lk(impl->mu);
    impl->busy = false;
  }
  impl->cv.notify_all();
  bool all = true;
  for (size_t i = 0; i < in.size(); ++i) {
    (*res)[i] = rs[i].ok;
    all = all && rs[i].ok;
  }
  return all;
}

bool SnappyGpuCodec::CompressBatch(const std::vector<const cord_buf*>& in,
                                   const std::vector<cord_buf*>& out, std::vector<bool>* ok) {
  return run_explicit(impl_, ok_, in, out, ok, true);
}

bool SnappyGpuCodec::UncompressBatch(const std::vector<const cord_buf*>& in,
                                     const std::vector<cord_buf*>& out, std::vector<bool>* ok) {
  return run_explicit(impl_, ok_, in, out, ok, false);
}

}  // namespace flare::gpu
