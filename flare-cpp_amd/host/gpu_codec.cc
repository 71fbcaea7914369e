// gpu_codec.cc -- see gpu_codec.h.
#include "gpu_codec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/flare_snappy_gpu.h"
#include "pinned.h"
#include "snappy_cpu.h"

namespace flare::gpu {

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    release();
    size_t want = n + n / 4 + 4096;
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {  // pinned host memory, so hipMemcpyAsync is a true DMA
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    release();
    size_t want = n + n / 4 + 4096;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

enum Kind { kCompress = 0, kDecompress = 1, kValidate = 2 };

struct Request {
  const cord_buf* in;
  cord_buf* out;
  Kind kind;
  bool ok = false;       // the verdict
  bool handled = false;  // a device (or the host codec) produced it
  bool done = false;
  void* latch = nullptr;
  void (*signal)(void*) = nullptr;
};

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Host threads for gather / scatter of large chunks (copies into pinned
// staging are CPU memcpy; one core moves ~10 GB/s).
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

// Flat copy of a cord_buf (the host codec works on contiguous bytes).
const uint8_t* flatten(const cord_buf& in, std::vector<uint8_t>* tmp) {
  if (in.backing_block_num() == 1) return reinterpret_cast<const uint8_t*>(in.backing_block(0).data());
  tmp->resize(in.size() + 1);
  in.copy_to(tmp->data(), in.size());
  return tmp->data();
}

// A valid stream expands at most 64/3x (a 3-byte COPY_2 of length 64) plus
// its header: a longer header length cannot decode (the reference would run
// out of input and return false), so nothing is allocated for it.
inline bool plausible_length(uint32_t ulen, size_t in_len) { return (uint64_t)ulen <= 22ull * in_len + 64; }

bool cpu_run(Kind kind, const cord_buf& in, cord_buf* out) {
  std::vector<uint8_t> tin, tout;  // per call: no thread_local (see snappy_cpu.cc)
  const uint8_t* p = flatten(in, &tin);
  const size_t n = in.size();
  if (kind == kCompress) {
    tout.resize(snappy::cpu::MaxCompressedLength(n));
    out->append(tout.data(), snappy::cpu::Compress(p, n, tout.data()));
    return true;
  }
  if (kind == kValidate) return snappy::cpu::IsValid(p, n);
  uint32_t ulen = 0;
  const size_t h = snappy::cpu::ReadHeader(p, n, &ulen, /*strict=*/false);
  if (h == 0 || !plausible_length(ulen, n)) return false;
  tout.resize((size_t)ulen + 32);
  if (!snappy::cpu::Decode(p, n, h, tout.data(), ulen, nullptr, tout.size())) return false;
  out->append(tout.data(), ulen);
  return true;
}

constexpr int kSlots = 3;
// Outputs at least this long are adopted from the pinned slab; shorter ones
// are copied (an adopted range costs a block header and a slab reference).
constexpr uint32_t kAdoptMin = 2048;

struct Counters {
  std::atomic<uint64_t> batches{0}, messages{0}, bytes_in{0}, bytes_out{0}, max_batch{0},
      failures{0}, cpu_messages{0}, fallbacks{0}, adopted{0};
};

// One HIP device's runtime.
struct Device {
  int id = -1;
  hipStream_t streams[kSlots] = {};
  // Decode is copy-bound end to end and pipelines well in 256 MiB chunks;
  // encode is latency-bound on the GPU and needs every message of the batch
  // in one launch, so it is not chunked.  FLARE_SNAPPY_GPU_CHUNK_BYTES
  // overrides both (tests force many small chunks).
  size_t chunk_bytes = 256ull << 20;
  size_t chunk_bytes_compress = ~size_t(0);
  DevBuf d_in, d_meta, d_out, d_ws[kSlots], d_gath;
  HostBuf h_in, h_meta, h_out, h_gath;

  bool start(int dev, std::string* err) {
    id = dev;
    if (fsg_init(dev) != FSG_SUCCESS) {
      *err = std::string("fsg_init failed: ") + fsg_last_error();
      return false;
    }
    for (auto& st : streams) {
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        st = nullptr;
        *err = "hipStreamCreate failed";
        return false;
      }
    }
    if (const char* cb = getenv("FLARE_SNAPPY_GPU_CHUNK_BYTES")) {
      chunk_bytes = std::max<size_t>(1, strtoull(cb, nullptr, 10));
      chunk_bytes_compress = chunk_bytes;
    }
    return true;
  }

  void stop() {
    if (id < 0) return;
    (void)hipSetDevice(id);
    for (auto& st : streams)
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
        st = nullptr;
      }
    d_in.release();
    d_meta.release();
    d_out.release();
    d_gath.release();
    for (auto& w : d_ws) w.release();
    h_in.release();
    h_meta.release();
    h_out.release();
    h_gath.release();
    id = -1;
  }

  // Runs one device batch for `reqs` (all of `kind`).  Every request it
  // finishes gets handled = true; returns false after a device error (the
  // unfinished requests are left to the host codec).
  bool run(const std::vector<Request*>& reqs, Kind kind, Counters* ctr);
};

std::atomic<int> g_inject_errors{0};  // test hook: fail the next n device batches

bool Device::run(const std::vector<Request*>& reqs, Kind kind, Counters* ctr) {
  const uint32_t n = (uint32_t)reqs.size();
  if (n == 0) return true;
  for (int k = g_inject_errors.load(); k > 0;)
    if (g_inject_errors.compare_exchange_weak(k, k - 1)) return false;
  if (hipSetDevice(id) != hipSuccess) return false;
  const bool compress = kind == kCompress, validate = kind == kValidate;
  // ---- sizes; messages whose verdict the header already decides are skipped
  std::vector<uint32_t> ulen(n, 0);
  std::vector<uint8_t> skip(n, 0);
  std::vector<uint32_t> blk_base(n + 1, 0);
  size_t total_out = 0;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const size_t len = reqs[i]->in->size();
    blk_base[i + 1] = blk_base[i];
    // beyond the format's uint32 lengths, or (compress) a worst-case output
    // the u32 slot sizes cannot describe: the host codec takes these
    if (len > 0xffffffffu || (compress && fsg_max_compressed_length(len) > 0xffffffffu)) {
      skip[i] = 2;
      continue;
    }
    if (compress) {
      total_out += align16(fsg_max_compressed_length(len));
      max_len = std::max<uint32_t>(max_len, (uint32_t)len);
    } else {
      uint8_t hdr[5];
      const size_t k = reqs[i]->in->copy_to(hdr, sizeof(hdr));
      uint32_t u = 0;
      if (fsg_get_uncompressed_length(hdr, k, &u, /*lenient=*/1) == 0 || !plausible_length(u, len)) {
        skip[i] = 1;  // the reference returns false
        continue;
      }
      ulen[i] = u;
      if (!validate) total_out += align16(u);
    }
    blk_base[i + 1] += (uint32_t)reqs[i]->in->backing_block_num();
  }
  const uint32_t n_blk = blk_base[n];
  // metadata: in_off u64, out_off u64, in_len u32, out_cap u32, out_len u32, status i32
  const size_t meta_bytes = (size_t)n * (8 + 8 + 4 + 4 + 4 + 4);
  const size_t gath_bytes = (size_t)n_blk * (8 + 8 + 4);
  size_t total_in = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!skip[i]) total_in += align16(reqs[i]->in->size());
  if (!h_in.reserve(total_in + 16) || !h_meta.reserve(meta_bytes) || !h_gath.reserve(gath_bytes + 16) ||
      !d_in.reserve(total_in + 16) || !d_meta.reserve(meta_bytes) || !d_gath.reserve(gath_bytes + 16) ||
      !d_out.reserve(total_out + 16))
    return false;
  // D2H target: a pinned slab the outputs are adopted from, else staging
  OutSlab* slab = validate ? nullptr : AcquireOutSlab(total_out + 16);
  // under slab pressure outputs are copied, so this slab returns to the pool
  // right after the batch instead of being held by long-lived cord_bufs
  const bool adopt = slab && !OutSlabsUnderPressure();
  if (!validate && slab == nullptr && !h_out.reserve(total_out + 16)) return false;
  uint8_t* hout = slab ? OutSlabData(slab) : h_out.as<uint8_t>();

  // Metadata columns, back to back in this order on host and device (the
  // one-chunk path below copies in_off..out_cap and out_len..status as two
  // contiguous spans, so the order and the packing are load-bearing):
  //   in_off u64[n] | out_off u64[n] | in_len u32[n] | out_cap u32[n] | out_len u32[n] | status i32[n]
  constexpr size_t kColInOff = 0, kColOutOff = 8, kColInLen = 16, kColOutCap = 20, kColOutLen = 24, kColStatus = 28;
  static_assert(kColOutOff == kColInOff + 8 && kColInLen == kColOutOff + 8 && kColOutCap == kColInLen + 4 &&
                    kColOutLen == kColOutCap + 4 && kColStatus == kColOutLen + 4,
                "the combined H2D (24n bytes from in_off) and D2H (8n bytes from out_len) copies need these "
                "columns contiguous and in this order");
  uint8_t* m = h_meta.as<uint8_t>();
  auto* in_off = reinterpret_cast<uint64_t*>(m + kColInOff * n);
  auto* out_off = reinterpret_cast<uint64_t*>(m + kColOutOff * n);
  auto* in_len = reinterpret_cast<uint32_t*>(m + kColInLen * n);
  auto* out_cap = reinterpret_cast<uint32_t*>(m + kColOutCap * n);
  auto* out_len = reinterpret_cast<uint32_t*>(m + kColOutLen * n);
  auto* status = reinterpret_cast<int32_t*>(m + kColStatus * n);
  uint8_t* dm = d_meta.as<uint8_t>();
  auto* d_in_off = reinterpret_cast<uint64_t*>(dm + kColInOff * n);
  auto* d_out_off = reinterpret_cast<uint64_t*>(dm + kColOutOff * n);
  auto* d_in_len = reinterpret_cast<uint32_t*>(dm + kColInLen * n);
  auto* d_out_cap = reinterpret_cast<uint32_t*>(dm + kColOutCap * n);
  auto* d_out_len = reinterpret_cast<uint32_t*>(dm + kColOutLen * n);
  auto* d_status = reinterpret_cast<int32_t*>(dm + kColStatus * n);
  // pinned-block descriptors: src u64, dst offset u64, length u32 (0 = staged)
  uint8_t* g = h_gath.as<uint8_t>();
  auto* g_src = reinterpret_cast<uint64_t*>(g);
  auto* g_dst = reinterpret_cast<uint64_t*>(g + 8ull * n_blk);
  auto* g_len = reinterpret_cast<uint32_t*>(g + 16ull * n_blk);
  uint8_t* dg = d_gath.as<uint8_t>();
  auto* dg_src = reinterpret_cast<uint64_t*>(dg);
  auto* dg_dst = reinterpret_cast<uint64_t*>(dg + 8ull * n_blk);
  auto* dg_len = reinterpret_cast<uint32_t*>(dg + 16ull * n_blk);
  uint8_t* hin = h_in.as<uint8_t>();

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
    const size_t cap = compress ? fsg_max_compressed_length(w) : (validate ? 0 : ulen[i]);
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
  uint64_t bytes_in = 0, bytes_out = 0, adopted = 0, corrupt = 0;
  auto finish = [&](int slot) {  // wait for a slot's chunk, scatter its results
    const int k = pending[slot];
    if (k < 0) return;
    pending[slot] = -1;
    if (hipStreamSynchronize(streams[slot]) != hipSuccess) {
      fprintf(stderr, "[flare-snappy-gpu] stream error on device %d\n", id);
      failed = true;
      return;
    }
    // ---- scatter: append results to the callers' cord_bufs (serial: page
    // faults from many threads at once measured 3x slower than one thread)
    for (uint32_t i = cut[k]; i < cut[k + 1]; ++i) {
      Request* r = reqs[i];
      if (skip[i] == 2) continue;  // for the host codec
      r->handled = true;
      if (skip[i] || status[i] != FSG_OK) {
        r->ok = false;
        ++corrupt;
        continue;
      }
      r->ok = true;
      bytes_in += in_len[i];
      if (validate) continue;
      const uint32_t L = out_len[i];
      if (adopt && L >= kAdoptMin) {
        OutSlabRef(slab);
        r->out->append_user_data(hout + out_off[i], L, AdoptedDeleter);
        ++adopted;
      } else {
        r->out->append(hout + out_off[i], L);
      }
      bytes_out += L;
    }
  };
  for (size_t k = 0; k < n_chunks && !failed; ++k) {
    const int slot = (int)(k % kSlots);
    finish(slot);  // its previous chunk (staging regions are disjoint, streams are not)
    if (failed) break;
    const uint32_t a = cut[k], b = cut[k + 1], cn = b - a;
    // ---- gather: cord_buf backing blocks (cord_buf.cc:1469-1475) -- pinned
    // ones become descriptors for the device gather, the rest is staged
    const size_t ia = in_off[a], ib = b < n ? in_off[b] : pos_in;
    std::atomic<uint64_t> staged{0}, direct{0};
    parallel_for(a, b, ib - ia, [&](uint32_t i) {
      if (skip[i]) return;
      const cord_buf& in = *reqs[i]->in;
      size_t w = 0;
      uint64_t st = 0, dr = 0;
      for (size_t blk = 0; blk < in.backing_block_num(); ++blk) {
        std::string_view v = in.backing_block(blk);
        const uint32_t j = blk_base[i] + (uint32_t)blk;
        g_dst[j] = in_off[i] + w;
        if (v.size() >= 1024 && IsPinned(v.data(), v.size())) {
          g_src[j] = reinterpret_cast<uint64_t>(v.data());
          g_len[j] = (uint32_t)v.size();
          dr += v.size();
        } else {
          g_src[j] = 0;
          g_len[j] = 0;
          memcpy(hin + in_off[i] + w, v.data(), v.size());
          st += v.size();
        }
        w += v.size();
      }
      staged += st;
      direct += dr;
    });
    hipStream_t st = streams[slot];
    const size_t oa = out_off[a], ob = b < n ? out_off[b] : pos_out;
    bool ok = true;
    if (staged.load() && ib > ia)
      ok = hipMemcpyAsync(d_in.as<uint8_t>() + ia, hin + ia, ib - ia, hipMemcpyHostToDevice, st) == hipSuccess;
    const uint32_t ja = blk_base[a], jn = blk_base[b] - blk_base[a];
    if (ok && direct.load() && jn) {
      ok = hipMemcpyAsync(dg_src + ja, g_src + ja, 8ull * jn, hipMemcpyHostToDevice, st) == hipSuccess &&
           hipMemcpyAsync(dg_dst + ja, g_dst + ja, 8ull * jn, hipMemcpyHostToDevice, st) == hipSuccess &&
           hipMemcpyAsync(dg_len + ja, g_len + ja, 4ull * jn, hipMemcpyHostToDevice, st) == hipSuccess &&
           fsg_gather_blocks(dg_src + ja, dg_len + ja, dg_dst + ja, jn, d_in.as<uint8_t>(), st) == FSG_SUCCESS;
    }
    // this chunk's offsets, lengths and caps: four column slices, or (one
    // chunk: the whole batch) the four columns in one copy -- per-copy
    // latency dominates a small batch
    if (n_chunks == 1) {
      ok = ok && hipMemcpyAsync(d_in_off, in_off, 24ull * n, hipMemcpyHostToDevice, st) == hipSuccess;
    } else {
      ok = ok && hipMemcpyAsync(d_in_off + a, in_off + a, 8ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
      ok = ok && hipMemcpyAsync(d_out_off + a, out_off + a, 8ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
      ok = ok && hipMemcpyAsync(d_in_len + a, in_len + a, 4ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
      ok = ok && hipMemcpyAsync(d_out_cap + a, out_cap + a, 4ull * cn, hipMemcpyHostToDevice, st) == hipSuccess;
    }
    if (!ok) {
      fprintf(stderr, "[flare-snappy-gpu] H2D copy failed on device %d\n", id);
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
      const size_t ws = validate ? 0 : fsg_decompress_workspace_bytes(cn, ib - ia);
      void* wsp = ws && d_ws[slot].reserve(ws) ? d_ws[slot].p : nullptr;
      rc = fsg_decompress_batch(d_in.as<uint8_t>(), d_in_off + a, d_in_len + a, cn,
                                validate ? nullptr : d_out.as<uint8_t>(), validate ? nullptr : d_out_off + a,
                                validate ? nullptr : d_out_cap + a, d_out_len + a, d_status + a,
                                validate ? FSG_FLAG_VALIDATE_ONLY : 0u, wsp, wsp ? ws : 0, st);
    }
    if (rc != FSG_SUCCESS) {
      fprintf(stderr, "[flare-snappy-gpu] batch launch failed on device %d: %s\n", id, fsg_last_error());
      failed = true;
      break;
    }
    ok = (n_chunks == 1
              ? hipMemcpyAsync(out_len, d_out_len, 8ull * n, hipMemcpyDeviceToHost, st) == hipSuccess
              : hipMemcpyAsync(out_len + a, d_out_len + a, 4ull * cn, hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipMemcpyAsync(status + a, d_status + a, 4ull * cn, hipMemcpyDeviceToHost, st) == hipSuccess) &&
         (validate || ob == oa ||
          hipMemcpyAsync(hout + oa, d_out.as<uint8_t>() + oa, ob - oa, hipMemcpyDeviceToHost, st) == hipSuccess);
    if (!ok) {
      fprintf(stderr, "[flare-snappy-gpu] D2H copy failed on device %d\n", id);
      failed = true;
      break;
    }
    pending[slot] = (int)k;
  }
  for (int s2 = 0; s2 < kSlots; ++s2) {  // drain (a failed batch leaves later chunks unhandled)
    if (failed) {
      if (pending[s2] >= 0) (void)hipStreamSynchronize(streams[s2]);
      pending[s2] = -1;
    } else {
      finish(s2);
    }
  }
  if (slab) OutSlabRelease(slab);  // the adopted ranges keep it alive
  ctr->batches += 1;
  ctr->messages += n;
  ctr->bytes_in += bytes_in;
  ctr->bytes_out += bytes_out;
  ctr->adopted += adopted;
  ctr->failures += corrupt;
  uint64_t mb = ctr->max_batch.load();
  while (n > mb && !ctr->max_batch.compare_exchange_weak(mb, n)) {
  }
  return !failed;
}

// Devices from FLARE_SNAPPY_GPU_DEVICES ("0x3" / "3" = a mask, "0,2" = a
// list) or FLARE_SNAPPY_GPU_DEVICE (one index); default device 0.
uint64_t env_device_mask() {
  if (const char* e = getenv("FLARE_SNAPPY_GPU_DEVICES")) {
    if (strchr(e, ',')) {
      uint64_t m = 0;
      for (const char* p = e; *p;) {
        m |= 1ull << (strtoul(p, nullptr, 10) & 63);
        p = strchr(p, ',');
        if (!p) break;
        ++p;
      }
      return m;
    }
    return strtoull(e, nullptr, 0);
  }
  if (const char* d = getenv("FLARE_SNAPPY_GPU_DEVICE")) return 1ull << (atoi(d) & 63);
  return 1;
}

size_t env_min_bytes() {
  const char* e = getenv("FLARE_SNAPPY_GPU_MIN_BYTES");
  return e ? (size_t)strtoull(e, nullptr, 10) : 16384;
}

}  // namespace

struct SnappyGpuCodec::Impl {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Request*> queue;
  std::vector<std::unique_ptr<Device>> devs;
  std::vector<char> busy;
  // double-checked start: read without the lock on every handler call,
  // published with release once start_locked has set the devices up
  std::atomic<bool> started{false};
  std::string err;
  std::atomic<int> n_devs{0};
  std::atomic<size_t> min_bytes{env_min_bytes()};
  ParkHooks hooks;
  Counters ctr;

  void ensure_started() {
    if (started.load(std::memory_order_acquire)) return;
    std::unique_lock<std::mutex> lk(mu);
    if (!started.load(std::memory_order_relaxed)) start_locked(env_device_mask());
  }

  int start_locked(uint64_t mask) {
    const int n = start_devices_locked(mask);
    started.store(true, std::memory_order_release);
    return n;
  }

  int start_devices_locked(uint64_t mask) {
    err.clear();
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
      err = "no HIP device";
      return 0;
    }
    for (int d = 0; d < 64 && d < count; ++d) {
      if (!(mask & (1ull << d))) continue;
      auto dev = std::make_unique<Device>();
      std::string e;
      if (dev->start(d, &e)) {
        devs.push_back(std::move(dev));
      } else {
        dev->stop();
        err += "device " + std::to_string(d) + ": " + e + "; ";
      }
    }
    busy.assign(devs.size(), 0);
    n_devs.store((int)devs.size());
    if (devs.empty() && err.empty()) err = "no device in the mask";
    return (int)devs.size();
  }

  // Waits until no device runs and nothing is queued (caller holds lk).
  void quiesce(std::unique_lock<std::mutex>& lk) {
    cv.wait(lk, [&] {
      return queue.empty() && std::none_of(busy.begin(), busy.end(), [](char b) { return b != 0; });
    });
  }

  void stop_locked() {
    for (auto& d : devs) d->stop();
    devs.clear();
    busy.clear();
    n_devs.store(0);
  }

  // Runs a mixed batch on device d; the host codec takes whatever the device
  // could not finish.
  void run_batch(Device& dev, const std::vector<Request*>& batch) {
    std::vector<Request*> by[3];
    for (Request* q : batch) by[q->kind].push_back(q);
    for (int k = 0; k < 3; ++k) {
      if (by[k].empty()) continue;
      dev.run(by[k], (Kind)k, &ctr);
      for (Request* q : by[k]) {
        if (q->handled) continue;
        q->ok = cpu_run(q->kind, *q->in, q->out);
        q->handled = true;
        ctr.fallbacks += 1;
        ctr.cpu_messages += 1;
      }
    }
  }

  // Leads device d (busy[d] set by the caller, lk held) until the queue is
  // empty, finishing and waking every request it takes.
  void lead(int d, std::unique_lock<std::mutex>& lk) {
    while (!queue.empty()) {
      std::vector<Request*> batch(queue.begin(), queue.end());
      queue.clear();
      lk.unlock();
      run_batch(*devs[d], batch);
      lk.lock();
      for (Request* q : batch) {
        q->done = true;
        if (q->latch) q->signal(q->latch);
      }
      cv.notify_all();
    }
  }

  // Queues r and returns once it is done; false if no device is running.
  bool submit(Request* r) {
    std::unique_lock<std::mutex> lk(mu);
    if (devs.empty()) return false;
    queue.push_back(r);
    int d = -1;
    for (size_t i = 0; i < busy.size(); ++i)
      if (!busy[i]) {
        d = (int)i;
        break;
      }
    if (d >= 0) {
      busy[d] = 1;
      lead(d, lk);
      busy[d] = 0;
      cv.notify_all();
      return true;
    }
    // follower: a leader (or an explicit batch releasing its device) drains
    // the queue before it lets its device go, so someone finishes r
    if (hooks.create && hooks.wait && hooks.signal && hooks.destroy) {
      const ParkHooks h = hooks;
      r->latch = h.create();
      r->signal = h.signal;
      lk.unlock();
      h.wait(r->latch);
      h.destroy(r->latch);
      lk.lock();
      cv.wait(lk, [&] { return r->done; });  // a latch that woke early
    } else {
      cv.wait(lk, [&] { return r->done; });
    }
    return true;
  }

  bool process(const cord_buf& in, cord_buf* out, Kind kind) {
    // devices start on the first body that needs one: a process whose bodies
    // all stay below the threshold never initialises HIP
    if (in.size() >= min_bytes.load(std::memory_order_relaxed)) {
      ensure_started();
      if (n_devs.load(std::memory_order_relaxed) > 0) {
        Request r{&in, out, kind};
        if (submit(&r)) return r.ok;
      }
    }
    ctr.cpu_messages += 1;
    return cpu_run(kind, in, out);
  }

  // Explicit batches: split by bytes over the devices, each part run on its
  // device as one batch (the part's thread then drains the queue before it
  // releases the device).
  bool explicit_batch(const std::vector<const cord_buf*>& in, const std::vector<cord_buf*>& out,
                      std::vector<bool>* ok, Kind kind) {
    if (in.size() != out.size()) return false;
    ensure_started();
    std::vector<Request> rs(in.size());
    for (size_t i = 0; i < in.size(); ++i) rs[i] = Request{in[i], out[i], kind};
    const size_t nd = (size_t)n_devs.load();
    if (nd == 0) {
      for (auto& r : rs) {
        r.ok = cpu_run(kind, *r.in, r.out);
        ctr.cpu_messages += 1;
      }
    } else {
      // contiguous ranges balanced by input bytes (shard.byte_balanced_ranges)
      size_t total = 0;
      for (auto& r : rs) total += r.in->size() + 64;
      std::vector<size_t> cuts{0};
      size_t acc = 0;
      for (size_t i = 0; i < rs.size() && cuts.size() < nd; ++i) {
        acc += rs[i].in->size() + 64;
        if (acc * nd >= total * cuts.size() && i + 1 < rs.size()) cuts.push_back(i + 1);
      }
      cuts.push_back(rs.size());
      auto part = [&](size_t p) {
        std::vector<Request*> batch;
        for (size_t i = cuts[p]; i < cuts[p + 1]; ++i) batch.push_back(&rs[i]);
        std::unique_lock<std::mutex> lk(mu);
        const size_t d = p % std::max<size_t>(1, devs.size());
        if (devs.empty()) {
          lk.unlock();
          for (Request* q : batch) {
            q->ok = cpu_run(kind, *q->in, q->out);
            ctr.cpu_messages += 1;
          }
          return;
        }
        cv.wait(lk, [&] { return !busy[d]; });
        busy[d] = 1;
        lk.unlock();
        run_batch(*devs[d], batch);
        lk.lock();
        lead((int)d, lk);
        busy[d] = 0;
        cv.notify_all();
      };
      const size_t parts = cuts.size() - 1;
      if (parts == 1) {
        part(0);
      } else {
        std::vector<std::thread> th;
        for (size_t p = 0; p < parts; ++p) th.emplace_back(part, p);
        for (auto& t : th) t.join();
      }
    }
    ok->assign(rs.size(), false);
    bool all = true;
    for (size_t i = 0; i < rs.size(); ++i) {
      (*ok)[i] = rs[i].ok;
      all = all && rs[i].ok;
    }
    return all;
  }
};

SnappyGpuCodec& SnappyGpuCodec::Instance() {
  static SnappyGpuCodec* inst = new SnappyGpuCodec();  // never destroyed: handlers may run at exit
  return *inst;
}

SnappyGpuCodec::SnappyGpuCodec() : impl_(new Impl) {}

SnappyGpuCodec::~SnappyGpuCodec() { delete impl_; }

int SnappyGpuCodec::InitDevices(uint64_t mask) {
  std::unique_lock<std::mutex> lk(impl_->mu);
  impl_->quiesce(lk);
  impl_->stop_locked();
  return impl_->start_locked(mask ? mask : env_device_mask());
}

void SnappyGpuCodec::Shutdown() {
  std::unique_lock<std::mutex> lk(impl_->mu);
  impl_->quiesce(lk);
  impl_->stop_locked();
  impl_->started.store(true, std::memory_order_release);  // stay on the host codec until InitDevices
  impl_->err = "shut down";
}

bool SnappyGpuCodec::available() {
  impl_->ensure_started();
  return impl_->n_devs.load() > 0;
}

std::string SnappyGpuCodec::error() {
  std::lock_guard<std::mutex> lk(impl_->mu);
  return impl_->err;
}

int SnappyGpuCodec::device_count() {
  impl_->ensure_started();
  return impl_->n_devs.load();
}

void SnappyGpuCodec::SetMinGpuBytes(size_t bytes) { impl_->min_bytes.store(bytes); }
size_t SnappyGpuCodec::min_gpu_bytes() const { return impl_->min_bytes.load(); }

void SnappyGpuCodec::SetParkHooks(const ParkHooks& hooks) {
  std::lock_guard<std::mutex> lk(impl_->mu);
  impl_->hooks = hooks;
}

bool SnappyGpuCodec::Compress(const cord_buf& in, cord_buf* out) { return impl_->process(in, out, kCompress); }
bool SnappyGpuCodec::Uncompress(const cord_buf& in, cord_buf* out) { return impl_->process(in, out, kDecompress); }
bool SnappyGpuCodec::IsValid(const cord_buf& in) { return impl_->process(in, nullptr, kValidate); }

bool SnappyGpuCodec::CompressBatch(const std::vector<const cord_buf*>& in, const std::vector<cord_buf*>& out,
                                   std::vector<bool>* ok) {
  return impl_->explicit_batch(in, out, ok, kCompress);
}

bool SnappyGpuCodec::UncompressBatch(const std::vector<const cord_buf*>& in, const std::vector<cord_buf*>& out,
                                     std::vector<bool>* ok) {
  return impl_->explicit_batch(in, out, ok, kDecompress);
}

CodecStats SnappyGpuCodec::stats() const {
  const Counters& c = impl_->ctr;
  CodecStats s;
  s.batches = c.batches.load();
  s.messages = c.messages.load();
  s.bytes_in = c.bytes_in.load();
  s.bytes_out = c.bytes_out.load();
  s.max_batch = c.max_batch.load();
  s.failures = c.failures.load();
  s.cpu_messages = c.cpu_messages.load();
  s.fallbacks = c.fallbacks.load();
  s.adopted = c.adopted.load();
  return s;
}

void InjectDeviceErrorsForTesting(int n) { g_inject_errors.store(n); }

bool CpuCompress(const cord_buf& in, cord_buf* out) { return cpu_run(kCompress, in, out); }
bool CpuUncompress(const cord_buf& in, cord_buf* out) { return cpu_run(kDecompress, in, out); }

}  // namespace flare::gpu
