// pinned.cc -- pinned host memory for the Snappy runtime: a registry of
// hipHostMalloc'd slabs, cord_buf's pinned block allocator (the
// blockmem_allocate hook, /root/reference/flare/io/cord_buf.cc:159-166), and
// refcounted output slabs whose ranges cord_bufs adopt with
// append_user_data (cord_buf.h:260, cord_buf.cc:1197).
//
// Slabs are allocated rarely and never returned to the driver (hipHostMalloc
// and hipHostFree are slow and synchronising): the registry only grows, so
// lookups need no lock.
#include "pinned.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "cord_buf.h"

namespace flare::gpu {

namespace {

struct Range {
  uintptr_t base;
  size_t size;
  OutSlab* slab;  // null: a block slab
};

constexpr int kMaxRanges = 1 << 14;
Range g_ranges[kMaxRanges];
std::atomic<int> g_nranges{0};
std::mutex g_reg_mu;  // writers only

int add_range(void* p, size_t n, OutSlab* slab) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  const int i = g_nranges.load(std::memory_order_relaxed);
  if (i >= kMaxRanges) return -1;
  g_ranges[i] = Range{reinterpret_cast<uintptr_t>(p), n, slab};
  g_nranges.store(i + 1, std::memory_order_release);
  return i;
}

std::atomic<int> g_last_hit{-1};  // a hint (no thread_local: see snappy_cpu.cc)

const Range* find_range(const void* p, size_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const int cnt = g_nranges.load(std::memory_order_acquire);
  auto hit = [&](int i) { return a >= g_ranges[i].base && a + n <= g_ranges[i].base + g_ranges[i].size; };
  const int last = g_last_hit.load(std::memory_order_relaxed);
  if (last >= 0 && last < cnt && hit(last)) return &g_ranges[last];
  for (int i = cnt - 1; i >= 0; --i)
    if (hit(i)) {
      g_last_hit.store(i, std::memory_order_relaxed);
      return &g_ranges[i];
    }
  return nullptr;
}

void* host_alloc(size_t n) {
  void* p = nullptr;
  return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

// ---- cord_buf blocks (8 KiB) carved from 64 MiB pinned slabs
constexpr size_t kBlockSlab = 64ull << 20;
std::mutex g_blk_mu;
std::vector<void*> g_blk_free;

void* block_allocate(size_t n) {
  if (n != cord_buf::kDefaultBlockSize) return ::malloc(n);
  std::lock_guard<std::mutex> lk(g_blk_mu);
  if (g_blk_free.empty()) {
    char* s = static_cast<char*>(host_alloc(kBlockSlab));
    if (s == nullptr || add_range(s, kBlockSlab, nullptr) < 0) return ::malloc(n);
    for (size_t off = kBlockSlab; off > 0; off -= cord_buf::kDefaultBlockSize)
      g_blk_free.push_back(s + off - cord_buf::kDefaultBlockSize);
  }
  void* p = g_blk_free.back();
  g_blk_free.pop_back();
  return p;
}

void block_deallocate(void* p) {
  const Range* r = find_range(p, 1);
  if (r == nullptr || r->slab != nullptr) {
    ::free(p);
    return;
  }
  std::lock_guard<std::mutex> lk(g_blk_mu);
  g_blk_free.push_back(p);
}

// ---- output slabs
std::mutex g_out_mu;
std::vector<OutSlab*> g_out_free;
size_t g_out_total = 0;

size_t out_cap_bytes() {
  static const size_t cap = [] {
    const char* e = getenv("FLARE_SNAPPY_GPU_PINNED_OUT_BYTES");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)(4ull << 30);
  }();
  return cap;
}

}  // namespace

struct OutSlab {
  uint8_t* data;
  size_t size;
  std::atomic<int64_t> refs{0};
};

bool IsPinned(const void* p, size_t n) { return find_range(p, n) != nullptr; }

int UsePinnedBlocks() {
  // one probe allocation: fail here (and keep malloc) when there is no HIP
  void* probe = block_allocate(cord_buf::kDefaultBlockSize);
  if (probe == nullptr || !IsPinned(probe, 1)) {
    if (probe) ::free(probe);
    return -1;
  }
  block_deallocate(probe);
  iobuf::blockmem_allocate = block_allocate;
  iobuf::blockmem_deallocate = block_deallocate;
  return 0;
}

OutSlab* AcquireOutSlab(size_t bytes) {
  std::lock_guard<std::mutex> lk(g_out_mu);
  OutSlab* best = nullptr;
  size_t bi = 0;
  for (size_t i = 0; i < g_out_free.size(); ++i)
    if (g_out_free[i]->size >= bytes && (best == nullptr || g_out_free[i]->size < best->size)) {
      best = g_out_free[i];
      bi = i;
    }
  if (best) {
    g_out_free.erase(g_out_free.begin() + (long)bi);
  } else {
    const size_t sz = std::max<size_t>(64ull << 20, (bytes + (16ull << 20) - 1) & ~((16ull << 20) - 1));
    if (g_out_total + sz > out_cap_bytes()) return nullptr;
    void* p = host_alloc(sz);
    if (p == nullptr) return nullptr;
    best = new OutSlab{static_cast<uint8_t*>(p), sz};
    if (add_range(p, sz, best) < 0) {  // leaks the slab's memory: registry full
      delete best;
      return nullptr;
    }
    g_out_total += sz;
  }
  best->refs.store(1, std::memory_order_relaxed);
  return best;
}

bool OutSlabsUnderPressure() {
  // more than half the cap allocated and no slab free: adopted outputs are
  // holding the pool, so new outputs are copied and their slab returns to
  // the pool right after the batch
  std::lock_guard<std::mutex> lk(g_out_mu);
  return g_out_free.empty() && 2 * g_out_total > out_cap_bytes();
}

uint8_t* OutSlabData(OutSlab* s) { return s->data; }

void OutSlabRef(OutSlab* s) { s->refs.fetch_add(1, std::memory_order_relaxed); }

void OutSlabRelease(OutSlab* s) {
  if (s->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  std::lock_guard<std::mutex> lk(g_out_mu);
  g_out_free.push_back(s);
}

void AdoptedDeleter(void* data) {
  const Range* r = find_range(data, 1);
  if (r && r->slab) OutSlabRelease(r->slab);
}

}  // namespace flare::gpu
