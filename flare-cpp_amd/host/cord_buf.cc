// cord_buf.cc -- see cord_buf.h.
#include "cord_buf.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>

namespace flare {

namespace iobuf {
void* (*blockmem_allocate)(size_t) = ::malloc;
void (*blockmem_deallocate)(void*) = ::free;
}  // namespace iobuf

// A block is either an 8 KiB allocation from blockmem_allocate (header kept
// inside the allocation, payload after kBlockHeader bytes, as the reference
// does) or adopted user data.
struct cord_buf::Block {
  std::atomic<int> nshared;
  uint32_t size;      // bytes written so far (owned blocks) / total (user data)
  uint32_t cap;       // payload capacity
  char* data;         // payload start
  void (*deleter)(void*);  // non-null: user data, freed with deleter(data)
};  // owned blocks live at the start of their own 8 KiB allocation

cord_buf::Block* cord_buf::new_block() {
  void* mem = iobuf::blockmem_allocate(kDefaultBlockSize);
  if (mem == nullptr) return nullptr;
  static_assert(sizeof(Block) <= kBlockHeader, "block header must fit in 32 bytes");
  Block* b = new (mem) Block;
  b->nshared.store(1, std::memory_order_relaxed);
  b->size = 0;
  b->cap = (uint32_t)kBlockPayload;
  b->data = static_cast<char*>(mem) + kBlockHeader;
  b->deleter = nullptr;
  return b;
}

void cord_buf::inc_ref(Block* b) { b->nshared.fetch_add(1, std::memory_order_relaxed); }

void cord_buf::dec_ref(Block* b) {
  if (b->nshared.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  if (b->deleter) {
    void (*d)(void*) = b->deleter;
    void* data = b->data;
    delete b;
    d(data);
  } else {
    b->~Block();
    iobuf::blockmem_deallocate(b);
  }
}

cord_buf::cord_buf(const cord_buf& o) : refs_(o.refs_), size_(o.size_) {
  for (auto& r : refs_) inc_ref(r.block);
}

cord_buf& cord_buf::operator=(const cord_buf& o) {
  if (this != &o) {
    cord_buf tmp(o);
    *this = std::move(tmp);
  }
  return *this;
}

cord_buf::cord_buf(cord_buf&& o) noexcept : refs_(std::move(o.refs_)), size_(o.size_) {
  o.refs_.clear();
  o.size_ = 0;
}

cord_buf& cord_buf::operator=(cord_buf&& o) noexcept {
  if (this != &o) {
    clear();
    refs_ = std::move(o.refs_);
    size_ = o.size_;
    o.refs_.clear();
    o.size_ = 0;
  }
  return *this;
}

cord_buf::~cord_buf() { clear(); }

void cord_buf::clear() {
  for (auto& r : refs_) dec_ref(r.block);
  refs_.clear();
  size_ = 0;
}

int cord_buf::append(const void* data, size_t n) {
  const char* p = static_cast<const char*>(data);
  while (n > 0) {
    Block* b = nullptr;
    // Extend the last ref in place when it ends at its block's write point
    // and we are the only holder of the block.
    if (!refs_.empty()) {
      Ref& last = refs_.back();
      Block* lb = last.block;
      if (lb->deleter == nullptr && last.offset + last.length == lb->size && lb->size < lb->cap &&
          lb->nshared.load(std::memory_order_relaxed) == 1)
        b = lb;
    }
    if (b == nullptr) {
      b = new_block();
      if (b == nullptr) return -1;
      refs_.push_back(Ref{b, 0, 0});
    }
    const size_t k = std::min<size_t>(n, b->cap - b->size);
    memcpy(b->data + b->size, p, k);
    b->size += (uint32_t)k;
    refs_.back().length += (uint32_t)k;
    size_ += k;
    p += k;
    n -= k;
  }
  return 0;
}

void cord_buf::append(const cord_buf& other) {
  // snapshot the count and index by position: `other` may be *this, whose
  // vector reallocates as it grows (the reference's append(self) works too)
  const size_t nrefs = other.refs_.size();
  const size_t nbytes = other.size_;
  refs_.reserve(refs_.size() + nrefs);
  for (size_t i = 0; i < nrefs; ++i) {
    const Ref r = other.refs_[i];
    inc_ref(r.block);
    refs_.push_back(r);
  }
  size_ += nbytes;
}

int cord_buf::append_user_data(void* data, size_t size, void (*deleter)(void*)) {
  if (size > 0xffffffffu) return -1;
  Block* b = new Block;
  b->nshared.store(1, std::memory_order_relaxed);
  b->size = (uint32_t)size;
  b->cap = (uint32_t)size;
  b->data = static_cast<char*>(data);
  b->deleter = deleter ? deleter : ::free;
  refs_.push_back(Ref{b, 0, (uint32_t)size});
  size_ += size;
  return 0;
}

std::string_view cord_buf::backing_block(size_t i) const {
  if (i >= refs_.size()) return {};
  const Ref& r = refs_[i];
  return std::string_view(r.block->data + r.offset, r.length);
}

size_t cord_buf::copy_to(void* dst, size_t n, size_t pos) const {
  char* d = static_cast<char*>(dst);
  size_t done = 0;
  for (const Ref& r : refs_) {
    if (done >= n) break;
    if (pos >= r.length) {
      pos -= r.length;
      continue;
    }
    const size_t k = std::min<size_t>(r.length - pos, n - done);
    memcpy(d + done, r.block->data + r.offset + pos, k);
    done += k;
    pos = 0;
  }
  return done;
}

std::string cord_buf::to_string() const {
  std::string s(size_, '\0');
  copy_to(&s[0], size_);
  return s;
}

size_t cord_buf::cutn(cord_buf* out, size_t n) {
  size_t moved = 0;
  size_t consumed_refs = 0;  // refs moved out entirely
  for (size_t j = 0; j < refs_.size() && moved < n; ++j) {
    Ref& r = refs_[j];
    const size_t k = std::min<size_t>(r.length, n - moved);
    if (out) {
      inc_ref(r.block);
      out->refs_.push_back(Ref{r.block, r.offset, (uint32_t)k});
      out->size_ += k;
    }
    moved += k;
    if (k == r.length) {
      dec_ref(r.block);
      ++consumed_refs;
    } else {
      r.offset += (uint32_t)k;  // partially cut: keep the tail
      r.length -= (uint32_t)k;
    }
  }
  refs_.erase(refs_.begin(), refs_.begin() + consumed_refs);
  size_ -= moved;
  return moved;
}

bool cord_buf::equals(std::string_view s) const {
  if (s.size() != size_) return false;
  size_t pos = 0;
  for (const Ref& r : refs_) {
    if (memcmp(s.data() + pos, r.block->data + r.offset, r.length) != 0) return false;
    pos += r.length;
  }
  return true;
}

}  // namespace flare
