// cord_buf.h -- the slice of flare::cord_buf the Snappy path touches.
//
// Mirrors /root/reference/flare/io/cord_buf.h: a non-contiguous, refcounted
// chain of block references.  Blocks are 8 KiB with a 32-byte header, i.e.
// 8160 payload bytes (cord_buf.h:67, cord_buf.cc:194-205,283-298); block
// memory comes from the swappable `blockmem_allocate`/`blockmem_deallocate`
// hooks (cord_buf.cc:159-166) so a GPU build can back blocks with pinned
// memory; `append_user_data` (cord_buf.h:260) adopts foreign memory with a
// deleter; `backing_block(i)` (cord_buf.cc:1469-1475) exposes each flat
// fragment for gather.  Only what the codec boundary needs is implemented:
// this is not the reference's zero-copy-stream / socket machinery.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace flare {

namespace iobuf {
// Swappable block allocator (cord_buf.cc:159-166).  Defaults to malloc/free.
extern void* (*blockmem_allocate)(size_t);
extern void (*blockmem_deallocate)(void*);
}  // namespace iobuf

class cord_buf {
 public:
  static constexpr size_t kDefaultBlockSize = 8192;  // cord_buf.h:67
  static constexpr size_t kBlockHeader = 32;
  static constexpr size_t kBlockPayload = kDefaultBlockSize - kBlockHeader;  // 8160

  cord_buf() = default;
  cord_buf(const cord_buf& other);
  cord_buf& operator=(const cord_buf& other);
  cord_buf(cord_buf&& other) noexcept;
  cord_buf& operator=(cord_buf&& other) noexcept;
  ~cord_buf();

  // Copy `n` bytes to the end (cord_buf.h:233).
  int append(const void* data, size_t n);
  int append(const std::string& s) { return append(s.data(), s.size()); }
  int append(std::string_view s) { return append(s.data(), s.size()); }
  // Reference-append another cord_buf's blocks (no byte copy).
  void append(const cord_buf& other);
  // Adopt `data` without copying; `deleter(data)` runs when the last
  // reference drops (cord_buf.h:260, cord_buf.cc:1197).
  int append_user_data(void* data, size_t size, void (*deleter)(void*));

  size_t size() const { return size_; }
  size_t length() const { return size_; }
  bool empty() const { return size_ == 0; }
  void clear();

  // Flat fragments (cord_buf.cc:1469-1475).
  size_t backing_block_num() const { return refs_.size(); }
  std::string_view backing_block(size_t i) const;

  // Copy out up to n bytes starting at `pos` (for headers / tests).
  size_t copy_to(void* dst, size_t n, size_t pos = 0) const;
  std::string to_string() const;

  // Remove the first n bytes into `out` (appended), like cutn.
  size_t cutn(cord_buf* out, size_t n);
  // Drop the first n bytes (cord_buf.h pop_front).
  size_t pop_front(size_t n) { return cutn(nullptr, n); }
  void swap(cord_buf& other) noexcept {
    refs_.swap(other.refs_);
    std::swap(size_, other.size_);
  }

  bool equals(std::string_view s) const;

 private:
  struct Block;
  struct Ref {
    Block* block;
    uint32_t offset;
    uint32_t length;
  };
  static Block* new_block();
  static void inc_ref(Block* b);
  static void dec_ref(Block* b);

  std::vector<Ref> refs_;
  size_t size_ = 0;
};

}  // namespace flare
