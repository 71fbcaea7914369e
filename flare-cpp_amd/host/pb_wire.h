// pb_wire.h -- the proto2 wire-format primitives the framing layer needs
// (varint, int32/int64, bool, length-delimited, tag), hand-written because the
// C++ protobuf runtime is not part of this build.
//
// Serialization follows what protobuf's SerializeWithCachedSizes emits for
// proto2 messages: known fields in field-number order, only fields whose
// has-bit is set, negative int32/int64 as 10-byte two's-complement varints.
// Parsing accepts fields in any order, keeps the last value of a repeated
// scalar occurrence, merges repeated occurrences of sub-messages (protobuf's
// MergeFrom semantics), and skips unknown fields of every wire type except
// the deprecated groups (3/4), which are rejected.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace flare::pb {

enum WireType : uint32_t { kVarint = 0, kFixed64 = 1, kLen = 2, kStartGroup = 3, kEndGroup = 4, kFixed32 = 5 };

inline void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back((char)(v | 0x80));
    v >>= 7;
  }
  o->push_back((char)v);
}
inline void put_tag(std::string* o, uint32_t field, WireType wt) { put_varint(o, ((uint64_t)field << 3) | wt); }
// int32 fields sign-extend to 64 bits on the wire (10 bytes when negative).
inline void put_int32(std::string* o, uint32_t field, int32_t v) {
  put_tag(o, field, kVarint);
  put_varint(o, (uint64_t)(int64_t)v);
}
inline void put_int64(std::string* o, uint32_t field, int64_t v) {
  put_tag(o, field, kVarint);
  put_varint(o, (uint64_t)v);
}
inline void put_bool(std::string* o, uint32_t field, bool v) {
  put_tag(o, field, kVarint);
  o->push_back(v ? 1 : 0);
}
inline void put_bytes(std::string* o, uint32_t field, std::string_view v) {
  put_tag(o, field, kLen);
  put_varint(o, v.size());
  o->append(v.data(), v.size());
}

// Cursor over a serialized message.
class Reader {
 public:
  explicit Reader(std::string_view s) : p_(s.data()), end_(s.data() + s.size()) {}
  bool done() const { return p_ == end_; }

  // Up to 10 bytes; bits past 64 are dropped, as protobuf's parser does.
  bool varint(uint64_t* v) {
    uint64_t r = 0;
    for (int i = 0; i < 10; ++i) {
      if (p_ == end_) return false;
      const uint8_t b = (uint8_t)*p_++;
      r |= (uint64_t)(b & 0x7f) << (7 * i);
      if (b < 0x80) {
        *v = r;
        return true;
      }
    }
    return false;
  }
  // Reads a field key. Field number 0 is malformed.
  bool tag(uint32_t* field, WireType* wt) {
    uint64_t k;
    if (!varint(&k) || k > 0xffffffffull) return false;
    *field = (uint32_t)(k >> 3);
    *wt = (WireType)(k & 7);
    return *field != 0;
  }
  bool bytes(std::string_view* v) {
    uint64_t n;
    if (!varint(&n) || n > (uint64_t)(end_ - p_)) return false;
    *v = std::string_view(p_, (size_t)n);
    p_ += n;
    return true;
  }
  bool skip(WireType wt) {
    uint64_t v;
    std::string_view s;
    switch (wt) {
      case kVarint: return varint(&v);
      case kFixed64: return advance(8);
      case kLen: return bytes(&s);
      case kFixed32: return advance(4);
      default: return false;  // groups are not used by these messages
    }
  }

 private:
  bool advance(size_t n) {
    if ((size_t)(end_ - p_) < n) return false;
    p_ += n;
    return true;
  }
  const char* p_;
  const char* end_;
};

}  // namespace flare::pb
