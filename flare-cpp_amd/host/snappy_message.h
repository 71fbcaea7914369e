// snappy_message.h -- SnappyMessageProto (/root/reference/test/snappy_message.proto:21-24)
//   message SnappyMessageProto { optional string text = 1; repeated int32 numbers = 2; }
// hand-serialized in proto2 wire format (field 1: LEN, field 2: unpacked
// varints, negative int32 as 10-byte sign-extended varints), which is what
// protobuf's SerializeToZeroCopyStream would emit for it.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "compress.h"

namespace snappy_message {

class SnappyMessageProto : public flare::rpc::Message {
 public:
  void set_text(const std::string& t) { text_ = t; has_text_ = true; }
  const std::string& text() const { return text_; }
  bool has_text() const { return has_text_; }
  void add_numbers(int32_t v) { numbers_.push_back(v); }
  int numbers_size() const { return (int)numbers_.size(); }
  int32_t numbers(int i) const { return numbers_[i]; }
  void Clear() { text_.clear(); has_text_ = false; numbers_.clear(); }

  std::string SerializeAsString() const {
    std::string out;
    if (has_text_) {
      out.push_back('\x0a');
      put_varint(&out, text_.size());
      out += text_;
    }
    for (int32_t v : numbers_) {
      out.push_back('\x10');
      put_varint(&out, (uint64_t)(int64_t)v);
    }
    return out;
  }
  bool ParseFromString(const std::string& s) {
    Clear();
    size_t p = 0;
    while (p < s.size()) {
      uint64_t key;
      if (!get_varint(s, &p, &key)) return false;
      const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
      if (field == 1 && wt == 2) {
        uint64_t len;
        if (!get_varint(s, &p, &len) || len > s.size() - p) return false;
        text_.assign(s, p, len);
        has_text_ = true;
        p += len;
      } else if (field == 2 && wt == 0) {
        uint64_t v;
        if (!get_varint(s, &p, &v)) return false;
        numbers_.push_back((int32_t)(uint32_t)v);
      } else if (field == 2 && wt == 2) {  // packed form is accepted on parse
        uint64_t len;
        if (!get_varint(s, &p, &len) || len > s.size() - p) return false;
        const size_t end = p + len;
        while (p < end) {
          uint64_t v;
          if (!get_varint(s, &p, &v)) return false;
          numbers_.push_back((int32_t)(uint32_t)v);
        }
      } else {
        return false;  // unknown fields are not needed by the tests
      }
    }
    return true;
  }
  bool SerializeToCordBuf(flare::cord_buf* out) const override {
    out->append(SerializeAsString());
    return true;
  }
  bool ParseFromCordBuf(const flare::cord_buf& in) override { return ParseFromString(in.to_string()); }

 private:
  static void put_varint(std::string* o, uint64_t v) {
    while (v >= 128) { o->push_back((char)(v | 128)); v >>= 7; }
    o->push_back((char)v);
  }
  static bool get_varint(const std::string& s, size_t* p, uint64_t* v) {
    uint64_t r = 0;
    for (int shift = 0; shift < 64 && *p < s.size(); shift += 7) {
      const uint8_t b = (uint8_t)s[(*p)++];
      r |= (uint64_t)(b & 127) << shift;
      if (b < 128) { *v = r; return true; }
    }
    return false;
  }

  std::string text_;
  bool has_text_ = false;
  std::vector<int32_t> numbers_;
};

}  // namespace snappy_message
