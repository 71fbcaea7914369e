// baidu_rpc_meta.h -- baidu_std's RpcMeta and rpc_dump's RpcDumpMeta as
// plain classes with proto2 wire serialization (pb_wire.h).
//
// Field numbers and types follow
//   /root/reference/flare/rpc/policy/baidu_rpc_meta.proto:26-50  (RpcMeta,
//       RpcRequestMeta, RpcResponseMeta)
//   /root/reference/flare/rpc/options.proto:77-80                (ChunkInfo)
//   /root/reference/flare/rpc/streaming_rpc_meta.proto:24-28     (StreamSettings)
//   /root/reference/flare/rpc/rpc_dump.proto:23-45               (RpcDumpMeta)
// Accessors mirror the generated protobuf API the reference's protocol code
// calls (set_x / has_x / x / mutable_x), so the framing code reads like
// baidu_rpc_protocol.cc.  Parse() is ParsePbFromCordBuf's contract
// (flare/rpc/protocol.cc:223-226): false on malformed input or on a missing
// required field (IsInitialized).  Enum fields are proto2 closed enums: a
// value outside the enum is kept out of the field (protobuf puts it in the
// unknown-field set).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace flare::rpc {

// flare/rpc/options.proto:38-67 (the values rpc_dump records).
enum ProtocolType {
  PROTOCOL_UNKNOWN = 0,
  PROTOCOL_BAIDU_STD = 1,
  PROTOCOL_STREAMING_RPC = 2,
  PROTOCOL_HULU_PBRPC = 3,
  PROTOCOL_SOFA_PBRPC = 4,
  PROTOCOL_PUBLIC_PBRPC = 8,
  PROTOCOL_NOVA_PBRPC = 9,
  PROTOCOL_H2 = 26,  // the last value
};

#define FLARE_PB_SCALAR(type, name)                                   \
 public:                                                              \
  bool has_##name() const { return has_##name##_; }                   \
  type name() const { return name##_; }                               \
  void set_##name(type v) {                                           \
    name##_ = v;                                                      \
    has_##name##_ = true;                                             \
  }                                                                   \
  void clear_##name() {                                               \
    name##_ = type();                                                 \
    has_##name##_ = false;                                            \
  }                                                                   \
                                                                      \
 private:                                                             \
  type name##_ = type();                                              \
  bool has_##name##_ = false;

#define FLARE_PB_STRING(name)                                         \
 public:                                                              \
  bool has_##name() const { return has_##name##_; }                   \
  const std::string& name() const { return name##_; }                 \
  void set_##name(std::string_view v) {                               \
    name##_.assign(v.data(), v.size());                               \
    has_##name##_ = true;                                             \
  }                                                                   \
  std::string* mutable_##name() {                                     \
    has_##name##_ = true;                                             \
    return &name##_;                                                  \
  }                                                                   \
  void clear_##name() {                                               \
    name##_.clear();                                                  \
    has_##name##_ = false;                                            \
  }                                                                   \
                                                                      \
 private:                                                             \
  std::string name##_;                                                \
  bool has_##name##_ = false;

#define FLARE_PB_MESSAGE(type, name)                                  \
 public:                                                              \
  bool has_##name() const { return has_##name##_; }                   \
  const type& name() const { return name##_; }                        \
  type* mutable_##name() {                                            \
    has_##name##_ = true;                                             \
    return &name##_;                                                  \
  }                                                                   \
  void clear_##name() {                                               \
    name##_ = type();                                                 \
    has_##name##_ = false;                                            \
  }                                                                   \
                                                                      \
 private:                                                             \
  type name##_;                                                       \
  bool has_##name##_ = false;

// options.proto:77-80
class ChunkInfo {
  FLARE_PB_SCALAR(int64_t, stream_id)  // = 1, required
  FLARE_PB_SCALAR(int64_t, chunk_id)   // = 2, required
 public:
  void SerializeTo(std::string* out) const;
  bool MergeFrom(std::string_view wire);
  bool IsInitialized() const { return has_stream_id_ && has_chunk_id_; }
};

// streaming_rpc_meta.proto:24-28
class StreamSettings {
  FLARE_PB_SCALAR(int64_t, stream_id)   // = 1, required
  FLARE_PB_SCALAR(bool, need_feedback)  // = 2
  FLARE_PB_SCALAR(bool, writable)       // = 3
 public:
  void SerializeTo(std::string* out) const;
  bool MergeFrom(std::string_view wire);
  bool IsInitialized() const { return has_stream_id_; }
};

namespace policy {

// baidu_rpc_meta.proto:37-45
class RpcRequestMeta {
  FLARE_PB_STRING(service_name)             // = 1, required
  FLARE_PB_STRING(method_name)              // = 2, required
  FLARE_PB_SCALAR(int64_t, log_id)          // = 3
  FLARE_PB_SCALAR(int64_t, trace_id)        // = 4
  FLARE_PB_SCALAR(int64_t, span_id)         // = 5
  FLARE_PB_SCALAR(int64_t, parent_span_id)  // = 6
  FLARE_PB_STRING(request_id)               // = 7
 public:
  void SerializeTo(std::string* out) const;
  bool MergeFrom(std::string_view wire);
  bool IsInitialized() const { return has_service_name_ && has_method_name_; }
};

// baidu_rpc_meta.proto:47-50
class RpcResponseMeta {
  FLARE_PB_SCALAR(int32_t, error_code)  // = 1
  FLARE_PB_STRING(error_text)           // = 2
 public:
  void SerializeTo(std::string* out) const;
  bool MergeFrom(std::string_view wire);
  bool IsInitialized() const { return true; }
};

// baidu_rpc_meta.proto:26-35
class RpcMeta {
  FLARE_PB_MESSAGE(RpcRequestMeta, request)          // = 1
  FLARE_PB_MESSAGE(RpcResponseMeta, response)        // = 2
  FLARE_PB_SCALAR(int32_t, compress_type)            // = 3
  FLARE_PB_SCALAR(int64_t, correlation_id)           // = 4
  FLARE_PB_SCALAR(int32_t, attachment_size)          // = 5
  FLARE_PB_MESSAGE(ChunkInfo, chunk_info)            // = 6
  FLARE_PB_STRING(authentication_data)               // = 7
  FLARE_PB_MESSAGE(StreamSettings, stream_settings)  // = 8
 public:
  void SerializeTo(std::string* out) const;
  std::string SerializeAsString() const {
    std::string s;
    SerializeTo(&s);
    return s;
  }
  size_t ByteSizeLong() const { return SerializeAsString().size(); }
  bool MergeFrom(std::string_view wire);
  // ParseFromString + IsInitialized, as ParsePbFromCordBuf does.
  bool Parse(std::string_view wire) {
    *this = RpcMeta();
    return MergeFrom(wire) && IsInitialized();
  }
  bool IsInitialized() const {
    return (!has_request_ || request_.IsInitialized()) &&
           (!has_chunk_info_ || chunk_info_.IsInitialized()) &&
           (!has_stream_settings_ || stream_settings_.IsInitialized());
  }
};

}  // namespace policy

// rpc_dump.proto:23-45
class RpcDumpMeta {
  FLARE_PB_STRING(service_name)              // = 1
  FLARE_PB_STRING(method_name)               // = 2
  FLARE_PB_SCALAR(int32_t, method_index)     // = 3
  FLARE_PB_SCALAR(int32_t, compress_type)    // = 4 (enum CompressType)
  FLARE_PB_SCALAR(int32_t, protocol_type)    // = 5 (enum ProtocolType)
  FLARE_PB_SCALAR(int32_t, attachment_size)  // = 6
  FLARE_PB_STRING(authentication_data)       // = 7
  FLARE_PB_STRING(user_data)                 // = 8
 public:
  void SerializeTo(std::string* out) const;
  std::string SerializeAsString() const {
    std::string s;
    SerializeTo(&s);
    return s;
  }
  bool MergeFrom(std::string_view wire);
  bool Parse(std::string_view wire) {
    *this = RpcDumpMeta();
    return MergeFrom(wire);
  }
};

#undef FLARE_PB_SCALAR
#undef FLARE_PB_STRING
#undef FLARE_PB_MESSAGE

}  // namespace flare::rpc
