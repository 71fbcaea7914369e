// baidu_rpc_meta.cc -- wire format of the framing metas (see baidu_rpc_meta.h).
#include "baidu_rpc_meta.h"

#include "pb_wire.h"

namespace flare::rpc {

using pb::Reader;
using pb::WireType;

namespace {

// Walks the fields of `wire`; `f(field, wire_type, reader)` returns 1 when it
// consumed a known field, 0 for an unknown one (skipped), -1 on malformed
// input.  A known field number with an unexpected wire type is an unknown
// field, as in protobuf.
template <class F>
bool for_each_field(std::string_view wire, F&& f) {
  Reader r(wire);
  while (!r.done()) {
    uint32_t field;
    WireType wt;
    if (!r.tag(&field, &wt)) return false;
    const int res = f(field, wt, r);
    if (res < 0) return false;
    if (res == 0 && !r.skip(wt)) return false;
  }
  return true;
}

// Nested message: tag, length, body.
template <class M>
void put_message(std::string* out, uint32_t field, const M& m) {
  std::string body;
  m.SerializeTo(&body);
  pb::put_bytes(out, field, body);
}

}  // namespace

#define PB_STR(num, name)                    \
  if (field == num && wt == pb::kLen) {      \
    std::string_view s_;                     \
    if (!r.bytes(&s_)) return -1;            \
    set_##name(s_);                          \
    return 1;                                \
  }
#define PB_VARINT(num, name, conv)           \
  if (field == num && wt == pb::kVarint) {   \
    uint64_t x_;                             \
    if (!r.varint(&x_)) return -1;           \
    set_##name(conv(x_));                    \
    return 1;                                \
  }
// proto2 closed enum: out-of-range values are consumed but not stored
#define PB_ENUM(num, name, lo, hi)                               \
  if (field == num && wt == pb::kVarint) {                       \
    uint64_t x_;                                                 \
    if (!r.varint(&x_)) return -1;                               \
    const int32_t v_ = (int32_t)(uint32_t)x_;                    \
    if (v_ >= (lo) && v_ <= (hi)) set_##name(v_);                \
    return 1;                                                    \
  }
#define PB_MSG(num, name)                                        \
  if (field == num && wt == pb::kLen) {                          \
    std::string_view s_;                                         \
    if (!r.bytes(&s_) || !mutable_##name()->MergeFrom(s_)) return -1; \
    return 1;                                                    \
  }

static inline int64_t as_i64(uint64_t x) { return (int64_t)x; }
static inline int32_t as_i32(uint64_t x) { return (int32_t)(uint32_t)x; }
static inline bool as_bool(uint64_t x) { return x != 0; }

// ---------------------------------------------------------------- ChunkInfo
void ChunkInfo::SerializeTo(std::string* out) const {
  if (has_stream_id_) pb::put_int64(out, 1, stream_id_);
  if (has_chunk_id_) pb::put_int64(out, 2, chunk_id_);
}
bool ChunkInfo::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_VARINT(1, stream_id, as_i64)
    PB_VARINT(2, chunk_id, as_i64)
    return 0;
  });
}

// ----------------------------------------------------------- StreamSettings
void StreamSettings::SerializeTo(std::string* out) const {
  if (has_stream_id_) pb::put_int64(out, 1, stream_id_);
  if (has_need_feedback_) pb::put_bool(out, 2, need_feedback_);
  if (has_writable_) pb::put_bool(out, 3, writable_);
}
bool StreamSettings::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_VARINT(1, stream_id, as_i64)
    PB_VARINT(2, need_feedback, as_bool)
    PB_VARINT(3, writable, as_bool)
    return 0;
  });
}

namespace policy {

// ----------------------------------------------------------- RpcRequestMeta
void RpcRequestMeta::SerializeTo(std::string* out) const {
  if (has_service_name_) pb::put_bytes(out, 1, service_name_);
  if (has_method_name_) pb::put_bytes(out, 2, method_name_);
  if (has_log_id_) pb::put_int64(out, 3, log_id_);
  if (has_trace_id_) pb::put_int64(out, 4, trace_id_);
  if (has_span_id_) pb::put_int64(out, 5, span_id_);
  if (has_parent_span_id_) pb::put_int64(out, 6, parent_span_id_);
  if (has_request_id_) pb::put_bytes(out, 7, request_id_);
}
bool RpcRequestMeta::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_STR(1, service_name)
    PB_STR(2, method_name)
    PB_VARINT(3, log_id, as_i64)
    PB_VARINT(4, trace_id, as_i64)
    PB_VARINT(5, span_id, as_i64)
    PB_VARINT(6, parent_span_id, as_i64)
    PB_STR(7, request_id)
    return 0;
  });
}

// ---------------------------------------------------------- RpcResponseMeta
void RpcResponseMeta::SerializeTo(std::string* out) const {
  if (has_error_code_) pb::put_int32(out, 1, error_code_);
  if (has_error_text_) pb::put_bytes(out, 2, error_text_);
}
bool RpcResponseMeta::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_VARINT(1, error_code, as_i32)
    PB_STR(2, error_text)
    return 0;
  });
}

// ------------------------------------------------------------------ RpcMeta
void RpcMeta::SerializeTo(std::string* out) const {
  if (has_request_) put_message(out, 1, request_);
  if (has_response_) put_message(out, 2, response_);
  if (has_compress_type_) pb::put_int32(out, 3, compress_type_);
  if (has_correlation_id_) pb::put_int64(out, 4, correlation_id_);
  if (has_attachment_size_) pb::put_int32(out, 5, attachment_size_);
  if (has_chunk_info_) put_message(out, 6, chunk_info_);
  if (has_authentication_data_) pb::put_bytes(out, 7, authentication_data_);
  if (has_stream_settings_) put_message(out, 8, stream_settings_);
}
bool RpcMeta::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_MSG(1, request)
    PB_MSG(2, response)
    PB_VARINT(3, compress_type, as_i32)
    PB_VARINT(4, correlation_id, as_i64)
    PB_VARINT(5, attachment_size, as_i32)
    PB_MSG(6, chunk_info)
    PB_STR(7, authentication_data)
    PB_MSG(8, stream_settings)
    return 0;
  });
}

}  // namespace policy

// -------------------------------------------------------------- RpcDumpMeta
void RpcDumpMeta::SerializeTo(std::string* out) const {
  if (has_service_name_) pb::put_bytes(out, 1, service_name_);
  if (has_method_name_) pb::put_bytes(out, 2, method_name_);
  if (has_method_index_) pb::put_int32(out, 3, method_index_);
  if (has_compress_type_) pb::put_int32(out, 4, compress_type_);
  if (has_protocol_type_) pb::put_int32(out, 5, protocol_type_);
  if (has_attachment_size_) pb::put_int32(out, 6, attachment_size_);
  if (has_authentication_data_) pb::put_bytes(out, 7, authentication_data_);
  if (has_user_data_) pb::put_bytes(out, 8, user_data_);
}
bool RpcDumpMeta::MergeFrom(std::string_view wire) {
  return for_each_field(wire, [&](uint32_t field, WireType wt, Reader& r) -> int {
    PB_STR(1, service_name)
    PB_STR(2, method_name)
    PB_VARINT(3, method_index, as_i32)
    PB_ENUM(4, compress_type, 0, 4)                 // options.proto:69-75
    PB_ENUM(5, protocol_type, 0, (int)PROTOCOL_H2)  // options.proto:38-67
    PB_VARINT(6, attachment_size, as_i32)
    PB_STR(7, authentication_data)
    PB_STR(8, user_data)
    return 0;
  });
}

#undef PB_STR
#undef PB_VARINT
#undef PB_ENUM
#undef PB_MSG

}  // namespace flare::rpc
