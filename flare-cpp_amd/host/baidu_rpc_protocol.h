// baidu_rpc_protocol.h -- baidu_std framing on either side of the codec
// (SURVEY.md §8(f) row 2).
//
// A baidu_std frame is
//   "PRPC" | body_size (u32 big-endian) | meta_size (u32 big-endian) |
//   RpcMeta (meta_size bytes) | payload (body_size - meta_size bytes)
// where payload = the (possibly compressed) message ++ attachment, and
// RpcMeta.attachment_size says where the attachment starts.  Follows
// /root/reference/flare/rpc/policy/baidu_rpc_protocol.cc:
//   PackRpcHeader :62-68, SerializeRpcHeaderAndMeta :70-90,
//   ParseRpcMessage :92-133, SendRpcResponse :136-266 (framing part),
//   ProcessRpcRequest :302-518 (meta / attachment / decompress part),
//   ProcessRpcResponse :544-620 (same), PackRpcRequest :622-687,
// and SerializeRequestDefault (/root/reference/flare/rpc/protocol.cc:130-151).
// Sockets, fibers, services, spans, streams and authentication are outside
// the hot path and not restated; the Controller below keeps only what these
// functions read and write.
//
// The batch entry point DecodeRpcFrames is the MI355X-native addition: it
// cuts every complete frame out of a receive buffer, and decompresses all
// SNAPPY bodies in ONE device batch (SnappyGpuCodec::UncompressBatch) instead
// of one handler call per frame.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "baidu_rpc_meta.h"
#include "compress.h"
#include "cord_buf.h"

namespace flare::rpc {

// flare/rpc/parse_result.h:25-50
enum ParseError {
  PARSE_OK = 0,
  PARSE_ERROR_TRY_OTHERS,
  PARSE_ERROR_NOT_ENOUGH_DATA,
  PARSE_ERROR_TOO_BIG_DATA,
  PARSE_ERROR_NO_RESOURCE,
  PARSE_ERROR_ABSOLUTELY_WRONG,
};
const char* ParseErrorToString(ParseError e);

// flare/rpc/errno.proto:25-47 (the codes these functions set)
enum Errno {
  ENOSERVICE = 1001,
  ENOMETHOD = 1002,
  EREQUEST = 1003,
  EINTERNAL = 2001,
  ERESPONSE = 2002,
};

// -max_body_size (flare/rpc/protocol.cc:45-46), default 64 MiB.
extern uint64_t FLAGS_max_body_size;

// A cut frame: the meta bytes and the payload (MostCommonMessage,
// flare/rpc/policy/most_common_message.h).
struct MostCommonMessage {
  cord_buf meta;
  cord_buf payload;
};

// The slice of flare/rpc/controller.h the framing reads and writes.
class Controller {
 public:
  void set_request_compress_type(CompressType t) { request_compress_type_ = t; }
  void set_response_compress_type(CompressType t) { response_compress_type_ = t; }
  CompressType request_compress_type() const { return request_compress_type_; }
  CompressType response_compress_type() const { return response_compress_type_; }

  void set_log_id(int64_t id) { log_id_ = id; has_log_id_ = true; }
  bool has_log_id() const { return has_log_id_; }
  int64_t log_id() const { return log_id_; }
  void set_request_id(const std::string& id) { request_id_ = id; }
  const std::string& request_id() const { return request_id_; }

  cord_buf& request_attachment() { return request_attachment_; }
  cord_buf& response_attachment() { return response_attachment_; }
  const cord_buf& request_attachment() const { return request_attachment_; }
  const cord_buf& response_attachment() const { return response_attachment_; }

  // printf-style text, as Controller::SetFailed.
  void SetFailed(int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
  bool Failed() const { return error_code_ != 0; }
  int ErrorCode() const { return error_code_; }
  const std::string& ErrorText() const { return error_text_; }

 private:
  CompressType request_compress_type_ = COMPRESS_TYPE_NONE;
  CompressType response_compress_type_ = COMPRESS_TYPE_NONE;
  int64_t log_id_ = 0;
  bool has_log_id_ = false;
  std::string request_id_;
  cord_buf request_attachment_;
  cord_buf response_attachment_;
  int error_code_ = 0;
  std::string error_text_;
};

// SerializeRequestDefault (protocol.cc:130-151): compress `request` into
// `buf` with the controller's request compress type; EREQUEST on failure.
void SerializeRequestDefault(cord_buf* buf, Controller* cntl, const Message* request);

namespace policy {

// "PRPC" + big-endian (meta_size + payload_size) + big-endian meta_size.
void PackRpcHeader(char* rpc_header, uint32_t meta_size, uint32_t payload_size);

// Header and serialized meta appended to `out`.
void SerializeRpcHeaderAndMeta(cord_buf* out, const RpcMeta& meta, size_t payload_size);

// Cut one frame from the front of `source`.  PARSE_OK fills `msg`.  A frame
// whose meta_size exceeds body_size is popped and reported as TRY_OTHERS.
ParseError ParseRpcMessage(cord_buf* source, MostCommonMessage* msg);

// Client: frame a request whose serialized (compressed) body is
// `request_body`; the controller's request attachment follows it.
// `service_name` is the service's full name (-baidu_protocol_use_fullname).
void PackRpcRequest(cord_buf* req_buf, uint64_t correlation_id,
                    const std::string& service_name, const std::string& method_name,
                    Controller* cntl, const cord_buf& request_body);

// Server: parse the frame's meta, split off the attachment into the
// controller, and decompress + parse the request body into `req`.  Returns
// false only when the meta itself is unparsable (the reference then fails
// the socket); otherwise request errors are on the controller (EREQUEST).
bool ProcessRpcRequest(MostCommonMessage* msg, Controller* cntl, Message* req, RpcMeta* meta_out);

// Server: frame the response to `correlation_id` (compressed with the
// controller's response compress type) into `out`.  A failed controller, or
// a failed serialization, sends the error code/text and no body.
void SendRpcResponse(int64_t correlation_id, Controller* cntl, const Message* res, cord_buf* out);

// Client: apply a response frame -- error code/text from the meta,
// attachment split, decompress + parse into `res` (if non-null).
void ProcessRpcResponse(MostCommonMessage* msg, Controller* cntl, Message* res);

// Batch receive path.  Cuts every complete frame from the front of `source`
// (stops at NOT_ENOUGH_DATA; a TRY_OTHERS/TOO_BIG frame ends the batch with
// that error in *stop).  For each frame: meta parsed, attachment split, and
// the body decompressed -- all SNAPPY bodies in one device batch; NONE
// bodies passed through.  ok[i] false = unparsable meta, attachment larger
// than the payload, unsupported compress type, or a corrupt body.
struct DecodedFrame {
  RpcMeta meta;
  cord_buf body;        // decompressed message bytes
  cord_buf attachment;
  bool ok = false;
};
size_t DecodeRpcFrames(cord_buf* source, std::vector<DecodedFrame>* frames, ParseError* stop);

}  // namespace policy
}  // namespace flare::rpc
