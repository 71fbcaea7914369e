// baidu_rpc_protocol.cc -- see baidu_rpc_protocol.h.
#include "baidu_rpc_protocol.h"

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "gpu_codec.h"

namespace flare::rpc {

uint64_t FLAGS_max_body_size = 64ull * 1024 * 1024;  // protocol.cc:45

const char* ParseErrorToString(ParseError e) {  // parse_result.h:34-50
  switch (e) {
    case PARSE_OK: return "ok";
    case PARSE_ERROR_TRY_OTHERS: return "try other protocols";
    case PARSE_ERROR_NOT_ENOUGH_DATA: return "not enough data";
    case PARSE_ERROR_TOO_BIG_DATA: return "too big data";
    case PARSE_ERROR_NO_RESOURCE: return "no resource for the message";
    case PARSE_ERROR_ABSOLUTELY_WRONG: return "absolutely wrong message";
  }
  return "unknown ParseError";
}

void Controller::SetFailed(int code, const char* fmt, ...) {
  error_code_ = code == 0 ? -1 : code;  // SetFailed never leaves code 0
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (!error_text_.empty()) error_text_ += "; ";
  error_text_ += buf;
}

void SerializeRequestDefault(cord_buf* buf, Controller* cntl, const Message* request) {
  if (request == nullptr) return cntl->SetFailed(EREQUEST, "`request' is nullptr");
  if (!SerializeAsCompressedData(*request, buf, cntl->request_compress_type()))
    return cntl->SetFailed(EREQUEST, "Fail to compress request, compress_tpye=%d",
                           (int)cntl->request_compress_type());
}

namespace policy {

namespace {
inline void put_be32(char* p, uint32_t v) {  // raw_packer::pack32 (raw_pack.h:52-56)
  p[0] = (char)(v >> 24);
  p[1] = (char)(v >> 16);
  p[2] = (char)(v >> 8);
  p[3] = (char)v;
}
inline uint32_t get_be32(const char* p) {
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  return ((uint32_t)u[0] << 24) | ((uint32_t)u[1] << 16) | ((uint32_t)u[2] << 8) | u[3];
}
}  // namespace

void PackRpcHeader(char* rpc_header, uint32_t meta_size, uint32_t payload_size) {
  memcpy(rpc_header, "PRPC", 4);
  put_be32(rpc_header + 4, meta_size + payload_size);
  put_be32(rpc_header + 8, meta_size);
}

void SerializeRpcHeaderAndMeta(cord_buf* out, const RpcMeta& meta, size_t payload_size) {
  const std::string m = meta.SerializeAsString();
  char header[12];
  PackRpcHeader(header, (uint32_t)m.size(), (uint32_t)payload_size);
  out->append(header, sizeof(header));
  out->append(m);
}

ParseError ParseRpcMessage(cord_buf* source, MostCommonMessage* msg) {
  char header_buf[12];
  const size_t n = source->copy_to(header_buf, sizeof(header_buf));
  if (n >= 4) {
    if (memcmp(header_buf, "PRPC", 4) != 0) return PARSE_ERROR_TRY_OTHERS;
  } else if (memcmp(header_buf, "PRPC", n) != 0) {
    return PARSE_ERROR_TRY_OTHERS;
  }
  if (n < sizeof(header_buf)) return PARSE_ERROR_NOT_ENOUGH_DATA;
  const uint32_t body_size = get_be32(header_buf + 4);
  const uint32_t meta_size = get_be32(header_buf + 8);
  if (body_size > FLAGS_max_body_size) {
    fprintf(stderr, "[ERROR] body_size=%u is too large\n", body_size);
    return PARSE_ERROR_TOO_BIG_DATA;
  }
  if (source->length() < sizeof(header_buf) + (size_t)body_size) return PARSE_ERROR_NOT_ENOUGH_DATA;
  if (meta_size > body_size) {
    fprintf(stderr, "[ERROR] meta_size=%u is bigger than body_size=%u\n", meta_size, body_size);
    source->pop_front(sizeof(header_buf) + body_size);  // pop the message
    return PARSE_ERROR_TRY_OTHERS;
  }
  source->pop_front(sizeof(header_buf));
  source->cutn(&msg->meta, meta_size);
  source->cutn(&msg->payload, body_size - meta_size);
  return PARSE_OK;
}

void PackRpcRequest(cord_buf* req_buf, uint64_t correlation_id, const std::string& service_name,
                    const std::string& method_name, Controller* cntl,
                    const cord_buf& request_body) {
  RpcMeta meta;
  RpcRequestMeta* request_meta = meta.mutable_request();
  request_meta->set_service_name(service_name);
  request_meta->set_method_name(method_name);
  meta.set_compress_type(cntl->request_compress_type());
  if (cntl->has_log_id()) request_meta->set_log_id(cntl->log_id());
  if (!cntl->request_id().empty()) request_meta->set_request_id(cntl->request_id());
  meta.set_correlation_id((int64_t)correlation_id);
  const size_t req_size = request_body.length();
  const size_t attached_size = cntl->request_attachment().length();
  if (attached_size) meta.set_attachment_size((int32_t)attached_size);
  SerializeRpcHeaderAndMeta(req_buf, meta, req_size + attached_size);
  req_buf->append(request_body);
  if (attached_size) req_buf->append(cntl->request_attachment());
}

namespace {
// The attachment split shared by request and response processing
// (baidu_rpc_protocol.cc:455-469, :587-602): the last attachment_size bytes of
// the payload become the attachment; `body` gets the rest.
bool SplitAttachment(const RpcMeta& meta, cord_buf* payload, cord_buf* body, cord_buf* attachment,
                     Controller* cntl, int err, const char* what) {
  const int size = (int)payload->size();
  if (!meta.has_attachment_size()) {
    body->swap(*payload);
    return true;
  }
  if (size < meta.attachment_size()) {
    cntl->SetFailed(err, "attachment_size=%d is larger than %s_size=%d", meta.attachment_size(),
                    what, size);
    return false;
  }
  payload->cutn(body, (size_t)(size - meta.attachment_size()));
  attachment->swap(*payload);
  return true;
}
}  // namespace

bool ProcessRpcRequest(MostCommonMessage* msg, Controller* cntl, Message* req, RpcMeta* meta_out) {
  RpcMeta meta;
  if (!meta.Parse(msg->meta.to_string())) {
    fprintf(stderr, "[WARNING] Fail to parse RpcMeta\n");
    return false;
  }
  const RpcRequestMeta& request_meta = meta.request();
  if (request_meta.has_log_id()) cntl->set_log_id(request_meta.log_id());
  if (request_meta.has_request_id()) cntl->set_request_id(request_meta.request_id());
  cntl->set_request_compress_type((CompressType)meta.compress_type());
  if (meta_out) *meta_out = meta;

  const int req_size = (int)msg->payload.size();
  cord_buf req_buf;
  if (!SplitAttachment(meta, &msg->payload, &req_buf, &cntl->request_attachment(), cntl, EREQUEST,
                       "request"))
    return true;
  const CompressType req_cmp_type = (CompressType)meta.compress_type();
  if (!ParseFromCompressedData(req_buf, req, req_cmp_type)) {
    cntl->SetFailed(EREQUEST, "Fail to parse request message, CompressType=%s, request_size=%d",
                    CompressTypeToCStr(req_cmp_type), req_size);
  }
  return true;
}

void SendRpcResponse(int64_t correlation_id, Controller* cntl, const Message* res, cord_buf* out) {
  bool append_body = false;
  cord_buf res_body;
  const CompressType type = cntl->response_compress_type();
  if (res != nullptr && !cntl->Failed()) {
    if (!SerializeAsCompressedData(*res, &res_body, type)) {
      cntl->SetFailed(ERESPONSE, "Fail to serialize response, CompressType=%s",
                      CompressTypeToCStr(type));
    } else {
      append_body = true;
    }
  }
  size_t res_size = 0, attached_size = 0;
  if (append_body) {
    res_size = res_body.length();
    attached_size = cntl->response_attachment().length();
  }
  int error_code = cntl->ErrorCode();
  if (error_code == -1) error_code = EINTERNAL;  // :188-193
  RpcMeta meta;
  RpcResponseMeta* response_meta = meta.mutable_response();
  response_meta->set_error_code(error_code);
  if (!cntl->ErrorText().empty()) response_meta->set_error_text(cntl->ErrorText());
  meta.set_correlation_id(correlation_id);
  meta.set_compress_type(cntl->response_compress_type());
  if (attached_size > 0) meta.set_attachment_size((int32_t)attached_size);
  SerializeRpcHeaderAndMeta(out, meta, res_size + attached_size);
  if (append_body) {
    out->append(res_body);
    if (attached_size) out->append(cntl->response_attachment());
  }
}

void ProcessRpcResponse(MostCommonMessage* msg, Controller* cntl, Message* res) {
  RpcMeta meta;
  if (!meta.Parse(msg->meta.to_string())) {
    fprintf(stderr, "[WARNING] Fail to parse from response meta\n");
    return;
  }
  const RpcResponseMeta& response_meta = meta.response();
  if (response_meta.error_code() != 0) {
    cntl->SetFailed(response_meta.error_code(), "%s", response_meta.error_text().c_str());
    return;
  }
  const int res_size = (int)msg->payload.length();
  cord_buf res_buf;
  if (!SplitAttachment(meta, &msg->payload, &res_buf, &cntl->response_attachment(), cntl,
                       ERESPONSE, "response"))
    return;
  const CompressType res_cmp_type = (CompressType)meta.compress_type();
  cntl->set_response_compress_type(res_cmp_type);
  if (res != nullptr && !ParseFromCompressedData(res_buf, res, res_cmp_type)) {
    cntl->SetFailed(ERESPONSE, "Fail to parse response message, CompressType=%s, response_size=%d",
                    CompressTypeToCStr(res_cmp_type), res_size);
  }
}

size_t DecodeRpcFrames(cord_buf* source, std::vector<DecodedFrame>* frames, ParseError* stop) {
  const size_t first = frames->size();
  ParseError err = PARSE_OK;
  std::vector<cord_buf> compressed;  // SNAPPY bodies, in frame order
  std::vector<size_t> owner;         // frame index of each
  for (;;) {
    MostCommonMessage msg;
    err = ParseRpcMessage(source, &msg);
    if (err != PARSE_OK) break;
    frames->emplace_back();
    DecodedFrame& f = frames->back();
    if (!f.meta.Parse(msg.meta.to_string())) continue;  // ok stays false
    Controller cntl;
    cord_buf body;
    if (!SplitAttachment(f.meta, &msg.payload, &body, &f.attachment, &cntl, EREQUEST, "payload"))
      continue;
    const int type = f.meta.compress_type();
    if (type == COMPRESS_TYPE_NONE) {
      f.body.swap(body);
      f.ok = true;
    } else if (type == COMPRESS_TYPE_SNAPPY) {
      compressed.emplace_back(std::move(body));
      owner.push_back(frames->size() - 1);
    }  // other codecs: no handler on this path, ok stays false
  }
  if (stop) *stop = err;
  if (!compressed.empty()) {
    std::vector<const cord_buf*> in(compressed.size());
    std::vector<cord_buf*> out(compressed.size());
    for (size_t i = 0; i < compressed.size(); ++i) {
      in[i] = &compressed[i];
      out[i] = &(*frames)[owner[i]].body;
    }
    std::vector<bool> ok;
    gpu::SnappyGpuCodec::Instance().UncompressBatch(in, out, &ok);
    for (size_t i = 0; i < compressed.size(); ++i) {
      DecodedFrame& f = (*frames)[owner[i]];
      f.ok = i < ok.size() && ok[i];
      if (!f.ok) f.body.clear();
    }
  }
  return frames->size() - first;
}

}  // namespace policy
}  // namespace flare::rpc
