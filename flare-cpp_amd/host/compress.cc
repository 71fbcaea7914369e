// compress.cc -- handler registry; behaviour follows
// /root/reference/flare/rpc/compress.cc:26-103.
#include "compress.h"

#include <cstdio>

namespace flare::rpc {

namespace {
constexpr int kMaxHandlerSize = 1024;  // compress.cc:26
CompressHandler s_handler_map[kMaxHandlerSize] = {};

void log_fatal(const char* what, int type) {
  // The reference uses FLARE_LOG(FATAL); a library cannot abort its host, so
  // the message is printed and -1 returned.
  fprintf(stderr, "[FATAL] CompressType=%d %s\n", type, what);
}
}  // namespace

int RegisterCompressHandler(CompressType type, CompressHandler handler) {
  if (handler.Compress == nullptr || handler.Decompress == nullptr) {
    log_fatal("Invalid parameter: handler function is NULL", (int)type);
    return -1;
  }
  const int index = type;
  if (index < 0 || index >= kMaxHandlerSize) {
    log_fatal("is out of range", index);
    return -1;
  }
  if (s_handler_map[index].Compress != nullptr) {
    log_fatal("was registered", index);
    return -1;
  }
  s_handler_map[index] = handler;
  return 0;
}

const CompressHandler* FindCompressHandler(CompressType type) {
  const int index = type;
  if (index < 0 || index >= kMaxHandlerSize) {
    fprintf(stderr, "[ERROR] CompressType=%d is out of range\n", index);
    return nullptr;
  }
  if (s_handler_map[index].Compress == nullptr) return nullptr;
  return &s_handler_map[index];
}

const char* CompressTypeToCStr(CompressType type) {
  if (type == COMPRESS_TYPE_NONE) return "none";
  const CompressHandler* h = FindCompressHandler(type);
  return h != nullptr ? h->name : "unknown";
}

void ListCompressHandler(std::vector<CompressHandler>* vec) {
  vec->clear();
  for (int i = 0; i < kMaxHandlerSize; ++i)
    if (s_handler_map[i].Compress != nullptr) vec->push_back(s_handler_map[i]);
}

bool ParseFromCompressedData(const cord_buf& data, Message* msg, CompressType compress_type) {
  if (compress_type == COMPRESS_TYPE_NONE) return msg->ParseFromCordBuf(data);
  const CompressHandler* h = FindCompressHandler(compress_type);
  return h != nullptr ? h->Decompress(data, msg) : false;
}

bool SerializeAsCompressedData(const Message& msg, cord_buf* buf, CompressType compress_type) {
  if (compress_type == COMPRESS_TYPE_NONE) return msg.SerializeToCordBuf(buf);
  const CompressHandler* h = FindCompressHandler(compress_type);
  return h != nullptr ? h->Compress(msg, buf) : false;
}

void ResetCompressHandlersForTesting() {
  for (auto& h : s_handler_map) h = CompressHandler{};
}

}  // namespace flare::rpc
