// compress.h -- flare's CompressType plugin surface, restated without
// protobuf (the C++ protobuf runtime is not available in this build).
//
// Mirrors /root/reference/flare/rpc/compress.h:28-61 and compress.cc:26-103:
// a static table of 1024 handlers indexed by CompressType, registration that
// is NOT thread-safe and FATAL on double registration, and the two helpers the
// protocols call (ParseFromCompressedData / SerializeAsCompressedData).
// `Message` stands in for google::protobuf::Message: anything that can
// serialize into / parse from a cord_buf.
#pragma once

#include <vector>

#include "cord_buf.h"

namespace flare::rpc {

// flare/rpc/options.proto:69-75 (wire-visible values).
enum CompressType {
  COMPRESS_TYPE_NONE = 0,
  COMPRESS_TYPE_SNAPPY = 1,
  COMPRESS_TYPE_GZIP = 2,
  COMPRESS_TYPE_ZLIB = 3,
  COMPRESS_TYPE_LZ4 = 4,
};

// Minimal protobuf::Message stand-in (SerializeToZeroCopyStream /
// ParsePbFromCordBuf roles, flare/rpc/protocol.cc:223-226).
class Message {
 public:
  virtual ~Message() = default;
  virtual bool SerializeToCordBuf(cord_buf* out) const = 0;
  virtual bool ParseFromCordBuf(const cord_buf& in) = 0;
};

struct CompressHandler {
  // Compress serialized `msg' into `buf'.  Returns true on success.
  bool (*Compress)(const Message& msg, cord_buf* buf);
  // Parse decompressed `data' as `msg'.  Returns true on success.
  bool (*Decompress)(const cord_buf& data, Message* msg);
  // Name of the compression algorithm, must be a string constant.
  const char* name;
};

// [NOT thread-safe] Register `handler' using key=`type'.  Returns 0 on
// success, -1 otherwise (null functions, out-of-range type, or type already
// registered -- the reference logs FATAL for all three, compress.cc:29-46).
int RegisterCompressHandler(CompressType type, CompressHandler handler);

// Returns the handler for `type`, or nullptr.
const CompressHandler* FindCompressHandler(CompressType type);

// "none" for NONE, the handler name if registered, "unknown" otherwise.
const char* CompressTypeToCStr(CompressType type);

// Put all registered handlers into `vec'.
void ListCompressHandler(std::vector<CompressHandler>* vec);

// Parse decompressed `data' as `msg' using registered `compress_type'.
bool ParseFromCompressedData(const cord_buf& data, Message* msg, CompressType compress_type);

// Compress serialized `msg' into `buf' using registered `compress_type'.
bool SerializeAsCompressedData(const Message& msg, cord_buf* buf, CompressType compress_type);

// Test hook (the reference's tests run with -Dprivate=public): forget every
// registration so a test can exercise registration from a clean table.
void ResetCompressHandlersForTesting();

}  // namespace flare::rpc
