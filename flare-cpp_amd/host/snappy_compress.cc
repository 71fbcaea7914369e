// snappy_compress.cc -- GPU-backed policy::Snappy{Compress,Decompress}.
// Control flow and logging follow /root/reference/flare/rpc/policy/
// snappy_compress.cc:28-61; the codec call is the batched GPU runtime.
#include "snappy_compress.h"

#include <cstdio>
#include <mutex>

#include "gpu_codec.h"

namespace flare::rpc::policy {

bool SnappyCompress(const Message& res, cord_buf* buf) {
  cord_buf serialized_pb;
  if (res.SerializeToCordBuf(&serialized_pb)) {
    return gpu::SnappyGpuCodec::Instance().Compress(serialized_pb, buf);
  }
  fprintf(stderr, "[WARNING] Fail to serialize input pb=%p\n", (const void*)&res);
  return false;
}

bool SnappyDecompress(const cord_buf& data, Message* req) {
  cord_buf binary_pb;
  if (gpu::SnappyGpuCodec::Instance().Uncompress(data, &binary_pb)) {
    return req->ParseFromCordBuf(binary_pb);
  }
  fprintf(stderr, "[WARNING] Fail to snappy::Uncompress, size=%zu\n", data.size());
  return false;
}

bool SnappyCompress(const cord_buf& in, cord_buf* out) {
  return gpu::SnappyGpuCodec::Instance().Compress(in, out);
}

bool SnappyDecompress(const cord_buf& in, cord_buf* out) {
  return gpu::SnappyGpuCodec::Instance().Uncompress(in, out);
}

}  // namespace flare::rpc::policy

namespace flare::rpc {

int GlobalInitializeSnappyGpu() {
  static std::once_flag once;
  static int rc = -1;
  std::call_once(once, [] {
    rc = RegisterCompressHandler(COMPRESS_TYPE_SNAPPY,
                                 CompressHandler{policy::SnappyCompress, policy::SnappyDecompress,
                                                 "snappy"});
  });
  return rc;
}

}  // namespace flare::rpc
