// lz4_compress.cc -- policy::Lz4{Compress,Decompress} (see lz4_compress.h).
#include "lz4_compress.h"

#include <cstdio>
#include <mutex>
#include <vector>

#include "lz4_cpu.h"

namespace flare::rpc::policy {

bool Lz4Compress(const cord_buf& in, cord_buf* out) {
  const size_t n = in.size();
  if (n > lz4::cpu::kMaxInput) return false;
  std::vector<uint8_t> src(n);
  in.copy_to(src.data(), n);
  std::vector<uint8_t> body(lz4::cpu::MaxCompressedLength(n));
  const size_t len = lz4::cpu::Compress(src.data(), n, body.data());
  return len != 0 && out->append(body.data(), len) == 0;
}

bool Lz4Decompress(const cord_buf& in, cord_buf* out) {
  const size_t n = in.size();
  std::vector<uint8_t> body(n);
  in.copy_to(body.data(), n);
  uint32_t ulen = 0;
  const size_t h = lz4::cpu::ReadHeader(body.data(), n, &ulen);
  // the header comes from the peer: bound it by what the block can hold
  // before allocating (a 5-byte body may claim 4 GiB)
  if (h == 0 || !lz4::cpu::PlausibleLength(ulen, n - h)) return false;
  std::vector<uint8_t> raw(ulen);
  if (!lz4::cpu::DecompressBlock(body.data() + h, n - h, raw.data(), ulen)) return false;
  return out->append(raw.data(), ulen) == 0;
}

bool Lz4Compress(const Message& res, cord_buf* buf) {
  cord_buf serialized_pb;
  if (res.SerializeToCordBuf(&serialized_pb)) return Lz4Compress(serialized_pb, buf);
  fprintf(stderr, "[WARNING] Fail to serialize input pb=%p\n", (const void*)&res);
  return false;
}

bool Lz4Decompress(const cord_buf& data, Message* req) {
  cord_buf binary_pb;
  if (Lz4Decompress(data, &binary_pb)) return req->ParseFromCordBuf(binary_pb);
  fprintf(stderr, "[WARNING] Fail to lz4 decompress, size=%zu\n", data.size());
  return false;
}

}  // namespace flare::rpc::policy

namespace flare::rpc {

int GlobalInitializeLz4() {
  static std::once_flag once;
  static int rc = -1;
  std::call_once(once, [] {
    rc = RegisterCompressHandler(COMPRESS_TYPE_LZ4,
                                 CompressHandler{policy::Lz4Compress, policy::Lz4Decompress, "lz4"});
  });
  return rc;
}

}  // namespace flare::rpc
