// snappy_flat.cc -- see snappy.h.
#include <cstring>

#include "../../include/flare_snappy_gpu.h"
#include "cord_buf.h"
#include "gpu_codec.h"
#include "snappy.h"

namespace flare::snappy {

size_t MaxCompressedLength(size_t n) { return fsg_max_compressed_length(n); }

size_t Compress(const char* input, size_t n, std::string* output) {
  cord_buf in, out;
  in.append(input, n);
  output->clear();
  if (!gpu::SnappyGpuCodec::Instance().Compress(in, &out)) return 0;
  *output = out.to_string();
  return output->size();
}

bool GetUncompressedLength(const char* compressed, size_t n, size_t* result) {
  uint32_t u = 0;
  if (fsg_get_uncompressed_length(compressed, n, &u, /*lenient=*/0) == 0) return false;
  *result = u;
  return true;
}

bool Uncompress(const char* compressed, size_t n, std::string* uncompressed) {
  size_t ulen = 0;
  if (!GetUncompressedLength(compressed, n, &ulen)) return false;
  cord_buf in, out;
  in.append(compressed, n);
  if (!gpu::SnappyGpuCodec::Instance().Uncompress(in, &out)) return false;
  *uncompressed = out.to_string();
  return true;
}

void RawCompress(const char* input, size_t n, char* compressed, size_t* compressed_length) {
  std::string s;
  Compress(input, n, &s);
  memcpy(compressed, s.data(), s.size());
  *compressed_length = s.size();
}

bool RawUncompress(const char* compressed, size_t n, char* uncompressed) {
  cord_buf in, out;
  in.append(compressed, n);
  if (!gpu::SnappyGpuCodec::Instance().Uncompress(in, &out)) return false;
  out.copy_to(uncompressed, out.size());
  return true;
}

bool IsValidCompressedBuffer(const char* compressed, size_t n) {
  cord_buf in, out;
  in.append(compressed, n);
  return gpu::SnappyGpuCodec::Instance().Uncompress(in, &out);
}

}  // namespace flare::snappy
