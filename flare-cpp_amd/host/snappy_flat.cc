// snappy_flat.cc -- see snappy.h.  Small inputs run the host codec in place
// (no cord_buf round trip); larger ones go through the batched runtime.
#include <sys/uio.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/flare_snappy_gpu.h"
#include "cord_buf.h"
#include "gpu_codec.h"
#include "snappy.h"
#include "snappy_cpu.h"

namespace flare::snappy {

namespace {
bool on_host(size_t n) {
  auto& c = gpu::SnappyGpuCodec::Instance();
  return n < c.min_gpu_bytes() || !c.available();
}
}  // namespace

size_t MaxCompressedLength(size_t n) { return fsg_max_compressed_length(n); }

size_t Compress(const char* input, size_t n, std::string* output) {
  if (on_host(n)) {
    output->resize(cpu::MaxCompressedLength(n));
    output->resize(cpu::Compress(reinterpret_cast<const uint8_t*>(input), n,
                                 reinterpret_cast<uint8_t*>(&(*output)[0])));
    return output->size();
  }
  cord_buf in, out;
  in.append(input, n);
  output->clear();
  gpu::SnappyGpuCodec::Instance().Compress(in, &out);  // never fails (host codec on device errors)
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
  if (on_host(n)) {
    std::string tmp(ulen, '\0');
    if (!cpu::Uncompress(reinterpret_cast<const uint8_t*>(compressed), n,
                         reinterpret_cast<uint8_t*>(&tmp[0]), ulen, /*strict=*/true))
      return false;
    uncompressed->swap(tmp);
    return true;
  }
  cord_buf in, out;
  in.append(compressed, n);
  if (!gpu::SnappyGpuCodec::Instance().Uncompress(in, &out)) return false;
  *uncompressed = out.to_string();
  return true;
}

void RawCompress(const char* input, size_t n, char* compressed, size_t* compressed_length) {
  if (on_host(n)) {
    *compressed_length = cpu::Compress(reinterpret_cast<const uint8_t*>(input), n,
                                       reinterpret_cast<uint8_t*>(compressed));
    return;
  }
  std::string s;
  Compress(input, n, &s);
  memcpy(compressed, s.data(), s.size());
  *compressed_length = s.size();
}

bool RawUncompress(const char* compressed, size_t n, char* uncompressed) {
  if (on_host(n)) {
    uint32_t ulen = 0;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(compressed);
    const size_t h = cpu::ReadHeader(p, n, &ulen, /*strict=*/false);
    return h != 0 && cpu::Decode(p, n, h, reinterpret_cast<uint8_t*>(uncompressed), ulen);
  }
  cord_buf in, out;
  in.append(compressed, n);
  if (!gpu::SnappyGpuCodec::Instance().Uncompress(in, &out)) return false;
  out.copy_to(uncompressed, out.size());
  return true;
}

bool IsValidCompressedBuffer(const char* compressed, size_t n) {
  if (on_host(n)) return cpu::IsValid(reinterpret_cast<const uint8_t*>(compressed), n);
  cord_buf in;
  in.append(compressed, n);
  return gpu::SnappyGpuCodec::Instance().IsValid(in);  // the device's validate-only pass
}

bool RawUncompressToIOVec(const char* compressed, size_t n, const struct iovec* iov, size_t iov_cnt) {
  // SnappyIOVecWriter (snappy.cc:963-1132): the output must fit the iovecs
  // and match the header length; bytes land in order across them.
  uint32_t ulen = 0;
  if (fsg_get_uncompressed_length(compressed, n, &ulen, /*lenient=*/1) == 0) return false;
  size_t room = 0;
  for (size_t i = 0; i < iov_cnt; ++i) room += iov[i].iov_len;
  // a header longer than any stream of n bytes can produce cannot decode
  if (room < ulen || (uint64_t)ulen > 22ull * n + 64) return false;
  std::string flat(ulen, '\0');
  if (!RawUncompress(compressed, n, &flat[0])) return false;
  size_t pos = 0;
  for (size_t i = 0; i < iov_cnt && pos < ulen; ++i) {
    const size_t k = std::min<size_t>(iov[i].iov_len, ulen - pos);
    memcpy(iov[i].iov_base, flat.data() + pos, k);
    pos += k;
  }
  return true;
}

size_t UncompressAsMuchAsPossible(const cord_buf& compressed, cord_buf* uncompressed) {
  std::vector<const uint8_t*> frag;
  std::vector<size_t> len;
  for (size_t i = 0; i < compressed.backing_block_num(); ++i) {
    std::string_view v = compressed.backing_block(i);
    frag.push_back(reinterpret_cast<const uint8_t*>(v.data()));
    len.push_back(v.size());
  }
  std::vector<uint8_t> out;
  const size_t r = cpu::UncompressAsMuchAsPossible(frag.data(), len.data(), frag.size(), &out);
  uncompressed->append(out.data(), out.size());
  return r;
}

}  // namespace flare::snappy
