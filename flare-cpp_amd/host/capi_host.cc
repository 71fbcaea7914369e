// capi_host.cc -- extern "C" surface of libflare_rpc_snappy.so
// (include/flare_snappy_host.h).
#include <cstring>
#include <vector>

#include "../../include/flare_snappy_host.h"
#include "gpu_codec.h"
#include "lz4_compress.h"
#include "lz4_cpu.h"
#include "snappy.h"
#include "snappy_cpu.h"

using flare::gpu::SnappyGpuCodec;

extern "C" {

int fsh_init_devices(uint64_t device_mask) { return SnappyGpuCodec::Instance().InitDevices(device_mask); }

void fsh_shutdown(void) { SnappyGpuCodec::Instance().Shutdown(); }

void fsh_set_gpu_min_bytes(size_t bytes) { SnappyGpuCodec::Instance().SetMinGpuBytes(bytes); }

void fsh_stats(uint64_t* out, size_t n) {
  const auto s = SnappyGpuCodec::Instance().stats();
  const uint64_t v[6] = {s.batches, s.messages, s.cpu_messages, s.fallbacks, s.failures, s.adopted};
  for (size_t i = 0; i < n && i < 6; ++i) out[i] = v[i];
}

void fsh_set_park_hooks(const fsh_park_hooks* hooks) {
  flare::gpu::ParkHooks h;
  if (hooks) {
    h.create = hooks->create;
    h.wait = hooks->wait;
    h.signal = hooks->signal;
    h.destroy = hooks->destroy;
  }
  SnappyGpuCodec::Instance().SetParkHooks(h);
}

int fsh_use_pinned_blocks(void) { return flare::gpu::UsePinnedBlocks(); }

size_t fsh_compress(const char* in, size_t n, char* out) {
  size_t r = 0;
  flare::snappy::RawCompress(in, n, out, &r);
  return r;
}

int fsh_raw_uncompress(const char* in, size_t n, char* out) {
  return flare::snappy::RawUncompress(in, n, out) ? 1 : 0;
}

int fsh_get_uncompressed_length(const char* in, size_t n, size_t* result) {
  return flare::snappy::GetUncompressedLength(in, n, result) ? 1 : 0;
}

int fsh_is_valid_compressed_buffer(const char* in, size_t n) {
  return flare::snappy::IsValidCompressedBuffer(in, n) ? 1 : 0;
}

size_t fsh_max_compressed_length(size_t n) { return flare::snappy::MaxCompressedLength(n); }

size_t fsh_cpu_compress(const uint8_t* in, size_t n, uint8_t* out) { return flare::snappy::cpu::Compress(in, n, out); }

int fsh_cpu_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int strict) {
  return flare::snappy::cpu::Uncompress(in, n, out, cap, strict != 0) ? 1 : 0;
}

int fsh_cpu_is_valid(const uint8_t* in, size_t n) { return flare::snappy::cpu::IsValid(in, n) ? 1 : 0; }

size_t fsh_cpu_uncompress_as_much(const uint8_t* in, size_t n, size_t frag, uint8_t* out, size_t cap,
                                  size_t* got) {
  std::vector<const uint8_t*> fp;
  std::vector<size_t> fl;
  if (frag == 0) frag = n ? n : 1;
  for (size_t p = 0; p < n; p += frag) {
    fp.push_back(in + p);
    fl.push_back(n - p < frag ? n - p : frag);
  }
  std::vector<uint8_t> o;
  const size_t r = flare::snappy::cpu::UncompressAsMuchAsPossible(fp.data(), fl.data(), fp.size(), &o);
  const size_t k = o.size() < cap ? o.size() : cap;
  if (k) memcpy(out, o.data(), k);
  *got = k;
  return r;
}

size_t fsh_lz4_max_compressed_length(size_t n) { return flare::lz4::cpu::MaxCompressedLength(n); }

size_t fsh_cpu_lz4_compress(const uint8_t* in, size_t n, uint8_t* out) { return flare::lz4::cpu::Compress(in, n, out); }

int fsh_cpu_lz4_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, uint32_t* ulen) {
  *ulen = 0;
  const size_t h = flare::lz4::cpu::ReadHeader(in, n, ulen);
  if (h == 0) return -1;
  if (*ulen > cap) return -2;
  if (!flare::lz4::cpu::PlausibleLength(*ulen, n - h)) return 0;
  return flare::lz4::cpu::DecompressBlock(in + h, n - h, out, *ulen) ? 1 : 0;
}

int fsh_register_lz4(void) { return flare::rpc::GlobalInitializeLz4(); }

}  // extern "C"
