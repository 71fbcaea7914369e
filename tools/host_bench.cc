// host_bench.cc -- end-to-end rate of the drop-in host path: C3-shaped bodies
// (64 KiB Zipf text, flare-cpp_amd/tools/datagen.c) held as cord_bufs of
// 8160-byte blocks, compressed and then decompressed through
// SnappyGpuCodec::CompressBatch / UncompressBatch (gather into pinned staging,
// H2D, kernels, D2H, append to the output cord_bufs -- the socket -> cord_buf
// -> socket path of BASELINE.json north_star, minus the socket).
//   ./build/host_bench [messages] [size] [reps] [pinned]   (defaults 16384 65536 3 0)
// pinned = 1 installs the pinned block allocator first (fsh_use_pinned_blocks):
// input blocks are then read by the GPU directly and no staging copy is made;
// outputs are adopted from pinned slabs either way (so the compressed
// cord_bufs feed the decompress leg without staging too).
// Prints one JSON line.  Byte-checks every round trip.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cord_buf.h"
#include "gpu_codec.h"

extern "C" void dg_text_body(uint64_t index, uint8_t* out, size_t n);

using flare::cord_buf;

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 16384;
  const size_t size = argc > 2 ? strtoull(argv[2], nullptr, 10) : 65536;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const bool pinned = argc > 4 && atoi(argv[4]) != 0;
  if (pinned && flare::gpu::UsePinnedBlocks() != 0) {
    fprintf(stderr, "pinned blocks unavailable\n");
    return 1;
  }
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  if (!codec.available()) {
    fprintf(stderr, "GPU codec unavailable: %s\n", codec.error().c_str());
    return 1;
  }
  std::vector<cord_buf> raw(n);
  std::string body(size, '\0');
  for (size_t i = 0; i < n; ++i) {
    dg_text_body(0x7E47ull * 1000003ull + i, reinterpret_cast<uint8_t*>(&body[0]), size);
    raw[i].append(body);  // 8160-byte blocks, as from a socket
  }
  std::vector<const cord_buf*> in(n);
  for (size_t i = 0; i < n; ++i) in[i] = &raw[i];
  const double raw_bytes = (double)n * size;
  using clk = std::chrono::steady_clock;
  double best_c = 1e30, best_d = 1e30;
  size_t comp_bytes = 0;
  bool ok_all = true;
  for (int r = 0; r < reps; ++r) {
    std::vector<cord_buf> comp(n), back(n);
    std::vector<cord_buf*> co(n), bo(n);
    std::vector<const cord_buf*> ci(n);
    for (size_t i = 0; i < n; ++i) {
      co[i] = &comp[i];
      bo[i] = &back[i];
      ci[i] = &comp[i];
    }
    std::vector<bool> ok;
    auto t0 = clk::now();
    codec.CompressBatch(in, co, &ok);
    auto t1 = clk::now();
    for (bool b : ok) ok_all = ok_all && b;
    codec.UncompressBatch(ci, bo, &ok);
    auto t2 = clk::now();
    for (bool b : ok) ok_all = ok_all && b;
    comp_bytes = 0;
    for (size_t i = 0; i < n; ++i) {
      comp_bytes += comp[i].size();
      if (r == 0 && !(back[i].size() == raw[i].size() && back[i].to_string() == raw[i].to_string())) ok_all = false;
    }
    best_c = std::min(best_c, std::chrono::duration<double>(t1 - t0).count());
    best_d = std::min(best_d, std::chrono::duration<double>(t2 - t1).count());
  }
  const double gib = 1024.0 * 1024.0 * 1024.0;
  const auto st = codec.stats();
  printf("{\"messages\": %zu, \"size\": %zu, \"ratio\": %.3f, \"compress_gib_s\": %.3f, "
         "\"decompress_gib_s\": %.3f, \"compress_ms\": %.2f, \"decompress_ms\": %.2f, \"round_trip_ok\": %s, "
         "\"pinned_blocks\": %s, \"adopted\": %llu, \"device_messages\": %llu, "
         "\"path\": \"cord_buf (8160-B blocks) -> %s -> kernels -> D2H into pinned slabs -> adopted "
         "(append_user_data), chunked over 3 streams\"}\n",
         n, size, raw_bytes / comp_bytes, raw_bytes / best_c / gib, raw_bytes / best_d / gib, best_c * 1e3,
         best_d * 1e3, ok_all ? "true" : "false", pinned ? "true" : "false", (unsigned long long)st.adopted,
         (unsigned long long)st.messages,
         pinned ? "GPU gather from pinned blocks" : "memcpy into pinned staging + H2D");
  return ok_all ? 0 : 2;
}
