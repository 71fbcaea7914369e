// lz4_host_check.hip -- TEST HELPER: runs the GPU LZ4 block codec
// (flare-cpp_amd/csrc/lz4.hip, its __host__ __device__ functions) on the CPU,
// built with AddressSanitizer by tests/test_lz4.py, so an out-of-bounds
// access in the kernels' code shows up without a GPU.  No HIP calls.
//   lz4_host_check c IN OUT   : IN = records [u32 n][n bytes]; OUT = bodies [u32 len][bytes]
//   lz4_host_check d IN OUT   : IN = records [u32 ulen][u32 n][block]; OUT = [i32 ok][ulen bytes if ok]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../flare-cpp_amd/csrc/lz4.hip"

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  FILE* in = fopen(argv[2], "rb");
  FILE* out = fopen(argv[3], "wb");
  if (!in || !out) return 2;
  std::vector<fsg::u8> table(16384);
  for (;;) {
    if (argv[1][0] == 'c') {
      uint32_t n;
      if (!rd(in, &n, 4)) break;
      std::vector<fsg::u8> src(n), dst(n + n / 255 + 16);
      if (n && !rd(in, src.data(), n)) return 3;
      std::fill(table.begin(), table.end(), 0);
      const uint32_t len = fsg::lz4_compress_block(src.data(), n, dst.data(), table.data());
      fwrite(&len, 4, 1, out);
      fwrite(dst.data(), 1, len, out);
    } else {
      uint32_t ulen, n;
      if (!rd(in, &ulen, 4)) break;
      if (!rd(in, &n, 4)) return 3;
      std::vector<fsg::u8> src(n), dst(ulen);
      if (n && !rd(in, src.data(), n)) return 3;
      const int32_t ok = fsg::lz4_decompress_block(src.data(), n, dst.data(), ulen) ? 1 : 0;
      fwrite(&ok, 4, 1, out);
      if (ok) fwrite(dst.data(), 1, ulen, out);
    }
  }
  fclose(out);
  return 0;
}
