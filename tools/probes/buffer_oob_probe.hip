// buffer_oob_probe.hip -- what a raw buffer load returns when it reaches past
// the descriptor's num_records, on gfx950.  The decoders load tag and literal
// bytes through a per-message buffer descriptor instead of clamping every
// 16-byte load by hand; this pins which bytes come back:
//   per dword: a dword entirely below num_records is loaded, one that reaches
//              past it returns 0 (the rest of the access is unaffected), or
//   per access: the whole access returns 0 once any byte is past the end.
// Memory holds byte i = (i * 7 + 1) & 0xff; num_records = 37.  For each
// width (4/8/16 bytes) and byte offset 20..44 it prints the returned bytes.
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/buffer_oob_probe tools/probes/buffer_oob_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32 u32x2 __attribute__((ext_vector_type(2)));

__global__ void probe(const uint8_t* b, u32 nrec, u32* out) {
  const u32 off = 20 + threadIdx.x;  // 0..24 -> offsets 20..44
  if (threadIdx.x >= 25) return;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, (int)nrec, 0x00020000);
  const u32x4 v16 = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  const u32x2 v8 = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  const u32 v4 = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  u32* o = out + threadIdx.x * 8;
  o[0] = v16[0]; o[1] = v16[1]; o[2] = v16[2]; o[3] = v16[3];
  o[4] = v8[0]; o[5] = v8[1]; o[6] = v4; o[7] = 0;
}

int main() {
  uint8_t* b = nullptr;
  u32* out = nullptr;
  uint8_t h[256];
  for (int i = 0; i < 256; ++i) h[i] = (uint8_t)(i * 7 + 1);
  if (hipMalloc(&b, 256) != hipSuccess || hipMalloc(&out, 25 * 8 * 4) != hipSuccess) return 1;
  (void)hipMemcpy(b, h, 256, hipMemcpyHostToDevice);
  const u32 nrec = 37;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, b, nrec, out);
  u32 r[25 * 8];
  if (hipMemcpy(r, out, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int per_dword = 1, per_byte = 1, per_access = 1;
  for (int t = 0; t < 25; ++t) {
    const u32 off = 20 + t;
    const uint8_t* g = reinterpret_cast<const uint8_t*>(r + t * 8);
    printf("off %2u  b128:", off);
    for (int i = 0; i < 16; ++i) printf(" %02x", g[i]);
    printf("  b64:");
    for (int i = 0; i < 8; ++i) printf(" %02x", g[16 + i]);
    printf("  b32:");
    for (int i = 0; i < 4; ++i) printf(" %02x", g[24 + i]);
    printf("\n");
    // classify the 16-byte load
    for (int i = 0; i < 16; ++i) {
      const u32 p = off + i;
      const uint8_t mem = h[p];
      const bool dword_in = off + 4 * (i / 4) + 4 <= nrec;
      const bool byte_in = p < nrec;
      const bool all_in = off + 16 <= nrec;
      if (g[i] != (dword_in ? mem : 0)) per_dword = 0;
      if (g[i] != (byte_in ? mem : 0)) per_byte = 0;
      if (g[i] != (all_in ? mem : 0)) per_access = 0;
    }
  }
  printf("b128 semantics: per_dword=%d per_byte=%d per_access=%d\n", per_dword, per_byte, per_access);
  return 0;
}
