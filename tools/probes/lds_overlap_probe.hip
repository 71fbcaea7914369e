// lds_overlap_probe.hip -- which lane's bytes survive when the lanes of ONE
// ds_write_b128 write overlapping, unaligned 16-byte ranges of LDS?
//
// Model under test: for every byte, the highest ACTIVE lane whose range
// covers it wins.  Each trial (one wave) writes 64 ranges, reads the LDS
// back, and the host compares against the model.  Layouts: "pieces"
// (increasing starts, gaps 1..16: what the decoder's piece stores look
// like), "random" (any start in [0, 1024)), and both with ~1/4 of the lanes
// masked off.
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/lds_overlap_probe tools/probes/lds_overlap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBuf = 1200;

__global__ __launch_bounds__(64) void probe(const u32* __restrict__ addr, const u32* __restrict__ act,
                                            uint8_t* __restrict__ out, int wide) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kBuf + 32];
  const u32 lane = threadIdx.x;
  const u32 t = blockIdx.x;
  for (u32 i = lane; i < (kBuf + 32) / 4; i += 64) reinterpret_cast<u32*>(buf)[i] = 0xffffffffu;
  __syncthreads();
  const u32 a = addr[t * 64 + lane];
  u32x4 v;
  for (int k = 0; k < 4; ++k) {
    u32 w = 0;
    for (int b = 0; b < 4; ++b) w |= ((lane | ((u32)((4 * k + b) & 3) << 6)) & 0xffu) << (8 * b);
    v[k] = w;
  }
  if (act[t * 64 + lane]) {
    if (wide == 16) __builtin_memcpy(buf + a, &v, 16);
    else if (wide == 8) { uint64_t x = (uint64_t)v[0] | ((uint64_t)v[1] << 32); __builtin_memcpy(buf + a, &x, 8); }
    else if (wide == 4) *reinterpret_cast<u32*>(buf + a) = v[0];
    else if (wide == 2) *reinterpret_cast<unsigned short*>(buf + a) = (unsigned short)v[0];
  }
  __syncthreads();
  for (u32 i = lane; i < kBuf; i += 64) out[(size_t)t * kBuf + i] = buf[i];
}

static uint64_t s = 0x1234567;
static u32 rnd() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (u32)s; }

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 20000;
  const char* names[4] = {"pieces", "random", "pieces+mask", "random+mask"};
  for (int wide : {16, 8, 4, 2}) {
    for (int kind = 0; kind < 4; ++kind) {
      std::vector<u32> A((size_t)trials * 64), M((size_t)trials * 64);
      for (int t = 0; t < trials; ++t) {
        u32 p = rnd() % 16;
        for (int l = 0; l < 64; ++l) {
          u32 a;
          if (kind % 2 == 0 && wide < 8) { a = (rnd() % 24) * wide; }
          else if (kind % 2 == 0) { a = p; p += 1 + rnd() % 16; if (p > kBuf - 16) p = kBuf - 16; }
          else a = wide >= 8 ? rnd() % (kBuf - 16) : (rnd() % 48) * wide;  // narrow: force collisions
          A[(size_t)t * 64 + l] = a;
          M[(size_t)t * 64 + l] = kind >= 2 ? (rnd() % 4 != 0) : 1;
        }
      }
      u32 *dA, *dM;
      uint8_t* dO;
      hipMalloc(&dA, A.size() * 4);
      hipMalloc(&dM, M.size() * 4);
      hipMalloc(&dO, (size_t)trials * kBuf);
      hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dM, M.data(), M.size() * 4, hipMemcpyHostToDevice);
      probe<<<trials, 64>>>(dA, dM, dO, wide);
      std::vector<uint8_t> O((size_t)trials * kBuf);
      if (hipMemcpy(O.data(), dO, O.size(), hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 1; }
      size_t bad_bytes = 0, bad_trials = 0, bad_lowwins = 0;
      for (int t = 0; t < trials; ++t) {
        bool tb = false;
        for (int i = 0; i < kBuf; ++i) {
          int win = -1, k = 0;
          for (int l = 63; l >= 0; --l) {
            const u32 a = A[(size_t)t * 64 + l];
            if (M[(size_t)t * 64 + l] && (u32)i >= a && (u32)i < a + (u32)wide) { win = l; k = i - a; break; }
          }
          const uint8_t want = win < 0 ? 0xff : (uint8_t)(win | ((k & 3) << 6));
          const uint8_t got = O[(size_t)t * kBuf + i];
          if (got != want) {
            ++bad_bytes; tb = true;
            if (win >= 0 && (got & 63) < win) ++bad_lowwins;
          }
        }
        bad_trials += tb;
      }
      printf("b%d %-12s trials %d  bad_trials %zu  bad_bytes %zu (lower lane won: %zu)\n", wide * 8, names[kind],
             trials, bad_trials, bad_bytes, bad_lowwins);
      hipFree(dA); hipFree(dM); hipFree(dO);
    }
  }
  return 0;
}
