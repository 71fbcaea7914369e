// fetch_probe.hip -- calibrates rocprofv3 FETCH_SIZE against known byte
// counts for the access patterns of the decode passes (MI355X_MICROARCH.md:
// "Other access widths are uncalibrated: calibrate on a known byte count in
// your own access pattern").  Run under `rocprofv3 --pmc FETCH_SIZE` and
// divide each kernel's FETCH_SIZE by the bytes printed here.
//
//   stream16   every lane loads 16 B, consecutive lanes consecutive (1 GiB)
//   rand_line  every lane loads 16 B at the start of a random 128-B line
//              of a 4 GiB buffer (one line per load; 2^24 loads)
//   rand_off   as rand_line, at a random 16-B-aligned offset in the line
//   rand_any   16 B at a random byte offset (a load may span two lines)
//   far_*      the exec pass's far-copy load itself: a 16-B buffer load with
//              sc1 (far_load, csrc/snappy_decode_v4.hip) at a random byte
//              offset, 2^24 loads, from a buffer left resident by a warm-up
//              kernel that every XCD runs over the whole buffer:
//              far_l2 (1 MiB: resident in every XCD's 4 MB L2), far_mall
//              (96 MiB: past the L2s, inside the 256 MiB Infinity Cache),
//              far_hbm (4 GiB, not resident)
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/fetch_probe tools/probes/fetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u64 mix(u64 z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void stream16(const u32x4* __restrict__ b, u64 n16, u32* sink) {
  u32 acc = 0;
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x) {
    const u32x4 v = b[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE>
__global__ void rand_load(const uint8_t* __restrict__ b, u64 bytes, u64 n, u32* sink) {
  u32 acc = 0;
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 r = mix(i * 0x9E3779B97F4A7C15ull + 12345);
    const u64 line = (r % (bytes / 128 - 1)) * 128;
    u64 off = line;
    if (MODE == 1) off += ((r >> 40) & 7) * 16;
    if (MODE == 2) off += (r >> 40) & 127;
    u32x4 v;
    __builtin_memcpy(&v, b + off, 16);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void warm(const u32x4* __restrict__ b, u64 n16, u32* sink) {
  // every workgroup reads the whole buffer: each XCD's L2 holds all of it
  u32 acc = 0;
  for (u64 i = threadIdx.x; i < n16; i += blockDim.x) {
    const u32x4 v = b[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int KIND>
__global__ void far_rand(const uint8_t* __restrict__ b, u64 bytes, u64 n, u32* sink) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(b), (short)0, (int)(bytes < 0x7fffffffull ? bytes : 0x7fffffffull), 0x00020000);
  u32 acc = 0;
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 x = mix(i * 0x9E3779B97F4A7C15ull + 777 + KIND);
    const u32 off = (u32)(x % ((bytes < 0x7fffffffull ? bytes : 0x7fffffffull) - 16));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);  // sc1, as far_load
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const u64 bytes = 4ull << 30;
  uint8_t* b = nullptr;
  u32* sink = nullptr;
  if (hipMalloc(&b, bytes + 256) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  (void)hipMemset(b, 1, bytes + 256);
  (void)hipDeviceSynchronize();
  const u64 n16 = (1ull << 30) / 16, n = 1ull << 24;
  stream16<<<4096, 256>>>(reinterpret_cast<const u32x4*>(b), n16, sink);
  (void)hipMemset(b, 2, 512ull << 20);  // evict
  rand_load<0><<<4096, 256>>>(b, bytes, n, sink);
  (void)hipMemset(b, 3, 512ull << 20);
  rand_load<1><<<4096, 256>>>(b, bytes, n, sink);
  (void)hipMemset(b, 4, 512ull << 20);
  rand_load<2><<<4096, 256>>>(b, bytes, n, sink);
  // far loads, L2-resident / Infinity-Cache-resident / not resident
  const u64 l2b = 1ull << 20, mallb = 96ull << 20;
  warm<<<256, 256>>>(reinterpret_cast<const u32x4*>(b), l2b / 16, sink);
  far_rand<0><<<4096, 256>>>(b, l2b, n, sink);
  warm<<<256, 256>>>(reinterpret_cast<const u32x4*>(b), l2b / 16, sink);
  far_rand<0><<<4096, 256>>>(b, l2b, n, sink);
  (void)hipMemset(b, 5, 512ull << 20);
  warm<<<8, 1024>>>(reinterpret_cast<const u32x4*>(b), mallb / 16, sink);
  far_rand<1><<<4096, 256>>>(b, mallb, n, sink);
  far_rand<1><<<4096, 256>>>(b, mallb, n, sink);
  (void)hipMemset(b, 6, 1024ull << 20);
  far_rand<2><<<4096, 256>>>(b, 2ull << 30, n, sink);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("stream16 bytes=%llu\n", (unsigned long long)(n16 * 16));
  printf("far_rand<0> (1 MiB, L2) / <1> (96 MiB, Infinity Cache) / <2> (2 GiB) loads=%llu each, 16 B at a random "
         "byte offset (sc1 buffer load)\n", (unsigned long long)n);
  printf("rand_line/rand_off/rand_any loads=%llu bytes_requested=%llu lines=%llu (x128 B = %llu)\n",
         (unsigned long long)n, (unsigned long long)(n * 16), (unsigned long long)n,
         (unsigned long long)(n * 128));
  (void)hipFree(b);
  (void)hipFree(sink);
  return 0;
}
