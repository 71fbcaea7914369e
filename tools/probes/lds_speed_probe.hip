// lds_speed_probe.hip -- cycles per LDS wave-instruction by instruction,
// address alignment and active lanes.  4 waves per CU (one per SIMD, one
// 256-thread workgroup per CU, 256 workgroups), each wave issuing a long
// unrolled chain of independent LDS instructions; s_memtime around the loop,
// averaged over waves.  With 4 waves sharing the CU's LDS, cycles/4 is the
// LDS's own time per instruction.
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/lds_speed_probe tools/probes/lds_speed_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 256;

enum Op { W128, W64, W32, W16, W8, R128, R64, R32, OR32, OR64, BPERM };
static const char* kNames[] = {"write_b128", "write_b64", "write_b32", "write_b16", "write_b8",
                               "read_b128",  "read_b64",  "read_b32",  "or_b32",    "or_b64",
                               "bpermute"};

template <int OP>
__global__ __launch_bounds__(256) void probe(u32 mis, u32 active, u32 stride, u64* out, u32* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4][64 * 24 + 64];
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* b = buf[wv];
  const u32 a = lane * stride + mis;
  u32x4 v = {lane, lane + 1, lane + 2, lane + 3};
  u32x4 acc = {0, 0, 0, 0};
  __syncthreads();
  const u64 t0 = __builtin_amdgcn_s_memtime();
  if (lane < active) {
#pragma unroll 16
    for (int i = 0; i < kIters; ++i) {
      if (OP == R128) { u32x4 x; __builtin_memcpy(&x, b + a, 16); acc += x; }
      if (OP == R64) { u64 x; __builtin_memcpy(&x, b + a, 8); acc.x += (u32)x; acc.y += (u32)(x >> 32); }
      if (OP == R32) { u32 x; __builtin_memcpy(&x, b + a, 4); acc.x += x; }
      if (OP == W128) __builtin_memcpy(b + a, &v, 16);
      if (OP == W64) { u64 x = ((u64)v[1] << 32) | v[0]; __builtin_memcpy(b + a, &x, 8); }
      if (OP == W32) { const u32 x = v[0]; __builtin_memcpy(b + a, &x, 4); }
      if (OP == W16) { const unsigned short x = (unsigned short)v[0]; __builtin_memcpy(b + a, &x, 2); }
      if (OP == W8) { b[a] = (uint8_t)v[0]; }
      if (OP == OR32) __hip_atomic_fetch_or(reinterpret_cast<u32*>(b + a), v[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (OP == OR64) __hip_atomic_fetch_or(reinterpret_cast<u64*>(b + a), (u64)v[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (OP == BPERM) acc.x += (u32)__builtin_amdgcn_ds_bpermute((int)(4 * ((lane + i) & 63)), (int)v[0]);
      v.x += 1;
      __builtin_amdgcn_wave_barrier();
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  const u64 t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 4 + wv] = t1 - t0;
  if (acc.x == 12345) sink[0] = acc.y;
}

template <int OP>
static void run(u32 mis, u32 active, u32 stride, u64* d, u32* sink) {
  const int blocks = 256;
  probe<OP><<<blocks, 256>>>(mis, active, stride, d, sink);
  u64 h[blocks * 4];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks * 4; ++i) s += (double)h[i];
  printf("%-10s stride %2u mis %2u active %2u : %6.1f cycles/instr/wave\n", kNames[OP], stride, mis, active,
         s / (blocks * 4) / kIters);
}

int main() {
  u64* d;
  u32* sink;
  (void)hipMalloc(&d, 256 * 4 * sizeof(u64));
  (void)hipMalloc(&sink, 64);
  for (u32 act : {64u, 16u}) {
    // aligned, natural stride
    run<W8>(0, act, 1, d, sink);
    run<W8>(0, act, 16, d, sink);
    run<W16>(0, act, 2, d, sink);
    run<W16>(1, act, 2, d, sink);
    run<W32>(0, act, 4, d, sink);
    run<W64>(0, act, 8, d, sink);
    run<R32>(0, act, 4, d, sink);
    run<R32>(1, act, 4, d, sink);
    run<R64>(0, act, 8, d, sink);
    run<R64>(0, act, 16, d, sink);
    run<R64>(4, act, 8, d, sink);
    run<R128>(0, act, 16, d, sink);
    run<OR32>(0, act, 4, d, sink);
    run<OR32>(0, act, 16, d, sink);
    run<OR64>(0, act, 8, d, sink);
    run<OR64>(0, act, 16, d, sink);
    run<BPERM>(0, act, 4, d, sink);
    // random-ish piece starts: stride 7 / 9, byte offsets
    run<R128>(0, act, 7, d, sink);
    run<W128>(0, act, 7, d, sink);
    run<R64>(0, act, 7, d, sink);
  }
  return 0;
}
