// salu_issue_probe.hip -- how many scalar-ALU instructions a CU issues per
// cycle as the number of waves on it grows (1, 2, 4 = one per SIMD, 8, 16,
// 24), against vector-ALU instructions and a mix of both.  Each wave runs a
// long unrolled chain of independent instructions (8 interleaved
// accumulators); s_memtime brackets the loop; aggregate rate per CU =
// waves x instructions / cycles of the slowest wave.
//
// Question it answers for the decoder's exec pass: is SALU issue
// a per-CU resource (then the pass's 2.8G SALU per launch is near its limit)
// or a per-SIMD one?
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/salu_issue_probe tools/probes/salu_issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kIters = 512;  // per launch of the memtime runs; event runs take a count

enum Mode { SALU, VALU, MIX, MIX2 };
static const char* kNames[] = {"salu", "valu", "salu+valu 1:1", "salu+valu 1:2"};

#define S8(op)                                                         \
  asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t" op \
                  " %3, %3, %8\n\t" op " %4, %4, %8\n\t" op " %5, %5, %8\n\t" op \
                  " %6, %6, %8\n\t" op " %7, %7, %8"                          \
               : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7) \
               : "s"(k) : "scc")
#define V8(op)                                                         \
  asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t" op \
                  " %3, %3, %8\n\t" op " %4, %4, %8\n\t" op " %5, %5, %8\n\t" op \
                  " %6, %6, %8\n\t" op " %7, %7, %8"                          \
               : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
               : "v"(kv))

__device__ __forceinline__ u64 memtime() {
  u64 t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int MODE>
__global__ __launch_bounds__(1024) void probe(u32 k, u64* cycles, u32* out, int iters) {
  u32 s0 = k, s1 = k + 1, s2 = k + 2, s3 = k + 3, s4 = k + 4, s5 = k + 5, s6 = k + 6, s7 = k + 7;
  u32 kv = threadIdx.x + k;
  u32 v0 = kv, v1 = kv + 1, v2 = kv + 2, v3 = kv + 3, v4 = kv + 4, v5 = kv + 5, v6 = kv + 6, v7 = kv + 7;
  __syncthreads();
  const u64 t0 = memtime();
  for (int i = 0; i < iters; ++i) {
    if (MODE == SALU) { S8("s_add_u32"); S8("s_xor_b32"); S8("s_add_u32"); S8("s_xor_b32"); }
    if (MODE == VALU) { V8("v_add_u32"); V8("v_xor_b32"); V8("v_add_u32"); V8("v_xor_b32"); }
    if (MODE == MIX) { S8("s_add_u32"); V8("v_add_u32"); S8("s_xor_b32"); V8("v_xor_b32"); }
    if (MODE == MIX2) { S8("s_add_u32"); V8("v_add_u32"); V8("v_xor_b32"); V8("v_add_u32");
                        S8("s_xor_b32"); V8("v_xor_b32"); }
  }
  const u64 t1 = memtime();
  if ((threadIdx.x & 63) == 0) cycles[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7 ^ v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
}

template <int MODE>
void run(int waves, u64* d_cyc, u32* d_out, u64* h_cyc) {
  const int blocks = 256;
  probe<MODE><<<blocks, waves * 64>>>(3, d_cyc, d_out, kIters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int big = 40 * kIters;
  hipEventRecord(e0);
  probe<MODE><<<blocks, waves * 64>>>(3, d_cyc, d_out, big);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(h_cyc, d_cyc, sizeof(u64) * blocks * 16, hipMemcpyDeviceToHost);
  u64 mx = 0, sum = 0;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < waves; ++w) {
      mx = h_cyc[b * 16 + w] > mx ? h_cyc[b * 16 + w] : mx;
      sum += h_cyc[b * 16 + w];
    }
  const double s_per_wave = MODE == VALU ? 0 : (MODE == MIX2 ? 16.0 : (MODE == MIX ? 16.0 : 32.0)) * kIters;
  const double v_per_wave = MODE == SALU ? 0 : (MODE == MIX2 ? 32.0 : (MODE == MIX ? 16.0 : 32.0)) * kIters;
  const double avg = (double)sum / (blocks * waves) / 40.0;  // per kIters
  // event time -> instructions per ns per CU (2.4 GHz shader clock: / 2.4 per cycle)
  const double ns = ms * 1e6;
  const double s_ns = waves * s_per_wave * 40.0 / ns, v_ns = waves * v_per_wave * 40.0 / ns;
  // cycles: s_memtime ticks (rate checked against events below)
  printf("{\"mode\": \"%s\", \"waves_per_cu\": %d, \"cycles_max\": %llu, \"cycles_avg\": %.0f, "
         "\"event_ms\": %.4f, \"salu_per_cu_ns\": %.3f, \"valu_per_cu_ns\": %.3f, \"memtime_ticks_per_wave_instr\": %.3f}\n",
         kNames[MODE], waves, (unsigned long long)mx, avg, ms, s_ns, v_ns, avg / (s_per_wave + v_per_wave));
}

int main() {
  u64* d_cyc;
  u32* d_out;
  hipMalloc(&d_cyc, sizeof(u64) * 256 * 16);
  hipMalloc(&d_out, sizeof(u32) * 256 * 1024);
  static u64 h_cyc[256 * 16];
  const int ws[] = {1, 2, 4, 8, 16};
  for (int w : ws) run<SALU>(w, d_cyc, d_out, h_cyc);
  for (int w : ws) run<VALU>(w, d_cyc, d_out, h_cyc);
  for (int w : ws) run<MIX>(w, d_cyc, d_out, h_cyc);
  for (int w : ws) run<MIX2>(w, d_cyc, d_out, h_cyc);
  // clock check: one timed launch
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  probe<SALU><<<256, 64>>>(3, d_cyc, d_out, 40 * kIters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(h_cyc, d_cyc, sizeof(u64) * 256 * 16, hipMemcpyDeviceToHost);
  printf("{\"clock_check_ms\": %.4f, \"memtime_cycles\": %llu, \"implied_mhz\": %.0f}\n", ms,
         (unsigned long long)h_cyc[0], h_cyc[0] / (ms * 1e3));
  return 0;
}
