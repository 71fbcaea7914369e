// lds_resident_probe.hip -- how many one-wave workgroups with L bytes of
// dynamic LDS are resident on one CU at once, on gfx950.  The wave encoder
// (csrc/snappy_encode_wave.hip) sizes its launch as 160 KiB / table bytes
// per CU; with 32 KiB tables that is 5, but a launch capped at 4 per CU ran
// in the same time.  Each wave records its CU (HW_ID, XCC_ID), its SIMD, and
// its start and end on the constant 100 MHz clock while it spins ~200 us;
// the host prints, per LDS size, the largest number of waves whose intervals
// overlap on one CU.
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/lds_resident_probe tools/probes/lds_resident_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;

__global__ void probe(u32* out, u32 lds_words) {
  extern __shared__ u32 s[];
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  // touch the allocation (first and last word) so it cannot be elided
  if (lds_words) {
    s[threadIdx.x % lds_words] = threadIdx.x;
    s[lds_words - 1 - (threadIdx.x % lds_words)] += 1;
  }
  u64 t = t0;
  while (t - t0 < 20000) t = __builtin_amdgcn_s_memrealtime();  // ~200 us
  const u32 hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
  const u32 xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  if (threadIdx.x == 0) {
    u32* o = out + 8 * blockIdx.x;
    o[0] = (u32)t0;
    o[1] = (u32)(t0 >> 32);
    o[2] = (u32)t;
    o[3] = (u32)(t >> 32);
    o[4] = hw;
    o[5] = xcc;
    o[6] = lds_words ? s[0] : 0u;
  }
}

int main() {
  const int blocks = 256 * 8;
  u32* d = nullptr;
  if (hipMalloc(&d, (size_t)blocks * 32) != hipSuccess) return 1;
  std::vector<u32> h((size_t)blocks * 8);
  const u32 sizes[] = {0, 16384, 30720, 31744, 32256, 32768, 40960, 53248, 65536};
  for (u32 L : sizes) {
    hipMemset(d, 0, (size_t)blocks * 32);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), L, 0, d, L / 4);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed for L=%u\n", L); return 1; }
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // per CU: intervals, max overlap; SIMD ids seen
    std::map<u64, std::vector<std::pair<u64, int>>> ev;
    std::map<u64, u32> simds;
    for (int b = 0; b < blocks; ++b) {
      const u32* o = &h[(size_t)b * 8];
      const u64 s0 = (u64)o[1] << 32 | o[0], s1 = (u64)o[3] << 32 | o[2];
      const u32 hw = o[4], xcc = o[5] & 0xf;
      const u64 cu = (u64)xcc << 16 | ((hw >> 8) & 0xff);  // cu_id, sh_id, se_id
      ev[cu].push_back({s0, +1});
      ev[cu].push_back({s1, -1});
      simds[cu] |= 1u << ((hw >> 4) & 3);
    }
    std::map<int, int> hist;
    for (auto& [cu, v] : ev) {
      std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
      int cur = 0, mx = 0;
      for (auto& e : v) { cur += e.second; mx = std::max(mx, cur); }
      hist[mx]++;
    }
    printf("L=%6u B: %zu CUs seen; max resident waves per CU:", L, ev.size());
    for (auto& [k, n] : hist) printf("  %d x%d", k, n);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
