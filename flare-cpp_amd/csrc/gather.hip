// gather.hip -- device-side gather of cord_buf blocks that live in pinned
// host memory (the blockmem_allocate hook, /root/reference/flare/io/
// cord_buf.cc:159-166): the GPU reads the blocks over PCIe itself, so the
// host runtime needs neither a staging memcpy nor one hipMemcpyAsync per
// 8 KiB block (cord_buf.cc:1469-1475 is the reference's per-block walk).
#include "../../include/flare_snappy_gpu.h"
#include "snappy_device.h"

namespace fsg {

// One wave per block: 16-byte loads when source and destination share
// 16-byte alignment (every whole cord_buf block: payload at +32 of an 8 KiB
// allocation, 8160-byte strides), bytes otherwise.
__global__ __launch_bounds__(256) void gather_blocks_kernel(const u64* __restrict__ src,
                                                            const u32* __restrict__ len,
                                                            const u64* __restrict__ dst_off,
                                                            u32 n, u8* __restrict__ dst) {
  const u32 w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const u32 lane = threadIdx.x & 63;
  if (w >= n) return;
  const u8* s = reinterpret_cast<const u8*>(src[w]);
  u8* d = dst + dst_off[w];
  const u32 L = len[w];
  const u32 head = (u32)((16 - (reinterpret_cast<uintptr_t>(s) & 15)) & 15);
  if (((reinterpret_cast<uintptr_t>(s) ^ reinterpret_cast<uintptr_t>(d)) & 15) == 0 && L > head) {
    for (u32 i = lane; i < head; i += 64) d[i] = s[i];
    const u32 body = (L - head) & ~15u;
    for (u32 i = head + 16 * lane; i < head + body; i += 1024)
      *reinterpret_cast<u32x4*>(d + i) = *reinterpret_cast<const u32x4*>(s + i);
    for (u32 i = head + body + lane; i < L; i += 64) d[i] = s[i];
  } else {
    for (u32 i = lane; i < L; i += 64) d[i] = s[i];
  }
}

hipError_t launch_gather_blocks(const u64* src, const u32* len, const u64* dst_off, u32 n, u8* dst,
                                hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const u32 blocks = (n + 3) / 4;  // 4 waves per 256-thread block
  gather_blocks_kernel<<<blocks, 256, 0, stream>>>(src, len, dst_off, n, dst);
  return hipGetLastError();
}

}  // namespace fsg
