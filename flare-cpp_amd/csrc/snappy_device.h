// snappy_device.h -- device-side constants and helpers shared by the gfx950
// Snappy kernels.  Format constants follow the reference's vendored Snappy
// 1.1.3 (/root/reference/flare/io/snappy/).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsg {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int32_t i32;
typedef int64_t i64;

constexpr u32 kBlockLog = 16;                    // snappy.h:201
constexpr u32 kBlockSize = 1u << kBlockLog;      // snappy.h:202
constexpr u32 kMaxHashTableBits = 14;            // snappy.h:204
constexpr u32 kMaxHashTableSize = 1u << kMaxHashTableBits;  // snappy.h:205
constexpr u32 kInputMarginBytes = 15;            // snappy.cc:346
constexpr u32 kHashMul = 0x1e35a7bdu;            // snappy.cc:47
constexpr int kWave = 64;                        // CDNA wavefront

// Status words (mirrors include/flare_snappy_gpu.h).
constexpr i32 kOk = 0;
constexpr i32 kCorrupt = 1;
constexpr i32 kBadHeader = 2;
constexpr i32 kSlotTooSmall = 3;
// Internal: message not indexed by the two-pass decoder (its bitmap did not
// fit the workspace); finished by v4's fallback_kernel (one lane, serial tag
// loop), or by the v3 kernel under kFlagFallbackOnly.
constexpr i32 kNeedFallback = 0x40000000;
constexpr u32 kFlagFallbackOnly = 0x80000000u;
// Internal: a large message left by the lane-per-message index pass for the
// wave-per-message one (decode v4), which writes its final status.
constexpr i32 kNeedBigIndex = 0x20000000;
// Internal: listed by the decode v4 plan pass for the lane walk.
constexpr i32 kNeedLaneWalk = 0x10000000;

__host__ __device__ inline u64 max_compressed_length(u64 n) {
  return 32 + n + n / 6;  // snappy.cc:55-77
}

// WorkingMemory::GetHashTable sizing, snappy.cc:247-271.
__host__ __device__ inline u32 table_size_for(u32 frag_len) {
  u32 ht = 256;
  while (ht < kMaxHashTableSize && ht < frag_len) ht <<= 1;
  return ht;
}

__host__ __device__ inline int varint32_len(u32 v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3
       : v < (1u << 28) ? 4 : 5;
}

// Unaligned little-endian loads/stores on global memory.  gfx950 runs in
// unaligned-access mode, so these lower to single dword/dwordx2/dwordx4 ops.
__device__ __forceinline__ u32 ldu32(const u8* p) {
  u32 v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
__device__ __forceinline__ u64 ldu64(const u8* p) {
  u64 v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__device__ __forceinline__ void stu64(u8* p, u64 v) { __builtin_memcpy(p, &v, 8); }
__device__ __forceinline__ void stu32(u8* p, u32 v) { __builtin_memcpy(p, &v, 4); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void copy16(u8* d, const u8* s) {
  u32x4 v;
  __builtin_memcpy(&v, s, 16);
  __builtin_memcpy(d, &v, 16);
}

__device__ __forceinline__ u32 hash_bytes(u32 bytes, int shift) {
  return (bytes * kHashMul) >> shift;  // snappy.cc:46-49
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// ---- encode work units (encode_plan_kernel's long list)
constexpr u32 kWaveEncMaxWaves = 5;      // waves per encode_wave_kernel workgroup (at most)
constexpr u32 kWholeUnit = 0x80000000u;  // unit = a whole message (not a fragment of a split one)

// Units [0, quota) of the long list go to the wave encoder, the rest to the
// lane encoder.  All of them when their bytes fit what the wave encoder does
// in about the time one lane needs for a 64 KiB fragment at full load (the
// lane path's floor: a lane taking a long unit late sets the batch's tail;
// measured on MI355X: one lane ~40 ms per 64 KiB fragment); otherwise the
// wave encoder's share of a bandwidth-bound batch (0.5 since round 5: the
// wave encoder alone does C3 in ~165 ms, the lanes in ~135 ms, and a sweep
// of 280 / 400 / 500 / 600 permille measured 97-101 / 94 / 87 / 101 ms).
// Both kernels compute it from the plan pass's counters.
__device__ __forceinline__ u32 wave_quota(const u32* ctr, u32 share_permille, u64 all_bytes) {
  const u32 n_long = ctr[1];
  const u64 bytes = *reinterpret_cast<const unsigned long long*>(ctr + 6);
  if (bytes <= all_bytes) return n_long;
  const u64 q = ((u64)n_long * share_permille + 999) / 1000;
  return q < n_long ? (u32)q : n_long;
}


}  // namespace fsg
