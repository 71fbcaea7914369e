// pinned.h -- pinned host memory of the Snappy runtime (pinned.cc).
#pragma once

#include <cstddef>
#include <cstdint>

namespace flare::gpu {

// Refcounted pinned output slab: one device batch's D2H target, whose
// message ranges cord_bufs adopt (append_user_data, deleter AdoptedDeleter).
// It returns to the pool when the runtime and every adopting cord_buf have
// released it.
struct OutSlab;
// nullptr when the pool is at its cap (FLARE_SNAPPY_GPU_PINNED_OUT_BYTES,
// default 4 GiB) or pinned memory is unavailable: the caller copies instead.
// An adopted output keeps its whole slab out of the pool until the last
// cord_buf holding a piece of it dies.
OutSlab* AcquireOutSlab(size_t bytes);  // holds one reference
// True when over half the cap is allocated and no slab is free (adopted
// outputs are holding the pool): callers copy outputs instead of adopting.
bool OutSlabsUnderPressure();
uint8_t* OutSlabData(OutSlab* s);
void OutSlabRef(OutSlab* s);
void OutSlabRelease(OutSlab* s);
// cord_buf deleter for adopted ranges: releases the slab holding `data`.
void AdoptedDeleter(void* data);

int UsePinnedBlocks();
bool IsPinned(const void* p, size_t n);

}  // namespace flare::gpu
