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
// default 16 GiB) or pinned memory is unavailable: the caller copies instead.
OutSlab* AcquireOutSlab(size_t bytes);  // holds one reference
uint8_t* OutSlabData(OutSlab* s);
void OutSlabRef(OutSlab* s);
void OutSlabRelease(OutSlab* s);
// cord_buf deleter for adopted ranges: releases the slab holding `data`.
void AdoptedDeleter(void* data);

int UsePinnedBlocks();
bool IsPinned(const void* p, size_t n);

}  // namespace flare::gpu
