// Page-locked host memory for record batches (runtime.cpp): a batch lowered
// into it (dp_lower_into DP_LOWER_PINNED) is copied to the device by DMA
// straight from where it lies.
#pragma once
#include <cstddef>

namespace dp {
// nullptr when no HIP device is present or the allocation fails
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);
}  // namespace dp
