// Hand-over between the device lowering (lower_device.hip) and the host
// lowering's result type (lower.cpp dp_lowered) and context (runtime.cpp).
#pragma once
#include <cstdint>

#include "../../include/deppy_hip.h"

namespace dp {

struct LoweredOut {
  int64_t *rec_off, *ident_off;
  int32_t *rec, *ivar, *icon;
};
// lw sized for P problems, rec_words record words and n_ident identities
// (page-locked when asked), every problem without an error.
LoweredOut lowered_prepare(dp_lowered* lw, int32_t P, int64_t rec_words, int64_t n_ident, bool pinned);
// Problems `which` lowered on the host from `sub` and spliced into lw.
int lowered_splice(dp_lowered* lw, const dp_wire* sub, int32_t flags, const int32_t* which, int32_t nw);
// The HIP ordinal of the context's first device (runtime.cpp).
int ctx_first_ordinal(const dp_ctx* ctx);

}  // namespace dp
