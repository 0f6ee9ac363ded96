// Internal helpers shared by the host-side translation units of libdeppy_hip.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/deppy_hip.h"

namespace dp {

// Text of the last failure that had no context to hang on (dp_create, dp_lower).
void set_global_error(const std::string& s);

// Go's strconv.Quote (used by fmt's %q), lit_mapping.go:15,86.  ASCII is exact;
// for non-ASCII runes the printable test covers the Unicode ranges Go rejects
// that identifiers plausibly contain (C1 controls, spaces, format characters,
// private use); see DESIGN.md §Errors.
std::string go_quote(const char* s, size_t n);

inline int64_t words_of(const int32_t* rec) { return rec[DP_H_WORDS]; }

}  // namespace dp
