// Host-side placement of a record and the multi-wave staged form, shared by
// the lowering (lower.cpp: DP_LOWER_NARROW emits each record in the form its
// placement stages) and the pipeline (runtime.cpp).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "layout.hpp"

namespace dp {

constexpr int kMaxLdsBytes = kLdsLimitBytes;  // LDS per CU on gfx950

// Problems whose one-wavefront LDS footprint exceeds kGroupAbove run as
// multi-wave workgroups: at two or one per CU a lone wavefront per problem
// leaves SIMDs idle.  Tuned on config 5 (profiles/r01_group_above_ab.jsonl):
// a tuning point of that workload's footprint buckets, not a derived constant.
constexpr int64_t kGroupAbove = 64 << 10;

inline int64_t group_above() {
  static const int64_t v = [] {
    const char* e = std::getenv("DEPPY_GROUP_ABOVE");  // diagnostic
    const int64_t x = e && *e ? std::atoll(e) : 0;
    return x > 0 ? std::min<int64_t>(x, kMaxLdsBytes) : kGroupAbove;
  }();
  return v;
}

// Does the record (header h, well formed) run one wavefront per problem on
// its 16-bit LDS image (without DP_OPT_FORCE_* flags)?
inline bool one_wave(const int32_t* h) {
  return fits16(h) && (int64_t)layout<M_LDS>(h).lds_bytes <= group_above();
}

// The all-LDS multi-wave placement (M_LDSG) for 16-bit records past
// group_above() that fit one CU's LDS.  Alone, such a catalog solves ~25%
// faster there than on the HBM-read 4-wave group (config 5's largest
// catalogs: kernel median 0.127 vs 0.169 ms), but a workgroup holding a
// whole CU's LDS keeps other launches off that CU: with many in flight,
// config 5 runs 705-718k res/s host to host against 877-917k on the 4-wave
// groups, which share CUs (profiles/r05_ldsg_ab.txt).  So the pipeline
// places them on M_LDSG only when a chunk holds at most kLdsgMaxProblems of
// them (a latency-bound chunk: each gets a CU), else on M_SPLIT4.
// DEPPY_LDSG (diagnostic, and tests of the HBM-read multi-wave records):
// 0 never, 1 always, unset/2 that rule.  Read once per lowering call and per
// planned chunk.
constexpr int32_t kLdsgMaxProblems = 256;  // MI355X CUs
enum { LDSG_NEVER = 0, LDSG_ALWAYS = 1, LDSG_AUTO = 2 };
inline int ldsg_env() {
  const char* e = std::getenv("DEPPY_LDSG");
  return e && *e == '0' ? LDSG_NEVER : e && *e == '1' ? LDSG_ALWAYS : LDSG_AUTO;
}
// Does the record fit the M_LDSG working set (one CU's LDS)?
inline bool ldsg_fits(const int32_t* h) { return fits16(h) && (int64_t)layout<M_LDSG>(h).lds_bytes <= kMaxLdsBytes; }
// Does the lowering emit the record in a 16-bit form (DP_LOWER_NARROW)?
// When it runs on one wavefront (M_LDS), or under DEPPY_LDSG=1 on M_LDSG; the
// mid-size ones stay int32 otherwise (the pipeline narrows them itself for
// an M_LDSG chunk).
inline bool lds_image(const int32_t* h, int ldsg) { return one_wave(h) || (ldsg == LDSG_ALWAYS && ldsg_fits(h)); }

// The watch lists of a multi-wave problem (layout.hpp img_layout), right
// after its int32 record r: rows in ascending order in every list.  Returns
// the extended length in words.
inline int64_t build_watches_host(int32_t* r) {
  const dp_rec_layout R = dp_rec_layout_of(r);
  const ImgLayout X = img_layout(r);
  const int32_t nv = r[DP_H_NV], nc = r[DP_H_NC], nk = r[DP_H_NK];
  const int32_t* clause_off = r + R.clause_off;
  const int32_t* clause_lits = r + R.clause_lits;
  const int32_t* card_off = r + R.card_off;
  const int32_t* card_lits = r + R.card_lits;
  int32_t* wo = r + X.w_off;
  int32_t* w = r + X.w;
  std::fill(wo, wo + 2 * (int64_t)nv + 1, 0);
  for (int32_t j = 0; j < r[DP_H_NCL]; ++j) wo[(clause_lits[j] ^ 1) + 1]++;
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t j = card_off[k]; j < card_off[k + 1]; ++j)
      if (j == card_off[k] || card_lits[j] != card_lits[j - 1]) wo[2 * card_lits[j] + 1]++;
  for (int64_t l = 0; l < 2 * (int64_t)nv; ++l) wo[l + 1] += wo[l];
  static thread_local std::vector<int32_t> cur;
  cur.assign(wo, wo + 2 * (int64_t)nv);
  for (int32_t rr = 0; rr < nc; ++rr)
    for (int32_t j = clause_off[rr]; j < clause_off[rr + 1]; ++j) w[cur[(size_t)(clause_lits[j] ^ 1)]++] = rr;
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t j = card_off[k]; j < card_off[k + 1]; ++j)
      if (j == card_off[k] || card_lits[j] != card_lits[j - 1]) w[cur[(size_t)(2 * card_lits[j])]++] = nc + k;
  return X.words;
}

}  // namespace dp
