// Working-set layout of one problem (one wavefront per problem).
// Shared by the host runtime (to size dynamic LDS and bucket launches) and the
// kernel (to carve the allocation).  Offsets and sizes are in BYTES.
//
// Two images of the same layout exist:
//   IX = uint16_t : the LDS image.  Record arrays are narrowed to 16 bits on
//                   load (every index of an eligible problem is < 65000), so a
//                   ~240-variable catalog needs ~18 KiB and 8-9 problems fit
//                   in one CU's 160 KiB of LDS.
//   IX = int32_t  : the HBM image for problems too large for LDS (or with
//                   larger indices), solved by one multi-wave workgroup
//                   (M_SPLIT / M_HBM below).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/deppy_hip.h"

namespace dp {

__host__ __device__ inline int32_t bits_words(int32_t n) { return (n + 31) >> 5; }

// learned-row store (oracle: L_MAX rows, lcap = 2*nv + 64 literals)
constexpr int32_t L_MAX = 64;

// Three placements of the same working set (one template instantiation each):
//   M_LDS   one wavefront per problem, the whole image narrowed to 16 bits and
//           the whole working set in LDS (the batched small-catalog path)
//   M_SPLIT one workgroup of BIG_WAVES wavefronts per problem (large catalogs,
//           e.g. config 4): the int32 image is read in place from HBM, the
//           per-literal arrays live in an HBM scratch region, and the hot
//           per-variable state (val, every bitset) plus the work lists live in
//           LDS
//   M_HBM   the same workgroup with everything but the work lists in HBM
//           (catalogs whose per-variable state exceeds the LDS)
// M_SPLIT4: M_SPLIT with MID_WAVES wavefronts (catalogs routed off the LDS
// path for their size, not for overflowing it; runtime.cpp kMidMaxVars)
// M_LDSG  the M_LDS image and working set, all of it in LDS, solved by one
//         workgroup of LDSG_WAVES wavefronts: catalogs whose one-wavefront
//         footprint is above placement.hpp group_above() (a lone wavefront
//         would leave the CU's other SIMDs idle) but still fits one CU's LDS.
//         No HBM scratch: every per-literal array, watch list and learned row
//         is LDS.
enum Mode { M_LDS = 0, M_SPLIT = 1, M_HBM = 2, M_SPLIT4 = 3, M_LDSG = 4 };
static_assert((int)M_LDS == DP_PLACE_LDS && (int)M_SPLIT == DP_PLACE_SPLIT && (int)M_HBM == DP_PLACE_HBM &&
                  (int)M_SPLIT4 == DP_PLACE_SPLIT4 && (int)M_LDSG == DP_PLACE_LDSG,
              "enum dp_place (include/deppy_hip.h) names the placements");
// The 16-bit LDS image (M_LDS, M_LDSG): record and working set in LDS
__host__ __device__ constexpr bool mode_n16(int mode) { return mode == M_LDS || mode == M_LDSG; }
#ifndef DP_BIG_WAVES
#define DP_BIG_WAVES 8
#endif
constexpr int32_t BIG_WAVES = DP_BIG_WAVES;

#ifndef DP_MID_WAVES
#define DP_MID_WAVES 4
#endif
constexpr int32_t MID_WAVES = DP_MID_WAVES;
#ifndef DP_LDSG_WAVES
#define DP_LDSG_WAVES 4
#endif
constexpr int32_t LDSG_WAVES = DP_LDSG_WAVES;
__host__ __device__ constexpr int32_t mode_waves(int mode) {
  return mode == M_LDS ? 1 : mode == M_SPLIT4 ? MID_WAVES : mode == M_LDSG ? LDSG_WAVES : BIG_WAVES;
}
// work list of one propagation chunk (rows watched by <= 64*waves frontier literals)
__host__ __device__ constexpr int32_t mode_wbuf(int mode) {
  return mode == M_LDS ? 128 : mode == M_LDSG ? 1024 : 4096;
}
// AtMost rows queued for wave-cooperative evaluation in one round
__host__ __device__ constexpr int32_t mode_cq(int mode) { return mode == M_LDS ? 64 : mode == M_LDSG ? 256 : 512; }
// The one-wavefront image stores imp (the lowest implying row per literal)
// in 16 bits, updated by a compare-and-swap; the multi-wave modes in 32
// bits, updated by atomicMin.  Two-watched-literal filters, row slots and
// 2-byte watch entries were built and measured slower on every placement
// (DESIGN.md §5.3, §9); occurrence lists with 8-byte entries ship.

// wave-shared scalars (S_*), then (multi-wave modes) per-wave reduction slots
constexpr int32_t NSCAL = 64;
__host__ __device__ constexpr int32_t mode_nscal(int mode) {
#ifdef DP_STAMPS
  return (mode == M_LDS ? 8 : NSCAL) + 64;  // diagnostic build: 32 int64 phase accumulators after the scalars
#else
  return mode == M_LDS ? 8 : NSCAL;
#endif
}

// dp_p16_tail_at / dp_p16_tail_bytes (include/deppy_hip.h) for device code.
__host__ __device__ inline bool fmt_derived(int32_t fmt) { return fmt == DP_FMT_P16D || fmt == DP_FMT_P8D; }
__host__ __device__ inline bool fmt_packed(int32_t fmt) { return fmt == DP_FMT_P16 || fmt_derived(fmt); }
__host__ __device__ inline int64_t p16_tail_at(const int32_t* h) {
  const int64_t ch = fmt_derived(h[DP_H_FMT]) ? 0 : h[DP_H_NCHL];
  return (2 * ((int64_t)h[DP_H_NCL] + h[DP_H_NKL] + h[DP_H_NK] + ch + h[DP_H_NA]) + 15) & ~(int64_t)15;
}
__host__ __device__ inline int64_t p16_tail_bytes(const int32_t* h) {
  const int64_t vc = fmt_derived(h[DP_H_FMT]) ? 0 : (int64_t)h[DP_H_NV];
  return (int64_t)h[DP_H_NC] + h[DP_H_NK] + h[DP_H_NCH] + vc + ((int64_t)h[DP_H_NID] + 7) / 8;
}
// DP_FMT_P8D: the body's bytes (header word DP_H_P8, bits 8..)
__host__ __device__ inline int32_t p8_bytes(const int32_t* h) { return (int32_t)((uint32_t)h[DP_H_P8] >> 8); }
// 16-bit words of a record's body (the arrays after the header) as the
// one-wavefront kernel decodes it into LDS: the int32 form's, except that
// DP_FMT_P16D's choice lists stay in the dependency rows they are implied
// by -- one row reference per list (nch words) in place of choice_off
// (nch + 1) and choice_lits (nchl).  The watch lists follow.
// The packed forms (DP_FMT_P16 / P16D) also keep their identities as the
// record's AtMost-identity mask (u32 words) with a prefix count per word, in
// place of clause_id (nc) and card_id (nk): every identity owns exactly one
// row, so the kernel works on rows and maps to identities only for the
// outputs (solve_kernel.hpp row_of).
__host__ __device__ inline int32_t id_mask_words16(const int32_t* h) {
  return 3 * bits_words(h[DP_H_NID]) + 2;  // mask (2 halves a word) + counts (nbi + 1) + alignment
}
__host__ __device__ inline int32_t lds_body_words(const int32_t* h) {
  int32_t b = h[DP_H_WORDS] - DP_H_SIZE;
  if (fmt_packed(h[DP_H_FMT])) b += id_mask_words16(h) - h[DP_H_NC] - h[DP_H_NK];
  return fmt_derived(h[DP_H_FMT]) ? b - 1 - h[DP_H_NCHL] : b;
}
// Byte offset (in the M_LDS body region) of the packed tail's copy while the
// kernel decodes it: the first 16-byte boundary past the decoded 16-bit
// arrays (lds_body_words).  DP_FMT_P8D: where its record lands (LDS-DMA),
// its DP_FMT_P16D tail decoded right after it (p8_tail).
__host__ __device__ inline int32_t p16_tail_copy(const int32_t* h) {
  return (2 * lds_body_words(h) + 15) & ~15;
}
__host__ __device__ inline int32_t p8_tail(const int32_t* h) {
  return p16_tail_copy(h) + ((p8_bytes(h) + 15) & ~15);
}

// dp_rec_layout_of (include/deppy_hip.h) for host and device code.
__host__ __device__ inline dp_rec_layout rec_layout(const int32_t* h) {
  dp_rec_layout L;
  int32_t o = DP_H_SIZE;
  L.clause_off = o;     o += h[DP_H_NC] + 1;
  L.clause_lits = o;    o += h[DP_H_NCL];
  L.clause_id = o;      o += h[DP_H_NC];
  L.card_off = o;       o += h[DP_H_NK] + 1;
  L.card_lits = o;      o += h[DP_H_NKL];
  L.card_bound = o;     o += h[DP_H_NK];
  L.card_id = o;        o += h[DP_H_NK];
  L.var_choice_off = o; o += h[DP_H_NV] + 1;
  L.choice_off = o;     o += h[DP_H_NCH] + 1;
  L.choice_lits = o;    o += h[DP_H_NCHL];
  L.anchors = o;        o += h[DP_H_NA];
  L.words = o;
  return L;
}

// The device copy of a problem is its record alone: nothing derived is built
// on the host or crosses PCIe.  A reserved header word of the device copy
// marks the 16-bit form (DP_FMT_U16): records of problems solved on the LDS
// path are narrowed by the host while it stages them (the int32 header stays,
// every word after it becomes a uint16), so PCIe and the LDS-DMA of init move
// half the bytes and the kernel has nothing to convert.
//
// Each record has watch lists
//   w_off[2nv+1], w[ncl+nkl]  rows to evaluate when literal l becomes true
//                             (clauses holding ~l; AtMost rows holding
//                             var(l) when l is positive, one entry per
//                             distinct variable)
// built on the device: in LDS during init for one-wavefront problems, right
// after the record (Group::build_watches); in the problem's HBM scratch for
// the multi-wave ones (Layout::wl: build_watches_wide, or watch_build.hip's
// passes above DEV_WATCH_VARS).  A DP_FMT_I32W record brings its own, and
// the host builds them after a record it converts while staging
// (runtime.cpp stage_one).  Rows that can fire on the empty assignment
// (clauses of length <= 1, AtMost rows in which some variable's multiplicity
// exceeds the bound) are found by a sweep of the row offsets
// (Group::base_propagate).

// Staged-copy formats besides the public ones: a record the host rejected
// while staging it (the kernel reports it as malformed without reading its
// body), and the 16-bit form of a record the host checked while narrowing it
// (the kernel validates only the DP_FMT_U16 copies the host passed through
// unread, Group::valid_record).
enum { DP_FMT_REJECT = 2, DP_FMT_U16_CHECKED = 16, DP_FMT_I32_CHECKED = 17 };

// Multi-wave problems cross PCIe as plain int32 records (DP_FMT_I32, no watch
// lists), and their watch lists are built on the device in the problem's HBM
// scratch (Layout::wl): up to DEV_WATCH_VARS variables by the solving
// workgroup with counters in the LDS work area (Group::build_watches_wide),
// above it by grid-wide passes before the launch (watch_build.hip).  A
// caller may also send DP_FMT_I32W (record + host-built lists).
constexpr int32_t DEV_WATCH_VARS = 2048;
__host__ __device__ inline bool device_watches(const int32_t* h) { return h[DP_H_NV] <= DEV_WATCH_VARS; }
// Its 2nv+1 counters span the work list and the AtMost queue after it
// (layout() takes them back to back, 16-byte aligned; both are free until the
// first round).
static_assert(2 * DEV_WATCH_VARS + 1 <= mode_wbuf(M_SPLIT) + mode_cq(M_SPLIT) &&
                  2 * DEV_WATCH_VARS + 1 <= mode_wbuf(M_SPLIT4) + mode_cq(M_SPLIT4) &&
                  2 * DEV_WATCH_VARS + 1 <= mode_wbuf(M_HBM) + mode_cq(M_HBM) && mode_wbuf(M_SPLIT) % 4 == 0,
              "build_watches_wide: the counters fit wbuf + cardq");

// A row's literal range in one word, for the 8-byte entries of device-built
// multi-wave watch lists (solve_kernel.hpp Group::w8): first position << 8 |
// length, or ROW_INFO_NONE (read the row's offsets) for a row of 255 or more
// positions or one starting at or past 2^24.
constexpr uint32_t ROW_INFO_NONE = 0xffffffffu;
__host__ __device__ inline uint32_t row_info(int32_t a, int32_t len) {
  return a >= 0 && a < (1 << 24) && len >= 0 && len < 255 ? ((uint32_t)a << 8) | (uint32_t)len : ROW_INFO_NONE;
}

struct ImgLayout {
  int32_t w_off, w, words;
};

// Words of the extended record (record + watch lists), in record-word units.
__host__ __device__ inline ImgLayout img_layout(const int32_t* h) {
  ImgLayout X;
  int32_t o = h[DP_H_WORDS];
  X.w_off = o; o += 2 * h[DP_H_NV] + 1;
  X.w = o;     o += h[DP_H_NCL] + h[DP_H_NKL];
  X.words = o;
  return X;
}

// Words of the staged (device) copy of a record: 16-byte aligned; the body in
// 16-bit form when narrow (one-wavefront problems), else int32 followed by the
// host-built watch lists.
__host__ __device__ inline int64_t staged_words(const int32_t* h, bool narrow) {
  const int64_t body = (int64_t)h[DP_H_WORDS] - DP_H_SIZE;
  const int64_t w = narrow ? DP_H_SIZE + (body + 1) / 2 : (int64_t)img_layout(h).words;
  return (w + 3) & ~3LL;
}

// Byte offsets of every working-set array.  An offset is into the LDS
// allocation when the mode places that array in LDS (in_lds below), else into
// the problem's HBM scratch region.
struct Layout {
  int32_t body;      // M_LDS / M_LDSG only: the extended record (header dropped), one IX per word;
                     // the watch-list build counts on the per-literal arrays (reason..touched)
  int32_t val;       // int8[nv]: 0 unassigned, 1 true, -1 false                  [LDS unless M_HBM]
  int32_t reason;    // IX[nv] implying row; R_DEC / R_EXTRA / a Solve() decision (-3 - index)
  int32_t rs;        // IX[nv] trail position where the assigning round started
  int32_t trail;     // IX[nv] true literals in assignment order
  int32_t touched;   // IX[2nv] literals implied this round; analysis work list
  int32_t d_mark;    // IX[nv] trail length before each Solve() decision (its literal is trail[d_mark])
  int32_t imp;       // IX[2nv] lowest row implying literal l this round (all ones: none)
  int32_t d_flip;    // bits[nv] decision already flipped                          [LDS unless M_HBM]
  int32_t inS;       // bits[nv] guessed set (search.assumptions)                  [LDS unless M_HBM]
  int32_t extra;     // bits[nv] SAT-epilogue extras                               [LDS unless M_HBM]
  int32_t seen;      // bits[nv] conflict analysis                                 [LDS unless M_HBM]
  int32_t model;     // bits[nv] last model (Value)                                [LDS unless M_HBM]
  int32_t dset;      // bits[nv] decisions met by the last conflict analysis       [LDS unless M_HBM]
  int32_t fg;        // bits[nv] guesses met by the refutation of a Solve()        [LDS unless M_HBM]
  int32_t used;      // bits[nid] identities met by a refutation                   [LDS unless M_HBM]
  int32_t en;        // bits[nid] identities enabled (core search)                 [LDS unless M_HBM]
  int32_t en2;       // bits[nid]                                                  [LDS unless M_HBM]
  int32_t crit;      // bits[nid] identities proven necessary by a core's model rotation [LDS unless M_HBM]
  int32_t idt;       // (M_LDS / M_LDSG) bits[nid] rows -> identities for the outputs (row_of)  [LDS]
  int32_t l_off;     // IX[L_MAX+1] learned rows (rows nrows..)
  int32_t l_lits;    // IX[lcap]
  int32_t dq;        // IX[2*cap] deque of choices (list, idx)
  int32_t stk;       // IX[3*cap] guess stack (list, idx | G_SKIP, mark)
  int32_t wbuf;      // IX[wbuf] flattened work list (watch-list positions)       [LDS]
  int32_t cardq;     // IX[cq] AtMost rows queued this round (multi-wave: then their row_info)  [LDS]
  int32_t scal;      // i32[nscal] wave-shared scalars and reduction slots        [LDS]
  // M_SPLIT / M_SPLIT4 round state in LDS (mode_lds_rounds): a round's
  // implications in an open-addressing table keyed by variable, the list of
  // first implications, and a ring of the latest trail entries (the next
  // round's frontier), so a round touches HBM only for the record
  int32_t hkey;      // i32[hc] variable of the slot (-1 empty)                    [LDS]
  int32_t hrp, hrn;  // u32[hc] lowest row implying +v / -v this round (INF none)  [LDS]
  int32_t tl;        // u16[2hc] first implications, (slot << 1) | negative       [LDS]
  int32_t fr;        // i32[hc] trail ring: trail[i] at fr[i & (hc - 1)]          [LDS]
  int32_t hc;        // slots (a power of two; 0 when the mode keeps rounds in HBM)
  int32_t wl;        // multi-wave, DP_FMT_I32 records: device-built w_off[2nv+2], then
                     // [ncl+nkl] int2 {row, row_info} entries  [HBM]
  int32_t bytes;     // HBM scratch bytes (0 for M_LDS / M_LDSG)
  int32_t lds_bytes; // LDS bytes
  int32_t cap, lcap;
};

// S_NTB / S_CVB / S_OVB: two banks each (alternate LDS-table rounds) of the
// round's first-implication count, lowest variable implied both ways (stored
// as INF - v, 0 none) and table-overflow flag.  S_POSROWS: the record has
// auxiliary variables (DP_H_NVU), so clause rows without a negative literal
// (an AtMost network's (g a b) rows) can be violated by the all-false
// completion (Group::first_violated scans every row).
// (M_LDS has slots 0..7 only.)
enum Scalar { S_NTOUCHED = 0, S_NWORK = 1, S_POSROWS = 2, S_APP = 3, S_NTB = 4, S_CVB = 6, S_OVB = 8, S_SLOT = 32 };

// Multi-wave modes whose per-variable state is in LDS keep a round's state
// there too (Layout::hkey..fr); M_HBM keeps it in HBM.
__host__ __device__ constexpr bool mode_lds_rounds(int mode) { return mode == M_SPLIT || mode == M_SPLIT4; }
// Implication-table slots: about one per 8 variables, 64..1024 (a round that
// implies more than the table holds is redone on the HBM arrays).
__host__ __device__ inline int32_t round_slots(int32_t nv) {
  int32_t c = 64;
  while (c < 1024 && c < nv / 8) c <<= 1;
  return c;
}

template <int MODE>
__host__ __device__ inline Layout layout_hc(const int32_t* h, int32_t hc) {
  constexpr bool N16 = mode_n16(MODE);
  using IX = typename std::conditional<N16, uint16_t, int32_t>::type;
  Layout L;
  const int32_t nv = h[DP_H_NV], nid = h[DP_H_NID];
  const int32_t nbv = bits_words(nv), nbi = bits_words(nid);
  const int32_t ix = (int32_t)sizeof(IX);
  int32_t og = 0, ol = 0;
  // every array 16-byte aligned; `hot` arrays go to LDS unless M_HBM, the
  // per-literal arrays to LDS only in M_LDS / M_LDSG, the work lists always to LDS
  auto take = [&](int32_t nbytes, int kind) {
    const bool lds = N16 || kind == 2 || (kind == 1 && (MODE == M_SPLIT || MODE == M_SPLIT4));
    int32_t& o = lds ? ol : og;
    const int32_t at = o;
    o += (nbytes + 15) & ~15;
    return at;
  };
  enum { COLD = 0, HOT = 1, WORK = 2 };
  L.cap = h[DP_H_NA] + h[DP_H_NCH] + 2;
  L.lcap = nv + 64;
  const ImgLayout X = img_layout(h);
  // M_LDS: the record (16-bit) and its watch lists, +8 words of dwordx4 copy
  // slack.  A packed record's tail is copied to p16_tail_copy (where the
  // watch lists go later) while it is decoded: the region covers that copy.
  int32_t body_bytes = (X.words - DP_H_SIZE + 8) * ix;
  if (N16) body_bytes = (lds_body_words(h) + (X.words - h[DP_H_WORDS]) + 8) * ix;
  if (N16 && fmt_packed(h[DP_H_FMT])) {
    const int32_t tail = h[DP_H_FMT] == DP_FMT_P8D ? p8_tail(h) : p16_tail_copy(h);
    const int32_t need = tail + (int32_t)((p16_tail_bytes(h) + 15) & ~15);
    body_bytes = body_bytes > need ? body_bytes : need;
  }
  L.body = N16 ? take(body_bytes, COLD) : 0;
  L.scal = take(mode_nscal(MODE) * 4, WORK);
  L.wbuf = take(mode_wbuf(MODE) * ix, WORK);
  // (multi-wave: each queued row's row_info after the queue, cardq[cq + i])
  L.cardq = take(mode_cq(MODE) * ix * (N16 ? 1 : 2), WORK);
  L.hc = mode_lds_rounds(MODE) ? hc : 0;
  L.hkey = take(L.hc * 4, WORK);
  L.hrp = take(L.hc * 4, WORK);
  L.hrn = take(L.hc * 4, WORK);
  L.tl = take(L.hc * 4, WORK);
  L.fr = take(L.hc * 4, WORK);
  L.val = take(nv, HOT);
  L.d_flip = take(nbv * 4, HOT);
  L.inS = take(nbv * 4, HOT);
  L.extra = take(nbv * 4, HOT);
  L.seen = take(nbv * 4, HOT);
  L.model = take(nbv * 4, HOT);
  L.dset = take(nbv * 4, HOT);
  L.fg = take(nbv * 4, HOT);
  L.used = take(nbi * 4, HOT);
  L.en = take(nbi * 4, HOT);
  L.en2 = take(nbi * 4, HOT);
  L.crit = take(nbi * 4, HOT);
  L.idt = N16 ? take(nbi * 4, HOT) : 0;
  L.reason = take(nv * ix, COLD);
  L.rs = take(nv * ix, COLD);
  L.trail = take(nv * ix, COLD);
  L.touched = take(2 * nv * ix, COLD);
  L.d_mark = take(nv * ix, COLD);
  L.imp = take(2 * nv * (N16 ? 2 : 4), COLD);
  L.l_off = take((L_MAX + 1) * ix, COLD);
  L.l_lits = take(L.lcap * ix, COLD);
  L.dq = take(2 * L.cap * ix, COLD);
  L.stk = take(3 * L.cap * ix, COLD);
  L.wl = !N16 && h[DP_H_FMT] == DP_FMT_I32 ? take((2 * nv + 2) * 4 + (h[DP_H_NCL] + h[DP_H_NKL]) * 8, COLD) : 0;
  L.bytes = og;
  L.lds_bytes = ol;
  return L;
}

// The round table shrinks (to 64 slots at least) when the catalog's
// per-variable state leaves less LDS, so it never moves a catalog off this
// placement.  The budget is the layout itself (every array layout_hc takes),
// not a formula beside it: round 5 added an identity bitset (crit) that a
// hand-written budget left out, and every OLM-scale catalog fell to M_HBM.
constexpr int32_t kLdsLimitBytes = 160 * 1024;  // LDS per CU on gfx950
template <int MODE>
__host__ __device__ inline Layout layout(const int32_t* h) {
  if (!mode_lds_rounds(MODE)) return layout_hc<MODE>(h, 0);
  int32_t hc = round_slots(h[DP_H_NV]);
  Layout L = layout_hc<MODE>(h, hc);
  while (hc > 64 && L.lds_bytes > kLdsLimitBytes) L = layout_hc<MODE>(h, hc >>= 1);
  return L;
}

// Can the record run on the 16-bit LDS image?  (dp_rec_fits16: the reasons
// encode Solve() decision d as 0xfffd - d above every row id.)
inline bool fits16(const int32_t* h) { return dp_rec_fits16(h) != 0; }

}  // namespace dp
