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
//                   larger indices); same code, working set in HBM scratch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/deppy_hip.h"

namespace dp {

__host__ __device__ inline int32_t bits_words(int32_t n) { return (n + 31) >> 5; }

// learned-row store (oracle: L_MAX rows, lcap = 2*nv + 64 literals)
constexpr int32_t L_MAX = 64;
// work list of one propagation chunk (rows watched by <= 64 frontier literals)
constexpr int32_t WBUF = 256;
// AtMost rows queued for wave-cooperative evaluation in one round
constexpr int32_t CQ = 64;

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

// Device image of a problem = the record followed by an extension the host
// runtime derives from it (runtime.cpp build_image), all int32 in HBM:
//   w_off[2nv+1], w[ncl+nkl]  watch lists: rows to evaluate when literal l
//                             becomes true (clauses holding ~l; AtMost rows
//                             holding var(l) when l is positive), row order
//   base[nbase]               rows that can fire on the empty assignment
//                             (clauses of length <= 1; AtMost rows in which
//                             some variable's multiplicity exceeds the bound)
// Two reserved header words of the device copy carry the extension sizes.
enum { DP_H_NBASE = 14, DP_H_IMG = 15 };

struct ImgLayout {
  int32_t w_off, w, base, words;
};

__host__ __device__ inline ImgLayout img_layout(const int32_t* h) {
  ImgLayout X;
  int32_t o = h[DP_H_WORDS];
  X.w_off = o; o += 2 * h[DP_H_NV] + 1;
  X.w = o;     o += h[DP_H_NCL] + h[DP_H_NKL];
  X.base = o;  o += h[DP_H_NBASE];
  X.words = o;
  return X;
}

struct Layout {
  int32_t body;      // image arrays (header dropped), one IX per image word
  int32_t val;       // int8[nv]: 0 unassigned, 1 true, -1 false
  int32_t reason;    // IX[nv] implying row; R_DEC / R_EXTRA
  int32_t rs;        // IX[nv] trail position where the assigning round started
  int32_t trail;     // IX[nv] true literals in assignment order
  int32_t touched;   // IX[2nv] literals implied this round; analysis work list
  int32_t d_lit;     // IX[nv] Solve() decision literals
  int32_t d_mark;    // IX[nv] trail length before each decision
  int32_t dix;       // IX[nv] decision index of a variable (NONE otherwise)
  int32_t imp;       // u32[2nv] lowest row implying literal l this round (INF: none)
  int32_t d_flip;    // bits[nv] decision already flipped
  int32_t inS;       // bits[nv] guessed set (search.assumptions)
  int32_t extra;     // bits[nv] SAT-epilogue extras
  int32_t seen;      // bits[nv] conflict analysis
  int32_t model;     // bits[nv] last model (Value)
  int32_t dset;      // bits[nv] decisions met by the last conflict analysis
  int32_t fg;        // bits[nv] guesses met by the refutation of a Solve()
  int32_t used;      // bits[nid] identities met by a refutation
  int32_t en;        // bits[nid] identities enabled (core search)
  int32_t en2;       // bits[nid]
  int32_t l_off;     // IX[L_MAX+1] learned rows (rows nrows..)
  int32_t l_lits;    // IX[lcap]
  int32_t dq;        // IX[2*cap] deque of choices (list, idx)
  int32_t stk;       // IX[5*cap] guess stack (list, idx, m, children, mark)
  int32_t wbuf;      // IX[WBUF] flattened work list (watch-list positions)
  int32_t cardq;     // i32[CQ] AtMost rows queued this round
  int32_t scal;      // i32[16] wave-shared scalars
  int32_t bytes;     // total
  int32_t cap, lcap;
};

enum Scalar { S_NTOUCHED = 0, S_NWORK = 1, S_NK = 2 };

template <class IX>
__host__ __device__ inline Layout layout(const int32_t* h) {
  Layout L;
  const int32_t nv = h[DP_H_NV], nid = h[DP_H_NID];
  const int32_t nbv = bits_words(nv), nbi = bits_words(nid);
  const int32_t ix = (int32_t)sizeof(IX);
  int32_t o = 0;
  auto take = [&](int32_t nbytes) {
    int32_t at = o;
    o += (nbytes + 15) & ~15;  // every array 16-byte aligned
    return at;
  };
  L.cap = h[DP_H_NA] + h[DP_H_NCH] + 2;
  L.lcap = 2 * nv + 64;
  L.body = take((h[DP_H_IMG] - DP_H_SIZE + 4) * ix);  // +4: dwordx4 copy slack
  L.val = take(nv);
  L.reason = take(nv * ix);
  L.rs = take(nv * ix);
  L.trail = take(nv * ix);
  L.touched = take(2 * nv * ix);
  L.d_lit = take(nv * ix);
  L.d_mark = take(nv * ix);
  L.dix = take(nv * ix);
  L.imp = take(2 * nv * 4);
  L.d_flip = take(nbv * 4);
  L.inS = take(nbv * 4);
  L.extra = take(nbv * 4);
  L.seen = take(nbv * 4);
  L.model = take(nbv * 4);
  L.dset = take(nbv * 4);
  L.fg = take(nbv * 4);
  L.used = take(nbi * 4);
  L.en = take(nbi * 4);
  L.en2 = take(nbi * 4);
  L.l_off = take((L_MAX + 1) * ix);
  L.l_lits = take(L.lcap * ix);
  L.dq = take(2 * L.cap * ix);
  L.stk = take(5 * L.cap * ix);
  L.wbuf = take(WBUF * ix);
  L.cardq = take(CQ * 4);
  L.scal = take(16 * 4);
  L.bytes = o;
  return L;
}

// Can the record run on the 16-bit LDS image?  Every index it holds, and every
// value the solve stores per variable / row, must stay below 0xfffe (0xffff and
// 0xfffe encode the no-row reasons).
__host__ __device__ inline bool fits16(const int32_t* h) {
  const int32_t nv = h[DP_H_NV];
  return h[DP_H_WORDS] < 65000 && nv < 16000 && h[DP_H_NID] < 65000 &&
         h[DP_H_NC] + h[DP_H_NK] + L_MAX < 65000 && h[DP_H_NA] + h[DP_H_NCH] < 65000 &&
         h[DP_H_NCL] + h[DP_H_NKL] < 65000;
}

}  // namespace dp
