// LDS layout of one problem's working set (one wavefront per problem).
// Shared by the host runtime (to size dynamic LDS and bucket launches) and the
// kernel (to carve the allocation).  All sizes in 32-bit words.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/deppy_hip.h"

namespace dp {

struct LdsLayout {
  // static problem image
  int32_t rec;       // record copy (header + arrays), DP_H_WORDS words, rounded to 4
  int32_t w_off;     // [2nv+1] watch offsets per literal
  int32_t w;         // [ncl+nkl] rows to evaluate when a literal becomes true
  // per-variable state
  int32_t val;       // int8[nv]: 0 unassigned, 1 true, -1 false
  int32_t reason;    // [nv] implying row, -1 decision/assumption, -2 extras bound
  int32_t rnd;       // [nv] propagation round of the assignment
  int32_t trail;     // [nv] true literals in assignment order
  int32_t imp_pos;   // [nv] lowest row implying +v this round   (also: watch-build cursor, 2nv)
  int32_t imp_neg;   // [nv] lowest row implying -v this round
  int32_t impflag;   // [nv] bit0 +v implied, bit1 -v implied this round
  int32_t touched;   // [nv] variables implied this round (also: analysis work list)
  int32_t d_lit;     // [nv] Solve() decision literals
  int32_t d_mark;    // [nv] trail length before each decision
  int32_t d_flip;    // bits[nv] decision already flipped
  int32_t inS;       // bits[nv] guessed set (search.assumptions)
  int32_t extra;     // bits[nv] SAT-epilogue extras
  int32_t seen;      // bits[nv] conflict analysis
  int32_t model;     // bits[nv] last model (Value)
  int32_t used;      // bits[nid] identities met by a refutation
  int32_t en;        // bits[nid] identities enabled (core search)
  int32_t en2;       // bits[nid]
  int32_t dix;       // [nv] Solve() decision index of a variable, -1 otherwise
  int32_t dset;      // bits[nv] decisions met by the last conflict analysis
  int32_t fg;        // bits[nv] guesses met by the refutation of a Solve()
  int32_t l_off;     // [L_MAX+1] learned rows (rows nrows..)
  int32_t l_lits;    // [lcap] learned literals
  int32_t lcap;
  int32_t dq;        // [2*cap] deque of choices (list, idx)
  int32_t stk;       // [5*cap] guess stack (list, idx, m, children, mark)
  int32_t pre;       // [64] exclusive prefix of watch-list lengths
  int32_t preA;      // [64] watch-list starts
  int32_t scal;      // [16] wave-shared scalars
  int32_t words;     // total
  int32_t cap;       // deque / stack capacity
};

enum Scalar {  // indices into the scal block
  S_CROW = 0,     // lowest conflicting row of the round
  S_CVAR = 1,     // lowest variable implied both ways
  S_NTOUCHED = 2, // implied variables this round
  S_NWORK = 3,    // analysis work list length
  S_TMP = 4
};

__host__ __device__ inline int32_t bits_words(int32_t n) { return (n + 31) >> 5; }

// learned-row store (oracle L_MAX, lcap = 4*nv + 256)
constexpr int32_t L_MAX = 64;

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

__host__ __device__ inline LdsLayout lds_layout(const int32_t* h) {
  LdsLayout L;
  const int32_t nv = h[DP_H_NV], nid = h[DP_H_NID];
  const int32_t nbv = bits_words(nv), nbi = bits_words(nid);
  int32_t o = 0;
  auto take = [&](int32_t n) {
    int32_t at = o;
    o += (n + 3) & ~3;  // keep every array 16-byte aligned
    return at;
  };
  L.cap = h[DP_H_NA] + h[DP_H_NCH] + 2;
  L.rec = take(h[DP_H_WORDS]);
  L.w_off = take(2 * nv + 1);
  L.w = take(h[DP_H_NCL] + h[DP_H_NKL]);
  L.val = take((nv + 3) >> 2);
  L.reason = take(nv);
  L.rnd = take(nv);
  L.trail = take(nv);
  L.imp_pos = take(nv);
  L.imp_neg = take(nv);
  L.impflag = take(nv);
  L.touched = take(nv);
  L.d_lit = take(nv);
  L.d_mark = take(nv);
  L.d_flip = take(nbv);
  L.inS = take(nbv);
  L.extra = take(nbv);
  L.seen = take(nbv);
  L.model = take(nbv);
  L.used = take(nbi);
  L.en = take(nbi);
  L.en2 = take(nbi);
  L.dix = take(nv);
  L.dset = take(nbv);
  L.fg = take(nbv);
  L.l_off = take(L_MAX + 1);
  L.lcap = 4 * nv + 256;
  L.l_lits = take(L.lcap);
  L.dq = take(2 * L.cap);
  L.stk = take(5 * L.cap);
  L.pre = take(64);
  L.preA = take(64);
  L.scal = take(16);
  L.words = o;
  return L;
}

// imp_pos and imp_neg are adjacent (2nv words) so they double as the per-literal
// cursor while watch lists are built.
static_assert(sizeof(int32_t) == 4, "");

}  // namespace dp
