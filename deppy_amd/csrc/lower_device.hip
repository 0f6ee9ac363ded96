// Lowering on the device (dp_lower_device): a compact 32-bit wire batch ->
// the DP_FMT_P8D records dp_lower_into(DP_LOWER_NARROW | DP_LOWER_PACKED)
// gives, byte for byte, without the host's constraint loop.
//
// One wavefront per problem runs the canonical-key lowering of lower.cpp
// (Lowerer::lower_fast, which restates newLitMapping + Constraint.Apply,
// pkg/sat/lit_mapping.go:40-77, constraints.go:54-204, and Order(),
// search.go:59-69) with the sequential loops turned into wave scans:
//   1. identifiers -> variables: an LDS hash of the problem's string ids
//      (a repeated one is a DuplicateIdentifier: the host reports it);
//   2. every constraint's canonical identity key (lower.cpp K_*), inserted
//      in an LDS table that keeps the first and last constraint of each key:
//      the first writer makes the identity and its row, the last is the
//      reported AppliedConstraint (lit_mapping.go:69-72);
//   3. in constraint order, chunks of 64: identities, clause rows, AtMost
//      rows and choice lists numbered by ballot counts and prefix sums;
//   4. the DP_FMT_P8D body (include/deppy_hip.h) assembled in LDS and written
//      to the problem's slot.
// A problem the kernel does not take -- one the keys cannot decide, one with
// an error to report, a record of another form (not P8D: choice lists not
// implied, multi-wave placement, ...), or past the kernel's sizes -- gets no
// record (0 words); dp_lower_device lowers those on the host pool and splices
// them in.  Then a scan gives the record and identity offsets, and a copy
// kernel packs the slots into the batch, which goes back to page-locked host
// memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "dlower.hpp"
#include "hostmem.hpp"
#include "layout.hpp"
#include "placement.hpp"
#include "pool.hpp"

namespace {

// the kernel's sizes (a problem past them is lowered on the host)
constexpr int DL_NV = 512;   // variables (DP_P8_MAX_VARS)
constexpr int DL_C = 512;    // constraints
constexpr int DL_A = 1536;   // constraint arguments
constexpr int DL_VH = 1024;  // identifier hash slots (>= 2 DL_NV)
constexpr int DL_KH = 1024;  // identity-key slots (>= 2 DL_C)
// a record's words at most: the LDS words the key table leaves to the record
// (the largest DP_FMT_P8D body these sizes allow is ~4.6 KB; a DP_FMT_P16
// record past 16 KB goes to the host)
constexpr int DL_SLOT = (DL_KH * 16) / 4;
constexpr int DL_T = 64;  // one wavefront per problem

// canonical keys, as lower.cpp's
enum : uint64_t { K_F = 0, K_POS = 1, K_NEG = 2, K_CONF = 3, K_NOR = 4, K_DEP = 5, K_CARD = 6 };
__device__ __forceinline__ uint64_t key1(uint64_t tag, uint32_t a) { return tag << 60 | a; }
__device__ __forceinline__ uint64_t key2(uint64_t tag, uint32_t a, uint32_t b) {
  const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
  return tag << 60 | (uint64_t)lo << 30 | hi;
}
__device__ __forceinline__ uint64_t hmix(uint64_t h, uint64_t x) {
  h ^= x + 0x9e3779b97f4a7c15ULL;
  h *= 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 31);
}
__device__ __forceinline__ uint64_t keyh(uint64_t tag, uint64_t h) { return tag << 60 | (h & ((1ULL << 60) - 1)); }

// a constraint's row if it is its key's first writer (cmeta)
enum { RT_SKIP = 0, RT_CLAUSE = 1, RT_CARD = 2 };
__device__ __forceinline__ uint32_t meta(int rt, bool hashed, bool list, int kind, int len) {
  return (uint32_t)rt | (hashed ? 4u : 0u) | (list ? 8u : 0u) | (uint32_t)kind << 4 | (uint32_t)len << 8;
}
__device__ __forceinline__ int m_rt(uint32_t m) { return (int)(m & 3u); }
__device__ __forceinline__ bool m_hashed(uint32_t m) { return (m & 4u) != 0; }
__device__ __forceinline__ bool m_list(uint32_t m) { return (m & 8u) != 0; }
__device__ __forceinline__ int m_kind(uint32_t m) { return (int)((m >> 4) & 15u); }
__device__ __forceinline__ int m_len(uint32_t m) { return (int)(m >> 8); }

// Arrays live in phases: the identifier table (1) shares its words with the
// rows (3-4), the key table (2-3) with the record (4), which keeps the
// working set at 4 workgroups per CU.
struct DlShared {
  union {
    struct {
      int32_t vkey[DL_VH];  // string id + 1 (0: empty)
      int16_t vval[DL_VH];
    };
    struct {
      int16_t clit[DL_A + DL_C];  // clause literals
      int16_t kv[DL_A];           // AtMost variables
    };
  };
  union {
    struct {
      unsigned long long kkey[DL_KH];  // key + 1 (0: empty)
      int32_t kfirst[DL_KH], klast[DL_KH];
    };
    uint32_t rec[DL_SLOT];
  };
  int16_t vstart[DL_NV + 2];  // constraints of variable i: [vstart[i], vstart[i+1])
  int16_t cs[DL_C];           // constraint -> subject variable
  int16_t ca[DL_A];           // argument -> variable
  int16_t cslot[DL_C];        // constraint -> key slot (-1: none)
  int16_t castart[DL_C + 1];  // arguments of constraint c: [castart[c], castart[c+1])
  uint32_t cmeta[DL_C];
  int16_t cid[DL_C];    // identity of a first writer
  int16_t clist[DL_C];  // choice list of a Dependency with candidates
  int16_t kb[DL_C];           // AtMost bounds
  uint8_t clen[DL_C], klen[DL_C], src[DL_C];
  uint32_t mask[DL_C / 32];   // identity is an AtMost row's
  uint32_t aflag[DL_NV / 32];  // variable has a Mandatory constraint
  int16_t av[DL_NV];
  uint8_t vcl[DL_NV];  // choice lists per variable (DP_FMT_P16)
  int32_t fb;  // the host lowers this problem
  int32_t big;  // a bound or row length past the packed forms'
  int32_t p16;  // the rows do not imply the choice lists: DP_FMT_P16
};

__device__ __forceinline__ uint64_t lt_mask() { return (1ull << __lane_id()) - 1ull; }
__device__ __forceinline__ int excl_scan(int x, int& total) {
  int y = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(y, d);
    if (__lane_id() >= d) y += t;
  }
  total = __shfl(y, 63);
  return y - x;
}

// dp_rec_fits16 (include/deppy_hip.h), on the device
__device__ __forceinline__ bool fits16_dev(const int32_t* h) {
  const int32_t nv = h[DP_H_NV];
  return h[DP_H_WORDS] < 65000 && nv < 16000 && h[DP_H_NID] < 65000 && h[DP_H_NC] + h[DP_H_NK] + 64 + nv < 65000 &&
         h[DP_H_NA] + h[DP_H_NCH] < 65000 && h[DP_H_NCL] + h[DP_H_NKL] < 65000;
}

struct DlArgs {
  // the batch's dp_wire32 ranges on the device
  const int32_t *pvo, *pco, *pao, *vid, *ckn, *arg;
  const uint16_t *vnc, *cna, *vid16, *arg16;  // (16-bit string indices when ids16)
  int32_t ids16;
  int32_t pbase, cbase, abase;  // absolute index of each range's first element
  int32_t nvars, ncons, nargs;
  int64_t n_strs;
  int64_t group_above;  // placement.hpp one_wave's bound
  int32_t p0;           // first problem of this launch
  int32_t* words;  // [P] padded record words, 0: lowered on the host
  int32_t* nid;    // [P]
  int32_t* slots;  // [P * DL_SLOT]
  int32_t* ivs;    // [P * DL_C] identity -> variable (last writer)
  int32_t* ics;    // [P * DL_C] identity -> constraint index within the variable
};

__global__ void __launch_bounds__(DL_T) lower_kernel(DlArgs a) {
  __shared__ DlShared S;
  const int p = a.p0 + (int)blockIdx.x;
  const int lane = (int)threadIdx.x;
  auto give_up = [&]() {
    if (lane == 0) {
      a.words[p] = 0;
      a.nid[p] = 0;
    }
  };
  const int v0 = a.pvo[p] - a.pbase, v1 = a.pvo[p + 1] - a.pbase;
  const int nv = v1 - v0;
  if (nv <= 0 || nv > DL_NV || v0 < 0 || v1 > a.nvars) return give_up();
  const int cb = a.pco[p] - a.cbase, ce = a.pco[p + 1] - a.cbase;
  const int C = ce - cb;
  if (cb < 0 || C < 0 || ce > a.ncons || C > DL_C) return give_up();
  const int ab = a.pao[p] - a.abase, ae = a.pao[p + 1] - a.abase;
  const int A = ae - ab;
  if (ab < 0 || A < 0 || ae > a.nargs || A > DL_A) return give_up();
  // the counts -> offsets within the problem (their sums must be C and A)
  {
    int run = 0;
    for (int i0 = 0; i0 < nv && run <= C; i0 += DL_T) {
      const int i = i0 + lane;
      int tot;
      const int ex = excl_scan(i < nv ? (int)a.vnc[v0 + i] : 0, tot);
      if (i < nv) S.vstart[i] = (int16_t)min(run + ex, 0x7fff);
      run += tot;
    }
    int arun = 0;
    for (int c0 = 0; c0 < C && arun <= A; c0 += DL_T) {
      const int c = c0 + lane;
      int tot;
      const int ex = excl_scan(c < C ? (int)a.cna[cb + c] : 0, tot);
      if (c < C) S.castart[c] = (int16_t)min(arun + ex, 0x7fff);
      arun += tot;
    }
    if (run != C || arun != A) return give_up();  // inconsistent counts: the host reports them
    if (lane == 0) {
      S.vstart[nv] = (int16_t)C;
      S.castart[C] = (int16_t)A;
    }
  }

  // ---- 0. tables ----
  for (int i = lane; i < DL_VH; i += DL_T) S.vkey[i] = 0;
  for (int i = lane; i < DL_KH; i += DL_T) {
    S.kkey[i] = 0ull;
    S.kfirst[i] = 0x7fffffff;
    S.klast[i] = -1;
  }
  for (int i = lane; i < DL_C / 32; i += DL_T) S.mask[i] = 0;
  for (int i = lane; i < DL_NV / 32; i += DL_T) S.aflag[i] = 0;
  if (lane == 0) {
    S.fb = 0;
    S.big = 0;
    S.p16 = 0;
  }
  __syncthreads();

  // ---- 1. identifiers -> variables (lit_mapping.go:50-57) ----
  for (int i = lane; i < nv; i += DL_T) {
    const int32_t sid = a.ids16 ? (int32_t)a.vid16[v0 + i] : a.vid[v0 + i];
    if (sid < 0 || (int64_t)sid >= a.n_strs) {
      S.fb = 1;  // malformed: the host reports it
      continue;
    }
    for (int c = S.vstart[i], c1 = S.vstart[i] + (int)a.vnc[v0 + i]; c < c1; ++c) S.cs[c] = (int16_t)i;
    uint32_t h = ((uint32_t)sid * 2654435761u) >> 22;  // log2(DL_VH) bits
    for (;;) {
      const int32_t old = atomicCAS(&S.vkey[h], 0, sid + 1);
      if (old == 0) {
        S.vval[h] = (int16_t)i;
        break;
      }
      if (old == sid + 1) {  // DuplicateIdentifier: the host reports it
        S.fb = 1;
        break;
      }
      h = (h + 1) & (DL_VH - 1);
    }
  }
  __syncthreads();
  if (S.fb) return give_up();
  // arguments (LitOf, lit_mapping.go:81-88: an unknown one is an error the host reports)
  for (int j = lane; j < A; j += DL_T) {
    const int32_t sid = a.ids16 ? (int32_t)a.arg16[ab + j] : a.arg[ab + j];
    if (sid < 0 || (int64_t)sid >= a.n_strs) {
      S.fb = 1;
      continue;
    }
    uint32_t h = ((uint32_t)sid * 2654435761u) >> 22;
    int v = -1;
    for (;;) {
      const int32_t k = S.vkey[h];
      if (k == sid + 1) {
        v = S.vval[h];
        break;
      }
      if (k == 0) break;
      h = (h + 1) & (DL_VH - 1);
    }
    if (v < 0) S.fb = 1;
    S.ca[j] = (int16_t)v;
  }
  __syncthreads();
  if (S.fb) return give_up();

  // ---- 2. identity keys (lower.cpp lower_fast's switch) ----
  for (int c = lane; c < C; c += DL_T) {
    const int32_t kn = a.ckn[cb + c];
    const int kind = kn & 7;
    const int n = kn >> 3;
    const int a0 = S.castart[c], a1 = S.castart[c + 1];
    const int ns = a1 - a0;
    const int vi = S.cs[c];
    bool bad = a0 < 0 || a1 > A || ns < 0;
    uint64_t key = 0;
    uint32_t m = 0;
    if (!bad) {
      if (kind == DP_DEPENDENCY && ns > 0) {
        if (ns + 1 > 255) {
          bad = true;
        } else if (S.ca[a0] == vi) {
          // Or(~x_s, x_s) = T: a choice list with no identity and no row
          // (lower.cpp: list_id -1); the lists are then not implied by the
          // rows, so the record is DP_FMT_P16 with the lists explicit
          m = meta(RT_SKIP, false, true, kind, 0);
          S.p16 = 1;
        } else {
          // the row (~s, d1..dn), each candidate once; s among the later
          // candidates folds the row to T while the identity stays (not a
          // packed form: the host)
          uint64_t h = hmix(0x646570ULL, (uint64_t)vi);
          int len = 1;
          for (int j = 0; j < ns && !bad; ++j) {
            const int d = S.ca[a0 + j];
            bad = d == vi;
            bool rep = false;
            for (int q = 0; q < j && !rep; ++q) rep = S.ca[a0 + q] == d;
            len += rep ? 0 : 1;
            h = hmix(h, (uint64_t)d);
          }
          if (len < ns + 1) S.p16 = 1;  // a repeated candidate: the row is shorter than its list
          key = keyh(K_DEP, h);
          m = meta(RT_CLAUSE, true, true, kind, len);
        }
      } else {
        switch (kind) {
          case DP_MANDATORY:
            bad = ns != 0;
            key = key1(K_POS, (uint32_t)vi);
            m = meta(RT_CLAUSE, false, false, kind, 1);
            atomicOr(&S.aflag[vi >> 5], 1u << (vi & 31));
            break;
          case DP_PROHIBITED:
            bad = ns != 0;
            key = key1(K_NEG, (uint32_t)vi);
            m = meta(RT_CLAUSE, false, false, kind, 1);
            break;
          case DP_DEPENDENCY:  // without candidates: ~x_s
            key = key1(K_NEG, (uint32_t)vi);
            m = meta(RT_CLAUSE, false, false, kind, 1);
            break;
          case DP_CONFLICT: {
            bad = ns != 1;
            if (bad) break;
            const int t = S.ca[a0];
            if (t == vi) {
              key = key1(K_NEG, (uint32_t)vi);
              m = meta(RT_CLAUSE, false, false, kind, 1);
            } else {
              key = key2(K_CONF, (uint32_t)vi, (uint32_t)t);
              m = meta(RT_CLAUSE, false, false, kind, 2);
            }
            break;
          }
          case DP_ATMOST: {
            if (n < 0) {
              key = key1(K_F, 0);
              m = meta(RT_CLAUSE, false, false, kind, 0);
              break;
            }
            if (n >= ns) {  // T: no identity
              m = meta(RT_SKIP, false, false, kind, 0);
              break;
            }
            for (int j = 1; j < ns && !bad; ++j)  // a repeated variable: the exact path
              for (int q = 0; q < j && !bad; ++q) bad = S.ca[a0 + q] == S.ca[a0 + j];
            if (bad) break;
            if (ns > 255 || n > 255) S.big = 1;
            if (ns == 1) {
              key = key1(K_NEG, (uint32_t)S.ca[a0]);
              m = meta(RT_CLAUSE, false, false, kind, 1);
            } else if (ns == 2) {
              key = key2(n == 0 ? K_NOR : K_CONF, (uint32_t)S.ca[a0], (uint32_t)S.ca[a0 + 1]);
              m = meta(RT_CARD, false, false, kind, 2);
            } else {
              // the set, order-free (an equal key is checked against the
              // first writer's sequence in order, as lower.cpp same_term)
              uint64_t s1 = 0, s2 = 0;
              for (int j = 0; j < ns; ++j) {
                const uint64_t x = (uint64_t)S.ca[a0 + j];
                s1 += hmix(0x1234ULL, x);
                s2 ^= hmix(0x5678ULL, x);
              }
              key = keyh(K_CARD, hmix(hmix(hmix(0x63617264ULL, (uint64_t)n), s1), s2 ^ (uint64_t)ns));
              m = meta(RT_CARD, true, false, kind, ns);
            }
            break;
          }
          default:
            bad = true;
        }
      }
    }
    if (bad) {
      S.fb = 1;
      continue;
    }
    S.cmeta[c] = m;
    if (m_rt(m) == RT_SKIP) {
      S.cslot[c] = -1;
      continue;
    }
    const unsigned long long kv1 = (unsigned long long)key + 1ull;
    uint32_t s = (uint32_t)hmix(key, 0) & (DL_KH - 1);
    for (;;) {
      const unsigned long long old = atomicCAS(&S.kkey[s], 0ull, kv1);
      if (old == 0ull || old == kv1) break;
      s = (s + 1) & (DL_KH - 1);
    }
    atomicMin(&S.kfirst[s], c);
    atomicMax(&S.klast[s], c);
    S.cslot[c] = (int16_t)s;
  }
  __syncthreads();
  if (S.fb || S.big) return give_up();

  // ---- 3. numbering in constraint order ----
  int nid = 0, nc = 0, ncl = 0, nk = 0, nkl = 0, nch = 0, nchl = 0;
  bool b1 = true, nib = true;
  for (int c0 = 0; c0 < C; c0 += DL_T) {
    const int c = c0 + lane;
    const bool act = c < C;
    const uint32_t m = act ? S.cmeta[c] : 0u;
    const int s = act ? S.cslot[c] : -1;
    const int first = s >= 0 ? S.kfirst[s] : -1;
    const bool isf = s >= 0 && first == c;
    const int kind = m_kind(m);
    const int a0 = act ? S.castart[c] : 0;
    const int ns = act ? S.castart[c + 1] - a0 : 0;
    const int vi = act ? S.cs[c] : 0;
    // an equal hashed key names the same term only for the same subject
    // (Dependency), bound (AtMost) and sequence (lower.cpp same_term)
    bool bad = false;
    if (s >= 0 && !isf && m_hashed(m)) {
      const int f0 = S.castart[first], fns = S.castart[first + 1] - f0;
      bad = fns != ns || (kind == DP_DEPENDENCY && S.cs[first] != vi) ||
            (kind == DP_ATMOST && a.ckn[cb + first] != a.ckn[cb + c]) || m_kind(S.cmeta[first]) != kind;
      for (int j = 0; j < ns && !bad; ++j) bad = S.ca[f0 + j] != S.ca[a0 + j];
    }
    if (__ballot(bad)) {
      if (lane == 0) S.fb = 1;
      break;
    }
    // identities
    const uint64_t bf = __ballot(isf);
    const int id = nid + __popcll(bf & lt_mask());
    if (isf) S.cid[c] = (int16_t)id;
    nid += __popcll(bf);
    // rows
    const bool isc = isf && m_rt(m) == RT_CLAUSE, isk = isf && m_rt(m) == RT_CARD;
    const int rlen = m_len(m);
    int tot;
    const int crow = nc + __popcll(__ballot(isc) & lt_mask());
    const int cat = ncl + excl_scan(isc ? rlen : 0, tot);
    nc += __popcll(__ballot(isc));
    ncl += tot;
    const int krow = nk + __popcll(__ballot(isk) & lt_mask());
    const int kat = nkl + excl_scan(isk ? rlen : 0, tot);
    nk += __popcll(__ballot(isk));
    nkl += tot;
    // choice lists: one per Dependency with candidates (search.go:59-69)
    const bool isl = act && m_list(m);
    const int k = nch + __popcll(__ballot(isl) & lt_mask());
    if (isl) S.clist[c] = (int16_t)k;
    nch += __popcll(__ballot(isl));
    (void)excl_scan(isl ? ns : 0, tot);
    nchl += tot;
    __syncthreads();  // the chunk's cid / clist before their readers
    bool far = false;
    if (isl) {
      const int d = isf || s < 0 ? 0 : k - S.clist[first];
      far = d > 255;
      S.src[k] = (uint8_t)d;
    }
    if (__ballot(far) && lane == 0) S.p16 = 1;  // a repeat too far back for a source byte
    if (isc) {
      S.clen[crow] = (uint8_t)rlen;
      if (kind == DP_DEPENDENCY && ns > 0) {
        S.clit[cat] = (int16_t)(2 * vi + 1);
        for (int j = 0, o = 1; j < ns; ++j) {
          const int d = S.ca[a0 + j];
          bool rep = false;
          for (int q = 0; q < j && !rep; ++q) rep = S.ca[a0 + q] == d;
          if (!rep) S.clit[cat + o++] = (int16_t)(2 * d);
        }
      } else if (rlen == 1) {
        const uint64_t key = S.kkey[s] - 1ull;
        S.clit[cat] = (int16_t)(2 * (int)(key & 0x3fffffffULL) + ((key >> 60) == K_NEG ? 1 : 0));
      } else if (rlen == 2) {  // Conflict(a, b): (~a ~b)
        S.clit[cat] = (int16_t)(2 * vi + 1);
        S.clit[cat + 1] = (int16_t)(2 * S.ca[a0] + 1);
      }
    }
    bool kb1 = true;
    if (isk) {
      const int n = a.ckn[cb + c] >> 3;
      S.klen[krow] = (uint8_t)rlen;
      S.kb[krow] = (int16_t)n;
      kb1 = n == 1;
      for (int j = 0; j < ns; ++j) S.kv[kat + j] = S.ca[a0 + j];
      atomicOr(&S.mask[id >> 5], 1u << (id & 31));
    }
    b1 = b1 && __ballot(!kb1) == 0;
    nib = nib && __ballot((isc || isk) && rlen > 15) == 0;
    // the reported AppliedConstraint: the key's last writer
    if (isf) {
      const int last = S.klast[s];
      const int ov = S.cs[last];
      a.ivs[(int64_t)p * DL_C + id] = ov;
      a.ics[(int64_t)p * DL_C + id] = last - S.vstart[ov];
    }
  }
  __syncthreads();
  if (S.fb) return give_up();
  // anchors (lit_mapping.go:163-174): variables with a Mandatory, in order
  int na = 0;
  for (int i0 = 0; i0 < nv; i0 += DL_T) {
    const int i = i0 + lane;
    const bool f = i < nv && ((S.aflag[i >> 5] >> (i & 31)) & 1u);
    const uint64_t bm = __ballot(f);
    if (f) S.av[na + __popcll(bm & lt_mask())] = (int16_t)i;
    na += __popcll(bm);
  }

  // ---- 4. the record (lower.cpp emit_p16d + p8_plan / p8_write) ----
  int32_t h[DP_H_SIZE];
#pragma unroll
  for (int i = 0; i < DP_H_SIZE; ++i) h[i] = 0;
  h[DP_H_MAGIC] = DP_REC_MAGIC;
  h[DP_H_NV] = nv;
  h[DP_H_NC] = nc;
  h[DP_H_NK] = nk;
  h[DP_H_NCH] = nch;
  h[DP_H_NA] = na;
  h[DP_H_NID] = nid;
  h[DP_H_NCL] = ncl;
  h[DP_H_NKL] = nkl;
  h[DP_H_NCHL] = nchl;
  h[DP_H_WORDS] = DP_H_SIZE + (nc + 1) + ncl + nc + (nk + 1) + nkl + 2 * nk + (nv + 1) + (nch + 1) + nchl + na;
  // one wavefront per problem (placement.hpp lds_image)
  if (!fits16_dev(h) || (int64_t)dp::layout<dp::M_LDS>(h).lds_bytes > a.group_above) return give_up();
  auto put_header = [&]() {
    for (int i = lane; i < DL_SLOT; i += DL_T) S.rec[i] = 0u;
    __syncthreads();
    if (lane < DP_H_SIZE) {
      int32_t x = 0;
#pragma unroll
      for (int i = 0; i < DP_H_SIZE; ++i)
        if (i == lane) x = h[i];
      S.rec[lane] = (uint32_t)x;
    }
  };
  auto put_out = [&](int padded) {
    __syncthreads();
    int32_t* out = a.slots + (int64_t)p * DL_SLOT;
    for (int i = lane; i < padded; i += DL_T) out[i] = (int32_t)S.rec[i];
    if (lane == 0) {
      a.words[p] = padded;
      a.nid[p] = nid;
    }
  };
  if (S.p16) {
    // DP_FMT_P16, the choice lists explicit (lower.cpp narrow_last -> pack16
    // when the rows do not imply them)
    bool bad16 = false;
    for (int i = lane; i < nv; i += DL_T) {
      int cnt = 0;
      for (int c = S.vstart[i]; c < S.vstart[i + 1]; ++c) cnt += m_list(S.cmeta[c]) ? 1 : 0;
      bad16 = bad16 || cnt > 255;
      S.vcl[i] = (uint8_t)cnt;
    }
    const int tb = nc + nk + nv + nch + (nid + 7) / 8;
    const int at = (2 * (ncl + nkl + nk + nchl + na) + 15) & ~15;
    const int phys = DP_H_SIZE + (at + tb + 3) / 4, padded = (phys + 3) & ~3;
    if (__ballot(bad16) || tb > DP_P16_TAIL_MAX || padded > DL_SLOT) return give_up();
    h[DP_H_FMT] = DP_FMT_P16;
    put_header();
    uint16_t* const u = reinterpret_cast<uint16_t*>(S.rec + DP_H_SIZE);
    uint8_t* const t = reinterpret_cast<uint8_t*>(S.rec + DP_H_SIZE) + at;
    for (int j = lane; j < ncl; j += DL_T) u[j] = (uint16_t)S.clit[j];
    for (int j = lane; j < nkl; j += DL_T) u[ncl + j] = (uint16_t)S.kv[j];
    for (int j = lane; j < nk; j += DL_T) u[ncl + nkl + j] = (uint16_t)S.kb[j];
    // the lists in list (= constraint) order, each its Dependency's candidates
    int run = 0;
    for (int c0 = 0; c0 < C; c0 += DL_T) {
      const int c = c0 + lane;
      const bool isl = c < C && m_list(S.cmeta[c]);
      const int ns = isl ? S.castart[c + 1] - S.castart[c] : 0;
      int tot;
      const int ex = excl_scan(ns, tot);
      if (isl) {
        for (int j = 0; j < ns; ++j) u[ncl + nkl + nk + run + ex + j] = (uint16_t)S.ca[S.castart[c] + j];
        t[nc + nk + nv + S.clist[c]] = (uint8_t)ns;
      }
      run += tot;
    }
    for (int j = lane; j < na; j += DL_T) u[ncl + nkl + nk + nchl + j] = (uint16_t)S.av[j];
    for (int i = lane; i < nc; i += DL_T) t[i] = S.clen[i];
    for (int i = lane; i < nk; i += DL_T) t[nc + i] = S.klen[i];
    for (int i = lane; i < nv; i += DL_T) t[nc + nk + i] = S.vcl[i];
    for (int b = lane; b < ((nid + 7) >> 3); b += DL_T)
      t[nc + nk + nv + nch + b] = (uint8_t)(S.mask[b >> 2] >> ((b & 3) * 8));
    put_out(padded);
    return;
  }
  if ((int64_t)nc + nk + nch + (nid + 7) / 8 > DP_P16_TAIL_MAX) return give_up();  // P16D's tail bound
  const int f = (nv > 256 ? DP_P8_HI : 0) | (b1 ? DP_P8_B1 : 0) | (nib ? DP_P8_NIB : 0);
  const bool hi = f & DP_P8_HI;
  // dp_p8_layout_of
  int o = 0;
  const int L_cvar = o; o += ncl;
  const int L_kvar = o; o += nkl;
  const int L_avar = o; o += na;
  const int L_bound = o; o += b1 ? 0 : nk;
  const int L_neg = o; o += (ncl + 7) >> 3;
  const int L_chi = o; o += hi ? (ncl + 7) >> 3 : 0;
  const int L_khi = o; o += hi ? (nkl + 7) >> 3 : 0;
  const int L_ahi = o; o += hi ? (na + 7) >> 3 : 0;
  const int rows = nc + nk;
  const int L_lens = o; o += nib ? (rows + 1) / 2 : rows;
  const int L_srcnz = o; o += (nch + 7) >> 3;
  const int L_srcval = o;
  int nnz = 0;
  for (int k0 = 0; k0 < nch; k0 += DL_T) nnz += __popcll(__ballot(k0 + lane < nch && S.src[k0 + lane] != 0));
  const int L_mask = L_srcval + nnz;
  const int bytes = L_mask + ((nid + 7) >> 3);
  const int phys = DP_H_SIZE + (bytes + 3) / 4, padded = (phys + 3) & ~3;
  if (padded > DL_SLOT) return give_up();
  h[DP_H_FMT] = DP_FMT_P8D;
  h[DP_H_P8] = (int32_t)((uint32_t)f | ((uint32_t)bytes << 8));
  put_header();
  uint8_t* const rb = reinterpret_cast<uint8_t*>(S.rec + DP_H_SIZE);
  for (int j = lane; j < ncl; j += DL_T) rb[L_cvar + j] = (uint8_t)(S.clit[j] >> 1);
  for (int j = lane; j < nkl; j += DL_T) rb[L_kvar + j] = (uint8_t)S.kv[j];
  for (int j = lane; j < na; j += DL_T) rb[L_avar + j] = (uint8_t)S.av[j];
  if (!b1)
    for (int j = lane; j < nk; j += DL_T) rb[L_bound + j] = (uint8_t)S.kb[j];
  for (int jb = lane; jb < ((ncl + 7) >> 3); jb += DL_T) {
    uint32_t ng = 0, hb = 0;
    for (int q = 0; q < 8 && 8 * jb + q < ncl; ++q) {
      const int x = S.clit[8 * jb + q];
      ng |= (uint32_t)(x & 1) << q;
      hb |= (uint32_t)((x >> 9) & 1) << q;
    }
    rb[L_neg + jb] = (uint8_t)ng;
    if (hi) rb[L_chi + jb] = (uint8_t)hb;
  }
  if (hi) {
    for (int jb = lane; jb < ((nkl + 7) >> 3); jb += DL_T) {
      uint32_t hb = 0;
      for (int q = 0; q < 8 && 8 * jb + q < nkl; ++q) hb |= (uint32_t)((S.kv[8 * jb + q] >> 8) & 1) << q;
      rb[L_khi + jb] = (uint8_t)hb;
    }
    for (int jb = lane; jb < ((na + 7) >> 3); jb += DL_T) {
      uint32_t hb = 0;
      for (int q = 0; q < 8 && 8 * jb + q < na; ++q) hb |= (uint32_t)((S.av[8 * jb + q] >> 8) & 1) << q;
      rb[L_ahi + jb] = (uint8_t)hb;
    }
  }
  auto len = [&](int i) { return i < nc ? (int)S.clen[i] : (int)S.klen[i - nc]; };
  if (nib) {
    for (int i = lane; i < (rows + 1) / 2; i += DL_T)
      rb[L_lens + i] = (uint8_t)(len(2 * i) | (2 * i + 1 < rows ? len(2 * i + 1) << 4 : 0));
  } else {
    for (int i = lane; i < rows; i += DL_T) rb[L_lens + i] = (uint8_t)len(i);
  }
  for (int jb = lane; jb < ((nch + 7) >> 3); jb += DL_T) {
    uint32_t b = 0;
    for (int q = 0; q < 8 && 8 * jb + q < nch; ++q) b |= (uint32_t)(S.src[8 * jb + q] != 0) << q;
    rb[L_srcnz + jb] = (uint8_t)b;
  }
  int q = 0;
  for (int k0 = 0; k0 < nch; k0 += DL_T) {
    const int k = k0 + lane;
    const bool nz = k < nch && S.src[k] != 0;
    const uint64_t bm = __ballot(nz);
    if (nz) rb[L_srcval + q + __popcll(bm & lt_mask())] = S.src[k];
    q += __popcll(bm);
  }
  for (int b = lane; b < ((nid + 7) >> 3); b += DL_T) rb[L_mask + b] = (uint8_t)(S.mask[b >> 2] >> ((b & 3) * 8));
  put_out(padded);
}

// Record and identity offsets of problems [q0, q1): one workgroup, a
// contiguous segment per thread, continuing from rec_off[q0] / ident_off[q0]
// (the previous piece's, on the same stream; 0 for the first).
constexpr int SCAN_T = 1024;
__global__ void __launch_bounds__(SCAN_T) scan_kernel(const int32_t* words, const int32_t* nid, int32_t q0, int32_t q1,
                                                     int64_t* rec_off, int64_t* ident_off) {
  __shared__ int64_t sw[SCAN_T], si[SCAN_T];
  const int t = (int)threadIdx.x;
  const int n = q1 - q0;
  const int seg = (n + SCAN_T - 1) / SCAN_T;
  const int b = q0 + min(n, t * seg), e = min(q1, b + seg);
  int64_t w = 0, d = 0;
  for (int i = b; i < e; ++i) {
    w += words[i];
    d += nid[i];
  }
  sw[t] = w;
  si[t] = d;
  __syncthreads();
  for (int s = 1; s < SCAN_T; s <<= 1) {
    const int64_t xw = t >= s ? sw[t - s] : 0, xd = t >= s ? si[t - s] : 0;
    __syncthreads();
    sw[t] += xw;
    si[t] += xd;
    __syncthreads();
  }
  const int64_t w0 = q0 ? rec_off[q0] : 0, d0 = q0 ? ident_off[q0] : 0;
  w = w0 + sw[t] - w;
  d = d0 + si[t] - d;
  __syncthreads();  // (every thread read the bases before any writes)
  if (t == 0 && q0 == 0) {
    rec_off[0] = 0;
    ident_off[0] = 0;
  }
  for (int i = b; i < e; ++i) {
    w += words[i];
    d += nid[i];
    rec_off[i + 1] = w;
    ident_off[i + 1] = d;
  }
}

// The slots of problems p0.. packed into the batch (records 16-byte aligned,
// as every offset is): device memory, or the caller's page-locked host
// memory through its device mapping (the copy back is the kernel's writes).
__global__ void __launch_bounds__(DL_T) pack_kernel(int32_t p0, const int32_t* words, const int32_t* nid,
                                                    const int32_t* slots, const int32_t* ivs, const int32_t* ics,
                                                    const int64_t* rec_off, const int64_t* ident_off, int32_t* rec,
                                                    int32_t* ivar, int32_t* icon) {
  const int p = p0 + (int)blockIdx.x, lane = (int)threadIdx.x;
  const int w4 = words[p] >> 2;
  const int4* s = reinterpret_cast<const int4*>(slots + (int64_t)p * DL_SLOT);
  int4* d = reinterpret_cast<int4*>(rec + rec_off[p]);
  for (int i = lane; i < w4; i += DL_T) d[i] = s[i];
  const int n = nid[p];
  const int64_t io = ident_off[p];
  for (int i = lane; i < n; i += DL_T) {
    ivar[io + i] = ivs[(int64_t)p * DL_C + i];
    icon[io + i] = ics[(int64_t)p * DL_C + i];
  }
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t need(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t c = std::max<size_t>(n + n / 8, 256);
    const hipError_t e = hipMalloc(&p, c * sizeof(T));
    if (e == hipSuccess) cap = c;
    return e;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

struct dp_dlower {
  int dev = 0;
  hipStream_t st = nullptr;   // kernels and the copies back
  hipStream_t cst = nullptr;  // the wire's copies to the device
  hipStream_t pst = nullptr;  // the packing (its writes to host memory run under the next piece's lowering)
  static constexpr int kMaxPieces = 8;
  hipEvent_t ev[kMaxPieces] = {}, es[kMaxPieces] = {};
  DevBuf<int32_t> pvo, pco, pao, vid, ckn, arg, words, nid, slots, ivs, ics, rec, ivar, icon;
  DevBuf<uint16_t> vnc, cna, vid16, arg16;
  DevBuf<int64_t> ro, io;
  int64_t* h_off = nullptr;  // page-locked: rec_off then ident_off
  size_t h_cap = 0;
  int64_t host_count = 0;
  // the problems lowered on the host, as a dp_wire of their own
  std::vector<int32_t> which;
  std::vector<int64_t> s_pvo, s_vid, s_vco, s_cao, s_arg;
  std::vector<int32_t> s_kind, s_cn;
  std::vector<uint8_t> s_bad;
  std::vector<int64_t> s_sz, s_off;
  std::mutex mu;  // one call at a time
  ~dp_dlower() {
    if (h_off) dp::pinned_free(h_off);
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : es)
      if (e) (void)hipEventDestroy(e);
    if (pst) (void)hipStreamDestroy(pst);
    if (st) (void)hipStreamDestroy(st);
    if (cst) (void)hipStreamDestroy(cst);
  }
};

namespace {
std::string hip_err(const char* what, hipError_t e) { return std::string("dp_lower_device: ") + what + ": " + hipGetErrorString(e); }
#define DL_OK(expr)                                  \
  do {                                               \
    const hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) {                          \
      dp::set_global_error(hip_err(#expr, e_));      \
      return -1;                                     \
    }                                                \
  } while (0)

// The problems d->which of w as a dp_wire of their own (64-bit, offsets
// from 0).  Inconsistent counts stay malformed (a negative identifier), so
// the host lowering reports the batch as dp_lower_into does.
void host_subwire(dp_dlower* d, const dp_wire32* w, dp_wire* sub) {
  const int64_t nw = (int64_t)d->which.size();
  dp::Pool& pool = dp::host_pool();
  // (a few large problems still spread over the pool: config 4's catalogs)
  const int64_t blk = std::max<int64_t>(1, std::min<int64_t>(64, nw / (4 * (int64_t)pool.size())));
  // sizes (on the host pool): a problem whose counts do not add up to its
  // ranges becomes one malformed variable
  std::vector<int64_t>& sz = d->s_sz;  // [3 nw]: variables, constraints, arguments
  sz.resize((size_t)(3 * nw + 3));
  std::vector<uint8_t>& bad = d->s_bad;
  bad.assign((size_t)nw, 0);
  pool.run(nw, std::function<void(int64_t)>([&](int64_t i) {
    const int32_t p = d->which[(size_t)i];
    const int32_t v0 = w->prob_var_off[p], v1 = w->prob_var_off[p + 1];
    const int64_t c0 = w->prob_con_off[p], ce = w->prob_con_off[p + 1];
    const int64_t x0 = w->prob_arg_off[p], xe = w->prob_arg_off[p + 1];
    int64_t sc = 0, sx = 0;
    for (int32_t v = v0; v < v1; ++v) sc += w->var_ncon[v];
    if (sc == ce - c0)
      for (int64_t k = c0; k < ce; ++k) sx += w->con_nargs[k];
    const bool b = sc != ce - c0 || sx != xe - x0;
    bad[(size_t)i] = b;
    sz[(size_t)(3 * i)] = b ? std::max(1, v1 - v0) : v1 - v0;
    sz[(size_t)(3 * i + 1)] = b ? 0 : ce - c0;
    sz[(size_t)(3 * i + 2)] = b ? 0 : xe - x0;
  }), blk);
  // offsets (serial), then the arrays (on the pool)
  std::vector<int64_t>& off = d->s_off;  // [3 (nw+1)]
  off.resize((size_t)(3 * nw + 3));
  off[0] = off[1] = off[2] = 0;
  for (int64_t i = 0; i < nw; ++i)
    for (int q = 0; q < 3; ++q) off[(size_t)(3 * (i + 1) + q)] = off[(size_t)(3 * i + q)] + sz[(size_t)(3 * i + q)];
  const int64_t tv = off[(size_t)(3 * nw)], tc = off[(size_t)(3 * nw + 1)], ta = off[(size_t)(3 * nw + 2)];
  d->s_pvo.resize((size_t)nw + 1);
  d->s_vid.resize((size_t)tv + 1);
  d->s_vco.resize((size_t)tv + 1);
  d->s_kind.resize((size_t)tc + 1);
  d->s_cn.resize((size_t)tc + 1);
  d->s_cao.resize((size_t)tc + 1);
  d->s_arg.resize((size_t)ta + 1);
  int64_t* const pvo = d->s_pvo.data();
  int64_t* const vid = d->s_vid.data();
  int64_t* const vco = d->s_vco.data();
  int32_t* const kind = d->s_kind.data();
  int32_t* const cn = d->s_cn.data();
  int64_t* const cao = d->s_cao.data();
  int64_t* const arg = d->s_arg.data();
  for (int64_t i = 0; i <= nw; ++i) pvo[i] = off[(size_t)(3 * i)];
  pool.run(nw, std::function<void(int64_t)>([&](int64_t i) {
    const int32_t p = d->which[(size_t)i];
    const int32_t v0 = w->prob_var_off[p], v1 = w->prob_var_off[p + 1];
    int64_t nv = off[(size_t)(3 * i)], nc = off[(size_t)(3 * i + 1)], na = off[(size_t)(3 * i + 2)];
    if (bad[(size_t)i]) {
      for (int32_t v = v0; v < std::max(v1, v0 + 1); ++v) {
        vid[nv] = -1;  // (a negative identifier: dp_lower_into reports the batch malformed)
        vco[nv++] = nc;
      }
      return;
    }
    int64_t c = w->prob_con_off[p];
    const int64_t xb = w->prob_arg_off[p];
    int64_t x = 0;
    for (int32_t v = v0; v < v1; ++v) {
      vid[nv] = w->var_id16 ? (int64_t)w->var_id16[v] : (int64_t)w->var_id[v];
      vco[nv++] = nc;
      for (int32_t k = 0; k < (int32_t)w->var_ncon[v]; ++k, ++c) {
        const int32_t kn = w->con_kn[c];
        kind[nc] = kn & 7;
        cn[nc] = kn >> 3;
        cao[nc++] = na;
        for (int32_t j = 0; j < (int32_t)w->con_nargs[c]; ++j, ++x)
          arg[na++] = w->con_arg16 ? (int64_t)w->con_arg16[xb + x] : (int64_t)w->con_arg[xb + x];
      }
    }
  }), blk);
  vco[tv] = tc;
  cao[tc] = ta;
  sub->n_problems = (int32_t)nw;
  sub->prob_var_off = pvo;
  sub->var_id = vid;
  sub->var_con_off = vco;
  sub->con_kind = kind;
  sub->con_n = cn;
  sub->con_arg_off = cao;
  sub->con_arg = arg;
  sub->n_strs = w->n_strs;
  sub->str_off = w->str_off;
  sub->str_bytes = w->str_bytes;
  sub->interned = 1;
}

// The whole batch on the host (flags the kernel does not emit).
int lower_on_host(const dp_wire32* w, int32_t flags, dp_lowered* lw, dp_dlower* d) {
  d->which.resize((size_t)w->n_problems);
  for (int32_t p = 0; p < w->n_problems; ++p) d->which[(size_t)p] = p;
  dp_wire sub{};
  host_subwire(d, w, &sub);
  d->host_count = w->n_problems;
  return dp_lower_into(&sub, flags, lw);
}

double dl_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// DEPPY_DL_TIMES=1 (diagnostic): each call's phases on stderr
bool dl_times() {
  static const bool on = [] {
    const char* e = std::getenv("DEPPY_DL_TIMES");
    return e && *e && *e != '0';
  }();
  return on;
}

bool monotone(const int32_t* o, int32_t P) {
  if (!o || o[0] < 0) return false;
  for (int32_t p = 0; p < P; ++p)
    if (o[p + 1] < o[p]) return false;
  return true;
}
}  // namespace

// The packing's stream at the highest priority: a queue of its own, so its
// writes to host memory run beside the next piece's lowering instead of
// behind it (DEPPY_DL_PACK_PRIORITY=0: a normal stream, A/B).
hipError_t dl_pack_stream(hipStream_t* s) {
  const char* e = std::getenv("DEPPY_DL_PACK_PRIORITY");
  int lo = 0, hi = 0;
  if ((e && *e == '0') || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess)
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
}

extern "C" {

dp_dlower* dp_dlower_new(dp_ctx* ctx) {
  const int dev = dp::ctx_first_ordinal(ctx);
  if (dev < 0) {
    dp::set_global_error("dp_dlower_new: no context");
    return nullptr;
  }
  auto* d = new dp_dlower;
  d->dev = dev;
  bool ok = hipSetDevice(dev) == hipSuccess && hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&d->cst, hipStreamNonBlocking) == hipSuccess &&
            dl_pack_stream(&d->pst) == hipSuccess;
  for (auto& e : d->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  for (auto& e : d->es) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    dp::set_global_error("dp_dlower_new: stream creation failed");
    delete d;
    return nullptr;
  }
  return d;
}

void dp_dlower_free(dp_dlower* d) { delete d; }
int64_t dp_dlower_host_count(const dp_dlower* d) { return d ? d->host_count : 0; }

int dp_lower_device(dp_dlower* d, const dp_wire32* w, int32_t flags, dp_lowered* lw) {
  if (!d || !lw || !w || w->n_problems < 0 || !monotone(w->prob_var_off, w->n_problems) ||
      !monotone(w->prob_con_off, w->n_problems) || !monotone(w->prob_arg_off, w->n_problems)) {
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  std::lock_guard<std::mutex> lk(d->mu);
  const double t0 = dl_ms();
  const int32_t P = w->n_problems;
  const bool ours = (flags & (DP_LOWER_NARROW | DP_LOWER_PACKED)) == (DP_LOWER_NARROW | DP_LOWER_PACKED) &&
                    !(flags & DP_LOWER_NO_P8) && dp::ldsg_env() != dp::LDSG_ALWAYS && P > 0;
  if (!ours) return lower_on_host(w, flags, lw, d);
  // problems past the kernel's sizes are lowered on the host: when they
  // hold most of the batch's arguments, the whole batch is (a device pass and
  // a splice would only add to the host's work)
  {
    int64_t fit_args = 0, all_args = (int64_t)w->prob_arg_off[P] - w->prob_arg_off[0];
    for (int32_t p = 0; p < P; ++p) {
      const int32_t nv = w->prob_var_off[p + 1] - w->prob_var_off[p];
      const int32_t nc = w->prob_con_off[p + 1] - w->prob_con_off[p];
      const int32_t na = w->prob_arg_off[p + 1] - w->prob_arg_off[p];
      if (nv >= 1 && nv <= DL_NV && nc <= DL_C && na <= DL_A) fit_args += na + 1;
    }
    if (2 * fit_args < all_args + P) return lower_on_host(w, flags, lw, d);
  }
  const int32_t pv0 = w->prob_var_off[0], cb0 = w->prob_con_off[0], ab0 = w->prob_arg_off[0];
  const int32_t nvars = w->prob_var_off[P] - pv0, ncons = w->prob_con_off[P] - cb0, nargs = w->prob_arg_off[P] - ab0;
  const bool ids16 = w->var_id16 != nullptr;
  if ((nvars > 0 && (!(ids16 ? (const void*)w->var_id16 : (const void*)w->var_id) || !w->var_ncon)) ||
      (ncons > 0 && (!w->con_kn || !w->con_nargs)) ||
      (nargs > 0 && !(ids16 ? (const void*)w->con_arg16 : (const void*)w->con_arg)) ||
      (ids16 && w->n_strs > 65536)) {
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  DL_OK(hipSetDevice(d->dev));
  DL_OK(d->pvo.need((size_t)P + 1));
  DL_OK(d->pco.need((size_t)P + 1));
  DL_OK(d->pao.need((size_t)P + 1));
  if (ids16) {
    DL_OK(d->vid16.need((size_t)nvars + 1));
    DL_OK(d->arg16.need((size_t)nargs + 1));
  } else {
    DL_OK(d->vid.need((size_t)nvars + 1));
    DL_OK(d->arg.need((size_t)nargs + 1));
  }
  DL_OK(d->vnc.need((size_t)nvars + 1));
  DL_OK(d->ckn.need((size_t)ncons + 1));
  DL_OK(d->cna.need((size_t)ncons + 1));
  DL_OK(d->words.need((size_t)P));
  DL_OK(d->nid.need((size_t)P));
  DL_OK(d->slots.need((size_t)P * DL_SLOT));
  DL_OK(d->ivs.need((size_t)P * DL_C));
  DL_OK(d->ics.need((size_t)P * DL_C));
  DL_OK(d->ro.need((size_t)P + 1));
  DL_OK(d->io.need((size_t)P + 1));
  if (d->h_cap < 2 * ((size_t)P + 1)) {
    if (d->h_off) dp::pinned_free(d->h_off);
    d->h_cap = 2 * ((size_t)P + 1) + P / 4;
    d->h_off = static_cast<int64_t*>(dp::pinned_alloc(d->h_cap * sizeof(int64_t)));
    if (!d->h_off) {
      d->h_cap = 0;
      dp::set_global_error("dp_lower_device: page-locked allocation failed");
      return -1;
    }
  }
  hipStream_t st = d->st, cst = d->cst;
  auto h2d = [&](auto* dst, const auto* src, int64_t n) {
    return n > 0 ? hipMemcpyAsync(dst, src, (size_t)n * sizeof(*src), hipMemcpyHostToDevice, cst) : hipSuccess;
  };
  DL_OK(h2d(d->pvo.p, w->prob_var_off, (int64_t)P + 1));
  DL_OK(h2d(d->pco.p, w->prob_con_off, (int64_t)P + 1));
  DL_OK(h2d(d->pao.p, w->prob_arg_off, (int64_t)P + 1));
  DlArgs a{};
  a.pvo = d->pvo.p;
  a.pco = d->pco.p;
  a.pao = d->pao.p;
  a.vid = d->vid.p;
  a.vnc = d->vnc.p;
  a.ckn = d->ckn.p;
  a.cna = d->cna.p;
  a.arg = d->arg.p;
  a.vid16 = d->vid16.p;
  a.arg16 = d->arg16.p;
  a.ids16 = ids16 ? 1 : 0;
  a.pbase = pv0;
  a.cbase = cb0;
  a.abase = ab0;
  a.nvars = nvars;
  a.ncons = ncons;
  a.nargs = nargs;
  a.n_strs = w->n_strs;
  a.group_above = dp::group_above();
  a.words = d->words.p;
  a.nid = d->nid.p;
  a.slots = d->slots.p;
  a.ivs = d->ivs.p;
  a.ics = d->ics.p;
  // Every size bounded from the batch's totals (a record's words: at most
  // 23 + (2 (args + constraints) + 2 variables + 4 constraints) / 4, an
  // identity per constraint), so the result is sized before the kernels run
  // and each piece is packed straight into place.
  const int64_t bound_words = 24 * (int64_t)P + (2 * ((int64_t)nargs + ncons) + 2 * (int64_t)nvars + 4 * (int64_t)ncons) / 4;
  const dp::LoweredOut O = dp::lowered_prepare(lw, P, bound_words, (int64_t)ncons + 1, (flags & DP_LOWER_PINNED) != 0);
  // page-locked results are written by the pack kernel through their device
  // mapping; otherwise into device buffers and copied back
  int32_t *trec = nullptr, *tivar = nullptr, *ticon = nullptr;
  if (flags & DP_LOWER_PINNED) {
    void *r = nullptr, *iv = nullptr, *ic = nullptr;
    if (hipHostGetDevicePointer(&r, O.rec, 0) == hipSuccess && hipHostGetDevicePointer(&iv, O.ivar, 0) == hipSuccess &&
        hipHostGetDevicePointer(&ic, O.icon, 0) == hipSuccess) {
      trec = static_cast<int32_t*>(r);
      tivar = static_cast<int32_t*>(iv);
      ticon = static_cast<int32_t*>(ic);
    }
    (void)hipGetLastError();
  }
  const bool mapped = trec != nullptr;
  if (!mapped) {
    DL_OK(d->rec.need((size_t)bound_words + 4));
    DL_OK(d->ivar.need((size_t)ncons + 1));
    DL_OK(d->icon.need((size_t)ncons + 1));
    trec = d->rec.p;
    tivar = d->ivar.p;
    ticon = d->icon.p;
  }
  // pieces: the wire's copy of piece k+1 runs under the lowering and packing
  // of piece k.  Every copy and its event is enqueued first: an event marker
  // may share a hardware queue with the packing's stream, and one enqueued
  // after pack(k) would hold lower(k+1) behind it.
  const int pieces = (int)std::min<int64_t>(dp_dlower::kMaxPieces, std::max<int64_t>(1, P / 2048));
  auto piece = [&](int k, int32_t& q0, int32_t& q1) {
    q0 = (int32_t)((int64_t)P * k / pieces);
    q1 = (int32_t)((int64_t)P * (k + 1) / pieces);
  };
  for (int k = 0; k < pieces; ++k) {
    int32_t q0, q1;
    piece(k, q0, q1);
    const int32_t v0 = w->prob_var_off[q0], v1 = w->prob_var_off[q1];
    const int32_t c0 = w->prob_con_off[q0], c1 = w->prob_con_off[q1];
    const int32_t x0 = w->prob_arg_off[q0], x1 = w->prob_arg_off[q1];
    if (ids16) DL_OK(h2d(d->vid16.p + (v0 - pv0), w->var_id16 + v0, v1 - v0));
    else DL_OK(h2d(d->vid.p + (v0 - pv0), w->var_id + v0, v1 - v0));
    DL_OK(h2d(d->vnc.p + (v0 - pv0), w->var_ncon + v0, v1 - v0));
    DL_OK(h2d(d->ckn.p + (c0 - cb0), w->con_kn + c0, c1 - c0));
    DL_OK(h2d(d->cna.p + (c0 - cb0), w->con_nargs + c0, c1 - c0));
    if (ids16) DL_OK(h2d(d->arg16.p + (x0 - ab0), w->con_arg16 + x0, x1 - x0));
    else DL_OK(h2d(d->arg.p + (x0 - ab0), w->con_arg + x0, x1 - x0));
    DL_OK(hipEventRecord(d->ev[k], cst));
  }
  for (int k = 0; k < pieces; ++k) {
    int32_t q0, q1;
    piece(k, q0, q1);
    DL_OK(hipStreamWaitEvent(st, d->ev[k], 0));
    if (q1 == q0) continue;
    a.p0 = q0;
    hipLaunchKernelGGL(lower_kernel, dim3((unsigned)(q1 - q0)), dim3(DL_T), 0, st, a);
    DL_OK(hipGetLastError());
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(SCAN_T), 0, st, d->words.p, d->nid.p, q0, q1, d->ro.p, d->io.p);
    DL_OK(hipGetLastError());
    DL_OK(hipEventRecord(d->es[k], st));
    DL_OK(hipStreamWaitEvent(d->pst, d->es[k], 0));
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)(q1 - q0)), dim3(DL_T), 0, d->pst, q0, d->words.p, d->nid.p,
                       d->slots.p, d->ivs.p, d->ics.p, d->ro.p, d->io.p, trec, tivar, ticon);
    DL_OK(hipGetLastError());
  }
  int64_t* h_ro = d->h_off;
  int64_t* h_io = d->h_off + P + 1;
  DL_OK(hipMemcpyAsync(h_ro, d->ro.p, ((size_t)P + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  DL_OK(hipMemcpyAsync(h_io, d->io.p, ((size_t)P + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  DL_OK(hipStreamSynchronize(st));
  const double t_dev = dl_ms();
  const int64_t rw = h_ro[P], ni = h_io[P];
  std::memcpy(O.rec_off, h_ro, ((size_t)P + 1) * sizeof(int64_t));
  std::memcpy(O.ident_off, h_io, ((size_t)P + 1) * sizeof(int64_t));
  if (!mapped) {  // (after the packs, on their stream)
    if (rw) DL_OK(hipMemcpyAsync(O.rec, d->rec.p, (size_t)rw * sizeof(int32_t), hipMemcpyDeviceToHost, d->pst));
    if (ni) {
      DL_OK(hipMemcpyAsync(O.ivar, d->ivar.p, (size_t)ni * sizeof(int32_t), hipMemcpyDeviceToHost, d->pst));
      DL_OK(hipMemcpyAsync(O.icon, d->icon.p, (size_t)ni * sizeof(int32_t), hipMemcpyDeviceToHost, d->pst));
    }
  }
  // the problems the kernel left to the host, found while the copies run
  d->which.clear();
  for (int32_t p = 0; p < P; ++p)
    if (h_ro[p + 1] == h_ro[p]) d->which.push_back(p);
  d->host_count = (int64_t)d->which.size();
  DL_OK(hipStreamSynchronize(d->pst));
  const double t_pack = dl_ms();
  if (d->which.empty()) {
    if (dl_times()) std::fprintf(stderr, "dp_lower_device: P %d device %.3f pack %.3f ms\n", P, t_dev - t0, t_pack - t0);
    return 0;
  }
  dp_wire sub{};
  host_subwire(d, w, &sub);
  const double t_sub = dl_ms();
  if (dp::lowered_splice(lw, &sub, flags, d->which.data(), (int32_t)d->which.size()) != 0) {
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  if (dl_times())
    std::fprintf(stderr, "dp_lower_device: P %d device %.3f pack %.3f sub-wire %.3f splice %.3f ms (%d on the host)\n", P,
                 t_dev - t0, t_pack - t0, t_sub - t_pack, dl_ms() - t_sub, (int)d->which.size());
  return 0;
}

}  // extern "C"
