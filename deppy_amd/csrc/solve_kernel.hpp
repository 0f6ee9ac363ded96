// Batched pkg/sat resolution on MI355X (gfx950).
//
// Small catalogs (the batched hot path, M_LDS): one 64-lane wavefront owns one
// problem.  The problem's device image is narrowed to 16 bits into LDS and the
// whole solve runs out of LDS.  Large catalogs (config 4, M_SPLIT / M_HBM):
// one workgroup of BIG_WAVES wavefronts owns one problem; the int32 image is
// read in place from HBM, the hot per-variable state stays in LDS, and every
// data-parallel loop is spread over the whole workgroup.
//
//   base scope + BCP        pkg/sat/solve.go:63-79           (base_propagate)
//   preference search       pkg/sat/search.go:34-203         (search)
//   Solve() under scopes    search.go:167-169, gini contract (dpll)
//   SAT epilogue            solve.go:86-110                  (epilogue)
//   NotSatisfiable          solve.go:114-115                 (core)
//
// Control flow is group-uniform: every thread runs the same scalar logic on
// broadcast LDS/HBM reads, and single-writer updates are made by thread 0.
// The data-parallel parts are row evaluation (threads over the rows watched by
// a round's frontier, flattened through an LDS work list), the
// all-false-completion check, candidate membership tests, AtMost counting
// (one wavefront per queued row), conflict analysis and every O(nv) sweep.
//
// Semantics are exactly those of oracle/sat_oracle.c (the test oracle): a
// round's implications are resolved to the lowest implying row with atomicMin,
// so reasons, cores and step counts are bit-identical.  (The oracle orders
// assignments by round number, this kernel by the trail position where the
// round started; the two orders agree on every pair of assigned variables, and
// nothing depends on the order of assignments within one round.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "kernel_api.hpp"
#include "layout.hpp"

namespace dp {

// Each mode's kernel is instantiated in its own translation unit
// (solve_lds.hip, solve_split.hip, solve_hbm.hip) so they compile in parallel.

namespace {

constexpr int32_t INF = 0x7fffffff;
constexpr int32_t R_DEC = -1;    // decision / assumption / guess
constexpr int32_t R_EXTRA = -2;  // epilogue bound over the extras
enum { CK_NONE = 0, CK_ROW, CK_VAR, CK_ASSUME, CK_EXTRA };
enum { RS_SAT = 1, RS_UNSAT = -1, RS_BUDGET = 2 };

// BCP-visited bytes, counted per thread (Group::vis_add).
#define DP_VIS_ADD(x) vis_add(x)

// Lanes of the wave hand values to each other through the working set (LDS,
// or HBM): complete every access before the next phase.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Inclusive prefix sum over the 64 lanes with DPP row shifts and row
// broadcasts (no LDS round trips).
__device__ __forceinline__ int wave_incl_scan(int x) {
  int y = x;
  y += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
  y += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
  y += __builtin_amdgcn_update_dpp(0, x, 0x113, 0xf, 0xf, true);   // row_shr:3
  y += __builtin_amdgcn_update_dpp(0, y, 0x114, 0xf, 0xe, false);  // row_shr:4, banks 1-3
  y += __builtin_amdgcn_update_dpp(0, y, 0x118, 0xf, 0xc, false);  // row_shr:8, banks 2-3
  y += __builtin_amdgcn_update_dpp(0, y, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  y += __builtin_amdgcn_update_dpp(0, y, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return y;
}

// Inclusive prefix maximum of non-negative values, the same DPP pattern.
__device__ __forceinline__ int wave_incl_max(int x) {
  int y = x;
  y = max(y, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true));   // row_shr:1
  y = max(y, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true));   // row_shr:2
  y = max(y, __builtin_amdgcn_update_dpp(0, x, 0x113, 0xf, 0xf, true));   // row_shr:3
  y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x114, 0xf, 0xe, false));  // row_shr:4, banks 1-3
  y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x118, 0xf, 0xc, false));  // row_shr:8, banks 2-3
  y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
  y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
  return y;
}

// Whole-wave minimum and sum, wave-uniform: the DPP scans' lane 63.  (A
// __shfl_xor butterfly takes a ds_bpermute address VGPR per step, which the
// compiler keeps live across the search loop: six of the register-capped
// build's spills.)
__device__ __forceinline__ int wave_min(int x) {
  constexpr int I = 0x7fffffff;  // lanes a shift does not reach keep the identity (bound_ctrl off)
  int y = x;
  y = min(y, __builtin_amdgcn_update_dpp(I, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  y = min(y, __builtin_amdgcn_update_dpp(I, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  y = min(y, __builtin_amdgcn_update_dpp(I, x, 0x113, 0xf, 0xf, false));  // row_shr:3
  y = min(y, __builtin_amdgcn_update_dpp(I, y, 0x114, 0xf, 0xe, false));  // row_shr:4, banks 1-3
  y = min(y, __builtin_amdgcn_update_dpp(I, y, 0x118, 0xf, 0xc, false));  // row_shr:8, banks 2-3
  y = min(y, __builtin_amdgcn_update_dpp(I, y, 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
  y = min(y, __builtin_amdgcn_update_dpp(I, y, 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
  return __builtin_amdgcn_readlane(y, 63);
}
__device__ __forceinline__ int wave_sum(int x) { return __builtin_amdgcn_readlane(wave_incl_scan(x), 63); }

__device__ __forceinline__ bool getb(const uint32_t* b, int i) { return (b[i >> 5] >> (i & 31)) & 1u; }

}  // namespace
// Diagnostic builds (-DDP_STAMPS, never the shipped library) record the
// shader-clock cycles of each phase; the release build compiles them away.
#ifdef DP_STAMPS
__device__ __forceinline__ int64_t stamp() {
  int64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ int64_t wallclock() {
  int64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define DP_STAMP(i) t[i] = stamp()
#else
#define DP_STAMP(i) (void)0
#endif
// Index checks of the diagnostic build (-DDP_STAMPS -DDP_CHECKS; the calls
// cost registers, so plain phase builds leave them out): a data-derived index outside its
// range is recorded (first failure per problem) and clamped to `lo`, so a
// broken invariant shows up as a report instead of a memory fault.
#if defined(DP_STAMPS) && defined(DP_CHECKS)
#define DP_CHK(x, lo, hi, code) chk((x), (lo), (hi), (code))
#else
#define DP_CHK(x, lo, hi, code) (x)
#endif
namespace {

// MINW: the waves per SIMD the kernel is built for (solve_kernel).  The
// register-capped one-wavefront build (config 3's small catalogs) does not
// count BCP-visited bytes: the counter's VGPR took its spills from 3 to 12
// VGPRs (an LDS counter per lane: 9).  The unbounded build counts them.
template <int MODE, int MINW = 1>
struct Group {
  // the 16-bit LDS image, the whole working set in LDS (M_LDS, M_LDSG)
  static constexpr bool N16 = mode_n16(MODE);
  using IX = typename std::conditional<N16, uint16_t, int32_t>::type;
  static constexpr bool NO_VIS = MODE == M_LDS && MINW > 1;
  static constexpr int NW = mode_waves(MODE);  // wavefronts per problem
  static constexpr int NT = 64 * NW;           // threads per problem
  static constexpr int WBUF = mode_wbuf(MODE);
  static constexpr int CQ = mode_cq(MODE);

  // the lowest implying row per literal: 16-bit in LDS, 32-bit (global
  // atomics) in the multi-wave modes; IMP_NONE = no implication this round
  static constexpr bool IMP16 = N16;
  using IMP = typename std::conditional<IMP16, uint16_t, uint32_t>::type;
  static constexpr uint32_t IMP_NONE = IMP16 ? 0xffffu : (uint32_t)INF;
  // guess-stack flag: the choice was already satisfied by a guess (m = none)
  static constexpr int G_SKIP = N16 ? 0x8000 : 0x40000000;

  // IX <-> int for the signed values: reasons R_DEC (-1), R_EXTRA (-2) and
  // Solve() decision d (-3 - d); in 16 bits every value from dthr up is one of
  // them (fits16 keeps rows below and decisions above)
  __device__ __forceinline__ int dec(IX x) const {
    if constexpr (!N16) return x;
    else return (int)x >= dthr ? (int)x - 0x10000 : (int)x;
  }
  __device__ __forceinline__ static IX enc(int x) { return (IX)x; }

  // Words updated by global atomics (imp; in M_HBM also the used / dset / fg
  // bitsets) are read from L2: the atomics are performed there and a plain
  // load from another wavefront of the workgroup can hit a stale L1 line.
  // LDS words need no such care.
  __device__ __forceinline__ static uint32_t ld_imp(const IMP* p) {
    if constexpr (N16) return *p;
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ static uint32_t ld_bits(const uint32_t* p) {
    if constexpr (MODE != M_HBM) return *p;
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- record views ----
  int nv, nc, nk, nid, nrows, nbv, nbi, na, nch, ncl, nkl, nchl;
  const IX *clause_off, *clause_lits, *clause_id;
  const IX *card_off, *card_lits, *card_bound, *card_id;
  const IX *var_choice_off, *choice_off, *choice_lits, *anchors;
  // DP_FMT_P16D in LDS: choice list k is dependency row rowref[k] after its
  // first literal (layout.hpp lds_body_words); else nullptr and the lists
  // are choice_off / choice_lits
  const IX* rowref;
  // Packed records on M_LDS (rowspace): identities as the AtMost-identity
  // mask (idmask, u32 words) and its per-word prefix counts (idpc), no
  // clause_id / card_id.  Identity i is AtMost row nc + rank1(i) when its
  // mask bit is set, else clause row i - rank1(i) (layout.hpp
  // lds_body_words).  `used`, `en`, `en2` and `enabled` are then indexed by
  // row; the outputs (cores, trace) go back to identities through idt.
  bool rowspace;
  const uint32_t* idmask;
  const uint16_t* idpc;
  uint32_t* idt;
  __device__ __forceinline__ int row_of(int id) const {
    const uint32_t m = idmask[id >> 5];
    const int sh = id & 31;
    const int r1 = (int)idpc[id >> 5] + __popc(m & ((1u << sh) - 1u));
    return (m >> sh) & 1u ? nc + r1 : id - r1;
  }
  // the bit a row sets in used / en / enabled
  __device__ __forceinline__ int row_key(int r) const { return rowspace ? r : row_ident(r); }
  const IX *w_off, *w;  // watch lists, built by build_watches
  // Multi-wave problems whose lists are built on the device (DP_FMT_I32,
  // layout.hpp Layout::wl): 8-byte entries {row, row_info(row)} carrying the
  // row's literal range, so a visit reads the row's literals without first
  // reading its offsets (one dependent HBM read less per row; w is unused).
  // nullptr: 4-byte row entries in w.
  const int2* w8;
  int nwatch, dthr;
  // BCP-visited bytes (this thread): the watch entries, row offsets, row
  // literals and their values that propagation reads
  uint32_t vis;
  __device__ __forceinline__ void vis_add(uint32_t x) {
    if constexpr (!NO_VIS) vis += x;
  }
  // the problem's BCP-visited bytes (group-uniform; 0: not counted)
  __device__ __forceinline__ uint32_t vis_total() {
    if constexpr (NO_VIS) return 0u;
    else return (uint32_t)g_sum((int)vis);
  }
  // ---- working set ----
  int8_t* val;
  IX *reason, *rs, *trail, *touched, *d_mark, *l_off, *l_lits, *dq, *stk;
  IMP* imp;  // imp[l] = lowest row implying literal l this round
  uint32_t *d_flip, *inS, *extra, *seen, *model, *used, *en, *en2, *crit, *dset, *fg;
  IX *wbuf, *cardq;
  int32_t* scal;
  // LDS round state (mode_lds_rounds; layout.hpp Layout::hkey..fr)
  static constexpr bool LR = mode_lds_rounds(MODE);
  int32_t *hkey, *fr;
  uint32_t *hrp, *hrn;
  uint16_t* tl;
  int hmask;   // hc - 1
  bool hmode;  // this round's implications go to the LDS table (else imp/touched in HBM)
  int rb;      // the LDS-table round's counter bank (S_NTB / S_CVB / S_OVB)
  int cap, lcap;
  int tid, lane, wid;
  // ---- group-uniform state (registers, identical in every thread) ----
  int tlen, qhead;
  int64_t steps, budget;
  bool budget_hit;
  int ck, c_row, c_var, c_rp, c_rn;
  bool collect_guess;
  int learn_lo;  // learned rows below learn_lo are switched off (core refutations)
  int nl;
  const uint32_t* enabled;  // nullptr: every row
  bool extra_mode;
  int extra_w;
  int32_t* tr;  // search trace of this problem (nullptr: not traced)
  int tr_cap, tr_len;
  bool tr_stop;
#ifdef DP_STAMPS
  // round eval cycles, round finish cycles, rounds, 1-literal rounds, push_guess cycles,
  // search Solve() cycles, pop_guess cycles, push_guess calls; within a
  // round: 1-literal visit cycles, flattened-frontier cycles, AtMost flush
  // cycles, learned-row cycles, watch entries visited, frontier literals of
  // flattened rounds, learned rows evaluated, AtMost rows flushed
  unsigned long long* lacc;  // LDS phase accumulators (thread 0 adds; no registers held)
  int64_t sub[6];           // init: record staging, validation, watch-list build cycles;
                            // the build's count, scan and fill
  unsigned long long* dbg;  // [first code, value, bound, failures]
  __device__ __noinline__ int chk_fail(int x, int hi, int code) {
    if (dbg) {
      if (atomicCAS(&dbg[0], 0ull, (unsigned long long)code) == 0ull) {
        dbg[1] = (unsigned long long)(long long)x;
        dbg[2] = (unsigned long long)(long long)hi;
      }
      atomicAdd(&dbg[3], 1ull);
    }
    return 0;
  }
  __device__ __forceinline__ int chk(int x, int lo, int hi, int code) {
    return (x < lo || x >= hi) ? (chk_fail(x, hi, code), lo) : x;
  }
#define DP_ACC(i, x) do { if (tid == 0) atomicAdd(&lacc[i], (unsigned long long)(x)); } while (0)
#else
#define DP_ACC(i, x) (void)0
#endif

  // ------------------------------------------------------------------
  // group primitives (one wavefront: wave barrier and ballots; several:
  // s_barrier and per-wave slots in LDS)
  // ------------------------------------------------------------------
  // Workgroup barrier of the multi-wave modes.  Their per-literal arrays are
  // in HBM and __syncthreads() only drains LDS traffic (lgkmcnt) before
  // s_barrier: a wavefront could pass it with global stores still in flight
  // and another wavefront read the old words.  Drain every counter first.
  // Within an LDS-table round (lds_sync) the wavefronts hand each other only
  // LDS words: the round's global stores (reason, rs, trail) are read by no
  // other wavefront before propagate() returns, which drains them.
  bool lds_sync;
  __device__ __forceinline__ void bar() const {
    if constexpr (mode_lds_rounds(MODE)) {
      if (lds_sync) {
        __syncthreads();
        return;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();
  }
  __device__ __forceinline__ void gsync() {
    if constexpr (NW == 1) wsync();
    else bar();
  }
  // Several wavefronts: publish one value per wavefront (from the lanes with
  // `writer`) and return the slots after one barrier.  Exchanges alternate
  // between two banks of slots: a wavefront writes bank b for exchange k+2
  // only after passing exchange k+1's barrier, which every wavefront reaches
  // after its reads of exchange k (bar() drains them first) -- so no
  // trailing barrier is needed.  Every exchange is group-uniform.
  int sbank;
  static_assert(NW == 1 || S_SLOT + 2 * NW <= NSCAL, "two banks of per-wave slots");
  __device__ __forceinline__ const int32_t* exchange(int v, bool writer) {
    int32_t* sl = scal + S_SLOT + sbank * NW;
    if (writer) sl[wid] = v;
    bar();
    sbank ^= 1;
    return sl;
  }
  __device__ __forceinline__ bool g_any(bool b) {
    const bool w = __ballot(b) != 0;
    if constexpr (NW == 1) {
      return w;
    } else {
      const int32_t* sl = exchange(w, lane == 0);
      int r = 0;
#pragma unroll
      for (int i = 0; i < NW; ++i) r |= sl[i];
      return r != 0;
    }
  }
  __device__ __forceinline__ int g_min(int x) {
    x = wave_min(x);
    if constexpr (NW == 1) {
      return x;
    } else {
      const int32_t* sl = exchange(x, lane == 0);
      int r = INF;
#pragma unroll
      for (int i = 0; i < NW; ++i) r = min(r, sl[i]);
      return r;
    }
  }
  __device__ __forceinline__ int g_sum(int x) {
    x = wave_sum(x);
    if constexpr (NW == 1) {
      return x;
    } else {
      const int32_t* sl = exchange(x, lane == 0);
      int r = 0;
#pragma unroll
      for (int i = 0; i < NW; ++i) r += sl[i];
      return r;
    }
  }
  // Unordered append: position of a flagged thread in a list that grows by
  // the flagged threads of every call.  One wavefront: ballot prefix on the
  // register `run`.  Several: wave-aggregated LDS atomic on S_APP; the caller
  // finishes with claim_end, which folds the appended count into `run`.
  __device__ __forceinline__ int claim(bool f, int& run) {
    const uint64_t m = __ballot(f);
    if constexpr (NW == 1) {
      const int at = run + __popcll(m & lanemask_lt());
      run += __popcll(m);
      return at;
    } else {
      int b = 0;
      if (m && lane == 0) b = atomicAdd(&scal[S_APP], __popcll(m));
      b = __builtin_amdgcn_readlane(b, 0);
      return run + b + __popcll(m & lanemask_lt());
    }
  }
  __device__ __forceinline__ void claim_end(int& run) {
    if constexpr (NW > 1) {
      bar();
      run += scal[S_APP];
      bar();
      if (tid == 0) scal[S_APP] = 0;
      bar();
    }
  }

  // ------------------------------------------------------------------
  // set-up (oracle: st_init)
  // ------------------------------------------------------------------
  // Returns false (nothing else initialised) for a malformed record.
  __device__ __forceinline__ bool init(char* lds, char* hbm, const int32_t* __restrict__ grec) {
    tid = (int)threadIdx.x;
    lane = lane_id();
    wid = tid >> 6;
    // the header by a 16-byte vector load on lanes 0..3 (one 64-byte read,
    // like the body's), broadcast by readlane
    int4 hv = make_int4(0, 0, 0, 0);
    if (lane < 4) hv = reinterpret_cast<const int4*>(grec)[lane];
    int32_t h[DP_H_SIZE];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      h[4 * q + 0] = __builtin_amdgcn_readlane(hv.x, q);
      h[4 * q + 1] = __builtin_amdgcn_readlane(hv.y, q);
      h[4 * q + 2] = __builtin_amdgcn_readlane(hv.z, q);
      h[4 * q + 3] = __builtin_amdgcn_readlane(hv.w, q);
    }
    if (h[DP_H_FMT] == DP_FMT_REJECT) return false;
#ifdef DP_STAMPS
    const int64_t ti0 = stamp();
#endif
    const Layout L = layout<MODE>(h);
    const dp_rec_layout R = rec_layout(h);
    const ImgLayout X = img_layout(h);
    // the group primitives' LDS words first (the decode's g_any uses them)
    scal = reinterpret_cast<int32_t*>(lds + L.scal);
    sbank = 0;
    ncl = h[DP_H_NCL]; nkl = h[DP_H_NKL]; nchl = h[DP_H_NCHL];
    nv = h[DP_H_NV]; nc = h[DP_H_NC]; nk = h[DP_H_NK]; nid = h[DP_H_NID]; na = h[DP_H_NA];
    nch = h[DP_H_NCH];
    nrows = nc + nk;
    nbv = bits_words(nv); nbi = bits_words(nid);
    const IX* body;
    bool packed = false;
    rowref = nullptr;
    rowspace = false;
    if constexpr (N16) {
      // The record -> LDS, as it is: the host stages one-wavefront records in
      // a 16-bit form (DP_FMT_U16, or DP_FMT_P16 whose tail is decoded below),
      // 16-byte aligned and padded to 4 words.
      IX* b = reinterpret_cast<IX*>(lds + L.body);
      const int4* src = reinterpret_cast<const int4*>(grec + DP_H_SIZE);
      const int fmt = h[DP_H_FMT];
      packed = fmt_packed(fmt);
      if (!packed && fmt != DP_FMT_U16 && fmt != DP_FMT_U16_CHECKED) return false;
      // DP_FMT_P8D lands past the arrays it decodes to (p16_tail_copy), the
      // other forms at the body's start
      const bool p8 = fmt == DP_FMT_P8D;
      const int land = p8 ? p16_tail_copy(h) : 0;
      const int groups = p8 ? (p8_bytes(h) + 15) >> 4
                            : packed ? (int)((p16_tail_at(h) + p16_tail_bytes(h) + 15) >> 4)
                                     : (h[DP_H_WORDS] - DP_H_SIZE + 7) >> 3;
      if (L.body == 0 && land + ((groups + 63) >> 6) * 1024 <= L.lds_bytes) {
        // LDS-DMA, every 1 KiB piece in flight at once, wavefront w taking
        // pieces w, w + NW, ... (lanes past the image re-read its last piece
        // into LDS the later arrays own; they are initialised after this)
        for (int c = 64 * wid; c < groups; c += NT) {
          const int i = min(c + lane, groups - 1);
          __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + i),
                                           (__attribute__((address_space(3))) void*)(lds + land + 16 * c), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        gsync();
      } else {
        for (int i = tid; i < groups; i += NT) reinterpret_cast<int4*>(reinterpret_cast<char*>(b) + land)[i] = src[i];
        gsync();
      }
      body = b;
      if (packed) {
        // DP_FMT_P16 / DP_FMT_P16D in LDS: the uint16 arrays where they
        // landed, then the offsets arrays and the identities decoded from the
        // tail (and, DP_FMT_P16D, the choice lists derived after them).
        // DP_FMT_P8D: its arrays first widened into DP_FMT_P16D's places and
        // its tail expanded after it (expand8), then decoded the same way.
        const bool derived = fmt_derived(fmt);
        IX* q = b;
        clause_lits = q; q += ncl;
        card_lits = q;   q += nkl;
        card_bound = q;  q += nk;
        if (!derived) { choice_lits = q; q += nchl; }
        anchors = q;     q += na;
        clause_off = q;  q += nc + 1;
        card_off = q;    q += nk + 1;
        var_choice_off = q; q += nv + 1;
        if (derived) { rowref = q; q += nch; }
        else { choice_off = q; q += nch + 1; }
        q += (q - b) & 1;  // (4-byte alignment)
        idmask = reinterpret_cast<const uint32_t*>(q); q += 2 * nbi;
        idpc = reinterpret_cast<const uint16_t*>(q);   q += nbi + 1;
        rowspace = true;
        // (one wavefront decodes; with several, the others wait at g_any's
        // barrier.  The one-wavefront build calls it unconditionally: the
        // call under a branch took its VGPRs from 161 to 202.)
        auto decode = [&] {
          uint8_t* raw = reinterpret_cast<uint8_t*>(b) + land;
          uint8_t* ex = reinterpret_cast<uint8_t*>(b) + p8_tail(h);
          const bool ok8 = !p8 || expand8(raw, h[DP_H_P8] & 0xff, p8_bytes(h), ex);
          const bool ok16 = unpack16(p8 ? reinterpret_cast<const char*>(ex)
                                        : reinterpret_cast<const char*>(b) + p16_tail_at(h),
                                     (int)p16_tail_bytes(h), derived, lds + L.reason,
                                     p8 ? ex : reinterpret_cast<uint8_t*>(b) + p16_tail_copy(h));
          return ok8 && ok16;
        };
        bool ok;
        if constexpr (NW == 1) {
          ok = decode();
        } else {
          ok = true;
          if (wid == 0) ok = decode();
          ok = !g_any(!ok);
        }
        if (!ok) return false;
      }
    } else {
      body = reinterpret_cast<const IX*>(grec + DP_H_SIZE);  // read in place (read-only)
    }
    auto rv = [&](int32_t word_off) { return body + (word_off - DP_H_SIZE); };
    if (!packed) {
      clause_off = rv(R.clause_off); clause_lits = rv(R.clause_lits); clause_id = rv(R.clause_id);
      card_off = rv(R.card_off); card_lits = rv(R.card_lits); card_bound = rv(R.card_bound);
      card_id = rv(R.card_id); var_choice_off = rv(R.var_choice_off); choice_off = rv(R.choice_off);
      choice_lits = rv(R.choice_lits); anchors = rv(R.anchors);
    }
    nwatch = h[DP_H_NCL] + h[DP_H_NKL];
    dthr = nrows + L_MAX;
    char* hot = MODE == M_HBM ? hbm : lds;  // val and the bitsets
    char* cold = N16 ? lds : hbm;           // per-literal arrays
    val = reinterpret_cast<int8_t*>(hot + L.val);
    reason = reinterpret_cast<IX*>(cold + L.reason);
    rs = reinterpret_cast<IX*>(cold + L.rs);
    trail = reinterpret_cast<IX*>(cold + L.trail);
    touched = reinterpret_cast<IX*>(cold + L.touched);
    d_mark = reinterpret_cast<IX*>(cold + L.d_mark);
    imp = reinterpret_cast<IMP*>(cold + L.imp);
    w8 = nullptr;
    d_flip = reinterpret_cast<uint32_t*>(hot + L.d_flip);
    inS = reinterpret_cast<uint32_t*>(hot + L.inS);
    extra = reinterpret_cast<uint32_t*>(hot + L.extra);
    seen = reinterpret_cast<uint32_t*>(hot + L.seen);
    model = reinterpret_cast<uint32_t*>(hot + L.model);
    dset = reinterpret_cast<uint32_t*>(hot + L.dset);
    fg = reinterpret_cast<uint32_t*>(hot + L.fg);
    used = reinterpret_cast<uint32_t*>(hot + L.used);
    en = reinterpret_cast<uint32_t*>(hot + L.en);
    en2 = reinterpret_cast<uint32_t*>(hot + L.en2);
    crit = reinterpret_cast<uint32_t*>(hot + L.crit);
    idt = reinterpret_cast<uint32_t*>(lds + L.idt);
    l_off = reinterpret_cast<IX*>(cold + L.l_off);
    l_lits = reinterpret_cast<IX*>(cold + L.l_lits);
    dq = reinterpret_cast<IX*>(cold + L.dq);
    stk = reinterpret_cast<IX*>(cold + L.stk);
    wbuf = reinterpret_cast<IX*>(lds + L.wbuf);
    cardq = reinterpret_cast<IX*>(lds + L.cardq);
    hkey = reinterpret_cast<int32_t*>(lds + L.hkey);
    hrp = reinterpret_cast<uint32_t*>(lds + L.hrp);
    hrn = reinterpret_cast<uint32_t*>(lds + L.hrn);
    tl = reinterpret_cast<uint16_t*>(lds + L.tl);
    fr = reinterpret_cast<int32_t*>(lds + L.fr);
    hmask = L.hc - 1;
    hmode = LR;
    lds_sync = false;
    rb = 0;
#ifdef DP_STAMPS
    lacc = reinterpret_cast<unsigned long long*>(scal + (MODE == M_LDS ? 8 : NSCAL));
#endif
    cap = L.cap; lcap = L.lcap;
    tlen = qhead = 0;
    pre_lo = -1;
    steps = 0;
    vis = 0;
    budget_hit = false;
    ck = CK_NONE; c_row = c_var = c_rp = c_rn = 0;
    collect_guess = false;
    learn_lo = 0;
    nl = 0;
    enabled = nullptr;
    extra_mode = false;
    extra_w = 0;
    tr = nullptr;
    tr_cap = tr_len = 0;
    tr_stop = false;
#ifdef DP_STAMPS
    dbg = nullptr;
#endif
#ifdef DP_STAMPS
    const int64_t ti1 = stamp();
    sub[0] = ti1 - ti0;
#endif
    if constexpr (N16)
      if ((h[DP_H_FMT] == DP_FMT_U16 || packed) && !valid_record(body, packed, fmt_derived(h[DP_H_FMT]))) return false;
    if constexpr (!N16)
      if ((h[DP_H_FMT] == DP_FMT_I32W || h[DP_H_FMT] == DP_FMT_I32) && !valid_wide(R, X, h[DP_H_FMT] == DP_FMT_I32W))
        return false;
#ifdef DP_STAMPS
    const int64_t ti2 = stamp();
    sub[1] = ti2 - ti1;
#endif
    // the watch lists follow the record (M_LDS) or live in the problem's
    // scratch; M_LDS / M_LDSG count on the per-literal arrays, initialised below
    if constexpr (N16) {
      IX* wo = const_cast<IX*>(body) + lds_body_words(h);  // right after the decoded arrays
      build_watches(wo, wo + 2 * nv + 1, reinterpret_cast<uint32_t*>(lds + L.reason));
      w_off = wo; w = wo + 2 * nv + 1;
    } else {
      if (h[DP_H_FMT] == DP_FMT_I32) {  // plain int32 record: the lists in scratch (layout.hpp wl)
        IX* wo = reinterpret_cast<IX*>(hbm + L.wl);
        if (device_watches(h)) build_watches_wide(wo, wo + 2 * nv + 2, reinterpret_cast<uint32_t*>(lds + L.wbuf));
        // (else built by the passes before this launch, watch_build.hip)
        w_off = wo; w = nullptr;
        w8 = reinterpret_cast<const int2*>(wo + 2 * nv + 2);
      } else {
        w_off = rv(X.w_off); w = rv(X.w);  // host-built, staged after the record
      }
    }
#ifdef DP_STAMPS
    sub[2] = stamp() - ti2;
#endif

    if constexpr (N16) {
      for (int v = tid; v < nv; v += NT) val[v] = 0;
    } else {
      for (int v = tid; v < (nv + 3) / 4; v += NT) reinterpret_cast<uint32_t*>(val)[v] = 0;
    }
    for (int l = tid; l < 2 * nv; l += NT) imp[l] = (IMP)IMP_NONE;
    if constexpr (LR)
      for (int i = tid; i <= hmask; i += NT) { hkey[i] = -1; hrp[i] = (uint32_t)INF; hrn[i] = (uint32_t)INF; }
    for (int i = tid; i < nbv; i += NT) {
      d_flip[i] = 0; inS[i] = 0; extra[i] = 0; seen[i] = 0; model[i] = 0; dset[i] = 0; fg[i] = 0;
    }
    for (int i = tid; i < mode_nscal(MODE); i += NT) scal[i] = 0;
    if (tid == 0) {  // (after the zeroing in program order: both are wavefront 0's stores)
      l_off[0] = 0;
      scal[S_POSROWS] = h[DP_H_NVU] > 0;
    }
    gsync();
    return true;
  }

  // dp_rec_validate on the device, for the records the host passed through
  // without reading them (16-bit records copied as they are, DP_FMT_U16):
  // offsets arrays start at 0, never decrease and end at their totals; every
  // literal, variable and identity is in range; the positions of a variable
  // in an AtMost row form one run (16-bit bounds cannot be negative).  The
  // host checked every other staged form (DP_FMT_U16_CHECKED, DP_FMT_I32).
  // Array by array, two 16-bit words per LDS load.  Group-uniform result.
  __device__ __forceinline__ bool valid_record(const IX* base, bool packed, bool derived) {
    static_assert(N16, "16-bit records run on the LDS image");
    // (base: the body's start, 16-byte aligned; arrays anywhere after it)
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(base);
    bool bad = false;
    auto range = [&](const IX* arr, int n, int hi) {
      const int a = (int)(arr - base), e = a + n;
      // four words per lane per step: the loads first
      for (int q0 = (a >> 1); 2 * q0 < e; q0 += 4 * NT) {
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = q0 + i * NT + tid;
          x[i] = 2 * q < e ? b32[q] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = q0 + i * NT + tid;
          bad |= 2 * q < e && ((2 * q >= a && (int)(x[i] & 0xffffu) >= hi) || (2 * q + 1 < e && (int)(x[i] >> 16) >= hi));
        }
      }
    };
    auto offsets = [&](const IX* arr, int n, int total) {  // n + 1 words
      const int a = (int)(arr - base), e = a + n + 1;
      for (int q = (a >> 1) + tid; 2 * q < e; q += NT) {
        const uint32_t x = b32[q];
        const int i0 = 2 * q, x0 = (int)(x & 0xffffu), x1 = (int)(x >> 16);
        const int prev = i0 > a ? (int)(b32[q - 1] >> 16) : 0;  // word i0 - 1
        if (i0 >= a) bad |= i0 == a ? x0 != 0 : x0 < prev;
        if (i0 + 1 < e) bad |= i0 + 1 == a ? x1 != 0 : x1 < x0;
        bad |= (i0 == e - 1 && x0 != total) || (i0 + 1 == e - 1 && x1 != total);
      }
    };
    if (packed) {
      // decoded (unpack16): offsets are prefix sums of byte lengths (from 0,
      // non-decreasing), identities come from the mask (in range); only the
      // totals remain to check
      if (tid == 0)  // (DP_FMT_P16D: unpack16 counted the lists' nchl variables)
        bad = (int)clause_off[nc] != ncl || (int)card_off[nk] != nkl || (int)var_choice_off[nv] != nch ||
              (!derived && (int)choice_off[nch] != nchl);
    } else {
      offsets(clause_off, nc, ncl);
      range(clause_id, nc, nid);
      offsets(card_off, nk, nkl);
      range(card_id, nk, nid);
      offsets(var_choice_off, nv, nch);
      offsets(choice_off, nch, nchl);
    }
    range(clause_lits, ncl, 2 * nv);
    range(card_lits, nkl, nv);
    if (!derived) range(choice_lits, nchl, nv);  // (derived lists are rows: clause_lits, above)
    range(anchors, na, nv);
    if (g_any(bad)) return false;  // the offsets below are now in range
    // a lane per AtMost row: its positions in registers (rows of up to 16:
    // independent loads, then register compares), longer rows in a loop
    for (int k = tid; k < nk; k += NT) {
      const int a = card_off[k], len = (int)card_off[k + 1] - a;
      if (len <= 16) {
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = i < len ? (int)card_lits[a + i] : -1 - i;
#pragma unroll
        for (int j = 2; j < 16; ++j) {
          bool dup = false;
#pragma unroll
          for (int i = 0; i < j - 1; ++i) dup |= v[i] == v[j];
          bad |= dup && v[j] != v[j - 1];
        }
      } else {
        for (int j = a + 1; j < a + len; ++j) {
          const int x = card_lits[j];
          if (x != (int)card_lits[j - 1])
            for (int i = a; i < j - 1; ++i) bad |= (int)card_lits[i] == x;
        }
      }
    }
    return !g_any(bad);
  }

  // dp_rec_validate for an int32 record the host passed through unread
  // (DP_FMT_I32W, read in place from HBM by a multi-wave group), with its
  // watch lists' bounds: offsets arrays from 0, non-decreasing, to their
  // totals; indices in range; AtMost bounds not negative and each variable's
  // positions one run; w_off from 0, non-decreasing, within w; every listed
  // row a row.  Group-uniform result.
  __device__ __forceinline__ bool valid_wide(const dp_rec_layout& R, const ImgLayout& X, bool watches) {
    static_assert(!N16, "the int32 form runs on the HBM-read multi-wave groups");
    const int32_t* r = reinterpret_cast<const int32_t*>(clause_off) - R.clause_off;  // the record
    bool bad = false;
    // VU independent loads per thread and step, so a thread has that many in
    // flight instead of one (an OLM-scale record is ~400k words: one load at
    // a time per thread took ~720k cycles, 0.3 ms a catalog)
    constexpr int VU = 8;
    auto offsets = [&](int at, int n, int total, bool exact) {
      for (int i0 = tid; i0 <= n; i0 += VU * NT) {
        int x[VU], y[VU];
#pragma unroll
        for (int u = 0; u < VU; ++u) {
          const int i = i0 + u * NT;
          x[u] = i <= n ? r[at + i] : 0;
          y[u] = i <= n && i > 0 ? r[at + i - 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < VU; ++u) {
          const int i = i0 + u * NT;
          if (i > n) continue;
          bad |= i == 0 ? x[u] != 0 : x[u] < y[u];
          bad |= i == n && (exact ? x[u] != total : x[u] > total);
        }
      }
    };
    auto range = [&](int at, int n, int lo, int hi) {
      for (int i0 = tid; i0 < n; i0 += VU * NT) {
        int x[VU];
#pragma unroll
        for (int u = 0; u < VU; ++u) x[u] = i0 + u * NT < n ? r[at + i0 + u * NT] : lo;
#pragma unroll
        for (int u = 0; u < VU; ++u) bad |= x[u] < lo || x[u] >= hi;
      }
    };
    offsets(R.clause_off, nc, ncl, true);
    offsets(R.card_off, nk, nkl, true);
    offsets(R.var_choice_off, nv, nch, true);
    offsets(R.choice_off, nch, nchl, true);
    if (watches) offsets(X.w_off, 2 * nv, ncl + nkl, false);
    range(R.clause_lits, ncl, 0, 2 * nv);
    range(R.clause_id, nc, 0, nid);
    range(R.card_lits, nkl, 0, nv);
    range(R.card_bound, nk, 0, 1 << 30);
    range(R.card_id, nk, 0, nid);
    range(R.choice_lits, nchl + na, 0, nv);  // choice_lits then anchors
    if (g_any(bad)) return false;  // the offsets below are now in range
    if (watches) range(X.w, r[X.w_off + 2 * nv], 0, nrows);
    // each variable's positions in an AtMost row form one run: rows of up to
    // 16 positions by independent loads into registers, longer ones in place
    for (int k = tid; k < nk; k += NT) {
      const int a = r[R.card_off + k], b = r[R.card_off + k + 1];
      const int32_t* cl = r + R.card_lits;
      if (b - a <= 16) {
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = a + i < b ? cl[a + i] : -1 - i;
#pragma unroll
        for (int j = 1; j < 16; ++j)
#pragma unroll
          for (int i = 0; i < j - 1; ++i) bad |= v[j] != v[j - 1] && v[i] == v[j];
        continue;
      }
      for (int j = a + 1; j < b; ++j)
        if (cl[j] != cl[j - 1])
          for (int i = a; i < j - 1; ++i) bad |= cl[i] == cl[j];
    }
    return !g_any(bad);
  }

  // DP_FMT_P8D (include/deppy_hip.h; lower.cpp p8_to_p16d) -> DP_FMT_P16D:
  // the 16-bit arrays at their places (clause_lits .. anchors, set up by
  // init) from the record's bytes at `raw`, and DP_FMT_P16D's tail (lengths,
  // list sources, identity mask) at `ex`, for unpack16.  One wavefront.
  // False when the sections overrun the body's `bytes` or a source marked
  // nonzero is zero (the rest is unpack16's and valid_record's).
  __device__ __forceinline__ bool expand8(const uint8_t* raw, int f, int bytes, uint8_t* ex) {
    static_assert(N16, "16-bit records run on the LDS image");
    const bool hi = f & DP_P8_HI, nib = f & DP_P8_NIB;
    const int o_kv = ncl, o_av = ncl + nkl, o_b = o_av + na;
    const int o_neg = o_b + ((f & DP_P8_B1) ? 0 : nk);
    const int o_chi = o_neg + ((ncl + 7) >> 3);
    const int o_khi = o_chi + (hi ? (ncl + 7) >> 3 : 0);
    const int o_ahi = o_khi + (hi ? (nkl + 7) >> 3 : 0);
    const int o_len = o_ahi + (hi ? (na + 7) >> 3 : 0);
    const int o_snz = o_len + (nib ? (nc + nk + 1) >> 1 : nc + nk);
    const int o_sv = o_snz + ((nch + 7) >> 3);
    bool bad = o_sv > bytes || (f & ~(DP_P8_B1 | DP_P8_HI | DP_P8_NIB)) != 0;
    const int lim = bytes > 0 ? bytes - 1 : 0;  // (reads stay inside the landed body)
    auto byte = [&](int i) -> int { return (int)raw[min(i, lim)]; };
    auto bit = [&](int at, int j) -> int { return (byte(at + (j >> 3)) >> (j & 7)) & 1; };
    IX* cl = const_cast<IX*>(clause_lits);
    IX* kl = const_cast<IX*>(card_lits);
    IX* kb = const_cast<IX*>(card_bound);
    IX* an = const_cast<IX*>(anchors);
    for (int j = lane; j < ncl; j += 64) cl[j] = enc(2 * (byte(j) | (hi ? bit(o_chi, j) << 8 : 0)) + bit(o_neg, j));
    for (int j = lane; j < nkl; j += 64) kl[j] = enc(byte(o_kv + j) | (hi ? bit(o_khi, j) << 8 : 0));
    for (int k = lane; k < nk; k += 64) kb[k] = enc((f & DP_P8_B1) ? 1 : byte(o_b + k));
    for (int i = lane; i < na; i += 64) an[i] = enc(byte(o_av + i) | (hi ? bit(o_ahi, i) << 8 : 0));
    for (int i = lane; i < nc + nk; i += 64)
      ex[i] = (uint8_t)(nib ? (byte(o_len + (i >> 1)) >> (4 * (i & 1))) & 15 : byte(o_len + i));
    const uint64_t lt = lanemask_lt();
    int q = o_sv;
    for (int c = 0; c < nch; c += 64) {
      const int k = c + lane;
      const bool nz = k < nch && bit(o_snz, k);
      const uint64_t m = __ballot(nz);
      const int v = nz ? byte(q + __popcll(m & lt)) : 0;
      bad |= nz && v == 0;
      if (k < nch) ex[nc + nk + k] = (uint8_t)v;
      q += __popcll(m);
    }
    const int mb = (nid + 7) >> 3;
    bad |= q + mb > bytes;
    for (int i = lane; i < mb; i += 64) ex[nc + nk + nch + i] = (uint8_t)byte(q + i);
    wsync();
    return !__ballot(bad);
  }

  // DP_FMT_P16 tail (include/deppy_hip.h) -> the offsets arrays and the row
  // identities, in place after the uint16 arrays.  The tail (at most
  // DP_P16_TAIL_MAX bytes) is first copied to `tcopy` (p16_tail_copy: past
  // the decoded arrays, where the watch lists go later; layout() sizes the
  // body for it), since the decoded arrays overwrite it; its bytes are then
  // plain LDS loads.  Lengths become offsets by a DPP scan, the mask becomes
  // clause / AtMost identities by ballot ranks.  False when the mask does
  // not have nc clear and nk set bits (a malformed record).
  // DP_FMT_P16D (derived): the choice lists from the dependency rows and the
  // lists' sources (include/deppy_hip.h; lower.cpp implied_choices), with
  // `scratch` (the per-literal arrays' LDS, not yet in use) for the
  // dependency rows by rank, each list's row and the per-subject counts.
  __device__ __forceinline__ bool unpack16(const char* tail, int tb, bool derived, char* scratch, uint8_t* tcopy) {
    static_assert(N16, "16-bit records run on the LDS image");
    if (tail != reinterpret_cast<const char*>(tcopy)) {  // (DP_FMT_P8D: expand8 wrote it there)
      uint4 r = make_uint4(0u, 0u, 0u, 0u);
      if (16 * lane < tb) r = *reinterpret_cast<const uint4*>(tail + 16 * lane);
      if (16 * lane < tb) *reinterpret_cast<uint4*>(tcopy + 16 * lane) = r;
      wsync();
    }
    auto tbyte = [&](int i) -> int { return (int)tcopy[i]; };  // i in [0, tb)
    int at = 0;
    auto lens = [&](const IX* off_c, int n) {
      IX* off = const_cast<IX*>(off_c);
      int carry = 0;
      for (int c = 0; c < n; c += 64) {
        const int j = c + lane;
        const int x = j < n ? tbyte(at + j) : 0;
        const int incl = wave_incl_scan(x) + carry;
        if (j < n) off[j + 1] = enc(incl);
        carry = __builtin_amdgcn_readlane(incl, 63);
      }
      if (lane == 0) off[0] = enc(0);
      at += n;
    };
    lens(clause_off, nc);
    lens(card_off, nk);
    const int src_at = at;
    if (!derived) {
      lens(var_choice_off, nv);
      lens(choice_off, nch);
    } else {
      at += nch;
    }
    const uint64_t lt = lanemask_lt();
    // the identity mask as u32 words (bits past nid clear) and the
    // popcount of the words before each (a DPP scan), for row_of
    uint32_t* mk = const_cast<uint32_t*>(idmask);
    uint16_t* pc = const_cast<uint16_t*>(idpc);
    int carry1 = 0;
    for (int c = 0; c < nbi; c += 64) {
      const int wd = c + lane;
      uint32_t x = 0;
      if (wd < nbi) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * wd + q < (nid + 7) / 8) x |= (uint32_t)tbyte(at + 4 * wd + q) << (8 * q);
        if (32 * wd + 32 > nid) x &= (1u << (nid & 31)) - 1u;
        mk[wd] = x;
      }
      const int n1 = __popc(x);
      const int incl = wave_incl_scan(n1) + carry1;
      if (wd < nbi) pc[wd + 1] = (uint16_t)incl;
      carry1 = __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) pc[0] = 0;
    wsync();
    if (carry1 != nk || nid != nc + nk) return false;
    if (!derived) return true;
    // -- DP_FMT_P16D: the choice lists --
    if ((int)clause_off[nc] != ncl) return false;  // (rows read below stay in clause_lits)
    uint16_t* depr = reinterpret_cast<uint16_t*>(scratch);  // [nch] dependency rows by rank
    IX* rowk = const_cast<IX*>(rowref);                      // [nch] each list's row (kept)
    uint32_t* cnt = reinterpret_cast<uint32_t*>(scratch + ((2 * nch + 15) & ~15));  // [nv + 1]
    IX* vco = const_cast<IX*>(var_choice_off);
    for (int i = lane; i <= nv; i += 64) cnt[i] = 0u;  // (one wavefront runs the decode)
    bool bad = false;
    int nd = 0;  // dependency rows
    for (int c = 0; c < nc; c += 64) {
      const int r = c + lane;
      bool dep = false;
      if (r < nc) {
        const int a = clause_off[r], e = clause_off[r + 1];
        // the row's first eight literals by independent loads, then the rest
        int l[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) l[q] = a + q < e ? (int)clause_lits[a + q] : 0;
        dep = e - a >= 2 && (l[0] & 1);
#pragma unroll
        for (int q = 1; q < 8; ++q) dep = dep && !(l[q] & 1);
        for (int j = a + 8; j < e && dep; ++j) dep = !((int)clause_lits[j] & 1);
      }
      const uint64_t m = __ballot(dep);
      const int j = nd + __popcll(m & lt);
      if (dep && j < nch) depr[j] = (uint16_t)r;
      nd += __popcll(m);
    }
    bad |= nd > nch;
    wsync();
    int taken = 0, n0 = 0, smax = -1;
    for (int c = 0; c < nch; c += 64) {
      const int k = c + lane;
      const int sv = k < nch ? tbyte(src_at + k) : 0;
      const bool zero = k < nch && sv == 0;
      const uint64_t mz = __ballot(zero);
      const int j = taken + __popcll(mz & lt);
      taken += __popcll(mz);
      // a repeat names an earlier list that took a row (written below, or
      // in an earlier chunk)
      const int ks = k - sv;
      const int ss = k < nch && ks >= 0 ? tbyte(src_at + ks) : 1;
      if (zero) {
        bad |= j >= nd;
        rowk[k] = j < nd ? enc(depr[j]) : enc(0);
      }
      wsync();
      if (k < nch && !zero) {
        bad |= ks < 0 || ss != 0;
        rowk[k] = ks >= 0 ? rowk[ks] : enc(0);
      }
      wsync();
      int x = 0, s = -1, a = 0;
      if (k < nch) {
        const int row = rowk[k];
        a = clause_off[row];
        x = (int)clause_off[row + 1] - a - 1;
        s = (int)clause_lits[a] >> 1;
      }
      const int incl = wave_incl_scan(x);
      const int n = n0 + incl - x;
      // the highest subject of the lists up to this one (a DPP max-scan of s + 1)
      const int pm = wave_incl_max(s + 1) - 1;
      const int up = __builtin_amdgcn_update_dpp(0, pm + 1, 0x138, 0xf, 0xf, false) - 1;  // wave_shr:1
      const int before = max(smax, lane > 0 ? up : -1);
      if (k < nch) {
        // the list is the row's literals after the first, read in place
        // (list_at); valid_record checks every clause literal below 2nv
        if (s >= nv || s < before || n + x > nchl) bad = true;
        else atomicAdd(&cnt[s], 1u);
      }
      n0 += __builtin_amdgcn_readlane(incl, 63);
      smax = max(smax, __builtin_amdgcn_readlane(pm, 63));
    }
    bad |= taken != nd || n0 != nchl;
    wsync();
    if (__ballot(bad)) return false;
    int carry = 0;
    for (int c = 0; c <= nv; c += 64) {
      const int v = c + lane;
      const int y = v < nv ? (int)cnt[v] : 0;
      const int incl = wave_incl_scan(y) + carry;
      if (v < nv) vco[v + 1] = enc(incl);
      carry = __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) vco[0] = enc(0);
    wsync();
    return true;
  }

  // Watch lists of a multi-wave problem sent as a plain int32 record
  // (DP_FMT_I32, layout.hpp device_watches): counters in the LDS work area
  // (cnt: 2nv+1 words, free until the first round), a scan by wavefront 0,
  // then the fill into the lists in HBM scratch through the counters as
  // cursors.  Row order within a list is left to the atomics, as in
  // build_watches.  Ends with a draining barrier: every wavefront reads the
  // lists after it.
  __device__ __forceinline__ void build_watches_wide(IX* wo, IX* wlist, uint32_t* cnt) {
    static_assert(!N16, "LDS-image problems build theirs in LDS");
    const int n2 = 2 * nv + 1;
    for (int i = tid; i < n2; i += NT) cnt[i] = 0u;
    gsync();
    for (int j = tid; j < ncl; j += NT) atomicAdd(&cnt[((int)clause_lits[j] ^ 1) + 1], 1u);
    for (int k = tid; k < nk; k += NT)
      for (int j = card_off[k]; j < (int)card_off[k + 1]; ++j)
        if (j == (int)card_off[k] || card_lits[j] != card_lits[j - 1]) atomicAdd(&cnt[2 * (int)card_lits[j] + 1], 1u);
    gsync();
    if (wid == 0) {
      int carry = 0;
      for (int b = 0; b < n2; b += 64) {
        const int i = b + lane;
        const int x = i < n2 ? (int)cnt[i] : 0;
        const int incl = wave_incl_scan(x) + carry;
        if (i < n2) { wo[i] = incl; cnt[i] = (uint32_t)incl; }
        carry = __builtin_amdgcn_readlane(incl, 63);
      }
    }
    gsync();
    int2* ww = reinterpret_cast<int2*>(wlist);
    auto put = [&](uint32_t at, int row, int a, int len) { ww[at] = make_int2(row, (int)row_info(a, len)); };
    for (int r = tid; r < nc; r += NT) {
      const int a = clause_off[r], b = clause_off[r + 1];
      for (int j = a; j < b; ++j) put(atomicAdd(&cnt[(int)clause_lits[j] ^ 1], 1u), r, a, b - a);
    }
    for (int k = tid; k < nk; k += NT) {
      const int a = card_off[k], b = card_off[k + 1];
      for (int j = a; j < b; ++j)
        if (j == a || card_lits[j] != card_lits[j - 1]) put(atomicAdd(&cnt[2 * (int)card_lits[j]], 1u), nc + k, a, b - a);
    }
    bar();  // (drains the lists' stores)
  }

  // Watch lists of a one-wavefront problem, built in LDS from its record
  // (the host ships the record alone): per-literal counts, an inclusive scan
  // into w_off, then a fill through per-literal cursors.  cnt[l + 1] counts
  // the rows literal l wakes: the clauses holding ~l, and (l positive) the
  // AtMost rows holding var(l), once per distinct variable.  Row order within
  // a list is left to the atomics: every outcome of a round is a minimum over
  // rows (reasons, conflicts, Solve()'s first violated row), so nothing
  // depends on it.  Rows are handled a lane each with their literals loaded 8
  // at a time (independent loads and atomics, not a dependent chain).
  // (Multi-wave problems get host-built lists in their staged image: at
  // OLM scale the counters live in HBM and the in-kernel build was
  // latency-bound, 4.7M cycles a catalog.)
  __device__ __forceinline__ void build_watches(IX* wo, IX* ww, uint32_t* cnt) {
    static_assert(N16, "the HBM-read multi-wave modes build theirs in scratch");
    const int n2 = 2 * nv + 1;
#ifdef DP_STAMPS
    const int64_t tb0 = stamp();
#endif
    for (int i = tid; i < n2; i += NT) cnt[i] = 0u;
    gsync();
    // four positions per lane per step: the loads first, then the atomics
    // (one LDS round trip per step instead of one per position)
    for (int j0 = 0; j0 < ncl; j0 += 4 * NT) {
      int l[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = j0 + i * NT + tid;
        l[i] = j < ncl ? (int)clause_lits[j] : -1;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (l[i] >= 0) atomicAdd(&cnt[(l[i] ^ 1) + 1], 1u);
    }
    for (int k = tid; k < nk; k += NT) {
      const int a = card_off[k], b = card_off[k + 1];
      for (int j0 = a; j0 < b; j0 += 8) {
        int v[9];
        v[0] = j0 == a ? -1 : (int)card_lits[j0 - 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i + 1] = j0 + i < b ? (int)card_lits[j0 + i] : -1;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (j0 + i < b && v[i + 1] != v[i]) atomicAdd(&cnt[2 * v[i + 1] + 1], 1u);
      }
    }
    gsync();
#ifdef DP_STAMPS
    const int64_t tb1 = stamp();
    sub[3] = tb1 - tb0;
#endif
    // eight consecutive counters per lane (independent loads), their sum
    // scanned across the wave by DPP, then each lane's running prefix: one
    // scan per 512 counters (a config-2 catalog has ~480); wavefront 0 scans
    int carry = 0;
    for (int b = 0; b < (wid == 0 ? n2 : 0); b += 8 * 64) {
      const int i0 = b + 8 * lane;
      int x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = i0 + q < n2 ? (int)cnt[i0 + q] : 0;
      int s = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) s += x[q];
      const int incl = wave_incl_scan(s);
      int run = carry + incl - s;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        run += x[q];
        if (i0 + q < n2) { wo[i0 + q] = enc(run); cnt[i0 + q] = (uint32_t)run; }
      }
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
    gsync();
#ifdef DP_STAMPS
    const int64_t tb2 = stamp();
    sub[4] = tb2 - tb1;
#endif
    for (int r = tid; r < nc; r += NT) {
      const int a = clause_off[r], b = clause_off[r + 1];
      for (int j0 = a; j0 < b; j0 += 8) {
        int l[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) l[i] = j0 + i < b ? (int)clause_lits[j0 + i] : -1;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (l[i] >= 0) ww[atomicAdd(&cnt[l[i] ^ 1], 1u)] = enc(r);
      }
    }
    for (int k = tid; k < nk; k += NT) {
      const int a = card_off[k], b = card_off[k + 1];
      for (int j0 = a; j0 < b; j0 += 8) {
        int v[9];
        v[0] = j0 == a ? -1 : (int)card_lits[j0 - 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i + 1] = j0 + i < b ? (int)card_lits[j0 + i] : -1;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (j0 + i < b && v[i + 1] != v[i]) ww[atomicAdd(&cnt[2 * v[i + 1]], 1u)] = enc(nc + k);
      }
    }
    gsync();
#ifdef DP_STAMPS
    sub[5] = stamp() - tb2;
#endif
  }

  // ------------------------------------------------------------------
  // unit propagation (oracle: eval_row / finish_round / propagate)
  // ------------------------------------------------------------------
  __device__ __forceinline__ int row_ident(int r) const {
    return r < nc ? (int)clause_id[r] : r < nrows ? (int)card_id[r - nc] : -1;
  }
  __device__ __forceinline__ bool row_on(int r) const { return !enabled || getb(enabled, row_key(r)); }
  // watch entry j: {row, row_info} (w8), or {row, ROW_INFO_NONE}
  __device__ __forceinline__ int2 went(int j) const {
    if constexpr (!N16) {
      if (w8) return w8[j];
    }
    return make_int2((int)w[j], (int)ROW_INFO_NONE);
  }
  // visit() of watch entry j, or of nothing (j < 0)
  __device__ __forceinline__ void visit_at(int j, int& crow, int& ncq) {
    const int2 e = j >= 0 ? went(j) : make_int2(-1, (int)ROW_INFO_NONE);
    visit(e.x, crow, ncq, (uint32_t)e.y);
  }
  __device__ __forceinline__ int lit_val(int l) const {
    const int x = val[l >> 1];
    return (l & 1) ? -x : x;
  }

  // imp[l] as an int (INF: none this round)
  __device__ __forceinline__ int imp_get(int l) const {
    const uint32_t x = ld_imp(&imp[l]);
    return x == IMP_NONE ? INF : (int)x;
  }
  // imp[l] = min(imp[l], r); true on the round's first implication of l.
  // 16-bit: a compare-and-swap on the 32-bit word holding l and l ^ 1.
  __device__ __forceinline__ bool imp_min(int l, int r) {
    if constexpr (IMP16) {
      uint32_t* w32 = reinterpret_cast<uint32_t*>(imp) + (l >> 1);
      const int sh = (l & 1) * 16;
      // optimistic first attempt: neither literal of the variable implied
      // yet this round (the common case) -- no load before the first CAS
      uint32_t old = 0xffffffffu;
      for (;;) {
        const uint32_t cur = (old >> sh) & 0xffffu;
        if ((uint32_t)r >= cur) return false;
        const uint32_t nw = (old & ~(0xffffu << sh)) | ((uint32_t)r << sh);
        const uint32_t prev = atomicCAS(w32, old, nw);
        if (prev == old) return cur == IMP_NONE;
        old = prev;
      }
    } else {
      return atomicMin(&imp[l], (uint32_t)r) == IMP_NONE;
    }
  }
  // record "row r implies literal l" (lowest row wins, oracle: note); the
  // first implication of a literal in the round lists it
  // LDS table: probe for variable l >> 1 (claiming an empty slot), keep the
  // lowest row per polarity, list the slot on the round's first implication
  // of l.  A full table flags the round for a redo on the HBM arrays.
  __device__ __forceinline__ void note_lds(int l, int r) {
    const int v = l >> 1;
    int h = (int)(((uint32_t)v * 2654435761u) >> 16) & hmask;
    for (int probe = 0;; ++probe) {
      const int k = hkey[h];
      if (k == v) break;
      if (k < 0) {
        const int old = atomicCAS(&hkey[h], -1, v);
        if (old < 0 || old == v) break;
      }
      if (probe == 32 || probe == hmask) {
        scal[S_OVB + rb] = 1;
        return;
      }
      h = (h + 1) & hmask;
    }
    uint32_t* rr = (l & 1) ? hrn : hrp;
    if (atomicMin(&rr[h], (uint32_t)r) == (uint32_t)INF) {
      tl[atomicAdd(&scal[S_NTB + rb], 1)] = (uint16_t)((h << 1) | (l & 1));
      // implied both ways?  Of the two first implications of v, the later
      // one (in the LDS's order of these atomics) sees the other's row.
      const uint32_t* ro = (l & 1) ? hrp : hrn;
      if (ro[h] != (uint32_t)INF) atomicMax(&scal[S_CVB + rb], INF - v);
    }
  }
  // the slot of variable v (listed this round)
  __device__ __forceinline__ int slot_of(int v) const {
    int h = (int)(((uint32_t)v * 2654435761u) >> 16) & hmask;
    while (hkey[h] != v) h = (h + 1) & hmask;
    return h;
  }
  // trail position i holds literal l (and the ring, for the next round's frontier)
  __device__ __forceinline__ void put_trail(int i, int l) {
    trail[DP_CHK(i, 0, nv, 9)] = enc(l);
    if constexpr (LR) fr[i & hmask] = l;
  }

  __device__ __forceinline__ void note(int l, int r) {
    l = DP_CHK(l, 0, 2 * nv, 1);
    if constexpr (LR) {
      if (hmode) {
        note_lds(l, r);
        return;
      }
    }
    if (imp_min(l, r))
      touched[DP_CHK(atomicAdd(&scal[S_NTOUCHED], 1), 0, 2 * nv, 2)] = enc(l);
  }

  // The same from wave-converged code: every lane passes its literal (or -1).
  // (Measured: a register count with ballot-placed appends instead of the LDS
  // counter raised the kernel's VGPRs 149 -> 156 and ran 3% slower.)
  __device__ __forceinline__ void note_all(int l, int r) {
    if (l >= 0) note(l, r);
  }

  // clause row evaluation; the literal loads are issued four at a time.
  // Returns the row's one unassigned literal when it is unit, else -1.
#ifndef DP_EVAL_UNROLL
#define DP_EVAL_UNROLL 4
#endif
  __device__ __forceinline__ int eval_clause(int r, const IX* lits, int a, int b, int& crow) {
    int nun = 0, ul = -1;
    DP_VIS_ADD(2 * sizeof(IX) + (uint32_t)(b - a) * (sizeof(IX) + 1));  // offsets, literals, their values
    constexpr int U = DP_EVAL_UNROLL;
    for (int j = a; j < b; j += U) {
      int l[U];
#pragma unroll
      for (int k = 0; k < U; ++k) l[k] = j + k < b ? (int)lits[j + k] : -1;
      int x[U];
#pragma unroll
      for (int k = 0; k < U; ++k) x[k] = l[k] >= 0 ? lit_val(l[k]) : -1;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (x[k] > 0) return -1;  // satisfied
        if (x[k] == 0) { ++nun; ul = l[k]; }
      }
    }
    if (nun == 0) crow = min(crow, r);
    return nun == 1 ? ul : -1;
  }
  // a clause row (r < nc) or a learned row (r >= nrows); info: the row's
  // literal range from its watch entry (row_info), or ROW_INFO_NONE
  __device__ __forceinline__ int clause_unit(int r, int& crow, uint32_t info = ROW_INFO_NONE) {
    if constexpr (!N16) {
      if (r < nc && info != ROW_INFO_NONE) {
        const int a = (int)(info >> 8);
        return eval_clause(r, clause_lits, a, a + (int)(info & 255u), crow);
      }
    }
    if (r < nc) return eval_clause(r, clause_lits, clause_off[r], clause_off[r + 1], crow);
    const int j = r - nrows;
    return eval_clause(r, l_lits, DP_CHK((int)l_off[j], 0, lcap + 1, 33), DP_CHK((int)l_off[j + 1], 0, lcap + 1, 34), crow);
  }

  // an AtMost row in one lane (several wavefronts, AtMost queue full)
  __device__ __forceinline__ void card_serial(int r, int& crow) {
    const int k = r - nc, a = card_off[k], b = card_off[k + 1];
    int cnt = 0, nun = 0;
    DP_VIS_ADD(3 * sizeof(IX) + (uint32_t)(b - a) * (sizeof(IX) + 1));
    for (int j = a; j < b; ++j) {
      const int x = val[card_lits[j]];
      cnt += (x > 0);
      nun += (x == 0);
    }
    const int bound = card_bound[k];
    if (cnt > bound) crow = min(crow, r);
    else if (nun > 0) {
      // a variable repeated m times is a run of m positions
      for (int j = a; j < b;) {
        const int v = card_lits[j];
        int e = j + 1;
        while (e < b && (int)card_lits[e] == v) ++e;
        if (val[v] == 0 && cnt + (e - j) > bound) note(2 * v + 1, r);
        j = e;
      }
    }
  }

  // A watched row reached in a round: clause rows are evaluated by the thread
  // that reached them; AtMost rows are queued (ballot compaction) and later
  // evaluated by the whole wavefront that queued them, one row at a time
  // (flush_cards).  Call from wave-converged code: every active lane passes
  // its row (or -1).  Each wavefront owns a segment of CQ / NW queue entries
  // (multi-wave: and their row_info after the queue) and counts it in ncq (a
  // register), so queueing and flushing need no barrier between wavefronts.
  static constexpr int CQW = CQ / NW;
  __device__ __forceinline__ void visit(int r, int& crow, int& ncq, uint32_t info = ROW_INFO_NONE) {
    DP_VIS_ADD(r >= 0 ? sizeof(IX) : 0);  // the watch entry
    const bool ok = r >= 0 && row_on(r);
    const bool card = ok && r >= nc && r < nrows;
    const uint64_t m = __ballot(card);
    const bool q = ncq + __popcll(m) <= CQW;  // queue full: evaluate in-lane
    const int pos = wid * CQW + ncq + __popcll(m & lanemask_lt());
    if (card && q) {
      cardq[pos] = enc(r);
      if constexpr (NW > 1 && !N16) cardq[CQ + pos] = (IX)info;  // (IX = int32 here; M_LDSG entries carry no range)
    } else if (card) card_serial(r, crow);
    else if (ok) {
      const int ul = clause_unit(r, crow, info);
      if (ul >= 0) note(ul, r);
    }
    if (q) ncq += __popcll(m);
  }

  // AtMost rows, one at a time per wavefront, lanes over positions (oracle:
  // eval_row): counts by ballot; a variable listed m times is a run of m
  // positions, forced false when the count plus m exceeds the bound.
  // (each wavefront its own queue segment: no barrier)
  __device__ __forceinline__ void flush_cards(int& crow, int ncq) {
    if (ncq == 0) return;
    wsync();
    for (int q = wid * CQW; q < wid * CQW + ncq; ++q) {
      const int r = DP_CHK((int)cardq[q], nc, nrows, 3), k = r - nc;
      int a, len;
      const uint32_t info = NW > 1 && !N16 ? (uint32_t)cardq[CQ + q] : ROW_INFO_NONE;
      if (info != ROW_INFO_NONE) {  // the range from the row's watch entry
        a = (int)(info >> 8);
        len = (int)(info & 255u);
      } else {
        a = card_off[k];
        len = (int)card_off[k + 1] - a;
      }
      const int bound = card_bound[k];
      if (len > 64) {  // long rows: the wavefront in chunks of 64 positions
        card_long(r, a, len, bound, crow);
        continue;
      }
      const int v = lane < len ? (int)card_lits[a + lane] : -1;
      const int x = v >= 0 ? val[v] : 0;
      DP_VIS_ADD((v >= 0 ? sizeof(IX) + 1 : 0) + (lane == 0 ? 3 * sizeof(IX) : 0));  // positions, values; offsets, bound
      const int cnt = __popcll(__ballot(v >= 0 && x > 0));
      if (cnt > bound) { crow = min(crow, r); continue; }
      if (!__ballot(v >= 0 && x == 0)) continue;
      const bool start = v >= 0 && (lane == 0 || (int)card_lits[a + lane - 1] != v);
      const uint64_t ms = __ballot(start);
      const uint64_t after = lane < 63 ? ms >> (lane + 1) : 0ull;
      const int run = (after ? lane + 1 + __ffsll((unsigned long long)after) - 1 : len) - lane;
      note_all(start && x == 0 && cnt + run > bound ? 2 * v + 1 : -1, r);
    }
  }
  __device__ __forceinline__ void card_long(int r, int a, int len, int bound, int& crow) {
    int cnt = 0;
    bool any = false;
    for (int j0 = 0; j0 < len; j0 += 64) {
      const int j = j0 + lane;
      const int v = j < len ? (int)card_lits[a + j] : -1;
      const int x = v >= 0 ? val[v] : 0;
      DP_VIS_ADD(v >= 0 ? sizeof(IX) + 1 : 0);
      cnt += __popcll(__ballot(v >= 0 && x > 0));
      any |= __ballot(v >= 0 && x == 0) != 0ull;
    }
    if (cnt > bound) { crow = min(crow, r); return; }
    if (!any) return;
    for (int j0 = 0; j0 < len; j0 += 64) {
      const int j = j0 + lane;
      const int v = j < len ? (int)card_lits[a + j] : -1;
      const bool start = v >= 0 && (j == 0 || (int)card_lits[a + j - 1] != v);
      int e = j + 1;
      if (start)
        while (e < len && (int)card_lits[a + e] == v) ++e;
      const bool f = start && val[v] == 0 && cnt + (e - j) > bound;
      note_all(f ? 2 * v + 1 : -1, r);
    }
  }

  // learned rows are evaluated in every round (threads over rows)
  __device__ __forceinline__ void eval_learned(int& crow) {
    for (int j0 = learn_lo; j0 < nl; j0 += NT) {
      const int j = j0 + tid;
      note_all(j < nl ? clause_unit(nrows + j, crow) : -1, nrows + j);
    }
  }

  __device__ __forceinline__ void clear_touched(int nt) {
    if constexpr (NW > 1) bar();  // every read of imp in this round is done
    for (int i = tid; i < nt; i += NT) imp[(int)touched[i]] = (IMP)IMP_NONE;
    gsync();
    if (tid == 0) scal[S_NTOUCHED] = 0;
    gsync();
  }

  __device__ __forceinline__ void commit(int l, int r, int start, int i) {
    const int v = l >> 1;
    val[v] = (l & 1) ? -1 : 1;
    reason[v] = enc(r);
    rs[v] = enc(start);
    put_trail(start + i, l);
    imp[l] = (IMP)IMP_NONE;
  }

  // The round's table slots back to empty (every thread has read them).
  __device__ __forceinline__ void clear_slots(int nt) {
    gsync();
    for (int i = tid; i < nt; i += NT) {
      const int h = tl[i] >> 1;
      hkey[h] = -1; hrp[h] = (uint32_t)INF; hrn[h] = (uint32_t)INF;
    }
    gsync();
  }

  // finish_round on the LDS table (hmode): one exchange, then the commit.
  // Returns 2 when the table overflowed: nothing was committed and the caller
  // redoes the round on the HBM arrays (the outcome does not depend on where
  // the round is kept).  The bank's counters are read here and reset at the
  // start of the round after next (run_round), past this round's last barrier.
  __device__ __forceinline__ int finish_round_lds(int crow) {
#ifdef DP_STAMPS
    const int64_t tx0 = stamp();
#endif
    const int cr = g_min(crow);  // the notes, the AtMost flush and the counters are complete
#ifdef DP_STAMPS
    const int64_t tx1 = stamp();
    DP_ACC(30, tx1 - tx0);  // the round's exchange
#endif
    const int nt = DP_CHK(scal[S_NTB + rb], 0, 2 * (hmask + 1) + 1, 4);
    const bool ovf = scal[S_OVB + rb] != 0;
    const int cvx = scal[S_CVB + rb];
    if (ovf) {
      clear_slots(nt);
      return 2;
    }
    if (cr != INF) {
      c_row = cr;
      clear_slots(nt);
      ck = CK_ROW;
      return -1;
    }
    if (cvx != 0) {
      c_var = INF - cvx;
      const int h = slot_of(c_var);
      c_rp = (int)hrp[h]; c_rn = (int)hrn[h];
      ck = CK_VAR; c_row = tlen;  // bound: every variable assigned so far
      clear_slots(nt);
      return -1;
    }
    // no variable is listed twice: each thread reads and empties its own slots
    const int start = tlen;
    for (int i = tid; i < nt; i += NT) {
      const int e = tl[i], h = e >> 1, v = hkey[h];
      const int l = 2 * v + (e & 1);
      const int r = (int)((e & 1) ? hrn[h] : hrp[h]);
      val[v] = (l & 1) ? -1 : 1;
      reason[v] = enc(r);
      rs[v] = enc(start);
      put_trail(start + i, l);
      hkey[h] = -1; hrp[h] = (uint32_t)INF; hrn[h] = (uint32_t)INF;
    }
    tlen += nt;
    gsync();
#ifdef DP_STAMPS
    DP_ACC(31, stamp() - tx1);  // the commit
#endif
    return 0;
  }

  // Commit the implications of the round, or report its conflict: the lowest
  // conflicting row, else the lowest variable implied both ways.
  __device__ __forceinline__ int finish_round(int crow) {
    if constexpr (LR) {
      if (hmode) return finish_round_lds(crow);
    }
    gsync();
    const int nt = DP_CHK(scal[S_NTOUCHED], 0, 2 * nv + 1, 4);
    if (g_any(crow != INF)) {
      c_row = g_min(crow);
      clear_touched(nt);
      ck = CK_ROW;
      return -1;
    }
    const int start = tlen;
    if (nt <= NT) {  // one literal per thread: a single pass
      const int l = tid < nt ? DP_CHK((int)touched[tid], 0, 2 * nv, 5) : 0;
      const int r = tid < nt ? DP_CHK(imp_get(l), 0, nrows + nl, 6) : 0,
                rn = tid < nt ? imp_get(l ^ 1) : INF;
      const int cv = rn != INF ? (l >> 1) : INF;
      if (g_any(cv != INF)) {
        c_var = g_min(cv);
        c_rp = imp_get(2 * c_var); c_rn = imp_get(2 * c_var + 1);
        ck = CK_VAR; c_row = tlen;  // bound: every variable assigned so far
        clear_touched(nt);
        return -1;
      }
      if (tid < nt) commit(l, r, start, tid);
    } else {
      int cv = INF;
      for (int i = tid; i < nt; i += NT) {
        const int l = touched[i];
        if (imp_get(l ^ 1) != INF) cv = min(cv, l >> 1);
      }
      if (g_any(cv != INF)) {
        c_var = g_min(cv);
        c_rp = imp_get(2 * c_var); c_rn = imp_get(2 * c_var + 1);
        ck = CK_VAR; c_row = tlen;
        clear_touched(nt);
        return -1;
      }
      for (int i = tid; i < nt; i += NT) {
        const int l = DP_CHK((int)touched[i], 0, 2 * nv, 7);
        commit(l, DP_CHK(imp_get(l), 0, nrows + nl, 8), start, i);
      }
    }
    if (tid == 0) scal[S_NTOUCHED] = 0;
    tlen += nt;
    gsync();
    return 0;
  }

  __device__ __forceinline__ int extra_check() {
    int cnt = 0, nun = 0;
    for (int b = 0; b < nv; b += NT) {
      const int v = b + tid;
      const bool ex = v < nv && getb(extra, v);
      const int x = ex ? val[v] : 0;
      cnt += ex && x > 0;
      nun += ex && x == 0;
    }
    cnt = g_sum(cnt);
    nun = g_sum(nun);
    if (cnt > extra_w) { ck = CK_EXTRA; return -1; }
    if (cnt == extra_w && nun > 0) {
      const int start = tlen;
      int run = tlen;
      for (int b = 0; b < nv; b += NT) {
        const int v = b + tid;
        const bool f = v < nv && getb(extra, v) && val[v] == 0;
        const int at = claim(f, run);
        if (f) {
          val[v] = -1; reason[v] = enc(R_EXTRA); rs[v] = enc(start);
          put_trail(at, 2 * v + 1);
        }
      }
      claim_end(run);
      tlen = run;
      gsync();
      return 1;
    }
    return 0;
  }

  __device__ __forceinline__ int propagate() {
    const int r = propagate_rounds();
    if constexpr (LR) bar();  // the rounds' global stores, for every wavefront
    return r;
  }
  __device__ __forceinline__ int propagate_rounds() {
    for (;;) {
      if (qhead == tlen) {
        if (extra_mode) {
          const int r = extra_check();
          if (r < 0) return -1;
          if (r > 0) continue;
        }
        return tlen == nv ? 1 : 0;
      }
      const int lo = qhead, hi = tlen;
      qhead = hi;
#ifdef DP_STAMPS
      const int64_t t0 = stamp();
      DP_ACC(2, 1);
      DP_ACC(3, hi - lo == 1);
#endif
      // the frontier from the trail ring (LDS) unless the ring has wrapped
      // over it; then from the trail in HBM, whose stores bar() drains
      const bool ring = LR && hi - lo <= hmask + 1;
      if constexpr (LR)
        if (!ring) bar();
      // (two instantiations: one accessor choosing between the LDS ring and
      // the trail in HBM compiled to flat loads, which wait on both the
      // vector-memory and the LDS counters, in every round's frontier read)
      int rr;
      if (LR && ring)
        rr = run_round([&](int& crow) { visit_frontier(lo, hi, crow, [&](int i) { return (int)fr[i & hmask]; }); });
      else
        rr = run_round([&](int& crow) { visit_frontier(lo, hi, crow, [&](int i) { return (int)trail[i]; }); });
      if (rr < 0) return -1;
#ifdef DP_STAMPS
      DP_ACC(0, stamp() - t0);
#endif
    }
  }

  // One round: `visit` evaluates the rows the round reaches (into crow and
  // the implication table), then the round is finished.  With the LDS table
  // full the round is redone on the HBM arrays (returns finish_round's value).
  template <class F>
  __device__ __forceinline__ int run_round(F&& visit) {
    int crow = INF;
    const uint32_t vis0 = vis;
    if constexpr (LR) {
      lds_sync = true;
      rb ^= 1;  // this round's bank; the other one was read before the last round's final barrier
      if (tid == 0) { scal[S_NTB + (rb ^ 1)] = 0; scal[S_CVB + (rb ^ 1)] = 0; scal[S_OVB + (rb ^ 1)] = 0; }
    }
    visit(crow);
    int r = finish_round(crow);
    if constexpr (LR) {
      lds_sync = false;
      if (r == 2) {
        DP_ACC(25, 1);  // diagnostic: rounds redone on the HBM arrays
        vis = vis0;
        hmode = false;
        crow = INF;
        visit(crow);
        r = finish_round(crow);
        hmode = true;
      }
      if (r < 0) bar();  // the callers' conflict analysis reads the trail
    }
    return r;
  }

  // The rows watched by the frontier trail[lo..hi) (front(i) = trail[i]),
  // then the AtMost queue and the learned rows.
  template <class FR>
  __device__ __forceinline__ void visit_frontier(int lo, int hi, int& crow, FR&& front) {
#ifdef DP_STAMPS
      const int64_t t0 = stamp();
#endif
      int ncq = 0;
      const int hint = pre_lo;  // (valid for this round only)
      pre_lo = -1;
      if (hi - lo == 1) {  // one new literal: threads over its watch list
        int a, e;
        if (lo == hint) {
          a = pre_a; e = pre_e;
        } else {
          const int l = DP_CHK(front(lo), 0, 2 * nv, 10);
          a = w_off[l]; e = w_off[l + 1];
        }
        for (int k0 = a; k0 < e; k0 += NT) {
          visit_at(k0 + tid < e ? k0 + tid : -1, crow, ncq);
        }
#ifdef DP_STAMPS
        DP_ACC(8, stamp() - t0);
        DP_ACC(12, e - a);
#endif
      } else {
        // Flattened: each wavefront takes 64 frontier literals of the chunk,
        // scans their watch-range lengths by DPP and visits the concatenated
        // entries 64 at a time from its own segment of the work list, with
        // no barrier between wavefronts (the round's exchange follows the
        // AtMost flush).  A wavefront whose entries overflow its segment
        // walks its literals' lists one at a time.
        // The frontier is dealt evenly: each wavefront takes S <= 64
        // consecutive literals per step (a frontier of 128 literals gives
        // each of 8 wavefronts 16, so their ~50 entries are one pass of its
        // lanes, not three passes of one wavefront's 64 literals).
        constexpr int SEGW = WBUF / NW;
        IX* wb = wbuf + wid * SEGW;
        const int S = NW == 1 ? 64 : min(64, (hi - lo + NW - 1) / NW);
        for (int b = lo; b < hi; b += S * NW) {
          const int i = b + wid * S + lane;
          int cnt = 0, a = 0;
          if (lane < S && i < hi) {
            const int l = DP_CHK(front(i), 0, 2 * nv, 11);
            a = w_off[l];
            cnt = (int)w_off[l + 1] - a;
          }
#ifdef DP_STAMPS
          const int64_t tf0 = stamp();
#endif
          const int incl = wave_incl_scan(cnt);
          const int total = __builtin_amdgcn_readlane(incl, 63);  // this wavefront's entries
#ifdef DP_STAMPS
          if constexpr (NW == 1) DP_ACC(26, total);  // watch entries a flattened chunk visits
#endif
          if (total <= SEGW) {
#ifdef DP_STAMPS
            const int64_t tf1 = stamp();
            if constexpr (NW > 1) DP_ACC(27, tf1 - tf0);  // ranges: scan
#endif
            // every frontier literal writes its watch range into the segment
            for (int k = 0, at = incl - cnt; k < cnt; ++k) wb[at + k] = enc(a + k);
            wsync();
#ifdef DP_STAMPS
            const int64_t tf2 = stamp();
            if constexpr (NW > 1) DP_ACC(28, tf2 - tf1);  // the work list
#endif
            for (int t0 = 0; t0 < total; t0 += 64) {
              visit_at(t0 + lane < total ? DP_CHK((int)wb[t0 + lane], 0, nwatch, 12) : -1, crow, ncq);
            }
#ifdef DP_STAMPS
            if constexpr (NW > 1) DP_ACC(29, stamp() - tf2);  // the visits
#endif
            wsync();  // (the segment is rewritten by the next chunk)
          } else {
            // a very large chunk: this wavefront's literals one at a time
            const int f0 = b + S * wid, n = max(0, min(S, hi - f0));
            for (int e = 0; e < n; ++e) {
              const int l = front(f0 + e);
              const int a2 = w_off[l], e2 = w_off[l + 1];
              for (int k0 = a2; k0 < e2; k0 += 64) {
                visit_at(k0 + lane < e2 ? k0 + lane : -1, crow, ncq);
              }
            }
          }
        }
#ifdef DP_STAMPS
        DP_ACC(9, stamp() - t0);
        DP_ACC(13, hi - lo);
#endif
      }
#ifdef DP_STAMPS
      const int64_t tf = stamp();
      DP_ACC(15, ncq);  // (multi-wave: wavefront 0's queue)
      flush_cards(crow, ncq);
      const int64_t tq = stamp();
      DP_ACC(10, tq - tf);
      DP_ACC(14, nl - learn_lo);
      eval_learned(crow);
      DP_ACC(11, stamp() - tq);
      DP_ACC(1, stamp() - t0);
#else
      flush_cards(crow, ncq);
      eval_learned(crow);
#endif
  }

  // Can AtMost row k fire on the empty assignment (a variable listed more
  // times than the bound)?
  __device__ __forceinline__ bool card_fires(int k) const {
    const int a = card_off[k], b = card_off[k + 1], bound = card_bound[k];
    if (b - a <= bound) return false;
    if (b - a <= 16) {  // the positions by independent loads, runs in registers
      int v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = a + i < b ? (int)card_lits[a + i] : -1 - i;
      int run = 1, best = 1;
#pragma unroll
      for (int i = 1; i < 16; ++i) {
        run = v[i] == v[i - 1] ? run + 1 : 1;
        best = max(best, run);
      }
      return best > bound;
    }
    for (int j = a; j < b;) {
      int e = j + 1;
      while (e < b && card_lits[e] == card_lits[j]) ++e;
      if (e - j > bound) return true;
      j = e;
    }
    return false;
  }

  // The base scope (solve.go:63-79): one round evaluates every (enabled) row;
  // on the empty assignment only clauses of length <= 1 and AtMost rows with
  // a multiplicity over the bound can fire, so a sweep visits just those.
  __device__ __forceinline__ int base_propagate() {
    const int r = run_round([&](int& crow) {
      int ncq = 0;
      for (int i0 = 0; i0 < nrows; i0 += NT) {
        const int row = i0 + tid;
        const bool f = row < nc ? (int)clause_off[row + 1] - (int)clause_off[row] <= 1
                                : row < nrows && card_fires(row - nc);
        visit(f ? row : -1, crow, ncq);
      }
      flush_cards(crow, ncq);
      eval_learned(crow);
    });
    if (r < 0) return -1;
    return propagate();
  }

  __device__ __forceinline__ void truncate_to(int mark) {
#ifdef DP_STAMPS
    const int64_t t0 = stamp();
    truncate_to_(mark);
    DP_ACC(19, stamp() - t0);
  }
  __device__ __forceinline__ void truncate_to_(int mark) {
#endif
    gsync();
    for (int i = mark + tid; i < tlen; i += NT) val[DP_CHK((int)trail[i], 0, 2 * nv, 14) >> 1] = 0;
    tlen = qhead = mark;
    gsync();
  }

  // gini Untest() (search.go:84): the learned rows decide the restored scope
  __device__ __forceinline__ int untest_to(int mark) {
    truncate_to(mark);
    if (nl > learn_lo) {
      if (run_round([&](int& crow) { eval_learned(crow); }) < 0) return -1;
      return propagate();
    }
    return tlen == nv ? 1 : 0;
  }

  __device__ __forceinline__ void assign_one(int l, int why, int decision) {
    // Callers decide on reads of val (test_assume's lit_val, dpll's
    // violated): with several wavefronts, no thread may still be reading when
    // thread 0 writes, or a late wavefront sees the new value and branches
    // differently (one wavefront reads before it writes, in program order).
    if constexpr (NW > 1) bar();
    if (tid == 0) {
      const int v = DP_CHK(l, 0, 2 * nv, 30) >> 1;
      val[v] = (l & 1) ? -1 : 1; reason[v] = enc(decision >= 0 ? -3 - decision : why);
      rs[v] = enc(tlen); put_trail(tlen, l);
    }
    ++tlen;
    gsync();
  }

  // gini Assume(m) + Test() (search.go:75-76)
  // (xv: val[l >> 1] when the caller has it already; wa, we: l's watch range)
  __device__ __forceinline__ int test_assume(int l, int xv = 2, int wa = 0, int we = -1) {
    ++steps;
    const int x = xv == 2 ? lit_val(l) : ((l & 1) ? -xv : xv);
    if (x > 0) return propagate();
    if (x < 0) { ck = CK_ASSUME; c_var = l >> 1; return -1; }
    if (we >= 0) { pre_lo = tlen; pre_a = wa; pre_e = we; }
    assign_one(l, R_DEC, -1);
    return propagate();
  }

  // ------------------------------------------------------------------
  // conflict analysis (oracle: analyze)
  // ------------------------------------------------------------------
  __device__ __forceinline__ void mark_push(int v) {
    const uint32_t bit = 1u << (v & 31);
    const uint32_t old = atomicOr(&seen[v >> 5], bit);
    if (!(old & bit)) touched[atomicAdd(&scal[S_NWORK], 1)] = enc(v);
  }
  __device__ __forceinline__ void set_bit_atomic(uint32_t* b, int i) { atomicOr(&b[i >> 5], 1u << (i & 31)); }

  // antecedents of row r for variable u, whose round started at trail
  // position bound (serial in the calling thread)
  __device__ __forceinline__ void ante_serial(int r, int u, int bound) {
    r = DP_CHK(r, 0, nrows + nl, 15);
    if (r < nc || r >= nrows) {
      const IX* lits = clause_lits;
      int a, b;
      if (r < nc) { a = clause_off[r]; b = clause_off[r + 1]; set_bit_atomic(used, row_key(r)); }
      else {
        lits = l_lits;
        a = DP_CHK((int)l_off[r - nrows], 0, lcap + 1, 35);
        b = DP_CHK((int)l_off[r - nrows + 1], 0, lcap + 1, 36);
      }
      for (int j = a; j < b; ++j) {
        const int v = (int)lits[j] >> 1;
        if (v != u) mark_push(v);
      }
    } else {
      const int k = r - nc;
      set_bit_atomic(used, row_key(r));
      for (int j = card_off[k]; j < card_off[k + 1]; ++j) {
        const int v = card_lits[j];
        if (v != u && val[v] > 0 && (int)rs[v] < bound) mark_push(v);
      }
    }
  }
  // the epilogue bound's antecedents (true extras assigned before bound)
  __device__ __forceinline__ void extra_serial(int u, int bound) {
    for (int v = 0; v < nv; ++v)
      if (v != u && getb(extra, v) && val[v] > 0 && (int)rs[v] < bound) mark_push(v);
  }

  __device__ __forceinline__ void analyze() {
#ifdef DP_STAMPS
    const int64_t t0 = stamp();
    analyze_();
    DP_ACC(17, stamp() - t0);
    DP_ACC(22, 1);
  }
  __device__ __forceinline__ void analyze_() {
#endif
    gsync();
    if (tid == 0) {
      scal[S_NWORK] = 0;
      if (ck == CK_ROW) ante_serial(c_row, -1, INF);
      else if (ck == CK_VAR) { ante_serial(c_rp, c_var, c_row); ante_serial(c_rn, c_var, c_row); }
      else if (ck == CK_EXTRA) extra_serial(-1, INF);
      else if (ck == CK_ASSUME) mark_push(c_var);  // the assumed literal is false: its reasons
    }
    gsync();
    int head = 0;
    for (;;) {
      const int nw = scal[S_NWORK];
      if constexpr (NW > 1) bar();  // every thread read nw before any grows it
      if (head >= nw) break;
      for (int i = head + tid; i < nw; i += NT) {
        const int u = DP_CHK((int)touched[i], 0, nv, 16);
        const int r = dec(reason[u]);
        if (r >= 0) ante_serial(r, u, rs[u]);
        else if (r == R_EXTRA) extra_serial(u, rs[u]);
        else if (r <= -3) set_bit_atomic(dset, DP_CHK(-3 - r, 0, nv, 32));  // Solve() decision
        else if (collect_guess && getb(inS, u)) set_bit_atomic(fg, u);
      }
      head = nw;
      gsync();
    }
    const int nw = scal[S_NWORK];
    for (int i = tid; i < nw; i += NT) {
      const int v = touched[i];
      atomicAnd(&seen[v >> 5], ~(1u << (v & 31)));
    }
    gsync();
  }

  // ------------------------------------------------------------------
  // Solve(): CDCL from a consistent fixpoint (oracle: first_violated / dpll)
  // ------------------------------------------------------------------
  // Is clause row c violated by the all-false completion of the current
  // assignment?  (oracle: first_violated)  fu = its first unassigned
  // positive literal.
  __device__ __forceinline__ bool violated(int c, int& fu, uint32_t info = ROW_INFO_NONE) const {
    fu = -1;
    int ja, jb;
    if (!N16 && info != ROW_INFO_NONE) {
      ja = (int)(info >> 8);
      jb = ja + (int)(info & 255u);
    } else {
      ja = clause_off[c];
      jb = clause_off[c + 1];
    }
    for (int j = ja; j < jb; ++j) {
      const int l = clause_lits[j];
      const int x = val[l >> 1];
      if (l & 1) {
        if (x != 1) return false;
      } else {
        if (x == 1) return false;
        if (x == 0 && fu < 0) fu = l;
      }
    }
    return true;
  }

  // The lowest clause row the all-false completion violates -> its first
  // unassigned positive literal (the decision), or -1.  Such a row has a
  // positive literal but no true one, and every negative literal on a true
  // variable, so, when it has a negative literal, it is in the watch list of
  // some variable assigned true: threads scan those lists instead of every
  // clause row (same answer as the oracle's full scan).  Rows without a
  // negative literal are units (assigned at the base) except an AtMost
  // network's (g a b) rows: records with auxiliary variables scan every row.
  __device__ __forceinline__ int first_violated() {
#ifdef DP_STAMPS
    const int64_t t0 = stamp();
    const int r = first_violated_();
    DP_ACC(16, stamp() - t0);
    DP_ACC(18, 1);
    return r;
  }
  __device__ __forceinline__ int first_violated_() {
#endif
    int best = INF;
    // (two-watched lists no longer hold every row a true literal occurs in:
    // scan the rows)
    if (nc <= 4 * NT || scal[S_POSROWS]) {
      // few rows: every thread scans its rows in ascending order (the
      // oracle's scan, a short dependent chain per thread)
      for (int c = tid; c < nc; c += NT) {
        int fu;
        if (row_on(c) && violated(c, fu)) { best = c; break; }
      }
      best = g_min(best);
      if (best == INF) return -1;
      int fu;
      violated(best, fu);
      return fu;
    }
    // Flattened: a wavefront takes 64 trail entries, scans their watch-list
    // lengths, and walks the concatenated (literal, entry) pairs 64 at a
    // time, so a long list does not hold the other lanes.  Loop bounds
    // are wave-uniform (i0 per wave, total by shuffle).
    for (int i0 = 64 * wid; i0 < tlen; i0 += NT) {
      const int i = i0 + lane;
      const int l = i < tlen ? (int)trail[i] : 1;
      int s = 0, n = 0;
      if (!(l & 1)) { s = (int)w_off[l]; n = (int)w_off[l + 1] - s; }
      const int inc = wave_incl_scan(n);
      const int total = __builtin_amdgcn_readlane(inc, 63);
      for (int base = 0; base < total; base += 64) {
        const int f = base + lane;
        int j = 0;  // lowest lane whose inclusive count exceeds f
        for (int step = 32; step; step >>= 1)
          if (__shfl(inc, j + step - 1) <= f) j += step;
        const int sj = __shfl(s, j), ej = __shfl(inc, j) - __shfl(n, j);
        if (f < total) {
          const int2 e = went(sj + f - ej);
          const int c = e.x;
          int fu;
          if (c < nc && c < best && row_on(c) && violated(c, fu, (uint32_t)e.y)) best = c;
        }
      }
    }
    best = g_min(best);
    if (best == INF) return -1;
    int fu;
    violated(best, fu);
    return fu;
  }

  __device__ __forceinline__ void save_model() {
#ifdef DP_STAMPS
    const int64_t t0 = stamp();
    save_model_();
    DP_ACC(20, stamp() - t0);
  }
  __device__ __forceinline__ void save_model_() {
#endif
    for (int b = 0; b < nv; b += NT) {
      const int v = b + tid;
      const uint64_t m = __ballot(v < nv && val[v] > 0);
      const int wd = (b + 64 * wid) >> 5;
      if (lane == 0 && wd < nbv) {
        model[wd] = (uint32_t)m;
        if (wd + 1 < nbv) model[wd + 1] = (uint32_t)(m >> 32);
      }
    }
    gsync();
  }

  __device__ __forceinline__ void clear_bits(uint32_t* bs, int n) {
    for (int i = tid; i < bits_words(n); i += NT) bs[i] = 0;
    gsync();
  }

  // Solve() decision i's literal: the trail entry at its mark, unflipped
  __device__ __forceinline__ int dlit(int i) const {
    return (int)trail[(int)d_mark[i]] ^ (int)getb(d_flip, i);
  }

  __device__ __forceinline__ int dpll() {
    const int root = tlen, nl0 = nl;
    int nd = 0, r;
    bool decide = true;
    for (;;) {
      if (decide) {
        const int l = first_violated();
        if (l < 0) { save_model(); r = RS_SAT; break; }
        if (++steps > budget) { budget_hit = true; r = RS_BUDGET; break; }
        if (tid == 0) {
          d_mark[nd] = enc(tlen);  // the decision's literal is trail[d_mark[nd]]
          d_flip[nd >> 5] &= ~(1u << (nd & 31));
        }
        assign_one(l, R_DEC, nd);
        ++nd;
      }
      // the one propagation site of Solve(): after a decision or an assertion
      if (propagate() >= 0) { decide = true; continue; }
      decide = false;
      clear_bits(dset, nd);
      analyze();
      // h = highest decision reached, b = the next one below (or -1)
      int h = -1, b = -1, n = 0;
      for (int wi = bits_words(nd) - 1; wi >= 0 && b < 0; --wi) {
        uint32_t x = ld_bits(&dset[wi]);
        while (x && b < 0) {
          const int i = wi * 32 + 31 - __clz(x);
          x &= ~(1u << (i & 31));
          if (h < 0) h = i; else b = i;
        }
      }
      for (int wi = 0; wi < bits_words(nd); ++wi) n += __popc(ld_bits(&dset[wi]));
      if (h < 0) { r = RS_UNSAT; break; }
      if (++steps > budget) { budget_hit = true; r = RS_BUDGET; break; }
      const int lat = DP_CHK((int)l_off[nl], 0, lcap + 1, 26);
      if (nl < L_MAX && lat + n <= lcap) {
        // learned row: the negated decisions it met
        int run = lat;
        for (int base = 0; base < nd; base += NT) {
          const int i = base + tid;
          const bool in = i < nd && ((ld_bits(&dset[i >> 5]) >> (i & 31)) & 1u);
          const int at = claim(in, run);
          if (in) l_lits[DP_CHK(at, 0, lcap, 27)] = enc(dlit(i) ^ 1);
        }
        claim_end(run);
        if (tid == 0) l_off[nl + 1] = enc(run);
        ++nl;
        gsync();
        const int lh = dlit(h);
        nd = b + 1;
        truncate_to(DP_CHK((int)d_mark[nd], 0, nv + 1, 24));
        assign_one(lh ^ 1, nrows + nl - 1, -1);
      } else {
        while (nd > 0 && getb(d_flip, nd - 1)) --nd;
        if (nd == 0) { r = RS_UNSAT; break; }
        const int lf = dlit(nd - 1);  // before its flip bit is set
        truncate_to(DP_CHK((int)d_mark[nd - 1], 0, nv + 1, 25));
        if (tid == 0) d_flip[(nd - 1) >> 5] |= 1u << ((nd - 1) & 31);
        gsync();
        assign_one(lf ^ 1, R_DEC, nd - 1);
      }
    }
    truncate_to(root);
    nl = nl0;
    return r;
  }

  // ------------------------------------------------------------------
  // search.Do (search.go:158-203)
  // ------------------------------------------------------------------
  int dq_head, dq_n, ng, result;
  // A guess's watch range, loaded with its other reads, for the round whose
  // frontier is the guess alone (trail[pre_lo])
  int pre_lo, pre_a, pre_e;
  bool class_b, solve_unsat, last_solve;
  bool final_from_solve;  // the search's last failure came from Solve() (else Test/Untest)

  // choice lists: rows 0..nch-1; the singleton list of anchor v is nch + v
  __device__ __forceinline__ int list_len(int list) const {
    if (list >= nch) return 1;
    if (rowref) {
      const int r = rowref[list];
      return (int)clause_off[r + 1] - (int)clause_off[r] - 1;
    }
    return (int)choice_off[list + 1] - (int)choice_off[list];
  }
  __device__ __forceinline__ int list_at(int list, int i) const {
    if (list >= nch) return list - nch;
    if (rowref) return (int)clause_lits[(int)clause_off[rowref[list]] + 1 + i] >> 1;
    return (int)choice_lits[(int)choice_off[list] + i];
  }
  __device__ __forceinline__ void dq_push_back(int list, int idx) {
    int at = dq_head + dq_n;
    if (at >= cap) at -= cap;
    if (tid == 0) { dq[2 * at] = enc(list); dq[2 * at + 1] = enc(idx); }
    ++dq_n;
  }
  __device__ __forceinline__ void dq_push_front(int list, int idx) {
    dq_head = dq_head == 0 ? cap - 1 : dq_head - 1;
    if (tid == 0) { dq[2 * dq_head] = enc(list); dq[2 * dq_head + 1] = enc(idx); }
    ++dq_n;
  }

  // the guessed variable of a stack entry (list, idx | G_SKIP), or -1
  __device__ __forceinline__ int guess_m(int list, int idxf) const {
    const int idx = idxf & ~G_SKIP;
    return !(idxf & G_SKIP) && idx < list_len(list) ? list_at(list, idx) : -1;
  }

  // PushGuess, search.go:34-77
  __device__ __forceinline__ void push_guess() {
#ifdef DP_STAMPS
    const int64_t tpg = stamp();
#endif
    gsync();
    const int list = DP_CHK((int)dq[2 * dq_head], 0, nch + nv, 17), idx = DP_CHK((int)dq[2 * dq_head + 1], 0, nv + 1, 18);
    dq_head = dq_head + 1 == cap ? 0 : dq_head + 1;
    --dq_n;
    // The list's entries are src[base + i] >> sh, i < len (list_len /
    // list_at with the list resolved once), and everything that depends on
    // the guessed variable is loaded together: the dependent LDS round trips
    // of a push are the list's row, its offsets, its entries, then their
    // inS words with m's child rows and value.
    const bool single = list >= nch;  // an anchor's singleton list
    int len = 1, base = 0, sh = 0;
    const IX* src = clause_lits;
    if (!single) {
      if (rowref) {
        const int r = rowref[list];
        base = (int)clause_off[r] + 1;
        len = (int)clause_off[r + 1] - base;
        sh = 1;
      } else {
        base = choice_off[list];
        len = (int)choice_off[list + 1] - base;
        src = choice_lits;
      }
    }
    auto entry = [&](int i) { return single ? list - nch : (int)src[base + i] >> sh; };
    int m = idx < len ? entry(idx) : -1;
    const int mc = m >= 0 ? m : 0;
    const int c0 = var_choice_off[mc], c1 = var_choice_off[mc + 1], xm = val[mc];
    const int wa = w_off[2 * mc], we = w_off[2 * mc + 1];
    bool any = false;
    for (int i = tid; i < len; i += NT) any |= getb(inS, entry(i));
    const bool skip = g_any(any);
    if (skip) m = -1;
    else if (idx >= len) class_b = true;  // exhausted choice
    // its children: one choice per choice row (pop_guess recounts them),
    // appended in row order, a thread per row
    const int nchild = m >= 0 ? c1 - c0 : 0;
    for (int k = tid; k < nchild; k += NT) {
      int at = dq_head + dq_n + k;
      if (at >= cap) at -= cap;
      dq[2 * at] = enc(c0 + k); dq[2 * at + 1] = enc(0);
    }
    dq_n += nchild;
    if (tid == 0) {
      IX* g = stk + 3 * ng;
      g[0] = enc(list); g[1] = enc(idx | (skip ? G_SKIP : 0)); g[2] = enc(tlen);
      if (m >= 0) atomicOr(&inS[m >> 5], 1u << (m & 31));
    }
    ++ng;
    gsync();
    if (m < 0) return;
    if (steps >= budget) { budget_hit = true; result = 0; return; }
#ifdef DP_STAMPS
    DP_ACC(21, stamp() - tpg);
#endif
    result = test_assume(2 * m, xm, wa, we);
    last_solve = false;
  }

  // PopGuess, search.go:79-98
  __device__ __forceinline__ void pop_guess() {
    gsync();
    --ng;
    const IX* g = stk + 3 * ng;
    const int list = DP_CHK((int)g[0], 0, nch + nv, 19), idxf = (int)g[1],
              mark = DP_CHK((int)g[2], 0, nv + 1, 23);
    const int idx = DP_CHK(idxf & ~G_SKIP, 0, nv + 1, 20);
    // guess_m with the list resolved once (as in push_guess)
    int m = -1;
    if (!(idxf & G_SKIP)) {
      if (list >= nch) {
        m = idx < 1 ? list - nch : -1;
      } else if (rowref) {
        const int r = rowref[list];
        const int a = (int)clause_off[r] + 1, len = (int)clause_off[r + 1] - a;
        if (idx < len) m = (int)clause_lits[a + idx] >> 1;
      } else {
        const int a = choice_off[list], len = (int)choice_off[list + 1] - a;
        if (idx < len) m = choice_lits[a + idx];
      }
    }
    m = DP_CHK(m, -1, nv, 21);
    const int children = m >= 0 ? (int)var_choice_off[m + 1] - (int)var_choice_off[m] : 0;
    gsync();
    if (m >= 0) {
      if (tid == 0) inS[m >> 5] &= ~(1u << (m & 31));
      gsync();
      result = untest_to(mark);
      last_solve = false;
    }
    dq_n -= children;
    dq_push_front(list, idx + (m >= 0 ? 1 : 0));
    gsync();
  }

  // Solve() within the search: a failure learns the nogood of the guesses its
  // refutation reached (oracle: be_solve / learn)
  __device__ __forceinline__ int search_solve() {
    clear_bits(fg, nv);
    collect_guess = true;
    const int r = dpll();
    collect_guess = false;
    if (r == RS_UNSAT) {
      int n = 0;
      for (int wi = tid; wi < nbv; wi += NT) n += __popc(ld_bits(&fg[wi]));
      n = g_sum(n);
      const int lat = l_off[nl];
      if (nl < L_MAX && lat + n <= lcap) {
        int run = lat;
        for (int b = 0; b < nv; b += NT) {
          const int v = b + tid;
          const bool in = v < nv && ((ld_bits(&fg[v >> 5]) >> (v & 31)) & 1u);
          const int at = claim(in, run);
          if (in) l_lits[at] = enc(2 * v + 1);
        }
        claim_end(run);
        if (tid == 0) l_off[nl + 1] = enc(run);
        ++nl;
        gsync();
      }
    }
    return r;
  }

  // Returns the search result; leaves the final guess set in inS.
  __device__ __forceinline__ int search() {
    dq_head = dq_n = ng = 0;
    result = 0;
    class_b = solve_unsat = last_solve = false;
    for (int i = 0; i < na; ++i) dq_push_back(nch + (int)anchors[i], 0);
    // `used` collects the identities of every conflict analysis of the
    // search's Solve() calls (the derivations of its learned nogoods): with
    // the final root conflict, an unsatisfiable set when the search fails
    // (oracle: search_do).  With tracing, `used` holds the current step's
    // identities and `en` the rest of the union.
    fill_bits(used, nid, false);
    fill_bits(en, nid, false);
    bool from_solve = false;
#ifdef DP_STAMPS
    const int64_t tloop = stamp();
    int64_t tgap = tloop;
#endif
    for (;;) {
#ifdef DP_STAMPS
      DP_ACC(24, stamp() - tgap);
#endif
      if (dq_n == 0 && result == 0) {
        if (tr) {
          or_bits(en, used, nid);
          fill_bits(used, nid, false);
        }
#ifdef DP_STAMPS
        const int64_t ts = stamp();
        const int r = search_solve();
        DP_ACC(5, stamp() - ts);
#else
        const int r = search_solve();
#endif
        from_solve = true;
        if (r == RS_BUDGET) { result = RS_BUDGET; break; }
        result = r;
        last_solve = (r == RS_SAT);
        if (r == RS_UNSAT) solve_unsat = true;
      }
      if (result < 0) {
        if (tr) trace_event(from_solve);  // h.tracer.Trace(h), search.go:173
        if (ng == 0) break;
#ifdef DP_STAMPS
        const int64_t tq = stamp();
        pop_guess();
        DP_ACC(6, stamp() - tq);
#else
        pop_guess();
#endif
        from_solve = false;
        continue;
      }
      if (dq_n == 0) break;
#ifdef DP_STAMPS
      const int64_t tp = stamp();
      push_guess();
      tgap = stamp();
      DP_ACC(4, tgap - tp);
      DP_ACC(7, 1);
#else
      push_guess();
#endif
      from_solve = false;
      if (budget_hit) { result = RS_BUDGET; break; }
    }
#ifdef DP_STAMPS
    DP_ACC(23, stamp() - tloop);
#endif
    final_from_solve = from_solve;
    or_bits(used, en, nid);
    // Value() after an ending on Test()==1 reads that scope's full assignment
    if (result == 1 && !last_solve) save_model();
    return result;
  }

  // ------------------------------------------------------------------
  // NotSatisfiable (oracle: refute / core_extract)
  // ------------------------------------------------------------------
  __device__ __forceinline__ void reset_all() { truncate_to(0); }

  // The set bits of bits[0..nw) as ascending indices into out; returns their
  // number.  Every thread writes the bits of its words at their exclusive
  // prefix (DPP scan per wavefront, per-wave slots across wavefronts).
  __device__ __forceinline__ int emit_bits(const uint32_t* bits, int nw, int32_t* out) {
    int len = 0;
    for (int b = 0; b < nw; b += NT) {
      const int i = b + tid;
      const uint32_t x = i < nw ? ld_bits(&bits[i]) : 0u;
      const int c = __popc(x);
      const int incl = wave_incl_scan(c);
      int before = incl - c, total = __builtin_amdgcn_readlane(incl, 63);
      if constexpr (NW > 1) {
        const int32_t* sl = exchange(incl, lane == 63);
        total = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const int s = sl[q];
          before += q < wid ? s : 0;
          total += s;
        }
      }
      for (uint32_t y = x; y; y &= y - 1) out[len + before++] = 32 * i + __ffs(y) - 1;
      len += total;
    }
    return len;
  }

  // Bits over rows (rowspace) -> the same set over identities, in idt (a
  // lane per identity: its row's bit, ballot per 64); outside rowspace the
  // set itself.  For the outputs, which list identities ascending.
  __device__ __forceinline__ const uint32_t* to_idents(const uint32_t* src) {
    if (!rowspace) return src;
    for (int b = 0; b < nid; b += NT) {
      const int id = b + tid;
      const uint64_t m = __ballot(id < nid && getb(src, row_of(id)));
      const int wd = (b + 64 * wid) >> 5;
      if (lane == 0 && wd < nbi) {
        idt[wd] = (uint32_t)m;
        if (wd + 1 < nbi) idt[wd + 1] = (uint32_t)(m >> 32);
      }
    }
    gsync();
    return idt;
  }

  // Tracer.Trace(SearchPosition) at an unsatisfiable search step
  // (search.go:173; oracle: trace_event).  Record [n, guessed variables in
  // stack order, m, identities ascending]: the identities of the failure's
  // conflict analysis -- a failed Test/Untest is analysed here, a failed
  // Solve() left the union of its refutation's analyses in `used`.
  __device__ __forceinline__ void trace_event(bool from_solve) {
    if (tr_stop) return;
    if (!from_solve) {  // a trace-only analysis: kept out of the union
      or_bits(en, used, nid);
      fill_bits(used, nid, false);
      analyze();
    }
    int ngv = 0, ni = 0;
    for (int i = tid; i < ng; i += NT) ngv += guess_m(stk[3 * i], stk[3 * i + 1]) >= 0;
    for (int i = tid; i < nbi; i += NT) ni += __popc(ld_bits(&used[i]));
    ngv = g_sum(ngv);
    ni = g_sum(ni);
    if (tr_len + 2 + ngv + ni > tr_cap) {
      tr_stop = true;
      if (!from_solve) fill_bits(used, nid, false);
      return;
    }
    int32_t* o = tr + tr_len;
    if (tid == 0) {
      int k = 0;
      o[k++] = ngv;
      for (int i = 0; i < ng; ++i) {
        const int m = guess_m(stk[3 * i], stk[3 * i + 1]);
        if (m >= 0) o[k++] = m;
      }
      o[k] = ni;
    }
    emit_bits(to_idents(used), nbi, o + 2 + ngv);
    tr_len += 2 + ngv + ni;
    gsync();
    if (!from_solve) fill_bits(used, nid, false);
  }

  __device__ __forceinline__ void fill_bits(uint32_t* bs, int n, bool ones) {
    const int nw = bits_words(n);
    for (int i = tid; i < nw; i += NT) {
      uint32_t x = 0;
      if (ones) x = (i == nw - 1 && (n & 31)) ? ((1u << (n & 31)) - 1u) : 0xffffffffu;
      bs[i] = x;
    }
    gsync();
  }
  __device__ __forceinline__ void copy_bits(uint32_t* dst, const uint32_t* src, int n) {
    for (int i = tid; i < bits_words(n); i += NT) dst[i] = ld_bits(&src[i]);
    gsync();
  }
  __device__ __forceinline__ void or_bits(uint32_t* dst, const uint32_t* src, int n) {
    for (int i = tid; i < bits_words(n); i += NT) dst[i] |= ld_bits(&src[i]);
    gsync();
  }

  __device__ __forceinline__ int refute(const uint32_t* K) {
    reset_all();
    // the search's learned rows are not part of the base formula; the rows
    // this refutation's own Solve() learns are (oracle: refute)
    const int lo = learn_lo;
    learn_lo = nl;
    enabled = K;
    fill_bits(used, nid, false);
    int r;
    if (base_propagate() < 0) { analyze(); r = RS_UNSAT; }
    else r = dpll();
    reset_all();
    enabled = nullptr;
    learn_lo = lo;
    return r;
  }

  // ---- recursive model rotation (oracle: rotate) ----
  // A refutation of K \ {c} that finds a model proves c necessary; flipping
  // one variable of c's row in that model and leaving exactly one other key
  // c' of K violated proves c' necessary too, without a refutation, and the
  // walk continues from that model.  Keys owning exactly one row only; depth
  // first over the row's positions in order; frames below the top in the
  // round work list (wbuf, free outside rounds), at most ROT_DEPTH.  The
  // working model is `extra` (free when the solve is UNSAT), K is `en`.
  static constexpr int ROT_DEPTH = 32;
  static_assert(3 * ROT_DEPTH <= WBUF, "rotation frames fit the work list");
  // Is row r violated by the working model?
  __device__ __forceinline__ bool row_viol_m(int r) const {
    if (r < nc) {
      for (int j = clause_off[r]; j < (int)clause_off[r + 1]; ++j) {
        const int l = clause_lits[j];
        if ((int)getb(extra, l >> 1) != (l & 1)) return false;  // a true literal
      }
      return true;
    }
    const int k = r - nc;
    int cnt = 0;
    for (int j = card_off[k]; j < (int)card_off[k + 1]; ++j) cnt += (int)getb(extra, card_lits[j]);
    return cnt > (int)card_bound[k];
  }
  // the one row of key c, or -1 (none or several; packed records: the row)
  __device__ __forceinline__ int single_row_of(int c) {
    if (rowspace) return c;
    int n = 0, first = INF;
    for (int r0 = 0; r0 < nrows; r0 += NT) {
      const int r = r0 + tid;
      if (r < nrows && row_ident(r) == c) { ++n; first = min(first, r); }
    }
    n = g_sum(n);
    first = g_min(first);
    return n == 1 ? first : -1;
  }
  // the variable at position t of row r, or -1 past its end
  __device__ __forceinline__ int row_var(int r, int t) const {
    const int a = r < nc ? (int)clause_off[r] : (int)card_off[r - nc];
    const int b = r < nc ? (int)clause_off[r + 1] : (int)card_off[r - nc + 1];
    if (a + t >= b) return -1;
    return r < nc ? (int)clause_lits[a + t] >> 1 : (int)card_lits[a + t];
  }
  __device__ __forceinline__ bool row_has(int r, int v) const {
    for (int t = 0;; ++t) {
      const int x = row_var(r, t);
      if (x < 0) return false;
      if (x == v) return true;
    }
  }
  __device__ __forceinline__ void flip_m(int v) {
    gsync();
    if (tid == 0) extra[v >> 5] ^= 1u << (v & 31);
    gsync();
  }
  // The one key of K violated among the rows holding v, or -1 (none or
  // several): the rows in v's two watch lists (every clause holding v or ~v,
  // every AtMost row holding v).
  __device__ __forceinline__ int viol_key(int v) {
    int lo = INF, hi = -1;
    auto one = [&](int r) {
      if (r < 0 || r >= nrows) return;
      const int k = row_key(r);
      if (!getb(en, k) || !row_viol_m(r)) return;
      lo = min(lo, k);
      hi = max(hi, k);
    };
    const int a = w_off[2 * v], b = w_off[2 * v + 2];
    for (int j0 = a; j0 < b; j0 += NT) {
      const int j = j0 + tid;
      if (j < b) one(went(j).x);
    }
    lo = g_min(lo);
    hi = -g_min(-hi);
    return lo == hi ? lo : -1;
  }
  __device__ __forceinline__ void rotate(int c0) {
    int r = single_row_of(c0);
    if (r < 0) return;
    int c = c0, t = 0, d = 1;
    IX* st = wbuf;  // frames 0 .. d-2 as (key, row, next position); the top in registers
    for (;;) {
      const int v = row_var(r, t);
      if (v < 0) {  // the frame is done: back to its parent, undoing the flip that opened it
        if (--d == 0) break;
        gsync();
        c = st[3 * (d - 1)]; r = st[3 * (d - 1) + 1]; t = st[3 * (d - 1) + 2];
        flip_m(row_var(r, t - 1));
        continue;
      }
      ++t;
      flip_m(v);
      const int k = viol_key(v);
      bool opened = false;
      if (k >= 0 && k != c && !getb(crit, k)) {
        // (several wavefronts: every one has read crit before thread 0 sets the bit)
        if constexpr (NW > 1) bar();
        if (tid == 0) crit[k >> 5] |= 1u << (k & 31);
        const int rn = single_row_of(k);
        if (d < ROT_DEPTH && rn >= 0) {  // continue from this model (v stays flipped)
          if (tid == 0) { st[3 * (d - 1)] = enc(c); st[3 * (d - 1) + 1] = enc(r); st[3 * (d - 1) + 2] = enc(t); }
          c = k; r = rn; t = 0; ++d;
          opened = true;
        }
      }
      if (!opened) flip_m(v);
    }
    gsync();
  }

  // thread 0's x in every thread
  __device__ __forceinline__ int g_bcast0(int x) {
    if constexpr (NW == 1) {
      return __builtin_amdgcn_readlane(x, 0);
    } else {
      return exchange(x, tid == 0)[0];
    }
  }

  // The explanation goes to a pool shared by the launch: its length is
  // counted first, then one atomic claims the words (*at = its position).
  __device__ __forceinline__ int core(int32_t* pool, int32_t* pool_len, int32_t& flags, int& at) {
    const int64_t saved = steps;
    steps = 0;
    int len = 0;
    // start from the identities of the solve's own refutation (`used`: the
    // base conflict, or the search's union), an unsatisfiable set: no fresh
    // refutation of the whole catalog (oracle: core_extract)
    copy_bits(en, used, nid);
    fill_bits(crit, nid, false);
    int any = 0;
    for (int i = tid; i < nbi; i += NT) any |= en[i] != 0u;
    int r = g_any(any) ? RS_UNSAT : RS_BUDGET;
    if (r == RS_UNSAT) {
      // identities in ascending order (rowspace: through their rows, with
      // the set mirrored over identities in idt for the empty-word skip);
      // one proven necessary by a model (crit) stays without a refutation
      const uint32_t* ids = to_idents(en);
      for (int id = 0; id < nid; ++id) {
        if ((id & 31) == 0 && ids[id >> 5] == 0) { id += 31; continue; }  // empty word
        if (!getb(ids, id)) continue;
        const int key = rowspace ? row_of(id) : id;
        if (getb(crit, key)) continue;
        copy_bits(en2, en, nid);
        if (tid == 0) en2[key >> 5] &= ~(1u << (key & 31));
        gsync();
        r = refute(en2);
        if (r == RS_UNSAT) {
          copy_bits(en, used, nid);
          ids = to_idents(en);
        } else if (r == RS_BUDGET) {
          flags |= DP_F_CORE_BUDGET;
          break;
        } else {  // a model of K \ {key}: key is necessary, and the model's rotations find others
          if (tid == 0) crit[key >> 5] |= 1u << (key & 31);
          copy_bits(extra, model, nv);
          rotate(key);
        }
      }
      int c = 0;
      for (int i = tid; i < nbi; i += NT) c += __popc(ld_bits(&en[i]));
      c = g_sum(c);
      int a0 = 0;
      if (tid == 0 && c > 0) a0 = atomicAdd(pool_len, c);
      at = g_bcast0(a0);
      len = emit_bits(to_idents(en), nbi, pool + at);  // ascending identity ids
    } else {
      flags |= DP_F_CORE_BUDGET;
    }
    budget_hit = false;
    steps += saved;
    return len;
  }

  // ------------------------------------------------------------------
  // SAT epilogue, solve.go:86-110 (oracle: epilogue)
  // ------------------------------------------------------------------
  // The extras, the fixed variables and the installed set are the input's
  // variables 0..nvu-1 only (litMap.Variables, solve.go:88-96): an AtMost
  // network's gates (DP_H_NVU) stay free.
  __device__ __forceinline__ int epilogue(int32_t& flags, uint32_t* __restrict__ out, int nvu) {
    auto ubits = [&](int i) -> uint32_t {
      const int r = nvu - 32 * i;
      return r >= 32 ? ~0u : r <= 0 ? 0u : (1u << r) - 1u;
    };
    int ne = 0;
    for (int i = tid; i < nbv; i += NT) {
      const uint32_t x = model[i] & ~inS[i] & ubits(i);
      extra[i] = x;
      ne += __popc(x);
    }
    ne = g_sum(ne);
    if (ne == 0) {
      for (int i = tid; i < nbv; i += NT) out[i] = inS[i];
      return DP_SAT;
    }
    flags |= DP_F_EPILOGUE;
    reset_all();
    if (base_propagate() < 0) return DP_ERROR;
    const int start = tlen;
    bool bad = false;
    int run = tlen;
    for (int b = 0; b < nv; b += NT) {
      const int v = b + tid;
      bool f = false;
      int l = 0;
      if (v < nvu && !getb(extra, v)) {
        const int want = getb(inS, v) ? 1 : -1;
        if (val[v] == -want) bad = true;
        if (val[v] == 0) { f = true; l = 2 * v + (want < 0 ? 1 : 0); }
      }
      const int at = claim(f, run);
      if (f) {
        val[v] = (l & 1) ? -1 : 1; reason[v] = enc(R_DEC); rs[v] = enc(start);
        put_trail(at, l);
      }
    }
    claim_end(run);
    tlen = run;
    gsync();
    if (g_any(bad)) return DP_ERROR;
    if (propagate() < 0) return DP_ERROR;
    const int mark = tlen;
    int f = 0;
    for (int v = tid; v < nv; v += NT) f += getb(extra, v) && val[v] > 0;
    f = g_sum(f);
    extra_mode = true;
    for (int wv = f; wv <= ne; ++wv) {
      truncate_to(mark);
      extra_w = wv;
      if (propagate() < 0) continue;
      const int r = dpll();
      if (r == RS_SAT) {
        extra_mode = false;
        for (int i = tid; i < nbv; i += NT) out[i] = model[i] & ubits(i);
        return DP_SAT;
      }
      if (r == RS_BUDGET) { extra_mode = false; return DP_INCOMPLETE; }
    }
    extra_mode = false;
    return DP_ERROR;
  }
};

}  // namespace

// One problem per workgroup; blockIdx.x indexes `order` (problems bucketed by
// working-set footprint; the multi-wave modes work partly in HBM scratch).
// Outputs: status / flags / installed / core / steps (oracle_solve).
#ifndef DP_LDS_MIN_WAVES
#define DP_LDS_MIN_WAVES 5
#endif
// (MINW: minimum waves per SIMD the kernel is compiled for.  The one-wavefront
// kernel has two builds: unbounded (105 VGPRs: 4 waves per SIMD, 16 per CU)
// and DP_LDS_MIN_WAVES = 5 (94 VGPRs: 20 per CU), neither with a spill
// (tests/test_placement.py reads the code objects).  The capped build only
// pays where LDS would let more than 16 problems share a CU (small
// catalogs, config 3); launch_solve picks the build per launch by
// footprint.  Before round 6 the whole-wave reductions were __shfl_xor
// butterflies whose ds_bpermute addresses the compiler kept live across the
// search loop: 163 VGPRs unbounded, and 13 spilled at a 128 cap.  A cap of 6
// waves (80 VGPRs) spills 11.)
// One problem's results as two 16-byte vector stores (kernel_api.hpp).
__device__ __forceinline__ void put_out(ProblemOut* o, int status, int32_t flags, int32_t clen, int32_t cat,
                                        int64_t steps, uint64_t bcp) {
  uint4 x, y;
  x.x = (uint32_t)(uint8_t)(int8_t)status;
  x.y = (uint32_t)flags;
  x.z = (uint32_t)clen;
  x.w = (uint32_t)cat;
  y.x = (uint32_t)(uint64_t)steps;
  y.y = (uint32_t)((uint64_t)steps >> 32);
  y.z = (uint32_t)bcp;
  y.w = (uint32_t)(bcp >> 32);
  uint4* p = reinterpret_cast<uint4*>(o);
  p[0] = x;
  p[1] = y;
}

// The input's variable count (DP_H_NVU; 0: every variable is the input's).
__device__ __forceinline__ int nvu_of(const int32_t* grec, int nv) {
  const int u = grec[DP_H_NVU];
  return u > 0 && u < nv ? u : nv;
}

// Item k of the launch: one problem, start to finish.
template <int MODE, int MINW>
__device__ __forceinline__ void solve_item(const KernelArgs& a, int k, int4* lds4) {
#ifdef DP_STAMPS
  int64_t t[6];
  const int64_t wall0 = wallclock();
#endif
  DP_STAMP(0);
  const WorkItem it = a.items[k];
  const int pid = it.pid;
  const int32_t* grec = a.rec + it.rec_off;
  Group<MODE, MINW> W;
  char* hbm = mode_n16(MODE) ? nullptr : reinterpret_cast<char*>(a.scratch + a.scratch_off[k]);
  if (!W.init(reinterpret_cast<char*>(lds4), hbm, grec)) {
    if (threadIdx.x == 0) {  // a malformed record: no solve (dp_rec_validate's verdict)
      put_out(a.out + pid, DP_ERROR, DP_F_MALFORMED, 0, 0, 0, 0);
      if (a.trace) a.trace_len[pid] = 0;
    }
    uint32_t* inst0 = a.installed + it.inst_off;
    for (int i = threadIdx.x; i < bits_words(grec[DP_H_NV]); i += blockDim.x) inst0[i] = 0;
    return;
  }
#ifdef DP_STAMPS
  if (a.stamps) W.dbg = reinterpret_cast<unsigned long long*>(a.stamps + (int64_t)DP_NSTAMP * pid + 12);
#endif
  W.budget = a.budget;
  if constexpr (Group<MODE, MINW>::LR)
    if (a.table_cap > 0 && a.table_cap - 1 < W.hmask) W.hmask = a.table_cap - 1;  // (a power of two)
  if (a.trace) {
    W.tr = a.trace + (int64_t)a.trace_cap * pid;
    W.tr_cap = a.trace_cap;
  }
  uint32_t* inst = a.installed + it.inst_off;
  int32_t flags = 0;
  int status;
  for (int i = W.tid; i < W.nbv; i += Group<MODE, MINW>::NT) inst[i] = 0;
  DP_STAMP(1);
  const int base = W.base_propagate();
  DP_STAMP(2);
  DP_STAMP(3);
  if (base < 0) {
    flags |= DP_F_BASE_UNSAT;
    status = DP_UNSAT;
    W.fill_bits(W.used, W.nid, false);
    W.analyze();  // the base conflict's identities start the explanation
  } else if (base == 1) {
    flags |= DP_F_SEARCH_SKIPPED;
    W.save_model();
    status = W.epilogue(flags, inst, nvu_of(grec, W.nv));
  } else {
    const int r = W.search();
    DP_STAMP(3);
    if (W.class_b) flags |= DP_F_CLASS_B;
    if (W.solve_unsat) flags |= DP_F_SOLVE_UNSAT;
    if (r == RS_BUDGET) {
      flags |= DP_F_BUDGET;
      status = DP_INCOMPLETE;
    } else if (r < 0) {
      status = DP_UNSAT;
      if (!W.final_from_solve) W.analyze();  // the final root conflict (an Untest)
    } else {
      status = W.epilogue(flags, inst, nvu_of(grec, W.nv));
      if (status == DP_INCOMPLETE) flags |= DP_F_BUDGET;
    }
  }
  DP_STAMP(4);
  int clen = 0, cat = 0;
  if (status == DP_UNSAT) clen = W.core(a.core, a.core_pool_len, flags, cat);
  DP_STAMP(5);
#ifdef DP_STAMPS
  if (W.tid == 0 && a.stamps) {
    int64_t* o = a.stamps + (int64_t)DP_NSTAMP * pid;
    for (int i = 0; i < 5; ++i) o[i] = t[i + 1] - t[i];
    for (int i = 0; i < 5; ++i) o[5 + i] = (int64_t)W.lacc[i];
    o[10] = wall0;
    o[11] = wallclock();
    for (int i = 5; i < 16; ++i) o[11 + i] = (int64_t)W.lacc[i];
    for (int i = 0; i < 3; ++i) o[27 + i] = W.sub[i];
    for (int i = 3; i < 6; ++i) o[45 + i] = W.sub[i];
    for (int i = 16; i < 32; ++i) o[16 + i] = (int64_t)W.lacc[i];
  }
#endif
  if (W.tr_stop) flags |= DP_F_TRACE_TRUNCATED;
  const uint64_t bcp = W.vis_total();  // (a problem reads well under 2 GB)
  if (W.tid == 0) {
    if (a.trace) a.trace_len[pid] = W.tr_len;
    put_out(a.out + pid, status, flags, clen, cat, W.steps, bcp);
  }
}

template <int MODE, int MINW>
__global__ void __launch_bounds__(64 * mode_waves(MODE), MINW)
solve_kernel(KernelArgs a) {
  extern __shared__ int4 lds4[];
  if constexpr (MODE != M_LDS) {
    if (a.queue) {
      // persistent workgroup: items in queue order until the queue is
      // drained (every workgroup reaches the exit).  The item number is
      // handed over in LDS word 0, the scalars' first word, which init
      // rewrites only after the third barrier.
      int32_t* slot = reinterpret_cast<int32_t*>(lds4);
      for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) *slot = atomicAdd(a.queue, 1);
        __syncthreads();
        const int k = *slot;
        __syncthreads();
        if (k >= a.n_items) return;
        solve_item<MODE, MINW>(a, k, lds4);
      }
    }
  }
  solve_item<MODE, MINW>(a, (int)blockIdx.x, lds4);
}

// Workgroups of a queued launch's kernel one CU holds at once, by (device,
// LDS bytes): computed once per pair (the serving loop launches the same few
// shapes chunk after chunk), with the device's CU count.
struct GridCache {
  std::mutex mu;
  std::map<std::pair<int, int>, int> per_cu;
  int cus[64] = {};
};
template <int MODE, int MINW>
int resident_grid(int lds_bytes) {
  static GridCache c;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lk(c.mu);
  if (c.cus[dev] == 0 && hipDeviceGetAttribute(&c.cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    c.cus[dev] = 0;
  auto it = c.per_cu.find({dev, lds_bytes});
  if (it == c.per_cu.end()) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, solve_kernel<MODE, MINW>, 64 * mode_waves(MODE),
                                                     lds_bytes) != hipSuccess)
      per = 0;
    it = c.per_cu.emplace(std::make_pair(dev, lds_bytes), per).first;
  }
  return it->second * c.cus[dev];
}
inline bool debug_grid() {
  static const bool on = std::getenv("DEPPY_DEBUG_GRID") != nullptr;  // diagnostic
  return on;
}

// Instantiate and launch one mode (included once per translation unit).
// A queued (persistent) launch gets as many workgroups as the device holds
// at once, at most one per item (and at most a.grid_cap when set).
#define DP_DEFINE_MODE(MODE, MINW, NAME)                                                    \
  hipError_t NAME(const KernelArgs& a, int n_blocks, int lds_bytes, hipStream_t stream) {   \
    if (n_blocks <= 0) return hipSuccess;                                                   \
    int grid = n_blocks;                                                                    \
    if (a.queue) {                                                                          \
      const int res = resident_grid<MODE, MINW>(lds_bytes);                                 \
      if (res > 0 && res < grid) grid = res;                                                \
      if (a.grid_cap > 0 && a.grid_cap < grid) grid = a.grid_cap;                           \
      if (debug_grid())                                                                     \
        fprintf(stderr, "solve launch mode %d: %d items, resident %d -> grid %d\n", MODE, n_blocks, res, grid); \
    }                                                                                       \
    hipLaunchKernelGGL((solve_kernel<MODE, MINW>), dim3((unsigned)grid), dim3(64 * mode_waves(MODE)), \
                       (size_t)lds_bytes, stream, a);                                       \
    return hipGetLastError();                                                               \
  }                                                                                         \
  hipError_t NAME##_configure(int max_lds_bytes) {                                          \
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&solve_kernel<MODE, MINW>),          \
                               hipFuncAttributeMaxDynamicSharedMemorySize, max_lds_bytes);  \
  }

}  // namespace dp
