// Watch lists of OLM-scale multi-wave problems, built on the device.
//
// A multi-wave record above DEV_WATCH_VARS variables crosses PCIe as a plain
// int32 record (DP_FMT_I32): its 2nv+1 list counters do not fit the LDS work
// area that build_watches_wide counts in, and a lone 8-wave workgroup filling
// ~330k list entries through HBM atomics spends millions of cycles on it.  So
// before a multi-wave launch holding such records, four grid-wide passes
// build the lists into each problem's scratch (layout.hpp Layout::wl):
//   zero   the 2nv+2 counters,
//   count  the rows each literal wakes (the clauses holding ~l, and for a
//          positive l the AtMost rows holding var(l), once per distinct
//          variable; the same rows as build_watches_host),
//   scan   the counts into list offsets (one workgroup per record),
//   fill   the lists through the offsets as cursors: 8-byte entries {row,
//          row_info(row)} (layout.hpp row_info).
// Counts go to wo[l + 2] and cursors run on wo[l + 1], so when the fill ends
// wo[l] is the start of list l (wo[2nv] their total) with no pass to shift
// the offsets back.  Row order within a list is left to the atomics, as in
// the in-kernel builds: every outcome of a round is a minimum over rows.
//
// The passes run before the solve kernel validates the record (valid_wide),
// so they touch memory only through checked indices: a row whose offsets are
// out of order or range is skipped, a literal or variable out of range is
// skipped, and a fill position past the lists' capacity is dropped.  A
// malformed record then gets lists that are wrong but in bounds, and the
// solve kernel reports it as DP_F_MALFORMED without reading them.
#include "kernel_api.hpp"
#include "layout.hpp"

namespace dp {
namespace {

constexpr int kWbThreads = 256;     // count / zero / fill workgroups
constexpr int kWbSlices = 32;       // workgroups per record in those passes
constexpr int kScanThreads = 1024;  // one scan workgroup per record

struct WbRec {
  const int32_t* h;
  int32_t* wo;  // [2nv + 2] counters / offsets, then the lists: [ncl + nkl] u16 rows or int2 {row, row_info}
  dp_rec_layout R;
};

// Item k of the launch, when its lists are built by these passes.
template <int MODE>
__device__ __forceinline__ bool wb_rec(const KernelArgs& a, int k, WbRec& x) {
  const int32_t* h = a.rec + a.items[k].rec_off;
  if (h[DP_H_FMT] != DP_FMT_I32 || device_watches(h)) return false;
  x.h = h;
  x.R = rec_layout(h);
  x.wo = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(a.scratch + a.scratch_off[k]) + layout<MODE>(h).wl);
  return true;
}

template <int MODE>
__global__ __launch_bounds__(kWbThreads) void wb_zero(KernelArgs a) {
  const int k = blockIdx.x / kWbSlices, s = blockIdx.x % kWbSlices;
  WbRec x;
  if (!wb_rec<MODE>(a, k, x)) return;
  const int n = 2 * x.h[DP_H_NV] + 2;
  for (int i = s * kWbThreads + (int)threadIdx.x; i < n; i += kWbSlices * kWbThreads) x.wo[i] = 0;
}

// The count (FILL false) and fill passes: rows one per thread across the
// record's slices, every position of a well-formed row (clauses, then AtMost
// rows at the first position of each variable run).
template <int MODE, bool FILL>
__global__ __launch_bounds__(kWbThreads) void wb_rows(KernelArgs a) {
  const int k = blockIdx.x / kWbSlices, s = blockIdx.x % kWbSlices;
  WbRec x;
  if (!wb_rec<MODE>(a, k, x)) return;
  const int32_t* h = x.h;
  const int nv = h[DP_H_NV], nc = h[DP_H_NC], nk = h[DP_H_NK], ncl = h[DP_H_NCL], nkl = h[DP_H_NKL];
  const int32_t* co = h + x.R.clause_off;
  const int32_t* cl = h + x.R.clause_lits;
  const int32_t* ko = h + x.R.card_off;
  const int32_t* kl = h + x.R.card_lits;
  int32_t* wo = x.wo;
  int2* ww = reinterpret_cast<int2*>(wo + 2 * nv + 2);
  const unsigned cap = (unsigned)(ncl + nkl), nl = (unsigned)(2 * nv);
  auto put = [&](unsigned at, int2 e) {
    if (at < cap) ww[at] = e;
  };
  const int t = s * kWbThreads + (int)threadIdx.x, T = kWbSlices * kWbThreads;
  for (int r = t; r < nc; r += T) {
    const int b0 = co[r], b1 = co[r + 1];
    if (b0 < 0 || b0 > b1 || b1 > ncl) continue;
    const int2 e = make_int2(r, (int)row_info(b0, b1 - b0));
    for (int j = b0; j < b1; ++j) {
      const int l = cl[j] ^ 1;  // the literal whose assignment falsifies position j
      if ((unsigned)l >= nl) continue;
      if constexpr (FILL) {
        put((unsigned)atomicAdd(&wo[l + 1], 1), e);
      } else {
        atomicAdd(&wo[l + 2], 1);
      }
    }
  }
  for (int q = t; q < nk; q += T) {
    const int b0 = ko[q], b1 = ko[q + 1];
    if (b0 < 0 || b0 > b1 || b1 > nkl) continue;
    const int2 e = make_int2(nc + q, (int)row_info(b0, b1 - b0));
    for (int j = b0; j < b1; ++j) {
      const int v = kl[j];
      if ((j > b0 && v == kl[j - 1]) || (unsigned)v >= (unsigned)nv) continue;
      if constexpr (FILL) {
        put((unsigned)atomicAdd(&wo[2 * v + 1], 1), e);
      } else {
        atomicAdd(&wo[2 * v + 2], 1);
      }
    }
  }
}

// wo[0..2nv+2) inclusive prefix sums in place, 1024 entries per step: a
// wavefront scan by lane shuffles, then the wavefront totals.
template <int MODE>
__global__ __launch_bounds__(kScanThreads) void wb_scan(KernelArgs a) {
  WbRec x;
  if (!wb_rec<MODE>(a, blockIdx.x, x)) return;
  __shared__ int wsum[kScanThreads / 64];
  const int n = 2 * x.h[DP_H_NV] + 2;
  const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
  int carry = 0;
  for (int b = 0; b < n; b += kScanThreads) {
    const int i = b + (int)threadIdx.x;
    int v = i < n ? x.wo[i] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(v, d, 64);
      if (lane >= d) v += y;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
      const int y = wsum[w];
      before += w < wv ? y : 0;
      total += y;
    }
    if (i < n) x.wo[i] = carry + before + v;
    carry += total;
    __syncthreads();  // (wsum is rewritten by the next step)
  }
}

template <int MODE>
hipError_t run(const KernelArgs& a, int n_items, hipStream_t s) {
  const dim3 rows((unsigned)n_items * kWbSlices), one((unsigned)n_items);
  hipLaunchKernelGGL((wb_zero<MODE>), rows, dim3(kWbThreads), 0, s, a);
  hipLaunchKernelGGL((wb_rows<MODE, false>), rows, dim3(kWbThreads), 0, s, a);
  hipLaunchKernelGGL((wb_scan<MODE>), one, dim3(kScanThreads), 0, s, a);
  hipLaunchKernelGGL((wb_rows<MODE, true>), rows, dim3(kWbThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_watch_build(const KernelArgs& a, int mode, int n_items, hipStream_t stream) {
  if (n_items <= 0) return hipSuccess;
  if (mode == M_SPLIT) return run<M_SPLIT>(a, n_items, stream);
  if (mode == M_SPLIT4) return run<M_SPLIT4>(a, n_items, stream);
  if (mode == M_HBM) return run<M_HBM>(a, n_items, stream);
  return hipSuccess;  // one-wavefront problems build theirs in LDS
}

}  // namespace dp
