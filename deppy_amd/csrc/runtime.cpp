// Host runtime of libdeppy_hip: device discovery, batch partitioning across
// MI355X devices, HBM residency, launch and result download.
//
// Problems are independent: a batch is cut into contiguous,
// cost-balanced slices, one per device, with no inter-device traffic.  On each
// device, problems are bucketed by working-set footprint so every launch
// requests only the dynamic LDS its largest problem needs (occupancy follows
// the footprint); adjacent buckets are merged while that costs at most half
// the workgroups per CU, since one launch per batch leaves the hardware
// queues to other batches in flight (measured: 13.7M -> 21M res/s at three
// batches in flight).  Problems beyond the 160 KiB LDS of a CU are solved by
// multi-wave workgroups with part of the working set in HBM scratch.
//
// Streams belong to the context: kLanes per device, one per hardware queue
// (GPU_MAX_HW_QUEUES is 4), created first so each maps to its own queue.
// Every dp_launch takes the next free lanes round-robin, one per bucket
// launch, so back-to-back batches in flight (dp_launch ... dp_wait) run
// concurrently and one batch's tail of hard problems overlaps the next
// batch's bulk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "kernel_api.hpp"
#include "layout.hpp"

namespace {

constexpr int kMaxLdsBytes = 160 * 1024;          // LDS per CU on gfx950
constexpr int64_t kDefaultBudget = 1 << 16;        // BCP invocations per problem
// LDS bucket ceilings (bytes); one launch per non-empty bucket (after
// merging).  Diagnostic DEPPY_LDS_LEVELS=1: one bucket per occupancy level
// instead (bucket k = the problems of which exactly kMaxLevel - k fit one
// CU's LDS).  Measured worse: more launches per batch take more of the four
// hardware queues, and batches in flight stop overlapping (config 2 at merge
// 0.75: 27.0M -> 18.3M res/s; config 5 at 0.5: 583k -> 568k).
constexpr int kMaxLevel = 16;
constexpr int kLdsGran = 512;
// (160 KiB / 10, / 5, / 3, / 2, / 1.  Config 5, 30 steps: 588k res/s with
// the earlier 8/16/24/32/48/64/96/160 ceilings, 608k with these;
// scripts/ab_ceil.sh.  Configs 2 and 3 make one launch either way.)
constexpr int kCeilings[] = {16 << 10, 32 << 10, 53 << 10, 80 << 10, 160 << 10};
constexpr int kNBuckets = kMaxLevel;
constexpr int kLanes = 4;
constexpr double kMergeRatio = 0.5;  // bucket merging (build_slice); 0 = off
constexpr double kSplitPct = 0.0;    // outlier split (build_slice); 0 = off

#define HIP_OK(expr)                                                         \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) {                                                  \
      fail(std::string(#expr) + ": " + hipGetErrorString(e_));               \
      return -1;                                                             \
    }                                                                        \
  } while (0)

}  // namespace

struct DevSlice {
  int device = 0;
  int32_t p0 = 0, p1 = 0;  // global problem range
  int64_t inst0 = 0, core0 = 0;
  // device buffers
  int32_t* rec = nullptr;
  int64_t* rec_off = nullptr;
  int32_t* order = nullptr;
  int8_t* status = nullptr;
  int32_t* flags = nullptr;
  uint32_t* installed = nullptr;
  int64_t* inst_off = nullptr;
  int32_t* core = nullptr;
  int64_t* core_off = nullptr;
  int32_t* core_len = nullptr;
  int64_t* steps = nullptr;
  int64_t n_inst = 0, n_core = 0;
  // launches: [bucket] -> (first order index, count, lds bytes)
  std::vector<int> b_first, b_count, b_lds;
  std::vector<int> b_chain;  // 1: runs after the previous bucket launch, on its queue
  std::vector<int32_t> too_large;             // local indices (-> DP_ERROR)
  // multi-wave launches for problems over the LDS limit: [i] -> (first order
  // index, count, mode, lds bytes); their scratch offsets are indexed from
  // big_base (the first order index of the big problems)
  std::vector<int> g_first, g_count, g_mode, g_lds;
  int big_base = 0;
  int32_t* scratch = nullptr;
  int64_t* scratch_off = nullptr;
  int64_t* stamps = nullptr;  // diagnostic builds only
  int32_t* trace = nullptr;   // search trace: trace_cap words per problem
  int32_t* trace_len = nullptr;
  int32_t trace_cap = 0;
  hipStream_t stream = nullptr;  // lane of the last launch (context-owned)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // bucket launches run concurrently on the other lanes, joined back by events
  hipEvent_t done[kLanes - 1] = {};
};

struct dp_resident {
  int32_t n = 0;
  bool inflight = false;
  std::vector<DevSlice> slices;
};

struct Lanes {
  hipStream_t s[kLanes] = {};
  int next = 0;
};

struct dp_ctx {
  std::vector<int> devices;
  std::vector<Lanes> lanes;  // per device
  int64_t budget = kDefaultBudget;
  int32_t flags = 0;  // dp_opt_flag
  std::string err;
  double last_ms = 0.0;
  std::mutex mu;
};

namespace {

thread_local dp_ctx* t_ctx = nullptr;
void fail(const std::string& s) {
  if (t_ctx) t_ctx->err = s;
  else dp::set_global_error(s);
}

Lanes& lanes_of(dp_ctx* ctx, int device) {
  for (size_t i = 0; i < ctx->devices.size(); ++i)
    if (ctx->devices[i] == device) return ctx->lanes[i];
  return ctx->lanes[0];
}

void free_slice(DevSlice& s) {
  (void)hipSetDevice(s.device);
  void* ptrs[] = {s.rec, s.rec_off, s.order, s.status, s.flags, s.installed,
                  s.inst_off, s.core, s.core_off, s.core_len, s.steps, s.scratch, s.scratch_off,
                  s.stamps, s.trace, s.trace_len};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s.ev0) (void)hipEventDestroy(s.ev0);
  if (s.ev1) (void)hipEventDestroy(s.ev1);
  for (auto& e : s.done)
    if (e) (void)hipEventDestroy(e);
  s = DevSlice{};
}

template <class T>
int upload_vec(T** dst, const T* src, size_t n, hipStream_t st) {
  HIP_OK(hipMalloc(reinterpret_cast<void**>(dst), std::max<size_t>(n, 1) * sizeof(T)));
  if (n) HIP_OK(hipMemcpyAsync(*dst, src, n * sizeof(T), hipMemcpyHostToDevice, st));
  return 0;
}

// Problems whose one-wavefront LDS footprint exceeds kGroupAbove run as
// multi-wave workgroups (M_SPLIT4 / M_SPLIT) instead: at two or one per CU, a
// lone wavefront per problem leaves SIMDs idle.  Config 5, 30 steps, same box,
// with 8-wave groups: 608k res/s with every LDS-fitting problem on one wave,
// 701k at 80 KiB (96 KiB 675k, 128 KiB 539k, 64 KiB 613k, 48 KiB 474k).  With
// 4-wave groups below kMidMaxVars: 737k at 80 KiB, 798k at 64 KiB (60 KiB
// 686k, 53 KiB 682k, 68 KiB 777k, 72 KiB 734k, 96 KiB 666k).  The optimum
// sits on the 53/80 KiB bucket structure of this workload; it is a tuning
// point, not a derived constant.  profiles/r01_group_above_ab.jsonl.
// DEPPY_GROUP_ABOVE=<bytes> overrides it (diagnostic; 163840 = off).
constexpr int64_t kGroupAbove = 64 << 10;
// Routed-off catalogs under kMidMaxVars variables run in 4-wave groups
// (M_SPLIT4), larger ones in 8-wave groups: config 5 (up to ~2.4k variables)
// 701k -> 737k res/s with 4 waves for all multi-wave work, while config 4
// (~55k variables) fell 6.3k -> 5.3k (profiles/r01_group_waves_ab.jsonl).
constexpr int32_t kMidMaxVars = 8192;
int64_t group_above() {
  static const int64_t v = [] {
    const char* e = std::getenv("DEPPY_GROUP_ABOVE");
    const int64_t x = e ? std::atoll(e) : 0;
    return x > 0 ? std::min<int64_t>(x, kMaxLdsBytes) : kGroupAbove;
  }();
  return v;
}

// Does an image (its header) run on the one-wavefront LDS path?  The same
// test places it in a bucket (build_slice).
bool lds_path(const int32_t* h) {
  return dp::fits16(h) && (int64_t)dp::layout<dp::M_LDS>(h).lds_bytes <= group_above();
}

// Device image of one record (layout.hpp img_layout): the record, then its
// watch lists and base rows.  Returns the image length.
int64_t build_image(const int32_t* rec, std::vector<int32_t>& out, bool narrow) {
  const dp_rec_layout R = dp::rec_layout(rec);
  const int32_t nv = rec[DP_H_NV], nc = rec[DP_H_NC], nk = rec[DP_H_NK];
  const int32_t* clause_off = rec + R.clause_off;
  const int32_t* clause_lits = rec + R.clause_lits;
  const int32_t* card_off = rec + R.card_off;
  const int32_t* card_lits = rec + R.card_lits;
  const int32_t* card_bound = rec + R.card_bound;
  const size_t at = out.size();
  out.insert(out.end(), rec, rec + rec[DP_H_WORDS]);
  // watch lists, rows in ascending order; one entry per distinct AtMost variable
  std::vector<int32_t> cnt((size_t)2 * nv + 1, 0);
  for (int32_t r = 0; r < nc; ++r)
    for (int32_t j = clause_off[r]; j < clause_off[r + 1]; ++j) cnt[(size_t)(clause_lits[j] ^ 1) + 1]++;
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t j = card_off[k]; j < card_off[k + 1]; ++j)
      if (j == card_off[k] || card_lits[j] != card_lits[j - 1]) cnt[(size_t)2 * card_lits[j] + 1]++;
  for (int32_t l = 0; l < 2 * nv; ++l) cnt[(size_t)l + 1] += cnt[(size_t)l];
  const size_t woff = out.size();
  out.insert(out.end(), cnt.begin(), cnt.end());
  const size_t wat = out.size();
  out.resize(wat + (size_t)cnt[(size_t)2 * nv], 0);
  for (int32_t r = 0; r < nc; ++r)
    for (int32_t j = clause_off[r]; j < clause_off[r + 1]; ++j) out[wat + (size_t)cnt[(size_t)(clause_lits[j] ^ 1)]++] = r;
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t j = card_off[k]; j < card_off[k + 1]; ++j)
      if (j == card_off[k] || card_lits[j] != card_lits[j - 1])
        out[wat + (size_t)cnt[(size_t)2 * card_lits[j]]++] = nc + k;
  (void)woff;
  // rows that can fire on the empty assignment
  int32_t nbase = 0;
  for (int32_t r = 0; r < nc; ++r)
    if (clause_off[r + 1] - clause_off[r] <= 1) { out.push_back(r); ++nbase; }
  for (int32_t k = 0; k < nk; ++k) {
    bool fires = false;
    for (int32_t j = card_off[k]; j < card_off[k + 1] && !fires;) {
      int32_t e = j + 1;
      while (e < card_off[k + 1] && card_lits[e] == card_lits[j]) ++e;
      fires = (e - j) > card_bound[k];
      j = e;
    }
    if (fires) { out.push_back(nc + k); ++nbase; }
  }
  const int64_t words = (int64_t)(out.size() - at);
  out[at + dp::DP_H_FMT] = dp::DP_FMT_I32;
  out[at + dp::DP_H_NBASE] = nbase;
  out[at + dp::DP_H_IMG] = (int32_t)words;
  if (narrow && lds_path(out.data() + at)) {
    // 16-bit form: body word j (after the header) -> uint16 j, two per int32
    int32_t* x = out.data() + at;
    const int64_t nb = words - DP_H_SIZE;
    for (int64_t j = 0; j < nb; j += 2) {
      const uint32_t lo = (uint32_t)x[DP_H_SIZE + j] & 0xffffu;
      const uint32_t hi = j + 1 < nb ? (uint32_t)x[DP_H_SIZE + j + 1] & 0xffffu : 0u;
      x[DP_H_SIZE + j / 2] = (int32_t)(lo | (hi << 16));
    }
    x[dp::DP_H_FMT] = dp::DP_FMT_U16;
    out.resize(at + (size_t)DP_H_SIZE + (size_t)((nb + 1) / 2));
  }
  const int64_t stored = (int64_t)(out.size() - at);
  out.resize(at + (size_t)((stored + 3) & ~3LL), 0);  // 16-byte aligned images
  return words;
}

extern "C" int dp_device_bytes(const dp_batch* b, int32_t opt_flags, int64_t* rec_bytes, int64_t* img_bytes) {
  if (!b || (b->n_problems > 0 && (!b->rec || !b->rec_off))) return -1;
  const bool forced = opt_flags & (DP_OPT_FORCE_GROUP | DP_OPT_FORCE_HBM | DP_OPT_FORCE_MID);
  int64_t rb = 0, ib = 0;
  std::vector<int32_t> tmp;
  for (int32_t p = 0; p < b->n_problems; ++p) {
    const int32_t* rec = b->rec + b->rec_off[p];
    tmp.clear();
    build_image(rec, tmp, !forced);
    const int64_t w = rec[DP_H_WORDS];
    rb += tmp[dp::DP_H_FMT] == dp::DP_FMT_U16 ? 4 * DP_H_SIZE + 2 * (w - DP_H_SIZE) : 4 * w;
    ib += 4 * (int64_t)tmp.size();
  }
  if (rec_bytes) *rec_bytes = rb;
  if (img_bytes) *img_bytes = ib;
  return 0;
}

// Build one device's slice: device images, bucketed launch order, outputs.
int build_slice(DevSlice& s, Lanes& L, const dp_batch* b, const int64_t* inst_off,
                const int64_t* core_off, int32_t opt_flags, int32_t trace_cap) {
  HIP_OK(hipSetDevice(s.device));
  s.stream = L.s[0];
  HIP_OK(hipEventCreate(&s.ev0));
  HIP_OK(hipEventCreate(&s.ev1));
  for (auto& e : s.done) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const int32_t n = s.p1 - s.p0;
  // device images, built by up to 16 host threads into contiguous parts
  // (each part is uploaded in place, no concatenation)
  const unsigned hw = std::thread::hardware_concurrency();
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>({16, hw ? (int64_t)hw : 1, n / 256}));
  std::vector<std::vector<int32_t>> parts((size_t)T);
  const bool forced = opt_flags & (DP_OPT_FORCE_GROUP | DP_OPT_FORCE_HBM | DP_OPT_FORCE_MID);
  std::vector<int64_t> len((size_t)n);
  auto part_lo = [&](int t) { return (int32_t)((int64_t)n * t / T); };
  auto build_part = [&](int t) {
    std::vector<int32_t>& out = parts[(size_t)t];
    for (int32_t i = part_lo(t); i < part_lo(t + 1); ++i) {
      const size_t at = out.size();
      build_image(b->rec + b->rec_off[s.p0 + i], out, !forced);
      len[(size_t)i] = (int64_t)(out.size() - at);
    }
  };
  if (T == 1) build_part(0);
  else {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(build_part, t);
    for (auto& x : th) x.join();
  }
  std::vector<int64_t> roff((size_t)n + 1, 0);
  std::vector<const int32_t*> img((size_t)n);
  for (int t = 0; t < T; ++t) {
    size_t at = 0;
    for (int32_t i = part_lo(t); i < part_lo(t + 1); ++i) {
      img[(size_t)i] = parts[(size_t)t].data() + at;
      at += (size_t)len[(size_t)i];
      roff[(size_t)i + 1] = roff[(size_t)i] + len[(size_t)i];
    }
  }
  std::vector<std::vector<int32_t>> bucket(kNBuckets), big(4);
  std::vector<int> ceil(std::begin(kCeilings), std::end(kCeilings));
  if (const char* e = std::getenv("DEPPY_LDS_CEILINGS")) {  // diagnostic: KiB list, ascending, last 160
    ceil.clear();
    for (const char* q = e; *q;) {
      ceil.push_back((int)(std::atof(q) * 1024));
      while (*q && *q != ',') ++q;
      if (*q == ',') ++q;
    }
    if (ceil.empty() || ceil.back() < kMaxLdsBytes || (int)ceil.size() > kNBuckets)
      ceil.assign(std::begin(kCeilings), std::end(kCeilings));
  }
  bool levels = false;
  if (const char* e = std::getenv("DEPPY_LDS_LEVELS")) levels = std::atoi(e) != 0;  // diagnostic
  for (int32_t i = 0; i < n; ++i) {
    const int32_t* r = img[(size_t)i];
    const int64_t lds = lds_path(r) && !forced ? (int64_t)dp::layout<dp::M_LDS>(r).lds_bytes : INT64_MAX;
    int k = kNBuckets;
    if (lds <= kMaxLdsBytes) {
      if (levels) {
        const int64_t q = kMaxLdsBytes / ((lds + kLdsGran - 1) / kLdsGran * kLdsGran);
        k = kMaxLevel - (int)std::min<int64_t>(q, kMaxLevel);
      } else {
        k = 0;
        while (lds > ceil[(size_t)k]) ++k;
      }
    }
    if (k < kNBuckets) {
      bucket[(size_t)k].push_back(i);
      continue;
    }
    const dp::Layout ls = dp::layout<dp::M_SPLIT>(r), lh = dp::layout<dp::M_HBM>(r);
    // (layout arithmetic is int32: variables are capped well below its range)
    const bool sized = r[DP_H_NV] < (1 << 24) && r[DP_H_NID] < (1 << 26);
    if (sized && ls.lds_bytes <= kMaxLdsBytes && !(opt_flags & DP_OPT_FORCE_HBM))
      big[(opt_flags & DP_OPT_FORCE_MID) || (!forced && r[DP_H_NV] < kMidMaxVars) ? dp::M_SPLIT4 : dp::M_SPLIT]
          .push_back(i);
    else if (sized && lh.lds_bytes <= kMaxLdsBytes) big[dp::M_HBM].push_back(i);
    else s.too_large.push_back(i);
  }
  std::vector<int32_t> order;
  // Adjacent buckets are merged into one launch while the merged LDS request
  // keeps at least kMergeRatio of the first bucket's workgroups per CU: fewer
  // launches per batch leave more hardware queues to the batches in flight.
  double merge = kMergeRatio;
  if (const char* m = std::getenv("DEPPY_BUCKET_MERGE")) merge = std::atof(m);  // diagnostic
  auto lds_of = [&](int32_t i) { return dp::layout<dp::M_LDS>(img[(size_t)i]).lds_bytes; };
  int first_lds = 0;  // largest footprint of the first bucket of the open launch
  for (int k = 0; k < kNBuckets; ++k) {
    if (bucket[(size_t)k].empty()) continue;
    int mx = 0;
    for (int32_t i : bucket[(size_t)k]) mx = std::max(mx, lds_of(i));
    const bool join = !s.b_lds.empty() && merge > 0 &&
                      (double)(kMaxLdsBytes / std::max(mx, s.b_lds.back())) >=
                          merge * (double)(kMaxLdsBytes / first_lds);
    if (!join) first_lds = mx;
    if (join) {
      s.b_count.back() += (int)bucket[(size_t)k].size();
      s.b_lds.back() = std::max(s.b_lds.back(), mx);
    } else {
      s.b_first.push_back((int)order.size());
      s.b_count.push_back((int)bucket[(size_t)k].size());
      s.b_lds.push_back(mx);
    }
    order.insert(order.end(), bucket[(size_t)k].begin(), bucket[(size_t)k].end());
  }
  // A launch requests its largest problem's LDS.  When a few outliers cost a
  // workgroup per CU, they are split off into a launch of their own that
  // follows on the same queue (b_chain), so the bulk runs at the higher
  // occupancy (kSplitPct: the footprint percentile the bulk is sized to).
  s.b_chain.assign(s.b_first.size(), 0);
  double pct = kSplitPct;
  if (const char* e = std::getenv("DEPPY_LDS_PCT")) pct = std::atof(e);  // diagnostic
  if (pct > 0 && pct < 100) {
    std::vector<int> f2, c2, l2, ch2;
    for (size_t g = 0; g < s.b_first.size(); ++g) {
      auto first = order.begin() + s.b_first[g], last = first + s.b_count[g];
      std::stable_sort(first, last, [&](int32_t x, int32_t y) { return lds_of(x) < lds_of(y); });
      const int cut = (int)((double)s.b_count[g] * pct / 100.0);
      const int q = cut > 0 ? lds_of(*(first + cut - 1)) : s.b_lds[g];
      int k = cut;  // bulk = every problem with footprint <= q
      while (k < s.b_count[g] && lds_of(*(first + k)) <= q) ++k;
      if (k < s.b_count[g] && kMaxLdsBytes / q > kMaxLdsBytes / s.b_lds[g]) {
        f2.push_back(s.b_first[g]); c2.push_back(k); l2.push_back(q); ch2.push_back(0);
        f2.push_back(s.b_first[g] + k); c2.push_back(s.b_count[g] - k); l2.push_back(s.b_lds[g]); ch2.push_back(1);
      } else {
        f2.push_back(s.b_first[g]); c2.push_back(s.b_count[g]); l2.push_back(s.b_lds[g]); ch2.push_back(0);
      }
    }
    s.b_first = f2; s.b_count = c2; s.b_lds = l2; s.b_chain = ch2;
  }
  // Within a launch, workgroups are dispatched in blockIdx order: largest
  // image first (longest-processing-time-first, the image size standing in
  // for the unknown solve time), so the long solves do not start last and
  // form the launch's tail.  (Results are indexed by problem: the order
  // changes nothing but the schedule.)
  bool lpt = true;
  if (const char* e = std::getenv("DEPPY_LPT")) lpt = std::atoi(e) != 0;  // diagnostic
  if (lpt)
    for (size_t g = 0; g < s.b_first.size(); ++g) {
      auto first = order.begin() + s.b_first[g], last = first + s.b_count[g];
      std::stable_sort(first, last, [&](int32_t x, int32_t y) {
        return img[(size_t)x][dp::DP_H_IMG] > img[(size_t)y][dp::DP_H_IMG];
      });
    }
  // diagnostic: DEPPY_LDS_PAD_KB raises every launch's LDS request (occupancy study)
  if (const char* pad = std::getenv("DEPPY_LDS_PAD_KB"))
    for (int& b : s.b_lds) b = std::max(b, std::atoi(pad) * 1024);
  s.big_base = (int)order.size();
  std::vector<int64_t> soff(1, 0);
  for (int mode : {(int)dp::M_SPLIT4, (int)dp::M_SPLIT, (int)dp::M_HBM}) {
    if (big[(size_t)mode].empty()) continue;
    if (lpt)
      std::stable_sort(big[(size_t)mode].begin(), big[(size_t)mode].end(), [&](int32_t x, int32_t y) {
        return img[(size_t)x][dp::DP_H_IMG] > img[(size_t)y][dp::DP_H_IMG];
      });
    s.g_first.push_back((int)order.size());
    s.g_count.push_back((int)big[(size_t)mode].size());
    s.g_mode.push_back(mode);
    int mx = 0;
    for (int32_t i : big[(size_t)mode]) {
      const int32_t* r = img[(size_t)i];
      const dp::Layout L = mode == dp::M_SPLIT    ? dp::layout<dp::M_SPLIT>(r)
                           : mode == dp::M_SPLIT4 ? dp::layout<dp::M_SPLIT4>(r)
                                                  : dp::layout<dp::M_HBM>(r);
      mx = std::max(mx, L.lds_bytes);
      soff.push_back(soff.back() + ((int64_t)L.bytes + 15) / 16 * 4);  // int32 words, 16-byte aligned
    }
    s.g_lds.push_back(mx);
    order.insert(order.end(), big[(size_t)mode].begin(), big[(size_t)mode].end());
  }
  s.inst0 = inst_off[s.p0];
  s.core0 = core_off[s.p0];
  s.n_inst = inst_off[s.p1] - s.inst0;
  s.n_core = core_off[s.p1] - s.core0;
  std::vector<int64_t> li((size_t)n + 1), lc((size_t)n + 1);
  for (int32_t i = 0; i <= n; ++i) {
    li[(size_t)i] = inst_off[s.p0 + i] - s.inst0;
    lc[(size_t)i] = core_off[s.p0 + i] - s.core0;
  }
  HIP_OK(hipMalloc(&s.rec, std::max<size_t>((size_t)roff[(size_t)n], 1) * 4));
  for (int t = 0; t < T; ++t)
    if (!parts[(size_t)t].empty())
      HIP_OK(hipMemcpyAsync(s.rec + roff[(size_t)part_lo(t)], parts[(size_t)t].data(),
                            parts[(size_t)t].size() * 4, hipMemcpyHostToDevice, s.stream));
  if (upload_vec(&s.rec_off, roff.data(), (size_t)n, s.stream)) return -1;
  if (upload_vec(&s.order, order.data(), order.size(), s.stream)) return -1;
  if (upload_vec(&s.inst_off, li.data(), (size_t)n + 1, s.stream)) return -1;
  if (upload_vec(&s.core_off, lc.data(), (size_t)n + 1, s.stream)) return -1;
  if (soff.size() > 1) {
    if (upload_vec(&s.scratch_off, soff.data(), soff.size() - 1, s.stream)) return -1;
    HIP_OK(hipMalloc(&s.scratch, (size_t)soff.back() * 4));
  }
  HIP_OK(hipMalloc(&s.status, std::max<size_t>((size_t)n, 1)));
  HIP_OK(hipMalloc(&s.flags, std::max<size_t>((size_t)n, 1) * 4));
  HIP_OK(hipMalloc(&s.core_len, std::max<size_t>((size_t)n, 1) * 4));
  HIP_OK(hipMalloc(&s.steps, std::max<size_t>((size_t)n, 1) * 8));
#ifdef DP_STAMPS
  HIP_OK(hipMalloc(&s.stamps, std::max<size_t>((size_t)n, 1) * dp::DP_NSTAMP * 8));
  HIP_OK(hipMemsetAsync(s.stamps, 0, std::max<size_t>((size_t)n, 1) * dp::DP_NSTAMP * 8, s.stream));
#endif
  if (trace_cap > 0) {
    s.trace_cap = trace_cap;
    HIP_OK(hipMalloc(&s.trace, std::max<size_t>((size_t)n, 1) * (size_t)trace_cap * 4));
    HIP_OK(hipMalloc(&s.trace_len, std::max<size_t>((size_t)n, 1) * 4));
    HIP_OK(hipMemsetAsync(s.trace_len, 0, std::max<size_t>((size_t)n, 1) * 4, s.stream));
  }
  HIP_OK(hipMalloc(&s.installed, (size_t)std::max<int64_t>(s.n_inst, 1) * 4));
  HIP_OK(hipMalloc(&s.core, (size_t)std::max<int64_t>(s.n_core, 1) * 4));
  // problems that fit no bucket are reported DP_ERROR | DP_F_TOO_LARGE
  HIP_OK(hipMemsetAsync(s.status, 0, std::max<size_t>((size_t)n, 1), s.stream));
  HIP_OK(hipMemsetAsync(s.flags, 0, std::max<size_t>((size_t)n, 1) * 4, s.stream));
  HIP_OK(hipMemsetAsync(s.core_len, 0, std::max<size_t>((size_t)n, 1) * 4, s.stream));
  HIP_OK(hipMemsetAsync(s.steps, 0, std::max<size_t>((size_t)n, 1) * 8, s.stream));
  HIP_OK(hipMemsetAsync(s.installed, 0, (size_t)std::max<int64_t>(s.n_inst, 1) * 4, s.stream));
  HIP_OK(hipStreamSynchronize(s.stream));
  return 0;
}

// Enqueue the slice's launches (no wait).  A slice with m launches takes the
// next m lanes (launch i on lane (base + i) % kLanes) and advances the cursor
// past them, so the next batch in flight starts on lanes this one does not
// use and the two overlap.
int launch_slice(DevSlice& s, Lanes& L, int64_t budget) {
  HIP_OK(hipSetDevice(s.device));
  // queue groups: launches that run back to back on one queue.  The
  // multi-wave launches (long-running large catalogs) first, then the bucket
  // launches by size (a chained launch follows its predecessor), so the
  // largest start earliest.
  std::vector<std::vector<int>> groups;
  for (size_t g = 0; g < s.g_first.size(); ++g) groups.push_back({-1 - (int)g});
  std::vector<std::vector<int>> bg;
  for (size_t k = 0; k < s.b_first.size(); ++k) {
    if (k < s.b_chain.size() && s.b_chain[k] && !bg.empty()) bg.back().push_back((int)k);
    else bg.push_back({(int)k});
  }
  auto cnt = [&](const std::vector<int>& v) {
    int c = 0;
    for (int k : v) c += s.b_count[(size_t)k];
    return c;
  };
  std::stable_sort(bg.begin(), bg.end(), [&](const std::vector<int>& x, const std::vector<int>& y) {
    return cnt(x) > cnt(y);
  });
  groups.insert(groups.end(), bg.begin(), bg.end());
  const int nlaunch = (int)groups.size();
  // lanes this batch spreads its launches over (diagnostic DEPPY_LANE_SERIAL=1:
  // one lane, launches back to back)
  int width = std::max(1, std::min(nlaunch, kLanes));
  if (const char* e = std::getenv("DEPPY_LANE_SERIAL")) width = std::atoi(e) ? 1 : width;
  const int base = L.next;
  L.next = (L.next + width) % kLanes;
  s.stream = L.s[base];
  dp::KernelArgs a;
  a.rec = s.rec;
  a.rec_off = s.rec_off;
  a.status = s.status;
  a.flags = s.flags;
  a.installed = s.installed;
  a.inst_off = s.inst_off;
  a.core = s.core;
  a.core_off = s.core_off;
  a.core_len = s.core_len;
  a.steps = s.steps;
  a.budget = budget;
  a.scratch = nullptr;
  a.scratch_off = nullptr;
  a.stamps = s.stamps;
  a.trace = s.trace;
  a.trace_len = s.trace_len;
  a.trace_cap = s.trace_cap;
  const int nside = std::min<int>(width - 1, nlaunch - 1);
  auto side = [&](int i) { return L.s[(base + 1 + i) % kLanes]; };
  HIP_OK(hipEventRecord(s.ev0, s.stream));
  for (int i = 0; i < nside; ++i) HIP_OK(hipStreamWaitEvent(side(i), s.ev0, 0));
  for (size_t i = 0; i < groups.size(); ++i)
  for (const int k : groups[i]) {
    hipStream_t st = (i % width == 0) ? s.stream : side((int)(i % width) - 1);
    if (k < 0) {
      const size_t g = (size_t)(-1 - k);
      a.order = s.order + s.g_first[g];
      a.scratch = s.scratch;
      a.scratch_off = s.scratch_off + (s.g_first[g] - s.big_base);
      HIP_OK(dp::launch_solve(a, s.g_mode[g], s.g_count[g], s.g_lds[g], st));
      a.scratch = nullptr;
      a.scratch_off = nullptr;
    } else {
      a.order = s.order + s.b_first[(size_t)k];
      HIP_OK(dp::launch_solve(a, dp::M_LDS, s.b_count[(size_t)k], s.b_lds[(size_t)k], st));
    }
  }
  for (int i = 0; i < nside; ++i) {
    HIP_OK(hipEventRecord(s.done[i], side(i)));
    HIP_OK(hipStreamWaitEvent(s.stream, s.done[i], 0));
  }
  HIP_OK(hipEventRecord(s.ev1, s.stream));
  return 0;
}

int wait_slice(DevSlice& s) {
  HIP_OK(hipSetDevice(s.device));
  HIP_OK(hipEventSynchronize(s.ev1));
  return 0;
}

int download_slice(DevSlice& s, dp_result* res) {
  HIP_OK(hipSetDevice(s.device));
  const int32_t n = s.p1 - s.p0;
  if (n == 0) return 0;
  HIP_OK(hipMemcpyAsync(res->status + s.p0, s.status, (size_t)n, hipMemcpyDeviceToHost, s.stream));
  HIP_OK(hipMemcpyAsync(res->flags + s.p0, s.flags, (size_t)n * 4, hipMemcpyDeviceToHost, s.stream));
  HIP_OK(hipMemcpyAsync(res->core_len + s.p0, s.core_len, (size_t)n * 4, hipMemcpyDeviceToHost, s.stream));
  if (res->steps)
    HIP_OK(hipMemcpyAsync(res->steps + s.p0, s.steps, (size_t)n * 8, hipMemcpyDeviceToHost, s.stream));
  if (s.n_inst)
    HIP_OK(hipMemcpyAsync(res->installed + s.inst0, s.installed, (size_t)s.n_inst * 4,
                          hipMemcpyDeviceToHost, s.stream));
  if (s.n_core)
    HIP_OK(hipMemcpyAsync(res->core + s.core0, s.core, (size_t)s.n_core * 4, hipMemcpyDeviceToHost,
                          s.stream));
  HIP_OK(hipStreamSynchronize(s.stream));
  for (int32_t i : s.too_large) {
    res->status[s.p0 + i] = DP_ERROR;
    res->flags[s.p0 + i] = DP_F_TOO_LARGE;
    res->core_len[s.p0 + i] = 0;
  }
  return 0;
}

// Run fn(slice) on every slice, one host thread per device.
template <class F>
int for_slices(dp_ctx* ctx, dp_resident* r, F fn) {
  if (r->slices.size() == 1) return fn(r->slices[0]);
  std::vector<int> rc(r->slices.size(), 0);
  std::vector<std::thread> th;
  for (size_t i = 0; i < r->slices.size(); ++i)
    th.emplace_back([&, i]() {
      t_ctx = ctx;
      rc[i] = fn(r->slices[i]);
    });
  for (auto& t : th) t.join();
  for (int x : rc)
    if (x) return x;
  return 0;
}

}  // namespace

extern "C" {

dp_ctx* dp_create(const dp_opts* opts) {
  t_ctx = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    dp::set_global_error(std::string("dp_create: no HIP device (") + hipGetErrorString(e) + ")");
    return nullptr;
  }
  int first = opts ? opts->first_device : 0;
  int cnt = opts && opts->n_devices > 0 ? opts->n_devices : n - first;
  if (first < 0 || cnt <= 0 || first + cnt > n) {
    dp::set_global_error("dp_create: device range out of bounds");
    return nullptr;
  }
  auto* ctx = new dp_ctx;
  for (int d = first; d < first + cnt; ++d) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      dp::set_global_error(std::string("dp_create: device ") + std::to_string(d) +
                           " is not gfx950 (" + prop.gcnArchName + ")");
      delete ctx;
      return nullptr;
    }
    if (hipSetDevice(d) != hipSuccess || dp::configure_solve_kernel(kMaxLdsBytes) != hipSuccess) {
      dp::set_global_error("dp_create: cannot configure the solve kernel");
      delete ctx;
      return nullptr;
    }
    Lanes L;
    for (auto& st : L.s) {
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        dp::set_global_error("dp_create: cannot create streams");
        dp_destroy(ctx);
        return nullptr;
      }
    }
    ctx->devices.push_back(d);
    ctx->lanes.push_back(L);
  }
  if (opts && opts->step_budget > 0) ctx->budget = opts->step_budget;
  if (opts) ctx->flags = opts->flags;
  return ctx;
}

void dp_destroy(dp_ctx* ctx) {
  if (!ctx) return;
  for (size_t i = 0; i < ctx->lanes.size(); ++i) {
    (void)hipSetDevice(ctx->devices.size() > i ? ctx->devices[i] : 0);
    for (auto& st : ctx->lanes[i].s)
      if (st) (void)hipStreamDestroy(st);
  }
  delete ctx;
}
const char* dp_last_error(const dp_ctx* ctx) { return ctx ? ctx->err.c_str() : dp_last_global_error(); }
int32_t dp_num_devices(const dp_ctx* ctx) { return ctx ? (int32_t)ctx->devices.size() : 0; }

int dp_result_layout(const dp_batch* b, int64_t* inst_off, int64_t* core_off) {
  if (!b || !inst_off || !core_off || b->n_problems < 0) return -1;
  inst_off[0] = core_off[0] = 0;
  for (int32_t i = 0; i < b->n_problems; ++i) {
    const int32_t* r = b->rec + b->rec_off[i];
    inst_off[i + 1] = inst_off[i] + dp::bits_words(r[DP_H_NV]);
    core_off[i + 1] = core_off[i] + r[DP_H_NID];
  }
  return 0;
}

int dp_upload(dp_ctx* ctx, const dp_batch* b, dp_resident** out) {
  return dp_upload_traced(ctx, b, 0, out);
}

int dp_upload_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_resident** out) {
  if (!ctx || !b || !out || trace_cap < 0) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  const int32_t P = b->n_problems;
  for (int32_t i = 0; i < P; ++i) {
    int64_t words = b->rec_off[i + 1] - b->rec_off[i];
    int rc = dp_rec_validate(b->rec + b->rec_off[i], words);
    if (rc) {
      fail("dp_upload: record " + std::to_string(i) + " malformed (" + std::to_string(rc) + ")");
      return -1;
    }
  }
  std::vector<int64_t> inst_off((size_t)P + 1), core_off((size_t)P + 1);
  dp_result_layout(b, inst_off.data(), core_off.data());
  auto* r = new dp_resident;
  r->n = P;
  // contiguous slices balanced by record words (a proxy of solve cost)
  const int nd = (int)ctx->devices.size();
  const int64_t total = P ? b->rec_off[P] - b->rec_off[0] : 0;
  int32_t p = 0;
  for (int d = 0; d < nd; ++d) {
    DevSlice s;
    s.device = ctx->devices[(size_t)d];
    s.p0 = p;
    const int64_t target = b->rec_off[0] + total * (d + 1) / nd;
    while (p < P && (d == nd - 1 || b->rec_off[p + 1] <= target)) ++p;
    s.p1 = p;
    r->slices.push_back(s);
  }
  int rc = for_slices(ctx, r, [&](DevSlice& s) {
    return build_slice(s, lanes_of(ctx, s.device), b, inst_off.data(), core_off.data(), ctx->flags,
                       trace_cap);
  });
  if (rc) {
    dp_resident_free(ctx, r);
    return -1;
  }
  *out = r;
  return 0;
}

namespace {
int wait_locked(dp_ctx* ctx, dp_resident* r) {
  if (!r->inflight) return 0;
  int rc = for_slices(ctx, r, [&](DevSlice& s) { return wait_slice(s); });
  r->inflight = false;
  if (rc) return -1;
  double mx = 0.0;
  for (auto& s : r->slices) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s.ev0, s.ev1) == hipSuccess) mx = std::max(mx, (double)ms);
  }
  ctx->last_ms = mx;
  return 0;
}

int launch_locked(dp_ctx* ctx, dp_resident* r) {
  if (r->inflight && wait_locked(ctx, r)) return -1;
  const int64_t budget = ctx->budget;
  int rc = 0;
  // launches are asynchronous: one host thread issues every device's slice
  for (auto& s : r->slices) rc = rc ? rc : launch_slice(s, lanes_of(ctx, s.device), budget);
  if (rc) return -1;
  r->inflight = true;
  return 0;
}
}  // namespace

int dp_launch(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  return launch_locked(ctx, r);
}

int dp_wait(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  return wait_locked(ctx, r);
}

int dp_run(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  if (launch_locked(ctx, r)) return -1;
  return wait_locked(ctx, r);
}

int dp_download(dp_ctx* ctx, dp_resident* r, dp_result* res) {
  if (!ctx || !r || !res) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  if (wait_locked(ctx, r)) return -1;
  return for_slices(ctx, r, [&](DevSlice& s) { return download_slice(s, res); });
}

int dp_download_trace(dp_ctx* ctx, dp_resident* r, int32_t* trace, int32_t* trace_len) {
  if (!ctx || !r || !trace || !trace_len) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  t_ctx = ctx;
  if (wait_locked(ctx, r)) return -1;
  return for_slices(ctx, r, [&](DevSlice& s) {
    HIP_OK(hipSetDevice(s.device));
    const int32_t n = s.p1 - s.p0;
    if (!s.trace) {
      fail("dp_download_trace: the batch was not uploaded with dp_upload_traced");
      return -1;
    }
    if (n == 0) return 0;
    HIP_OK(hipMemcpyAsync(trace_len + s.p0, s.trace_len, (size_t)n * 4, hipMemcpyDeviceToHost, s.stream));
    HIP_OK(hipMemcpyAsync(trace + (int64_t)s.trace_cap * s.p0, s.trace, (size_t)n * s.trace_cap * 4,
                          hipMemcpyDeviceToHost, s.stream));
    HIP_OK(hipStreamSynchronize(s.stream));
    return 0;
  });
}

int dp_solve_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_result* res,
                    int32_t* trace, int32_t* trace_len) {
  dp_resident* r = nullptr;
  if (dp_upload_traced(ctx, b, trace_cap, &r)) return -1;
  int rc = dp_run(ctx, r);
  if (!rc) rc = dp_download(ctx, r, res);
  if (!rc) rc = dp_download_trace(ctx, r, trace, trace_len);
  dp_resident_free(ctx, r);
  return rc;
}

void dp_resident_free(dp_ctx* ctx, dp_resident* r) {
  if (!r) return;
  if (ctx && r->inflight) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    t_ctx = ctx;
    (void)wait_locked(ctx, r);
  }
  for (auto& s : r->slices) free_slice(s);
  delete r;
}

int dp_solve(dp_ctx* ctx, const dp_batch* b, dp_result* res) {
  dp_resident* r = nullptr;
  if (dp_upload(ctx, b, &r)) return -1;
  int rc = dp_run(ctx, r);
  if (!rc) rc = dp_download(ctx, r, res);
  dp_resident_free(ctx, r);
  return rc;
}

#ifdef DP_STAMPS
// Diagnostic builds only: per-problem phase cycles [init, base, search,
// epilogue, core] of the last run (not part of include/deppy_hip.h).
int dp_debug_stamps(dp_ctx* ctx, dp_resident* r, int64_t* out) {
  t_ctx = ctx;
  for (auto& s : r->slices) {
    HIP_OK(hipSetDevice(s.device));
    HIP_OK(hipMemcpy(out + dp::DP_NSTAMP * (size_t)s.p0, s.stamps, (size_t)(s.p1 - s.p0) * dp::DP_NSTAMP * 8,
                     hipMemcpyDeviceToHost));
  }
  return 0;
}
#endif

int dp_last_kernel_ms(const dp_ctx* ctx, double* ms) {
  if (!ctx || !ms) return -1;
  *ms = ctx->last_ms;
  return 0;
}

}  // extern "C"
