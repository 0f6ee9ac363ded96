// Host runtime of libdeppy_hip: device discovery, the host-to-host solve
// pipeline, the device-resident form, launch placement and result stitching.
//
// The reference's Solve is a host-memory-to-host-memory call
// (pkg/sat/solve.go:53-119).  dp_submit / dp_job_wait / dp_solve are the
// batched form of it: lowered records in host memory -> results in host
// memory.  A batch is cut into chunks of contiguous problems; every chunk
// goes through one lane (a HIP stream on its own hardware queue, with its own
// persistent pinned and device buffers):
//
//   host pool: stage the chunk's records into the lane's pinned buffer
//              (16-bit form for the LDS path), plan its launches
//   lane:      one H2D copy -> solve kernel launch(es) -> one D2H copy
//   host:      scatter the lane's results into the caller's dp_result
//
// Lanes are taken round-robin over devices and hardware queues, so while
// the host stages chunk i+1, chunks i, i-1, ... copy and solve on the GPU,
// and H2D, kernels and D2H of different chunks overlap.  Nothing is
// allocated per call once the buffers have grown to the chunk size: no
// hipMalloc, hipHostMalloc or event creation on the steady-state path.
// Watch lists are built by the kernel (layout.hpp), so only records cross
// PCIe.
//
// Problems are independent: chunks on different devices
// need no inter-device traffic, and results are stitched by problem index.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "dlower.hpp"
#include "kernel_api.hpp"
#include "layout.hpp"
#include "hostmem.hpp"
#include "placement.hpp"
#include "pool.hpp"

namespace {

using dp::kMaxLdsBytes;  // (placement.hpp)
constexpr int64_t kDefaultBudget = 1 << 16;        // BCP invocations per problem
// LDS bucket ceilings (bytes); one launch per non-empty bucket after merging.
// (160 KiB / 10, / 5, / 3, / 2, / 1.  Config 5, 30 steps: 588k res/s with
// 8/16/24/32/48/64/96/160 ceilings, 608k with these; configs 2 and 3 make
// one launch either way.)
// Coarse ceilings (the default): 160 KiB / 10, / 5, / 3, / 2, / 1.
// DEPPY_CEILINGS=fine: one bucket per residency, the largest footprint of
// which k problems share a CU (160 KiB / k, in 512-byte LDS allocation
// units), k = 16 .. 1.  The one-wavefront kernel is latency-bound per wave:
// its throughput follows residency almost linearly (config 2, kernel only:
// 2 per CU 6.2M res/s, 4: 11.5M, 6: 16.7M, 8: 20.4M, 9: 22.3M;
// profiles/r03_config2_residency_sweep.jsonl).  But a chunk's launches run
// one after another on its stream, each as long as its slowest problem:
// fine buckets split config 2 into 2-3 launches and it fell from 22.1M to
// 14.3M res/s (profiles/r03_buckets_ab.jsonl).  Residency has to come from
// smaller footprints, not from more launches.
constexpr int kNBuckets = 16;
struct Ceilings {
  int c[kNBuckets];
  int n;
};
const Ceilings& ceilings() {
  static const Ceilings t = [] {
    Ceilings x{};
    const char* e = std::getenv("DEPPY_CEILINGS");
    if (!e || std::strcmp(e, "fine") != 0) {
      const int coarse[] = {16 << 10, 32 << 10, 53 << 10, 80 << 10, 160 << 10};
      x.n = 5;
      for (int i = 0; i < 5; ++i) x.c[i] = coarse[i];
    } else {
      x.n = kNBuckets;
      for (int k = kNBuckets; k >= 1; --k) x.c[kNBuckets - k] = (160 * 1024 / k) / 512 * 512;
      x.c[kNBuckets - 1] = 160 * 1024;
    }
    return x;
  }();
  return t;
}
constexpr int kXcds = 8;             // MI355X: the dispatcher deals workgroups round-robin to 8 XCDs
constexpr int kStreams = 4;          // streams per device, one per hardware queue (DEPPY_STREAMS)
constexpr int kMaxStreams = 16;
constexpr int kMaxLanes = 2 * kMaxStreams;  // chunk slots per device, two per stream: a stream always
                                            // has the next chunk queued behind the running one (no host gap)
constexpr double kMergeRatio = 0.5;  // bucket merging (plan_chunk)
constexpr int32_t kMinLaunch = 512;   // a smaller bucket rides along in a larger one's launch
// Routed-off catalogs under kMidMaxVars variables run in 4-wave groups
// (M_SPLIT4), larger ones in 8-wave groups (profiles/r01_group_waves_ab.jsonl).
constexpr int32_t kMidMaxVars = 8192;
// Pipeline chunks: at most this many problems or record bytes each.  A
// chunk's kernels last as long as its slowest problem, and at most one chunk
// per lane is in flight, so chunks are large (config 3 host to host: 11.0M
// res/s with 4096-problem / 24 MiB chunks, 45.1M with 65536 / 64 MiB;
// config 2: 10.0M -> 12.4M, one chunk per 10,000-catalog batch,
// profiles/r02_h2h_sweep_b.jsonl; config 5: 363k at 64 MiB, 456k at 256 MiB;
// config 4: 1.6k -> 3.0k, profiles/r02_h2h_sweep_c.jsonl; a directly copied
// batch needs no pinned staging room, so the cap is the device image).
constexpr int32_t kChunkProblems = 65536;
constexpr int64_t kChunkBytes = 1ll << 30;
// several devices (cut_chunks): chunks per device for the shared queue to
// balance, and the smallest such chunk (config 2: 5000-problem chunks ran 3%
// under whole 10k ones, 2500-problem ones 32%; profiles/r05_chunk_ab.txt)
constexpr int32_t kChunksPerDevice = 3;
constexpr int kCostClasses = 16;  // plan_chunk: dispatch classes of one-wavefront problems (anchors, capped)
constexpr int32_t kMinSharedChunk = 4096;
// D2H of the explanation pool per chunk: this many words per problem are
// copied with the fixed outputs; a chunk whose cores need more fetches the
// rest with a second copy.
constexpr int64_t kCoreWordsPerProblem = 8;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int64_t env_i64(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoll(e) : dflt;
}

bool forced_of(int32_t opt_flags) {
  return opt_flags & (DP_OPT_FORCE_GROUP | DP_OPT_FORCE_HBM | DP_OPT_FORCE_MID | DP_OPT_FORCE_LDSG);
}

// Header sanity needed before any layout arithmetic on it: the counts bound
// every array, so the kernel can stage and validate the body (valid_record)
// without reading past the record.
bool header_ok(const int32_t* h, int64_t avail) {
  if (avail < DP_H_SIZE || h[DP_H_MAGIC] != DP_REC_MAGIC) return false;
  for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
    if (h[i] < 0 || h[i] > (1 << 28)) return false;
  const int32_t fmt = h[DP_H_FMT];
  if (fmt != DP_FMT_I32 && fmt != DP_FMT_I32W && ((fmt != DP_FMT_U16 && !dp_fmt_packed(fmt)) || !dp_rec_fits16(h)))
    return false;
  if (dp_fmt_packed(fmt) && dp_p16_tail_bytes(h) > DP_P16_TAIL_MAX) return false;
  const int64_t w = dp_rec_layout_of(h).words;
  return w == h[DP_H_WORDS] && dp_rec_phys_words(h) <= avail;
}

}  // namespace

namespace dp {

// ---------------------------------------------------------------------------
// Launch plan of one chunk (pure host logic; no HIP)
// ---------------------------------------------------------------------------
struct Launch {
  int first, count, mode, lds;
  bool dev_lists;  // holds DP_FMT_I32 records above DEV_WATCH_VARS variables, whose watch lists the
                   // grid-wide passes build (watch_build.hip); copied as they lie or by stage_one alike
};

// What the plan needs of one record, from its header alone (one cache line
// per record: the header pass runs on the host pool, since the headers of a
// chunk sit a record apart and every one is a cache miss).
struct Head {
  int8_t place;   // -1 malformed, -2 too large, else the Mode
  bool ldsg_ok;   // a mid-size 16-bit-able record the chunk may place on M_LDSG (plan_chunk)
  int8_t bucket;  // M_LDS: the LDS bucket (ceilings())
  // (M_LDSG problems are staged like M_LDS ones: `lds` is their M_LDSG footprint)
  bool direct;    // the record is its own staged form (16-bit, 16-byte aligned)
  int32_t lds, inst_words, nid;
  int64_t sw, rec_bytes;
  uint8_t cls;    // cost class of a one-wavefront problem: its anchors (plan_chunk's dispatch order)
};

// One block of plan_chunk's passes: its sums, then (after the scan) its
// image and installed-word bases.
constexpr int32_t kPlanBlock = 512;
constexpr int32_t kPlanPoolMin = 32768;  // chunks this large run every plan pass on the pool
struct PlanBlock {
  int64_t img = 0, inst = 0, core = 0, rbytes = 0, other = 0;
  int32_t ndirect = 0, nother = 0, nok = 0;
  int32_t bcount[kNBuckets] = {}, bmax[kNBuckets] = {};
};

struct Plan {
  int32_t n = 0;
  int32_t n_ldsg = 0;             // problems placed on M_LDSG
  std::vector<int64_t> img_off;   // [n+1] staged word offsets
  std::vector<uint8_t> narrow;    // [n] staged in 16-bit form
  std::vector<int32_t> order;     // workgroup -> local problem
  std::vector<Launch> launches;   // in enqueue order (multi-wave first)
  int big_base = 0;               // first order index of the multi-wave problems
  std::vector<int64_t> scratch_off;  // [order.size() - big_base] int32-word offsets
  int64_t scratch_words = 0;
  std::vector<int32_t> skip;      // local problems not launched (-> DP_ERROR)
  std::vector<int32_t> skip_flags; // their dp_flag (DP_F_TOO_LARGE / DP_F_MALFORMED)
  std::vector<int64_t> inst_off;  // [n+1] local installed-word offsets
  int64_t core_cap = 0;           // sum of identity counts (pool capacity)
  int64_t rec_bytes = 0;          // staged record bytes
  // Device image: word offset of each problem's record, and the image's
  // length (img_off and its total unless start_chunk copies records as they
  // lie, see there)
  std::vector<int64_t> dev_off;
  int64_t img_words = 0;
  std::vector<uint8_t> direct;    // [n] the source record is its own staged form
  int32_t n_direct = 0;
  int64_t other_words = 0;        // source words of the other problems
  // planning scratch, kept across chunks (no allocation or page fault per
  // chunk once grown)
  std::vector<Head> head;
  std::vector<PlanBlock> blk;
  std::vector<int32_t> segcnt;             // [block][segment] one-wavefront counts, then write cursors
  std::vector<int64_t> segpos, segxs;       // segment starts in order; per segment, each XCD's first member
  std::vector<int32_t> big[5], cnt, tmp, grp;
};

// A mid-size record moved onto M_LDSG: staged (or copied) in 16-bit form.
void place_ldsg(Head& H, const int32_t* h, bool aligned) {
  H.lds = layout<M_LDSG>(h).lds_bytes;
  H.sw = staged_words(h, true);
  H.rec_bytes = dp_fmt_packed(h[DP_H_FMT]) ? 4 * dp_rec_phys_words(h)
                                           : 4 * DP_H_SIZE + 2 * ((int64_t)h[DP_H_WORDS] - DP_H_SIZE);
  H.place = M_LDSG;
  H.direct = aligned && (h[DP_H_FMT] == DP_FMT_U16 || dp_fmt_packed(h[DP_H_FMT]));
}

void read_head(Head& H, const int32_t* h, int64_t avail, int32_t opt_flags, bool aligned) {
  H = Head{};
  if (!header_ok(h, avail)) { H.place = -1; return; }
  H.inst_words = bits_words(h[DP_H_NV]);
  H.nid = h[DP_H_NID];
  H.cls = (uint8_t)std::min<int32_t>(h[DP_H_NA], kCostClasses - 1);
  // lds_path, with the one-wavefront layout computed once; past
  // group_above(), a record whose 16-bit image fits a CU may go to the
  // all-LDS multi-wave group (ldsg_ok: plan_chunk decides per chunk;
  // DP_OPT_FORCE_LDSG: always)
  bool nar = false;
  if (dp::fits16(h)) {
    if (!forced_of(opt_flags)) {
      H.lds = layout<M_LDS>(h).lds_bytes;
      nar = H.lds <= dp::group_above();
    }
    if (!nar && (!forced_of(opt_flags) || (opt_flags & DP_OPT_FORCE_LDSG)) && dp::ldsg_fits(h)) {
      if (opt_flags & DP_OPT_FORCE_LDSG) {
        place_ldsg(H, h, aligned);
        return;
      }
      H.ldsg_ok = true;
    }
  }
  H.sw = staged_words(h, nar);
  // algorithmic input bytes (roofline.achieved): the record as the kernel
  // reads it -- the packed form as it is, else the 16-bit form (LDS path) or
  // the int32 form.  Watch lists are derived data and not counted, whether
  // the device builds them (in LDS, or in HBM scratch by the multi-wave
  // passes) or they come with the record (DP_FMT_I32W, host staging): the
  // lists' HBM traffic shows in the PMC figure, not in the compulsory bytes.
  H.rec_bytes = nar ? (dp_fmt_packed(h[DP_H_FMT]) ? 4 * dp_rec_phys_words(h)
                                                 : 4 * DP_H_SIZE + 2 * ((int64_t)h[DP_H_WORDS] - DP_H_SIZE))
                    : 4 * (int64_t)h[DP_H_WORDS];
  if (nar) {
    H.place = M_LDS;
    int k = 0;
    const Ceilings& C = ceilings();
    while (k < C.n - 1 && H.lds > C.c[k]) ++k;
    H.bucket = (int8_t)k;
    H.direct = aligned && (h[DP_H_FMT] == DP_FMT_U16 || dp_fmt_packed(h[DP_H_FMT]));
    return;
  }
  // the multi-wave staged forms: with host-built watch lists, or plain int32
  // for the device to build them (layout.hpp DEV_WATCH_VARS)
  H.direct = aligned && (h[DP_H_FMT] == DP_FMT_I32W || h[DP_H_FMT] == DP_FMT_I32);
  const bool forced = forced_of(opt_flags);
  // (layout arithmetic is int32: variables are capped well below its range)
  const bool sized = h[DP_H_NV] < (1 << 24) && h[DP_H_NID] < (1 << 26) && h[DP_H_WORDS] < (1 << 28);
  if (sized && layout<M_SPLIT>(h).lds_bytes <= kMaxLdsBytes && !(opt_flags & DP_OPT_FORCE_HBM))
    H.place = (opt_flags & DP_OPT_FORCE_MID) || (!forced && h[DP_H_NV] < kMidMaxVars) ? M_SPLIT4 : M_SPLIT;
  else if (sized && layout<M_HBM>(h).lds_bytes <= kMaxLdsBytes)
    H.place = M_HBM;
  else
    H.place = -2;
}

// rec + rec_off[p0 + i] is local problem i.  Problems whose header is not
// well formed are planned as skipped (the caller reports them).  pool (may
// be null) reads the headers in parallel.
// ldsg_busy: M_LDSG problems already in flight on the device (the
// pipeline's other lanes), counted against kLdsgMaxProblems with the chunk's.
void plan_chunk(Plan& P, const int32_t* rec, const int64_t* rec_off, int32_t p0, int32_t n,
                int32_t opt_flags, std::vector<uint8_t>* bad, Pool* pool = nullptr, int32_t ldsg_busy = 0) {
  P.n = n;
  P.n_ldsg = 0;
  P.img_off.resize((size_t)n + 1);
  P.inst_off.resize((size_t)n + 1);
  P.narrow.resize((size_t)n);
  P.direct.resize((size_t)n);
  P.head.resize((size_t)n);
  P.order.clear();
  P.launches.clear();
  P.scratch_off.clear();
  P.skip.clear();
  P.skip_flags.clear();
  P.scratch_words = P.core_cap = P.rec_bytes = P.other_words = 0;
  P.n_direct = 0;
  P.big_base = 0;
  Head* head = P.head.data();
  // Three passes over blocks of kPlanBlock problems (on the pool when there
  // are several blocks; the per-problem work is a header cache miss and its
  // layout arithmetic, ~25 ns a header on one core): the headers, then each
  // block's sums, then the offsets from the scanned sums.  The lists of
  // multi-wave and skipped problems are built in problem order afterwards,
  // only when the chunk has some.
  const int32_t nblk = (n + kPlanBlock - 1) / kPlanBlock;
  P.blk.resize((size_t)std::max(nblk, 1));
  // (a pool run costs its wake-ups: measured on the box, 10k-problem chunks
  // planned faster with only the header pass on the pool -- config 6 0.12-0.16
  // against 0.44 ms with every pass on it -- while 62.5k-problem chunks gain
  // from all of them; kPlanPoolMin)
  auto over_blocks_if = [&](bool par, const std::function<void(int64_t)>& fn) {
    if (pool && nblk > 1 && par) pool->run(nblk, fn, 1);
    else for (int32_t b = 0; b < nblk; ++b) fn(b);
  };
  const bool wide = n >= kPlanPoolMin;
  auto over_blocks = [&](const std::function<void(int64_t)>& fn) { over_blocks_if(wide, fn); };
  over_blocks_if(n > 256, [&](int64_t b) {
    const int32_t i0 = (int32_t)b * kPlanBlock, i1 = std::min(n, i0 + kPlanBlock);
    int32_t nok = 0;
    for (int32_t i = i0; i < i1; ++i) {
      // every header is a cache miss: keep the next ones in flight
      if (i + 8 < i1) {
        const int32_t* h8 = rec + rec_off[p0 + i + 8];
        __builtin_prefetch(h8);
        __builtin_prefetch(h8 + 15);
      }
      read_head(head[i], rec + rec_off[p0 + i], rec_off[p0 + i + 1] - rec_off[p0 + i], opt_flags,
                (rec_off[p0 + i] & 3) == 0);
      nok += head[i].ldsg_ok;
    }
    P.blk[(size_t)b].nok = nok;
  });
  // mid-size catalogs onto the all-LDS group when the chunk holds few of
  // them (placement.hpp kLdsgMaxProblems), else the HBM-read 4-wave groups
  {
    const int lm = dp::ldsg_env();
    int32_t n_ok = 0;
    for (int32_t b = 0; b < nblk; ++b) n_ok += P.blk[(size_t)b].nok;
    // (with other M_LDSG chunks in flight on the device -- concurrent small
    // jobs -- their problems count too: the rule is per device load, so many
    // small chunks do not each take the all-LDS group, the regime measured
    // slower under load)
    if (n_ok > 0 && (lm == dp::LDSG_ALWAYS || (lm == dp::LDSG_AUTO && n_ok + ldsg_busy <= dp::kLdsgMaxProblems))) {
      for (int32_t i = 0; i < n; ++i)
        if (head[i].ldsg_ok) place_ldsg(head[i], rec + rec_off[p0 + i], (rec_off[p0 + i] & 3) == 0);
      P.n_ldsg = n_ok;
    }
  }
  // per block: totals and per-bucket counts / LDS maxima
  const bool rec_aligned = ((uintptr_t)rec & 15) == 0;
  over_blocks([&](int64_t b) {
    PlanBlock& B = P.blk[(size_t)b];
    const int32_t nok = B.nok;
    B = PlanBlock{};
    B.nok = nok;
    const int32_t i0 = (int32_t)b * kPlanBlock, i1 = std::min(n, i0 + kPlanBlock);
    for (int32_t i = i0; i < i1; ++i) {
      const Head& H = head[i];
      const bool d = rec_aligned && H.direct;
      B.ndirect += d;
      B.other += d ? 0 : rec_off[p0 + i + 1] - rec_off[p0 + i];
      if (H.place == M_LDS) {
        B.bcount[H.bucket]++;
        B.bmax[H.bucket] = std::max(B.bmax[H.bucket], H.lds);
      } else {
        B.nother++;
      }
      if (H.place != -1) {
        B.img += H.sw;
        B.inst += H.inst_words;
        B.core += H.nid;
        B.rbytes += H.rec_bytes;
      }
    }
  });
  for (auto& v : P.big) v.clear();
  int32_t bcount[kNBuckets] = {}, bmax[kNBuckets] = {};
  int64_t img = 0, inst = 0;
  bool others = false;
  for (int32_t b = 0; b < nblk; ++b) {  // the scan
    PlanBlock& B = P.blk[(size_t)b];
    const int64_t bi = B.img, bn = B.inst;
    B.img = img;
    B.inst = inst;
    img += bi;
    inst += bn;
    P.n_direct += B.ndirect;
    P.other_words += B.other;
    P.core_cap += B.core;
    P.rec_bytes += B.rbytes;
    others |= B.nother > 0;
    for (int k = 0; k < kNBuckets; ++k) {
      bcount[k] += B.bcount[k];
      bmax[k] = std::max(bmax[k], B.bmax[k]);
    }
  }
  P.dev_off.resize((size_t)n);
  P.img_off[0] = P.inst_off[0] = 0;
  over_blocks([&](int64_t b) {
    const PlanBlock& B = P.blk[(size_t)b];
    int64_t im = B.img, in = B.inst;
    const int32_t i0 = (int32_t)b * kPlanBlock, i1 = std::min(n, i0 + kPlanBlock);
    for (int32_t i = i0; i < i1; ++i) {
      const Head& H = head[i];
      P.direct[(size_t)i] = rec_aligned && H.direct;
      P.narrow[(size_t)i] = H.place == M_LDS || H.place == M_LDSG;
      P.dev_off[(size_t)i] = im;
      if (H.place != -1) {
        im += H.sw;
        in += H.inst_words;
      }
      P.img_off[(size_t)i + 1] = im;
      P.inst_off[(size_t)i + 1] = in;
    }
  });
  if (others)
    for (int32_t i = 0; i < n; ++i) {
      const Head& H = head[i];
      if (H.place == M_LDS) continue;
      if (H.place >= 0) {
        P.big[(size_t)H.place].push_back(i);
      } else {
        if (H.place == -1 && bad) (*bad)[(size_t)i] = 1;
        P.skip.push_back(i);
        P.skip_flags.push_back(H.place == -1 ? DP_F_MALFORMED : DP_F_TOO_LARGE);
      }
    }
  P.img_words = img;
  // Within a launch, workgroups are dispatched in blockIdx order: largest
  // record first (longest-processing-time-first), so the long solves do not
  // form the launch's tail.
  // (a counting sort on the staged size, stable: ties keep problem order)
  auto cost = [&](int32_t i) { return P.img_off[(size_t)i + 1] - P.img_off[(size_t)i]; };
  auto lpt = [&](int32_t* v, size_t m) {
    if (m < 2) return;
    int64_t lo = INT64_MAX, hi = 0;
    for (size_t j = 0; j < m; ++j) { lo = std::min(lo, cost(v[j])); hi = std::max(hi, cost(v[j])); }
    if (hi - lo > 4 * (int64_t)m + 65536) {  // a wide range: comparison sort
      std::stable_sort(v, v + m, [&](int32_t x, int32_t y) { return cost(x) > cost(y); });
      return;
    }
    P.cnt.assign((size_t)(hi - lo) + 2, 0);
    for (size_t j = 0; j < m; ++j) P.cnt[(size_t)(hi - cost(v[j])) + 1]++;
    for (size_t k = 1; k < P.cnt.size(); ++k) P.cnt[k] += P.cnt[k - 1];
    P.tmp.resize(m);
    for (size_t j = 0; j < m; ++j) P.tmp[(size_t)P.cnt[(size_t)(hi - cost(v[j]))]++] = v[j];
    std::copy(P.tmp.begin(), P.tmp.begin() + (int64_t)m, v);
  };
  // multi-wave launches first: the long-running large catalogs start earliest
  for (int mode : {(int)M_LDSG, (int)M_SPLIT4, (int)M_SPLIT, (int)M_HBM}) {
    auto& bg = P.big[(size_t)mode];
    if (bg.empty()) continue;
    lpt(bg.data(), bg.size());
    int mx = 0;
    Launch L{(int)P.order.size(), (int)bg.size(), mode, 0, false};
    for (int32_t i : bg) {
      const int32_t* h = rec + rec_off[p0 + i];
      L.dev_lists |= h[DP_H_FMT] == DP_FMT_I32 && !dp::device_watches(h);
      const Layout Y = mode == M_SPLIT    ? layout<M_SPLIT>(h)
                       : mode == M_SPLIT4 ? layout<M_SPLIT4>(h)
                       : mode == M_LDSG   ? layout<M_LDSG>(h)
                                          : layout<M_HBM>(h);
      mx = std::max(mx, Y.lds_bytes);
      if (P.scratch_words == 0) P.scratch_words = dp::kQueueWords;  // the launches' queues first
      P.scratch_off.push_back(P.scratch_words);
      P.scratch_words += ((int64_t)Y.bytes + 15) / 16 * 4;  // int32 words, 16-byte aligned
    }
    L.lds = mx;
    P.launches.push_back(L);
    P.order.insert(P.order.end(), bg.begin(), bg.end());
  }
  P.big_base = 0;  // scratch_off is indexed from the first multi-wave workgroup (order index 0)
  // LDS buckets, largest footprint first, are merged into the launch of the
  // bucket before them (whose largest footprint the launch requests) while
  // their members keep at least kMergeRatio of their own residency, or when
  // they are too few for a launch of their own (its tail would be most of it).
  static const double merge = [] {  // diagnostic DEPPY_BUCKET_MERGE
    const char* m = std::getenv("DEPPY_BUCKET_MERGE");
    return m ? std::atof(m) : kMergeRatio;
  }();
  int group_of[kNBuckets];
  Launch bl[kNBuckets];
  int64_t gsize[kNBuckets] = {};
  int ng = 0;
  for (int k = kNBuckets - 1; k >= 0; --k) {
    if (!bcount[k]) continue;
    const bool join = ng > 0 && (bcount[k] < kMinLaunch ||
                                 (merge > 0 && (double)(kMaxLdsBytes / bl[ng - 1].lds) >=
                                                   merge * (double)(kMaxLdsBytes / bmax[k])));
    if (!join) bl[ng++] = Launch{0, 0, M_LDS, bmax[k]};
    group_of[k] = ng - 1;
    gsize[ng - 1] += bcount[k];
  }
  // the bucket launches, the most problems first; members in problem order,
  // then each launch's members by LPT
  int ix[kNBuckets];
  for (int g = 0; g < ng; ++g) ix[g] = g;
  std::stable_sort(ix, ix + ng, [&](int x, int y) { return gsize[x] > gsize[y]; });
  int64_t o = (int64_t)P.order.size();
  for (int r = 0; r < ng; ++r) {
    const int g = ix[r];
    bl[g].first = (int)o;
    bl[g].count = (int)gsize[g];
    o += gsize[g];
  }
  P.order.resize((size_t)o);
  // XCD-contiguous order for one-wavefront launches up to this LDS request
  // (DEPPY_XCD_ORDER, bytes; 0: longest record first everywhere).  Measured
  // on one box against LPT: config 2 host to host 18.4-18.5M -> 20.3-20.6M
  // res/s, kernel only 22.4M -> 23.9-24.2M; config 3 PMC writes per run
  // 10.9 -> 6.5 MB; config 5 and 6 unchanged (scripts/xcd_ab.sh,
  // profiles/r03_xcd_order_ab.txt).
  // Within such a launch, dispatch order by cost class, the costliest
  // first: a catalog's anchors (Mandatory roots, lit_mapping.go:163-174)
  // start its search, and on config 2 they predict its steps (correlation
  // 0.7 with their log; 89 of the 100 slowest of 10k catalogs have 3 or 4
  // of 4), so the slow ones start with the launch instead of forming its
  // tail.  Within a class XCD-contiguous: workgroup b runs on XCD b % kXcds,
  // so XCD x takes the x-th contiguous range of the class's members in
  // problem order: neighbouring records (sharing their boundary lines) are
  // read, and neighbouring results written, through one XCD's L2 at about
  // the same time.
  // Built as one stable counting sort of the one-wavefront problems by
  // segment (launch rank, class) over the plan's blocks, then every segment
  // dealt to the XCDs, both passes on the pool.
  static const int64_t xcd_order = env_i64("DEPPY_XCD_ORDER", kMaxLdsBytes);
  static const bool anchor_order = env_i64("DEPPY_ANCHOR_ORDER", 1) != 0;  // diagnostic A/B
  if (ng > 0) {
    int rank_of[kNBuckets];
    bool xo[kNBuckets];
    for (int r = 0; r < ng; ++r) {
      rank_of[ix[r]] = r;
      xo[ix[r]] = xcd_order && bl[ix[r]].lds <= xcd_order;
    }
    const int nseg = ng * kCostClasses;
    auto seg_of = [&](const Head& H) {
      const int g = group_of[H.bucket];
      const int c = anchor_order && xo[g] ? H.cls : 0;
      return rank_of[g] * kCostClasses + (kCostClasses - 1 - c);
    };
    P.segcnt.assign((size_t)nblk * nseg, 0);
    over_blocks([&](int64_t b) {
      int32_t* c = P.segcnt.data() + (size_t)b * nseg;
      const int32_t i0 = (int32_t)b * kPlanBlock, i1 = std::min(n, i0 + kPlanBlock);
      for (int32_t i = i0; i < i1; ++i)
        if (head[i].place == M_LDS) c[seg_of(head[i])]++;
    });
    P.segpos.resize((size_t)nseg + 1);
    int64_t run = bl[ix[0]].first;  // (the one-wavefront launches follow the multi-wave ones)
    for (int sg = 0; sg < nseg; ++sg) {
      P.segpos[(size_t)sg] = run;
      for (int32_t b = 0; b < nblk; ++b) {
        int32_t& c = P.segcnt[(size_t)b * nseg + sg];
        const int32_t x = c;
        c = (int32_t)run;
        run += x;
      }
    }
    P.segpos[(size_t)nseg] = run;
    P.tmp.resize((size_t)o);
    over_blocks([&](int64_t b) {
      int32_t* c = P.segcnt.data() + (size_t)b * nseg;
      const int32_t i0 = (int32_t)b * kPlanBlock, i1 = std::min(n, i0 + kPlanBlock);
      for (int32_t i = i0; i < i1; ++i)
        if (head[i].place == M_LDS) P.tmp[(size_t)c[seg_of(head[i])]++] = i;
    });
    // each segment [pos, end): slot b (XCD x = b % kXcds) takes the next of
    // XCD x's contiguous range of the segment's members
    P.segxs.resize((size_t)nseg * kXcds);
    // (XCDs count from the launch's first workgroup: slot t of launch g is
    // workgroup t - bl[g].first)
    auto first_on = [&](int sg, int64_t pos, int x) {  // the segment's first slot on XCD x
      const int64_t rel = pos - bl[ix[sg / kCostClasses]].first;
      return pos + ((x - rel % kXcds) % kXcds + kXcds) % kXcds;
    };
    for (int sg = 0; sg < nseg; ++sg) {
      const int64_t pos = P.segpos[(size_t)sg], end = P.segpos[(size_t)sg + 1];
      int64_t st = pos;
      for (int x = 0; x < kXcds; ++x) {
        P.segxs[(size_t)sg * kXcds + x] = st;
        const int64_t first = first_on(sg, pos, x);
        st += first < end ? (end - 1 - first) / kXcds + 1 : 0;
      }
    }
    const int64_t o0 = bl[ix[0]].first, nslot = o - o0;
    const int32_t sblk = (int32_t)((nslot + kPlanBlock - 1) / kPlanBlock);
    auto deal = [&](int64_t b) {
      const int64_t s0 = o0 + b * kPlanBlock, s1 = std::min<int64_t>(o, s0 + kPlanBlock);
      int sg = (int)(std::upper_bound(P.segpos.begin(), P.segpos.end(), s0) - P.segpos.begin()) - 1;
      for (int64_t t = s0; t < s1; ++t) {
        while (P.segpos[(size_t)sg + 1] <= t) ++sg;
        const int g = ix[sg / kCostClasses];
        if (!xo[g]) {
          P.order[(size_t)t] = P.tmp[(size_t)t];
          continue;
        }
        const int x = (int)((t - bl[g].first) % kXcds);
        const int64_t first = first_on(sg, P.segpos[(size_t)sg], x);
        P.order[(size_t)t] = P.tmp[(size_t)(P.segxs[(size_t)sg * kXcds + x] + (t - first) / kXcds)];
      }
    };
    if (pool && sblk > 1 && wide) pool->run(sblk, std::function<void(int64_t)>(deal), 1);
    else for (int32_t b = 0; b < sblk; ++b) deal(b);
    for (int r = 0; r < ng; ++r) {
      const int g = ix[r];
      if (!xo[g]) lpt(P.order.data() + bl[g].first, (size_t)bl[g].count);
      P.launches.push_back(bl[g]);
    }
  }
  static const int pad_kb = (int)env_i64("DEPPY_LDS_PAD_KB", 0);  // diagnostic (occupancy study)
  if (pad_kb > 0)
    for (auto& L : P.launches)
      if (L.mode == M_LDS) L.lds = std::max(L.lds, pad_kb * 1024);
}

// Copy n words of s into d (narrowing or widening), checking lo <= x < hi
// for each (one pass: the min/max reductions and the stores vectorise).
template <class S, class D>
__attribute__((always_inline)) static inline bool copy_range(const S* __restrict s, D* __restrict d, int32_t n,
                                                             int32_t lo, int32_t hi) {
  int32_t mn = INT32_MAX, mx = INT32_MIN;
  for (int32_t j = 0; j < n; ++j) {
    const int32_t x = (int32_t)s[j];
    mn = x < mn ? x : mn;
    mx = x > mx ? x : mx;
    d[j] = (D)x;
  }
  return n == 0 || (mn >= lo && mx < hi);
}
// An offsets array: s[0] == 0, non-decreasing, s[n] == total.
template <class S, class D>
__attribute__((always_inline)) static inline bool copy_offsets(const S* __restrict s, D* __restrict d, int32_t n,
                                                               int32_t total) {
  int32_t dec = 0;
  for (int32_t j = 0; j < n; ++j) dec |= (int32_t)s[j + 1] < (int32_t)s[j];
  for (int32_t j = 0; j <= n; ++j) d[j] = (D)s[j];
  return (int32_t)s[0] == 0 && (int32_t)s[n] == total && !dec;
}

// The checked copy of a record's body (header h, which passed header_ok;
// source body in S words, destination body in D words): dp_rec_validate's
// checks fused into the copy.  Into 16 bits, AtMost bounds over the row
// length are stored as the row length (the same row: neither can be
// exceeded by the count).
template <class S, class D>
__attribute__((always_inline)) static inline bool convert_body(const int32_t* h, const S* sb, D* db) {
  const dp_rec_layout L = dp_rec_layout_of(h);
  const int32_t nv = h[DP_H_NV], nc = h[DP_H_NC], nk = h[DP_H_NK], nch = h[DP_H_NCH];
  const int32_t nid = h[DP_H_NID], ncl = h[DP_H_NCL], nkl = h[DP_H_NKL], nchl = h[DP_H_NCHL];
  auto s = [&](int32_t word) { return sb + (word - DP_H_SIZE); };
  auto d = [&](int32_t word) { return db + (word - DP_H_SIZE); };
  bool ok = copy_offsets(s(L.clause_off), d(L.clause_off), nc, ncl);
  ok &= copy_range(s(L.clause_lits), d(L.clause_lits), ncl, 0, 2 * nv);
  ok &= copy_range(s(L.clause_id), d(L.clause_id), nc, 0, nid);
  ok &= copy_offsets(s(L.card_off), d(L.card_off), nk, nkl);
  ok &= copy_range(s(L.card_lits), d(L.card_lits), nkl, 0, nv);
  ok &= copy_range(s(L.card_id), d(L.card_id), nk, 0, nid);
  ok &= copy_offsets(s(L.var_choice_off), d(L.var_choice_off), nv, nch);
  ok &= copy_offsets(s(L.choice_off), d(L.choice_off), nch, nchl);
  ok &= copy_range(s(L.choice_lits), d(L.choice_lits), nchl, 0, nv);
  ok &= copy_range(s(L.anchors), d(L.anchors), h[DP_H_NA], 0, nv);
  if (!ok) return false;
  // the positions of a variable form one run: run starts are distinct within
  // a row (a per-thread mark array, one tag per row)
  static thread_local std::vector<uint32_t> mark;
  static thread_local uint32_t tag = 0;
  if (mark.size() < (size_t)nv) mark.assign((size_t)nv + 1024, 0);
  const S* co = s(L.card_off);
  const S* cl = s(L.card_lits);
  const S* cb = s(L.card_bound);
  D* ob = d(L.card_bound);
  for (int32_t k = 0; k < nk; ++k) {
    const int32_t a = (int32_t)co[k], b = (int32_t)co[k + 1], bound = (int32_t)cb[k];
    if (bound < 0) return false;
    ob[k] = (D)(sizeof(D) == 2 ? std::min(bound, b - a) : bound);
    if (++tag == 0) {
      std::fill(mark.begin(), mark.end(), 0u);
      tag = 1;
    }
    for (int32_t j = a; j < b; ++j)
      if (j == a || cl[j] != cl[j - 1]) {
        if (mark[(size_t)cl[j]] == tag) return false;
        mark[(size_t)cl[j]] = tag;
      }
  }
  return true;
}
// (AVX2 clones of the three checked copies, picked at run time)
template <class S, class D>
__attribute__((target("avx2"))) static bool convert_avx2(const int32_t* h, const S* sb, D* db) {
  return convert_body(h, sb, db);
}
template <class S, class D>
static bool convert_generic(const int32_t* h, const S* sb, D* db) { return convert_body(h, sb, db); }
template <class S, class D>
static bool convert(const int32_t* h, const S* sb, D* db) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  return avx2 ? convert_avx2(h, sb, db) : convert_generic(h, sb, db);
}

// Problems per pool work item when staging n records: a few items per
// thread at least (a chunk of 28 OLM-scale records must not go to one thread).
int64_t stage_block(int64_t n, const Pool& pool) {
  return std::max<int64_t>(1, std::min<int64_t>(32, n / (8 * (int64_t)std::max(1, pool.size()))));
}

// Stage local problem i of the plan into dst (the staged image area): the
// int32 header with its format word, then the body in the form the plan
// chose.  A 16-bit record to a 16-bit copy, or a plain int32 record to a
// multi-wave group, is copied as it is; a 16-bit record for a multi-wave
// problem is widened.  Every body is checked once: a record copied as it is
// by the kernel (valid_record for DP_FMT_U16, valid_wide for DP_FMT_I32, whose
// watch lists the device builds), any other here, while narrowing it
// (DP_FMT_U16_CHECKED) or before building its watch lists.  Returns false for
// a malformed record:
// its staged copy is marked DP_FMT_REJECT and the kernel reports DP_ERROR /
// DP_F_MALFORMED for it.
bool stage_one(const Plan& P, const int32_t* rec, const int64_t* rec_off, int32_t p0, int32_t i,
               int32_t* dst, bool host_check) {
  const int64_t at = P.dev_off[(size_t)i], sw = P.img_off[(size_t)i + 1] - P.img_off[(size_t)i];
  if (sw == 0) return true;  // skipped (header already rejected)
  const int32_t* src = rec + rec_off[p0 + i];
  int32_t* d = dst + at;
  const int64_t words = src[DP_H_WORDS], body = words - DP_H_SIZE;
  const int32_t fmt = src[DP_H_FMT];
  std::memcpy(d, src, 4 * DP_H_SIZE);
  if (P.narrow[(size_t)i]) {
    if (fmt == DP_FMT_I32 || fmt == DP_FMT_I32W) {
      d[DP_H_FMT] = DP_FMT_U16_CHECKED;
      uint16_t* o = reinterpret_cast<uint16_t*>(d + DP_H_SIZE);
      if (!convert(src, src + DP_H_SIZE, o)) {
        d[DP_H_FMT] = DP_FMT_REJECT;
        return false;
      }
      for (int64_t j = body; j < 2 * (sw - DP_H_SIZE); ++j) o[j] = 0;
    } else if (host_check) {
      // a 16-bit form checked and expanded here (the latency path: one
      // catalog's decode and validation cost the kernel more than the host)
      static thread_local std::vector<int32_t> wide;
      wide.resize((size_t)words);
      d[DP_H_FMT] = DP_FMT_U16_CHECKED;
      uint16_t* o = reinterpret_cast<uint16_t*>(d + DP_H_SIZE);
      if (dp_rec_widen(src, rec_off[p0 + i + 1] - rec_off[p0 + i], wide.data()) != 0 ||
          !convert(wide.data(), wide.data() + DP_H_SIZE, o)) {
        d[DP_H_FMT] = DP_FMT_REJECT;
        return false;
      }
      for (int64_t j = body; j < 2 * (sw - DP_H_SIZE); ++j) o[j] = 0;
    } else {  // a 16-bit form, copied as it is (validated by the kernel)
      const int64_t phys = dp_rec_phys_words(src);
      std::memcpy(d + DP_H_SIZE, src + DP_H_SIZE, 4 * (size_t)(phys - DP_H_SIZE));
      for (int64_t j = phys; j < sw; ++j) d[j] = 0;
    }
  } else if (fmt == DP_FMT_I32) {
    // a plain int32 record for a multi-wave group: copied as it is, like a
    // record DMA'd as it lies -- the kernel checks it (valid_wide) and the
    // device builds its watch lists (the solving workgroup, or the grid-wide
    // passes above DEV_WATCH_VARS).  Building them here cost one host thread
    // ~2 ms per OLM-scale catalog inside a latency call.
    std::memcpy(d + DP_H_SIZE, src + DP_H_SIZE, 4 * (size_t)body);
    for (int64_t j = words; j < sw; ++j) d[j] = 0;
  } else {
    d[DP_H_FMT] = dp::DP_FMT_I32_CHECKED;  // checked here, watch lists built here
    bool ok;
    if (dp_fmt_packed(fmt)) {  // its int32 form, then the checked copy
      static thread_local std::vector<int32_t> wide;
      wide.resize((size_t)words);
      ok = dp_rec_widen(src, rec_off[p0 + i + 1] - rec_off[p0 + i], wide.data()) == 0 &&
           convert(src, wide.data() + DP_H_SIZE, d + DP_H_SIZE);
    } else {
      ok = fmt == DP_FMT_U16 ? convert(src, reinterpret_cast<const uint16_t*>(src + DP_H_SIZE), d + DP_H_SIZE)
                             : convert(src, src + DP_H_SIZE, d + DP_H_SIZE);
    }
    // the watch lists are built here, from the checked int32 copy
    if (!ok) {
      d[DP_H_FMT] = DP_FMT_REJECT;
      return false;
    }
    const int64_t end = build_watches_host(d);
    for (int64_t j = end; j < sw; ++j) d[j] = 0;
  }
  return true;
}

void* pinned_alloc(size_t bytes) {
  int n = 0;
  void* p = nullptr;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}
void pinned_free(void* p) { (void)hipHostFree(p); }

}  // namespace dp

namespace {

using dp::Plan;

// Are the first and the last byte of [p, p + bytes) page-locked host memory?
bool pinned_range(const void* p, size_t bytes) {
  auto locked = [](const void* q) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeHost;
  };
  return bytes > 0 && locked(p) && locked(static_cast<const char*>(p) + bytes - 1);
}

// Byte layout of a chunk's input region (identical in pinned host memory and
// on the device, so one copy moves it) and of its output region.
struct InLayout {
  size_t img, items, pool_len, scratch_off, end;
};
struct OutLayout {
  size_t prob, installed, pool_len, pool, end;
  size_t d2h;  // bytes copied back by the pipelined D2H
};

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

InLayout in_layout(const Plan& P) {
  InLayout L;
  size_t o = 0;
  L.img = o;         o = al(o + (size_t)P.img_words * 4);
  L.items = o;       o = al(o + P.order.size() * sizeof(dp::WorkItem));
  L.pool_len = o;    o = al(o + 4);  // the core pool's counter, zeroed by the chunk's H2D copy
  L.scratch_off = o; o = al(o + P.scratch_off.size() * 8);
  L.end = o;
  return L;
}

OutLayout out_layout(const Plan& P) {
  OutLayout L;
  const size_t n = (size_t)P.n;
  size_t o = 0;
  L.prob = o;      o = al(o + n * sizeof(dp::ProblemOut));
  L.installed = o; o = al(o + (size_t)P.inst_off[n] * 4);
  L.pool_len = o;  o = al(o + 4);
  L.pool = o;      o = al(o + (size_t)std::max<int64_t>(P.core_cap, 1) * 4);
  L.end = o;
  L.d2h = L.pool + (size_t)std::min<int64_t>(P.core_cap, kCoreWordsPerProblem * (int64_t)n) * 4;
  return L;
}

// Fill the non-image parts of an input region.
void fill_in_tables(const Plan& P, const InLayout& L, char* base) {
  dp::WorkItem* it = reinterpret_cast<dp::WorkItem*>(base + L.items);
  for (size_t k = 0; k < P.order.size(); ++k) {
    const int32_t i = P.order[k];
    it[k] = dp::WorkItem{P.dev_off[(size_t)i], (int32_t)P.inst_off[(size_t)i], i};
  }
  *reinterpret_cast<int32_t*>(base + L.pool_len) = 0;
  if (!P.scratch_off.empty()) std::memcpy(base + L.scratch_off, P.scratch_off.data(), P.scratch_off.size() * 8);
}

// Results of a chunk (output region `out`, local problems) -> the caller's
// dp_result at global problems p0...  Cores come from the pool.
// Returns the chunk's BCP-visited bytes.  One pass over the per-problem
// results (in blocks on `pool` when given and the chunk is large).
uint64_t scatter(const Plan& P, const OutLayout& L, const char* out, int32_t p0, dp_result* res,
                 dp::Pool* pool = nullptr) {
  const int32_t n = P.n;
  const dp::ProblemOut* po = reinterpret_cast<const dp::ProblemOut*>(out + L.prob);
  const uint32_t* inst = reinterpret_cast<const uint32_t*>(out + L.installed);
  const int32_t* cpool = reinterpret_cast<const int32_t*>(out + L.pool);
  const bool same_inst = res->inst_off[p0 + n] - res->inst_off[p0] == P.inst_off[(size_t)n];
  constexpr int32_t kBlock = 1024;
  const int32_t nb = (n + kBlock - 1) / kBlock;
  static thread_local std::vector<uint64_t> part_tl;  // (per calling thread: no allocation once grown)
  std::vector<uint64_t>& part = part_tl;  // (a local name: the pool's threads write the caller's vector)
  part.assign((size_t)std::max(nb, 1), 0);
  auto block = [&](int64_t b) {
    const int32_t i0 = (int32_t)b * kBlock, i1 = std::min(n, i0 + kBlock);
    uint64_t bcp = 0;
    for (int32_t i = i0; i < i1; ++i) {
      const dp::ProblemOut& o = po[i];
      res->status[p0 + i] = o.status;
      res->flags[p0 + i] = o.flags;
      res->core_len[p0 + i] = o.core_len;
      if (res->steps) res->steps[p0 + i] = o.steps;
      bcp += o.bcp;
      if (o.core_len > 0) {
        const int64_t cap = res->core_off[p0 + i + 1] - res->core_off[p0 + i];
        std::memcpy(res->core + res->core_off[p0 + i], cpool + o.core_at,
                    (size_t)std::min<int64_t>(o.core_len, cap) * 4);
      }
      if (!same_inst) {  // a caller layout of its own: problem by problem
        const int64_t w = std::min(P.inst_off[(size_t)i + 1] - P.inst_off[(size_t)i],
                                   res->inst_off[p0 + i + 1] - res->inst_off[p0 + i]);
        std::memcpy(res->installed + res->inst_off[p0 + i], inst + P.inst_off[(size_t)i], (size_t)w * 4);
      }
    }
    if (same_inst) {
      const int64_t w0 = P.inst_off[(size_t)i0], w1 = P.inst_off[(size_t)i1];
      std::memcpy(res->installed + res->inst_off[p0] + w0, inst + w0, (size_t)(w1 - w0) * 4);
    }
    part[(size_t)b] = bcp;
  };
  if (pool && nb >= 4) pool->run(nb, std::function<void(int64_t)>(block), 1);
  else for (int32_t b = 0; b < nb; ++b) block(b);
  uint64_t bcp = 0;
  for (uint64_t x : part) bcp += x;
  for (size_t q = 0; q < P.skip.size(); ++q) {
    const int32_t i = P.skip[q];
    res->status[p0 + i] = DP_ERROR;
    res->flags[p0 + i] = P.skip_flags[q];
    res->core_len[p0 + i] = 0;
    if (res->steps) res->steps[p0 + i] = 0;
    for (int64_t w = res->inst_off[p0 + i]; w < res->inst_off[p0 + i + 1]; ++w) res->installed[w] = 0;
  }
  return bcp;
}

template <class T>
T* at(char* base, size_t off) {
  return reinterpret_cast<T*>(base + off);
}

dp::KernelArgs kernel_args(const InLayout& I, const OutLayout& O, char* din, char* dout, int32_t* scratch,
                           int64_t budget) {
  dp::KernelArgs a{};
  a.rec = at<int32_t>(din, I.img);
  a.items = at<dp::WorkItem>(din, I.items);
  a.out = at<dp::ProblemOut>(dout, O.prob);
  a.installed = at<uint32_t>(dout, O.installed);
  a.core = at<int32_t>(dout, O.pool);
  a.core_pool_len = at<int32_t>(dout, O.pool_len);
  a.budget = budget;
  a.scratch = scratch;
  a.scratch_off = at<int64_t>(din, I.scratch_off);
  return a;
}

// Allocations made by growing buffers (hipMalloc / hipHostMalloc), process
// wide: dp_stats.allocs reports the ones made on behalf of a context.
std::atomic<int64_t> g_buf_allocs{0};

// A growable buffer, device or pinned host.
struct Buf {
  char* p = nullptr;
  size_t cap = 0;
  bool host = false;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    n = std::max<size_t>(al(n + n / 8), 4096);
    hipError_t e = host ? hipHostMalloc(reinterpret_cast<void**>(&p), n,
                                        hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent)
                        : hipMalloc(reinterpret_cast<void**>(&p), n);
    if (e != hipSuccess) { p = nullptr; cap = 0; return e; }
    g_buf_allocs.fetch_add(1, std::memory_order_relaxed);
    dev = p;
    if (host && hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), p, 0) != hipSuccess) dev = p;
    cap = n;
    return hipSuccess;
  }
  char* dev = nullptr;  // device address of a mapped host buffer (zero-copy)
  void release() {
    if (p) (void)(host ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct dp_job;

// One stream with its own buffers; holds at most one chunk in flight.
// A chunk's one-wavefront launches after its first, spread over other
// lane streams of the device (DEPPY_SPREAD=1, A/B): each waits for the
// chunk's copies (`start`, recorded on the chunk's stream before its first
// launch) and the chunk's stream waits for each (`fin`), so launches of
// different LDS buckets run side by side -- the dispatcher packs workgroups
// of both onto a CU -- instead of one after another, each with its own tail.
constexpr int kMaxSpread = 4;
struct Spread {
  hipStream_t s[kMaxSpread] = {};
  int n = 0;
  hipEvent_t start = nullptr, fin[kMaxSpread] = {};
  int create() {
    if (hipEventCreateWithFlags(&start, hipEventDisableTiming) != hipSuccess) return -1;
    for (auto& e : fin)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return -1;
    return 0;
  }
  void destroy() {
    if (start) (void)hipEventDestroy(start);
    for (auto& e : fin)
      if (e) (void)hipEventDestroy(e);
    start = nullptr;
    for (auto& e : fin) e = nullptr;
  }
};

struct Lane {
  int device = 0;
  hipStream_t s = nullptr;
  hipEvent_t k0 = nullptr, k1 = nullptr, done = nullptr;
  // copy stream of the lane's records (shared like s): the next chunk's H2D
  // runs while the stream's current kernel does; `copied` orders the launch
  hipStream_t cs = nullptr;
  hipEvent_t copied = nullptr;
  Spread spread;  // (DEPPY_SPREAD) its events; the sibling streams are set per chunk
  Buf h_in{nullptr, 0, true}, d_in, h_out{nullptr, 0, true}, d_out, scratch;
  bool zc_out = false;  // the chunk's kernels wrote their results straight into h_out
  // the chunk in flight
  dp_job* job = nullptr;
  int32_t p0 = 0;
  // its results being scattered by the device's finisher thread (under
  // Device::fmu): the lane's buffers and plan are the finisher's until then
  dp_job* fjob = nullptr;
  bool scattering = false;
  Plan plan;
  OutLayout ol{};
  std::vector<uint8_t> bad;  // per-problem malformed marks of the chunk being started
};

// One piece of a submitted job for a device's worker: problems [p0, p0+n).
struct Task {
  dp_job* job;
  int32_t p0, n;
};

// A device of the context.  Its pipeline lanes belong to one host worker
// thread (worker_main): dp_submit only cuts a batch into chunks and queues
// them here, so a caller thread never plans, stages, waits or scatters, and
// every device of a multi-device context has its own submitting thread.
// The latency path of a small synchronous dp_solve (the reference's one
// problem per Solve, solve.go:53-119): on the caller's thread, through a
// stream of its own, with the records read by the kernel from mapped pinned
// memory (no H2D copy) and the results written back into it, completion
// polled without sleeping.  Buffers grow once and stay.
struct FastLane {
  std::mutex mu;
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  Buf h_in{nullptr, 0, true}, h_out{nullptr, 0, true};
  Plan plan;
  std::vector<uint8_t> bad;
};
constexpr int32_t kFastProblems = 16;    // dp_solve batches up to this many problems
constexpr int64_t kFastWords = 1 << 16;  // and this many record words take the latency path

struct Device {
  int ordinal = 0;
  Lane lanes[kMaxLanes];
  int nstreams = kStreams, nlanes = 2 * kStreams;
  // the event after the last chunk's record copies, and the chunks left of
  // the current pipeline fill (worker only; start_chunk)
  hipEvent_t last_copied = nullptr;
  int fill_left = 0;
  int next = 0;  // resident launches: next lane
  FastLane fast;
  // -- the worker's --
  std::thread worker;
  std::mutex qmu;                 // q and stop (and the wake-ups)
  std::condition_variable qcv;
  std::deque<Task> q;             // chunks waiting for a lane
  bool stop = false;
  int cursor = 0;                 // next lane (round robin)
  std::deque<Lane*> inflight;     // lanes holding a chunk, oldest first (worker only)
  dp::Pool* pool = nullptr;       // staging and planning threads of this device
  bool own_pool = false;
  // -- the finisher's: chunks done on the GPU, their results scattered into
  // their jobs' dp_result off the worker's path (finisher_main) --
  std::thread finisher;
  std::mutex fmu;
  std::condition_variable fcv;
  std::deque<Lane*> fq;
  bool fstop = false;
  dp::Pool* fpool = nullptr;  // its scatter threads
  std::mutex smu;                 // st
  dp_stats st{};                  // this device's pipeline counters
};

struct dp_job {
  int32_t n = 0;
  const int32_t* rec = nullptr;
  const int64_t* rec_off = nullptr;
  bool pinned = false;  // the records are page-locked (pinned_range)
  dp_result res{};
  // completion: chunks not yet delivered; the waiter sleeps on cv
  std::mutex m;
  std::condition_variable cv;
  int chunks_left = 0;
  std::atomic<bool> waiting{false};  // dp_job_wait is blocked on it: its chunks are finished eagerly
  int rc = 0;
  std::string err;
};

struct dp_ctx {
  std::deque<Device> dev;  // (a deque: a Device holds a thread and mutexes, it never moves)
  int64_t budget = kDefaultBudget;
  int32_t flags = 0;  // dp_opt_flag
  std::string err;
  std::atomic<double> last_ms{0.0};
  std::mutex mu;
  dp::Pool* pool = nullptr;
  mutable std::mutex err_mu;  // err: written by any caller thread (set_err), read by dp_last_error
  int next_dev = 0;  // pipeline cursor over devices (under mu)
  bool zc_in = false, zc_out = true;  // zero-copy records / results (start_chunk)
  bool copy_streams = false;          // records' H2D on a stream of its own (DEPPY_COPY_STREAM=1)
  bool direct = true;  // copy page-locked batches of staged-form records as they are
  int32_t chunk_problems = kChunkProblems;
  int64_t chunk_bytes = kChunkBytes;
  int32_t min_shared_chunk = kMinSharedChunk;  // (DEPPY_MIN_SHARED_CHUNK: tests of the shared queue)
  int32_t grid_cap = 0;  // test: workgroups of a queued launch (DEPPY_GRID_CAP; 0 = resident maximum)
  bool fast_path = true;  // small dp_solve batches on the latency path (DEPPY_FAST_PATH=0: off)
  bool spread = false;    // DEPPY_SPREAD=1: a chunk's later one-wavefront launches on sibling streams
  // Several devices: the chunks of every job wait here, the costliest
  // first, and a device's submitting thread takes the next one whenever it
  // has a free lane (worker_main), so the devices balance dynamically.
  std::mutex sqmu;
  std::deque<Task> sq;
  dp_stats st{};         // the caller-thread paths (resident batches)
  ~dp_ctx() { delete pool; }
};

// A batch resident in HBM (dp_upload): its own buffers per device slice.
struct Slice {
  int d = 0;        // index into ctx->dev
  int ordinal = 0;  // its HIP device
  int32_t p0 = 0, p1 = 0;
  Plan plan;
  InLayout il{};
  OutLayout ol{};
  Buf d_in, d_out, scratch;
  int32_t* trace = nullptr;
  int32_t* trace_len = nullptr;
  int64_t* stamps = nullptr;
  hipStream_t stream = nullptr;  // lane of the last launch
  hipEvent_t k0 = nullptr, k1 = nullptr;
  Spread spread;
};

struct dp_resident {
  int32_t n = 0;
  int32_t trace_cap = 0;
  bool inflight = false;
  std::vector<Slice> slices;
};

namespace {

// The failing call's text, per thread (a device worker reports it to the
// job, an API function to ctx->err through api_fail).
thread_local std::string t_err;
#define HIP_OK(expr)                                                         \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) {                                                  \
      (void)ctx;                                                             \
      t_err = std::string(#expr) + ": " + hipGetErrorString(e_);             \
      return -1;                                                             \
    }                                                                        \
  } while (0)
// The context's last error.  Jobs may be submitted and waited on from any
// number of caller threads, so every write takes err_mu, and dp_last_error
// hands each thread its own copy.
void set_err(dp_ctx* ctx, std::string e) {
  std::lock_guard<std::mutex> lk(ctx->err_mu);
  ctx->err = std::move(e);
}
int api_fail(dp_ctx* ctx) {
  set_err(ctx, t_err);
  return -1;
}
// HIP_OK in an API function on the caller's thread: the text to ctx->err.
#define API_OK(expr)                                                         \
  do {                                                                       \
    if (hipError_t e_ = (expr); e_ != hipSuccess) {                          \
      set_err(ctx, std::string(#expr) + ": " + hipGetErrorString(e_));       \
      return -1;                                                             \
    }                                                                        \
  } while (0)

void add_stats(dp_stats& a, const dp_stats& b) {
  a.problems += b.problems; a.chunks += b.chunks; a.launches += b.launches; a.kernel_ms += b.kernel_ms;
  a.h2d_bytes += b.h2d_bytes; a.d2h_bytes += b.d2h_bytes; a.rec_bytes += b.rec_bytes; a.stage_ms += b.stage_ms;
  a.plan_ms += b.plan_ms; a.wait_ms += b.wait_ms; a.scatter_ms += b.scatter_ms; a.direct_chunks += b.direct_chunks;
  a.bcp_bytes += b.bcp_bytes; a.allocs += b.allocs;
  for (int m = 0; m < 5; ++m) {
    a.placed[m] += b.placed[m];
    a.placed_launches[m] += b.placed_launches[m];
  }
}
void add_device_stats(Device& D, const dp_stats& b) {
  std::lock_guard<std::mutex> lk(D.smu);
  add_stats(D.st, b);
}

// Enqueue a planned chunk's launches on stream s.
// Multi-wave launches take their items from a queue (kernel_api.hpp
// KernelArgs::queue) in the scratch's first words, zeroed here.
int enqueue_launches(dp_ctx* ctx, const Plan& P, const dp::KernelArgs& base, hipStream_t s, dp_stats& st,
                     Spread* sp = nullptr) {
  static const bool no_queue = [] {  // diagnostic DEPPY_NO_QUEUE=1: one workgroup per item
    const char* e = std::getenv("DEPPY_NO_QUEUE");
    return e && *e && *e != '0';
  }();
  if (!P.scratch_off.empty()) HIP_OK(hipMemsetAsync(base.scratch, 0, 4 * dp::kQueueWords, s));
  int nlds = 0;
  for (const auto& L : P.launches) nlds += L.mode == dp::M_LDS;
  const bool spread = sp && sp->n > 0 && nlds > 1;
  if (spread) HIP_OK(hipEventRecord(sp->start, s));
  int q = 0, jl = 0, nf = 0;
  for (const auto& L : P.launches) {
    hipStream_t t = s;
    if (spread && L.mode == dp::M_LDS && jl++ > 0 && nf < kMaxSpread) {
      t = sp->s[(jl - 2) % sp->n];
      HIP_OK(hipStreamWaitEvent(t, sp->start, 0));
    }
    dp::KernelArgs a = base;
    a.items = base.items + L.first;
    if (L.mode != dp::M_LDS) {
      a.scratch_off = base.scratch_off + (L.first - P.big_base);
      a.queue = no_queue ? nullptr : base.scratch + q;
      a.n_items = L.count;
      if (ctx->flags & DP_OPT_TINY_TABLE) a.table_cap = 4;
      a.grid_cap = ctx->grid_cap;
      ++q;
      if (L.dev_lists) HIP_OK(dp::launch_watch_build(a, L.mode, L.count, s));
    }
    HIP_OK(dp::launch_solve(a, L.mode, L.count, L.lds, t));
    if (t != s) {
      HIP_OK(hipEventRecord(sp->fin[nf], t));
      HIP_OK(hipStreamWaitEvent(s, sp->fin[nf], 0));
      ++nf;
    }
    st.launches++;
    st.placed[L.mode] += L.count;
    st.placed_launches[L.mode]++;
  }
  return 0;
}

// The sibling streams of lane stream i (the device's other lane streams).
void set_siblings(const Device& D, int i, Spread& sp, bool on) {
  sp.n = 0;
  if (!on) return;
  for (int j = 1; j < D.nstreams && sp.n < kMaxSpread; ++j) sp.s[sp.n++] = D.lanes[(i + j) % D.nstreams].s;
}

// Wait for a lane's chunk and scatter its results into its job's dp_result
// (the job's bookkeeping is deliver()'s).
int finish_lane(dp_ctx* ctx, Device& D, Lane& L) {
  if (!L.job) return 0;
  dp_job* job = L.job;
  L.job = nullptr;
  dp_stats st{};
  HIP_OK(hipSetDevice(L.device));
  const double t0 = now_ms();
  HIP_OK(hipEventSynchronize(L.done));
  const double t1 = now_ms();
  st.wait_ms += t1 - t0;
  float ms = 0.f;
  if (!L.plan.launches.empty() && hipEventElapsedTime(&ms, L.k0, L.k1) == hipSuccess) {
    st.kernel_ms += ms;
    ctx->last_ms.store(ms);
  }
  const int32_t used = L.zc_out ? 0 : *at<int32_t>(L.h_out.p, L.ol.pool_len);
  const size_t need = L.ol.pool + (size_t)used * 4;
  if (!L.zc_out && need > L.ol.d2h) {  // cores beyond the pipelined window
    HIP_OK(hipMemcpyAsync(L.h_out.p + L.ol.d2h, L.d_out.p + L.ol.d2h, need - L.ol.d2h, hipMemcpyDeviceToHost, L.s));
    HIP_OK(hipStreamSynchronize(L.s));
    st.d2h_bytes += (int64_t)(need - L.ol.d2h);
  }
  add_device_stats(D, st);
  // the results to the caller on the finisher thread, so the worker goes on
  // planning and enqueueing the next chunks (config 2: planning and scatter
  // took 0.15 + 0.17 ms of the worker's 0.45 ms per 10k-catalog chunk)
  {
    std::lock_guard<std::mutex> lk(D.fmu);
    L.fjob = job;
    L.scattering = true;
    D.fq.push_back(&L);
  }
  D.fcv.notify_all();
  return 0;
}

void chunk_done(dp_job* job, int rc);

// Wait until lane L's results are scattered (the worker, before it reuses
// the lane's buffers or plan).
void wait_scatter(Device& D, Lane& L) {
  std::unique_lock<std::mutex> lk(D.fmu);
  D.fcv.wait(lk, [&] { return !L.scattering; });
}

// A device's finisher thread: scatters finished chunks' results into their
// jobs (oldest first) and accounts them.  Exits once stopped and drained.
void finisher_main(dp_ctx* ctx, Device* Dp) {
  Device& D = *Dp;
  std::unique_lock<std::mutex> lk(D.fmu);
  for (;;) {
    if (D.fq.empty()) {
      if (D.fstop) return;
      D.fcv.wait(lk);
      continue;
    }
    Lane* L = D.fq.front();
    D.fq.pop_front();
    lk.unlock();
    dp_stats st{};
    const double t0 = now_ms();
    dp_job* job = L->fjob;
    st.bcp_bytes += (int64_t)scatter(L->plan, L->ol, L->h_out.p, L->p0, &job->res, D.fpool);
    st.scatter_ms += now_ms() - t0;
    add_device_stats(D, st);
    lk.lock();
    L->scattering = false;
    L->fjob = nullptr;
    lk.unlock();
    D.fcv.notify_all();
    chunk_done(job, 0);  // (may free the job: not touched after this)
    lk.lock();
  }
}

// One chunk of `job` is over (delivered, failed or skipped).
void chunk_done(dp_job* job, int rc) {
  std::lock_guard<std::mutex> lk(job->m);
  if (rc && !job->rc) {
    job->rc = rc;
    job->err = t_err;
  }
  if (--job->chunks_left == 0) job->cv.notify_all();
}

// Finish lane L (on its device's worker) and account its chunk to its job.
void deliver(dp_ctx* ctx, Device& D, Lane& L) {
  dp_job* job = L.job;
  if (!job) return;
  auto it = std::find(D.inflight.begin(), D.inflight.end(), &L);
  if (it != D.inflight.end()) D.inflight.erase(it);
  const int rc = finish_lane(ctx, D, L);
  if (rc) chunk_done(job, rc);  // (else the finisher completes the chunk)
}

// Planning storage of `dst` grown to (at least) the sizes `src` uses, with
// its pages touched, so plan_chunk on dst allocates and faults nothing for a
// chunk like src's.
template <class T>
void grow_vec(std::vector<T>& d, size_t n) {
  if (d.capacity() >= n) return;
  const size_t keep = d.size();
  d.resize(n);
  d.resize(keep);
}
void grow_plan(Plan& dst, const Plan& src) {
  grow_vec(dst.img_off, src.img_off.size());
  grow_vec(dst.narrow, src.narrow.size());
  grow_vec(dst.order, src.order.size());
  grow_vec(dst.launches, src.launches.size());
  grow_vec(dst.scratch_off, src.scratch_off.size());
  grow_vec(dst.skip, src.skip.size());
  grow_vec(dst.skip_flags, src.skip_flags.size());
  grow_vec(dst.inst_off, src.inst_off.size());
  grow_vec(dst.dev_off, src.dev_off.size());
  grow_vec(dst.direct, src.direct.size());
  grow_vec(dst.head, src.head.size());
  grow_vec(dst.blk, src.blk.size());
  grow_vec(dst.segcnt, src.segcnt.size());
  grow_vec(dst.segpos, src.segpos.size());
  grow_vec(dst.segxs, src.segxs.size());
  for (int k = 0; k < 5; ++k) grow_vec(dst.big[k], src.big[k].size());
  grow_vec(dst.cnt, src.cnt.capacity());
  grow_vec(dst.tmp, src.tmp.capacity());
}

// Buffer sizes a planned chunk needs on its lane.
struct LaneNeed {
  size_t h_in, d_in, h_out, d_out, scratch;
  bool fits(const Lane& L) const {
    return h_in <= L.h_in.cap && d_in <= L.d_in.cap && h_out <= L.h_out.cap && d_out <= L.d_out.cap &&
           scratch <= L.scratch.cap;
  }
};

int reserve_lane(dp_ctx* ctx, Lane& L, const LaneNeed& n) {
  HIP_OK(L.h_in.reserve(n.h_in));
  HIP_OK(L.d_in.reserve(n.d_in));
  HIP_OK(L.h_out.reserve(n.h_out));
  HIP_OK(L.d_out.reserve(n.d_out));
  HIP_OK(L.scratch.reserve(n.scratch));
  return 0;
}

// Bytes of planning storage a plan holds (a change means plan_chunk allocated).
size_t plan_cap(const Plan& P) {
  size_t c = P.img_off.capacity() + P.inst_off.capacity() + P.dev_off.capacity() + P.scratch_off.capacity() +
             P.narrow.capacity() + P.direct.capacity() + P.order.capacity() + P.launches.capacity() +
             P.skip.capacity() + P.skip_flags.capacity() + P.head.capacity() + P.cnt.capacity() + P.tmp.capacity() +
             P.blk.capacity() + P.segcnt.capacity() + P.segpos.capacity() + P.segxs.capacity();
  for (const auto& b : P.big) c += b.capacity();
  return c;
}

// A chunk that does not fit its lane's buffers grows every lane of the
// device to its sizes (and their planning storage to its plan's), not just
// its own: lanes are taken round-robin, so otherwise each of them would make
// its first allocation on its first chunk, the last ones well into a serving
// loop (or a timed region).  After the first batch of a shape no chunk on the
// device allocates (dp_stats.allocs).  A lane with a chunk in flight is
// finished first, since the GPU may still use its buffers.
int grow_device_lanes(dp_ctx* ctx, Device& D, Lane& L, const LaneNeed& need) {
  if (reserve_lane(ctx, L, need)) return -1;
  for (int li = 0; li < D.nlanes; ++li) {
    Lane& O = D.lanes[li];
    if (&O == &L) continue;
    wait_scatter(D, O);
    grow_plan(O.plan, L.plan);
    grow_vec(O.bad, L.bad.size());
    if (need.fits(O)) continue;
    deliver(ctx, D, O);  // (an error of its chunk goes to that chunk's job)
    wait_scatter(D, O);
    if (reserve_lane(ctx, O, need)) return -1;
  }
  return 0;
}

// Stage and enqueue problems [p0, p0+n) of a job on lane L.
int start_chunk(dp_ctx* ctx, Device& D, Lane& L, dp_job* job, int32_t p0, int32_t n) {
  HIP_OK(hipSetDevice(L.device));
  dp_stats st{};
  const int64_t allocs0 = g_buf_allocs.load(std::memory_order_relaxed);
  const size_t bad_cap = L.bad.capacity(), plan_cap0 = plan_cap(L.plan);
  const double t0 = now_ms();
  // The records' DMA ahead of the plan (the plan adds only the tables after
  // them): a page-locked batch whose first record is in a staged form sends
  // its source range to the image's front at once when it fits the lane and
  // its copy is not one the fill would chain (below), so the copy runs under
  // the planning.  (A chunk that then turns out not to be direct stages its
  // image over it, later on the same stream.)
  static const int64_t chain_mb = env_i64("DEPPY_COPY_CHAIN_MB", 64);
  static const bool early_dma = env_i64("DEPPY_EARLY_DMA", 1) != 0;  // diagnostic A/B
  const int64_t W = job->rec_off[p0 + n] - job->rec_off[p0];
  hipStream_t cs = L.cs ? L.cs : L.s;
  const int32_t f0 = n > 0 && W >= DP_H_SIZE ? job->rec[job->rec_off[p0] + DP_H_FMT] : -1;
  const bool early = early_dma && job->pinned && !ctx->zc_in && W > 0 && (size_t)4 * W <= L.d_in.cap &&
                     (f0 == DP_FMT_U16 || dp_fmt_packed(f0)) &&
                     !(chain_mb > 0 && (size_t)4 * W >= (size_t)chain_mb << 20);
  if (early) HIP_OK(hipMemcpyAsync(L.d_in.p, job->rec + job->rec_off[p0], 4 * (size_t)W, hipMemcpyHostToDevice, cs));
  L.bad.assign((size_t)n, 0);
  std::vector<uint8_t>& bad = L.bad;
  int32_t ldsg_busy = 0;  // M_LDSG problems of the chunks in flight on this device
  for (const Lane* o : D.inflight) ldsg_busy += o->plan.n_ldsg;
  dp::plan_chunk(L.plan, job->rec, job->rec_off, p0, n, ctx->flags, &bad, D.pool, ldsg_busy);
  const double t_plan = now_ms();
  st.plan_ms += t_plan - t0;
  // Direct: records already in their staged form (16-bit, on a 16-byte
  // boundary; dp_lower_into DP_LOWER_NARROW) in page-locked memory are
  // copied to the device from where they lie: the chunk's source range goes
  // by one DMA to the front of the image, each such record at its own
  // offset, and only the other problems' records are staged, after it.
  // (Worth it while the others' source words, copied for nothing, are not
  // the larger part.)
  const bool direct = job->pinned && L.plan.n_direct > 0 && !ctx->zc_in && 2 * L.plan.other_words <= W;
  if (direct) {
    Plan& Q = L.plan;
    int64_t o = W;
    for (int32_t i = 0; i < n; ++i) {
      if (Q.direct[(size_t)i]) {
        Q.dev_off[(size_t)i] = job->rec_off[p0 + i] - job->rec_off[p0];
      } else {
        Q.dev_off[(size_t)i] = o;
        o += Q.img_off[(size_t)i + 1] - Q.img_off[(size_t)i];
      }
    }
    Q.img_words = o;
  }
  const InLayout il = in_layout(L.plan);
  L.ol = out_layout(L.plan);
  // The host side of the input region: all of it, or (direct) only what
  // follows the copied source range -- the staged records and the tables --
  // with `hin` the address the region's offset 0 would have.
  const size_t rest = direct ? il.img + 4 * (size_t)W : 0;
  const LaneNeed need{il.end - rest, il.end, L.ol.end, L.ol.end,
                      (size_t)std::max<int64_t>(L.plan.scratch_words, 1) * 4};
  const char* const d_in0 = L.d_in.p;
  if (!need.fits(L) && grow_device_lanes(ctx, D, L, need)) return -1;
  const bool early_in = early && L.d_in.p == d_in0;  // (a grown lane has a new buffer: copy again)
  char* const hin = L.h_in.p - rest;  // (only offsets >= rest are used)
  const Plan& P = L.plan;
  if (!direct || P.n_direct < n) {  // stage the records (host pool)
    int32_t* img = at<int32_t>(hin, il.img);
    D.pool->run(n, [&](int64_t i) {
      if (direct && P.direct[(size_t)i]) return;
      if (!dp::stage_one(P, job->rec, job->rec_off, p0, (int32_t)i, img, false)) bad[(size_t)i] = 1;
    }, dp::stage_block(n, *D.pool));
    // (records found malformed while staging are reported by the kernel)
  }
  fill_in_tables(P, il, hin);
  st.stage_ms += now_ms() - t_plan;
  // Zero-copy results: the kernels write their results straight into the
  // lane's mapped pinned buffer.  With a D2H copy per chunk instead, copies
  // from every stream queue on the same copy engine: a chunk's H2D waited
  // behind the previous chunk's D2H, which waits for that chunk's kernel, and
  // the lanes ran one after another (config 2: 3.0M res/s with H2D + D2H,
  // 5.9M with zero-copy results; profiles/r02_zero_copy_ab.jsonl).  Records
  // go by H2D copy: once staging got faster, the copy engine (8.4M res/s at
  // 3 jobs in flight) beat kernels reading them over PCIe (6.9M;
  // DEPPY_ZC_IN=1, only for chunks without multi-wave problems, which re-read
  // their record; profiles/r02_h2h_sweep.jsonl).
  const bool zc_in = ctx->zc_in && !direct && P.scratch_off.empty();
  L.zc_out = ctx->zc_out;
  char* din = zc_in ? L.h_in.dev : L.d_in.p;
  char* dout = L.zc_out ? L.h_out.dev : L.d_out.p;
  size_t h2d = 0;
  // (lane buffers are free: finish_lane waited for the lane's last chunk)
  // Filling an idle pipeline with large chunks, copies go in submission
  // order: the first chunks (one per stream) each wait for the previous
  // one's copy instead of sharing PCIe with all of them, so the first
  // kernels start after one chunk's copy rather than after every stream's.
  // Only while filling (the streams are idle, so a copy never waits behind
  // another stream's kernel), and only for chunks of at least
  // DEPPY_COPY_CHAIN_MB (default 64; 0: off): measured on one box, configs 4
  // and 5 (564 / 322 MB chunks) gain 10-11% host to host at 20 steps, while
  // configs 2 and 6 (19 / 10 MB) lose half (profiles/r03_copy_chain_ab_unsized.txt).
  const size_t copy_bytes = direct ? 4 * (size_t)W + (il.end - rest) : zc_in ? 0 : il.end;
  if (D.inflight.empty()) D.fill_left = D.nstreams;
  const bool chain = chain_mb > 0 && D.fill_left > 0 && copy_bytes >= (size_t)chain_mb << 20;
  if (D.fill_left > 0) --D.fill_left;
  if (chain && D.last_copied && hipEventQuery(D.last_copied) == hipErrorNotReady)
    HIP_OK(hipStreamWaitEvent(cs, D.last_copied, 0));
  (void)hipGetLastError();  // (hipEventQuery's not-ready status)
  if (direct) {
    const size_t src_bytes = 4 * (size_t)W;
    if (src_bytes && !early_in)
      HIP_OK(hipMemcpyAsync(L.d_in.p + il.img, job->rec + job->rec_off[p0], src_bytes, hipMemcpyHostToDevice, cs));
    HIP_OK(hipMemcpyAsync(L.d_in.p + rest, L.h_in.p, il.end - rest, hipMemcpyHostToDevice, cs));
    h2d = src_bytes + il.end - rest;
    st.direct_chunks++;
  } else if (!zc_in) {
    HIP_OK(hipMemcpyAsync(L.d_in.p, L.h_in.p, il.end, hipMemcpyHostToDevice, cs));
    h2d = il.end + (early ? 4 * (size_t)W : 0);
  }
  if (cs != L.s || chain) HIP_OK(hipEventRecord(L.copied, cs));
  if (cs != L.s) HIP_OK(hipStreamWaitEvent(L.s, L.copied, 0));
  D.last_copied = chain ? L.copied : nullptr;  // (a chain restarts after an unchained chunk)
  dp::KernelArgs a = kernel_args(il, L.ol, din, dout, reinterpret_cast<int32_t*>(L.scratch.p), ctx->budget);
  static const bool pool_memset = env_i64("DEPPY_POOL_MEMSET", 0) != 0;  // diagnostic: 1 = the fill kernel
  if (!zc_in && L.zc_out && !pool_memset) {
    // the pool's counter in the input region, zeroed by the copy above: one
    // dispatch fewer per chunk (a fill kernel, ~58 us under load in the
    // r05_final kernel traces); host to host measured the same either way
    // (profiles/r05_pool_ab.txt)
    a.core_pool_len = at<int32_t>(din, il.pool_len);
  } else {  // (the host reads the counter back from the output region)
    HIP_OK(hipMemsetAsync(L.d_out.p + L.ol.pool_len, 0, 4, L.s));
    a.core_pool_len = at<int32_t>(L.d_out.p, L.ol.pool_len);
  }
  a.items = at<dp::WorkItem>(din, il.items);
  HIP_OK(hipEventRecord(L.k0, L.s));
  set_siblings(D, (int)(&L - D.lanes) % D.nstreams, L.spread, ctx->spread);
  if (enqueue_launches(ctx, P, a, L.s, st, &L.spread)) return -1;
  HIP_OK(hipEventRecord(L.k1, L.s));
  if (!L.zc_out) HIP_OK(hipMemcpyAsync(L.h_out.p, L.d_out.p, L.ol.d2h, hipMemcpyDeviceToHost, L.s));
  HIP_OK(hipEventRecord(L.done, L.s));
  L.job = job;
  L.p0 = p0;
  st.chunks++;
  st.problems += n;
  st.h2d_bytes += (int64_t)h2d;
  st.d2h_bytes += L.zc_out ? 0 : (int64_t)L.ol.d2h;
  st.rec_bytes += P.rec_bytes;
  st.allocs += g_buf_allocs.load(std::memory_order_relaxed) - allocs0 + (L.bad.capacity() != bad_cap) +
               (plan_cap(L.plan) != plan_cap0);
  add_device_stats(D, st);
  return 0;
}

// The chunk starting at p: up to chunk_problems problems and chunk_bytes
// record bytes (at least one problem).
int32_t next_chunk(const int64_t* rec_off, int32_t p, int32_t P, int32_t chunk_problems, int64_t chunk_bytes) {
  int32_t q = p;
  const int64_t w0 = rec_off[p];
  while (q < P && q - p < chunk_problems && (q == p || (rec_off[q + 1] - w0) * 4 <= chunk_bytes)) ++q;
  return q;
}

// Start task t on the device's next lane (delivering the chunk that lane
// holds first).  A job that already failed skips its later chunks.
void run_task(dp_ctx* ctx, Device& D, const Task& t) {
  dp_job* job = t.job;
  bool failed;
  {
    std::lock_guard<std::mutex> lk(job->m);
    failed = job->rc != 0;
  }
  if (failed) {
    chunk_done(job, 0);
    return;
  }
  Lane& L = D.lanes[D.cursor];
  D.cursor = (D.cursor + 1) % D.nlanes;
  deliver(ctx, D, L);
  wait_scatter(D, L);
  if (start_chunk(ctx, D, L, job, t.p0, t.n)) {
    L.job = nullptr;
    chunk_done(job, -1);
    return;
  }
  D.inflight.push_back(&L);
}

// A device's submitting thread: starts queued chunks on its lanes in order,
// and in between delivers finished chunks, oldest first -- at once when a
// waiter is blocked on their job, else when their `done` event has fired
// (polled every 50 us while chunks are in flight).  Exits once stopped and
// drained.
// The next chunk of the context's shared queue when this device has a free
// lane (its oldest lane delivered), so a busy device leaves the queue's
// chunks to the others.  (Called with D.qmu held: qmu, then sqmu.)
bool take_shared(dp_ctx* ctx, Device& D, Task& t) {
  if ((int)D.inflight.size() >= D.nlanes) return false;
  std::lock_guard<std::mutex> g(ctx->sqmu);
  if (ctx->sq.empty()) return false;
  t = ctx->sq.front();
  ctx->sq.pop_front();
  return true;
}

void worker_main(dp_ctx* ctx, Device* Dp) {
  Device& D = *Dp;
  (void)hipSetDevice(D.ordinal);
  std::unique_lock<std::mutex> lk(D.qmu);
  for (;;) {
    Task t;
    if (!D.q.empty()) {
      t = D.q.front();
      D.q.pop_front();
      lk.unlock();
      run_task(ctx, D, t);
      lk.lock();
      continue;
    }
    if (take_shared(ctx, D, t)) {
      lk.unlock();
      run_task(ctx, D, t);
      lk.lock();
      continue;
    }
    if (!D.inflight.empty()) {
      Lane* o = D.inflight.front();
      const bool now = D.stop || o->job->waiting.load(std::memory_order_acquire) ||
                       hipEventQuery(o->done) != hipErrorNotReady;
      if (now) {
        lk.unlock();
        deliver(ctx, D, *o);
        lk.lock();
      } else {
        D.qcv.wait_for(lk, std::chrono::microseconds(50));
      }
      continue;
    }
    if (D.stop) {
      std::lock_guard<std::mutex> g(ctx->sqmu);
      if (ctx->sq.empty()) return;
      continue;
    }
    D.qcv.wait(lk);
  }
}

// The latency path (FastLane): 0 solved, -1 error (ctx->err), 1 the batch
// needs the pipeline (a multi-wave or malformed problem).
int fast_solve(dp_ctx* ctx, Device& D, const dp_batch* b, dp_result* res) {
  FastLane& F = D.fast;
  std::lock_guard<std::mutex> lk(F.mu);
  const int32_t n = b->n_problems;
  F.bad.assign((size_t)n, 0);
  dp::plan_chunk(F.plan, b->rec, b->rec_off, 0, n, ctx->flags, &F.bad, nullptr);
  const Plan& P = F.plan;
  if (!P.skip.empty() || !P.scratch_off.empty()) return 1;
  if (hipSetDevice(D.ordinal) != hipSuccess) return 1;
  const InLayout il = in_layout(P);
  const OutLayout ol = out_layout(P);
  if (F.h_in.reserve(il.end) != hipSuccess || F.h_out.reserve(ol.end) != hipSuccess) return 1;
  int32_t* img = at<int32_t>(F.h_in.p, il.img);
  for (int32_t i = 0; i < n; ++i)
    if (!dp::stage_one(P, b->rec, b->rec_off, 0, i, img, true)) F.bad[(size_t)i] = 1;
  fill_in_tables(P, il, F.h_in.p);
  *at<int32_t>(F.h_out.p, ol.pool_len) = 0;
  dp::KernelArgs a = kernel_args(il, ol, F.h_in.dev, F.h_out.dev, nullptr, ctx->budget);
  dp_stats st{};
  if (enqueue_launches(ctx, P, a, F.s, st) || hipEventRecord(F.done, F.s) != hipSuccess) return api_fail(ctx);
  // poll: a sleeping wait costs more than the solve of one small catalog
  hipError_t e;
  while ((e = hipEventQuery(F.done)) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) {
    set_err(ctx, std::string("dp_solve (latency path): ") + hipGetErrorString(e));
    return -1;
  }
  scatter(P, ol, F.h_out.p, 0, res);
  return 0;
}

// The chunks of a batch: at most chunk_problems problems and chunk_bytes
// record bytes each, and (several devices) at least one per device.
void cut_chunks(const dp_ctx* ctx, const dp_job* job, std::vector<std::pair<int32_t, int32_t>>& out) {
  const int32_t P = job->n;
  const int nd = (int)ctx->dev.size();
  int32_t cp = ctx->chunk_problems;
  // several devices: about kChunksPerDevice chunks each (but not below
  // kMinSharedChunk problems: a chunk's launches last as long as its slowest
  // catalog, so small chunks are tail-bound), for the shared queue to balance
  if (nd > 1 && P >= nd)
    cp = std::min<int32_t>(cp, std::max<int32_t>((P + kChunksPerDevice * nd - 1) / (kChunksPerDevice * nd),
                                                 std::min<int32_t>(ctx->min_shared_chunk, (P + nd - 1) / nd)));
  for (int32_t p = 0; p < P;) {
    const int32_t q = next_chunk(job->rec_off, p, P, cp, ctx->chunk_bytes);
    out.emplace_back(p, q - p);
    p = q;
  }
}

// Lane streams per device (two lanes each): one per hardware queue the HIP
// runtime opened, at most 8 (16 streams measured far slower host to host,
// and 8 streams on 4 queues 5% slower than 4; profiles/r03_streams_ab.txt).
// HIP opens GPU_MAX_HW_QUEUES queues (4 by default) when it initialises; the
// binding (deppy_amd/_lib.py, the cgo shim) raises the setting before that
// and reports in DEPPY_HW_QUEUES how many HIP actually runs with -- which
// differs from the setting when something initialised HIP first.  Without
// the binding the setting is the best guess.  DEPPY_STREAMS overrides (A/B).
int lane_streams() {
  // DEPPY_HW_QUEUES = "q@s": q queues, valid while GPU_MAX_HW_QUEUES still
  // reads s (a child process that inherited it with another setting uses its own)
  int64_t hwq = env_i64("GPU_MAX_HW_QUEUES", kStreams);
  if (const char* e = std::getenv("DEPPY_HW_QUEUES")) {
    const char* at = std::strchr(e, '@');
    const char* g = std::getenv("GPU_MAX_HW_QUEUES");
    if (!at || std::strcmp(at + 1, g ? g : "") == 0) hwq = std::atoll(e);
  }
  return (int)std::min<int64_t>(kMaxStreams,
                                std::max<int64_t>(1, env_i64("DEPPY_STREAMS", std::min<int64_t>(hwq, 8))));
}

}  // namespace

namespace dp {
int ctx_first_ordinal(const dp_ctx* ctx) { return ctx && !ctx->dev.empty() ? ctx->dev[0].ordinal : -1; }
}  // namespace dp

extern "C" {

dp_ctx* dp_create(const dp_opts* opts) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    dp::set_global_error(std::string("dp_create: no HIP device (") + hipGetErrorString(e) + ")");
    return nullptr;
  }
  int first = opts ? opts->first_device : 0;
  int cnt = opts && opts->n_devices > 0 ? opts->n_devices : n - first;
  // (test) every logical device on first_device's GPU
  const bool share = opts && (opts->flags & DP_OPT_SHARE_ORDINAL) && opts->n_devices > 0;
  if (first < 0 || cnt <= 0 || (share ? first >= n || cnt > 8 : first + cnt > n)) {
    dp::set_global_error("dp_create: device range out of bounds");
    return nullptr;
  }
  auto* ctx = new dp_ctx;
  for (int i = 0; i < cnt; ++i) ctx->dev.emplace_back();
  for (int i = 0; i < cnt; ++i) {
    const int d = share ? first : first + i;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      dp::set_global_error(std::string("dp_create: device ") + std::to_string(d) + " is not gfx950 (" +
                           prop.gcnArchName + ")");
      dp_destroy(ctx);
      return nullptr;
    }
    if (hipSetDevice(d) != hipSuccess || dp::configure_solve_kernel(kMaxLdsBytes) != hipSuccess) {
      dp::set_global_error("dp_create: cannot configure the solve kernel");
      dp_destroy(ctx);
      return nullptr;
    }
    Device& D = ctx->dev[(size_t)i];
    D.ordinal = d;
    ctx->copy_streams = env_i64("DEPPY_COPY_STREAM", 0) != 0;
    D.nstreams = lane_streams();
    D.nlanes = 2 * D.nstreams;
    for (int li = 0; li < D.nlanes; ++li) {
      Lane& L = D.lanes[li];
      L.device = d;
      if (li >= D.nstreams) {  // lane li shares the streams of lane li % nstreams
        L.s = D.lanes[li % D.nstreams].s;
        L.cs = D.lanes[li % D.nstreams].cs;
      }
      if ((li < D.nstreams && (hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking) != hipSuccess ||
                             (ctx->copy_streams && hipStreamCreateWithFlags(&L.cs, hipStreamNonBlocking) != hipSuccess))) ||
          hipEventCreateWithFlags(&L.copied, hipEventDisableTiming) != hipSuccess ||
          hipEventCreate(&L.k0) != hipSuccess || hipEventCreate(&L.k1) != hipSuccess ||
          hipEventCreateWithFlags(&L.done, hipEventDisableTiming) != hipSuccess || L.spread.create() != 0) {
        dp::set_global_error("dp_create: cannot create streams");
        dp_destroy(ctx);
        return nullptr;
      }
    }
  }
  if (opts && opts->step_budget > 0) ctx->budget = opts->step_budget;
  if (opts) ctx->flags = opts->flags;
  ctx->chunk_problems = (int32_t)std::max<int64_t>(1, env_i64("DEPPY_CHUNK_PROBLEMS", kChunkProblems));
  ctx->chunk_bytes = std::max<int64_t>(1, env_i64("DEPPY_CHUNK_BYTES", kChunkBytes));
  ctx->min_shared_chunk = (int32_t)std::max<int64_t>(1, env_i64("DEPPY_MIN_SHARED_CHUNK", kMinSharedChunk));
  ctx->zc_in = env_i64("DEPPY_ZC_IN", 0) != 0;   // diagnostic: 1 = kernels read staged records over PCIe
  ctx->zc_out = env_i64("DEPPY_ZC_OUT", 1) != 0; // diagnostic: 0 = D2H copy of every chunk
  ctx->direct = env_i64("DEPPY_DIRECT", 1) != 0; // diagnostic: 0 = stage every chunk
  ctx->grid_cap = (int32_t)std::max<int64_t>(0, env_i64("DEPPY_GRID_CAP", 0));
  ctx->fast_path = env_i64("DEPPY_FAST_PATH", 1) != 0;
  ctx->spread = env_i64("DEPPY_SPREAD", 0) != 0;
  const int ht = dp::host_threads();
  ctx->pool = new dp::Pool(ht);
  const int per = std::max(2, ht / cnt);
  for (auto& D : ctx->dev) {
    if (hipSetDevice(D.ordinal) != hipSuccess || hipStreamCreateWithFlags(&D.fast.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&D.fast.done, hipEventDisableTiming) != hipSuccess) {
      dp::set_global_error("dp_create: cannot create the latency stream");
      dp_destroy(ctx);
      return nullptr;
    }
    D.own_pool = cnt > 1;
    D.pool = D.own_pool ? new dp::Pool(per) : ctx->pool;
    // the finisher's scatter on threads of its own: on the worker's pool it
    // held the pool's run lock while the worker waited to plan the next
    // chunk's headers (config 6: planning 0.27 -> 0.44 ms per 10k chunk)
    D.fpool = new dp::Pool(std::max(2, std::min(4, per / 4)));
    D.worker = std::thread(worker_main, ctx, &D);
    D.finisher = std::thread(finisher_main, ctx, &D);
  }
  return ctx;
}

void dp_destroy(dp_ctx* ctx) {
  if (!ctx) return;
  for (auto& D : ctx->dev) {  // the workers drain their queues and lanes, then exit
    if (!D.worker.joinable()) continue;
    {
      std::lock_guard<std::mutex> lk(D.qmu);
      D.stop = true;
    }
    D.qcv.notify_all();
    D.worker.join();
    if (D.finisher.joinable()) {  // (the worker handed it every chunk it delivered)
      {
        std::lock_guard<std::mutex> lk(D.fmu);
        D.fstop = true;
      }
      D.fcv.notify_all();
      D.finisher.join();
    }
    delete D.fpool;
    D.fpool = nullptr;
    if (D.own_pool) delete D.pool;
    D.pool = nullptr;
  }
  for (auto& D : ctx->dev) {
    (void)hipSetDevice(D.ordinal);
    if (D.fast.s) (void)hipStreamSynchronize(D.fast.s);
    D.fast.h_in.release();
    D.fast.h_out.release();
    if (D.fast.done) (void)hipEventDestroy(D.fast.done);
    if (D.fast.s) (void)hipStreamDestroy(D.fast.s);
  }
  for (auto& D : ctx->dev) {
    (void)hipSetDevice(D.ordinal);
    for (int li = 0; li < D.nstreams; ++li)
      if (D.lanes[li].s) (void)hipStreamSynchronize(D.lanes[li].s);
    for (int li = 0; li < D.nlanes; ++li) {
      Lane& L = D.lanes[li];
      for (Buf* b : {&L.h_in, &L.d_in, &L.h_out, &L.d_out, &L.scratch}) b->release();
      if (L.k0) (void)hipEventDestroy(L.k0);
      if (L.k1) (void)hipEventDestroy(L.k1);
      if (L.done) (void)hipEventDestroy(L.done);
      if (L.copied) (void)hipEventDestroy(L.copied);
      L.spread.destroy();
    }
    for (int li = 0; li < D.nstreams; ++li) {  // (lanes li + nstreams... share these)
      if (D.lanes[li].s) (void)hipStreamDestroy(D.lanes[li].s);
      if (D.lanes[li].cs) (void)hipStreamDestroy(D.lanes[li].cs);
    }
  }
  delete ctx;
}

const char* dp_last_error(const dp_ctx* ctx) {
  if (!ctx) return dp_last_global_error();
  static thread_local std::string copy;  // valid until this thread's next call
  std::lock_guard<std::mutex> lk(ctx->err_mu);
  copy = ctx->err;
  return copy.c_str();
}
int32_t dp_num_devices(const dp_ctx* ctx) { return ctx ? (int32_t)ctx->dev.size() : 0; }
int32_t dp_lanes(const dp_ctx* ctx) { return ctx && !ctx->dev.empty() ? (int32_t)ctx->dev[0].nlanes : 0; }
void* dp_host_alloc(int64_t bytes) { return bytes > 0 ? dp::pinned_alloc((size_t)bytes) : nullptr; }
void dp_host_free(void* p) {
  if (p) dp::pinned_free(p);
}

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

int dp_device_bytes(const dp_batch* b, int32_t opt_flags, int64_t* rec_bytes, int64_t* img_bytes) {
  if (!b || (b->n_problems > 0 && (!b->rec || !b->rec_off))) return -1;
  Plan P;
  dp::plan_chunk(P, b->rec, b->rec_off, 0, b->n_problems, opt_flags, nullptr);
  if (rec_bytes) *rec_bytes = P.rec_bytes;
  if (img_bytes) *img_bytes = 4 * P.img_words;
  return 0;
}

int dp_plan_order(const dp_batch* b, int32_t opt_flags, int32_t* order, int32_t* launch_first) {
  if (!b || !order || b->n_problems < 0 || (b->n_problems > 0 && (!b->rec || !b->rec_off))) return -1;
  static thread_local Plan P;
  dp::plan_chunk(P, b->rec, b->rec_off, 0, b->n_problems, opt_flags, nullptr, &dp::host_pool());
  std::copy(P.order.begin(), P.order.end(), order);
  if (launch_first)
    for (size_t k = 0; k < P.launches.size(); ++k) launch_first[k] = P.launches[k].first;
  return (int)P.launches.size();
}

int dp_plan_placements(const dp_batch* b, int32_t opt_flags, int8_t* place) {
  if (!b || !place || b->n_problems < 0 || (b->n_problems > 0 && (!b->rec || !b->rec_off))) return -1;
  static thread_local Plan P;  // (reused, as a lane's: no allocation once grown)
  dp::plan_chunk(P, b->rec, b->rec_off, 0, b->n_problems, opt_flags, nullptr, &dp::host_pool());
  for (int32_t i = 0; i < b->n_problems; ++i) place[i] = (int8_t)P.head[(size_t)i].place;
  return 0;
}

// ---- host-to-host pipeline ----

int dp_submit(dp_ctx* ctx, const dp_batch* b, dp_result* res, dp_job** out) {
  if (!ctx || !b || !res || !out || b->n_problems < 0 || (b->n_problems > 0 && (!b->rec || !b->rec_off)))
    return -1;
  auto* job = new dp_job;
  job->n = b->n_problems;
  job->rec = b->rec;
  job->rec_off = b->rec_off;
  job->pinned = ctx->direct && job->n > 0 && pinned_range(b->rec, 4 * (size_t)b->rec_off[job->n]);
  job->res = *res;
  std::vector<std::pair<int32_t, int32_t>> chunks;
  cut_chunks(ctx, job, chunks);
  job->chunks_left = (int)chunks.size();
  const int nd = (int)ctx->dev.size();
  if (nd == 1) {
    Device& D = ctx->dev[0];
    {
      std::lock_guard<std::mutex> lk(D.qmu);
      for (const auto& c : chunks) D.q.push_back(Task{job, c.first, c.second});
    }
    D.qcv.notify_one();
    *out = job;
    return 0;
  }
  // several devices: the shared queue, costliest chunk first (record words,
  // the cost the plan can see before solving), pulled by whichever device
  // has a lane free (worker_main take_shared)
  std::stable_sort(chunks.begin(), chunks.end(), [&](const auto& x, const auto& y) {
    return b->rec_off[x.first + x.second] - b->rec_off[x.first] > b->rec_off[y.first + y.second] - b->rec_off[y.first];
  });
  {
    std::lock_guard<std::mutex> g(ctx->sqmu);
    for (const auto& c : chunks) ctx->sq.push_back(Task{job, c.first, c.second});
  }
  for (auto& D : ctx->dev) {  // (taking qmu orders the wake-up after a worker's check)
    { std::lock_guard<std::mutex> lk(D.qmu); }
    D.qcv.notify_one();
  }
  *out = job;
  return 0;
}

int dp_job_wait(dp_ctx* ctx, dp_job* job) {
  if (!ctx || !job) return -1;
  job->waiting.store(true, std::memory_order_release);
  for (auto& D : ctx->dev) {  // workers deliver the job's chunks as soon as they are done
    std::lock_guard<std::mutex> lk(D.qmu);
    D.qcv.notify_all();
  }
  int rc;
  {
    std::unique_lock<std::mutex> lk(job->m);
    job->cv.wait(lk, [&] { return job->chunks_left == 0; });
    rc = job->rc;
  }
  if (rc) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    set_err(ctx, job->err);
  }
  delete job;
  return rc;
}

int dp_solve(dp_ctx* ctx, const dp_batch* b, dp_result* res) {
  if (!ctx || !b || !res || b->n_problems < 0 || (b->n_problems > 0 && (!b->rec || !b->rec_off))) return -1;
  if (b->n_problems > 0 && b->n_problems <= kFastProblems && b->rec_off[b->n_problems] <= kFastWords &&
      ctx->fast_path) {
    const int r = fast_solve(ctx, ctx->dev[0], b, res);
    if (r <= 0) return r;  // (1: not for the latency path)
  }
  dp_job* job = nullptr;
  if (dp_submit(ctx, b, res, &job)) return -1;
  return dp_job_wait(ctx, job);
}

int dp_get_device_stats(dp_ctx* ctx, int32_t device, dp_stats* out, int32_t reset) {
  if (!ctx || !out || device < 0 || device >= (int32_t)ctx->dev.size()) return -1;
  Device& D = ctx->dev[(size_t)device];
  std::lock_guard<std::mutex> dl(D.smu);
  *out = D.st;
  if (reset) D.st = dp_stats{};
  return 0;
}

int dp_get_stats(dp_ctx* ctx, dp_stats* out, int32_t reset) {
  if (!ctx || !out) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  *out = ctx->st;
  if (reset) ctx->st = dp_stats{};
  for (auto& D : ctx->dev) {
    std::lock_guard<std::mutex> dl(D.smu);
    add_stats(*out, D.st);
    if (reset) D.st = dp_stats{};
  }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device-resident batches (dp_upload / dp_launch / dp_wait / dp_download)
// ---------------------------------------------------------------------------
namespace {

void free_slice(Slice& s) {
  (void)hipSetDevice(s.ordinal);
  for (Buf* b : {&s.d_in, &s.d_out, &s.scratch}) b->release();
  for (void* p : {(void*)s.trace, (void*)s.trace_len, (void*)s.stamps})
    if (p) (void)hipFree(p);
  if (s.k0) (void)hipEventDestroy(s.k0);
  if (s.k1) (void)hipEventDestroy(s.k1);
  s.spread.destroy();
  s = Slice{};
}

int build_slice(dp_ctx* ctx, Slice& s, const dp_batch* b, int32_t trace_cap) {
  HIP_OK(hipSetDevice(s.ordinal));
  HIP_OK(hipEventCreate(&s.k0));
  HIP_OK(hipEventCreate(&s.k1));
  if (s.spread.create()) HIP_OK(hipErrorOutOfMemory);
  const int32_t n = s.p1 - s.p0;
  std::vector<uint8_t> bad((size_t)std::max(n, 1), 0);
  dp::plan_chunk(s.plan, b->rec, b->rec_off, s.p0, n, ctx->flags, &bad, ctx->pool);
  s.il = in_layout(s.plan);
  s.ol = out_layout(s.plan);
  std::vector<char> host(s.il.end);
  int32_t* img = reinterpret_cast<int32_t*>(host.data() + s.il.img);
  const Plan& P = s.plan;
  ctx->pool->run(n, [&](int64_t i) {
    if (!dp::stage_one(P, b->rec, b->rec_off, s.p0, (int32_t)i, img, false)) bad[(size_t)i] = 1;
  }, dp::stage_block(n, *ctx->pool));
  fill_in_tables(P, s.il, host.data());
  s.d_in.host = s.d_out.host = s.scratch.host = false;
  HIP_OK(s.d_in.reserve(s.il.end));
  HIP_OK(s.d_out.reserve(s.ol.end));
  HIP_OK(s.scratch.reserve((size_t)std::max<int64_t>(P.scratch_words, 1) * 4));
  HIP_OK(hipMemcpy(s.d_in.p, host.data(), s.il.end, hipMemcpyHostToDevice));
  if (trace_cap > 0) {
    HIP_OK(hipMalloc(&s.trace, std::max<size_t>((size_t)n, 1) * (size_t)trace_cap * 4));
    HIP_OK(hipMalloc(&s.trace_len, std::max<size_t>((size_t)n, 1) * 4));
    HIP_OK(hipMemset(s.trace_len, 0, std::max<size_t>((size_t)n, 1) * 4));
  }
#ifdef DP_STAMPS
  HIP_OK(hipMalloc(&s.stamps, std::max<size_t>((size_t)n, 1) * dp::DP_NSTAMP * 8));
  HIP_OK(hipMemset(s.stamps, 0, std::max<size_t>((size_t)n, 1) * dp::DP_NSTAMP * 8));
#endif
  return 0;
}

int launch_slice(dp_ctx* ctx, Slice& s, int32_t trace_cap) {
  Device& D = ctx->dev[(size_t)s.d];
  HIP_OK(hipSetDevice(D.ordinal));
  s.stream = D.lanes[D.next].s;
  set_siblings(D, D.next % D.nstreams, s.spread, ctx->spread);
  D.next = (D.next + 1) % D.nlanes;
  HIP_OK(hipMemsetAsync(s.d_out.p + s.ol.pool_len, 0, 4, s.stream));
  dp::KernelArgs a = kernel_args(s.il, s.ol, s.d_in.p, s.d_out.p, reinterpret_cast<int32_t*>(s.scratch.p),
                                 ctx->budget);
  a.items = at<dp::WorkItem>(s.d_in.p, s.il.items);
  a.stamps = s.stamps;
  a.trace = s.trace;
  a.trace_len = s.trace_len;
  a.trace_cap = trace_cap;
  HIP_OK(hipEventRecord(s.k0, s.stream));
  if (enqueue_launches(ctx, s.plan, a, s.stream, ctx->st, &s.spread)) return -1;
  HIP_OK(hipEventRecord(s.k1, s.stream));
  return 0;
}

int wait_locked(dp_ctx* ctx, dp_resident* r) {
  if (!r->inflight) return 0;
  r->inflight = false;
  double mx = 0.0;
  for (auto& s : r->slices) {
    HIP_OK(hipSetDevice(ctx->dev[(size_t)s.d].ordinal));
    HIP_OK(hipEventSynchronize(s.k1));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s.k0, s.k1) == hipSuccess) mx = std::max(mx, (double)ms);
  }
  ctx->last_ms.store(mx);
  return 0;
}

int launch_locked(dp_ctx* ctx, dp_resident* r) {
  if (r->inflight && wait_locked(ctx, r)) return -1;
  for (auto& s : r->slices)
    if (launch_slice(ctx, s, r->trace_cap)) return -1;
  r->inflight = true;
  return 0;
}

}  // namespace

namespace dp {
// Contiguous slices of a batch, one per device, balanced by record words (a
// proxy of solve cost): slice d is [cut[d], cut[d+1]).
void partition_by_words(const int64_t* rec_off, int32_t P, int nd, std::vector<int32_t>& cut) {
  cut.assign((size_t)nd + 1, P);
  cut[0] = 0;
  const int64_t total = P ? rec_off[P] - rec_off[0] : 0;
  int32_t p = 0;
  for (int d = 0; d < nd; ++d) {
    cut[(size_t)d] = p;
    const int64_t target = rec_off[0] + total * (d + 1) / nd;
    while (p < P && (d == nd - 1 || rec_off[p + 1] <= target)) ++p;
  }
  cut[(size_t)nd] = P;
}
}  // namespace dp

extern "C" {

int dp_upload(dp_ctx* ctx, const dp_batch* b, dp_resident** out) { return dp_upload_traced(ctx, b, 0, out); }

int dp_upload_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_resident** out) {
  if (!ctx || !b || !out || trace_cap < 0 || b->n_problems < 0) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto* r = new dp_resident;
  r->n = b->n_problems;
  r->trace_cap = trace_cap;
  std::vector<int32_t> cut;
  dp::partition_by_words(b->rec_off, b->n_problems, (int)ctx->dev.size(), cut);
  for (size_t d = 0; d < ctx->dev.size(); ++d) {
    Slice s;
    s.d = (int)d;
    s.ordinal = ctx->dev[d].ordinal;
    s.p0 = cut[d];
    s.p1 = cut[d + 1];
    r->slices.push_back(std::move(s));
  }
  for (auto& s : r->slices)
    if (build_slice(ctx, s, b, trace_cap)) {
      for (auto& x : r->slices) free_slice(x);
      delete r;
      return api_fail(ctx);
    }
  *out = r;
  return 0;
}

int dp_launch(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return launch_locked(ctx, r) ? api_fail(ctx) : 0;
}

int dp_wait(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return wait_locked(ctx, r) ? api_fail(ctx) : 0;
}

int dp_run(dp_ctx* ctx, dp_resident* r) {
  if (!ctx || !r) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (launch_locked(ctx, r)) return api_fail(ctx);
  return wait_locked(ctx, r) ? api_fail(ctx) : 0;
}

int dp_download(dp_ctx* ctx, dp_resident* r, dp_result* res) {
  if (!ctx || !r || !res) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (wait_locked(ctx, r)) return api_fail(ctx);
  for (auto& s : r->slices) {
    if (s.p1 == s.p0) continue;
    API_OK(hipSetDevice(ctx->dev[(size_t)s.d].ordinal));
    std::vector<char> host(s.ol.end);
    API_OK(hipMemcpy(host.data(), s.d_out.p, s.ol.end, hipMemcpyDeviceToHost));
    scatter(s.plan, s.ol, host.data(), s.p0, res);
  }
  return 0;
}

int dp_download_trace(dp_ctx* ctx, dp_resident* r, int32_t* trace, int32_t* trace_len) {
  if (!ctx || !r || !trace || !trace_len) return -1;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (wait_locked(ctx, r)) return api_fail(ctx);
  if (r->trace_cap <= 0) {
    set_err(ctx, "dp_download_trace: the batch was not uploaded with dp_upload_traced");
    return -1;
  }
  for (auto& s : r->slices) {
    const int32_t n = s.p1 - s.p0;
    if (n == 0) continue;
    API_OK(hipSetDevice(ctx->dev[(size_t)s.d].ordinal));
    API_OK(hipMemcpy(trace_len + s.p0, s.trace_len, (size_t)n * 4, hipMemcpyDeviceToHost));
    API_OK(hipMemcpy(trace + (int64_t)r->trace_cap * s.p0, s.trace, (size_t)n * r->trace_cap * 4,
                     hipMemcpyDeviceToHost));
  }
  return 0;
}

void dp_resident_free(dp_ctx* ctx, dp_resident* r) {
  if (!r) return;
  if (ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (r->inflight) (void)wait_locked(ctx, r);
    for (auto& s : r->slices) free_slice(s);
  }
  delete r;
}

int dp_solve_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_result* res, int32_t* trace,
                    int32_t* trace_len) {
  dp_resident* r = nullptr;
  if (dp_upload_traced(ctx, b, trace_cap, &r)) return -1;
  int rc = dp_run(ctx, r);
  if (!rc) rc = dp_download(ctx, r, res);
  if (!rc) rc = dp_download_trace(ctx, r, trace, trace_len);
  dp_resident_free(ctx, r);
  return rc;
}

#ifdef DP_STAMPS
// Diagnostic builds only: per-problem phase cycles [init, base, search,
// epilogue, core] of the last run (not part of include/deppy_hip.h).
int dp_debug_stamps(dp_ctx* ctx, dp_resident* r, int64_t* out) {
  for (auto& s : r->slices) {
    API_OK(hipSetDevice(ctx->dev[(size_t)s.d].ordinal));
    API_OK(hipMemcpy(out + dp::DP_NSTAMP * (size_t)s.p0, s.stamps, (size_t)(s.p1 - s.p0) * dp::DP_NSTAMP * 8,
                     hipMemcpyDeviceToHost));
  }
  return 0;
}
#endif

int dp_last_kernel_ms(const dp_ctx* ctx, double* ms) {
  if (!ctx || !ms) return -1;
  *ms = ctx->last_ms.load();
  return 0;
}

// ---- host-only test hooks (include/deppy_hip.h) ----

static dp::Pool& hook_pool() { return dp::host_pool(); }

int dp_stage_roundtrip(const dp_batch* b, int32_t opt_flags, int32_t chunk_problems, int64_t chunk_bytes,
                       int32_t* out_rec, int32_t* chunk_first, int32_t cap) {
  if (!b || b->n_problems < 0) return -1;
  if (chunk_problems <= 0) chunk_problems = kChunkProblems;
  if (chunk_bytes <= 0) chunk_bytes = kChunkBytes;
  const int32_t P = b->n_problems;
  int32_t nchunks = 0;
  Plan plan;
  static std::vector<int32_t> staged, wide;  // (test hook: one caller at a time)
  for (int32_t p = 0; p < P;) {
    const int32_t q = next_chunk(b->rec_off, p, P, chunk_problems, chunk_bytes);
    if (chunk_first && nchunks < cap) chunk_first[nchunks] = p;
    ++nchunks;
    std::vector<uint8_t> bad((size_t)(q - p), 0);
    dp::plan_chunk(plan, b->rec, b->rec_off, p, q - p, opt_flags, &bad, &hook_pool());
    if (staged.size() < (size_t)plan.img_off[(size_t)plan.n] + 1) staged.resize((size_t)plan.img_off[(size_t)plan.n] + 1);
    hook_pool().run(q - p, [&](int64_t i) {
      if (!dp::stage_one(plan, b->rec, b->rec_off, p, (int32_t)i, staged.data(), false)) bad[(size_t)i] = 1;
    }, dp::stage_block(q - p, hook_pool()));
    for (auto x : bad)
      if (x) return -1;
    for (int32_t i = 0; out_rec && i < q - p; ++i) {  // out_rec NULL: staging only (timing)
      // the staged copy back in the source record's own form
      const int32_t* src = b->rec + b->rec_off[p + i];
      const int32_t* st = staged.data() + plan.img_off[(size_t)i];
      int32_t* o = out_rec + b->rec_off[p + i];
      const int64_t words = src[DP_H_WORDS];
      wide.resize((size_t)words);
      std::memcpy(wide.data(), st, 4 * DP_H_SIZE);
      if (dp_fmt_packed(src[DP_H_FMT])) {  // staged as it is (one-wavefront), else not shown
        if (dp_fmt_packed(st[DP_H_FMT])) std::memcpy(o, st, 4 * (size_t)dp_rec_phys_words(src));
        continue;
      }
      if (st[DP_H_FMT] == DP_FMT_U16 || st[DP_H_FMT] == dp::DP_FMT_U16_CHECKED) {
        const uint16_t* u = reinterpret_cast<const uint16_t*>(st + DP_H_SIZE);
        for (int64_t j = DP_H_SIZE; j < words; ++j) wide[(size_t)j] = u[j - DP_H_SIZE];
      } else {
        std::memcpy(wide.data() + DP_H_SIZE, st + DP_H_SIZE, 4 * (size_t)(words - DP_H_SIZE));
      }
      std::memcpy(o, wide.data(), 4 * DP_H_SIZE);
      o[DP_H_FMT] = src[DP_H_FMT];
      if (src[DP_H_FMT] == DP_FMT_U16) {
        uint16_t* u = reinterpret_cast<uint16_t*>(o + DP_H_SIZE);
        for (int64_t j = DP_H_SIZE; j < words; ++j) u[j - DP_H_SIZE] = (uint16_t)wide[(size_t)j];
      } else {
        std::memcpy(o + DP_H_SIZE, wide.data() + DP_H_SIZE, 4 * (size_t)(words - DP_H_SIZE));
      }
    }
    p = q;
  }
  return nchunks;
}

int dp_stitch_selftest(const dp_batch* b, int32_t chunk_problems, dp_result* res) {
  if (!b || !res || b->n_problems < 0) return -1;
  if (chunk_problems <= 0) chunk_problems = kChunkProblems;
  const int32_t P = b->n_problems;
  int32_t nchunks = 0;
  Plan plan;
  std::vector<char> out;
  for (int32_t p = 0; p < P; ++nchunks) {
    const int32_t q = next_chunk(b->rec_off, p, P, chunk_problems, kChunkBytes);
    dp::plan_chunk(plan, b->rec, b->rec_off, p, q - p, 0, nullptr);
    const OutLayout ol = out_layout(plan);
    out.assign(ol.end, 0);
    int32_t pool_len = 0;
    for (int32_t i = q - p - 1; i >= 0; --i) {  // pool claims in reverse problem order
      const int64_t g = p + i;
      const int32_t* h = b->rec + b->rec_off[g];
      const int32_t nid = h[DP_H_NID];
      const bool unsat = g % 3 == 0 && nid > 0;
      dp::ProblemOut& po = at<dp::ProblemOut>(out.data(), ol.prob)[i];
      po.status = (int8_t)(unsat ? DP_UNSAT : DP_SAT);
      po.flags = (int32_t)(g & 0xff);
      po.steps = 7 * g;
      uint32_t* inst = at<uint32_t>(out.data(), ol.installed) + plan.inst_off[(size_t)i];
      for (int64_t w = 0; w < plan.inst_off[(size_t)i + 1] - plan.inst_off[(size_t)i]; ++w)
        inst[w] = (uint32_t)(g * 2654435761u) ^ (uint32_t)w;
      const int32_t len = unsat ? std::min<int32_t>(nid, 1 + (int32_t)(g % 4)) : 0;
      po.core_len = len;
      po.core_at = pool_len;
      for (int32_t j = 0; j < len; ++j) at<int32_t>(out.data(), ol.pool)[pool_len + j] = (int32_t)((g + j) % nid);
      pool_len += len;
    }
    *at<int32_t>(out.data(), ol.pool_len) = pool_len;
    scatter(plan, ol, out.data(), p, res);
    p = q;
  }
  return nchunks;
}

int dp_partition(const int64_t* rec_off, int32_t n_problems, int32_t nd, int32_t* cut) {
  if (!rec_off || !cut || nd <= 0 || n_problems < 0) return -1;
  std::vector<int32_t> c;
  dp::partition_by_words(rec_off, n_problems, nd, c);
  std::copy(c.begin(), c.end(), cut);
  return 0;
}

}  // extern "C"
