// Host <-> kernel interface of the solve kernel (solve_kernel.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dp {

// diagnostic stamps per problem: 5 phase cycles, 5 counters, wall-clock
// start/end, then the first failed index check (code, value, bound) and the
// number of failed checks, then 3 more counters (Solve, pop_guess, pushes)
constexpr int DP_NSTAMP = 56;

// A problem's fixed-size results, written by one lane as two 16-byte stores:
// one transaction per problem whether the output region is device memory or
// mapped host memory (zero-copy results cross PCIe as written).
struct alignas(32) ProblemOut {
  int8_t status;
  int8_t pad[3];
  int32_t flags;
  int32_t core_len;  // identities at core[core_at ...]
  int32_t core_at;
  int64_t steps;
  uint64_t bcp;      // BCP-visited bytes
};
static_assert(sizeof(ProblemOut) == 32, "two 16-byte stores");

// What one workgroup needs to find its problem: one 16-byte read, in launch
// order, so consecutive workgroups read consecutive items.
struct alignas(16) WorkItem {
  int64_t rec_off;   // word offset of the record in the image
  int32_t inst_off;  // word offset of its installed bitmap
  int32_t pid;       // local problem index (results, traces)
};
static_assert(sizeof(WorkItem) == 16, "one 16-byte read");

struct KernelArgs {
  const int32_t* rec;      // staged records (layout.hpp), each 16-byte aligned
  const WorkItem* items;   // [grid] the workgroup's problem (launch order)
  ProblemOut* out;         // [n] per-problem results (one 32-byte store each)
  uint32_t* installed;
  // NotSatisfiable explanations: problem p's core_len[p] identities are at
  // core[core_at[p]...], claimed from *core_pool_len (the pool holds the sum
  // of the problems' identity counts, so it cannot overflow)
  int32_t* core;
  int32_t* core_pool_len;
  int64_t budget;
  // HBM scratch of the multi-wave modes (M_SPLIT / M_HBM, problems over the
  // LDS limit): workgroup b works in scratch + scratch_off[b] (and in LDS)
  int32_t* scratch;
  const int64_t* scratch_off;
  // diagnostic builds only (-DDP_STAMPS): per-problem phase cycle counts
  int64_t* stamps;
  // search trace (Tracer, search.go:173); null: not traced.  trace_cap words
  // per problem, indexed by problem like status
  int32_t* trace;
  int32_t* trace_len;
  int32_t trace_cap;
  // Multi-wave launches run a persistent grid (as many workgroups as the
  // device holds at once): each workgroup takes the next item from *queue
  // (zeroed before the launch) until n_items are taken, so the longest
  // catalogs (first, in LPT order) never wait behind a dispatch order.
  // nullptr: one workgroup per item.
  int32_t* queue;
  int32_t n_items;
  // test (DP_OPT_TINY_TABLE): round tables of this many slots (0: the layout's)
  int32_t table_cap;
  // test (DEPPY_GRID_CAP): a queued launch starts at most this many
  // workgroups (0: as many as the device holds), so each takes several items
  int32_t grid_cap;
};
// Words at the front of the multi-wave scratch holding the launches' queues.
constexpr int kQueueWords = 64;

// Launch one workgroup per problem of order[0..n_blocks) with lds_bytes of
// LDS: one wavefront (mode M_LDS) or a multi-wave workgroup (M_LDSG, M_SPLIT4,
// M_SPLIT, M_HBM; layout.hpp mode_waves).
hipError_t launch_solve(const KernelArgs& a, int mode, int n_blocks, int lds_bytes, hipStream_t stream);
// Before a multi-wave launch (mode M_SPLIT / M_SPLIT4 / M_HBM) of n_items
// items: the watch lists of its DP_FMT_I32 records above DEV_WATCH_VARS
// variables into their scratch (watch_build.hip).  Other items are skipped.
hipError_t launch_watch_build(const KernelArgs& a, int mode, int n_items, hipStream_t stream);
// Raise the kernel's dynamic-LDS limit to the device maximum.
hipError_t configure_solve_kernel(int max_lds_bytes);

}  // namespace dp
