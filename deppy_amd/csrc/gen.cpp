// Synthetic operator catalogs emitted in the wire format.
// Bench / test tooling: the reference's BenchmarkInput (pkg/sat/bench_test.go:10-64)
// depends on Go's math/rand stream and cannot be regenerated, so the build owns
// this generator.  Deterministic: problem i uses SplitMix64(base_seed + i).
//
// Per problem: P packages, package q has n_q ~ U{1..9} versions; one bundle
// variable per (package, version), listed package-major, newest first.
//   * with p = 0.4 a bundle gets 1-3 Dependency rows, each on a random package
//     of higher index, candidates = a random contiguous version range, newest
//     first (a DAG, so chains form);
//   * with p = 0.05 one Conflict on a random bundle of another package;
//   * one uniqueness variable per package: AtMost(1, all its versions);
//   * R ~ U{1..4} required variables: Mandatory + Dependency(all versions of a
//     random package, newest first).
// Input order: bundles, uniqueness variables, required variables.
// config 2: P = 40;  config 3: P ~ U{4..12};  config 5: P ~ U{4..400} and half
// the problems get an injected infeasibility (half BCP-level, half search-level);
// config 4 (OLM-scale): P = 5000, n_q ~ U{5..15} (V ~ 55k), Dependency targets
// only in packages (q, q+8] (deep chains), R = 50.
// config 6: the shape of the reference's own benchmark input, BenchmarkInput
// (pkg/sat/bench_test.go:10-64): 256 variables "0".."255", each with p = 0.1
// Mandatory, with p = 0.15 one Dependency on 1-5 random other variables, with
// p = 0.05 1-2 Conflicts with random other variables, in that constraint
// order (the draws come from SplitMix64, not Go's math/rand, so the problems
// are of the same distribution, not the same problems).
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

namespace {

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  int64_t uniform(int64_t lo, int64_t hi) {  // inclusive
    return lo + (int64_t)(next() % (uint64_t)(hi - lo + 1));
  }
  bool bernoulli(double p) { return (double)(next() >> 11) * (1.0 / 9007199254740992.0) < p; }
};

struct Builder {
  std::vector<int64_t> prob_var_off{0}, var_id, var_con_off{0}, con_arg_off{0}, con_arg, str_off{0};
  std::vector<int32_t> con_kind, con_n;
  std::vector<char> bytes;
  std::unordered_map<std::string, int64_t> intern;

  int64_t s(const std::string& x) {
    auto it = intern.find(x);
    if (it != intern.end()) return it->second;
    int64_t id = (int64_t)str_off.size() - 1;
    bytes.insert(bytes.end(), x.begin(), x.end());
    str_off.push_back((int64_t)bytes.size());
    intern.emplace(x, id);
    return id;
  }
  void var(const std::string& id) {
    var_id.push_back(s(id));
    var_con_off.push_back(var_con_off.back());
  }
  void con(int32_t kind, int32_t n, const std::vector<std::string>& args) {
    con_kind.push_back(kind);
    con_n.push_back(n);
    for (auto& a : args) con_arg.push_back(s(a));
    con_arg_off.push_back((int64_t)con_arg.size());
    var_con_off.back() += 1;
  }
  void end_problem() { prob_var_off.push_back((int64_t)var_id.size()); }
};

std::string bname(int q, int v) { return "p" + std::to_string(q) + "-v" + std::to_string(v); }

// bench_test.go:10-64 (BenchmarkInput), distribution for distribution.
void gen_bench_input(Builder& B, uint64_t seed) {
  SplitMix64 r(seed);
  constexpr int length = 256, nDependency = 6, nConflict = 3;
  auto other = [&](int i) {
    int y = i;
    while (y == i) y = (int)r.uniform(0, length - 1);
    return std::to_string(y);
  };
  for (int i = 0; i < length; ++i) {
    B.var(std::to_string(i));
    if (r.bernoulli(0.1)) B.con(DP_MANDATORY, 0, {});
    if (r.bernoulli(0.15)) {
      const int n = (int)r.uniform(0, nDependency - 2) + 1;  // rand.Intn(nDependency-1) + 1
      std::vector<std::string> d;
      for (int x = 0; x < n; ++x) d.push_back(other(i));
      B.con(DP_DEPENDENCY, 0, d);
    }
    if (r.bernoulli(0.05)) {
      const int n = (int)r.uniform(0, nConflict - 2) + 1;  // rand.Intn(nConflict-1) + 1
      for (int x = 0; x < n; ++x) B.con(DP_CONFLICT, 0, {other(i)});
    }
  }
  B.end_problem();
}

void gen_problem(Builder& B, int config, uint64_t seed) {
  if (config == 6) {
    gen_bench_input(B, seed);
    return;
  }
  SplitMix64 r(seed);
  int P = config == 2 ? 40 : config == 3 ? (int)r.uniform(4, 12) : config == 4 ? 5000 : (int)r.uniform(4, 400);
  const int vlo = config == 4 ? 5 : 1, vhi = config == 4 ? 15 : 9;
  std::vector<int> nver((size_t)P);
  for (int q = 0; q < P; ++q) nver[(size_t)q] = (int)r.uniform(vlo, vhi);
  // injected infeasibility (config 5): 0 none, 1 BCP-level, 2 search-level
  int inject = 0, ia = -1, ic = -1;
  if (config == 5 && r.bernoulli(0.5)) {
    inject = r.bernoulli(0.5) ? 1 : 2;
    // pick packages with >= 2 versions (ic > ia for the two-hop form)
    for (int t = 0; t < 64 && (ia < 0 || ic < 0); ++t) {
      int a = (int)r.uniform(0, P - 1), c = (int)r.uniform(0, P - 1);
      if (nver[(size_t)a] < 2 || nver[(size_t)c] < 2) continue;
      if (inject == 1) { ia = ic = a; break; }
      if (a < c) { ia = a; ic = c; }
    }
    if (ia < 0 || ic < 0) {  // force a shape
      nver[0] = std::max(nver[0], 2);
      nver[(size_t)P - 1] = std::max(nver[(size_t)P - 1], 2);
      ia = 0;
      ic = inject == 1 ? 0 : P - 1;
    }
  }
  const int khalf = ic >= 0 ? nver[(size_t)ic] / 2 : 0;  // C versions [0, khalf) vs [khalf, n)
  for (int q = 0; q < P; ++q) {
    for (int v = nver[(size_t)q] - 1; v >= 0; --v) {
      B.var(bname(q, v));
      if (inject == 2 && q == ia) {
        // every A version requires C in the lower half (newest first)
        std::vector<std::string> ids;
        for (int x = khalf - 1; x >= 0; --x) ids.push_back(bname(ic, x));
        B.con(DP_DEPENDENCY, 0, ids);
      }
      if (r.bernoulli(0.4)) {
        int nd = (int)r.uniform(1, 3);
        for (int d = 0; d < nd; ++d) {
          if (q == P - 1) break;
          int t = (int)r.uniform(q + 1, config == 4 ? std::min(q + 8, P - 1) : P - 1);
          int lo = (int)r.uniform(0, nver[(size_t)t] - 1);
          int hi = (int)r.uniform(lo, nver[(size_t)t] - 1);
          std::vector<std::string> ids;
          for (int x = hi; x >= lo; --x) ids.push_back(bname(t, x));
          B.con(DP_DEPENDENCY, 0, ids);
        }
      }
      if (P > 1 && r.bernoulli(0.05)) {
        int t = (int)r.uniform(0, P - 2);
        if (t >= q) ++t;
        B.con(DP_CONFLICT, 0, {bname(t, (int)r.uniform(0, nver[(size_t)t] - 1))});
      }
    }
  }
  for (int q = 0; q < P; ++q) {
    B.var("u" + std::to_string(q));
    std::vector<std::string> ids;
    for (int v = nver[(size_t)q] - 1; v >= 0; --v) ids.push_back(bname(q, v));
    B.con(DP_ATMOST, 1, ids);
  }
  int R = config == 4 ? 50 : (int)r.uniform(1, 4);
  for (int i = 0; i < R; ++i) {
    B.var("r" + std::to_string(i));
    B.con(DP_MANDATORY, 0, {});
    int t = (int)r.uniform(0, P - 1);
    std::vector<std::string> ids;
    for (int v = nver[(size_t)t] - 1; v >= 0; --v) ids.push_back(bname(t, v));
    B.con(DP_DEPENDENCY, 0, ids);
  }
  if (inject == 1) {  // two required variables pinning different single versions of one package
    int v1 = (int)r.uniform(0, nver[(size_t)ia] - 1);
    int v2 = (int)r.uniform(0, nver[(size_t)ia] - 2);
    if (v2 >= v1) ++v2;
    B.var("x0");
    B.con(DP_MANDATORY, 0, {});
    B.con(DP_DEPENDENCY, 0, {bname(ia, v1)});
    B.var("x1");
    B.con(DP_MANDATORY, 0, {});
    B.con(DP_DEPENDENCY, 0, {bname(ia, v2)});
  } else if (inject == 2) {  // required A (any version) and C from the upper half
    B.var("x0");
    B.con(DP_MANDATORY, 0, {});
    std::vector<std::string> a, c;
    for (int v = nver[(size_t)ia] - 1; v >= 0; --v) a.push_back(bname(ia, v));
    B.con(DP_DEPENDENCY, 0, a);
    B.var("x1");
    B.con(DP_MANDATORY, 0, {});
    for (int v = nver[(size_t)ic] - 1; v >= khalf; --v) c.push_back(bname(ic, v));
    B.con(DP_DEPENDENCY, 0, c);
  }
  B.end_problem();
}

}  // namespace

struct dp_gen {
  Builder b;
  dp_wire w;
};

extern "C" {

dp_gen* dp_gen_catalogs(int32_t config, int32_t n_problems, uint64_t base_seed) {
  if (config < 2 || config > 6) {
    dp::set_global_error("dp_gen_catalogs: config must be 2, 3, 4, 5 or 6");
    return nullptr;
  }
  if (n_problems < 0) return nullptr;
  auto* g = new dp_gen;
  for (int32_t i = 0; i < n_problems; ++i) gen_problem(g->b, config, base_seed + (uint64_t)i);
  Builder& B = g->b;
  B.intern.clear();
  dp_wire& w = g->w;
  std::memset(&w, 0, sizeof w);
  w.n_problems = n_problems;
  w.prob_var_off = B.prob_var_off.data();
  w.var_id = B.var_id.data();
  w.var_con_off = B.var_con_off.data();
  w.con_kind = B.con_kind.data();
  w.con_n = B.con_n.data();
  w.con_arg_off = B.con_arg_off.data();
  w.con_arg = B.con_arg.data();
  w.n_strs = (int64_t)B.str_off.size() - 1;
  w.str_off = B.str_off.data();
  w.str_bytes = B.bytes.data();
  w.interned = 1;
  return g;
}

const dp_wire* dp_gen_wire(const dp_gen* g) { return &g->w; }
void dp_gen_free(dp_gen* g) { delete g; }

}  // extern "C"
