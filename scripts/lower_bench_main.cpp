// Standalone host-lowering benchmark (scripts/lower_ab.sh): dp_lower_into of a
// generated batch, best of R calls, microseconds per catalog.  Built with
//   hipcc -O3 -std=c++17 -Iinclude deppy_amd/csrc/lower.cpp deppy_amd/csrc/gen.cpp scripts/lower_bench_main.cpp
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include "deppy_hip.h"
namespace dp { void* pinned_alloc(size_t b) { return nullptr; } void pinned_free(void* p) {} }
int main(int argc, char** argv) {
  int cfg = argc > 1 ? atoi(argv[1]) : 2, n = argc > 2 ? atoi(argv[2]) : 10000, reps = argc > 3 ? atoi(argv[3]) : 10;
  dp_gen* g = dp_gen_catalogs(cfg, n, 1000);
  dp_wire w = *dp_gen_wire(g);
  dp_lowered* lw = dp_lowered_new();
  double best = 1e9;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    dp_lower_into(&w, DP_LOWER_NARROW | DP_LOWER_PACKED, lw);
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt < best) best = dt;
  }
  printf("config %d: %.3f us/catalog (best of %d), exact %ld\n", cfg, best / n * 1e6, reps, (long)dp_lowered_exact_count(lw));
}
