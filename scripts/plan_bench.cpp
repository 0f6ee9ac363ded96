// Host-side planning cost of dp_submit (runtime.cpp plan_chunk) per problem,
// on a given number of pool threads: the header pass alone, and the whole
// plan.  Build: scripts/build_plan_bench.sh; run: plan_bench CONFIG N REPS THREADS
#include "../deppy_amd/csrc/runtime.cpp"
#include <chrono>
int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const int cfg = atoi(argv[1]), n = atoi(argv[2]), reps = atoi(argv[3]), nt = atoi(argv[4]);
  dp_gen* g = dp_gen_catalogs(cfg, n, 1000);
  dp_lowered* lw = dp_lowered_new();
  dp_lower_into(dp_gen_wire(g), DP_LOWER_NARROW, lw);
  const int64_t* ro = dp_lowered_rec_off(lw);
  const int32_t* rec = dp_lowered_rec(lw);
  dp::Pool pool(nt);
  auto secs = [](auto t0) { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  std::vector<dp::Head> hd((size_t)n);
  auto rd = [&](int64_t i) { dp::read_head(hd[(size_t)i], rec + ro[i], ro[i + 1] - ro[i], 0, true); };
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) pool.run(n, std::function<void(int64_t)>(rd), 64);
  const double th = secs(t0);
  Plan P;
  std::vector<uint8_t> bad((size_t)n);
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) dp::plan_chunk(P, rec, ro, 0, n, 0, &bad, &pool);
  const double tp = secs(t0);
  printf("{\"config\": %d, \"problems\": %d, \"threads\": %d, \"header_ns\": %.1f, \"plan_ns\": %.1f, \"launches\": %zu}\n",
         cfg, n, nt, th / reps / n * 1e9, tp / reps / n * 1e9, P.launches.size());
  dp_lowered_free(lw);
  dp_gen_free(g);
}
