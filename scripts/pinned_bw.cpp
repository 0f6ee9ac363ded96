// Host memcpy bandwidth into pinned buffers of different hipHostMalloc flags
// (one thread), and into pageable memory: which mapping the staging writes.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
int main() {
  const size_t n = 64 << 20;
  std::vector<char> src(n, 1), dstp(n, 0);
  struct { const char* name; unsigned flags; } v[] = {
      {"default", hipHostMallocDefault},
      {"portable|mapped", hipHostMallocPortable | hipHostMallocMapped},
      {"portable|mapped|coherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent},
      {"portable|mapped|noncoherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocNonCoherent},
      {"writecombined", hipHostMallocWriteCombined | hipHostMallocMapped}};
  auto bw = [&](char* dst) {
    memcpy(dst, src.data(), n);
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 5; ++r) memcpy(dst, src.data(), n);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 5.0 * n / s / 1e9;
  };
  printf("pageable: %.1f GB/s\n", bw(dstp.data()));
  for (auto& x : v) {
    char* p = nullptr;
    if (hipHostMalloc((void**)&p, n, x.flags) != hipSuccess) { printf("%s: alloc failed\n", x.name); continue; }
    printf("%s: write %.1f GB/s", x.name, bw(p));
    auto t0 = std::chrono::steady_clock::now();
    volatile long acc = 0;
    for (size_t i = 0; i < n; i += 64) acc += p[i];
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf(", read %.1f GB/s\n", n / s / 1e9);
    hipHostFree(p);
  }
}
