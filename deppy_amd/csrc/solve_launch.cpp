// Mode dispatch of the solve kernel launches (kernel_api.hpp).
#include <cstdlib>

#include "kernel_api.hpp"
#include "layout.hpp"

namespace dp {

hipError_t launch_lds(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_lds_dense(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_split(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_split4(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_hbm(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_ldsg(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_lds_configure(int);
hipError_t launch_lds_dense_configure(int);
hipError_t launch_split_configure(int);
hipError_t launch_split4_configure(int);
hipError_t launch_hbm_configure(int);
hipError_t launch_ldsg_configure(int);

// The unbounded one-wavefront build runs 4 waves per SIMD (105 VGPRs, 16 per
// CU).  A launch whose footprint lets LDS hold more problems than that per
// CU takes the register-capped build (5 per SIMD, 20 per CU; 94 VGPRs);
// larger footprints are LDS-bound (solve_kernel.hpp DP_LDS_MIN_WAVES).
constexpr int kUnboundedWavesPerCU = 16;
constexpr int kLdsPerCU = 160 * 1024;

hipError_t launch_solve(const KernelArgs& a, int mode, int n_blocks, int lds_bytes, hipStream_t stream) {
  if (mode == M_LDS) {
    static const bool no_dense = [] {  // diagnostic DEPPY_NO_DENSE=1: the unbounded build only
      const char* e = std::getenv("DEPPY_NO_DENSE");
      return e && *e && *e != '0';
    }();
    const bool dense = !no_dense && lds_bytes > 0 && kLdsPerCU / lds_bytes > kUnboundedWavesPerCU;
    return dense ? launch_lds_dense(a, n_blocks, lds_bytes, stream) : launch_lds(a, n_blocks, lds_bytes, stream);
  }
  if (mode == M_SPLIT) return launch_split(a, n_blocks, lds_bytes, stream);
  if (mode == M_SPLIT4) return launch_split4(a, n_blocks, lds_bytes, stream);
  if (mode == M_LDSG) return launch_ldsg(a, n_blocks, lds_bytes, stream);
  return launch_hbm(a, n_blocks, lds_bytes, stream);
}

hipError_t configure_solve_kernel(int max_lds_bytes) {
  hipError_t e = launch_lds_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_lds_dense_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_split_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_split4_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_hbm_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_ldsg_configure(max_lds_bytes);
  return e;
}

}  // namespace dp
