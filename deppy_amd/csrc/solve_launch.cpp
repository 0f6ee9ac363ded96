// Mode dispatch of the solve kernel launches (kernel_api.hpp).
#include "kernel_api.hpp"
#include "layout.hpp"

namespace dp {

hipError_t launch_lds(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_split(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_hbm(const KernelArgs&, int, int, hipStream_t);
hipError_t launch_lds_configure(int);
hipError_t launch_split_configure(int);
hipError_t launch_hbm_configure(int);

hipError_t launch_solve(const KernelArgs& a, int mode, int n_blocks, int lds_bytes, hipStream_t stream) {
  if (mode == M_LDS) return launch_lds(a, n_blocks, lds_bytes, stream);
  if (mode == M_SPLIT) return launch_split(a, n_blocks, lds_bytes, stream);
  return launch_hbm(a, n_blocks, lds_bytes, stream);
}

hipError_t configure_solve_kernel(int max_lds_bytes) {
  hipError_t e = launch_lds_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_split_configure(max_lds_bytes);
  if (e == hipSuccess) e = launch_hbm_configure(max_lds_bytes);
  return e;
}

}  // namespace dp
