// M_LDS instantiation of the solve kernel (solve_kernel.hpp).
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_LDS, launch_lds)
}  // namespace dp
