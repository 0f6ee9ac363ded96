// M_HBM instantiation of the solve kernel (solve_kernel.hpp).
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_HBM, 2, launch_hbm)
}  // namespace dp
