// M_SPLIT instantiation of the solve kernel (solve_kernel.hpp).
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_SPLIT, 2, launch_split)
}  // namespace dp
