// M_LDS instantiation of the solve kernel (solve_kernel.hpp), unbounded
// registers: for footprints that LDS limits to <= 12 problems per CU.
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_LDS, 1, launch_lds)
}  // namespace dp
