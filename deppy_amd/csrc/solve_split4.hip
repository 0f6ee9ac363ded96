// M_SPLIT4 instantiation of the solve kernel (solve_kernel.hpp): the M_SPLIT
// layout run by MID_WAVES wavefronts per problem.
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_SPLIT4, 2, launch_split4)
}  // namespace dp
