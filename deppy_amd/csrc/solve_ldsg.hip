// M_LDSG instantiation of the solve kernel (solve_kernel.hpp): the M_LDS image
// and working set, all in LDS, run by LDSG_WAVES wavefronts per problem.
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_LDSG, 1, launch_ldsg)
}  // namespace dp
