// M_LDS instantiation of the solve kernel (solve_kernel.hpp) capped at
// DP_LDS_MIN_WAVES waves per SIMD: for small footprints, where LDS would let
// more problems share a CU than the unbounded build's registers allow.
// Clause rows evaluated two literals per step (the unbounded build: four),
// and the BCP counter left out (Group::NO_VIS).
#define DP_EVAL_UNROLL 2
#include "solve_kernel.hpp"

namespace dp {
DP_DEFINE_MODE(M_LDS, DP_LDS_MIN_WAVES, launch_lds_dense)
}  // namespace dp
