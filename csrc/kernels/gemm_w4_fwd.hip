// w4 GEMM instantiations: K-contiguous A and B (forward).
#include "gemm_w4.h"

namespace ftw4 {

void launch_fwd(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st) {
  launch_l<false, false>(st_, nj, p, epi, st);
}

}  // namespace ftw4
