// w4 GEMM instantiations: k-major A and B (dW).
#include "gemm_w4.h"

namespace ftw4 {

void launch_dw(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st) {
  launch_l<true, true>(st_, nj, p, epi, st);
}

}  // namespace ftw4
