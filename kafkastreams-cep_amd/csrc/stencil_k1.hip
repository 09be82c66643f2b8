// stencil_k1.hip -- stencil_kernel instantiated for K = 1 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k1(const StencilLaunch& L, hipStream_t st) {
  return launch_k<1>(L, st);
}
}  // namespace kcep
