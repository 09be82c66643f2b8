// stencil_k2.hip -- stencil_kernel instantiated for K = 2 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k2(const StencilLaunch& L, hipStream_t st) {
  return launch_k<2>(L, st);
}
}  // namespace kcep
