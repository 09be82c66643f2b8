// stencil_k4.hip -- stencil_kernel instantiated for K = 4 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k4(const StencilLaunch& L, hipStream_t st) {
  if (L.chain) return launch_k<4, true>(L, st);
  return launch_k<4>(L, st);
}
}  // namespace kcep
