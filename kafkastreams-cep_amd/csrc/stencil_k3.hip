// stencil_k3.hip -- stencil_kernel instantiated for K = 3 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k3(const StencilLaunch& L, hipStream_t st) {
  if (L.chain) return launch_k<3, true>(L, st);
  return launch_k<3>(L, st);
}
}  // namespace kcep
