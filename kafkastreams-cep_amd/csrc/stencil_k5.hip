// stencil_k5.hip -- stencil_kernel instantiated for K = 5 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k5(const StencilLaunch& L, hipStream_t st) {
  return launch_k<5>(L, st);
}
}  // namespace kcep
