// stencil_k7.hip -- stencil_kernel instantiated for K = 7 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k7(const StencilLaunch& L, hipStream_t st) {
  return launch_k<7>(L, st);
}
}  // namespace kcep
