// stencil_k6.hip -- stencil_kernel instantiated for K = 6 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k6(const StencilLaunch& L, hipStream_t st) {
  return launch_k<6>(L, st);
}
}  // namespace kcep
