// stencil_k8.hip -- stencil_kernel instantiated for K = 8 (see stencil_kernel.h)
#include "stencil_kernel.h"

namespace kcep {
hipError_t stencil_count_k8(const StencilLaunch& L, hipStream_t st) {
  return launch_k<8>(L, st);
}
}  // namespace kcep
