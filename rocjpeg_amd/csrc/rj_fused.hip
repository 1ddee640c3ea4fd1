// rj_fused.hip -- K2 fused output kernel (placeholder until the fast path lands).
#include "rj_kernels.h"
namespace rj {
hipError_t LaunchFusedOutput(hipStream_t, const RjImageDev *, int, const uint32_t *, uint32_t, const int16_t *,
                             const RjTableSet *) {
  return hipErrorNotSupported;
}
}  // namespace rj
