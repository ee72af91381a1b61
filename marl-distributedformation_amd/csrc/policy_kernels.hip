// Batched actor-critic MLP forward (SB3 MlpPolicy default for a Box action space; call site
// /root/reference/vectorized_env.py:126, /root/reference/visualize_policy.py:16).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "fenv.h"
#include "fenv_internal.h"

namespace fenvk {

hipError_t launch_policy_forward(const float *, int32_t, const float *, int64_t, float *, float *,
                                 float *, float *, float *, uint64_t, uint64_t, int32_t,
                                 hipStream_t) {
    return hipErrorNotSupported;
}

}  // namespace fenvk
