// Batched actor-critic MLP forward (policy_forward) and GAE (rollout_gae) on gfx950.
// The per-tile policy math lives in policy_device.h and is shared with the fused rollout
// (policy_rollout.hip), so both paths produce the same bits for the same observations.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "fenv.h"
#include "fenv_internal.h"
#include "policy_device.h"

namespace fenvk {

// Persistent workgroups of 4 waves share one LDS weight image; each wave walks 32-agent tiles.
__global__ __launch_bounds__(256) void k_policy(const float *__restrict__ params, int32_t D,
                                               const float *__restrict__ obs, int64_t B,
                                               int64_t row0,
                                               float *__restrict__ mu_out,
                                               float *__restrict__ value_out,
                                               float *__restrict__ act_out,
                                               float *__restrict__ logp_out,
                                               float *__restrict__ clip_out, uint64_t seed,
                                               uint64_t offset, int32_t deterministic) {
    __shared__ __attribute__((aligned(16))) float lds[kPolicyLds];
    stage_policy_weights(lds, params, D, threadIdx.x, blockDim.x);
    __syncthreads();

    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int waves_per_block = blockDim.x >> 6;
    const int64_t ntiles = (B + 31) / 32;
    const bool value_only = !mu_out && !act_out && !logp_out && !clip_out;
    for (int64_t tile = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6); tile < ntiles;
         tile += (int64_t)gridDim.x * waves_per_block) {
        asm volatile("" ::: "memory");  // no hoisting of the LDS weight image into registers
        const int64_t row = tile * 32 + j;
        const bool valid = row < B;
        float o[8];
#pragma unroll
        for (int col = 0; col < 8; ++col) o[col] = (valid && col < D) ? obs[row * D + col] : 0.0f;
        const uint2 nb = deterministic ? make_uint2(0u, 0u) : policy_noise_bits(row0 + row, seed, offset);
        const PolicyLane r = policy_tile(lds, obs_operand(o, h), lane, nb, deterministic != 0,
                                         value_only);
        if (valid) {
            if (mu_out) mu_out[row * 2 + h] = r.mu;
            if (act_out) act_out[row * 2 + h] = r.act;
            if (clip_out) clip_out[row * 2 + h] = r.clip;
            if (h == 0) {
                if (value_out) value_out[row] = r.value;
                if (logp_out) logp_out[row] = r.logp;
            }
        }
    }
}

hipError_t launch_policy_forward(const float *params, int32_t D, const float *obs, int64_t B,
                                 int64_t row0, float *mu, float *value, float *action, float *logp,
                                 float *clipped, uint64_t seed, uint64_t offset,
                                 int32_t deterministic, hipStream_t st) {
    // Persistent grid sized to exactly the resident workgroups (no partial second round).
    static int resident = 0;
    if (resident == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_policy, 256, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus < 1)
            cus = 256;
        resident = per_cu * cus;
    }
    const int64_t tiles = (B + 31) / 32;
    int64_t blocks = (tiles + 3) / 4;
    if (blocks > resident) {
        // equalise tiles per wave over the resident grid
        const int64_t rounds = (blocks + resident - 1) / resident;
        blocks = (tiles + 4 * rounds - 1) / (4 * rounds);
        if (blocks > resident) blocks = resident;
    }
    hipLaunchKernelGGL(k_policy, dim3((unsigned)blocks), dim3(256), 0, st, params, D, obs, B, row0,
                       mu, value, action, logp, clipped, seed, offset, deterministic);
    return hipGetLastError();
}

// SB3 RolloutBuffer.compute_returns_and_advantage (GAE(lambda)), one lane per env column,
// backwards over the T steps of the [T][A] buffers.  Elementwise/HBM-bound: per agent-step
// reads reward, value, episode_start (4+4+1 B) and writes advantage, return (8 B).
__global__ __launch_bounds__(256) void k_gae(const float *__restrict__ rew,
                                             const float *__restrict__ values,
                                             const uint8_t *__restrict__ episode_starts,
                                             const float *__restrict__ last_values,
                                             const uint8_t *__restrict__ last_dones, int32_t T,
                                             int64_t A, float gamma, float lam,
                                             float *__restrict__ adv, float *__restrict__ ret) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= A) return;
    float last = 0.0f;
    float next_v = last_values[a];
    float next_nt = 1.0f - (float)last_dones[a];
    for (int32_t k = T - 1; k >= 0; --k) {
        const int64_t r = (int64_t)k * A + a;
        const float v = values[r];
        last = gae_step(rew[r], v, next_v, next_nt, gamma, lam, last);
        adv[r] = last;
        ret[r] = last + v;
        next_v = v;
        next_nt = 1.0f - (float)episode_starts[r];
    }
}

hipError_t launch_gae(const float *rew, const float *values, const uint8_t *episode_starts,
                      const float *last_values, const uint8_t *last_dones, int32_t T, int64_t A,
                      float gamma, float lam, float *adv, float *ret, hipStream_t st) {
    hipLaunchKernelGGL(k_gae, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, st, rew, values,
                       episode_starts, last_values, last_dones, T, A, gamma, lam, adv, ret);
    return hipGetLastError();
}

}  // namespace fenvk
