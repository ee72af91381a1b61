// Fused PPO rollout collection on gfx950: per step, the policy forward on the MFMA cores ->
// Gaussian sample -> clip -> formation-env step -> next observation, T steps in one launch,
// then the value of the final observation.
//
// Reference: SB3 OnPolicyAlgorithm.collect_rollouts + RolloutBuffer as driven by
// PPO('MlpPolicy', env, n_steps=10, ...) (/root/reference/vectorized_env.py:126-134) over
// FormationEnv.step (vectorized_env.py:68-82) -> FormationSimulator.step (simulate.py:70-118).
// Bit-identical to the unfused path (policy_forward + fenv_step per step, then rollout_gae):
// the policy math is policy_device.h, the env math env_device.h, GAE gae_step.
//
// Mapping.  A wavefront owns fpw = 64/N whole formations (M = fpw*N <= 64 agents, lane = agent)
// for all T steps, exactly as k_rollout_wave; its agents are two 32-agent MFMA tiles.  Per step
// the observation rows are staged in the wave's private 2 KiB LDS slice (coalesced store to
// observations[k] and the MFMA B operands come from the same slice), the policy outputs are
// staged in the same slice (coalesced stores of mu/action/clipped/value/log_prob, and the lane
// that owns agent l picks up its clipped action), then the env step runs on registers.
// 4 waves per workgroup share one 42.8 KB weight image (50.8 KB of LDS with the stage slices:
// 3 workgroups per CU).  A wave in its MFMA phase raises its issue priority
// (s_setprio) so the VALU/LDS work of the other waves fills around it.  Measured against 8-wave
// workgroups with and without the priority (build_variants, tools/gpu_policy.sh): 4 waves +
// priority is +9 % at F = 65,536 x 10 and +2 % at F = 262,144 x 10.
// GAE runs as one short HBM-bound launch after it (k_gae: 17 B per agent-step, ~2 % of the
// rollout; holding T rewards and values in registers would cost the occupancy).
//
// Work: 18,816 fp32-equivalent FLOP per agent-step (+9,344 per agent for the last value) as
// split-f16 MFMAs (policy_device.h), plus ~256 tanh per agent-step on the VALU;
// HBM output is ~78 B per agent-step, an order of magnitude below the MFMA time.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <atomic>

#ifndef FENV_POLICY_PRIO
#define FENV_POLICY_PRIO 1
#endif
#include "env_device.h"
#include "policy_device.h"

namespace fenvk {

#ifndef FENV_PR_WAVES
#define FENV_PR_WAVES 4
#endif
constexpr int kPRWaves = FENV_PR_WAVES;
// LDS (50.8 KB per 4-wave workgroup) allows 3 workgroups = 3 waves per SIMD, so the register
// budget is 168 VGPRs; the compiler is told so (at a 128 budget it spills)
#ifndef FENV_PR_OCCUPANCY
#define FENV_PR_OCCUPANCY __attribute__((amdgpu_waves_per_eu(3)))
#endif
constexpr size_t kPRLdsBytes = (size_t)(kPolicyLds + kPRWaves * 512) * sizeof(float);
static_assert(kPolicyLds % 4 == 0, "stage slices must stay 16-byte aligned");

// The layer-1 MFMA B operands of the wave's two tiles from the staged observation rows.
template <int D>
__device__ __forceinline__ void tile_operands(const float *stage, int j, int h, h8 (&bo)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        float o[8];
#pragma unroll
        for (int col = 0; col < 8; ++col) o[col] = col < D ? stage[(32 * t + j) * D + col] : 0.0f;
        bo[t] = obs_operand(o, h);
    }
}

// One wave-unit: the fpw whole formations starting at formation f_first, all T steps (the body
// of the persistent loop below).
template <int D, int MODE>
__device__ __forceinline__ void policy_rollout_unit(const Consts &c, const DevState &st,
                                                    const DevPending &p, const PRArgs &g,
                                                    const float *wimg, float *stage,
                                                    int64_t f_first) {
    const int lane = threadIdx.x & 63;
    const int N = c.N;
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = f_first + fi;
    const bool active = fi < c.fpw && f < c.F;
    const int64_t a = f * N + i;
    const WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    const int64_t f_left = c.F - f_first;
    const int M = (int)((f_left < c.fpw ? f_left : c.fpw) * N);
    const int64_t a_first = f_first * N;
    const int64_t A = c.F * (int64_t)N;
    const fenv_rollout_bufs &b = g.b;
    const bool det = g.deterministic != 0;

    Agent s{0.f, 0.f, 0.f, 0.f, 0, 0u};
    uint32_t start = 0;  // episode_start of the current step (SB3: previous step's done)
    if (active) {
        s.px = st.px[a];
        s.py = st.py[a];
        s.gx = st.gx[f];
        s.gy = st.gy[f];
        s.t = st.t[f];
        s.ep = st.ep[f];
        start = b.last_done[a] ? 1u : 0u;
    }
    bool any_reset = false;

    float o[8];
    env_obs<D>(x, s, o);
    for (int32_t k = 0; k < g.T; ++k) {
        // weights are re-read from LDS every step: keeps the compiler from hoisting the
        // loop-invariant LDS image into (spilled) registers
        asm volatile("" ::: "memory");
        // an opaque copy of the lane index: every LDS address derived from it is recomputed per
        // step instead of being hoisted into ~85 loop-invariant VGPRs
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int j = ln & 31, h = ln >> 5;
        const int64_t rk = (int64_t)k * A;
        // the observation the action is taken on -> observations[k]
        store_obs_rows<D>(stage, o, ln, M, b.obs + (rk + a_first) * D);
        h8 bo[2];
        tile_operands<D>(stage, j, h, bo);
        __builtin_amdgcn_wave_barrier();
        // Gaussian noise words: lane (j, h) draws them for agent j of tile h, so one Philox call
        // per lane covers both tiles (each agent keeps its own (global row, step) counter)
        const uint2 mine = det ? make_uint2(0u, 0u)
                               : policy_noise_bits(c.f0 * N + a_first + 32 * h + j, g.seed,
                                                   g.offset + k);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            // one tile at a time, outputs parked in LDS at once
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            uint2 nb = mine;
            if (!det) nb = make_uint2(__shfl(mine.x, j + 32 * t, 64), __shfl(mine.y, j + 32 * t, 64));
            const PolicyLane pl = policy_tile(wimg, bo[t], ln, nb, det, false);
            const int r = 32 * t + j;
            stage[2 * r + h] = pl.mu;
            stage[128 + 2 * r + h] = pl.act;
            stage[256 + 2 * r + h] = pl.clip;
            if (h == 0) {
                stage[384 + r] = pl.value;
                stage[448 + r] = pl.logp;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // one store per output: lane l writes agent a_first + l (bases are wave-uniform, so the
        // per-lane part of every address is a 32-bit offset)
        const int64_t o1 = rk + a_first;
        const float2 *s2 = reinterpret_cast<const float2 *>(stage);
        if (ln < M) {
            if (b.mu) reinterpret_cast<float2 *>(b.mu + 2 * o1)[ln] = s2[ln];
            reinterpret_cast<float2 *>(b.action + 2 * o1)[ln] = s2[64 + ln];
            if (b.clipped) reinterpret_cast<float2 *>(b.clipped + 2 * o1)[ln] = s2[128 + ln];
            (b.value + o1)[ln] = stage[384 + ln];
            (b.log_prob + o1)[ln] = stage[448 + ln];
        }
        const float2 ac = s2[128 + ln];
        __builtin_amdgcn_wave_barrier();

        // env.step(clipped actions) (collect_rollouts clips to the Box, vectorized_env.py:68-82)
        float rw;
        bool dn, rs;
        env_step<MODE>(c, p, x, f, a, i, active, ac, s, rw, dn, rs);
        any_reset |= rs;
        if (active) {  // active <=> ln < M; agent a = a_first + ln
            (b.reward + o1)[ln] = rw;
            (b.episode_start + o1)[ln] = (uint8_t)start;
            if (b.done) (b.done + o1)[ln] = (uint8_t)dn;
        }
        start = dn ? 1u : 0u;
        env_obs<D>(x, s, o);
    }

    // the observation after the last step (SB3's self._last_obs) and its value
    if (b.last_obs) {
        store_obs_rows<D>(stage, o, lane, M, b.last_obs + a_first * D);
    } else {
        stage_obs_rows<D>(stage, o, lane);
        __builtin_amdgcn_wave_barrier();
    }
    float lv = 0.0f;
    if (b.last_value) {
        const int j = lane & 31, h = lane >> 5;
        h8 bo[2];
        tile_operands<D>(stage, j, h, bo);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const PolicyLane pv = policy_tile(wimg, bo[t], lane, make_uint2(0u, 0u), true, true);
            if (h == 0) stage[384 + 32 * t + j] = pv.value;
        }
        __builtin_amdgcn_wave_barrier();
        lv = stage[384 + lane];
        __builtin_amdgcn_wave_barrier();  // the slice is reused by the wave's next unit
    }
    if (active) {
        b.last_done[a] = (uint8_t)start;
        if (b.last_value) b.last_value[a] = lv;
        st.px[a] = s.px;
        st.py[a] = s.py;
        if (i == 0) {
            st.t[f] = s.t;
            if (any_reset) {
                st.gx[f] = s.gx;
                st.gy[f] = s.gy;
                st.ep[f] = s.ep;
            }
        }
    }
}

// Persistent workgroups (grid = the resident workgroup count, or fewer): the weight image is
// staged once per workgroup, then every wave walks wave-units wave, wave + G, ... (G = the
// grid's wave count) with no further barrier, so a finished wave's slot never waits for its
// workgroup siblings and no workgroup re-stages the weights.
template <int D, int MODE>
__global__ __launch_bounds__(64 * kPRWaves) FENV_PR_OCCUPANCY void k_policy_rollout(Consts c, DevState st,
                                                                  DevPending p, PRArgs g) {
    // Dynamic LDS (kPRLdsBytes, set at launch): with a static declaration of this size the
    // compiler budgets registers for fewer waves/SIMD than the LDS allows.
    extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
    float *wimg = lds_dyn;
    float(*stage_all)[512] = reinterpret_cast<float(*)[512]>(lds_dyn + kPolicyLds);
    stage_policy_weights(wimg, g.params, D, threadIdx.x, blockDim.x);
    __syncthreads();  // the only workgroup barrier: waves are independent from here on

    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR
    const int64_t stride = (int64_t)gridDim.x * kPRWaves;
#pragma unroll 1
    for (int64_t wave = (int64_t)blockIdx.x * kPRWaves + w; wave * c.fpw < c.F; wave += stride)
        policy_rollout_unit<D, MODE>(c, st, p, g, wimg, stage_all[w], wave * c.fpw);
}

template <int D, int MODE>
static hipError_t policy_rollout_dm(const Consts &c, const DevState &s, const DevPending &p,
                                    const PRArgs &g, hipStream_t st) {
    const int64_t waves = (c.F + c.fpw - 1) / c.fpw;
    int64_t blocks = (waves + kPRWaves - 1) / kPRWaves;
    {
        // resident workgroups, per template instance (D, MODE) and device (devices may differ)
        static std::atomic<int> resident_by_dev[64];
        int dev = 0;
        (void)hipGetDevice(&dev);
        int resident = (dev >= 0 && dev < 64) ? resident_by_dev[dev].load() : 0;
        if (resident == 0) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_policy_rollout<D, MODE>,
                                                             64 * kPRWaves, kPRLdsBytes) !=
                    hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                    hipSuccess ||
                cus < 1)
                cus = 256;
            resident = per_cu * cus;
            if (dev >= 0 && dev < 64) resident_by_dev[dev].store(resident);
        }
        if (blocks > resident) blocks = resident;
    }
    hipLaunchKernelGGL((k_policy_rollout<D, MODE>), dim3((unsigned)blocks), dim3(64 * kPRWaves),
                       kPRLdsBytes, st, c, s, p, g);
    return hipGetLastError();
}

hipError_t launch_policy_rollout(const Consts &c, const DevState &s, const DevPending &p,
                                 int32_t D, const PRArgs &g, hipStream_t st) {
    const bool mt = c.reset_mode == FENV_RESET_MT19937;
    if (D == 8)
        return mt ? policy_rollout_dm<8, FENV_RESET_MT19937>(c, s, p, g, st)
                  : policy_rollout_dm<8, FENV_RESET_PHILOX>(c, s, p, g, st);
    return mt ? policy_rollout_dm<6, FENV_RESET_MT19937>(c, s, p, g, st)
              : policy_rollout_dm<6, FENV_RESET_PHILOX>(c, s, p, g, st);
}

}  // namespace fenvk
