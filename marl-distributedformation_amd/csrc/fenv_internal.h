// Internal interface between the C-ABI host layer (fenv_api.cpp) and the gfx950 kernels
// (fenv_kernels.hip, policy_kernels.hip).  Not installed; the public ABI is include/fenv.h.
#pragma once

#include <hip/hip_runtime.h>  // __host__ __device__ for the staged-set tag helpers
#include <stdint.h>

#include "fenv.h"

namespace fenvk {

// Device-resident env state, structure-of-arrays (one lane reads 8 B of position per agent,
// formation scalars are broadcast from one cache line to the formation's lanes).
struct DevState {
    float *px, *py;  // [A]  agent positions (simulate.py:133-135 self.agents)
    float *gx, *gy;  // [F]  goal (simulate.py:140-143)
    int32_t *t;      // [F]  steps_since_reset (simulate.py:147, :111)
    uint32_t *ep;    // [F]  episode counter (Philox reset key; not in the reference)
};

// Reset-side buffers: the host-staged next reset draw set (FENV_RESET_MT19937 mode) and the
// terminal (pre-reset, post-clip) state of the formations reset by their latest done step, which
// compute_reward_and_done's logged components (simulate.py:183-208) are taken from on a done step
// (written only on done steps; read by the metrics kernel).
//
// A staged set is px[A] py[A] gx[F] gy[F] atag[A] gtag[F] (stage_floats): every agent's and every
// formation's draw carries a tag the host computes from its bits, its index and the set's
// generation (stage_tag_agent / stage_tag_goal).  The kernels recompute the tag from what they
// read; a mismatch -- a set read before its copy landed, a stale line, the other slot -- is
// recorded in the handle's error words (host memory, read by every later API call, which then
// fails with FENV_ESTATE) instead of being applied silently.
struct DevPending {
    const float *pend;  // staged draw set of this launch (NULL in Philox mode)
    float4 *term;       // terminal (px, py, gx, gy)[A] (the goal repeated per agent: one
                        // store, one index)
    float *lf;          // N > kMaxN only: per-agent exchange scratch of the large-formation
                        // kernels (fenv_large.hip), 7 x [A] floats; NULL otherwise
    uint32_t *err;      // MT19937 mode: the handle's error words [4] (mapped host memory)
    uint32_t gen;       // generation of the set in `pend` (1 = the ctor's set)
};

// Tag of one staged draw (host and device compute the same bits; murmur3's 32-bit finaliser).
__host__ __device__ inline uint32_t stage_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    return x ^ (x >> 16);
}
__host__ __device__ inline uint32_t stage_rotl13(uint32_t x) { return (x << 13) | (x >> 19); }
// One finaliser round over the draw's bits, the generation and the index: a bijection of the
// combined word, so a draw read under another generation (or a stale value) mismatches unless
// the combination collides (~2^-32 per draw); one round keeps the host's tagging of a config-3
// set (5.2M agents) off the refill's critical path.
__host__ __device__ inline uint32_t stage_tag_agent(uint32_t gen, int64_t a, uint32_t bx,
                                                    uint32_t by) {
    return stage_mix(bx ^ stage_rotl13(by) ^ (gen * 0x85EBCA6Bu) ^ ((uint32_t)a * 0x9E3779B1u));
}
__host__ __device__ inline uint32_t stage_tag_goal(uint32_t gen, int64_t f, uint32_t bx,
                                                   uint32_t by) {
    return stage_mix(bx ^ stage_rotl13(by) ^ (gen * 0x85EBCA6Bu) ^ 0x5BD1E995u ^
                     ((uint32_t)f * 0x9E3779B1u));
}
// floats of one staged set (tags are 32-bit words in float slots)
inline int64_t stage_floats(int64_t A, int64_t F) { return 3 * A + 3 * F; }
// error words: [0] kind (0 none; kStageStale: the slot's previous set, two refills back;
// kStageOther: the set of the other slot; kStageBad: neither), [1] the generation expected,
// [2] the (shard-local) formation, [3] the number of the launch's lanes that saw it (capped)
enum : uint32_t { kStageStale = 1, kStageOther = 2, kStageBad = 3 };

struct Consts {
    int64_t F;          // formations in this shard
    int64_t f0;         // global index of formation 0 of the shard (Philox key)
    int32_t N;          // agents per formation
    int32_t fpw;        // formations per 64-lane wavefront (N <= 64 path)
    int32_t max_steps;  // simulate.py:20
    int32_t reset_mode; // FENV_RESET_*
    float c_self, c_nb; // (1 - 2 share), share (simulate.py:228-229)
    float d_nb;         // desired neighbour distance, fp32 (simulate.py:26)
    uint32_t key0, key1;// Philox key
};

// Geometry: N <= 64   -> `fpw` whole formations per wavefront, 256-thread workgroups.
//           N <= 1024 -> one formation per workgroup of round_up(N, 64) threads (LDS exchange).
//           N  > 1024 -> one formation per 1024-thread workgroup, several agents per thread,
//                        exchanges through global scratch (fenv_large.hip).
inline bool wave_path(int32_t N) { return N <= 64; }
constexpr int32_t kBlockMaxN = 1024;
inline bool large_path(int32_t N) { return N > kBlockMaxN; }
constexpr int kLargeScratchPerAgent = 7;  // floats of DevPending::lf per agent
int64_t group_count(const Consts &c);  // 4-wave workgroups (N<=64) or formations (N>64)
// workgroups of the rollout/step launch = records of its stats partials
int64_t rollout_group_count(const Consts &c);

// In-kernel synthetic actions (fenv_rollout_random): U(-1, 1) per component from Philox4x32-10
// keyed by act_seed, counter (global agent, global step / 2); one call serves two steps.
struct ActGen {
    uint32_t k0, k1;  // Philox key = act_seed
    uint64_t offset;  // global step index of the launch's local step 0
    float *out;       // optional [T][A][2] copy of the actions (NULL: not written)
};

// Launch plan of a T-step rollout call (fenv_rollout / fenv_rollout_random / fenv_step): calls
// of at least kNTMinAgentSteps agent-steps store their outputs non-temporally (rollout_nt) and
// run as kernel launches of at most rollout_launch_steps() steps each (fenv_api.cpp splits them,
// as it splits at MT19937 reset events); the state makes the round trip between the launches.
bool rollout_nt(const Consts &c, int64_t T);
int32_t rollout_launch_steps(const Consts &c, int64_t T);
hipError_t launch_rollout(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                          int32_t D, const float *act, float *obs, float *rew, uint8_t *done,
                          float *partial, bool accumulate, bool nt, hipStream_t st,
                          const ActGen *gen = nullptr);
hipError_t launch_reset_observe(const Consts &c, const DevState &s, const DevPending &p,
                                int32_t D, bool do_reset, float *obs, hipStream_t st);
// kMetricCols columns per formation (include/fenv.h fenv_metrics); `terminal`: formations with
// steps_since_reset == 0 take their reward components from the terminal state (the env's last
// state-changing call was a step, so t == 0 means "reset by that step").
constexpr int kMetricCols = 8;
hipError_t launch_metrics(const Consts &c, const DevState &s, const DevPending &p, bool terminal,
                          const float *rew, float *out, double *sums, hipStream_t st);
const char *rollout_kernel_name(const Consts &c, int32_t T);
// large formations (large_path(N)): the same entry points' kernels, fenv_large.hip
hipError_t launch_rollout_large(const Consts &c, const DevState &s, const DevPending &p,
                                int32_t T, int32_t D, const float *act, float *obs, float *rew,
                                uint8_t *done, float *partial, bool accumulate, hipStream_t st,
                                const ActGen *gen);
hipError_t launch_reset_observe_large(const Consts &c, const DevState &s, const DevPending &p,
                                      int32_t D, bool do_reset, float *obs, hipStream_t st);
hipError_t launch_metrics_large(const Consts &c, const DevState &s, const DevPending &p,
                                bool terminal, const float *rew, float *out, hipStream_t st);
// delay_sleeps > 0 (test hook fenv_test_stage_hook): every workgroup first waits that many
// s_sleep 127 periods (~3.4 us each), so a consumer not ordered behind the copy would read the
// slot's old set
hipError_t launch_stage_copy(float *dst, const float *src, int64_t n, int32_t delay_sleeps,
                             hipStream_t st);
hipError_t launch_reduce_partials(const float *partial, int64_t count, double *out,
                                  hipStream_t st);
hipError_t launch_stream_gate(const uint32_t *flag, uint32_t value, uint64_t timeout_ticks,
                              uint32_t khz, uint32_t *status, hipStream_t st);
hipError_t launch_fp_probe(int32_t op, const float *a, const float *b, float *out, int64_t n,
                           hipStream_t st);

hipError_t launch_policy_forward(const float *params, int32_t D, const float *obs, int64_t B,
                                 int64_t row0, float *mu, float *value, float *action, float *logp,
                                 float *clipped, uint64_t seed, uint64_t offset,
                                 int32_t deterministic, hipStream_t st);

// Fused policy->env rollout (policy_rollout.hip); GAE follows as a launch_gae.
struct PRArgs {
    fenv_rollout_bufs b;
    const float *params;
    int32_t T;
    int32_t deterministic;
    uint64_t seed, offset;
    float gamma, lam;
};
hipError_t launch_policy_rollout(const Consts &c, const DevState &s, const DevPending &p,
                                 int32_t D, const PRArgs &g, hipStream_t st);

hipError_t launch_gae(const float *rew, const float *values, const uint8_t *episode_starts,
                      const float *last_values, const uint8_t *last_dones, int32_t T, int64_t A,
                      float gamma, float lam, float *adv, float *ret, hipStream_t st);

hipError_t launch_ppo_update(float *params, float *exp_avg, float *exp_avg_sq, float *step,
                             int32_t D, const float *obs, const float *act,
                             const float *old_log_prob, const float *adv, const float *ret,
                             int64_t n, const int64_t *perm, int32_t n_epochs,
                             int32_t batch_size, const ppo_hparams &hp, double *stats,
                             void *workspace, hipStream_t st);
size_t ppo_workspace_bytes_impl();
void ppo_set_inject(int n);
hipError_t launch_ppo_grad(const float *params, int32_t D, const float *obs, const float *act,
                           const float *old_log_prob, const float *adv, const float *ret,
                           const int64_t *rows, int32_t b_local, int32_t b_global,
                           float adv_mean, float adv_std, int32_t adv_normalize,
                           int32_t entropy_term, const ppo_hparams &hp, float *grad,
                           double *stats, hipStream_t st);
hipError_t launch_ppo_apply(float *params, float *exp_avg, float *exp_avg_sq, float *step,
                            const float *grad, int32_t D, const ppo_hparams &hp,
                            hipStream_t st);

}  // namespace fenvk
