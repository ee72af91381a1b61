// Device-side SB3 MlpPolicy evaluation on the gfx950 matrix cores, shared by the standalone
// policy forward (policy_kernels.hip: k_policy) and the fused policy->env rollout
// (policy_rollout.hip: k_policy_rollout), so the two produce bit-identical outputs.
//
// Reference: SB3 `PPO('MlpPolicy', env, ...)` (/root/reference/vectorized_env.py:126) builds an
// ActorCriticPolicy with net_arch pi=[64,64], vf=[64,64], Tanh, a Linear(64,2) action head with a
// state-independent log_std[2], and a Linear(64,1) value head; collect_rollouts samples
// a = mu + exp(log_std) * eps, stores log_prob, and hands clip(a, -1, 1) to env.step;
// predict(deterministic=True) (/root/reference/visualize_policy.py:16) returns clip(mu).
//
// Mapping (one wavefront = one 32-agent tile):
//   layer 1  H1^T[64 x 32] = W1[64 x D] . O^T[D x 32]     v_mfma_f32_32x32x2_f32, 2 row tiles x D/2
//   layer 2  H2^T[64 x 32] = W2[64 x 64] . tanh(H1^T)     the layer-1 accumulator registers ARE the
//            B operands (lane l holds hidden rows rho(r, l>>5) of agent l&31), so no data moves
//            between layers; W2 is read from LDS pre-permuted into that k order (ds_read_b128).
//   heads    mu[2], value on the VALU from the layer-2 accumulators, halves joined across lanes
//            l and l^32.
// Both networks: 144 MFMAs of 32x32x2 per 32 agents = 18,816 FLOP/agent.
//
// tanh.  Hidden-layer weights and biases are staged pre-multiplied by 2/ln2, so an accumulator
// holds y = 2x*log2(e) and tanh(x) = 1 - 2 / (1 + 2^y): v_exp_f32, v_add, v_rcp_f32, v_fma --
// 4 VALU instructions instead of a 13-instruction rational, which is what lets the VALU work hide
// under the MFMAs.  |abs err| < 5e-7 (tests/test_gpu_policy.py bounds the network outputs).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fenvk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef FENV_POLICY_PRIO
#define FENV_POLICY_PRIO 0
#endif

constexpr int kHid = 64;
constexpr float kTanhScale = 2.88539008177792681f;  // 2 / ln(2)

// row of accumulator register `reg` held by lane half `h` (32x32 C/D layout)
__host__ __device__ constexpr int rho(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Flat parameter offsets (include/fenv.h policy_forward layout = SB3 state_dict order)
struct PLayout {
    int pi0W, pi0b, pi2W, pi2b, vf0W, vf0b, vf2W, vf2b, actW, actb, valW, valb, logstd, total;
    __host__ __device__ explicit PLayout(int D) {
        pi0W = 0;
        pi0b = pi0W + kHid * D;
        pi2W = pi0b + kHid;
        pi2b = pi2W + kHid * kHid;
        vf0W = pi2b + kHid;
        vf0b = vf0W + kHid * D;
        vf2W = vf0b + kHid;
        vf2b = vf2W + kHid * kHid;
        actW = vf2b + kHid;
        actb = actW + 2 * kHid;
        valW = actb + 2;
        valb = valW + kHid;
        logstd = valb + 1;
        total = logstd + 2;
    }
};

// LDS image (floats).  net 0 = actor (pi), 1 = critic (vf).
constexpr int kW1F = 2 * 2 * 4 * 64;       // [net][ht][s][lane]           W1 * kTanhScale
constexpr int kW2F = 2 * 2 * 2 * 16 * 64;  // [net][ot][kt][r/4][lane][4]  W2 * kTanhScale
constexpr int oW1 = 0;
constexpr int oW2 = oW1 + kW1F;
constexpr int oB1 = oW2 + kW2F;            // [net][64]  b1 * kTanhScale
constexpr int oB2 = oB1 + 2 * kHid;        // [net][64]  b2 * kTanhScale
constexpr int oHA0 = oB2 + 2 * kHid;       // action_net.weight[0][64]
constexpr int oHA1 = oHA0 + kHid;          // action_net.weight[1][64]
constexpr int oHV = oHA1 + kHid;           // value_net.weight[0][64]
constexpr int oSc = oHV + kHid;            // ba0 ba1 bv log_std0 log_std1 (+3 pad)
constexpr int kPolicyLds = oSc + 8;        // 9,672 floats = 38.7 KB

// Cooperative copy of the flat parameters into the LDS image (all threads of the block).
__device__ __forceinline__ void stage_policy_weights(float *lds, const float *__restrict__ params,
                                                     int D, int tid, int nthreads) {
    const PLayout L(D);
    for (int e = tid; e < kW1F; e += nthreads) {
        const int lane = e & 63, s = (e >> 6) & 3, ht = (e >> 8) & 1, net = e >> 9;
        const int row = 32 * ht + (lane & 31), col = 2 * s + (lane >> 5);
        const int base = net ? L.vf0W : L.pi0W;
        lds[oW1 + e] = col < D ? params[base + row * D + col] * kTanhScale : 0.0f;
    }
    for (int e = tid; e < kW2F; e += nthreads) {
        const int q = e & 3, lane = (e >> 2) & 63, r4 = (e >> 8) & 3, kt = (e >> 10) & 1,
                  ot = (e >> 11) & 1, net = e >> 12;
        const int r = 4 * r4 + q;
        const int row = 32 * ot + (lane & 31), col = 32 * kt + rho(r, lane >> 5);
        lds[oW2 + e] = params[(net ? L.vf2W : L.pi2W) + row * kHid + col] * kTanhScale;
    }
    for (int e = tid; e < kHid; e += nthreads) {
        lds[oB1 + e] = params[L.pi0b + e] * kTanhScale;
        lds[oB1 + kHid + e] = params[L.vf0b + e] * kTanhScale;
        lds[oB2 + e] = params[L.pi2b + e] * kTanhScale;
        lds[oB2 + kHid + e] = params[L.vf2b + e] * kTanhScale;
        lds[oHA0 + e] = params[L.actW + e];
        lds[oHA1 + e] = params[L.actW + kHid + e];
        lds[oHV + e] = params[L.valW + e];
    }
    if (tid < 8) {
        float v = 0.0f;
        if (tid < 2) v = params[L.actb + tid];
        else if (tid == 2) v = params[L.valb];
        else if (tid < 5) v = params[L.logstd + tid - 3];
        lds[oSc + tid] = v;
    }
}

// tanh(x) from y = x * 2/ln2 (see header)
__device__ __forceinline__ float tanh_s(float y) {
    const float e = __builtin_amdgcn_exp2f(y);
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
}

// accumulator <- bias rows rho(reg, h) of hidden rows [32*ht, 32*ht + 32): 4 x ds_read_b128
__device__ __forceinline__ f32x16 bias_acc(const float *b, int ht, int h) {
    f32x16 a;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 v = *reinterpret_cast<const f32x4 *>(&b[32 * ht + 8 * r4 + 4 * h]);
        a[4 * r4 + 0] = v[0];
        a[4 * r4 + 1] = v[1];
        a[4 * r4 + 2] = v[2];
        a[4 * r4 + 3] = v[3];
    }
    return a;
}

// One network (net 0 actor / 1 critic) over one 32-agent tile: layer 1, tanh, layer 2, tanh.
// Leaves tanh(H2) rows rho(reg, h) (+32*ot) of agent l&31 in c0 (ot 0) and c1 (ot 1).
__device__ __forceinline__ void net_tile(const float *lds, int net, const float (&ob)[4], int D,
                                         int lane, int h, f32x16 &c0, f32x16 &c1) {
    f32x16 a0 = bias_acc(lds + oB1 + net * kHid, 0, h);
    f32x16 a1 = bias_acc(lds + oB1 + net * kHid, 1, h);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (2 * s >= D) break;
        a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + ((net * 2 + 0) * 4 + s) * 64 + lane],
                                                  ob[s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + ((net * 2 + 1) * 4 + s) * 64 + lane],
                                                  ob[s], a1, 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        a0[reg] = tanh_s(a0[reg]);
        a1[reg] = tanh_s(a1[reg]);
    }
    c0 = bias_acc(lds + oB2 + net * kHid, 0, h);
    c1 = bias_acc(lds + oB2 + net * kHid, 1, h);
#if FENV_POLICY_PRIO
    __builtin_amdgcn_s_setprio(1);  // a wave in its MFMA phase wins issue arbitration
#endif
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
            const f32x4 w0 = *reinterpret_cast<const f32x4 *>(
                &lds[oW2 + ((((net * 2 + 0) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
            const f32x4 w1 = *reinterpret_cast<const f32x4 *>(
                &lds[oW2 + ((((net * 2 + 1) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float b = kt == 0 ? a0[4 * r4 + q] : a1[4 * r4 + q];
                c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[q], b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[q], b, c1, 0, 0, 0);
            }
        }
    }
#if FENV_POLICY_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        c0[reg] = tanh_s(c0[reg]);
        c1[reg] = tanh_s(c1[reg]);
    }
}

// sum_rows w[row] * hid[row] over this lane's 32 hidden rows, fixed order (ot, r4, q)
__device__ __forceinline__ float head_dot(const float *w, const f32x16 &c0, const f32x16 &c1,
                                          int h) {
    float p = 0.0f;
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
            const f32x4 wv = *reinterpret_cast<const f32x4 *>(&w[32 * ot + 8 * r4 + 4 * h]);
#pragma unroll
            for (int q = 0; q < 4; ++q) p = __builtin_fmaf(wv[q], (ot ? c1 : c0)[4 * r4 + q], p);
        }
    }
    return p;
}

// join the two lane halves in a fixed order (half 0 + half 1)
__device__ __forceinline__ float join_halves(float v, int h) {
    const float o = __shfl_xor(v, 32, 64);
    return h == 0 ? v + o : o + v;
}

__device__ __forceinline__ uint4 philox4x32(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// What one lane (agent l&31 of the tile, action component h = l>>5) gets from the policy.
struct PolicyLane {
    float mu;     // mu[h]
    float act;    // unclipped action[h] (= mu[h] when deterministic)
    float clip;   // clamp(act, -1, 1)
    float value;  // critic value (both halves)
    float logp;   // sum over both components of Normal(mu, std).log_prob(act) (both halves)
};

// Full policy evaluation of one 32-agent tile.  ob[s] = obs[agent][2s + h] (0 for 2s+h >= D);
// `row` is the agent's row in the batch (Philox counter); value_only skips the actor.
__device__ __forceinline__ PolicyLane policy_tile(const float *lds, const float (&ob)[4], int D,
                                                  int lane, int64_t row, uint64_t seed,
                                                  uint64_t offset, bool deterministic,
                                                  bool value_only) {
    const int h = lane >> 5;
    PolicyLane o;
    f32x16 c0, c1;
    float pa = 0.0f;
    if (!value_only) {
        net_tile(lds, 0, ob, D, lane, h, c0, c1);
        const float p0 = head_dot(lds + oHA0, c0, c1, h);
        const float p1 = head_dot(lds + oHA1, c0, c1, h);
        // keep component h: own partial + the partner half's partial of the same component
        const float other = __shfl_xor(h == 0 ? p1 : p0, 32, 64);
        pa = h == 0 ? p0 + other : other + p1;
    }
    __builtin_amdgcn_sched_barrier(0);  // actor, then critic: overlapping them costs registers
    net_tile(lds, 1, ob, D, lane, h, c0, c1);
    o.value = join_halves(head_dot(lds + oHV, c0, c1, h), h) + lds[oSc + 2];
    if (value_only) {
        o.mu = o.act = o.clip = o.logp = 0.0f;
        return o;
    }
    const float std_h = expf(lds[oSc + 3 + h]);
    o.mu = pa + lds[oSc + h];
    float a = o.mu;
    if (!deterministic) {
        const uint4 r = philox4x32(make_uint4((uint32_t)row, (uint32_t)((uint64_t)row >> 32),
                                              (uint32_t)offset, (uint32_t)(offset >> 32)),
                                   (uint32_t)seed, (uint32_t)(seed >> 32));
        const float u1 = (float)((r.x >> 8) + 1u) * 0x1.0p-24f;  // (0, 1]
        const float u2 = (float)(r.y >> 8) * 0x1.0p-24f;          // [0, 1)
        // Box-Muller on the hardware transcendentals: v_log_f32 is log2, v_sin/v_cos_f32 take
        // the angle in turns (sin(2 pi u2) directly, no range reduction needed for u2 in [0,1))
        const float rad = __builtin_amdgcn_sqrtf(-1.38629436111989061f * __builtin_amdgcn_logf(u1));
        const float eps = rad * (h == 0 ? __builtin_amdgcn_cosf(u2) : __builtin_amdgcn_sinf(u2));
        a = o.mu + std_h * eps;
    }
    o.act = a;
    o.clip = a < -1.0f ? -1.0f : (a > 1.0f ? 1.0f : a);
    // torch Normal.log_prob: -(a-mu)^2 / (2 var) - log(scale) - log(sqrt(2 pi)), scale = exp(ls)
    const float inv_2var = 0.5f / (std_h * std_h);
    const float d = a - o.mu;
    const float lp_h = -(d * d) * inv_2var - logf(std_h) - 0.918938533204672742f;
    o.logp = join_halves(lp_h, h);
    return o;
}

// SB3 RolloutBuffer.compute_returns_and_advantage, one backward step (GAE(lambda)):
// delta = r + gamma * V' * nnt - V;  A = delta + gamma * lambda * nnt * A'
__device__ __forceinline__ float gae_step(float rew, float v, float next_v, float next_nt,
                                          float gamma, float lam, float last) {
    const float delta = rew + gamma * next_v * next_nt - v;
    return delta + gamma * lam * next_nt * last;
}

}  // namespace fenvk
