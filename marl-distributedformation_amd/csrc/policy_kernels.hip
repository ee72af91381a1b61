// Batched actor-critic MLP forward on the gfx950 matrix cores (fp32 in, fp32 accumulate).
//
// Reference: SB3 `PPO('MlpPolicy', env, ...)` (/root/reference/vectorized_env.py:126) builds an
// ActorCriticPolicy with net_arch pi=[64,64], vf=[64,64], Tanh, a Linear(64,2) action head with a
// state-independent log_std[2], and a Linear(64,1) value head; collect_rollouts samples
// a = mu + exp(log_std) * eps, stores log_prob, and hands clip(a, -1, 1) to env.step;
// predict(deterministic=True) (/root/reference/visualize_policy.py:16) returns clip(mu).
//
// Mapping (one wavefront = 32 agents per tile, persistent workgroups of 4 waves):
//   layer 1  H1^T[64 x 32] = W1[64 x D] . O^T[D x 32]     v_mfma_f32_32x32x2_f32, 2 row tiles x D/2
//   layer 2  H2^T[64 x 32] = W2[64 x 64] . tanh(H1^T)     the layer-1 accumulator registers ARE the
//            B operands (lane l holds hidden rows rho(r, l>>5) of agent l&31), so no data moves
//            between layers; W2 is read from LDS pre-permuted into that k order (ds_read_b128).
//   heads    mu[2], value on the VALU from the layer-2 accumulators, halves joined across lanes
//            l and l^32.
// Both networks: 144 MFMAs of 32x32x2 per 32 agents = 18,816 FLOP/agent.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "fenv.h"
#include "fenv_internal.h"

namespace fenvk {

#ifndef FENV_POLICY_V2
#define FENV_POLICY_V2 0
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kHid = 64;

// row of accumulator register `reg` held by lane half `h` (32x32 C/D layout)
__host__ __device__ constexpr int rho(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Flat parameter offsets (include/fenv.h policy_forward layout)
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

// LDS image (floats)
constexpr int kW1F = 2 * 2 * 4 * 64;          // [net][ht][s][lane]
constexpr int kW2F = 2 * 2 * 2 * 16 * 64;     // [net][ot][kt][r/4][lane][4]
constexpr int kB = 2 * 2 * kHid;              // b1[net][64], b2[net][64]
constexpr int kHead = 3 * kHid + 3 + 2;       // Wa[2][64], Wv[64], ba[2], bv, log_std[2]
constexpr int kLds = kW1F + kW2F + kB + kHead;
constexpr int oW1 = 0, oW2 = kW1F, oB1 = kW1F + kW2F, oB2 = oB1 + 2 * kHid, oHead = oB1 + kB;

// Single-precision tanh without libm calls: odd/even minimax rational x P(x^2) / Q(x^2) on
// [-7.9988, 7.9988] (clamped outside; Eigen's float tanh coefficients), one v_rcp_f32.
// |abs err| < 4e-7 over all inputs (tests/test_gpu_policy.py bounds the network outputs).
__device__ __forceinline__ float tanh_f(float x) {
    const float xc = __builtin_amdgcn_fmed3f(x, -7.99881172180175781f, 7.99881172180175781f);
    const float x2 = xc * xc;
    float p = -2.76076847742355e-16f;
    p = __builtin_fmaf(p, x2, 2.00018790482477e-13f);
    p = __builtin_fmaf(p, x2, -8.60467152213735e-11f);
    p = __builtin_fmaf(p, x2, 5.12229709037114e-08f);
    p = __builtin_fmaf(p, x2, 1.48572235717979e-05f);
    p = __builtin_fmaf(p, x2, 6.37261928875436e-04f);
    p = __builtin_fmaf(p, x2, 4.89352455891786e-03f);
    float q = 1.19825839466702e-06f;
    q = __builtin_fmaf(q, x2, 1.18534705686654e-04f);
    q = __builtin_fmaf(q, x2, 2.26843463243900e-03f);
    q = __builtin_fmaf(q, x2, 4.89352518554385e-03f);
    return (p * xc) * __builtin_amdgcn_rcpf(q);
}

__device__ __forceinline__ uint4 philox_p(uint4 c, uint32_t k0, uint32_t k1) {
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

__global__ __launch_bounds__(256) void k_policy(const float *__restrict__ params, int32_t D,
                                               const float *__restrict__ obs, int64_t B,
                                               float *__restrict__ mu_out,
                                               float *__restrict__ value_out,
                                               float *__restrict__ act_out,
                                               float *__restrict__ logp_out,
                                               float *__restrict__ clip_out, uint64_t seed,
                                               uint64_t offset, int32_t deterministic) {
    __shared__ __attribute__((aligned(16))) float lds[kLds];
    const PLayout L(D);
    const int tid = threadIdx.x;
    // ---- stage weights into the fragment-ordered LDS image
    for (int e = tid; e < kW1F; e += blockDim.x) {
        const int lane = e & 63, s = (e >> 6) & 3, ht = (e >> 8) & 1, net = e >> 9;
        const int row = 32 * ht + (lane & 31), col = 2 * s + (lane >> 5);
        const int base = net ? L.vf0W : L.pi0W;
        lds[oW1 + e] = col < D ? params[base + row * D + col] : 0.0f;
    }
    for (int e = tid; e < kW2F; e += blockDim.x) {
        const int q = e & 3, lane = (e >> 2) & 63, r4 = (e >> 8) & 3, kt = (e >> 10) & 1,
                  ot = (e >> 11) & 1, net = e >> 12;
        const int r = 4 * r4 + q;
        const int row = 32 * ot + (lane & 31), col = 32 * kt + rho(r, lane >> 5);
        lds[oW2 + e] = params[(net ? L.vf2W : L.pi2W) + row * kHid + col];
    }
    for (int e = tid; e < kHid; e += blockDim.x) {
        lds[oB1 + e] = params[L.pi0b + e];
        lds[oB1 + kHid + e] = params[L.vf0b + e];
        lds[oB2 + e] = params[L.pi2b + e];
        lds[oB2 + kHid + e] = params[L.vf2b + e];
        lds[oHead + e] = params[L.actW + e];
        lds[oHead + kHid + e] = params[L.actW + kHid + e];
        lds[oHead + 2 * kHid + e] = params[L.valW + e];
    }
    if (tid < 2) {
        lds[oHead + 3 * kHid + tid] = params[L.actb + tid];
        lds[oHead + 3 * kHid + 3 + tid] = params[L.logstd + tid];
    }
    if (tid == 0) lds[oHead + 3 * kHid + 2] = params[L.valb];
    __syncthreads();

    const int lane = tid & 63, j = lane & 31, h = lane >> 5;
    const int waves_per_block = blockDim.x >> 6;
    const int64_t ntiles = (B + 31) / 32;
    const float ls_h = lds[oHead + 3 * kHid + 3 + h];
    const float std_h = expf(ls_h);
    const float ba_h = lds[oHead + 3 * kHid + h];
    const float ba_o = lds[oHead + 3 * kHid + (h ^ 1)];
    const float bv = lds[oHead + 3 * kHid + 2];
    const float log_scale = logf(std_h);
    const float half_log_2pi = 0.918938533204672742f;  // log(sqrt(2*pi))

    for (int64_t tile = (int64_t)blockIdx.x * waves_per_block + (tid >> 6); tile < ntiles;
         tile += (int64_t)gridDim.x * waves_per_block) {
        const int64_t row = tile * 32 + j;
        const bool valid = row < B;
        float o[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int col = 2 * s + h;
            o[s] = (valid && col < D) ? obs[row * D + col] : 0.0f;
        }
#if FENV_POLICY_V2
        float head[3] = {0.f, 0.f, 0.f};  // mu0, mu1 partials (actor), value partial (critic)
        // Both networks in one straight-line body, ordered so that each MFMA phase has
        // independent VALU work beside it: L1(pi,vf) | L2(pi) || tanh L1(vf) | L2(vf) || tanh
        // L2(pi) + actor head | tanh L2(vf) + value head.
        f32x16 pa0, pa1, va0, va1;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            pa0[reg] = lds[oB1 + rho(reg, h)];
            pa1[reg] = lds[oB1 + 32 + rho(reg, h)];
            va0[reg] = lds[oB1 + kHid + rho(reg, h)];
            va1[reg] = lds[oB1 + kHid + 32 + rho(reg, h)];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (2 * s >= D) break;
            pa0 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + (0 * 4 + s) * 64 + lane], o[s], pa0, 0, 0, 0);
            pa1 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + (1 * 4 + s) * 64 + lane], o[s], pa1, 0, 0, 0);
            va0 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + (2 * 4 + s) * 64 + lane], o[s], va0, 0, 0, 0);
            va1 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + (3 * 4 + s) * 64 + lane], o[s], va1, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            pa0[reg] = tanh_f(pa0[reg]);
            pa1[reg] = tanh_f(pa1[reg]);
        }
        f32x16 pc0, pc1, vc0, vc1;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            pc0[reg] = lds[oB2 + rho(reg, h)];
            pc1[reg] = lds[oB2 + 32 + rho(reg, h)];
            vc0[reg] = lds[oB2 + kHid + rho(reg, h)];
            vc1[reg] = lds[oB2 + kHid + 32 + rho(reg, h)];
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const f32x4 w0 = *reinterpret_cast<const f32x4 *>(&lds[oW2 + ((((0 * 2 + 0) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
                const f32x4 w1 = *reinterpret_cast<const f32x4 *>(&lds[oW2 + ((((0 * 2 + 1) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float b = kt == 0 ? pa0[4 * r4 + q] : pa1[4 * r4 + q];
                    pc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[q], b, pc0, 0, 0, 0);
                    pc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[q], b, pc1, 0, 0, 0);
                    // independent VALU beside the actor's layer-2 MFMAs
                    va0[4 * r4 + q + 0] = kt == 0 ? tanh_f(va0[4 * r4 + q]) : va0[4 * r4 + q];
                    va1[4 * r4 + q + 0] = kt == 1 ? tanh_f(va1[4 * r4 + q]) : va1[4 * r4 + q];
                }
            }
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const f32x4 w0 = *reinterpret_cast<const f32x4 *>(&lds[oW2 + ((((1 * 2 + 0) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
                const f32x4 w1 = *reinterpret_cast<const f32x4 *>(&lds[oW2 + ((((1 * 2 + 1) * 2 + kt) * 4 + r4) * 64 + lane) * 4]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float b = kt == 0 ? va0[4 * r4 + q] : va1[4 * r4 + q];
                    vc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[q], b, vc0, 0, 0, 0);
                    vc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[q], b, vc1, 0, 0, 0);
                    // actor head beside the critic's layer-2 MFMAs (same order as v1)
                    const int reg = 4 * r4 + q;
                    const f32x16 &pc = kt ? pc1 : pc0;
                    const float hv = tanh_f(pc[reg]);
                    const int idx = 32 * kt + rho(reg, h);
                    head[0] = __builtin_fmaf(lds[oHead + idx], hv, head[0]);
                    head[1] = __builtin_fmaf(lds[oHead + kHid + idx], hv, head[1]);
                }
            }
        }
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const float hv = tanh_f(ot ? vc1[reg] : vc0[reg]);
                head[2] = __builtin_fmaf(lds[oHead + 2 * kHid + 32 * ot + rho(reg, h)], hv, head[2]);
            }
        }
#else
        float head[3] = {0.f, 0.f, 0.f};  // mu0, mu1 partials (actor), value partial (critic)
#pragma unroll 1
        for (int net = 0; net < 2; ++net) {
            f32x16 a0, a1;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                a0[reg] = lds[oB1 + net * kHid + rho(reg, h)];
                a1[reg] = lds[oB1 + net * kHid + 32 + rho(reg, h)];
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (2 * s >= D) break;
                a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + ((net * 2 + 0) * 4 + s) * 64 + lane],
                                                          o[s], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(lds[oW1 + ((net * 2 + 1) * 4 + s) * 64 + lane],
                                                          o[s], a1, 0, 0, 0);
            }
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                a0[reg] = tanh_f(a0[reg]);
                a1[reg] = tanh_f(a1[reg]);
            }
            f32x16 c0, c1;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                c0[reg] = lds[oB2 + net * kHid + rho(reg, h)];
                c1[reg] = lds[oB2 + net * kHid + 32 + rho(reg, h)];
            }
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
            // heads over this lane's 32 hidden rows (ot = 0, 1; reg order), fma chain
            if (net == 0) {
                float p0 = 0.f, p1 = 0.f;
#pragma unroll
                for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const float hv = tanh_f(ot ? c1[reg] : c0[reg]);
                        const int idx = 32 * ot + rho(reg, h);
                        p0 = __builtin_fmaf(lds[oHead + idx], hv, p0);
                        p1 = __builtin_fmaf(lds[oHead + kHid + idx], hv, p1);
                    }
                }
                head[0] = p0;
                head[1] = p1;
            } else {
                float pv = 0.f;
#pragma unroll
                for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const float hv = tanh_f(ot ? c1[reg] : c0[reg]);
                        pv = __builtin_fmaf(lds[oHead + 2 * kHid + 32 * ot + rho(reg, h)], hv, pv);
                    }
                }
                head[2] = pv;
            }
        }
#endif
        // join the two lane halves in a fixed order (half 0 + half 1), add biases
        float full[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const float other = __shfl_xor(head[m], 32, 64);
            full[m] = h == 0 ? head[m] + other : other + head[m];
        }
        const float mu_h = (h == 0 ? full[0] : full[1]) + ba_h;
        const float mu_o = (h == 0 ? full[1] : full[0]) + ba_o;
        (void)mu_o;
        const float value = full[2] + bv;
        float a_h = mu_h;
        if (!deterministic) {
            const uint4 r = philox_p(make_uint4((uint32_t)row, (uint32_t)((uint64_t)row >> 32),
                                                (uint32_t)offset, (uint32_t)(offset >> 32)),
                                     (uint32_t)seed, (uint32_t)(seed >> 32));
            const float u1 = (float)((r.x >> 8) + 1u) * 0x1.0p-24f;  // (0, 1]
            const float u2 = (float)(r.y >> 8) * 0x1.0p-24f;          // [0, 1)
            const float rad = sqrtf(-2.0f * logf(u1));
            float sn, cs;
            sincosf(6.28318530717958648f * u2, &sn, &cs);
            const float eps = h == 0 ? rad * cs : rad * sn;
            a_h = mu_h + std_h * eps;
        }
        // Normal(mu, std).log_prob(a) summed over the 2 action dims
        const float var = std_h * std_h;
        const float d = a_h - mu_h;
        const float lp_h = -(d * d) / (2.0f * var) - log_scale - half_log_2pi;
        const float lp_o = __shfl_xor(lp_h, 32, 64);
        const float logp = h == 0 ? lp_h + lp_o : lp_o + lp_h;
        if (valid) {
            if (mu_out) mu_out[row * 2 + h] = mu_h;
            if (act_out) act_out[row * 2 + h] = a_h;
            if (clip_out) clip_out[row * 2 + h] = a_h < -1.0f ? -1.0f : (a_h > 1.0f ? 1.0f : a_h);
            if (h == 0) {
                if (value_out) value_out[row] = value;
                if (logp_out) logp_out[row] = logp;
            }
        }
    }
}

hipError_t launch_policy_forward(const float *params, int32_t D, const float *obs, int64_t B,
                                 float *mu, float *value, float *action, float *logp,
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
    hipLaunchKernelGGL(k_policy, dim3((unsigned)blocks), dim3(256), 0, st, params, D, obs, B, mu,
                       value, action, logp, clipped, seed, offset, deterministic);
    return hipGetLastError();
}

}  // namespace fenvk

namespace fenvk {

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
        const float delta = rew[r] + gamma * next_v * next_nt - v;
        last = delta + gamma * lam * next_nt * last;
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
