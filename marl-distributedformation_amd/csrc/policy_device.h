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
// Arithmetic: split-f16 MFMA ("3xf16").  Every fp32 operand x is split as x = hi + lo with
// hi = x truncated to 11 significant bits and lo = the exact remainder rounded to f16, and each
// fp32 product is taken as hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16 (products exact,
// fp32 accumulation; the dropped lo*lo term and lo's rounding are < 2^-21 relative).  Three
// 32-cycle f16 MFMAs replace eight 64-cycle f32 32x32x2 MFMAs per 16-deep k-chunk: the policy
// tile's MFMA time drops ~5x while the results stay within the fp32 tolerance
// (tests/test_gpu_policy.py; numpy emulation tools/split_f16_error.py: worst error 17 % of the
// 2e-5 + 2e-5|ref| bound).  Operand-map, subnormal and exactness facts this relies on are probed
// on the hardware by tools/mfma_f16_probe.hip.  Inputs must satisfy |x| < 65504 (f16 range);
// the env's observations are within [-1.5, 1.5].
//
// Mapping (one wavefront = one 32-agent tile, lane l: agent r = l&31, half h = l>>5):
//   layer 1  H1^T[64 x 32] = W1[64 x D] . O^T[D x 32]: per 32-row tile two MFMAs over a 16-slot
//            k: slots 0-7 (half 0) carry (W1hi, Ohi), slots 8-15 (half 1) (W1hi, Olo); then
//            (W1lo, Ohi) in half 0 and zeros in half 1.
//   layer 2  H2^T[64 x 32] = W2[64 x 64] . tanh(H1^T): the layer-1 accumulator registers ARE the
//            B operands (chunk c = registers 8(c&1)..+7 of row tile c>>1, i.e. hidden rows
//            32(c>>1) + rho(8(c&1)+j, h)); W2 is staged in LDS pre-permuted into that k order as
//            hi and lo fragments (one ds_read_b128 each).  4 chunks x 3 products per row tile.
//   heads    mu[2], value on the VALU (fp32 FMA) from the layer-2 accumulators, halves joined
//            across lanes l and l^32.
// Both networks: 56 f16 MFMAs per 32 agents carrying 18,816 fp32-equivalent FLOP/agent
// (SURVEY §8(a) R10).
//
// tanh.  Hidden-layer weights and biases are staged pre-multiplied by 2/ln2, so an accumulator
// holds y = 2x*log2(e); the layers pass on r = 1/(1 + 2^y) = (1 - tanh x)/2 (v_exp_f32, v_add,
// v_rcp_f32) and the consumers fold tanh = 1 - 2r into their weights and biases (see rsig).
// |abs err of tanh| < 5e-7.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fenvk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

// LDS image (floats).  net 0 = actor (pi), 1 = critic (vf).  An MFMA A fragment is 64 lanes x
// 8 f16 = 256 floats (1 KiB), read with one ds_read_b128 per lane.
constexpr int kFrag = 64 * 4;
constexpr int oW1 = 0;                     // fragments [net][ht][m]          W1 * kTanhScale
constexpr int oW2 = oW1 + 8 * kFrag;       // fragments [net][ot][c][hi/lo]   -2 * W2 * kTanhScale
constexpr int oB1 = oW2 + 32 * kFrag;      // [net][64]  b1 * kTanhScale (fp32)
constexpr int oB2 = oB1 + 2 * kHid;        // [net][64]  (b2 + rowsum W2) * kTanhScale
constexpr int oHA0 = oB2 + 2 * kHid;       // -2 * action_net.weight[0][64]
constexpr int oHA1 = oHA0 + kHid;          // -2 * action_net.weight[1][64]
constexpr int oHV = oHA1 + kHid;           // -2 * value_net.weight[0][64]
constexpr int oSc = oHV + kHid;            // ba0 ba1 bv (each + rowsum), log_std[2], then per
                                           // component h: std[2] at +5, 0.5/var[2] at +7,
                                           // log(std)[2] at +9 (hoisted out of the step loop)
constexpr int kPolicyLds = oSc + 12;       // 10,700 floats = 42.8 KB

// x = hi + lo: hi = x truncated to 11 significant bits (exact in f16 for 2^-14 <= |x| < 65504),
// lo = f16(x - hi) (x - hi is exact).  Two values per v_cvt_pkrtz_f16_f32.
__device__ __forceinline__ uint32_t pk_rtz(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
// Weights (staged once per workgroup): hi rounded to nearest (ties away) on the integer bits.
// Every conversion goes through these explicit integer ops and v_cvt_pkrtz, never a compiler
// f32->f16 cast: hipcc lowers casts to v_cvt_f16_f32 or v_cvt_pk_f16_f32 depending on the
// surrounding code, and the two kernels that share this image must stage the same bits.
__device__ __forceinline__ float hi11_rn(float x) {
    return __uint_as_float((__float_as_uint(x) + 0x1000u) & 0xFFFFE000u);
}
__device__ __forceinline__ _Float16 to_f16(float x) {
    return __builtin_bit_cast(_Float16, (uint16_t)(pk_rtz(x, 0.0f) & 0xFFFFu));
}
template <class V>
__device__ __forceinline__ void split8(const V &v, int base, h8 &hi, h8 &lo) {
    u32x4 H, L;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const float x = v[base + 2 * p], y = v[base + 2 * p + 1];
        // hi = RTZ to f16 (the 11 leading significant bits); the exact remainder x - f32(hi)
        // straight from the packed halves with v_fma_mix_f32 (f16 operand, f32 math)
        const uint32_t hh = pk_rtz(x, y);
        float lx, ly;
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lx) : "v"(hh), "v"(x));
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "=v"(ly) : "v"(hh), "v"(y));
        H[p] = hh;
        L[p] = pk_rtz(lx, ly);
    }
    hi = __builtin_bit_cast(h8, H);
    lo = __builtin_bit_cast(h8, L);
}

// Cooperative copy of the flat parameters into the LDS image (all threads of the block).
__device__ __forceinline__ void stage_policy_weights(float *lds, const float *__restrict__ params,
                                                     int D, int tid, int nthreads) {
    const PLayout L(D);
    _Float16 *fh = reinterpret_cast<_Float16 *>(lds);
    // layer 1: fragment (net, ht, m), lane (r, hh), slot j -> W1[32 ht + r][j]
    for (int e = tid; e < 8 * 64 * 8; e += nthreads) {
        const int j = e & 7, lane = (e >> 3) & 63, m = (e >> 9) & 1, ht = (e >> 10) & 1,
                  net = e >> 11;
        const int row = 32 * ht + (lane & 31), hh = lane >> 5;
        const float w = j < D ? params[(net ? L.vf0W : L.pi0W) + row * D + j] * kTanhScale : 0.0f;
        const float whi = hi11_rn(w);
        fh[2 * oW1 + e] = to_f16(m == 0 ? whi : (hh == 0 ? w - whi : 0.0f));
    }
    // layer 2: fragment (net, ot, c, hl), lane (r, hh), slot j -> W2[32 ot + r][k(c, hh, j)]
    for (int e = tid; e < 32 * 64 * 8; e += nthreads) {
        const int j = e & 7, lane = (e >> 3) & 63, hl = (e >> 9) & 1, c = (e >> 10) & 3,
                  ot = (e >> 12) & 1, net = e >> 13;
        const int row = 32 * ot + (lane & 31);
        const int col = 32 * (c >> 1) + rho(8 * (c & 1) + j, lane >> 5);
        const float w = -2.0f * (params[(net ? L.vf2W : L.pi2W) + row * kHid + col] * kTanhScale);
        const float whi = hi11_rn(w);
        fh[2 * oW2 + e] = to_f16(hl == 0 ? whi : w - whi);
    }
    // layers fed with r = (1 - tanh) / 2 (see rsig): W.tanh + b = (b + rowsum W) - 2 W.r
    for (int e = tid; e < 2 * kHid; e += nthreads) {
        const int net = e >> 6, row = e & 63;
        lds[oB1 + e] = params[(net ? L.vf0b : L.pi0b) + row] * kTanhScale;
        const float *w2 = params + (net ? L.vf2W : L.pi2W) + row * kHid;
        float sum = params[(net ? L.vf2b : L.pi2b) + row] * kTanhScale;
        for (int k = 0; k < kHid; ++k) sum += w2[k] * kTanhScale;
        lds[oB2 + e] = sum;
    }
    for (int e = tid; e < kHid; e += nthreads) {
        lds[oHA0 + e] = -2.0f * params[L.actW + e];
        lds[oHA1 + e] = -2.0f * params[L.actW + kHid + e];
        lds[oHV + e] = -2.0f * params[L.valW + e];
    }
    if (tid < 8) {
        float v = 0.0f;
        if (tid < 3) {  // head biases + rowsum of the head weights
            const float *w = params + (tid < 2 ? L.actW + tid * kHid : L.valW);
            v = params[tid < 2 ? L.actb + tid : L.valb];
            for (int k = 0; k < kHid; ++k) v += w[k];
        } else if (tid < 5) {
            v = params[L.logstd + tid - 3];
        }
        lds[oSc + tid] = v;
    }
    if (tid < 2) {  // the Gaussian's per-component constants (torch Normal, scale = exp(log_std))
        const float sd = expf(params[L.logstd + tid]);
        lds[oSc + 5 + tid] = sd;
        lds[oSc + 7 + tid] = 0.5f / (sd * sd);
        lds[oSc + 9 + tid] = logf(sd);
    }
}

// r = 1 / (1 + 2^y) = (1 - tanh(x)) / 2 for y = x * 2/ln2: v_exp_f32, v_add, v_rcp_f32.  The
// hidden layers hand r on instead of tanh = 1 - 2r; the next layer and the heads absorb the
// affine map (weights -2W, bias b + rowsum W, staged above), which saves the v_fma per unit.
__device__ __forceinline__ float rsig(float y) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y));
}

// Layer-1 B operand of a lane from its agent's observation row o[0..8) (zero-padded past D):
// half 0 carries the hi parts, half 1 the lo parts (see the mapping above).
__device__ __forceinline__ h8 obs_operand(const float (&o)[8], int h) {
    h8 hi, lo;
    split8(o, 0, hi, lo);
    return h == 0 ? hi : lo;
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

__device__ __forceinline__ f32x16 mma16(const h8 &a, const h8 &b, const f32x16 &c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// One network (net 0 actor / 1 critic) over one 32-agent tile: layer 1, tanh, layer 2, tanh.
// Leaves r(H2) = (1 - tanh(H2)) / 2, rows rho(reg, h) (+32*ot) of agent l&31, in c0 (ot 0) and
// c1 (ot 1).
__device__ __forceinline__ void net_tile(const float *lds, int net, const h8 &bo, int lane, int h,
                                         f32x16 &c0, f32x16 &c1) {
    const h8 *fr = reinterpret_cast<const h8 *>(lds) + lane;  // fragment f: fr[64 f]
    f32x16 a0 = bias_acc(lds + oB1 + net * kHid, 0, h);
    f32x16 a1 = bias_acc(lds + oB1 + net * kHid, 1, h);
    {
        const int f1 = oW1 / kFrag + net * 4;
        a0 = mma16(fr[64 * (f1 + 0)], bo, a0);
        a1 = mma16(fr[64 * (f1 + 2)], bo, a1);
        a0 = mma16(fr[64 * (f1 + 1)], bo, a0);
        a1 = mma16(fr[64 * (f1 + 3)], bo, a1);
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        a0[reg] = rsig(a0[reg]);
        a1[reg] = rsig(a1[reg]);
    }
    h8 bh[4], bl[4];
    split8(a0, 0, bh[0], bl[0]);
    split8(a0, 8, bh[1], bl[1]);
    split8(a1, 0, bh[2], bl[2]);
    split8(a1, 8, bh[3], bl[3]);
    c0 = bias_acc(lds + oB2 + net * kHid, 0, h);
    c1 = bias_acc(lds + oB2 + net * kHid, 1, h);
#if FENV_POLICY_PRIO
    __builtin_amdgcn_s_setprio(1);  // a wave in its MFMA phase wins issue arbitration
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int f0 = oW2 / kFrag + ((net * 2 + 0) * 4 + c) * 2;
        const int f1 = oW2 / kFrag + ((net * 2 + 1) * 4 + c) * 2;
        const h8 w0h = fr[64 * f0], w0l = fr[64 * (f0 + 1)];
        const h8 w1h = fr[64 * f1], w1l = fr[64 * (f1 + 1)];
        // small terms first
        c0 = mma16(w0h, bl[c], c0);
        c1 = mma16(w1h, bl[c], c1);
        c0 = mma16(w0l, bh[c], c0);
        c1 = mma16(w1l, bh[c], c1);
        c0 = mma16(w0h, bh[c], c0);
        c1 = mma16(w1h, bh[c], c1);
    }
#if FENV_POLICY_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        c0[reg] = rsig(c0[reg]);
        c1[reg] = rsig(c1[reg]);
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

// The Philox4x32-10 words (x, y) a row's Gaussian noise is made from (Box-Muller below):
// counter (row, offset), key seed.  The oracle regenerates them (policy_oracle.philox_normals).
__device__ __forceinline__ uint2 policy_noise_bits(int64_t row, uint64_t seed, uint64_t offset) {
    const uint4 r = philox4x32(make_uint4((uint32_t)row, (uint32_t)((uint64_t)row >> 32),
                                          (uint32_t)offset, (uint32_t)(offset >> 32)),
                               (uint32_t)seed, (uint32_t)(seed >> 32));
    return make_uint2(r.x, r.y);
}

// Full policy evaluation of one 32-agent tile.  bo = obs_operand(agent's observation row, h);
// nb = policy_noise_bits of the lane's agent (unused when deterministic); value_only skips the
// actor.
__device__ __forceinline__ PolicyLane policy_tile(const float *lds, const h8 &bo, int lane,
                                                  uint2 nb, bool deterministic, bool value_only) {
    const int h = lane >> 5;
    PolicyLane o;
    f32x16 c0, c1;
    float pa = 0.0f;
    if (!value_only) {
        net_tile(lds, 0, bo, lane, h, c0, c1);
        const float p0 = head_dot(lds + oHA0, c0, c1, h);
        const float p1 = head_dot(lds + oHA1, c0, c1, h);
        // keep component h: own partial + the partner half's partial of the same component
        const float other = __shfl_xor(h == 0 ? p1 : p0, 32, 64);
        pa = h == 0 ? p0 + other : other + p1;
    }
    __builtin_amdgcn_sched_barrier(0);  // actor, then critic: overlapping them costs registers
    net_tile(lds, 1, bo, lane, h, c0, c1);
    o.value = join_halves(head_dot(lds + oHV, c0, c1, h), h) + lds[oSc + 2];
    if (value_only) {
        o.mu = o.act = o.clip = o.logp = 0.0f;
        return o;
    }
    const float std_h = lds[oSc + 5 + h];
    o.mu = pa + lds[oSc + h];
    float a = o.mu;
    if (!deterministic) {
        const float u1 = (float)((nb.x >> 8) + 1u) * 0x1.0p-24f;  // (0, 1]
        const float u2 = (float)(nb.y >> 8) * 0x1.0p-24f;          // [0, 1)
        // Box-Muller on the hardware transcendentals: v_log_f32 is log2, v_sin/v_cos_f32 take
        // the angle in turns (sin(2 pi u2) directly, no range reduction needed for u2 in [0,1))
        const float rad = __builtin_amdgcn_sqrtf(-1.38629436111989061f * __builtin_amdgcn_logf(u1));
        const float eps = rad * (h == 0 ? __builtin_amdgcn_cosf(u2) : __builtin_amdgcn_sinf(u2));
        a = o.mu + std_h * eps;
    }
    o.act = a;
    o.clip = a < -1.0f ? -1.0f : (a > 1.0f ? 1.0f : a);
    // torch Normal.log_prob: -(a-mu)^2 / (2 var) - log(scale) - log(sqrt(2 pi)), scale = exp(ls)
    const float inv_2var = lds[oSc + 7 + h];
    const float d = a - o.mu;
    const float lp_h = -(d * d) * inv_2var - lds[oSc + 9 + h] - 0.918938533204672742f;
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
