// gfx950 kernels for the batched formation env (reference: /root/reference/simulate.py:70-254,
// /root/reference/vectorized_env.py:52-82).
//
// Mapping.  One lane owns one agent for the whole launch; its position, its formation's goal,
// steps_since_reset and episode counter live in registers.  For N <= 64 a 64-lane wavefront
// holds fpw = 64/N whole formations (lanes fi*N .. fi*N+N-1), so every ring-neighbour exchange
// (simulate.py:162-167, 197-198, 223-229) is a ds_bpermute inside the wavefront: no LDS
// traffic, no barriers, waves are fully independent.  For N > 64 one workgroup holds one
// formation and exchanges through LDS with one barrier per exchange round.
//
// Numerics.  Bit-for-bit the reference's torch-CPU fp32: contraction is off for this file,
// division and sqrt are the correctly rounded IEEE ops, and the 2-vector norm is
// sqrtf(fmaf(y, y, x*x)) as torch's CPU linalg.norm computes it.  Every expression keeps the
// reference's operation order (comments cite the line).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "fenv.h"
#include "fenv_internal.h"

namespace fenvk {

constexpr float kW = 400.0f;  // simulate.py:13
constexpr float kH = 600.0f;  // simulate.py:14

__device__ __forceinline__ float norm2(float x, float y) {
    const float xx = x * x;
    return __builtin_sqrtf(__builtin_fmaf(y, y, xx));
}

// torch.clip(v, 0, hi) incl. NaN propagation (simulate.py:89-90)
__device__ __forceinline__ float clip0(float v, float hi) {
    return v < 0.0f ? 0.0f : (v > hi ? hi : v);
}

// - 0.01 * where(d < 0, d**2, d)   (simulate.py:204-205)
__device__ __forceinline__ float nb_reward(float d) { return -0.01f * (d < 0.0f ? d * d : d); }

// Philox4x32-10 (Salmon et al., SC'11), throughput-mode reset RNG.
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
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

// torch.rand float32 from 32 random bits: (r & 0xFFFFFF) * 2^-24 (exact).
__device__ __forceinline__ float u24(uint32_t r) { return (float)(r & 0xFFFFFFu) * 0x1.0p-24f; }

// simulate.py:133-143 for agent i of formation f (local indices), episode `ep_new`.
template <int MODE>
__device__ __forceinline__ void draw_reset(const Consts &c, const DevPending &p, int64_t f,
                                           int64_t a, int i, uint32_t ep_new, float &px,
                                           float &py, float &gx, float &gy) {
    if (MODE == FENV_RESET_MT19937) {
        px = p.px[a];
        py = p.py[a];
        gx = p.gx[f];
        gy = p.gy[f];
    } else {
        const uint64_t fg = (uint64_t)(c.f0 + f);
        const uint64_t ag = fg * (uint64_t)c.N + (uint64_t)i;
        const uint4 r = philox(make_uint4((uint32_t)ag, (uint32_t)(ag >> 32), ep_new, 0x41474E54u),
                               c.key0, c.key1);
        px = u24(r.x) * 400.0f;
        py = u24(r.y) * 100.0f;
        const uint4 g = philox(make_uint4((uint32_t)fg, (uint32_t)(fg >> 32), ep_new, 0x474F414Cu),
                               c.key0, c.key1);
        gx = u24(g.x) * 280.0f + 60.0f;
        gy = u24(g.y) * 480.0f + 60.0f;
    }
}

// ---------------------------------------------------------------- ring-neighbour exchange
// Four exchange rounds per env step: A {px,py}->next, B {drr}->prev, C {ind}->prev,next,
// D {nx,ny}->prev,next.

struct WaveX {  // N <= 64: lanes of one formation are contiguous in the wavefront
    int lp, ln;
    __device__ __forceinline__ void a_next(float u, float v, float &un, float &vn) const {
        un = __shfl(u, ln, 64);
        vn = __shfl(v, ln, 64);
    }
    __device__ __forceinline__ float b_prev(float v) const { return __shfl(v, lp, 64); }
    __device__ __forceinline__ void c_pn(float v, float &vp, float &vn) const {
        vp = __shfl(v, lp, 64);
        vn = __shfl(v, ln, 64);
    }
    __device__ __forceinline__ void d_pn(float u, float v, float &up, float &un, float &vp,
                                         float &vn) const {
        up = __shfl(u, lp, 64);
        un = __shfl(u, ln, 64);
        vp = __shfl(v, lp, 64);
        vn = __shfl(v, ln, 64);
    }
};

constexpr int kMaxN = 1024;

// N > 64: one formation per workgroup, slots in LDS.  Each slot's next write is separated from
// its previous reads by at least one barrier (rounds are used in the order A,B,C,D).
struct BlockX {
    float *lds;  // 6 * kMaxN floats
    int i, ip, in;
    __device__ __forceinline__ void a_next(float u, float v, float &un, float &vn) const {
        lds[0 * kMaxN + i] = u;
        lds[1 * kMaxN + i] = v;
        __syncthreads();
        un = lds[0 * kMaxN + in];
        vn = lds[1 * kMaxN + in];
    }
    __device__ __forceinline__ float b_prev(float v) const {
        lds[2 * kMaxN + i] = v;
        __syncthreads();
        return lds[2 * kMaxN + ip];
    }
    __device__ __forceinline__ void c_pn(float v, float &vp, float &vn) const {
        lds[3 * kMaxN + i] = v;
        __syncthreads();
        vp = lds[3 * kMaxN + ip];
        vn = lds[3 * kMaxN + in];
    }
    __device__ __forceinline__ void d_pn(float u, float v, float &up, float &un, float &vp,
                                         float &vn) const {
        lds[4 * kMaxN + i] = u;
        lds[5 * kMaxN + i] = v;
        __syncthreads();
        up = lds[4 * kMaxN + ip];
        un = lds[4 * kMaxN + in];
        vp = lds[5 * kMaxN + ip];
        vn = lds[5 * kMaxN + in];
    }
};

// ---------------------------------------------------------------- one env step of one agent
struct Agent {
    float px, py, gx, gy;
    int32_t t;
    uint32_t ep;
};

// FormationSimulator.step (simulate.py:70-118) for this lane's agent.  Returns the reward
// (pre-reset state) and done; leaves the post-(auto-)reset state in `s`.
template <int MODE, class X>
__device__ __forceinline__ void env_step(const Consts &c, const DevPending &p, const X &x,
                                         int64_t f, int64_t a, int i, float2 act, Agent &s,
                                         float &rw, bool &dn, bool &did_reset) {
    // vectorized_env.py:69-70 (v = 10 * a), simulate.py:82 (agents += v)
    const float x1 = s.px + 10.0f * act.x;
    const float y1 = s.py + 10.0f * act.y;
    // simulate.py:86-87: out of bounds tested on the unclipped position
    const bool oob = (x1 <= 0.0f) | (y1 <= 0.0f) | (x1 >= kW) | (y1 >= kH);
    s.px = clip0(x1, kW);
    s.py = clip0(y1, kH);

    // compute_reward_and_done, simulate.py:180-211
    const float dg = norm2(s.px - s.gx, s.py - s.gy);
    float pnx, pny;
    x.a_next(s.px, s.py, pnx, pny);
    const float drr = norm2(s.px - pnx, s.py - pny);  // ||p_i - p_{i+1}||  (:197)
    const float drl = x.b_prev(drr);                  // ||p_i - p_{i-1}|| == drr_{i-1} bitwise
    const float ctg = dg < 100.0f ? 10.0f : 0.0f;     // :183-187
    const float rd = -0.1f * dg;                      // :191
    const float rr = nb_reward(drr - c.d_nb);         // :202-205
    const float rl = nb_reward(drl - c.d_nb);
    float ind = ((rd + ctg) + rr) + rl;               // :211
    if (oob) ind = ind + -100.0f;                     // :214-217 (else + (-0.0): identity)
    float ip, in;
    x.c_pn(ind, ip, in);
    rw = c.c_self * ind + c.c_nb * (ip + in);         // :228-229

    dn = s.t > c.max_steps;                           // :231 (before the increment at :111)
    s.t += 1;
    did_reset = false;
    if (dn) {                                         // :113-116 auto-reset
        const uint32_t ep_new = s.ep + 1;
        draw_reset<MODE>(c, p, f, a, i, ep_new, s.px, s.py, s.gx, s.gy);
        s.t = 0;
        s.ep = ep_new;
        did_reset = true;
    }
}

// compute_obs (simulate.py:150-174) of this lane's agent into o[0..D).
template <int D, class X>
__device__ __forceinline__ void env_obs(const X &x, const Agent &s, float (&o)[8]) {
    const float nx = s.px / kW;  // :156, normalise first
    const float ny = s.py / kH;
    float npx, nnx, npy, nny;
    x.d_pn(nx, ny, npx, nnx, npy, nny);
    o[0] = nx;
    o[1] = ny;
    o[2] = npx - nx;  // :166
    o[3] = npy - ny;
    o[4] = nnx - nx;  // :167
    o[5] = nny - ny;
    if (D == 8) {
        o[6] = (s.gx - s.px) / kW;  // :172, subtract first, then divide
        o[7] = (s.gy - s.py) / kH;
    }
}

// Wave-cooperative store of the wave's observation rows.  Lanes 0..M-1 own the rows of M
// consecutive agents starting at `dst`; each lane stages its D floats in the wave's private
// LDS slice (2 KiB) and the wave then writes the whole contiguous span with full-width vector
// stores (1 KiB per instruction) instead of 64 strided rows (tools/ubench_hbm: 3.45 -> 4.7 TB/s
// on this access pattern).  No barrier: the slice is private to the wave and a wave's LDS
// operations complete in order.
template <int D>
__device__ __forceinline__ void store_obs_rows(float *stage, const float (&o)[8], int lane, int M,
                                               float *dst) {
    if (D == 8) {
        reinterpret_cast<float4 *>(stage)[2 * lane] = make_float4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<float4 *>(stage)[2 * lane + 1] = make_float4(o[4], o[5], o[6], o[7]);
    } else {
        reinterpret_cast<float2 *>(stage)[3 * lane] = make_float2(o[0], o[1]);
        reinterpret_cast<float2 *>(stage)[3 * lane + 1] = make_float2(o[2], o[3]);
        reinterpret_cast<float2 *>(stage)[3 * lane + 2] = make_float2(o[4], o[5]);
    }
    __builtin_amdgcn_wave_barrier();
    const int nf = M * D;
    if (((reinterpret_cast<uintptr_t>(dst) & 15) == 0) && ((nf & 3) == 0)) {
        const int nq = nf >> 2;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int q = lane + 64 * k;
            if (q < nq)
                reinterpret_cast<float4 *>(dst)[q] = reinterpret_cast<const float4 *>(stage)[q];
        }
    } else {
        const int nq = nf >> 1;  // D is even, rows are 8-byte aligned
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = lane + 64 * k;
            if (q < nq)
                reinterpret_cast<float2 *>(dst)[q] = reinterpret_cast<const float2 *>(stage)[q];
        }
    }
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// ---------------------------------------------------------------- fused T-step rollout
template <int D, int MODE, class X>
__device__ __forceinline__ void rollout_body(const Consts &c, const DevState &st,
                                             const DevPending &p, const X &x, bool active,
                                             int64_t f, int64_t a, int i, float *stage, int lane,
                                             int M, int64_t a_first, int32_t T,
                                             const float2 *__restrict__ act,
                                             float *__restrict__ obs, float *__restrict__ rew,
                                             uint8_t *__restrict__ done, float &rsum,
                                             float &dsum) {
    const int64_t A = c.F * (int64_t)c.N;
    Agent s{0.f, 0.f, 0.f, 0.f, 0, 0u};
    if (active) {
        s.px = st.px[a];
        s.py = st.py[a];
        s.gx = st.gx[f];
        s.gy = st.gy[f];
        s.t = st.t[f];
        s.ep = st.ep[f];
    }
    bool any_reset = false;
    // Rolling action prefetch: a ring of kPF registers keeps the loads of the next kPF steps in
    // flight while a step computes (kPF = 1: load step k+1 during step k).
#ifndef FENV_ACT_PREFETCH
#define FENV_ACT_PREFETCH 1
#endif
    constexpr int kPF = FENV_ACT_PREFETCH;
    float2 ring[kPF];
#pragma unroll
    for (int j = 0; j < kPF; ++j)
        ring[j] = (active && j < T) ? act[(int64_t)j * A + a] : make_float2(0.f, 0.f);
    for (int32_t k0 = 0; k0 < T; k0 += kPF) {
#pragma unroll
        for (int j = 0; j < kPF; ++j) {
            const int32_t k = k0 + j;
            if (k >= T) break;
            const float2 ac = ring[j];
            if (active && k + kPF < T) ring[j] = act[(int64_t)(k + kPF) * A + a];
            float rw;
            bool dn, rs;
            env_step<MODE>(c, p, x, f, a, i, ac, s, rw, dn, rs);
            any_reset |= rs;
            const int64_t row = (int64_t)k * A + a;
            float o[8];
            env_obs<D>(x, s, o);
            if (obs) store_obs_rows<D>(stage, o, lane, M, obs + ((int64_t)k * A + a_first) * D);
            if (active) {
                if (rew) rew[row] = rw;
                if (done) done[row] = (uint8_t)dn;
                rsum += rw;
                dsum += dn ? 1.0f : 0.0f;
            }
        }
    }
    if (active) {
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

template <int D, int MODE>
__global__ __launch_bounds__(256) void k_rollout_wave(Consts c, DevState st, DevPending p,
                                                      int32_t T, const float2 *__restrict__ act,
                                                      float *__restrict__ obs,
                                                      float *__restrict__ rew,
                                                      uint8_t *__restrict__ done,
                                                      float2 *__restrict__ partial,
                                                      bool accum) {
    // No early exit for waves past the last formation: they idle through the loop with every
    // lane inactive so that the workgroup reduction below can use a barrier.
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8];
    __shared__ float2 red[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int N = c.N;
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = wave * c.fpw + fi;
    const bool active = fi < c.fpw && f < c.F;
    const int64_t a = f * N + i;
    WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    const int64_t f_first = wave * c.fpw;
    const int64_t f_left = c.F - f_first;
    const int M = (int)((f_left <= 0 ? 0 : (f_left < c.fpw ? f_left : c.fpw)) * N);
    float rsum = 0.f, dsum = 0.f;
    if (M > 0)
        rollout_body<D, MODE>(c, st, p, x, active, f, a, i, stage[w], lane, M, f_first * N, T,
                              act, obs, rew, done, rsum, dsum);
    if (partial) {  // one {sum reward, sum done} record per workgroup, fixed summation order
        rsum = wave_sum(rsum);
        dsum = wave_sum(dsum);
        if (lane == 0) red[w] = make_float2(rsum, dsum);
        __syncthreads();
        if (threadIdx.x == 0) {
            float2 v = red[0];
            for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
                v = make_float2(v.x + red[k].x, v.y + red[k].y);
            if (accum) v = make_float2(partial[blockIdx.x].x + v.x, partial[blockIdx.x].y + v.y);
            partial[blockIdx.x] = v;
        }
    }
}

template <int D, int MODE>
__global__ __launch_bounds__(1024) void k_rollout_block(Consts c, DevState st, DevPending p,
                                                        int32_t T,
                                                        const float2 *__restrict__ act,
                                                        float *__restrict__ obs,
                                                        float *__restrict__ rew,
                                                        uint8_t *__restrict__ done,
                                                        float2 *__restrict__ partial,
                                                        bool accum) {
    __shared__ float lds[6 * kMaxN];
    __shared__ float red[2][kMaxN / 64];
    const int N = c.N;
    const int i = threadIdx.x;
    const int64_t f = blockIdx.x;
    const bool active = i < N;
    const int64_t a = f * N + i;
    BlockX x{lds, i, active ? (i == 0 ? N - 1 : i - 1) : i, active ? (i == N - 1 ? 0 : i + 1) : i};
    __shared__ __attribute__((aligned(16))) float stage[kMaxN / 64][64 * 8];
    const int w = i >> 6;
    const int M = N - 64 * w < 64 ? (N - 64 * w > 0 ? N - 64 * w : 0) : 64;
    float rsum = 0.f, dsum = 0.f;
    rollout_body<D, MODE>(c, st, p, x, active, f, a, i, stage[w], i & 63, M, f * N + 64 * w, T,
                          act, obs, rew, done, rsum, dsum);
    if (partial) {
        rsum = wave_sum(rsum);
        dsum = wave_sum(dsum);
        const int w = i >> 6, nw = blockDim.x >> 6;
        if ((i & 63) == 0) {
            red[0][w] = rsum;
            red[1][w] = dsum;
        }
        __syncthreads();
        if (i == 0) {
            float r = 0.f, d = 0.f;
            for (int k = 0; k < nw; ++k) {
                r += red[0][k];
                d += red[1][k];
            }
            if (accum) {
                r = partial[f].x + r;
                d = partial[f].y + d;
            }
            partial[f] = make_float2(r, d);
        }
    }
}

// ---------------------------------------------------------------- reset + observe
template <int D, int MODE, bool RESET, class X>
__device__ __forceinline__ void reset_obs_body(const Consts &c, const DevState &st,
                                               const DevPending &p, const X &x, bool active,
                                               int64_t f, int64_t a, int i, float *stage,
                                               int lane, int M, int64_t a_first, float *obs) {
    Agent s{0.f, 0.f, 0.f, 0.f, 0, 0u};
    if (active) {
        if (RESET) {
            const uint32_t ep_new = st.ep[f] + 1;
            draw_reset<MODE>(c, p, f, a, i, ep_new, s.px, s.py, s.gx, s.gy);
            s.t = 0;
            s.ep = ep_new;
        } else {
            s.px = st.px[a];
            s.py = st.py[a];
            s.gx = st.gx[f];
            s.gy = st.gy[f];
        }
    }
    float o[8];
    env_obs<D>(x, s, o);
    if (obs) store_obs_rows<D>(stage, o, lane, M, obs + a_first * D);
    if (RESET && active) {
        st.px[a] = s.px;
        st.py[a] = s.py;
        if (i == 0) {
            st.gx[f] = s.gx;
            st.gy[f] = s.gy;
            st.t[f] = 0;
            st.ep[f] = s.ep;
        }
    }
}

template <int D, int MODE, bool RESET>
__global__ __launch_bounds__(256) void k_reset_obs_wave(Consts c, DevState st, DevPending p,
                                                        float *obs) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave * c.fpw >= c.F) return;
    const int N = c.N;
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = wave * c.fpw + fi;
    const bool active = fi < c.fpw && f < c.F;
    WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8];
    const int64_t f_first = wave * c.fpw;
    const int M = (int)((c.F - f_first < c.fpw ? c.F - f_first : c.fpw) * N);
    reset_obs_body<D, MODE, RESET>(c, st, p, x, active, f, f * N + i, i, stage[threadIdx.x >> 6],
                                   lane, M, f_first * N, obs);
}

template <int D, int MODE, bool RESET>
__global__ __launch_bounds__(1024) void k_reset_obs_block(Consts c, DevState st, DevPending p,
                                                          float *obs) {
    __shared__ float lds[6 * kMaxN];
    const int N = c.N;
    const int i = threadIdx.x;
    const int64_t f = blockIdx.x;
    const bool active = i < N;
    BlockX x{lds, i, active ? (i == 0 ? N - 1 : i - 1) : i, active ? (i == N - 1 ? 0 : i + 1) : i};
    __shared__ __attribute__((aligned(16))) float stage[kMaxN / 64][64 * 8];
    const int w = i >> 6;
    const int M = N - 64 * w < 64 ? (N - 64 * w > 0 ? N - 64 * w : 0) : 64;
    reset_obs_body<D, MODE, RESET>(c, st, p, x, active, f, f * N + i, i, stage[w], i & 63, M,
                                   f * N + 64 * w, obs);
}

// ---------------------------------------------------------------- metrics (simulate.py:238-254)
// Per formation: mean ||p - goal||, mean ||p_i - p_{i+1}||, its unbiased std, mean reward.
// Each formation's values are staged in LDS and summed by its first lane in agent order
// (deterministic), in double.
template <class X>
__device__ __forceinline__ void metrics_body(const Consts &c, const DevState &st, const X &x,
                                             bool active, int64_t f, int64_t a, int i,
                                             const float *rew, float *stage, int base,
                                             float *out) {
    float px = 0.f, py = 0.f, gx = 0.f, gy = 0.f, r = 0.f;
    if (active) {
        px = st.px[a];
        py = st.py[a];
        gx = st.gx[f];
        gy = st.gy[f];
        r = rew ? rew[a] : 0.f;
    }
    float pnx, pny;
    x.a_next(px, py, pnx, pny);
    const float dg = norm2(px - gx, py - gy);
    const float dr = norm2(px - pnx, py - pny);
    const int N = c.N;
    stage[3 * (base + i) + 0] = dg;
    stage[3 * (base + i) + 1] = dr;
    stage[3 * (base + i) + 2] = r;
    __syncthreads();
    if (active && i == 0) {
        double sg = 0, sr = 0, sr2 = 0, rw = 0;
        for (int k = 0; k < N; ++k) {
            const double d = stage[3 * (base + k) + 1];
            sg += stage[3 * (base + k) + 0];
            sr += d;
            sr2 += d * d;
            rw += stage[3 * (base + k) + 2];
        }
        const double mr = sr / N;
        out[f * 4 + 0] = (float)(sg / N);
        out[f * 4 + 1] = (float)mr;
        out[f * 4 + 2] = N > 1 ? (float)sqrt(fmax(0.0, (sr2 - N * mr * mr) / (N - 1)))
                               : __builtin_nanf("");
        out[f * 4 + 3] = (float)(rw / N);
    }
}

__global__ __launch_bounds__(256) void k_metrics_wave(Consts c, DevState st, const float *rew,
                                                      float *out) {
    __shared__ float stage[3 * 256];
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int N = c.N;
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = wave * c.fpw + fi;
    const bool active = fi < c.fpw && f < c.F;
    WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    metrics_body(c, st, x, active, f, f * N + i, i, rew, stage, (threadIdx.x & ~63) + fi * N,
                 out);
}

__global__ __launch_bounds__(1024) void k_metrics_block(Consts c, DevState st, const float *rew,
                                                        float *out) {
    __shared__ float lds[6 * kMaxN];
    __shared__ float stage[3 * kMaxN];
    const int N = c.N;
    const int i = threadIdx.x;
    const int64_t f = blockIdx.x;
    const bool active = i < N;
    BlockX x{lds, i, active ? (i == 0 ? N - 1 : i - 1) : i, active ? (i == N - 1 ? 0 : i + 1) : i};
    metrics_body(c, st, x, active, f, f * N + i, i, rew, stage, 0, out);
}

// ---------------------------------------------------------------- deterministic reductions
// One workgroup; thread k sums elements k, k+1024, ... in double; then a fixed tree.
template <int K, class T>
__global__ __launch_bounds__(1024) void k_reduce_rows(const T *in, int64_t rows, double *out) {
    __shared__ double red[K][1024];
    double acc[K][4];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[j][u] = 0.0;
    // 4 independent rows in flight per thread per iteration (fixed assignment: deterministic)
    int64_t r = threadIdx.x;
    for (; r + 3 * 1024 < rows; r += 4 * 1024) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) acc[j][u] += (double)in[(r + u * 1024) * K + j];
    }
    for (; r < rows; r += 1024)
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j][0] += (double)in[r * K + j];
#pragma unroll
    for (int j = 0; j < K; ++j) red[j][threadIdx.x] = (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
#pragma unroll
            for (int j = 0; j < K; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < K; ++j) out[j] = red[j][0];
    }
}

// ---------------------------------------------------------------- fp probe (diagnostic)
__global__ void k_fp_probe(int32_t op, const float *a, const float *b, float *out, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const float x = a[k];
        float r;
        switch (op) {
            case 0: r = x / kW; break;
            case 1: r = x / kH; break;
            case 2: r = __builtin_sqrtf(x); break;
            default: r = norm2(x, b[k]); break;
        }
        out[k] = r;
    }
}

// ---------------------------------------------------------------- launchers
int64_t group_count(const Consts &c) {
    if (wave_path(c.N)) return ((c.F + c.fpw - 1) / c.fpw + 3) / 4;  // 4-wave workgroups
    return c.F;
}

static inline unsigned block_threads(int32_t N) { return (unsigned)((N + 63) / 64 * 64); }

template <int D, int MODE>
static hipError_t rollout_dm(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                             const float *act, float *obs, float *rew, uint8_t *done,
                             float *partial, bool accum, hipStream_t st) {
    const float2 *a2 = reinterpret_cast<const float2 *>(act);
    float2 *p2 = reinterpret_cast<float2 *>(partial);
    if (wave_path(c.N)) {
        const unsigned blocks = (unsigned)group_count(c);
        hipLaunchKernelGGL((k_rollout_wave<D, MODE>), dim3(blocks), dim3(256), 0, st, c, s, p, T,
                           a2, obs, rew, done, p2, accum);
    } else {
        hipLaunchKernelGGL((k_rollout_block<D, MODE>), dim3((unsigned)c.F), dim3(block_threads(c.N)),
                           0, st, c, s, p, T, a2, obs, rew, done, p2, accum);
    }
    return hipGetLastError();
}

hipError_t launch_rollout(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                          int32_t D, const float *act, float *obs, float *rew, uint8_t *done,
                          float *partial, bool accum, hipStream_t st) {
    const bool mt = c.reset_mode == FENV_RESET_MT19937;
    if (D == 8)
        return mt ? rollout_dm<8, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done, partial, accum, st)
                  : rollout_dm<8, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done, partial, accum, st);
    return mt ? rollout_dm<6, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done, partial, accum, st)
              : rollout_dm<6, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done, partial, accum, st);
}

template <int D, int MODE, bool RESET>
static hipError_t reset_obs_dmr(const Consts &c, const DevState &s, const DevPending &p,
                                float *obs, hipStream_t st) {
    if (wave_path(c.N)) {
        hipLaunchKernelGGL((k_reset_obs_wave<D, MODE, RESET>), dim3((unsigned)group_count(c)),
                           dim3(256), 0, st, c, s, p, obs);
    } else {
        hipLaunchKernelGGL((k_reset_obs_block<D, MODE, RESET>), dim3((unsigned)c.F),
                           dim3(block_threads(c.N)), 0, st, c, s, p, obs);
    }
    return hipGetLastError();
}

template <int D>
static hipError_t reset_obs_d(const Consts &c, const DevState &s, const DevPending &p,
                              bool do_reset, float *obs, hipStream_t st) {
    if (!do_reset) return reset_obs_dmr<D, FENV_RESET_PHILOX, false>(c, s, p, obs, st);
    if (c.reset_mode == FENV_RESET_MT19937)
        return reset_obs_dmr<D, FENV_RESET_MT19937, true>(c, s, p, obs, st);
    return reset_obs_dmr<D, FENV_RESET_PHILOX, true>(c, s, p, obs, st);
}

hipError_t launch_reset_observe(const Consts &c, const DevState &s, const DevPending &p,
                                int32_t D, bool do_reset, float *obs, hipStream_t st) {
    return D == 8 ? reset_obs_d<8>(c, s, p, do_reset, obs, st)
                  : reset_obs_d<6>(c, s, p, do_reset, obs, st);
}

hipError_t launch_metrics(const Consts &c, const DevState &s, const float *rew, float *out,
                          double *sums, double *scratch, hipStream_t st) {
    (void)scratch;
    if (wave_path(c.N)) {
        hipLaunchKernelGGL(k_metrics_wave, dim3((unsigned)group_count(c)), dim3(256), 0, st, c,
                           s, rew, out);
    } else {
        hipLaunchKernelGGL(k_metrics_block, dim3((unsigned)c.F), dim3(block_threads(c.N)), 0, st,
                           c, s, rew, out);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || sums == nullptr) return e;
    hipLaunchKernelGGL((k_reduce_rows<4, float>), dim3(1), dim3(1024), 0, st, out, c.F, sums);
    return hipGetLastError();
}

hipError_t launch_reduce_partials(const float *partial, int64_t count, double *out,
                                  hipStream_t st) {
    hipLaunchKernelGGL((k_reduce_rows<2, float>), dim3(1), dim3(1024), 0, st, partial, count, out);
    return hipGetLastError();
}

hipError_t launch_fp_probe(int32_t op, const float *a, const float *b, float *out, int64_t n,
                           hipStream_t st) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_fp_probe, dim3((unsigned)blocks), dim3(256), 0, st, op, a, b, out, n);
    return hipGetLastError();
}

}  // namespace fenvk
