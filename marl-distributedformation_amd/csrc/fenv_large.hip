// Large formations (N > kMaxN = 1024 agents per formation): the env kernels for formations too
// big for one workgroup's lanes and LDS slots (reference: /root/reference/simulate.py:70-254,
// which takes any num_agents_per_formation).
//
// Mapping.  One workgroup of kLT = 1024 threads per formation; thread j owns agents j, j + kLT,
// j + 2 kLT, ... of it.  The formation's scalars (goal, steps_since_reset, episode counter) live
// in every thread's registers for the whole launch; agent positions stay in HBM (the state
// arrays themselves), and the ring exchanges go through a per-agent scratch in global memory
// (16 B per agent, L2-resident for any realistic formation) with one workgroup barrier per
// exchange round: clipped positions -> individual rewards -> shared rewards -> observations.
// Same fp32 operations and order as env_step / env_obs (env_device.h), so the results are the
// reference's bit for bit.  These launches are rare-path code: correctness, not the roofline.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "env_device.h"

namespace fenvk {

constexpr int kLT = 1024;

// per-agent action of local step k (fenv_rollout's [T][A][2] input, or in-kernel Philox for
// fenv_rollout_random: the same words k_rollout_wave draws, computed per step)
template <bool RA>
__device__ __forceinline__ float2 lf_action(const Consts &c, const float2 *act, const ActGen &gen,
                                            int64_t A, int64_t a, int32_t k) {
    if (!RA) return act[(int64_t)k * A + a];
    const int64_t ga = c.f0 * c.N + a;
    const uint64_t gs = gen.offset + (uint64_t)k;
    const uint4 w = philox(make_uint4((uint32_t)ga, (uint32_t)((uint64_t)ga >> 32),
                                      (uint32_t)(gs >> 1), (uint32_t)(gs >> 33)),
                           gen.k0, gen.k1);
    const float2 ac = (gs & 1) ? make_float2((float)((int32_t)(w.z >> 8) - (1 << 23)) * 0x1.0p-23f,
                                             (float)((int32_t)(w.w >> 8) - (1 << 23)) * 0x1.0p-23f)
                               : make_float2((float)((int32_t)(w.x >> 8) - (1 << 23)) * 0x1.0p-23f,
                                             (float)((int32_t)(w.y >> 8) - (1 << 23)) * 0x1.0p-23f);
    if (gen.out) reinterpret_cast<float2 *>(gen.out)[(int64_t)k * A + a] = ac;
    return ac;
}

// compute_obs (simulate.py:150-174) of agent i from the positions in HBM: the neighbours'
// normalised positions are recomputed here with the same correctly rounded division, so they
// are the bits the neighbours compute for themselves.
template <int D>
__device__ __forceinline__ void lf_obs(const Consts &c, const DevState &st, int64_t a0, int i,
                                       float gx, float gy, float *dst) {
    const int N = c.N;
    const int ip = i == 0 ? N - 1 : i - 1, in = i == N - 1 ? 0 : i + 1;
    const float px = st.px[a0 + i], py = st.py[a0 + i];
    const float nx = div_const<400>(px), ny = div_const<600>(py);
    const float npx = div_const<400>(st.px[a0 + ip]), npy = div_const<600>(st.py[a0 + ip]);
    const float nnx = div_const<400>(st.px[a0 + in]), nny = div_const<600>(st.py[a0 + in]);
    float o[8];
    o[0] = nx;
    o[1] = ny;
    o[2] = npx - nx;
    o[3] = npy - ny;
    o[4] = nnx - nx;
    o[5] = nny - ny;
    if (D == 8) {
        o[6] = div_const<400>(gx - px);
        o[7] = div_const<600>(gy - py);
    }
    if (D == 8) {
        reinterpret_cast<float4 *>(dst)[0] = make_float4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<float4 *>(dst)[1] = make_float4(o[4], o[5], o[6], o[7]);
    } else {
        reinterpret_cast<float2 *>(dst)[0] = make_float2(o[0], o[1]);
        reinterpret_cast<float2 *>(dst)[1] = make_float2(o[2], o[3]);
        reinterpret_cast<float2 *>(dst)[2] = make_float2(o[4], o[5]);
    }
}

// {sum, sum} over the workgroup in a fixed order, into partial[f] (accumulated if `accum`)
__device__ __forceinline__ void lf_record(float rsum, float dsum, float2 *partial, int64_t f,
                                          bool accum) {
    __shared__ float2 red[kLT / 64];
    rsum = wave_sum(rsum);
    dsum = wave_sum(dsum);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_float2(rsum, dsum);
    __syncthreads();
    if (threadIdx.x == 0) {
        float2 v = red[0];
        for (int k = 1; k < kLT / 64; ++k) v = make_float2(v.x + red[k].x, v.y + red[k].y);
        if (accum) v = make_float2(partial[f].x + v.x, partial[f].y + v.y);
        partial[f] = v;
    }
}

// T fused steps of formation blockIdx.x (FormationSimulator.step, simulate.py:70-118).
template <int D, int MODE, bool RA>
__global__ __launch_bounds__(kLT) void k_rollout_large(Consts c, DevState st, DevPending p,
                                                       int32_t T, const float2 *__restrict__ act,
                                                       ActGen gen, float *__restrict__ obs,
                                                       float *__restrict__ rew,
                                                       uint8_t *__restrict__ done,
                                                       float2 *__restrict__ partial, bool accum) {
    const int N = c.N;
    const int64_t f = blockIdx.x;
    const int64_t A = c.F * (int64_t)N;
    const int64_t a0 = f * N;
    float *qx = p.lf, *qy = p.lf + A, *qind = p.lf + 2 * A, *qoob = p.lf + 3 * A;
    float gx = st.gx[f], gy = st.gy[f];
    int32_t t = st.t[f];
    uint32_t ep = st.ep[f];
    bool any_reset = false;
    float rsum = 0.f, dsum = 0.f;
    for (int32_t k = 0; k < T; ++k) {
        const int64_t row = (int64_t)k * A;
        // vectorized_env.py:69-70, simulate.py:82-90: move, out-of-bounds test, clip
        for (int i = threadIdx.x; i < N; i += kLT) {
            const float2 ac = lf_action<RA>(c, act, gen, A, a0 + i, k);
            const float x1 = st.px[a0 + i] + 10.0f * ac.x;
            const float y1 = st.py[a0 + i] + 10.0f * ac.y;
            const bool oob = (x1 <= 0.0f) | (y1 <= 0.0f) | (x1 >= kW) | (y1 >= kH);
            qx[a0 + i] = clip0(x1, kW);
            qy[a0 + i] = clip0(y1, kH);
            qoob[a0 + i] = oob ? 1.0f : 0.0f;
        }
        __syncthreads();
        // simulate.py:180-217: individual reward from the clipped positions of i-1, i, i+1
        for (int i = threadIdx.x; i < N; i += kLT) {
            const int ip = i == 0 ? N - 1 : i - 1, in = i == N - 1 ? 0 : i + 1;
            const float x = qx[a0 + i], y = qy[a0 + i];
            const float dg = norm2(x - gx, y - gy);
            const float drr = norm2(x - qx[a0 + in], y - qy[a0 + in]);
            const float drl = norm2(x - qx[a0 + ip], y - qy[a0 + ip]);
            const float ctg = dg < 100.0f ? 10.0f : 0.0f;
            const float rd = -0.1f * dg;
            const float rr = nb_reward(drr - c.d_nb);
            const float rl = nb_reward(drl - c.d_nb);
            float ind = ((rd + ctg) + rr) + rl;
            if (qoob[a0 + i] != 0.0f) ind = ind + -100.0f;
            qind[a0 + i] = ind;
        }
        __syncthreads();
        // simulate.py:223-236, :111-116: shared reward, done, auto-reset
        const bool dn = t > c.max_steps;
        float ngx = gx, ngy = gy;
        for (int i = threadIdx.x; i < N; i += kLT) {
            const int ip = i == 0 ? N - 1 : i - 1, in = i == N - 1 ? 0 : i + 1;
            const int64_t a = a0 + i;
            const float rw = c.c_self * qind[a] + c.c_nb * (qind[a0 + ip] + qind[a0 + in]);
            if (rew) rew[row + a] = rw;
            if (done) done[row + a] = (uint8_t)dn;
            rsum += rw;
            dsum += dn ? 1.0f : 0.0f;
            float px = qx[a], py = qy[a];
            if (dn) {
                p.term[a] = make_float4(px, py, gx, gy);
                draw_reset<MODE>(c, p, f, a, i, ep + 1, px, py, ngx, ngy);
            }
            st.px[a] = px;
            st.py[a] = py;
        }
        t += 1;
        if (dn) {
            t = 0;
            ep += 1;
            gx = ngx;
            gy = ngy;
            any_reset = true;
        }
        __syncthreads();
        if (obs)
            for (int i = threadIdx.x; i < N; i += kLT)
                lf_obs<D>(c, st, a0, i, gx, gy, obs + (row + a0 + i) * D);
    }
    if (threadIdx.x == 0) {
        st.t[f] = t;
        if (any_reset) {
            st.gx[f] = gx;
            st.gy[f] = gy;
            st.ep[f] = ep;
        }
    }
    if (partial) lf_record(rsum, dsum, partial, f, accum);
}

// reset (simulate.py:120-147) and/or compute_observations (vectorized_env.py:57-66)
template <int D, int MODE, bool RESET>
__global__ __launch_bounds__(kLT) void k_reset_obs_large(Consts c, DevState st, DevPending p,
                                                         float *obs) {
    const int N = c.N;
    const int64_t f = blockIdx.x;
    const int64_t a0 = f * N;
    float gx = st.gx[f], gy = st.gy[f];
    const uint32_t ep_new = st.ep[f] + 1;
    if (RESET) {
        for (int i = threadIdx.x; i < N; i += kLT) {
            float px, py;
            draw_reset<MODE>(c, p, f, a0 + i, i, ep_new, px, py, gx, gy);
            st.px[a0 + i] = px;
            st.py[a0 + i] = py;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            st.gx[f] = gx;
            st.gy[f] = gy;
            st.t[f] = 0;
            st.ep[f] = ep_new;
        }
    }
    if (obs)
        for (int i = threadIdx.x; i < N; i += kLT) lf_obs<D>(c, st, a0, i, gx, gy, obs + (a0 + i) * D);
}

// compute_metrics (simulate.py:238-254) + the logged reward components (:183-208), as
// metrics_body: per-agent values to the scratch (column-major, kMS columns), then one thread per
// column sums the formation's agents in order, in double.
constexpr int kMSL = 7;
__global__ __launch_bounds__(kLT) void k_metrics_large(Consts c, DevState st, DevPending p,
                                                       bool terminal, const float *rew,
                                                       float *out) {
    __shared__ double sums[kMSL + 1];
    const int N = c.N;
    const int64_t f = blockIdx.x;
    const int64_t A = c.F * (int64_t)N;
    const int64_t a0 = f * N;
    const float gx = st.gx[f], gy = st.gy[f];
    const bool term = terminal && st.t[f] == 0;
    float *sv = p.lf;  // [kMSL][A]
    for (int i = threadIdx.x; i < N; i += kLT) {
        const int ip = i == 0 ? N - 1 : i - 1, in = i == N - 1 ? 0 : i + 1;
        const int64_t a = a0 + i;
        const float px = st.px[a], py = st.py[a];
        const float dg = norm2(px - gx, py - gy);
        const float dr = norm2(px - st.px[a0 + in], py - st.py[a0 + in]);
        // the state the last step's reward scored: terminal state of a formation it reset
        float4 q = make_float4(px, py, gx, gy), qp, qn;
        if (term) {
            q = p.term[a];
            qp = p.term[a0 + ip];
            qn = p.term[a0 + in];
        } else {
            qp = make_float4(st.px[a0 + ip], st.py[a0 + ip], gx, gy);
            qn = make_float4(st.px[a0 + in], st.py[a0 + in], gx, gy);
        }
        const float qg = norm2(q.x - q.z, q.y - q.w);
        sv[0 * A + a] = dg;
        sv[1 * A + a] = dr;
        sv[2 * A + a] = rew ? rew[a] : 0.f;
        sv[3 * A + a] = qg < 100.0f ? 10.0f : 0.0f;
        sv[4 * A + a] = -0.1f * qg;
        sv[5 * A + a] = nb_reward(norm2(q.x - qn.x, q.y - qn.y) - c.d_nb);
        sv[6 * A + a] = nb_reward(norm2(q.x - qp.x, q.y - qp.y) - c.d_nb);
    }
    __syncthreads();
    const int col = threadIdx.x;
    if (col < kMSL) {
        double s = 0, s2 = 0;
        for (int k = 0; k < N; ++k) {
            const double d = sv[col * A + a0 + k];
            s += d;
            s2 += d * d;
        }
        sums[col] = s;
        if (col == 1) sums[kMSL] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double mr = sums[1] / N;
        float *o = out + f * kMetricCols;
        o[0] = (float)(sums[0] / N);
        o[1] = (float)mr;
        o[2] = (float)sqrt(fmax(0.0, (sums[kMSL] - N * mr * mr) / (N - 1)));
        o[3] = (float)(sums[2] / N);
        o[4] = (float)(sums[3] / N);
        o[5] = (float)(sums[4] / N);
        o[6] = (float)(sums[5] / N);
        o[7] = (float)(sums[6] / N);
    }
}

// ---------------------------------------------------------------- launchers
template <int D, int MODE>
static hipError_t rollout_large_dm(const Consts &c, const DevState &s, const DevPending &p,
                                   int32_t T, const float *act, float *obs, float *rew,
                                   uint8_t *done, float *partial, bool accum, hipStream_t st,
                                   const ActGen *gen) {
    const float2 *a2 = reinterpret_cast<const float2 *>(act);
    float2 *p2 = reinterpret_cast<float2 *>(partial);
    if (gen)
        hipLaunchKernelGGL((k_rollout_large<D, MODE, true>), dim3((unsigned)c.F), dim3(kLT), 0, st,
                           c, s, p, T, a2, *gen, obs, rew, done, p2, accum);
    else
        hipLaunchKernelGGL((k_rollout_large<D, MODE, false>), dim3((unsigned)c.F), dim3(kLT), 0,
                           st, c, s, p, T, a2, ActGen{}, obs, rew, done, p2, accum);
    return hipGetLastError();
}

hipError_t launch_rollout_large(const Consts &c, const DevState &s, const DevPending &p,
                                int32_t T, int32_t D, const float *act, float *obs, float *rew,
                                uint8_t *done, float *partial, bool accum, hipStream_t st,
                                const ActGen *gen) {
    const bool mt = c.reset_mode == FENV_RESET_MT19937;
    if (D == 8)
        return mt ? rollout_large_dm<8, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done,
                                                            partial, accum, st, gen)
                  : rollout_large_dm<8, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done,
                                                           partial, accum, st, gen);
    return mt ? rollout_large_dm<6, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done, partial,
                                                        accum, st, gen)
              : rollout_large_dm<6, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done, partial,
                                                       accum, st, gen);
}

template <int D>
static hipError_t reset_obs_large_d(const Consts &c, const DevState &s, const DevPending &p,
                                    bool do_reset, float *obs, hipStream_t st) {
    const dim3 g((unsigned)c.F), b(kLT);
    if (!do_reset)
        hipLaunchKernelGGL((k_reset_obs_large<D, FENV_RESET_PHILOX, false>), g, b, 0, st, c, s, p,
                           obs);
    else if (c.reset_mode == FENV_RESET_MT19937)
        hipLaunchKernelGGL((k_reset_obs_large<D, FENV_RESET_MT19937, true>), g, b, 0, st, c, s, p,
                           obs);
    else
        hipLaunchKernelGGL((k_reset_obs_large<D, FENV_RESET_PHILOX, true>), g, b, 0, st, c, s, p,
                           obs);
    return hipGetLastError();
}

hipError_t launch_reset_observe_large(const Consts &c, const DevState &s, const DevPending &p,
                                      int32_t D, bool do_reset, float *obs, hipStream_t st) {
    return D == 8 ? reset_obs_large_d<8>(c, s, p, do_reset, obs, st)
                  : reset_obs_large_d<6>(c, s, p, do_reset, obs, st);
}

hipError_t launch_metrics_large(const Consts &c, const DevState &s, const DevPending &p,
                                bool terminal, const float *rew, float *out, hipStream_t st) {
    hipLaunchKernelGGL(k_metrics_large, dim3((unsigned)c.F), dim3(kLT), 0, st, c, s, p, terminal,
                       rew, out);
    return hipGetLastError();
}

}  // namespace fenvk
