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

#include "env_device.h"

namespace fenvk {

// ---------------------------------------------------------------- fused T-step rollout
// Synthetic action component in [-1, 1) from 24 random bits, exactly: (w >> 8) / 2^23 - 1.
__device__ __forceinline__ float act_u24(uint32_t w) {
    return (float)((int32_t)(w >> 8) - (1 << 23)) * 0x1.0p-23f;
}

// Workgroup-staged reward/done rows (k_rollout_wave_rs): the kRS waves of a workgroup cover one
// contiguous agent slice (8 x 60 = 480 agents at N = 5: a 1,920-B reward row = 15 whole 128-B
// lines, where a wave's own 240-B row straddles lines shared with its neighbours).  Rewards and
// dones of kRSTB steps are buffered in LDS and written as whole slice rows after one barrier;
// observations and actions stay per wave (their rows are already 128-B-line multiples).
#ifndef FENV_RS
#define FENV_RS 1  // 0: k_rollout_wave with per-wave reward/done stores
#endif
#ifndef FENV_RS_TB
#define FENV_RS_TB 8
#endif
// action-prefetch depth of the staged kernel (1: step k + 1's actions load during step k)
#ifndef FENV_RS_PF
#define FENV_RS_PF 1
#endif
// Register budget: left to the compiler for the Philox kernels (69 VGPRs -> 7 waves/SIMD).  The
// MT19937 kernel with HBM actions is held to 7 waves/SIMD too: left alone it takes 73 VGPRs (6
// waves); at 72 it spills only SGPRs (to VGPR lanes) and its rollout runs 1 % faster
// (profiles/r5_mt_mode/occupancy_ab, 3 interleaved rounds).  Forcing 64 VGPRs (8 waves) spills VGPRs and runs
// ~12 % slower (archive: tools/env_ab.sh).
#ifndef FENV_RS_OCC
#define FENV_RS_OCC __attribute__((amdgpu_waves_per_eu((MODE == 0 && !RA) ? 7 : 1)))
#endif
constexpr int kRS = 8;
constexpr int kRSA = 64 * kRS;
constexpr int kRSTB = FENV_RS_TB;

struct RSStage {
    float *rbuf;    // [kRSTB][kRSA]
    uint8_t *dbuf;  // [kRSTB][kRSA]
    int li;         // this lane's slot in the slice (w * agents-per-wave + lane)
    int nwg;        // agents in the slice
    int64_t g0;     // first agent of the slice
};

// rows [kfirst, kfirst + nrows) of the slice from the LDS buffers (all kRSA threads).  Vector
// path: thread (c4 = tid & 127, tid >> 7) stores 16 B of reward / 4 B of done per row, 4 rows per
// pass (a slice has at most kRSA = 512 agents = 128 float4).
template <bool NT>
__device__ __forceinline__ void rs_flush(const RSStage &r, int kfirst, int nrows, int64_t A,
                                         float *__restrict__ rew, uint8_t *__restrict__ done) {
    const int tid = threadIdx.x, n = r.nwg;
    const int c4 = tid & 127, r0 = tid >> 7;
    const bool vec = ((n | (int)(A & 3)) & 3) == 0;
    if (rew) {
        float *base = rew + (int64_t)kfirst * A + r.g0;
        if (vec && (reinterpret_cast<uintptr_t>(base) & 15) == 0) {
            if (c4 < (n >> 2))
                for (int row = r0; row < nrows; row += 4)
                    st_out<NT>(reinterpret_cast<float4 *>(base + (int64_t)row * A) + c4,
                           reinterpret_cast<const float4 *>(r.rbuf + row * kRSA)[c4]);
        } else if (tid < n) {
            for (int row = 0; row < nrows; ++row)
                base[(int64_t)row * A + tid] = r.rbuf[row * kRSA + tid];
        }
    }
    if (done) {
        uint8_t *base = done + (int64_t)kfirst * A + r.g0;
        if (vec && (reinterpret_cast<uintptr_t>(base) & 3) == 0) {
            if (c4 < (n >> 2))
                for (int row = r0; row < nrows; row += 4)
                    st_out<NT>(reinterpret_cast<uint32_t *>(base + (int64_t)row * A) + c4,
                           reinterpret_cast<const uint32_t *>(r.dbuf + row * kRSA)[c4]);
        } else if (tid < n) {
            for (int row = 0; row < nrows; ++row)
                base[(int64_t)row * A + tid] = r.dbuf[row * kRSA + tid];
        }
    }
}

// Roles of a wave in rollout_body.  kRoleAll: the whole step.  The split kernel (small grids,
// k_rollout_wave_split) gives one formation group two waves that both carry the state (the
// kinematics, done and auto-reset are recomputed bit-identically by each): kRoleState writes
// reward / done / the stats sums / the terminal and final state, kRoleObs only the observations.
// (A third role splitting the observations by step parity measured slower at config 1,
// profiles/ab/r3_config1_split3_ab.txt; source at commit 2c54623.)
constexpr int kRoleAll = 0, kRoleState = 1, kRoleObs = 2;

template <int D, int MODE, bool RA, bool RS, int PF, class X, int ROLE = kRoleAll, bool NT = false>
__device__ __forceinline__ void rollout_body(const Consts &c, const DevState &st,
                                             const DevPending &p, const X &x, bool active,
                                             int64_t f, int64_t a, int i, float *stage, int lane,
                                             int M, int64_t a_first, int32_t T,
                                             const float2 *__restrict__ act, const ActGen &gen,
                                             float *__restrict__ obs, float *__restrict__ rew,
                                             uint8_t *__restrict__ done, float &rsum,
                                             float &dsum, const RSStage &rsg = RSStage{}) {
    const int64_t A = c.F * (int64_t)c.N;
    constexpr bool kObsR = ROLE == kRoleObs;
    Agent s{0.f, 0.f, 0.f, 0.f, 0, 0u};
    if (active) {
        s.px = st.px[a];
        s.py = st.py[a];
        s.gx = st.gx[f];
        s.gy = st.gy[f];
        s.t = st.t[f];
        s.ep = st.ep[f];
    }
    // split kernel: every wave of the workgroup has read the state before a kRoleState wave
    // may write it back (the partner kRoleObs wave of the same formations sits in the same
    // workgroup)
    if (ROLE != kRoleAll) __syncthreads();
    bool any_reset = false;
    // Rolling action prefetch: a ring of kPF registers keeps the loads of the next kPF steps in
    // flight while a step computes (kPF = 1: load step k+1 during step k).  The step loop is
    // unrolled by kPF, which also lets the scheduler overlap one step's observation / reward
    // tail with the next step's head: what a latency-bound small grid wants (see use_pf).
    // staged rows: FENV_RS_PF steps (the chunk loop below is unrolled by it); in-kernel actions:
    // one step
    constexpr int kPF = RA ? 1 : (RS ? FENV_RS_PF : PF);
    float2 ring[kPF];
    const int64_t ga = c.f0 * c.N + a;  // global agent index (shard-invariant actions)
    uint4 words = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int j = 0; j < kPF; ++j)
        ring[j] = (!RA && active && j < T) ? act[(int64_t)j * A + a] : make_float2(0.f, 0.f);
    // one env step k with action slot j of the prefetch ring
    auto step = [&](int32_t k, int j) {
        float2 ac = ring[j];
        if (RA) {
            const uint64_t gs = gen.offset + (uint64_t)k;
            if (k == 0 || (gs & 1) == 0)
                words = philox(make_uint4((uint32_t)ga, (uint32_t)((uint64_t)ga >> 32),
                                          (uint32_t)(gs >> 1), (uint32_t)(gs >> 33)),
                               gen.k0, gen.k1);
            ac = (gs & 1) ? make_float2(act_u24(words.z), act_u24(words.w))
                          : make_float2(act_u24(words.x), act_u24(words.y));
            if (!kObsR && gen.out && active)
                reinterpret_cast<float2 *>(gen.out)[(int64_t)k * A + a] = ac;
        } else if (active && k + kPF < T) {
            ring[j] = act[(int64_t)(k + kPF) * A + a];
        }
        float rw;
        bool dn, rs;
        env_step<MODE, X, !kObsR>(c, p, x, f, a, i, active, ac, s, rw, dn, rs);
        any_reset |= rs;
        const int64_t row = (int64_t)k * A + a;
        if (ROLE != kRoleState && obs) {
            float o[8];
            env_obs<D>(x, s, o);
            store_obs_rows<D, NT>(stage, o, lane, M, obs + ((int64_t)k * A + a_first) * D);
        }
        if (!kObsR && active) {
            if (RS) {
                const int kb = k % kRSTB;
                rsg.rbuf[kb * kRSA + rsg.li] = rw;
                rsg.dbuf[kb * kRSA + rsg.li] = (uint8_t)dn;
            } else {
                if (rew) st_out<NT>(rew + row, rw);
                if (done) st_out<NT>(done + row, (uint8_t)dn);
            }
            rsum += rw;
            dsum += dn ? 1.0f : 0.0f;
        }
    };
    if constexpr (RS) {  // chunks of kRSTB steps, each followed by one workgroup flush of its rows
#pragma unroll 1
        for (int32_t kc = 0; kc < T; kc += kRSTB) {
            const int32_t ke = T - kc < kRSTB ? T : kc + kRSTB;
            if constexpr (kPF == 1) {
#pragma unroll 1
                for (int32_t k = kc; k < ke; ++k) step(k, 0);
            } else {  // kRSTB is even: step k uses ring slot k & 1
                static_assert(kPF == 2 && kRSTB % 2 == 0, "FENV_RS_PF is 1 or 2");
#pragma unroll 1
                for (int32_t k = kc; k < ke; k += 2) {
                    step(k, 0);
                    if (k + 1 < ke) step(k + 1, 1);
                }
            }
            __syncthreads();
            rs_flush<NT>(rsg, kc, ke - kc, A, rew, done);
            if (ke < T) __syncthreads();
        }
    } else {
        for (int32_t k0 = 0; k0 < T; k0 += kPF) {
#pragma unroll
            for (int j = 0; j < kPF; ++j) {
                const int32_t k = k0 + j;
                if (k >= T) break;
                step(k, j);
            }
        }
    }
    if (!kObsR && active) {
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

template <int D, int MODE, bool RA, int PF, bool NT>
__global__ __launch_bounds__(256) void k_rollout_wave(Consts c, DevState st, DevPending p,
                                                      int32_t T, const float2 *__restrict__ act,
                                                      ActGen gen,
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
        rollout_body<D, MODE, RA, false, PF, WaveX, kRoleAll, NT>(c, st, p, x, active, f, a, i,
                                                                  stage[w], lane, M,
                                             f_first * N, T, act, gen, obs, rew, done, rsum,
                                             dsum);
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

// Small latency-bound grids (use_split): a 4-wave group of formation-waves (k_rollout_wave's
// workgroup) is run by 8 waves.  Waves 0-3 take kRoleState, waves 4-7 kRoleObs for the same
// formations, so each wave issues about half of a step's instructions and a SIMD holds two
// waves whose latencies hide each other.  The stats record is the 4 kRoleState waves' sums in
// k_rollout_wave's order: the same records.
template <int D, int MODE, bool RA, int PF>
__global__ __launch_bounds__(512) void k_rollout_wave_split(Consts c, DevState st, DevPending p,
                                                            int32_t T,
                                                            const float2 *__restrict__ act,
                                                            ActGen gen, float *__restrict__ obs,
                                                            float *__restrict__ rew,
                                                            uint8_t *__restrict__ done,
                                                            float2 *__restrict__ partial,
                                                            bool accum) {
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8];
    __shared__ float2 red[4];
    const int lane = threadIdx.x & 63;
    const int w8 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = w8 & 3;  // formation-wave of the group
    const int64_t wave = (int64_t)blockIdx.x * 4 + w;
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
    // every wave runs its body (each holds one barrier), also the waves with no formation
    if (w8 < 4)
        rollout_body<D, MODE, RA, false, PF, WaveX, kRoleState>(
            c, st, p, x, active, f, a, i, nullptr, lane, M, f_first * N, T, act, gen, nullptr,
            rew, done, rsum, dsum);
    else
        rollout_body<D, MODE, RA, false, PF, WaveX, kRoleObs>(
            c, st, p, x, active, f, a, i, stage[w], lane, M, f_first * N, T, act, gen, obs,
            nullptr, nullptr, rsum, dsum);
    if (partial) {
        if (w8 < 4) {
            rsum = wave_sum(rsum);
            dsum = wave_sum(dsum);
            if (lane == 0) red[w] = make_float2(rsum, dsum);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float2 v = red[0];
            for (int k = 1; k < 4; ++k) v = make_float2(v.x + red[k].x, v.y + red[k].y);
            if (accum) v = make_float2(partial[blockIdx.x].x + v.x, partial[blockIdx.x].y + v.y);
            partial[blockIdx.x] = v;
        }
    }
}

template <int D, int MODE, bool RA, bool NT>
__global__ __launch_bounds__(kRSA) FENV_RS_OCC void k_rollout_wave_rs(Consts c, DevState st, DevPending p,
                                                          int32_t T,
                                                          const float2 *__restrict__ act,
                                                          ActGen gen, float *__restrict__ obs,
                                                          float *__restrict__ rew,
                                                          uint8_t *__restrict__ done,
                                                          float2 *__restrict__ partial,
                                                          bool accum) {
    // Every wave runs the step loop (the flushes are workgroup barriers); waves past the last
    // formation have no active lane and write nothing.
    __shared__ __attribute__((aligned(16))) float stage[kRS][64 * 8];
    __shared__ __attribute__((aligned(16))) float rbuf[kRSTB * kRSA];
    __shared__ __attribute__((aligned(16))) uint8_t dbuf[kRSTB * kRSA];
    __shared__ float2 red[kRS];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t blk = blockIdx.x;
    const int64_t wave = blk * kRS + w;
    const int N = c.N;
    const int Mw = c.fpw * N;  // agents of a full wave
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = wave * c.fpw + fi;
    const bool active = fi < c.fpw && f < c.F;
    const int64_t a = f * N + i;
    WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    const int64_t f_first = wave * c.fpw;
    const int64_t f_left = c.F - f_first;
    const int M = (int)((f_left <= 0 ? 0 : (f_left < c.fpw ? f_left : c.fpw)) * N);
    const int64_t A = c.F * (int64_t)N;
    RSStage rsg;
    rsg.rbuf = rbuf;
    rsg.dbuf = dbuf;
    rsg.li = w * Mw + lane;
    rsg.g0 = blk * kRS * Mw;
    rsg.nwg = (int)((A - rsg.g0) < (int64_t)kRS * Mw ? (A - rsg.g0) : (int64_t)kRS * Mw);
    float rsum = 0.f, dsum = 0.f;
    rollout_body<D, MODE, RA, true, 1, WaveX, kRoleAll, NT>(c, st, p, x, active, f, a, i, stage[w],
                                                           lane, M,
                                       f_first * N, T, act, gen, obs, rew, done, rsum, dsum, rsg);
    if (partial) {  // one {sum reward, sum done} record per 4 waves -- the same records, in the
                    // same summation order, as k_rollout_wave's 4-wave workgroups
        rsum = wave_sum(rsum);
        dsum = wave_sum(dsum);
        if (lane == 0) red[w] = make_float2(rsum, dsum);
        __syncthreads();
        const int64_t groups = ((c.F + c.fpw - 1) / c.fpw + 3) / 4;
        const int hq = (int)threadIdx.x;
        if (hq < kRS / 4 && blk * (kRS / 4) + hq < groups) {
            const int64_t gi = blk * (kRS / 4) + hq;
            float2 v = red[4 * hq];
            for (int k = 1; k < 4; ++k)
                v = make_float2(v.x + red[4 * hq + k].x, v.y + red[4 * hq + k].y);
            if (accum) v = make_float2(partial[gi].x + v.x, partial[gi].y + v.y);
            partial[gi] = v;
        }
    }
}

template <int D, int MODE, bool RA, bool NT>
__global__ __launch_bounds__(1024) void k_rollout_block(Consts c, DevState st, DevPending p,
                                                        int32_t T,
                                                        const float2 *__restrict__ act,
                                                        ActGen gen,
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
    rollout_body<D, MODE, RA, false, 1, BlockX, kRoleAll, NT>(c, st, p, x, active, f, a, i,
                                                             stage[w], i & 63, M,
                                        f * N + 64 * w, T, act, gen, obs, rew, done, rsum, dsum);
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
// Per formation: mean ||p - goal||, mean ||p_i - p_{i+1}||, its unbiased std, mean reward
// (compute_metrics on the current, post-reset state, simulate.py:117 + vectorized_env.py:80-81),
// then the means of the four reward components compute_reward_and_done logs
// (simulate.py:183-208: close-to-goal bonus, distance reward, right / left neighbour rewards) of
// the state the last step scored -- the terminal state for a formation that step reset.  Each
// formation's values are staged in LDS and summed by its first lane in agent order, in double.
constexpr int kMS = 7;  // staged values per agent
template <class X>
__device__ __forceinline__ void metrics_body(const Consts &c, const DevState &st,
                                             const DevPending &p, bool terminal, const X &x,
                                             bool active, int64_t f, int64_t a, int i,
                                             const float *rew, float *stage, int base,
                                             float *out) {
    float px = 0.f, py = 0.f, gx = 0.f, gy = 0.f, r = 0.f;
    bool term = false;
    if (active) {
        px = st.px[a];
        py = st.py[a];
        gx = st.gx[f];
        gy = st.gy[f];
        r = rew ? rew[a] : 0.f;
        term = terminal && st.t[f] == 0;
    }
    float qx = px, qy = py, qgx = gx, qgy = gy;  // the state the last step's reward scored
    if (term) {
        const float4 tq = p.term[a];
        qx = tq.x;
        qy = tq.y;
        qgx = tq.z;
        qgy = tq.w;
    }
    float pnx, pny;
    x.a_next(px, py, pnx, pny);
    const float dg = norm2(px - gx, py - gy);
    const float dr = norm2(px - pnx, py - pny);
    float qpx, qnx, qpy, qny;
    x.d_pn(qx, qy, qpx, qnx, qpy, qny);
    const float qg = norm2(qx - qgx, qy - qgy);                  // simulate.py:180
    const float ctg = qg < 100.0f ? 10.0f : 0.0f;               // :183-187
    const float rd = -0.1f * qg;                                // :191
    const float rr = nb_reward(norm2(qx - qnx, qy - qny) - c.d_nb);  // :197, 202, 204
    const float rl = nb_reward(norm2(qx - qpx, qy - qpy) - c.d_nb);  // :198, 203, 205
    const int N = c.N;
    float *sv = stage + kMS * (base + i);
    sv[0] = dg;
    sv[1] = dr;
    sv[2] = r;
    sv[3] = ctg;
    sv[4] = rd;
    sv[5] = rr;
    sv[6] = rl;
    __syncthreads();
    if (active && i == 0) {
        double sg = 0, sr = 0, sr2 = 0, rw = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0;
        for (int k = 0; k < N; ++k) {
            const float *v = stage + kMS * (base + k);
            const double d = v[1];
            sg += v[0];
            sr += d;
            sr2 += d * d;
            rw += v[2];
            s3 += v[3];
            s4 += v[4];
            s5 += v[5];
            s6 += v[6];
        }
        const double mr = sr / N;
        float *o = out + f * kMetricCols;
        o[0] = (float)(sg / N);
        o[1] = (float)mr;
        o[2] = N > 1 ? (float)sqrt(fmax(0.0, (sr2 - N * mr * mr) / (N - 1))) : __builtin_nanf("");
        o[3] = (float)(rw / N);
        o[4] = (float)(s3 / N);
        o[5] = (float)(s4 / N);
        o[6] = (float)(s5 / N);
        o[7] = (float)(s6 / N);
    }
}

__global__ __launch_bounds__(256) void k_metrics_wave(Consts c, DevState st, DevPending p,
                                                      bool terminal, const float *rew,
                                                      float *out) {
    __shared__ float stage[kMS * 256];
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int N = c.N;
    const int fi = lane / N;
    const int i = lane - fi * N;
    const int64_t f = wave * c.fpw + fi;
    const bool active = fi < c.fpw && f < c.F;
    WaveX x{i == 0 ? lane + N - 1 : lane - 1, i == N - 1 ? lane - N + 1 : lane + 1};
    metrics_body(c, st, p, terminal, x, active, f, f * N + i, i, rew, stage,
                 (threadIdx.x & ~63) + fi * N, out);
}

__global__ __launch_bounds__(1024) void k_metrics_block(Consts c, DevState st, DevPending p,
                                                        bool terminal, const float *rew,
                                                        float *out) {
    __shared__ float lds[6 * kMaxN];
    __shared__ float stage[kMS * kMaxN];
    const int N = c.N;
    const int i = threadIdx.x;
    const int64_t f = blockIdx.x;
    const bool active = i < N;
    BlockX x{lds, i, active ? (i == 0 ? N - 1 : i - 1) : i, active ? (i == N - 1 ? 0 : i + 1) : i};
    metrics_body(c, st, p, terminal, x, active, f, f * N + i, i, rew, stage, 0, out);
}

// ---------------------------------------------------------------- deterministic reductions
// One workgroup of NT threads; thread k sums elements k, k+NT, ... in double; then a fixed tree.
template <int K, class T, int NT>
__global__ __launch_bounds__(NT) void k_reduce_rows(const T *in, int64_t rows, double *out) {
    __shared__ double red[K][NT];
    double acc[K][4];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[j][u] = 0.0;
    // 4 independent rows in flight per thread per iteration (fixed assignment: deterministic)
    int64_t r = threadIdx.x;
    for (; r + 3 * NT < rows; r += 4 * NT) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) acc[j][u] += (double)in[(r + u * NT) * K + j];
    }
    for (; r < rows; r += NT)
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j][0] += (double)in[r * K + j];
#pragma unroll
    for (int j = 0; j < K; ++j) red[j][threadIdx.x] = (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
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

// Workgroup-staged rows (k_rollout_wave_rs) only where they pay (same-box A/B): a
// wave's reward row must straddle 128-B lines (agents per wave not a multiple of 32; at N = 64
// the rows are whole lines and the staging costs 1.4 %), and the grid must be large enough to
// be store-bound: a small launch (BASELINE config 1, 342 waves) is latency-bound and runs 13 %
// faster as 4-wave workgroups spread over 4x as many CUs, with no flush barriers.
// A single-step launch pays the flush barrier without amortising it (T = 1: 70.6 µs staged vs
// 64.2 µs plain at config 3; T = 2-6 tie within 3 % either way).  Both kernels write the same
// per-4-wave stats records, so the choice may change from launch to launch.
#ifndef FENV_RS_MIN_WAVES
#define FENV_RS_MIN_WAVES 2048
#endif
#ifndef FENV_RS_MIN_T
#define FENV_RS_MIN_T 2
#endif
static inline bool use_rs(const Consts &c, int32_t T) {
    if (!FENV_RS || !wave_path(c.N) || T < FENV_RS_MIN_T) return false;
    const int64_t waves = (c.F + c.fpw - 1) / c.fpw;
    return (c.fpw * c.N) % 32 != 0 && waves >= FENV_RS_MIN_WAVES;
}

// Small latency-bound grids (fewer waves than FENV_RS_MIN_WAVES: the per-step dependency chain
// of one wave, not HBM, sets the time) take a 4-deep action prefetch / 4x unrolled step loop:
// same-box A/B at BASELINE config 1 (4,096 x 5) 10.04-10.08 vs 10.47 us per 10-step launch,
// while it costs 5-7 % at config 4 (16,384 x 64, 16,384 waves), which keeps depth 1
// (profiles/ab/r2_env_cfg_ab.txt).
#ifndef FENV_SMALL_PF
#define FENV_SMALL_PF 4
#endif
static inline bool use_pf(const Consts &c, int32_t T) {
    const int64_t waves = (c.F + c.fpw - 1) / c.fpw;
    return FENV_SMALL_PF > 1 && T >= FENV_SMALL_PF && waves < FENV_RS_MIN_WAVES;
}

// Small latency-bound grids: the role-split kernel (two waves per formation-wave, see
// k_rollout_wave_split) where the grid leaves most SIMDs idle.  FENV_SPLIT=0 turns it off (A/B).
#ifndef FENV_SPLIT
#define FENV_SPLIT 1
#endif
static inline bool use_split(const Consts &c) {
    const int64_t waves = (c.F + c.fpw - 1) / c.fpw;
    return FENV_SPLIT && wave_path(c.N) && waves < FENV_RS_MIN_WAVES;
}

int64_t rollout_group_count(const Consts &c) {
    return group_count(c);
}

// grid of k_rollout_wave_rs: kRS waves per workgroup
static inline int64_t rs_blocks(const Consts &c) {
    return ((c.F + c.fpw - 1) / c.fpw + kRS - 1) / kRS;
}

static inline unsigned block_threads(int32_t N) { return (unsigned)((N + 63) / 64 * 64); }

template <int D, int MODE, bool NT>
static hipError_t rollout_dmn(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                             const float *act, float *obs, float *rew, uint8_t *done,
                             float *partial, bool accum, hipStream_t st, const ActGen *gen) {
    const float2 *a2 = reinterpret_cast<const float2 *>(act);
    float2 *p2 = reinterpret_cast<float2 *>(partial);
    if (gen) {  // in-kernel actions
        if (use_rs(c, T))
            hipLaunchKernelGGL((k_rollout_wave_rs<D, MODE, true, NT>),
                               dim3((unsigned)rs_blocks(c)), dim3(kRSA), 0, st, c, s, p,
                               T, a2, *gen, obs, rew, done, p2, accum);
        else if (wave_path(c.N))
            hipLaunchKernelGGL((k_rollout_wave<D, MODE, true, 1, NT>), dim3((unsigned)group_count(c)),
                               dim3(256), 0, st, c, s, p, T, a2, *gen, obs, rew, done, p2, accum);
        else
            hipLaunchKernelGGL((k_rollout_block<D, MODE, true, NT>), dim3((unsigned)c.F),
                               dim3(block_threads(c.N)), 0, st, c, s, p, T, a2, *gen, obs, rew,
                               done, p2, accum);
        return hipGetLastError();
    }
    const ActGen g0{};
    if (use_rs(c, T)) {
        hipLaunchKernelGGL((k_rollout_wave_rs<D, MODE, false, NT>),
                           dim3((unsigned)rs_blocks(c)), dim3(kRSA), 0, st, c, s, p, T, a2, g0,
                           obs, rew, done, p2, accum);
    } else if (use_split(c)) {
        const unsigned blocks = (unsigned)group_count(c);
        if (use_pf(c, T))
            hipLaunchKernelGGL((k_rollout_wave_split<D, MODE, false, FENV_SMALL_PF>), dim3(blocks),
                               dim3(512), 0, st, c, s, p, T, a2, g0, obs, rew, done, p2, accum);
        else
            hipLaunchKernelGGL((k_rollout_wave_split<D, MODE, false, 1>), dim3(blocks), dim3(512),
                               0, st, c, s, p, T, a2, g0, obs, rew, done, p2, accum);
    } else if (wave_path(c.N)) {
        const unsigned blocks = (unsigned)group_count(c);
        if (use_pf(c, T))
            hipLaunchKernelGGL((k_rollout_wave<D, MODE, false, FENV_SMALL_PF, NT>), dim3(blocks),
                               dim3(256), 0, st, c, s, p, T, a2, g0, obs, rew, done, p2, accum);
        else
            hipLaunchKernelGGL((k_rollout_wave<D, MODE, false, 1, NT>), dim3(blocks), dim3(256), 0, st,
                               c, s, p, T, a2, g0, obs, rew, done, p2, accum);
    } else {
        hipLaunchKernelGGL((k_rollout_block<D, MODE, false, NT>), dim3((unsigned)c.F),
                           dim3(block_threads(c.N)), 0, st, c, s, p, T, a2, g0, obs, rew, done, p2,
                           accum);
    }
    return hipGetLastError();
}

// Non-temporal output stores (st_out) where a call's outputs stream far past the caches: at
// least kNTMinAgentSteps agent-steps (45 B each at D = 8: >= 135 MB, half the Infinity Cache).
// Same-box A/B (profiles/ab/r2_nt_out_ab.txt): config 3 447 vs 470 us per 10-step launch,
// config 4 74-75 vs 94 us, single-step launches at config 3 52 vs 70 us; config 1 (200k
// agent-steps, latency-bound) 8.2 vs 7.7 us, so small calls keep plain stores.
#ifndef FENV_NT_OUT
#define FENV_NT_OUT 1
#endif
constexpr double kNTMinAgentSteps = 3.0e6;
bool rollout_nt(const Consts &c, int64_t T) {
    return FENV_NT_OUT && (double)c.F * (double)c.N * (double)T >= kNTMinAgentSteps;
}
// Steps per kernel launch of a large call.  With non-temporal stores, launches of <= 4 steps
// stream at 0.89 of the HBM spec at config 3 against 0.69-0.70 for 6-10 (five steps is
// address-dependent: either): the T output planes written concurrently by a launch are what the
// memory system handles badly, so long calls run as short launches and pay the state round trip
// (16 B per agent per launch) instead (profiles/ab/r2_chunk_ab.txt).  0: one launch per call.
#ifndef FENV_LAUNCH_CHUNK
#define FENV_LAUNCH_CHUNK 0
#endif
int32_t rollout_launch_steps(const Consts &c, int64_t T) {
    if (FENV_LAUNCH_CHUNK <= 0 || !rollout_nt(c, T) || large_path(c.N)) return (int32_t)T;
    return T < FENV_LAUNCH_CHUNK ? (int32_t)T : FENV_LAUNCH_CHUNK;
}

template <int D, int MODE>
static hipError_t rollout_dm(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                             const float *act, float *obs, float *rew, uint8_t *done,
                             float *partial, bool accum, bool nt, hipStream_t st,
                             const ActGen *gen) {
    return nt ? rollout_dmn<D, MODE, true>(c, s, p, T, act, obs, rew, done, partial, accum, st,
                                           gen)
              : rollout_dmn<D, MODE, false>(c, s, p, T, act, obs, rew, done, partial, accum, st,
                                            gen);
}

const char *rollout_kernel_name(const Consts &c, int32_t T) {
    if (large_path(c.N)) return "k_rollout_large";
    if (use_rs(c, T)) return "k_rollout_wave_rs";
    if (use_split(c))
        return use_pf(c, T) ? "k_rollout_wave_split (prefetch 4)" : "k_rollout_wave_split";
    if (wave_path(c.N)) return use_pf(c, T) ? "k_rollout_wave (prefetch 4)" : "k_rollout_wave";
    return "k_rollout_block";
}

hipError_t launch_rollout(const Consts &c, const DevState &s, const DevPending &p, int32_t T,
                          int32_t D, const float *act, float *obs, float *rew, uint8_t *done,
                          float *partial, bool accum, bool nt, hipStream_t st,
                          const ActGen *gen) {
    if (large_path(c.N))
        return launch_rollout_large(c, s, p, T, D, act, obs, rew, done, partial, accum, st, gen);
    const bool mt = c.reset_mode == FENV_RESET_MT19937;
    if (D == 8)
        return mt ? rollout_dm<8, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done, partial,
                                                      accum, nt, st, gen)
                  : rollout_dm<8, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done, partial,
                                                     accum, nt, st, gen);
    return mt ? rollout_dm<6, FENV_RESET_MT19937>(c, s, p, T, act, obs, rew, done, partial, accum, nt,
                                                  st, gen)
              : rollout_dm<6, FENV_RESET_PHILOX>(c, s, p, T, act, obs, rew, done, partial, accum, nt,
                                                 st, gen);
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
    if (large_path(c.N)) return launch_reset_observe_large(c, s, p, D, do_reset, obs, st);
    return D == 8 ? reset_obs_d<8>(c, s, p, do_reset, obs, st)
                  : reset_obs_d<6>(c, s, p, do_reset, obs, st);
}

hipError_t launch_metrics(const Consts &c, const DevState &s, const DevPending &p, bool terminal,
                          const float *rew, float *out, double *sums, hipStream_t st) {
    if (large_path(c.N)) {
        hipError_t e = launch_metrics_large(c, s, p, terminal, rew, out, st);
        if (e != hipSuccess) return e;
    } else if (wave_path(c.N)) {
        hipLaunchKernelGGL(k_metrics_wave, dim3((unsigned)group_count(c)), dim3(256), 0, st, c,
                           s, p, terminal, rew, out);
    } else {
        hipLaunchKernelGGL(k_metrics_block, dim3((unsigned)c.F), dim3(block_threads(c.N)), 0, st,
                           c, s, p, terminal, rew, out);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || sums == nullptr) return e;
    hipLaunchKernelGGL((k_reduce_rows<kMetricCols, float, 512>), dim3(1), dim3(512), 0, st, out,
                       c.F, sums);
    return hipGetLastError();
}

hipError_t launch_reduce_partials(const float *partial, int64_t count, double *out,
                                  hipStream_t st) {
    hipLaunchKernelGGL((k_reduce_rows<2, float, 1024>), dim3(1), dim3(1024), 0, st, partial, count,
                       out);
    return hipGetLastError();
}

// Launch gate (fenv_stream_gate): one wavefront that holds the stream's later launches until the
// host stores `value` into the word at `flag` (coherent, device-mapped host memory: every poll is
// a system-scope load that crosses the bus, ~1-2 us), or until `timeout_ticks` of the
// constant-rate wall clock have passed -- an exit every wave reaches, whatever the host does.
// status[0] = 1 released / 2 timed out, status[1] = polls, status[2..3] = the time the wave held
// the stream (entry to exit, ns, 64-bit); written by lane 0 with system-scope stores (vector
// memory), status[0] last, so a host that sees it also sees the rest.
__global__ __launch_bounds__(64) void k_stream_gate(const uint32_t *flag, uint32_t value,
                                                    uint64_t timeout_ticks, uint32_t khz,
                                                    uint32_t *status) {
    const uint64_t t0 = wall_clock64();
    uint64_t t = t0;
    uint32_t polls = 0, how = 2;
    for (;;) {
        const uint32_t v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        ++polls;
        t = wall_clock64();
        if (v == value) {
            how = 1;
            break;
        }
        if (t - t0 > timeout_ticks) break;
        __builtin_amdgcn_s_sleep(8);  // ~0.2 us between polls; a poll itself takes ~1 us
    }
    if (status && threadIdx.x == 0) {
        const uint64_t held_ns = (t - t0) * 1000000ull / khz;
        __hip_atomic_store(status + 1, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(status + 2, (uint32_t)held_ns, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(status + 3, (uint32_t)(held_ns >> 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(status, how, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_stream_gate(const uint32_t *flag, uint32_t value, uint64_t timeout_ticks,
                              uint32_t khz, uint32_t *status, hipStream_t st) {
    hipLaunchKernelGGL(k_stream_gate, dim3(1), dim3(64), 0, st, flag, value, timeout_ticks, khz,
                       status);
    return hipGetLastError();
}

// Staged MT19937 reset set: pinned host buffer -> HBM, as a kernel on the launch stream (the
// refill is then ordered with the rollout kernels by the stream's in-order AQL queue alone; the
// host buffer is read over the bus through its mapped device address).  n floats, any n.
// delay > 0: test hook (fenv_test_stage_hook), every workgroup sleeps first.
__global__ __launch_bounds__(256) void k_stage_copy(float *__restrict__ dst,
                                                    const float *__restrict__ src, int64_t n,
                                                    int32_t delay) {
    if (delay > 0) {
        if (threadIdx.x == 0)
            for (int32_t k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(127);
        __syncthreads();
    }
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        d4[i] = s4[i];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n - 4 * n4) dst[4 * n4 + t] = src[4 * n4 + t];
}

hipError_t launch_stage_copy(float *dst, const float *src, int64_t n, int32_t delay_sleeps,
                             hipStream_t st) {
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_stage_copy, dim3((unsigned)blocks), dim3(256), 0, st, dst, src, n,
                       delay_sleeps);
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
