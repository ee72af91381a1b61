// Device-side building blocks of one formation-env step (reference: /root/reference/simulate.py
// :70-254), shared by the env kernels (fenv_kernels.hip) and the fused policy rollout
// (policy_rollout.hip) so both compute bit-identical results.  Every translation unit that
// includes it compiles with contraction off.
#pragma once
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

// x / Y (Y = 400 or 600), correctly rounded: the IEEE division.  (A reciprocal-product form with
// one fma residual correction, exact for every finite |x| >= 2^-100 by tools/div_const_check.c,
// was A/B'd per config in rounds 1-2 and not kept: DESIGN.md section 4.)
template <int Y>
__device__ __forceinline__ float div_const(float x) {
    return x / (float)Y;
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

// A staged MT19937 draw failed its tag check (fenv_internal.h DevPending): classify it against the
// generations the slot and the other slot held, and record it in the handle's error words (host
// memory; relaxed system-scope vector stores -- any lane's values will do).
__device__ __forceinline__ void stage_tag_fail(const DevPending &p, int64_t f, int64_t a,
                                                         uint32_t tag, uint32_t bx, uint32_t by) {
    uint32_t kind = kStageBad;
    if (tag == stage_tag_agent(p.gen - 2u, a, bx, by)) kind = kStageStale;
    else if (tag == stage_tag_agent(p.gen - 1u, a, bx, by) ||
             tag == stage_tag_agent(p.gen + 1u, a, bx, by)) kind = kStageOther;
    if (p.err == nullptr) return;
    __hip_atomic_store(p.err + 0, kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.err + 1, p.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.err + 2, (uint32_t)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// simulate.py:133-143 for agent i of formation f (local indices), episode `ep_new`.
template <int MODE>
__device__ __forceinline__ void draw_reset(const Consts &c, const DevPending &p, int64_t f,
                                           int64_t a, int i, uint32_t ep_new, float &px,
                                           float &py, float &gx, float &gy) {
    if (MODE == FENV_RESET_MT19937) {
        // indices laundered here: a and f are loop-invariant in the kernels' step loops, so the
        // compiler would otherwise hoist the six addresses below (12 VGPRs) out of the loop for
        // this rarely taken branch -- one occupancy step down on every MT19937 kernel
        int64_t la = a, lf = f;
        asm volatile("" : "+v"(la));
        asm volatile("" : "+v"(lf));
        const int64_t A = c.F * (int64_t)c.N;
        px = p.pend[la];
        py = p.pend[A + la];
        gx = p.pend[2 * A + lf];
        gy = p.pend[2 * A + c.F + lf];
        // the tags of the lane's draws (a lane owning no agent -- env_step's `live` -- may index
        // past the set; it applies nothing, so it is not checked there)
        if (f < c.F && a < A) {
            const uint32_t *tg = reinterpret_cast<const uint32_t *>(p.pend + 2 * A + 2 * c.F);
            const uint32_t ta = tg[la], tf = tg[A + lf];
            const uint32_t bx = __float_as_uint(px), by = __float_as_uint(py);
            if (ta != stage_tag_agent(p.gen, a, bx, by))
                stage_tag_fail(p, f, a, ta, bx, by);
            else if (tf != stage_tag_goal(p.gen, f, __float_as_uint(gx), __float_as_uint(gy)))
                stage_tag_fail(p, f, a, 0u, 0u, 0u);  // the goal's tag: kStageBad
        }
    } else {
        // the same laundering (the counters depend only on loop-invariant indices): 7-10 VGPRs
        // fewer per Philox kernel; the random-action kernel 5 -> 7 waves/SIMD, -6 % per launch
        int64_t lf = f;
        int li = i;
        asm volatile("" : "+v"(lf));
        asm volatile("" : "+v"(li));
        const uint64_t fg = (uint64_t)(c.f0 + lf);
        const uint64_t ag = fg * (uint64_t)c.N + (uint64_t)li;
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
// Three exchange rounds per env step: A {px,py}->prev,next, C {ind}->prev,next, D {nx,ny}->
// prev,next (round 1 had four: A {px,py}->next, B {drr}->prev, C, D).

struct WaveX {  // N <= 64: lanes of one formation are contiguous in the wavefront
    int lp, ln;
    __device__ __forceinline__ void a_next(float u, float v, float &un, float &vn) const {
        un = __shfl(u, ln, 64);
        vn = __shfl(v, ln, 64);
    }
    __device__ __forceinline__ void a_pn(float u, float v, float &up, float &un, float &vp,
                                         float &vn) const {
        up = __shfl(u, lp, 64);
        un = __shfl(u, ln, 64);
        vp = __shfl(v, lp, 64);
        vn = __shfl(v, ln, 64);
    }
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
// its previous reads by at least one barrier (rounds are used in the order A,[B,]C,D; A and a_pn
// share slots 0-1).
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
    __device__ __forceinline__ void a_pn(float u, float v, float &up, float &un, float &vp,
                                         float &vn) const {
        lds[0 * kMaxN + i] = u;
        lds[1 * kMaxN + i] = v;
        __syncthreads();
        up = lds[0 * kMaxN + ip];
        un = lds[0 * kMaxN + in];
        vp = lds[1 * kMaxN + ip];
        vn = lds[1 * kMaxN + in];
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
// TERM = false: leave the terminal-state record to another wave (the split kernel's kRoleState).
// live = false: a lane that owns no agent (the grid's padding, a wave's lanes past its last
// whole formation, a workgroup's threads past N).  It still runs the step -- the ring exchanges
// are wave-wide -- from a zero state whose steps_since_reset starts at 0 every launch, so it has
// a phantom done step max_steps + 1 steps into a launch.  It must store nothing there: its
// (f, a) index a formation that is not its own, or none (the round-2/3
// post-reset failures were these lanes' terminal-state stores of zeros, past the end of the
// terminal buffer into the staged reset set that follows it in memory).
template <int MODE, class X, bool TERM = true>
__device__ __forceinline__ void env_step(const Consts &c, const DevPending &p, const X &x,
                                         int64_t f, int64_t a, int i, bool live, float2 act,
                                         Agent &s, float &rw, bool &dn, bool &did_reset) {
    // vectorized_env.py:69-70 (v = 10 * a), simulate.py:82 (agents += v)
    const float x1 = s.px + 10.0f * act.x;
    const float y1 = s.py + 10.0f * act.y;
    // simulate.py:86-87: out of bounds tested on the unclipped position
    const bool oob = (x1 <= 0.0f) | (y1 <= 0.0f) | (x1 >= kW) | (y1 >= kH);
    s.px = clip0(x1, kW);
    s.py = clip0(y1, kH);

    // compute_reward_and_done, simulate.py:180-211
    const float dg = norm2(s.px - s.gx, s.py - s.gy);
    // one exchange round for both neighbours' positions; both distances computed here as the
    // reference does (:197-198: norm(p - roll(p, -1)), norm(p - roll(p, 1)))
    float ppx, pnx, ppy, pny;
    x.a_pn(s.px, s.py, ppx, pnx, ppy, pny);
    const float drr = norm2(s.px - pnx, s.py - pny);  // ||p_i - p_{i+1}||  (:197)
    const float drl = norm2(s.px - ppx, s.py - ppy);  // ||p_i - p_{i-1}||  (:198)
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
        // keep the terminal (post-clip, pre-reset) state: the step's logged reward components
        // (simulate.py:183-208) describe it, not the freshly drawn one
        // (indices laundered inside the branch: otherwise the compiler hoists these rarely used
        // addresses out of the step loop into 4 loop-invariant VGPRs)
        if (TERM && live) {
            int64_t ta = a;
            asm volatile("" : "+v"(ta));
            p.term[ta] = make_float4(s.px, s.py, s.gx, s.gy);
        }
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
    const float nx = div_const<400>(s.px);  // :156, normalise first
    const float ny = div_const<600>(s.py);
    float npx, nnx, npy, nny;
    x.d_pn(nx, ny, npx, nnx, npy, nny);
    o[0] = nx;
    o[1] = ny;
    o[2] = npx - nx;  // :166
    o[3] = npy - ny;
    o[4] = nnx - nx;  // :167
    o[5] = nny - ny;
    if (D == 8) {
        o[6] = div_const<400>(s.gx - s.px);  // :172, subtract first, then divide
        o[7] = div_const<600>(s.gy - s.py);
    }
}

// Wave-cooperative store of the wave's observation rows.  Lanes 0..M-1 own the rows of M
// consecutive agents starting at `dst`; each lane stages its D floats in the wave's private
// LDS slice (2 KiB) and the wave then writes the whole contiguous span with full-width vector
// stores (1 KiB per instruction) instead of 64 strided rows (tools/ubench_hbm: 3.45 -> 4.7 TB/s
// on this access pattern).  No barrier: the slice is private to the wave and a wave's LDS
// operations complete in order.
template <int D>
__device__ __forceinline__ void stage_obs_rows(float *stage, const float (&o)[8], int lane) {
    if (D == 8) {
        reinterpret_cast<float4 *>(stage)[2 * lane] = make_float4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<float4 *>(stage)[2 * lane + 1] = make_float4(o[4], o[5], o[6], o[7]);
    } else {
        reinterpret_cast<float2 *>(stage)[3 * lane] = make_float2(o[0], o[1]);
        reinterpret_cast<float2 *>(stage)[3 * lane + 1] = make_float2(o[2], o[3]);
        reinterpret_cast<float2 *>(stage)[3 * lane + 2] = make_float2(o[4], o[5]);
    }
}

// Output stores (observations, rewards, dones).  NT: non-temporal (`nt`), for launches whose
// outputs stream far past the caches: they are not allocated in L2 / the Infinity Cache, which
// measured 5 % faster at BASELINE config 3, 20 % at config 4 and 26 % for single-step launches,
// and 6 % slower for a small latency-bound grid (config 1) (profiles/ab/r2_nt_out_ab.txt).
template <bool NT, class V>
__device__ __forceinline__ void st_out(V *p, V v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ void st_out(float4 *p, float4 v) {
    if (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}
template <bool NT>
__device__ __forceinline__ void st_out(float2 *p, float2 v) {
    if (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
    } else {
        *p = v;
    }
}

template <int D, bool NT = false>
__device__ __forceinline__ void store_obs_rows(float *stage, const float (&o)[8], int lane, int M,
                                               float *dst) {
    stage_obs_rows<D>(stage, o, lane);
    __builtin_amdgcn_wave_barrier();
    const int nf = M * D;
    if (((reinterpret_cast<uintptr_t>(dst) & 15) == 0) && ((nf & 3) == 0)) {
        const int nq = nf >> 2;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int q = lane + 64 * k;
            if (q < nq)
                st_out<NT>(reinterpret_cast<float4 *>(dst) + q,
                           reinterpret_cast<const float4 *>(stage)[q]);
        }
    } else {
        const int nq = nf >> 1;  // D is even, rows are 8-byte aligned
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = lane + 64 * k;
            if (q < nq)
                st_out<NT>(reinterpret_cast<float2 *>(dst) + q,
                           reinterpret_cast<const float2 *>(stage)[q]);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Sum over the 64 lanes, returned in every lane.  DPP form: row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast 15 / 31 carry the row sums up, so lane 63 holds the total (a fixed order:
// deterministic), read back with v_readlane.  Six VALU ops instead of six LDS-latency swizzles.
__device__ __forceinline__ float wave_sum(float v) {
    int x = __float_as_int(v);
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xe, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xc, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false)));
    x = __float_as_int(__int_as_float(x) + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false)));
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

}  // namespace fenvk
