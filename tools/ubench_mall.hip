// Does a per-step launch shape with the env state kept in the Infinity Cache (MALL) beat the
// fused T-step rollout's T-plane write shape?  Byte mix of config 3 (A = 5,242,880 agents,
// D = 8): per agent-step 8 B of actions read, 32 B obs + 4 B reward + 1 B done written; per
// step-launch the state (px, py: 8 B read + 8 B written per agent) round-trips through memory.
//   fused  : one launch, every thread T steps, state in registers (the rollout's T-plane shape)
//   step   : T launches, state read + written every step, plain stores
//   step_nt: T launches, outputs stored non-temporally (hoping they do not evict the state)
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_mall ubench_mall.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int T = 10;

template <bool NT>
__device__ __forceinline__ void st4(float4 *p, float4 v) {
    if (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}
template <bool NT, class V>
__device__ __forceinline__ void st1(V *p, V v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one env-like step of agent a: the arithmetic is a stand-in (a few flops), the bytes are exact
template <bool NT, bool COAL>
__device__ __forceinline__ void step_body(int64_t A, int64_t a, int k, float &px, float &py,
                                          const float2 *act, float4 *obs, float *rew,
                                          uint8_t *done) {
    const float2 ac = act[(int64_t)k * A + a];
    px = fminf(fmaxf(px + 10.f * ac.x, 0.f), 400.f);
    py = fminf(fmaxf(py + 10.f * ac.y, 0.f), 600.f);
    if (COAL) {
        // the wave's 64 obs rows (2 KiB) as two fully contiguous 1 KiB float4 stores, as the
        // env kernels' LDS-staged store_obs_rows issue them (values are stand-ins)
        const int64_t w0 = (a & ~(int64_t)63) * 2, l = a & 63;
        float4 *o = obs + (int64_t)k * A * 2 + w0;
        st4<NT>(o + l, make_float4(px * 0.0025f, py * 0.001666f, px, py));
        st4<NT>(o + 64 + l, make_float4(py, px, py * 0.5f, px * 0.5f));
    } else {
        float4 *o = obs + ((int64_t)k * A + a) * 2;
        st4<NT>(o, make_float4(px * 0.0025f, py * 0.001666f, px, py));
        st4<NT>(o + 1, make_float4(py, px, py * 0.5f, px * 0.5f));
    }
    st1<NT>(rew + (int64_t)k * A + a, px - py);
    st1<NT>(done + (int64_t)k * A + a, (uint8_t)(px > 399.f));
}

template <bool COAL>
__global__ __launch_bounds__(256) void k_fused(int64_t A, float *spx, float *spy, const float2 *act,
                                               float4 *obs, float *rew, uint8_t *done) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    float px = spx[a], py = spy[a];
    for (int k = 0; k < T; ++k) step_body<false, COAL>(A, a, k, px, py, act, obs, rew, done);
    spx[a] = px;
    spy[a] = py;
}

template <bool NT, bool COAL>
__global__ __launch_bounds__(256) void k_step(int64_t A, int k, float *spx, float *spy,
                                              const float2 *act, float4 *obs, float *rew,
                                              uint8_t *done) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    float px = spx[a], py = spy[a];
    step_body<NT, COAL>(A, a, k, px, py, act, obs, rew, done);
    spx[a] = px;
    spy[a] = py;
}

template <class F>
void timeit(const char *name, double bytes, F f, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 5; ++w) f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-40s best %.3f ms (%.1f us/step) %7.1f GB/s of 45 B/agent-step   median %.3f ms\n", name,
           t[0], t[0] * 1e3 / T, bytes / t[0] / 1e6, t[reps / 2]);
    fflush(stdout);
}

int main() {
    const int64_t A = 5242880;
    float *spx, *spy;
    float2 *act;
    float4 *obs;
    float *rew;
    uint8_t *done;
    CK(hipMalloc(&spx, A * 4));
    CK(hipMalloc(&spy, A * 4));
    CK(hipMalloc(&act, T * A * 8));
    CK(hipMalloc(&obs, T * A * 32));
    CK(hipMalloc(&rew, T * A * 4));
    CK(hipMalloc(&done, T * A));
    CK(hipMemset(spx, 0, A * 4));
    CK(hipMemset(spy, 0, A * 4));
    CK(hipMemset(act, 0, T * A * 8));
    const unsigned g = (unsigned)((A + 255) / 256);
    const double byt = 45.0 * A * T;  // the fused rollout's per-step bytes (state excluded)
    for (int round = 0; round < 3; ++round) {
        timeit("fused (T-plane, state in registers)", byt, [&] {
            hipLaunchKernelGGL((k_fused<false>), dim3(g), dim3(256), 0, 0, A, spx, spy, act, obs,
                               rew, done);
        });
        timeit("fused, coalesced obs", byt, [&] {
            hipLaunchKernelGGL((k_fused<true>), dim3(g), dim3(256), 0, 0, A, spx, spy, act, obs,
                               rew, done);
        });
        timeit("step launches, plain stores", byt, [&] {
            for (int k = 0; k < T; ++k)
                hipLaunchKernelGGL((k_step<false, false>), dim3(g), dim3(256), 0, 0, A, k, spx, spy,
                                   act, obs, rew, done);
        });
        timeit("step launches, coalesced obs", byt, [&] {
            for (int k = 0; k < T; ++k)
                hipLaunchKernelGGL((k_step<false, true>), dim3(g), dim3(256), 0, 0, A, k, spx, spy,
                                   act, obs, rew, done);
        });
        timeit("step launches, coalesced, non-temporal", byt, [&] {
            for (int k = 0; k < T; ++k)
                hipLaunchKernelGGL((k_step<true, true>), dim3(g), dim3(256), 0, 0, A, k, spx, spy,
                                   act, obs, rew, done);
        });
    }
    CK(hipDeviceSynchronize());
    return 0;
}
