// Where does the rollout's write pattern lose bandwidth against a plain stream?  tools/ubench_bw
// measured 6.9-7.1 TB/s for float4 writes of one 4 KiB chunk per 256-thread block, but the
// rollout's byte mix (k_mix: a block keeps CH agents for T steps and writes one row of each of
// the obs / reward / done planes per step) reaches 5.0-5.4 TB/s.  This morphs one into the other:
//   planes<T,U> : a block writes its 4U KiB chunk in each of T planes (plane stride = buffer/T)
//   mix<CH>     : the rollout's exact streams (tools/ubench_ceiling.hip's k_mix), T = 10 or 1,
//                 obs only or all streams, linear or XCD-major chunk order
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_bw2 ubench_bw2.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float v4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ size_t chunk_of(size_t b, size_t nch, int scatter) {
    if (scatter == 0 || (nch & 7)) return b;
    return (b & 7) * (nch >> 3) + (b >> 3);   // XCD-major: blocks b, b+8, ... take one contiguous run
}

template <int U>
__global__ __launch_bounds__(256) void k_planes(v4 *__restrict__ out, size_t nch, size_t pstride, int T, int scatter) {
    const size_t c = chunk_of(blockIdx.x, nch, scatter);
    const size_t base = c * (size_t)(256 * U) + threadIdx.x;
    for (int k = 0; k < T; ++k) {
#pragma unroll
        for (int j = 0; j < U; ++j) out[k * pstride + base + (size_t)j * 256] = (v4){(float)j, (float)k, 2.f, (float)c};
    }
}

// k_mix: CH agents per 256-thread block for T steps; act [T][A][2] read, obs [T][A][8], rew [T][A],
// done [T][A] (bytes) written; obs_only skips rew/done.
template <int CH>
__global__ __launch_bounds__(256) void k_mix(const v4 *__restrict__ act, v4 *__restrict__ obs, v4 *__restrict__ rew,
                                             v4 *__restrict__ done, long A, int T, int scatter, int obs_only) {
    constexpr int NA = CH * 8 / 16, NO = CH * 32 / 16, NR = CH * 4 / 16, ND = CH / 16;
    constexpr int PA = (NA + 255) / 256;
    const int tid = threadIdx.x;
    const long nch = A / CH;
    const long c0 = (long)chunk_of(blockIdx.x, nch, scatter) * CH;
    v4 a[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) a[j] = (tid + 256 * j < NA) ? act[(c0 * 8) / 16 + tid + 256 * j] : (v4){0, 0, 0, 0};
    for (int k = 0; k < T; ++k) {
        v4 cur[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) cur[j] = a[j];
        if (k + 1 < T) {
#pragma unroll
            for (int j = 0; j < PA; ++j)
                if (tid + 256 * j < NA) a[j] = act[((long)(k + 1) * A * 8 + c0 * 8) / 16 + tid + 256 * j];
        }
        const float s = cur[0].x + cur[PA - 1].w;
        v4 *o = obs + ((long)k * A * 32 + c0 * 32) / 16;
#pragma unroll
        for (int j = 0; j < NO / 256; ++j) o[tid + 256 * j] = (v4){s, cur[j % PA].y, cur[j % PA].z, 1.f};
        if (obs_only) continue;
        v4 *r = rew + ((long)k * A * 4 + c0 * 4) / 16;
        for (int q = tid; q < NR; q += 256) r[q] = (v4){s, s, s, s};
        v4 *d = done + ((long)k * A + c0) / 16;
        if (tid < ND) d[tid] = (v4){s, 0.f, s, 0.f};
    }
}

template <class F>
void timeit(const char *name, double bytes, F f, int reps = 20) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-52s best %.3f ms %7.1f GB/s   median %.3f ms %7.1f GB/s\n", name, t[0], bytes / t[0] / 1e6,
           t[reps / 2], bytes / t[reps / 2] / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main() {
    char nm[128];
    {
        const size_t bytes = (size_t)2 << 30, n = bytes / 16;
        v4 *y; CK(hipMalloc(&y, bytes)); CK(hipMemset(y, 0, bytes));
        for (int T : {1, 2, 10}) for (int sc : {0, 1}) {
            const size_t ps = n / T, nch1 = ps / 256, nch4 = ps / 1024;
            snprintf(nm, sizeof nm, "planes U=1 T=%d scatter=%d", T, sc);
            timeit(nm, 1.0 * nch1 * 4096 * T, [&] { hipLaunchKernelGGL((k_planes<1>), dim3(nch1), dim3(256), 0, 0, y, nch1, ps, T, sc); });
            snprintf(nm, sizeof nm, "planes U=4 T=%d scatter=%d", T, sc);
            timeit(nm, 1.0 * nch4 * 16384 * T, [&] { hipLaunchKernelGGL((k_planes<4>), dim3(nch4), dim3(256), 0, 0, y, nch4, ps, T, sc); });
        }
        CK(hipFree(y));
    }
    const long A = 5242880;   // BASELINE config 3 at N = 5
    const int TT = 10;
    v4 *act, *obs, *rew, *done;
    CK(hipMalloc(&act, (size_t)TT * A * 8)); CK(hipMalloc(&obs, (size_t)TT * A * 32));
    CK(hipMalloc(&rew, (size_t)TT * A * 4)); CK(hipMalloc(&done, (size_t)TT * A));
    CK(hipMemset(act, 0, (size_t)TT * A * 8));
#define MIX(CH, T, SC, OO) { const unsigned nb = (unsigned)(A / CH); \
        snprintf(nm, sizeof nm, "mix CH=%d T=%d scatter=%d obs_only=%d", CH, T, SC, OO); \
        timeit(nm, (double)A * T * ((OO) ? 40.0 : 45.0), [&] { hipLaunchKernelGGL((k_mix<CH>), dim3(nb), dim3(256), 0, 0, act, obs, rew, done, A, T, SC, OO); }); }
    MIX(512, 10, 0, 0) MIX(512, 10, 1, 0) MIX(512, 10, 0, 1) MIX(512, 10, 1, 1)
    MIX(512, 1, 0, 0) MIX(512, 1, 1, 0) MIX(512, 2, 0, 0) MIX(512, 2, 1, 0)
    MIX(1024, 10, 0, 0) MIX(1024, 10, 1, 0) MIX(128, 10, 0, 0) MIX(128, 10, 1, 0)
    return 0;
}
