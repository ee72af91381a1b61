// Follow-up of tools/ubench_bw2: float4 writes of one chunk per block into T planes fall from
// 7.07 TB/s (T = 1) to 6.7 (T = 2) and 5.1 (T = 10).  Is it the number of planes written at the
// same moment (blocks at different steps), or the resident block count (the width of the write
// front)?  Planes are 160 MiB apart, like the rollout's obs planes at config 3.
//   planes  bpc : non-persistent grid, resident blocks per CU capped at bpc by dynamic LDS
//   inter   R   : persistent grid, loops interchanged over R rounds of chunks (see k_inter)
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_bw3 ubench_bw3.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float v4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_planes(v4 *__restrict__ out, size_t pstride, int T) {
    extern __shared__ float pad[];
    const size_t c = blockIdx.x;
    const size_t base = c * (size_t)(256 * U) + threadIdx.x;
    for (int k = 0; k < T; ++k) {
#pragma unroll
        for (int j = 0; j < U; ++j) out[k * pstride + base + (size_t)j * 256] = (v4){(float)j, (float)k, 2.f, (float)c};
    }
    if (T < 0) pad[threadIdx.x] = 0.f;  // keep the allocation
}

// interchanged loops: a persistent block takes R consecutive rounds of chunks at a time and
// writes plane k of all R before plane k + 1 (R = all rounds: the whole grid sweeps one plane at a
// time; R = 1: k_planes' order on a persistent grid)
template <int U>
__global__ __launch_bounds__(256) void k_inter(v4 *__restrict__ out, size_t pstride, int T, size_t nch, int R) {
    const size_t G = gridDim.x;
    for (size_t q = 0; q * G < nch; q += R) {
        for (int k = 0; k < T; ++k) {
            for (int rr = 0; rr < R; ++rr) {
                const size_t c = (q + rr) * G + blockIdx.x;
                if (c >= nch) break;
                const size_t base = c * (size_t)(256 * U) + threadIdx.x;
#pragma unroll
                for (int j = 0; j < U; ++j) out[k * pstride + base + (size_t)j * 256] = (v4){(float)j, (float)k, 2.f, (float)c};
            }
        }
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
    const size_t plane = (size_t)160 << 20;  // bytes per plane (the obs plane at config 3)
    const int TMAX = 10;
    v4 *y; CK(hipMalloc(&y, plane * TMAX)); CK(hipMemset(y, 0, plane * TMAX));
    const size_t ps = plane / 16;
    char nm[128];
    for (int T : {1, 10}) for (int bpc : {1, 2, 4, 8}) {
        const size_t lds = (160 * 1024) / bpc - 1024;
        // T = 1: one 1.6 GiB plane (a 160 MiB one would live in the 256 MiB Infinity Cache)
        const size_t pl = T == 1 ? ps * TMAX : ps, n1 = pl / 256, n4 = pl / 1024;
        const double byt = 16.0 * pl * T;
        snprintf(nm, sizeof nm, "planes U=1 T=%d bpc<=%d", T, bpc);
        timeit(nm, byt, [&] { hipLaunchKernelGGL((k_planes<1>), dim3(n1), dim3(256), lds, 0, y, pl, T); });
        snprintf(nm, sizeof nm, "planes U=4 T=%d bpc<=%d", T, bpc);
        timeit(nm, byt, [&] { hipLaunchKernelGGL((k_planes<4>), dim3(n4), dim3(256), lds, 0, y, pl, T); });
    }
    for (int bpc : {2, 8}) for (int R : {1, 2, 4, 1 << 20}) {
        const unsigned G = 256 * bpc;
        const size_t n1 = ps / 256, n4 = ps / 1024;
        snprintf(nm, sizeof nm, "inter U=1 T=10 blocks=%u R=%d", G, R);
        timeit(nm, (double)plane * 10, [&] { hipLaunchKernelGGL((k_inter<1>), dim3(G), dim3(256), 0, 0, y, ps, 10, n1, R); });
        snprintf(nm, sizeof nm, "inter U=4 T=10 blocks=%u R=%d", G, R);
        timeit(nm, (double)plane * 10, [&] { hipLaunchKernelGGL((k_inter<4>), dim3(G), dim3(256), 0, 0, y, ps, 10, n4, R); });
    }
    return 0;
}
