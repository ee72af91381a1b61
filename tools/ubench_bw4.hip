// Follow-up of tools/ubench_bw3: T = 10 planes of writes run at 5.1-6.7 TB/s against 7.1 for one
// plane.  At any moment the resident blocks are spread over the T steps, and every block writes
// the SAME in-plane offset range in each plane, so ten write fronts sit at addresses that differ
// by multiples of the plane stride (160 MiB at config 3 = 5 x 2^25 B).  If those alias in the
// HBM channel / bank map, the fronts collide.  This pads the plane stride by delta bytes:
//   planes delta : float4 writes of one 4 KiB chunk per block in each of 10 planes
//   mix    delta : the rollout's byte mix (tools/ubench_bw2.hip k_mix) with every plane (obs,
//                  reward, done, actions) padded by delta bytes
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_bw4 ubench_bw4.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float v4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_planes(v4 *__restrict__ out, size_t pstride, int T) {
    const size_t c = blockIdx.x;
    const size_t base = c * 256 + threadIdx.x;
    for (int k = 0; k < T; ++k) out[k * pstride + base] = (v4){1.f, (float)k, 2.f, (float)c};
}

// strides in float4 units: sa (actions), so (obs), sr (reward), sd (done)
template <int CH>
__global__ __launch_bounds__(256) void k_mix(const v4 *__restrict__ act, v4 *__restrict__ obs, v4 *__restrict__ rew,
                                             v4 *__restrict__ done, int T, size_t sa, size_t so, size_t sr, size_t sd) {
    constexpr int NA = CH * 8 / 16, NO = CH * 32 / 16, NR = CH * 4 / 16, ND = CH / 16;
    constexpr int PA = (NA + 255) / 256;
    const int tid = threadIdx.x;
    const long c0 = (long)blockIdx.x * CH;
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
                if (tid + 256 * j < NA) a[j] = act[(k + 1) * sa + (c0 * 8) / 16 + tid + 256 * j];
        }
        const float s = cur[0].x + cur[PA - 1].w;
        v4 *o = obs + k * so + (c0 * 32) / 16;
#pragma unroll
        for (int j = 0; j < NO / 256; ++j) o[tid + 256 * j] = (v4){s, cur[j % PA].y, cur[j % PA].z, 1.f};
        v4 *r = rew + k * sr + (c0 * 4) / 16;
        for (int q = tid; q < NR; q += 256) r[q] = (v4){s, s, s, s};
        v4 *d = done + k * sd + c0 / 16;
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
    printf("%-44s best %.3f ms %7.1f GB/s   median %.3f ms %7.1f GB/s\n", name, t[0], bytes / t[0] / 1e6,
           t[reps / 2], bytes / t[reps / 2] / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main() {
    const int T = 10;
    const long A = 5242880;                        // config 3 agents
    const size_t plane = (size_t)A * 32;           // obs plane, 160 MiB
    const long deltas[] = {0, 4096, 65536, 1 << 20, (1 << 20) + 4096, 3 * 4096 + 256, 2621440 + 12288};
    size_t maxd = 0;  // allocations are padded by the largest delta (checked on the host)
    for (long dl : deltas) maxd = std::max(maxd, (size_t)dl);
    maxd = (maxd + 4095) & ~(size_t)4095;
    v4 *y; CK(hipMalloc(&y, (plane + maxd) * T)); CK(hipMemset(y, 0, (plane + maxd) * T));
    char nm[128];
    for (long dl : deltas) {
        const size_t ps = (plane + dl) / 16, nch = plane / 4096;
        snprintf(nm, sizeof nm, "planes T=10 delta=%ld", dl);
        timeit(nm, (double)plane * T, [&] { hipLaunchKernelGGL(k_planes, dim3(nch), dim3(256), 0, 0, y, ps, T); });
    }
    CK(hipFree(y));
    v4 *act, *obs, *rew, *done;
    CK(hipMalloc(&act, ((size_t)A * 8 + maxd) * T)); CK(hipMalloc(&obs, ((size_t)A * 32 + maxd) * T));
    CK(hipMalloc(&rew, ((size_t)A * 4 + maxd) * T)); CK(hipMalloc(&done, ((size_t)A + maxd) * T));
    CK(hipMemset(act, 0, ((size_t)A * 8 + maxd) * T));
    for (long dl : deltas) {
        const size_t sa = ((size_t)A * 8 + dl) / 16, so = ((size_t)A * 32 + dl) / 16;
        const size_t sr = ((size_t)A * 4 + dl) / 16, sd = ((size_t)A + dl) / 16;
        snprintf(nm, sizeof nm, "mix CH=512 T=10 delta=%ld", dl);
        timeit(nm, (double)A * T * 45.0, [&] { hipLaunchKernelGGL((k_mix<512>), dim3(A / 512), dim3(256), 0, 0, act, obs, rew, done, T, sa, so, sr, sd); });
    }
    return 0;
}
