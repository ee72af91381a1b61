// Same-box HBM ceiling for the env rollout's byte mix (gfx950).  Runs next to bench.py in one
// gpurun call so the kernel's fraction can be read against what this box's HBM delivers:
//   copy4  : float4 copy, 4 loads in flight per thread (the guide's 6.3 TB/s form)
//   write4 : float4 stores only
//   mix    : the rollout's exact streams and layout (actions [T][A][2] read; obs [T][A][8],
//            reward [T][A], done [T][A] written; 8 + 37 B per agent-step) with no arithmetic,
//            every access a whole, 128-B-aligned float4 run: chunks of CH agents per workgroup.
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_ceiling ubench_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_copy4(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        float4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
    }
}
__global__ __launch_bounds__(256) void k_write4(float4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

// CH agents per workgroup of 256 threads; CH multiple of 512 (done row = CH B = whole float4s).
template <class V>
__device__ __forceinline__ void st(V *p, V v, bool nt) {
    if (nt) __builtin_nontemporal_store(v, p); else *p = v;
}
typedef float v4 __attribute__((ext_vector_type(4)));
template <int CH, bool NT = false, bool PERSIST = false>
__global__ __launch_bounds__(256) void k_mix(const float4 *__restrict__ act, float4 *__restrict__ obs,
                                             float4 *__restrict__ rew, float4 *__restrict__ done,
                                             long A, int T) {
    constexpr int NA = CH * 8 / 16, NO = CH * 32 / 16, NR = CH * 4 / 16, ND = CH / 16;
    constexpr int PA = (NA + 255) / 256;
    const int tid = threadIdx.x;
    const long nch = A / CH;
  for (long cb = blockIdx.x; cb < nch; cb += PERSIST ? gridDim.x : nch) {
    const long c0 = cb * CH;
    float4 a[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) a[j] = (tid + 256 * j < NA) ? act[(c0 * 8) / 16 + tid + 256 * j] : make_float4(0, 0, 0, 0);
    for (int k = 0; k < T; ++k) {
        float4 cur[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) cur[j] = a[j];
        if (k + 1 < T) {
#pragma unroll
            for (int j = 0; j < PA; ++j)
                if (tid + 256 * j < NA) a[j] = act[((long)(k + 1) * A * 8 + c0 * 8) / 16 + tid + 256 * j];
        }
        const float s = cur[0].x + cur[PA - 1].w;
        v4 *o = reinterpret_cast<v4 *>(obs + ((long)k * A * 32 + c0 * 32) / 16);
#pragma unroll
        for (int j = 0; j < NO / 256; ++j) st(o + tid + 256 * j, (v4){s, cur[j % PA].y, cur[j % PA].z, 1.f}, NT);
        v4 *r = reinterpret_cast<v4 *>(rew + ((long)k * A * 4 + c0 * 4) / 16);
        for (int q = tid; q < NR; q += 256) st(r + q, (v4){s, s, s, s}, NT);
        v4 *d = reinterpret_cast<v4 *>(done + ((long)k * A + c0) / 16);
        if (tid < ND) st(d + tid, (v4){s, 0.f, s, 0.f}, NT);
    }
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void k_copy4nt(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const v4 *vi = reinterpret_cast<const v4 *>(in);
    v4 *vo = reinterpret_cast<v4 *>(out);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        v4 a = __builtin_nontemporal_load(vi + i), b = __builtin_nontemporal_load(vi + i + stride);
        v4 c = __builtin_nontemporal_load(vi + i + 2 * stride), d = __builtin_nontemporal_load(vi + i + 3 * stride);
        st(vo + i, a, NT); st(vo + i + stride, b, NT); st(vo + i + 2 * stride, c, NT); st(vo + i + 3 * stride, d, NT);
    }
}
__global__ __launch_bounds__(256) void k_write4nt(float4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    v4 *vo = reinterpret_cast<v4 *>(out);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store((v4){(float)i, 1.f, 2.f, 3.f}, vo + i);
}

template <class F>
float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    float4 *x, *y; CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
    const size_t n = bytes / 16;
    for (int blocks : {2048, 8192, 32768}) {
        float ms = timeit([&] { hipLaunchKernelGGL(k_copy4, dim3(blocks), dim3(256), 0, 0, x, y, n); }, 20);
        printf("copy4  blocks=%6d  %.3f ms  %.1f GB/s (read+write)\n", blocks, ms, 2.0 * bytes / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_write4, dim3(blocks), dim3(256), 0, 0, y, n); }, 20);
        printf("write4 blocks=%6d  %.3f ms  %.1f GB/s\n", blocks, ms, 1.0 * bytes / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_copy4nt<true>, dim3(blocks), dim3(256), 0, 0, x, y, n); }, 20);
        printf("copy4 nt-load nt-store blocks=%6d  %.3f ms  %.1f GB/s\n", blocks, ms, 2.0 * bytes / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_copy4nt<false>, dim3(blocks), dim3(256), 0, 0, x, y, n); }, 20);
        printf("copy4 nt-load blocks=%6d  %.3f ms  %.1f GB/s\n", blocks, ms, 2.0 * bytes / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_write4nt, dim3(blocks), dim3(256), 0, 0, y, n); }, 20);
        printf("write4 nt blocks=%6d  %.3f ms  %.1f GB/s\n", blocks, ms, 1.0 * bytes / ms / 1e6);
    }
    CK(hipFree(x)); CK(hipFree(y));
    const long A = 5242880; const int T = 10;  // BASELINE config 3 at N = 5, one 10-step launch
    float4 *act, *obs, *rew, *done;
    CK(hipMalloc(&act, (size_t)T * A * 8)); CK(hipMalloc(&obs, (size_t)T * A * 32));
    CK(hipMalloc(&rew, (size_t)T * A * 4)); CK(hipMalloc(&done, (size_t)T * A));
    CK(hipMemset(act, 0, (size_t)T * A * 8));
    const double algo = (double)A * T * 45.0;
#define RUNM(CH) { const unsigned nb = (unsigned)(A / CH); \
        float ms = timeit([&] { hipLaunchKernelGGL((k_mix<CH>), dim3(nb), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 50); \
        printf("mix CH=%5d  %.3f ms  %.1f GB/s (8 B read + 37 B written per agent-step)\n", CH, ms, algo / ms / 1e6); }
    RUNM(512) RUNM(1024) RUNM(2048) RUNM(4096)
#define RUNV(CH, NT, PE, NB) { const unsigned nb = PE ? NB : (unsigned)(A / CH); \
        float ms = timeit([&] { hipLaunchKernelGGL((k_mix<CH, NT, PE>), dim3(nb), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 50); \
        printf("mix CH=%5d nt=%d persistent=%d blocks=%u  %.3f ms  %.1f GB/s\n", CH, NT, PE, nb, ms, algo / ms / 1e6); }
    RUNV(1024, true, false, 0) RUNV(512, true, false, 0)
    RUNV(1024, false, true, 1024) RUNV(1024, false, true, 2048) RUNV(512, false, true, 3072) RUNV(512, false, true, 6144)
    RUNV(1024, true, true, 2048)
    return 0;
}
