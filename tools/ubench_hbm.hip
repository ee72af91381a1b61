// HBM calibration micro-benchmark for the env rollout's access pattern (gfx950).
// Measures the bandwidth ceiling of: float4 copy, float4 write-only, and the rollout's
// per-agent-step pattern (8 B action read, 32 B obs + 4 B reward + 1 B done written), with and
// without non-temporal stores.  Build: hipcc --offload-arch=gfx950 -O3 -o ubench_hbm ubench_hbm.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_copy(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}
__global__ void k_write(float4 *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
// one lane per agent, 60 active lanes per wave (N=5 packing), T steps
template <bool NT, bool DONE, bool PF>
__global__ __launch_bounds__(256) void k_pattern(const float2 *__restrict__ act, float *__restrict__ obs,
                                                 float *__restrict__ rew, unsigned char *__restrict__ done,
                                                 long A, int T) {
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long a = wave * 60 + lane;
    const bool active = lane < 60 && a < A;
    float acc = 0.f;
    float2 an = active ? act[a] : make_float2(0, 0);
    float2 an2 = (PF && active && T > 1) ? act[A + a] : make_float2(0, 0);
    for (int k = 0; k < T; ++k) {
        float2 ac = an;
        if (PF) { an = an2; if (active && k + 2 < T) an2 = act[(long)(k + 2) * A + a]; }
        else if (active && k + 1 < T) an = act[(long)(k + 1) * A + a];
        acc += ac.x * 0.5f + ac.y;
        if (active) {
            long row = (long)k * A + a;
            float4 o0 = make_float4(acc, ac.x, ac.y, 1.f), o1 = make_float4(ac.y, acc, 2.f, 3.f);
            float4 *o = reinterpret_cast<float4 *>(obs + row * 8);
            if (NT) {
                v4f *ov = reinterpret_cast<v4f *>(o);
                __builtin_nontemporal_store((v4f){o0.x, o0.y, o0.z, o0.w}, ov);
                __builtin_nontemporal_store((v4f){o1.x, o1.y, o1.z, o1.w}, ov + 1);
                __builtin_nontemporal_store(acc, rew + row);
                if (DONE) __builtin_nontemporal_store((unsigned char)(acc > 0.f), done + row);
            } else {
                o[0] = o0; o[1] = o1; rew[row] = acc;
                if (DONE) done[row] = (unsigned char)(acc > 0.f);
            }
        }
    }
}


// variant with wave-private LDS transpose: each store instruction writes 1 KiB contiguous
template <bool NT, bool PACKDONE>
__global__ __launch_bounds__(256) void k_pattern_lds(const float2 *__restrict__ act, float *__restrict__ obs,
                                                     float *__restrict__ rew, unsigned char *__restrict__ done,
                                                     long A, int T) {
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8 + 16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long a0 = wave * 60;
    const long a = a0 + lane;
    const bool active = lane < 60 && a < A;
    const int nact = (int)((A - a0) < 60 ? (A - a0) : 60);
    float acc = 0.f;
    float2 an = active ? act[a] : make_float2(0, 0);
    float *st = stage[w];
    for (int k = 0; k < T; ++k) {
        float2 ac = an;
        if (active && k + 1 < T) an = act[(long)(k + 1) * A + a];
        acc += ac.x * 0.5f + ac.y;
        const long row0 = (long)k * A + a0;
        v4f o0 = {acc, ac.x, ac.y, 1.f}, o1 = {ac.y, acc, 2.f, 3.f};
        *reinterpret_cast<v4f *>(&st[lane * 8]) = o0;
        *reinterpret_cast<v4f *>(&st[lane * 8 + 4]) = o1;
        if (PACKDONE) reinterpret_cast<unsigned char *>(&st[512])[lane] = (unsigned char)(acc > 0.f);
        __builtin_amdgcn_wave_barrier();
        v4f *ob = reinterpret_cast<v4f *>(obs + row0 * 8);
        const int nq = nact * 2;  // float4 count of this wave's obs rows
        v4f q0 = *reinterpret_cast<v4f *>(&st[lane * 4]);
        v4f q1 = *reinterpret_cast<v4f *>(&st[(lane + 64) * 4]);
        if (NT) {
            if (lane < nq) __builtin_nontemporal_store(q0, ob + lane);
            if (lane + 64 < nq) __builtin_nontemporal_store(q1, ob + lane + 64);
            if (active) __builtin_nontemporal_store(acc, rew + row0 + lane);
        } else {
            if (lane < nq) ob[lane] = q0;
            if (lane + 64 < nq) ob[lane + 64] = q1;
            if (active) rew[row0 + lane] = acc;
        }
        if (PACKDONE) {
            unsigned int dw = reinterpret_cast<unsigned int *>(&st[512])[lane];
            if (lane < nact / 4) {
                if (NT) __builtin_nontemporal_store(dw, reinterpret_cast<unsigned int *>(done + row0) + lane);
                else reinterpret_cast<unsigned int *>(done + row0)[lane] = dw;
            }
        } else if (active) {
            if (NT) __builtin_nontemporal_store((unsigned char)(acc > 0.f), done + row0 + lane);
            else done[row0 + lane] = (unsigned char)(acc > 0.f);
        }
        __builtin_amdgcn_wave_barrier();
    }
}


// explore: PFALL = prefetch all T action loads at entry; TWO = each lane owns 2 agents (2 groups
// of 60 in one wave); PERSIST = grid of 256*8 blocks striding over wave tiles.
template <bool PFALL, bool TWO, bool PERSIST>
__global__ __launch_bounds__(256) void k_explore(const float2 *__restrict__ act, float *__restrict__ obs,
                                                 float *__restrict__ rew, unsigned char *__restrict__ done,
                                                 long A, int T, long ntiles) {
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *st = stage[w];
    const long wstride = PERSIST ? (long)gridDim.x * 4 : 0;
    for (long tile = (long)blockIdx.x * 4 + w; tile < ntiles; tile += (PERSIST ? wstride : ntiles)) {
        constexpr int G = TWO ? 2 : 1;
        long a0[G]; bool active[G]; float acc[G]; float2 an[G];
        float2 pre[16];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            a0[g] = (tile * G + g) * 60;
            active[g] = lane < 60 && a0[g] + lane < A;
            acc[g] = 0.f;
            an[g] = active[g] ? act[a0[g] + lane] : make_float2(0, 0);
        }
        if (PFALL) {
#pragma unroll
            for (int k = 0; k < 16; ++k) pre[k] = (k < T && active[0]) ? act[(long)k * A + a0[0] + lane] : make_float2(0, 0);
        }
        for (int k = 0; k < T; ++k) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float2 ac = an[g];
                if (PFALL && g == 0) {
                    ac = make_float2(0, 0);
#pragma unroll
                    for (int q = 0; q < 16; ++q) if (q == k) ac = pre[q];
                } else if (active[g] && k + 1 < T) an[g] = act[(long)(k + 1) * A + a0[g] + lane];
                acc[g] += ac.x * 0.5f + ac.y;
                const long row0 = (long)k * A + a0[g];
                v4f o0 = {acc[g], ac.x, ac.y, 1.f}, o1 = {ac.y, acc[g], 2.f, 3.f};
                *reinterpret_cast<v4f *>(&st[lane * 8]) = o0;
                *reinterpret_cast<v4f *>(&st[lane * 8 + 4]) = o1;
                __builtin_amdgcn_wave_barrier();
                v4f *ob = reinterpret_cast<v4f *>(obs + row0 * 8);
                v4f q0 = *reinterpret_cast<v4f *>(&st[lane * 4]);
                v4f q1 = *reinterpret_cast<v4f *>(&st[(lane + 64) * 4]);
                const long left = A - a0[g];
                const int nq = 2 * (int)(left <= 0 ? 0 : (left < 60 ? left : 60));
                if (lane < nq) ob[lane] = q0;
                if (lane + 64 < nq) ob[lane + 64] = q1;
                if (active[g]) { rew[row0 + lane] = acc[g]; done[row0 + lane] = (unsigned char)(acc[g] > 0.f); }
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

template <class F>
float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t bytes = (size_t)2 << 30;  // 2 GiB per buffer
    float4 *x, *y; CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
    size_t n = bytes / 16;
    for (int blocks : {2048, 8192, 65536}) {
        float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, x, y, n); }, 10);
        printf("copy   blocks=%6d  %.1f GB/s (read+write)\n", blocks, 2.0 * bytes / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_write, dim3(blocks), dim3(256), 0, 0, y, n); }, 10);
        printf("write  blocks=%6d  %.1f GB/s\n", blocks, 1.0 * bytes / ms / 1e6);
    }
    const long A = 5242880; const int T = 10;
    float2 *act; float *obs, *rew; unsigned char *done;
    CK(hipMalloc(&act, (size_t)T * A * 8)); CK(hipMalloc(&obs, (size_t)T * A * 32));
    CK(hipMalloc(&rew, (size_t)T * A * 4)); CK(hipMalloc(&done, (size_t)T * A));
    CK(hipMemset(act, 0, (size_t)T * A * 8));
    const long waves = (A + 59) / 60; const unsigned blocks = (unsigned)((waves + 3) / 4);
    const double algo = (double)A * T * 45.0;
#define RUN(NT, DN, PF) { float ms = timeit([&] { hipLaunchKernelGGL((k_pattern<NT, DN, PF>), dim3(blocks), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20); \
        printf("pattern nt=%d done=%d pf2=%d  %.3f ms  %.1f GB/s (algorithmic 45 B/agent-step)\n", NT, DN, PF, ms, algo / ms / 1e6); }
    RUN(false, true, false) RUN(true, true, false) RUN(false, false, false) RUN(true, false, false)
    RUN(false, true, true) RUN(true, true, true)
#define RUNL(NT, PD) { float ms = timeit([&] { hipLaunchKernelGGL((k_pattern_lds<NT, PD>), dim3(blocks), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20); \
        printf("lds-transpose nt=%d packdone=%d  %.3f ms  %.1f GB/s\n", NT, PD, ms, algo / ms / 1e6); }
    RUNL(false, false) RUNL(true, false) RUNL(false, true) RUNL(true, true)
#define RUNX(PF, TW, PE, NB) { const long nt = (waves + (TW ? 1 : 0)) / (TW ? 2 : 1); unsigned nb = PE ? NB : (unsigned)((nt + 3) / 4); \
        float ms = timeit([&] { hipLaunchKernelGGL((k_explore<PF, TW, PE>), dim3(nb), dim3(256), 0, 0, act, obs, rew, done, A, T, nt); }, 20); \
        printf("explore pfall=%d two=%d persist=%d blocks=%u  %.3f ms  %.1f GB/s\n", PF, TW, PE, nb, ms, algo / ms / 1e6); }
    RUNX(false, false, false, 0) RUNX(true, false, false, 0) RUNX(false, true, false, 0)
    RUNX(false, false, true, 2048) RUNX(false, false, true, 4096) RUNX(false, false, true, 8192)
    RUNX(true, false, true, 2048) RUNX(false, true, true, 2048)
    return 0;
}
