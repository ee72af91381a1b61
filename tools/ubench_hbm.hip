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
// copy with 4 independent float4 loads in flight per thread (the guide's 6.3 TB/s form)
__global__ __launch_bounds__(256) void k_copy4(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        float4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
    }
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


// component ablation of the lds-transpose pattern: bit 0 action loads, 1 obs stores, 2 reward
// stores, 3 done stores (what each stream costs on its own and in the mix)
// blockIdx -> logical block so that the blocks one XCD receives (b, b+8, b+16, ...: round-robin
// dispatch over the 8 XCDs) cover one contiguous range of the data: lines shared by neighbouring
// blocks are then written through one L2.  A bijection for any grid size.
__device__ __forceinline__ long xcd_block(long b, long nb) {
    const long q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}
template <int M, int LN = 60, bool XCD = false>
__global__ __launch_bounds__(256) void k_ablate(const float2 *__restrict__ act, float *__restrict__ obs,
                                                float *__restrict__ rew, unsigned char *__restrict__ done,
                                                long A, int T) {
    __shared__ __attribute__((aligned(16))) float stage[4][64 * 8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long blk = XCD ? xcd_block(blockIdx.x, gridDim.x) : (long)blockIdx.x;
    const long wave = blk * 4 + (threadIdx.x >> 6);
    const long a0 = wave * LN;
    const long a = a0 + lane;
    const bool active = lane < LN && a < A;
    const int nact = (int)((A - a0) < LN ? (A - a0) : LN);
    float acc = 0.f;
    float2 an = (M & 1) && active ? act[a] : make_float2(0.25f, (float)lane);
    float *st = stage[w];
    for (int k = 0; k < T; ++k) {
        float2 ac = an;
        if ((M & 1) && active && k + 1 < T) an = act[(long)(k + 1) * A + a];
        acc += ac.x * 0.5f + ac.y;
        const long row0 = (long)k * A + a0;
        if (M & 2) {
            v4f o0 = {acc, ac.x, ac.y, 1.f}, o1 = {ac.y, acc, 2.f, 3.f};
            *reinterpret_cast<v4f *>(&st[lane * 8]) = o0;
            *reinterpret_cast<v4f *>(&st[lane * 8 + 4]) = o1;
            __builtin_amdgcn_wave_barrier();
            v4f *ob = reinterpret_cast<v4f *>(obs + row0 * 8);
            const int nq = nact * 2;
            v4f q0 = *reinterpret_cast<v4f *>(&st[lane * 4]);
            v4f q1 = *reinterpret_cast<v4f *>(&st[(lane + 64) * 4]);
            if (lane < nq) ob[lane] = q0;
            if (lane + 64 < nq) ob[lane + 64] = q1;
            __builtin_amdgcn_wave_barrier();
        }
        if ((M & 4) && active) rew[row0 + lane] = acc;
        if ((M & 8) && active) done[row0 + lane] = (unsigned char)(acc > 0.f);
    }
    if (!(M & 14) && acc == 12345.f) rew[a] = acc;
}

// two consecutive agents per lane (PW agents per wave, PW <= 128): float4 action loads, float2
// reward stores, 2-byte done stores, obs rows staged through a 4 KiB wave slice
template <int PW>
__global__ __launch_bounds__(256) void k_pair(const float2 *__restrict__ act, float *__restrict__ obs,
                                              float *__restrict__ rew, unsigned char *__restrict__ done,
                                              long A, int T) {
    __shared__ __attribute__((aligned(16))) float stage[4][128 * 8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long a0 = wave * PW;
    const long a = a0 + 2 * lane;
    const bool active = 2 * lane < PW && a + 1 < A;
    const int nact = (int)((A - a0) < PW ? (A - a0) : PW);
    float acc0 = 0.f, acc1 = 0.f;
    float4 an = active ? *reinterpret_cast<const float4 *>(act + a) : make_float4(0, 0, 0, 0);
    float *st = stage[w];
    for (int k = 0; k < T; ++k) {
        float4 ac = an;
        if (active && k + 1 < T) an = *reinterpret_cast<const float4 *>(act + (long)(k + 1) * A + a);
        acc0 += ac.x * 0.5f + ac.y;
        acc1 += ac.z * 0.5f + ac.w;
        const long row0 = (long)k * A + a0;
        v4f o0 = {acc0, ac.x, ac.y, 1.f}, o1 = {ac.y, acc0, 2.f, 3.f};
        v4f o2 = {acc1, ac.z, ac.w, 1.f}, o3 = {ac.w, acc1, 2.f, 3.f};
        v4f *sv = reinterpret_cast<v4f *>(st);
        sv[4 * lane] = o0; sv[4 * lane + 1] = o1; sv[4 * lane + 2] = o2; sv[4 * lane + 3] = o3;
        __builtin_amdgcn_wave_barrier();
        v4f *ob = reinterpret_cast<v4f *>(obs + row0 * 8);
        const int nq = nact * 2;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (lane + 64 * q < nq) ob[lane + 64 * q] = sv[lane + 64 * q];
        __builtin_amdgcn_wave_barrier();
        if (active) {
            *reinterpret_cast<float2 *>(rew + row0 + 2 * lane) = make_float2(acc0, acc1);
            *reinterpret_cast<unsigned short *>(done + row0 + 2 * lane) =
                (unsigned short)((acc0 > 0.f) | ((acc1 > 0.f) << 8));
        }
    }
}

// workgroup-staged pattern: 11 waves compute 60-agent groups (whole N=5 formations, lane = agent)
// but the workgroup covers 640 agents (128 formations) = an exact number of 128-B lines in every
// stream; actions come in and outputs go out through LDS as line-aligned full-width accesses.
// One workgroup barrier per step (double-buffered staging).
template <int kWG, int kWGW>
__global__ __launch_bounds__(64 * kWGW) void k_wgstage(const float2 *__restrict__ act, float *__restrict__ obs,
                                                        float *__restrict__ rew, unsigned char *__restrict__ done,
                                                        long A, int T) {
    __shared__ __attribute__((aligned(16))) float s_obs[2][kWG * 8];
    __shared__ __attribute__((aligned(16))) float s_rew[2][kWG];
    __shared__ __attribute__((aligned(16))) unsigned char s_done[2][kWG];
    __shared__ __attribute__((aligned(16))) float2 s_act[2][kWG];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long base = (long)blockIdx.x * kWG;
    const int li = w * 60 + lane;                 // agent index inside the workgroup
    const bool active = lane < 60 && li < kWG && base + li < A;
    const int nag = (int)((A - base) < kWG ? (A - base) : kWG);
    // actions of step 0 and 1 -> LDS (float4 = 2 agents per thread)
    auto load_act = [&](int k, int buf) {
        if (k >= T) return;
        const float4 *src = reinterpret_cast<const float4 *>(act + (long)k * A + base);
        for (int q = tid; q < nag / 2; q += 64 * kWGW) reinterpret_cast<float4 *>(s_act[buf])[q] = src[q];
    };
    load_act(0, 0);
    __syncthreads();
    float acc = 0.f;
    for (int k = 0; k < T; ++k) {
        const int b = k & 1;
        load_act(k + 1, b ^ 1);
        const float2 ac = active ? s_act[b][li] : make_float2(0, 0);
        acc += ac.x * 0.5f + ac.y;
        if (active) {
            v4f o0 = {acc, ac.x, ac.y, 1.f}, o1 = {ac.y, acc, 2.f, 3.f};
            reinterpret_cast<v4f *>(s_obs[b])[2 * li] = o0;
            reinterpret_cast<v4f *>(s_obs[b])[2 * li + 1] = o1;
            s_rew[b][li] = acc;
            s_done[b][li] = (unsigned char)(acc > 0.f);
        }
        __syncthreads();
        const long row0 = (long)k * A + base;
        v4f *ob = reinterpret_cast<v4f *>(obs + row0 * 8);
        for (int q = tid; q < nag * 2; q += 64 * kWGW) ob[q] = reinterpret_cast<v4f *>(s_obs[b])[q];
        for (int q = tid; q < nag / 4; q += 64 * kWGW)
            reinterpret_cast<v4f *>(rew + row0)[q] = reinterpret_cast<v4f *>(s_rew[b])[q];
        for (int q = tid; q < nag / 4; q += 64 * kWGW)
            reinterpret_cast<unsigned int *>(done + row0)[q] = reinterpret_cast<unsigned int *>(s_done[b])[q];
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
        ms = timeit([&] { hipLaunchKernelGGL(k_copy4, dim3(blocks), dim3(256), 0, 0, x, y, n); }, 10);
        printf("copy4  blocks=%6d  %.1f GB/s (read+write)\n", blocks, 2.0 * bytes / ms / 1e6);
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
        {
#define RUNA(M) { float ms = timeit([&] { hipLaunchKernelGGL((k_ablate<M>), dim3(blocks), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20); \
        const double b = (double)A * T * (((M) & 1 ? 8 : 0) + ((M) & 2 ? 32 : 0) + ((M) & 4 ? 4 : 0) + ((M) & 8 ? 1 : 0)); \
        printf("ablate act=%d obs=%d rew=%d done=%d  %.3f ms  %.1f GB/s of its own bytes\n", (M) & 1, ((M) >> 1) & 1, ((M) >> 2) & 1, ((M) >> 3) & 1, ms, b / ms / 1e6); }
        RUNA(15) RUNA(14) RUNA(7) RUNA(11) RUNA(13) RUNA(6) RUNA(2) RUNA(3) RUNA(4) RUNA(8) RUNA(1)
        // same with 64 agents per wave: every wave's reward row is 2 whole 128-B lines
        const unsigned blocks64 = (unsigned)(((A + 63) / 64 + 3) / 4);
#define RUNB(M) { float ms = timeit([&] { hipLaunchKernelGGL((k_ablate<M, 64>), dim3(blocks64), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20); \
        const double b = (double)A * T * (((M) & 1 ? 8 : 0) + ((M) & 2 ? 32 : 0) + ((M) & 4 ? 4 : 0) + ((M) & 8 ? 1 : 0)); \
        printf("ablate64 act=%d obs=%d rew=%d done=%d  %.3f ms  %.1f GB/s of its own bytes\n", (M) & 1, ((M) >> 1) & 1, ((M) >> 2) & 1, ((M) >> 3) & 1, ms, b / ms / 1e6); }
        RUNB(15) RUNB(7) RUNB(11) RUNB(3) RUNB(4) RUNB(8)
#define RUNC(M, LN) { float ms = timeit([&] { hipLaunchKernelGGL((k_ablate<M, LN, true>), dim3(LN == 64 ? blocks64 : blocks), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20); \
        const double b = (double)A * T * (((M) & 1 ? 8 : 0) + ((M) & 2 ? 32 : 0) + ((M) & 4 ? 4 : 0) + ((M) & 8 ? 1 : 0)); \
        printf("ablate-xcd lanes=%d act=%d obs=%d rew=%d done=%d  %.3f ms  %.1f GB/s of its own bytes\n", LN, (M) & 1, ((M) >> 1) & 1, ((M) >> 2) & 1, ((M) >> 3) & 1, ms, b / ms / 1e6); }
        RUNC(15, 60) RUNC(15, 64) RUNC(7, 60) RUNC(11, 60) RUNC(3, 60) RUNC(8, 60)
        RUNA(15) RUNB(15)
        for (int pw : {120, 128}) {
            const unsigned bp = (unsigned)(((A + pw - 1) / pw + 3) / 4);
            float ms = pw == 120 ? timeit([&] { hipLaunchKernelGGL((k_pair<120>), dim3(bp), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20)
                                 : timeit([&] { hipLaunchKernelGGL((k_pair<128>), dim3(bp), dim3(256), 0, 0, act, obs, rew, done, A, T); }, 20);
            printf("pair agents/wave=%d  %.3f ms  %.1f GB/s (algorithmic 45 B/agent-step)\n", pw, ms, algo / ms / 1e6);
        }
#define RUNW(G, W) { const unsigned bw = (unsigned)((A + G - 1) / G); \
            float ms = timeit([&] { hipLaunchKernelGGL((k_wgstage<G, W>), dim3(bw), dim3(64 * W), 0, 0, act, obs, rew, done, A, T); }, 20); \
            printf("wgstage %d agents/WG, %d waves  %.3f ms  %.1f GB/s (algorithmic 45 B/agent-step)\n", G, W, ms, algo / ms / 1e6); }
        RUNW(640, 11) RUNW(240, 4) RUNW(480, 8) RUNW(960, 16)
    }
    return 0;
}
