// Does the ORDER in which a launch's workgroups walk the T output planes move the HBM rate of the
// env rollout's byte mix?  (Round 5: the headline launch sits at ~0.99 of k_mix, which walks
// slice-major like the env kernel -- each workgroup writes its agents' rows in all T planes in
// turn, so the chip's write front spans all T planes at once.)
//   slice  k_mix's order: block b owns agents [b*CH, (b+1)*CH) for all T steps (grid A/CH)
//   plane  persistent blocks, block b owns S consecutive chunks and walks them step-major:
//          step t of all its chunks, then step t+1 -- the chip's write front sits in ~1 plane
// Same bytes (actions 8 B read, obs 32 + reward 4 + done 1 B written per agent-step), no
// arithmetic, whole float4 runs, plain and non-temporal stores.  Config 3's shape by default.
//   hipcc --offload-arch=gfx950 -O3 -o tools/plane_order_ubench tools/plane_order_ubench.hip
//   slice_split  slice order as S back-to-back launches over consecutive chunk ranges
//                (reported as grid -S): does a smaller footprint PER LAUNCH help?
//   tools/plane_order_ubench [A] [T]       -> one JSON line per variant (SPLIT_ONLY=1: no plane;
//                                             NOACT=1: no action reads; NTLOAD=1: non-temporal
//                                             action loads; ALLOC=contig|one)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

constexpr int CH = 1024;  // agents per chunk (one workgroup of 256 threads, 4 agents each)
__constant__ int act_stride0;  // 1: NOACT, 2: NTLOAD (set from the host, hipMemcpyToSymbol)

template <bool NT>
__device__ __forceinline__ void st(float4 *p, float4 v) {
    if (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}

// one chunk's step k: read its actions, write its obs / reward / done rows of plane k
template <bool NT>
__device__ __forceinline__ void chunk_step(const float4 *__restrict__ act, float4 *__restrict__ obs,
                                           float4 *__restrict__ rew, float4 *__restrict__ done,
                                           int64_t A, int k, int64_t c0) {
    const int tid = threadIdx.x;
    const float4 *a = act + ((int64_t)k * A * 8 + c0 * 8) / 16;
    float4 a0, a1;
    if (act_stride0 == 1) {  // NOACT: no action reads (a write-only mix), values from the indices
        a0 = make_float4((float)tid, (float)k, 1.f, 2.f);
        a1 = make_float4((float)c0, 0.5f, 3.f, (float)tid);
    } else if (act_stride0 == 2) {  // NTLOAD: non-temporal action loads
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 *av = reinterpret_cast<const f4 *>(a);
        const f4 x0 = __builtin_nontemporal_load(av + tid), x1 = __builtin_nontemporal_load(av + tid + 256);
        a0 = make_float4(x0.x, x0.y, x0.z, x0.w);
        a1 = make_float4(x1.x, x1.y, x1.z, x1.w);
    } else {
        a0 = a[tid];
        a1 = a[tid + 256];
    }
    const float s = a0.x + a1.w;
    float4 *o = obs + ((int64_t)k * A * 32 + c0 * 32) / 16;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        st<NT>(o + tid + 256 * j, make_float4(s, (j & 1 ? a1 : a0).y, (j & 1 ? a1 : a0).z, 1.f));
    st<NT>(rew + ((int64_t)k * A * 4 + c0 * 4) / 16 + tid, make_float4(s, s, s, s));
    if (tid < CH / 16) st<NT>(done + ((int64_t)k * A + c0) / 16 + tid, make_float4(s, 0.f, s, 0.f));
}

template <bool NT>
__global__ __launch_bounds__(256) void k_slice(const float4 *act, float4 *obs, float4 *rew,
                                               float4 *done, int64_t A, int T, int64_t b0 = 0) {
    const int64_t c0 = ((int64_t)blockIdx.x + b0) * CH;
    for (int k = 0; k < T; ++k) chunk_step<NT>(act, obs, rew, done, A, k, c0);
}

template <bool NT>
__global__ __launch_bounds__(256) void k_plane(const float4 *act, float4 *obs, float4 *rew,
                                               float4 *done, int64_t A, int T, int64_t nchunk) {
    const int64_t per = (nchunk + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per;
    const int64_t b1 = std::min<int64_t>(b0 + per, nchunk);
    for (int k = 0; k < T; ++k)
        for (int64_t c = b0; c < b1; ++c) chunk_step<NT>(act, obs, rew, done, A, k, c * CH);
}

int main(int argc, char **argv) {
    const int64_t A = argc > 1 ? std::atoll(argv[1]) : 5242880;
    const int T = argc > 2 ? std::atoi(argv[2]) : 10;
    if (A % CH) return 2;
    const int64_t nchunk = A / CH;
    float4 *act, *obs, *rew, *done;
    // ALLOC=contig: hipExtMallocWithFlags(hipDeviceMallocContiguous) (physically contiguous, so
    // the page tables can use large fragments); ALLOC=one: the four streams carved from one
    // hipMalloc; default: one hipMalloc each
    const char *al = std::getenv("ALLOC");
    const std::string mode = al ? al : "";
    auto alloc = [&](float4 **p, size_t b) {
        if (mode == "contig")
            return hipExtMallocWithFlags(reinterpret_cast<void **>(p), b,
                                         hipDeviceMallocContiguous);
        return hipMalloc(p, b);
    };
    if (mode == "one") {
        char *base = nullptr;
        const size_t b0 = (size_t)T * A * 8, b1 = (size_t)T * A * 32, b2 = (size_t)T * A * 4;
        if (hipMalloc(&base, b0 + b1 + b2 + (size_t)T * A) != hipSuccess) return 3;
        act = reinterpret_cast<float4 *>(base);
        obs = reinterpret_cast<float4 *>(base + b0);
        rew = reinterpret_cast<float4 *>(base + b0 + b1);
        done = reinterpret_cast<float4 *>(base + b0 + b1 + b2);
    } else if (alloc(&act, (size_t)T * A * 8) != hipSuccess ||
               alloc(&obs, (size_t)T * A * 32) != hipSuccess ||
               alloc(&rew, (size_t)T * A * 4) != hipSuccess ||
               alloc(&done, (size_t)T * A) != hipSuccess)
        return 3;
    (void)hipMemset(act, 0, (size_t)T * A * 8);
    const int noact = std::getenv("NOACT") ? 1 : (std::getenv("NTLOAD") ? 2 : 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(act_stride0), &noact, sizeof(int)) != hipSuccess) return 5;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double bytes = 45.0 * (double)A * T;
    struct V {
        const char *name;
        int grid;  // 0: slice-major (A / CH blocks)
        bool nt;
    };
    std::vector<V> vs;
    const bool split_only = std::getenv("SPLIT_ONLY") != nullptr;
    for (bool nt : {false, true}) {
        vs.push_back({"slice", 0, nt});
        if (!split_only)
            for (int g : {256, 512, 768, 1024, 1536, 2048}) vs.push_back({"plane", g, nt});
        // slice order in S back-to-back launches over consecutive chunk ranges (grid = -S)
        for (int S : {2, 4, 8}) vs.push_back({"slice_split", -S, nt});
    }
    for (int round = 0; round < 2; ++round)
        for (const V &v : vs) {
            auto launch = [&] {
                if (v.grid < 0) {
                    const int S = -v.grid;
                    const int64_t per = nchunk / S;
                    for (int k = 0; k < S; ++k) {
                        const int64_t b0 = k * per, nb = k + 1 < S ? per : nchunk - b0;
                        if (v.nt)
                            hipLaunchKernelGGL(k_slice<true>, dim3((unsigned)nb), dim3(256), 0, 0,
                                               act, obs, rew, done, A, T, b0);
                        else
                            hipLaunchKernelGGL(k_slice<false>, dim3((unsigned)nb), dim3(256), 0,
                                               0, act, obs, rew, done, A, T, b0);
                    }
                } else if (v.grid == 0) {
                    if (v.nt)
                        hipLaunchKernelGGL(k_slice<true>, dim3((unsigned)nchunk), dim3(256), 0, 0,
                                           act, obs, rew, done, A, T);
                    else
                        hipLaunchKernelGGL(k_slice<false>, dim3((unsigned)nchunk), dim3(256), 0, 0,
                                           act, obs, rew, done, A, T);
                } else {
                    if (v.nt)
                        hipLaunchKernelGGL(k_plane<true>, dim3(v.grid), dim3(256), 0, 0, act, obs,
                                           rew, done, A, T, nchunk);
                    else
                        hipLaunchKernelGGL(k_plane<false>, dim3(v.grid), dim3(256), 0, 0, act,
                                           obs, rew, done, A, T, nchunk);
                }
            };
            for (int w = 0; w < 3; ++w) launch();
            std::vector<float> ms;
            for (int r = 0; r < 10; ++r) {
                (void)hipEventRecord(e0, 0);
                launch();
                (void)hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) return 4;
                float m = 0.f;
                (void)hipEventElapsedTime(&m, e0, e1);
                ms.push_back(m);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            std::printf("{\"round\": %d, \"order\": \"%s\", \"grid\": %d, \"nt\": %d, \"A\": %lld, "
                        "\"T\": %d, \"ms\": %.4f, \"tb_s\": %.3f}\n",
                        round, v.name, v.grid > 0 ? v.grid : (v.grid < 0 ? v.grid : (int)nchunk),
                        v.nt ? 1 : 0, (long long)A,
                        T, med, bytes / (med * 1e-3) / 1e12);
            std::fflush(stdout);
        }
    return 0;
}
