// Same-box HBM ceiling of the env rollout's byte mix, measured inside bench.py next to the
// kernel it calibrates (measurement support, not product: bench.py loads it with ctypes when
// built; __graft_entry__.build() builds it into tools/calib/libhbm_ceiling.so).
//
// k_mix streams exactly the bytes of one fenv_rollout launch -- actions [T][A][2] f32 read,
// obs [T][A][8] f32, reward [T][A] f32 and done [T][A] u8 written, 45 B per agent-step -- into
// the caller's own rollout buffers, with no arithmetic and every access a whole, 128-B-aligned
// float4 run (a workgroup owns a chunk of CH agents for all T steps, like the env kernel's
// agents-per-lane mapping).  Its rate is what this box's HBM delivers for this read/write mix
// (tools/ubench_ceiling.hip: CH = 1,024 is the best of 512 ... 4,096 and of persistent
// variants); the writes are timed both plain and non-temporal and the faster counts (the env
// kernels store non-temporally on large launches).  The fraction kernel / ceiling says how much
// of the reachable bandwidth the env kernel leaves on the table.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int CH = 1024;

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

template <bool NT>
__global__ __launch_bounds__(256) void k_mix(const float4 *__restrict__ act,
                                             float4 *__restrict__ obs, float4 *__restrict__ rew,
                                             float4 *__restrict__ done, int64_t A, int T) {
    constexpr int NA = CH * 8 / 16, NO = CH * 32 / 16, NR = CH * 4 / 16, ND = CH / 16;
    constexpr int PA = (NA + 255) / 256;
    const int64_t c0 = (int64_t)blockIdx.x * CH;
    const int tid = threadIdx.x;
    float4 a[PA];
#pragma unroll
    for (int j = 0; j < PA; ++j) a[j] = act[(c0 * 8) / 16 + tid + 256 * j];
    for (int k = 0; k < T; ++k) {
        float4 cur[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) cur[j] = a[j];
        if (k + 1 < T) {
#pragma unroll
            for (int j = 0; j < PA; ++j)
                a[j] = act[((int64_t)(k + 1) * A * 8 + c0 * 8) / 16 + tid + 256 * j];
        }
        const float s = cur[0].x + cur[PA - 1].w;
        float4 *o = obs + ((int64_t)k * A * 32 + c0 * 32) / 16;
#pragma unroll
        for (int j = 0; j < NO / 256; ++j)
            st<NT>(o + tid + 256 * j, make_float4(s, cur[j % PA].y, cur[j % PA].z, 1.f));
        float4 *r = rew + ((int64_t)k * A * 4 + c0 * 4) / 16;
        st<NT>(r + tid, make_float4(s, s, s, s));
        float4 *d = done + ((int64_t)k * A + c0) / 16;
        if (tid < ND) st<NT>(d + tid, make_float4(s, 0.f, s, 0.f));
    }
    static_assert(NR == 256 && NA == 512, "one reward float4 per thread, 2 action float4s");
}

}  // namespace

extern "C" {

// Chunk size the buffers must be a multiple of (agents).
int hbm_ceiling_chunk(void) { return CH; }

// Average ms per launch of `reps` back-to-back k_mix launches over A agents x T steps on
// `stream` (HIP events on that stream; 3 untimed launches first), the faster of the plain and
// the non-temporal store variant.  A must be a positive multiple
// of hbm_ceiling_chunk() and the buffers 16-B aligned and at least T*A*{8, 32, 4, 1} bytes.
// Returns a negative value on error.
double hbm_ceiling_mix_ms(const void *act, void *obs, void *rew, void *done, int64_t A,
                          int32_t T, int32_t reps, void *stream) {
    if (A <= 0 || A % CH != 0 || T < 1 || reps < 1) return -1.0;
    for (const void *p : {act, (const void *)obs, (const void *)rew, (const void *)done})
        if (p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) != 0) return -2.0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)(A / CH)), block(256);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return -3.0;
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return -3.0;
    }
    double best = -4.0;
    for (int nt = 0; nt < 2; ++nt) {
        auto launch = [&] {
            if (nt)
                hipLaunchKernelGGL(k_mix<true>, grid, block, 0, st,
                                   reinterpret_cast<const float4 *>(act),
                                   reinterpret_cast<float4 *>(obs), reinterpret_cast<float4 *>(rew),
                                   reinterpret_cast<float4 *>(done), A, T);
            else
                hipLaunchKernelGGL(k_mix<false>, grid, block, 0, st,
                                   reinterpret_cast<const float4 *>(act),
                                   reinterpret_cast<float4 *>(obs), reinterpret_cast<float4 *>(rew),
                                   reinterpret_cast<float4 *>(done), A, T);
        };
        for (int w = 0; w < 3; ++w) launch();
        (void)hipEventRecord(e0, st);
        for (int r = 0; r < reps; ++r) launch();
        (void)hipEventRecord(e1, st);
        float ms = -4.0f;
        if (hipGetLastError() == hipSuccess && hipEventSynchronize(e1) == hipSuccess)
            (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms > 0.0f && (best < 0.0 || (double)ms / reps < best)) best = (double)ms / reps;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

}  // extern "C"
