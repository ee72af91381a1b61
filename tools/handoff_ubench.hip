// cost the PPO update's cross-CU norm exchange before changing it.
// The exact exchange pattern of k_ppo_update's split launch (csrc/ppo_update.hip, the norm
// phase): a cooperative 9-block grid of 256 threads, blocks 0 and 8 active; per iteration thread
// 0 of each posts {seq, value} with a relaxed agent-scope 64-bit store into its word of the
// iteration's parity, loads the partner's word, spins (s_sleep 1 between loads, as shipped, or
// none) until the sequence matches, then the block barriers.  Optionally W cycles of
// s_sleep-free VALU work per iteration on each block, with a skew of S extra cycles on block 0
// (the actor is the late block).  Reports ns per iteration; the exchange's cost is the period
// minus the work alone (same kernel, exchange off).
//   hipcc --offload-arch=gfx950 -O3 -o tools/handoff_ubench tools/handoff_ubench.hip
//   tools/handoff_ubench                 (prints one JSON line per configuration)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

struct Args {
    uint64_t *xch;
    float *out;
    int iters;
    int work;     // busy cycles per iteration (both blocks)
    int skew;     // extra busy cycles on block 0
    int sleep;    // 1: s_sleep(1) between polls (shipped); 0: tight poll
    int exchange; // 0: work alone (no post, no wait)
};

__device__ __forceinline__ float busy(int cycles, float x) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) x = x * 1.0000001f + 1e-7f;
    return x;
}

__global__ void __launch_bounds__(256) k_handoff(Args a) {
    const int b = blockIdx.x;
    if (b != 0 && b != 8) return;
    const int net = b == 0 ? 0 : 1;
    float x = (float)threadIdx.x;
    __shared__ float sh;
    for (int k = 0; k < a.iters; ++k) {
        x = busy(a.work + (net == 0 ? a.skew : 0), x);
        if (a.exchange && threadIdx.x == 0) {
            const uint64_t seq = (uint64_t)(k + 1);
            __hip_atomic_store(a.xch + 2 * net + (k & 1), (seq << 32) | __float_as_uint(x),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint64_t o = __hip_atomic_load(a.xch + 2 * (net ^ 1) + (k & 1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            for (int spin = 0; spin < (1 << 22) && (o >> 32) != seq; ++spin) {
                if (a.sleep) __builtin_amdgcn_s_sleep(1);
                o = __hip_atomic_load(a.xch + 2 * (net ^ 1) + (k & 1), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
            }
            sh = __uint_as_float((uint32_t)o);
        }
        __syncthreads();
        x += sh * 0.0f;
    }
    a.out[b * 256 + threadIdx.x] = x;
}

int main() {
    uint64_t *xch;
    float *out;
    if (hipMalloc(&xch, 4 * sizeof(uint64_t)) != hipSuccess) return 2;
    if (hipMalloc(&out, 9 * 256 * sizeof(float)) != hipSuccess) return 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 20000;
    // work 0: the bare exchange; 18k cycles ~ one minibatch's per-block work
    const int works[] = {0, 18000};
    const int skews[] = {0, 700};
    for (int w : works)
        for (int sk : skews)
            for (int sl = 1; sl >= 0; --sl)
                for (int ex = 1; ex >= 0; --ex) {
                    if (!ex && sl == 0) continue;  // work alone: one measurement per (w, skew)
                    Args a{xch, out, iters, w, sk, sl, ex};
                    double best = 1e30;
                    for (int rep = 0; rep < 3; ++rep) {
                        (void)hipMemset(xch, 0, 4 * sizeof(uint64_t));
                        void *args[] = {&a};
                        (void)hipEventRecord(e0, nullptr);
                        hipError_t e = hipLaunchCooperativeKernel(
                            reinterpret_cast<const void *>(&k_handoff), dim3(9), dim3(256), args,
                            0, nullptr);
                        (void)hipEventRecord(e1, nullptr);
                        if (e != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
                            std::printf("launch failed\n");
                            return 3;
                        }
                        float ms = 0.f;
                        (void)hipEventElapsedTime(&ms, e0, e1);
                        best = ms < best ? ms : best;
                    }
                    std::printf("{\"work_cycles\": %d, \"skew_cycles\": %d, \"sleep\": %d, "
                                "\"exchange\": %d, \"ns_per_iter\": %.1f}\n",
                                w, sk, sl, ex, best * 1e6 / iters);
                    std::fflush(stdout);
                }
    (void)hipFree(xch);
    (void)hipFree(out);
    return 0;
}
