// Probe for VERDICT r3 weak #1 (wrong post-reset rewards after an MT19937 reset, staged set read
// stale?).  Replays the staging protocol of fenv_api.cpp gen_pending in isolation: two slots, the
// host rewrites a pinned (mapped, coherent) host slot, a copy kernel on the launch stream moves it
// to HBM, a consumer kernel reads it the way draw_reset does; every word is checked on the host.
//
// Variants of the copy's host-memory loads:
//   plain  : k_stage_copy as shipped in round 3 (plain global loads of the mapped host pointer)
//   sys    : system-scope relaxed atomic loads (global_load ... sc0 sc1: bypass the GPU caches)
//   dma    : hipMemcpyAsync H2D from the same pinned buffer (no kernel reads host memory)
// A word is "stale" when the consumer sees the value the slot held two refills ago.
//
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/host_stage_probe tools/host_stage_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,               \
                         hipGetErrorString(e_));                                         \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void k_copy_plain(float *__restrict__ dst,
                                                    const float *__restrict__ src, int64_t n) {
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        d4[i] = s4[i];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n - 4 * n4) dst[4 * n4 + t] = src[4 * n4 + t];
}

__global__ __launch_bounds__(256) void k_copy_sys(float *__restrict__ dst, const float *src,
                                                  int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        d[i] = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// consumer: reads the slot like draw_reset (one lane per word) into out
__global__ __launch_bounds__(256) void k_consume(const float *__restrict__ slot, float *out,
                                                 int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = slot[i];
}

// unrelated traffic between refills (what the test suite's other kernels do to the caches)
__global__ __launch_bounds__(256) void k_noise(float *buf, int64_t n, float v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        buf[i] = buf[i] * 0.5f + v;
}

static inline float tagval(int trial, int64_t i) {
    // exact in fp32: trial in the high bits, index in the low ones
    uint32_t u = 0x3F800000u ^ (((uint32_t)trial & 0xFFFu) << 11) ^ (uint32_t)(i & 0x7FF);
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 6000;  // pend_floats at F=500, N=5
    const int trials = argc > 2 ? std::atoi(argv[2]) : 2000;
    const char *variants[] = {"plain", "sys", "dma"};
    const size_t stride = (size_t)((n + 63) & ~63);
    float *hbuf = nullptr, *hdev = nullptr, *dslot = nullptr, *dout = nullptr, *noise = nullptr;
    CK(hipHostMalloc((void **)&hbuf, 2 * stride * 4,
                     hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    CK(hipHostGetDevicePointer((void **)&hdev, hbuf, 0));
    CK(hipMalloc(&dslot, 2 * stride * 4));
    CK(hipMalloc(&dout, stride * 4));
    const int64_t nn = 1 << 22;
    CK(hipMalloc(&noise, nn * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t ev[2];
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::vector<float> out(n);
    const unsigned cblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (n / 4 + 255) / 256));
    for (int v = 0; v < 3; ++v) {
        long long stale = 0, other = 0, bad_trials = 0;
        int first_bad = -1;
        bool recorded[2] = {false, false};
        for (int tr = 0; tr < trials; ++tr) {
            const int s = tr & 1;
            if (recorded[s]) CK(hipEventSynchronize(ev[s]));  // host slot free (as gen_pending)
            float *hs = hbuf + s * stride;
            for (int64_t i = 0; i < n; ++i) hs[i] = tagval(tr, i);
            float *ds = dslot + s * stride;
            if (v == 0)
                hipLaunchKernelGGL(k_copy_plain, dim3(cblocks), dim3(256), 0, st, ds, hdev + s * stride, n);
            else if (v == 1)
                hipLaunchKernelGGL(k_copy_sys, dim3(cblocks), dim3(256), 0, st, ds, hdev + s * stride, n);
            else
                CK(hipMemcpyAsync(ds, hs, n * 4, hipMemcpyHostToDevice, st));
            CK(hipGetLastError());
            CK(hipEventRecord(ev[s], st));
            recorded[s] = true;
            if (tr % 3 == 1)
                hipLaunchKernelGGL(k_noise, dim3(256), dim3(256), 0, st, noise, (tr % 6 == 1) ? nn : 4096, 1.0f);
            hipLaunchKernelGGL(k_consume, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ds, dout, n);
            CK(hipMemcpyAsync(out.data(), dout, n * 4, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            long long bad = 0;
            for (int64_t i = 0; i < n; ++i) {
                if (std::memcmp(&out[i], &hs[i], 4) == 0) continue;
                ++bad;
                float old = tagval(tr - 2, i);
                if (tr >= 2 && std::memcmp(&out[i], &old, 4) == 0) ++stale;
                else ++other;
            }
            if (bad) {
                ++bad_trials;
                if (first_bad < 0) first_bad = tr;
            }
        }
        std::printf("{\"variant\": \"%s\", \"n\": %lld, \"trials\": %d, \"bad_trials\": %lld, "
                    "\"stale_words\": %lld, \"other_wrong_words\": %lld, \"first_bad_trial\": %d}\n",
                    variants[v], (long long)n, trials, bad_trials, stale, other, first_bad);
        std::fflush(stdout);
    }
    return 0;
}
