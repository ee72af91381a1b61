// Host write bandwidth into the three kinds of host memory a staging buffer can be: plain
// malloc, malloc + hipHostRegister, and hipHostMalloc(Mapped | Coherent | Portable) (the MT19937
// staging pool until round 5).  One thread writes 75 MB (a config-3 draw set with its tags) as
// floats, best of 5.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pinned_write_probe tools/pinned_write_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double fill_ms(float *p, size_t n) {
    double best = 1e30;
    for (int r = 0; r < 5; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < n; ++i) p[i] = (float)(i & 1023) * 0.5f;
        auto t1 = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    const size_t n = (size_t)75 << 18;  // 75 MB of floats
    const size_t bytes = n * sizeof(float);
    float *a = static_cast<float *>(std::aligned_alloc(4096, bytes));
    std::memset(a, 0, bytes);
    std::printf("{\"plain_ms\": %.2f", fill_ms(a, n));
    float *b = static_cast<float *>(std::aligned_alloc(4096, bytes));
    std::memset(b, 0, bytes);
    if (hipHostRegister(b, bytes, hipHostRegisterDefault) != hipSuccess) return 2;
    std::printf(", \"registered_ms\": %.2f", fill_ms(b, n));
    void *c = nullptr;
    if (hipHostMalloc(&c, bytes, hipHostMallocMapped | hipHostMallocCoherent |
                                     hipHostMallocPortable) != hipSuccess)
        return 3;
    std::printf(", \"hostmalloc_coherent_ms\": %.2f", fill_ms(static_cast<float *>(c), n));
    void *d = nullptr;
    if (hipHostMalloc(&d, bytes, hipHostMallocDefault) != hipSuccess) return 4;
    std::printf(", \"hostmalloc_default_ms\": %.2f", fill_ms(static_cast<float *>(d), n));
    void *e = nullptr;
    if (hipHostMalloc(&e, bytes, hipHostMallocMapped | hipHostMallocNonCoherent |
                                     hipHostMallocPortable) != hipSuccess)
        return 5;
    std::printf(", \"hostmalloc_noncoherent_ms\": %.2f, \"MB\": %.1f}\n",
                fill_ms(static_cast<float *>(e), n), bytes / 1e6);
    (void)hipHostUnregister(b);
    (void)hipHostFree(c);
    (void)hipHostFree(d);
    (void)hipHostFree(e);
    std::free(a);
    std::free(b);
    return 0;
}
