// Which access shapes reach the most HBM bandwidth on this box (gfx950)?  The rollout kernel
// runs at 1.00 of the same-box ceiling that tools/ubench_ceiling.hip measures (5.0-5.7 TB/s of
// streaming writes, 4.6-4.8 TB/s float4 copy), while MI355X_MICROARCH.md quotes 6.29 TB/s for a
// float4 copy and 6.0-6.2 TB/s for dword stores into random 2,304-B rows.  This sweeps the
// shapes that differ between the two: block-contiguous chunks with U accesses in flight per
// thread, chunk order (linear vs a bijective scatter of the chunk index), workgroup size, and
// the guide's random-row dword stores.  4 GiB buffers (far past the 256 MiB Infinity Cache).
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_bw ubench_bw.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float v4 __attribute__((ext_vector_type(4)));

// chunk index of block b: linear, or a bijective scatter over a power-of-two chunk count
__device__ __forceinline__ size_t chunk_of(size_t b, size_t nch, int scatter) {
    if (scatter == 0) return b;
    if (scatter == 1) return (b * 0x9E3779B1ull) & (nch - 1);          // odd multiplier mod 2^k
    // scatter == 2: XCD-major: blocks b, b+8, ... (one XCD) take one contiguous run of chunks
    const size_t per = nch / 8;
    return (b & 7) * per + (b >> 3);
}

template <int U, int BS>
__global__ __launch_bounds__(BS) void k_copy(const v4 *__restrict__ in, v4 *__restrict__ out, size_t nch, int scatter) {
    const size_t c = chunk_of(blockIdx.x, nch, scatter);
    const size_t base = c * (size_t)(BS * U) + threadIdx.x;
    v4 r[U];
#pragma unroll
    for (int j = 0; j < U; ++j) r[j] = in[base + (size_t)j * BS];
#pragma unroll
    for (int j = 0; j < U; ++j) out[base + (size_t)j * BS] = r[j];
}
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_read(const v4 *__restrict__ in, v4 *__restrict__ out, size_t nch, int scatter) {
    const size_t c = chunk_of(blockIdx.x, nch, scatter);
    const size_t base = c * (size_t)(BS * U) + threadIdx.x;
    v4 s = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < U; ++j) s += in[base + (size_t)j * BS];
    if (s.x == 1234.5f && s.y == -1.f) out[threadIdx.x] = s;  // never true on the zeroed input
}
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_write(v4 *__restrict__ out, size_t nch, int scatter) {
    const size_t c = chunk_of(blockIdx.x, nch, scatter);
    const size_t base = c * (size_t)(BS * U) + threadIdx.x;
#pragma unroll
    for (int j = 0; j < U; ++j) out[base + (size_t)j * BS] = (v4){(float)j, 1.f, 2.f, (float)c};
}
// the guide's shape: one wave per 2,304-B row (9 dword stores of 256 B), rows in random order
__global__ __launch_bounds__(256) void k_rows(float *__restrict__ out, const unsigned *__restrict__ rows,
                                              unsigned nrows) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nrows) return;
    float *p = out + (size_t)rows[w] * 576;
#pragma unroll
    for (int j = 0; j < 9; ++j) p[j * 64 + lane] = (float)(j + lane);
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
    printf("%-40s  best %.3f ms %7.1f GB/s   median %.3f ms %7.1f GB/s\n", name, t[0], bytes / t[0] / 1e6,
           t[reps / 2], bytes / t[reps / 2] / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main() {
    const size_t bytes = (size_t)4 << 30, n = bytes / 16;
    v4 *x, *y; CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
    char nm[96];
#define SWEEP(U, BS) for (int sc = 0; sc < 3; ++sc) { const size_t nch = n / ((size_t)(BS) * (U)); \
        snprintf(nm, sizeof nm, "copy  U=%d BS=%d scatter=%d", U, BS, sc); \
        timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<U, BS>), dim3(nch), dim3(BS), 0, 0, x, y, nch, sc); }); \
        snprintf(nm, sizeof nm, "read  U=%d BS=%d scatter=%d", U, BS, sc); \
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_read<U, BS>), dim3(nch), dim3(BS), 0, 0, x, y, nch, sc); }); \
        snprintf(nm, sizeof nm, "write U=%d BS=%d scatter=%d", U, BS, sc); \
        timeit(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((k_write<U, BS>), dim3(nch), dim3(BS), 0, 0, y, nch, sc); }); }
    SWEEP(1, 256) SWEEP(4, 256) SWEEP(8, 256) SWEEP(4, 512) SWEEP(4, 1024) SWEEP(16, 256)
    // guide's random-row dword stores, and the same rows in order
    const unsigned nrows = (unsigned)(bytes / 2304);
    std::vector<unsigned> h(nrows);
    for (unsigned i = 0; i < nrows; ++i) h[i] = i;
    unsigned *rows; CK(hipMalloc(&rows, (size_t)nrows * 4));
    CK(hipMemcpy(rows, h.data(), (size_t)nrows * 4, hipMemcpyHostToDevice));
    timeit("rows 2304B dword, in order", 2304.0 * nrows,
           [&] { hipLaunchKernelGGL(k_rows, dim3((nrows + 3) / 4), dim3(256), 0, 0, (float *)y, rows, nrows); });
    srand(1);
    for (unsigned i = nrows - 1; i > 0; --i) std::swap(h[i], h[(unsigned)(((size_t)rand() * RAND_MAX + rand()) % (i + 1))]);
    CK(hipMemcpy(rows, h.data(), (size_t)nrows * 4, hipMemcpyHostToDevice));
    timeit("rows 2304B dword, random order", 2304.0 * nrows,
           [&] { hipLaunchKernelGGL(k_rows, dim3((nrows + 3) / 4), dim3(256), 0, 0, (float *)y, rows, nrows); });
    CK(hipFree(rows)); CK(hipFree(x)); CK(hipFree(y));
    return 0;
}
