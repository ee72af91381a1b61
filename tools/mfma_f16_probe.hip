// Probe for the split-f16 policy MFMA (csrc/policy_device.h): checks on the real gfx950
//  (1) the A/B operand lane map of v_mfma_f32_32x32x16_f16 (A[r][8h+j], B[8h+j][r]) and the
//      C/D map rows rho(reg, h), with exact integer data and an asymmetric B;
//  (2) whether f16 SUBNORMAL A/B inputs are honoured or flushed (the lo halves of the split
//      operands are subnormal for |x| < ~0.1, so a flush would break the fp32-grade accuracy);
//  (3) that the products are exact and accumulate in fp32 (2^-11 * 2^-11 terms survive);
//  (4) whether a dependent MFMA chain rounds the same when issued back to back (accumulator
//      forwarded) as when the producer has retired (accumulator read from the register file).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/mfma_f16_probe tools/mfma_f16_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k_mma(const _Float16 *A, const _Float16 *B, float *C) {
    // A [32][16] row-major, B [16][32] row-major, C [32][32] row-major
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    h8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[r * 16 + 8 * h + j];
        b[j] = B[(8 * h + j) * 32 + r];
    }
    f16v c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        C[row * 32 + r] = c[reg];
    }
}

// (4): C <- A1 B1 + C, C <- A2 B2 + C, back to back (GAP = 0) or with the first retired (GAP = 1)
template <int GAP>
__global__ void k_chain(const h8 *A1, const h8 *B1, const h8 *A2, const h8 *B2, const f16v *C0,
                        f16v *C) {
    const int l = threadIdx.x + 64 * blockIdx.x;
    f16v c = C0[l];
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1[l], B1[l], c, 0, 0, 0);
    if (GAP) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
        c = c + 0.0f;  // a VALU read of the whole accumulator: the producer has retired
        __builtin_amdgcn_sched_barrier(0);
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2[l], B2[l], c, 0, 0, 0);
    C[l] = c;
}

static int run(const std::vector<float> &A, const std::vector<float> &B, std::vector<float> &C) {
    std::vector<_Float16> Ah(A.size()), Bh(B.size());
    for (size_t i = 0; i < A.size(); ++i) Ah[i] = (_Float16)A[i];
    for (size_t i = 0; i < B.size(); ++i) Bh[i] = (_Float16)B[i];
    _Float16 *dA, *dB;
    float *dC;
    if (hipMalloc(&dA, Ah.size() * 2) || hipMalloc(&dB, Bh.size() * 2) || hipMalloc(&dC, 32 * 32 * 4))
        return 1;
    hipMemcpy(dA, Ah.data(), Ah.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, Bh.data(), Bh.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mma, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    C.resize(32 * 32);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    hipFree(dA);
    hipFree(dB);
    hipFree(dC);
    return hipGetLastError() != hipSuccess;
}

int main() {
    int fails = 0;
    std::vector<float> A(32 * 16), B(16 * 32), C;
    // (1) layout, exact integers, asymmetric B
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 16; ++k) A[i * 16 + k] = (float)((i * 3 + k * 7) % 11 - 5);
    for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 32; ++j) B[k * 32 + j] = (float)((k * 5 + j * 2 + k * j) % 13 - 6);
    if (run(A, B, C)) return 2;
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            float s = 0;
            for (int k = 0; k < 16; ++k) s += A[i * 16 + k] * B[k * 32 + j];
            bad += C[i * 32 + j] != s;
        }
    printf("layout A[r][8h+j] B[8h+j][r] C rho(reg,h): %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    fails += bad != 0;
    // (2) subnormal f16 inputs: 2^-20 (f16 min normal is 2^-14)
    for (auto &v : A) v = std::ldexp(1.0f, -20);
    for (auto &v : B) v = 1.0f;
    run(A, B, C);
    printf("subnormal A (2^-20) x 1, K=16: C = %g (honoured: %g, flushed: 0) -> %s\n", C[0],
           std::ldexp(16.0, -20), C[0] == std::ldexp(16.0f, -20) ? "honoured" : "FLUSHED/other");
    fails += C[0] != std::ldexp(16.0f, -20);
    for (auto &v : A) v = 1.0f;
    for (auto &v : B) v = std::ldexp(1.0f, -24);
    run(A, B, C);
    printf("subnormal B (2^-24) x 1, K=16: C = %g (honoured: %g) -> %s\n", C[0],
           std::ldexp(16.0, -24), C[0] == std::ldexp(16.0f, -24) ? "honoured" : "FLUSHED/other");
    fails += C[0] != std::ldexp(16.0f, -24);
    // (3) exact products + fp32 accumulation: 1 + 2^-11 * 2^-11 (needs > f16 accumulators)
    for (auto &v : A) v = 0.0f;
    for (auto &v : B) v = 0.0f;
    A[0] = 1.0f;  B[0] = 1.0f;
    A[1] = std::ldexp(1.0f, -11) * 3;  B[32] = std::ldexp(1.0f, -11) * 5;
    run(A, B, C);
    const float want = 1.0f + 15.0f * std::ldexp(1.0f, -22);
    printf("1 + (3*2^-11)(5*2^-11) = %.9g (want %.9g) -> %s\n", C[0], want, C[0] == want ? "ok" : "FAIL");
    fails += C[0] != want;
    // (4) chain rounding, random operands (1024 waves)
    {
        const int W = 1024, L = 64 * W;
        std::vector<_Float16> a(4 * (size_t)L * 8);
        std::vector<float> c0((size_t)L * 16);
        uint32_t x = 12345;
        auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (x >> 8) * 0x1.0p-24f * 2.0f - 1.0f; };
        for (auto &v : a) v = (_Float16)rnd();
        for (auto &v : c0) v = rnd() * 4.0f;
        _Float16 *dA;
        float *dC0, *dC[2];
        hipMalloc(&dA, a.size() * 2);
        hipMalloc(&dC0, c0.size() * 4);
        hipMalloc(&dC[0], c0.size() * 4);
        hipMalloc(&dC[1], c0.size() * 4);
        hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dC0, c0.data(), c0.size() * 4, hipMemcpyHostToDevice);
        const h8 *p = reinterpret_cast<const h8 *>(dA);
        hipLaunchKernelGGL(k_chain<0>, dim3(W), dim3(64), 0, 0, p, p + L, p + 2 * L, p + 3 * L,
                           reinterpret_cast<const f16v *>(dC0), reinterpret_cast<f16v *>(dC[0]));
        hipLaunchKernelGGL(k_chain<1>, dim3(W), dim3(64), 0, 0, p, p + L, p + 2 * L, p + 3 * L,
                           reinterpret_cast<const f16v *>(dC0), reinterpret_cast<f16v *>(dC[1]));
        std::vector<float> r0(c0.size()), r1(c0.size());
        hipMemcpy(r0.data(), dC[0], r0.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(r1.data(), dC[1], r1.size() * 4, hipMemcpyDeviceToHost);
        size_t diff = 0;
        for (size_t i = 0; i < r0.size(); ++i) diff += r0[i] != r1[i];
        printf("chain back-to-back vs retired: %zu of %zu results differ -> %s\n", diff, r0.size(),
               diff ? "forwarding CHANGES rounding" : "identical");
    }
    printf("%s\n", fails ? "PROBE FAILED" : "PROBE OK");
    return fails ? 1 : 0;
}
