// Issue cost per wave64 instruction on gfx950 for the ops the policy rollout's sampling uses
// (Philox: v_mul_lo_u32 / v_mul_hi_u32), against v_add_u32, v_mul_u32_u24, v_fma_f32, v_exp_f32.
// One wave per SIMD (grid = 1024 x 64 threads), 8 independent chains per lane, s_memtime around
// a fixed count of instructions: cycles per instruction = elapsed / count.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIt = 256;

template <int OP>
__global__ __launch_bounds__(64) void k_rate(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t v[8];
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] = seed + threadIdx.x * 8 + j;
        f[j] = (float)v[j] * 1e-9f;
    }
    const uint32_t c = 0xD2511F53u ^ seed;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIt; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
            if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
            if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[j]) : "s"(c));
            if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[j]) : "s"(c));
            if (OP == 4) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(f[j]));
            if (OP == 5) asm volatile("v_exp_f32 %0, %0" : "+v"(f[j]));
            if (OP == 6) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(*(uint64_t *)&v[(j & 3) * 2]) : "v"(v[j]), "s"(c) : "vcc");
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j] ^ __float_as_uint(f[j]);
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int blocks = 1024;
    uint32_t *out; uint64_t *cyc;
    CK(hipMalloc(&out, blocks * 64 * 4)); CK(hipMalloc(&cyc, blocks * 8));
    uint64_t *h = (uint64_t *)malloc(blocks * 8);
    const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_fma_f32", "v_exp_f32", "v_mad_u64_u32"};
    for (int rep = 0; rep < 2; ++rep)
        for (int op = 0; op < 7; ++op) {
            switch (op) {
                case 0: hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 1: hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 2: hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 3: hipLaunchKernelGGL(k_rate<3>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 4: hipLaunchKernelGGL(k_rate<4>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 5: hipLaunchKernelGGL(k_rate<5>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
                case 6: hipLaunchKernelGGL(k_rate<6>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1u); break;
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost));
            double s = 0;
            for (int b = 0; b < blocks; ++b) s += (double)h[b];
            // s_memtime: the shader clock counter (v_add_u32 reads ~4 per instruction)
            const double ticks = s / blocks / (kIt * 8.0);
            if (rep) printf("%-14s %.2f s_memtime cycles per instruction\n", names[op], ticks);
        }
    return 0;
}
