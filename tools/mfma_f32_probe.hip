// Hardware check of the fp32 MFMA operand/result maps the fused PPO update assumes:
//   v_mfma_f32_32x32x2f32: A[i][k] in lane i + 32k, B[k][j] in lane j + 32k,
//                          D[i][j] in reg (i&3) + 4(i>>3), lane j + 32((i>>2)&1)
//   v_mfma_f32_16x16x4f32: A[i][k] in lane i + 16k, B[k][j] in lane j + 16k,
//                          D[i][j] in reg i&3, lane j + 16(i>>2)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/mfma_f32_probe tools/mfma_f32_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k32(const float *a, const float *b, float *d) {
    const int l = threadIdx.x;
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = 0.f;
    c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[l], b[l], c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) d[r * 64 + l] = c[r];
}
__global__ void k16(const float *a, const float *b, float *d) {
    const int l = threadIdx.x;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[l], b[l], c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[r * 64 + l] = c[r];
}

int main() {
    float ha[64], hb[64], hd[1024];
    float *a, *b, *d;
    hipMalloc(&a, 256); hipMalloc(&b, 256); hipMalloc(&d, 4096);
    int bad = 0;
    // 32x32x2: A[i][k] = i + 1 + 100 k, B[k][j] = (j + 1) * (k ? 1000 : 1)
    for (int l = 0; l < 64; ++l) {
        const int i = l & 31, k = l >> 5;
        ha[l] = (float)(i + 1 + 100 * k);
        hb[l] = (float)((i + 1) * (k ? 1000 : 1));
    }
    hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
    k32<<<1, 64>>>(a, b, d);
    hipMemcpy(hd, d, 4096, hipMemcpyDeviceToHost);
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            const double want = (double)(i + 1) * (j + 1) + (double)(i + 101) * (j + 1) * 1000;
            const int r = (i & 3) + 4 * (i >> 3), l = j + 32 * ((i >> 2) & 1);
            if (hd[r * 64 + l] != (float)want) {
                if (bad++ < 5) printf("32x32x2 D[%d][%d]: got %g want %g\n", i, j, hd[r * 64 + l], want);
            }
        }
    printf("32x32x2f32 map: %s\n", bad ? "MISMATCH" : "ok");
    int bad16 = 0;
    for (int l = 0; l < 64; ++l) {
        const int i = l & 15, k = l >> 4;
        ha[l] = (float)(i + 1 + 20 * k);
        hb[l] = (float)((i + 1) * (k == 0 ? 1 : (k == 1 ? 50 : (k == 2 ? 2500 : 125000))));
    }
    hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
    k16<<<1, 64>>>(a, b, d);
    hipMemcpy(hd, d, 4096, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double want = 0;
            const double sc[4] = {1, 50, 2500, 125000};
            for (int k = 0; k < 4; ++k) want += (double)(i + 1 + 20 * k) * (j + 1) * sc[k];
            const int r = i & 3, l = j + 16 * (i >> 2);
            if (hd[r * 64 + l] != (float)want) {
                if (bad16++ < 5) printf("16x16x4 D[%d][%d]: got %g want %g\n", i, j, hd[r * 64 + l], want);
            }
        }
    printf("16x16x4f32 map: %s\n", bad16 ? "MISMATCH" : "ok");
    return bad || bad16;
}
