// Minimal repro for the rocprofv3 exit-time SIGSEGV, with no torch and no
// libfenv in the process: one trivial kernel launched cooperatively (9 workgroups, like the PPO
// update's split launch) or plainly, synchronised, then a normal return from main.
//   hipcc --offload-arch=gfx950 -O2 -o tools/coop_exit_min tools/coop_exit_min.hip
//   rocprofv3 --kernel-trace --stats -d OUT -o p -- tools/coop_exit_min coop|plain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void k_touch(float *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = (float)blockIdx.x;
}

int main(int argc, char **argv) {
    const bool coop = argc > 1 && std::strcmp(argv[1], "coop") == 0;
    float *d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(float)) != hipSuccess) return 2;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 2;
    hipError_t e;
    if (coop) {
        void *args[] = {&d};
        e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(&k_touch), dim3(9), dim3(256),
                                       args, 0, st);
    } else {
        hipLaunchKernelGGL(k_touch, dim3(9), dim3(256), 0, st, d);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        std::printf("launch failed: %s\n", hipGetErrorString(e));
        return 3;
    }
    if (hipStreamSynchronize(st) != hipSuccess) return 4;
    float h[9];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 5;
    std::printf("%s launch ok: %g .. %g\n", coop ? "cooperative" : "plain", h[0], h[8]);
    std::fflush(stdout);  // the exit-time crash under the profiler would lose a buffered line
    (void)hipStreamDestroy(st);
    (void)hipFree(d);
    return 0;
}
