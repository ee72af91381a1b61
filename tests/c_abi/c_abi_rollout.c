/* The C ABI (include/fenv.h) driven from plain C, without Python or torch in the process: the
 * way a C / C++ training loop would bind libfenv.so.  A small env (F = 37 formations x N
 * agents, both obs layouts, MT19937 resets every 11 steps) is reset, rolled out in fused chunks
 * that straddle reset events, stepped once more, then once through device-mapped host memory
 * (fenv_host_alloc); every observation, reward and done byte and the final state are compared
 * with the CPU oracle (oracle/fenv_oracle.c, test infrastructure).
 * Also checks the ABI's error contract (negative code + fenv_last_error) on bad arguments.
 * Built by tests/c_abi/Makefile (from __graft_entry__.build()); run by
 * tests/test_gpu_c_abi.py on the GPU box.  Exit 0 = all bit-exact. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fenv.h"

/* oracle/fenv_oracle.c (liboracle.so) */
typedef struct orc_env orc_env;
orc_env *orc_env_create(int64_t F, int32_t N, int32_t goal_in_obs, double share,
                        int32_t max_steps, uint32_t seed);
void orc_env_destroy(orc_env *e);
void orc_env_reset(orc_env *e, float *obs);
void orc_env_step(orc_env *e, const float *act, float *obs, float *rew, uint8_t *done);
void orc_env_get_state(const orc_env *e, float *px, float *py, float *gx, float *gy, int32_t *t);

#define HIP(x)                                                            \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            exit(2);                                                      \
        }                                                                 \
    } while (0)
#define ABI(x)                                                            \
    do {                                                                  \
        int rc_ = (x);                                                    \
        if (rc_ != FENV_OK) {                                             \
            fprintf(stderr, "%s -> %d: %s\n", #x, rc_, fenv_last_error()); \
            exit(3);                                                      \
        }                                                                 \
    } while (0)

/* deterministic actions in [-1.2, 1.2) (splitmix64 bits) */
static uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int same(const void *a, const void *b, size_t n, const char *what, int step) {
    if (memcmp(a, b, n) == 0) return 1;
    fprintf(stderr, "mismatch: %s at step %d\n", what, step);
    return 0;
}

static int run(int32_t N, int goal) {
    const int64_t F = 37, A = F * N;
    const int D = goal ? 8 : 6, max_steps = 9;
    const uint32_t seed = 123u + (uint32_t)N;
    fenv_t *env = NULL;
    ABI(fenv_create(&env, 0, F, N, goal, 0.25, max_steps, seed, FENV_RESET_MT19937, 0, 0));
    orc_env *ref = orc_env_create(F, N, goal, 0.25, max_steps, seed);
    const int TMAX = 14;
    float *act, *obs, *rew;
    uint8_t *done;
    HIP(hipMalloc((void **)&act, sizeof(float) * TMAX * A * 2));
    HIP(hipMalloc((void **)&obs, sizeof(float) * TMAX * A * D));
    HIP(hipMalloc((void **)&rew, sizeof(float) * TMAX * A));
    HIP(hipMalloc((void **)&done, (size_t)TMAX * A));
    float *h_act = malloc(sizeof(float) * TMAX * A * 2), *h_obs = malloc(sizeof(float) * TMAX * A * D);
    float *h_rew = malloc(sizeof(float) * TMAX * A), *r_obs = malloc(sizeof(float) * A * D);
    float *r_rew = malloc(sizeof(float) * A);
    uint8_t *h_done = malloc((size_t)TMAX * A), *r_done = malloc((size_t)A);
    int ok = 1, step = 0;

    ABI(fenv_reset(env, obs, NULL));
    HIP(hipDeviceSynchronize());
    HIP(hipMemcpy(h_obs, obs, sizeof(float) * A * D, hipMemcpyDeviceToHost));
    orc_env_reset(ref, r_obs);
    ok &= same(h_obs, r_obs, sizeof(float) * A * D, "reset obs", 0);

    uint64_t s = 0x5EED0000ull + (uint64_t)N;
    const int chunks[] = {10, 1, 14, 3};  /* crosses the resets at steps 11 and 22 */
    for (int c = 0; c < 4 && ok; ++c) {
        const int T = chunks[c];
        for (int64_t q = 0; q < (int64_t)T * A * 2; ++q)
            h_act[q] = (float)((double)(sm64(&s) >> 40) * 0x1.0p-24 * 2.4 - 1.2);
        HIP(hipMemcpy(act, h_act, sizeof(float) * T * A * 2, hipMemcpyHostToDevice));
        if (T == 1)
            ABI(fenv_step(env, act, obs, rew, done, NULL));
        else
            ABI(fenv_rollout(env, T, act, obs, rew, done, NULL, NULL));
        HIP(hipDeviceSynchronize());
        HIP(hipMemcpy(h_obs, obs, sizeof(float) * T * A * D, hipMemcpyDeviceToHost));
        HIP(hipMemcpy(h_rew, rew, sizeof(float) * T * A, hipMemcpyDeviceToHost));
        HIP(hipMemcpy(h_done, done, (size_t)T * A, hipMemcpyDeviceToHost));
        for (int k = 0; k < T && ok; ++k) {
            ++step;
            orc_env_step(ref, h_act + (int64_t)k * A * 2, r_obs, r_rew, r_done);
            ok &= same(h_obs + (int64_t)k * A * D, r_obs, sizeof(float) * A * D, "obs", step);
            ok &= same(h_rew + (int64_t)k * A, r_rew, sizeof(float) * A, "reward", step);
            ok &= same(h_done + (int64_t)k * A, r_done, (size_t)A, "done", step);
        }
    }
    /* one more step through device-mapped host memory (fenv_host_alloc): the kernel reads the
     * actions and writes obs / reward / done in the host block, no copies */
    if (ok) {
        const size_t sa = (size_t)A * 8, so = (size_t)A * D * 4, sr = (size_t)A * 4;
        const size_t oa = 0, oo = (sa + 255) / 256 * 256, orw = oo + (so + 255) / 256 * 256,
                     od = orw + (sr + 255) / 256 * 256;
        void *hb = NULL, *db = NULL;
        ABI(fenv_host_alloc(0, (int64_t)(od + (size_t)A), &hb, &db));
        char *h = (char *)hb, *d = (char *)db;
        for (int64_t q = 0; q < A * 2; ++q)
            ((float *)(h + oa))[q] = (float)((double)(sm64(&s) >> 40) * 0x1.0p-24 * 2.4 - 1.2);
        ABI(fenv_step(env, (const float *)(d + oa), (float *)(d + oo), (float *)(d + orw),
                      (uint8_t *)(d + od), NULL));
        HIP(hipDeviceSynchronize());
        ++step;
        orc_env_step(ref, (const float *)(h + oa), r_obs, r_rew, r_done);
        ok &= same(h + oo, r_obs, so, "host-block obs", step);
        ok &= same(h + orw, r_rew, sr, "host-block reward", step);
        ok &= same(h + od, r_done, (size_t)A, "host-block done", step);
        ABI(fenv_host_free(0, hb));
        if (fenv_host_free(0, hb) >= 0) {  /* a second free is refused */
            fprintf(stderr, "fenv_host_free accepted a freed block\n");
            ok = 0;
        }
    }
    /* final state */
    float *px, *py, *gx, *gy, *hp = malloc(sizeof(float) * (2 * A + 2 * F)), *rp = malloc(sizeof(float) * (2 * A + 2 * F));
    int32_t *t, ht[64], rt[64];
    HIP(hipMalloc((void **)&px, sizeof(float) * (2 * A + 2 * F)));
    HIP(hipMalloc((void **)&t, sizeof(int32_t) * F));
    py = px + A;
    gx = py + A;
    gy = gx + F;
    ABI(fenv_get_state(env, px, py, gx, gy, t, NULL));
    HIP(hipDeviceSynchronize());
    HIP(hipMemcpy(hp, px, sizeof(float) * (2 * A + 2 * F), hipMemcpyDeviceToHost));
    HIP(hipMemcpy(ht, t, sizeof(int32_t) * F, hipMemcpyDeviceToHost));
    orc_env_get_state(ref, rp, rp + A, rp + 2 * A, rp + 2 * A + F, rt);
    if (ok) ok &= same(hp, rp, sizeof(float) * (2 * A + 2 * F), "final positions/goals", step);
    if (ok) ok &= same(ht, rt, sizeof(int32_t) * F, "final steps_since_reset", step);

    HIP(hipFree(px));
    HIP(hipFree(t));
    HIP(hipFree(act));
    HIP(hipFree(obs));
    HIP(hipFree(rew));
    HIP(hipFree(done));
    free(hp); free(rp); free(h_act); free(h_obs); free(h_rew); free(r_obs); free(r_rew);
    free(h_done); free(r_done);
    orc_env_destroy(ref);
    ABI(fenv_destroy(env));
    printf("N=%d D=%d: %d steps bit-exact vs the C oracle: %s\n", N, D, step, ok ? "yes" : "NO");
    return ok;
}

int main(void) {
    int ok = 1;
    if (fenv_abi_version() != FENV_ABI_VERSION) {  /* built against another header revision */
        fprintf(stderr, "libfenv ABI %d, header %d\n", fenv_abi_version(), FENV_ABI_VERSION);
        return 1;
    }
    /* error contract: a negative code and a message, nothing allocated */
    fenv_t *bad = (fenv_t *)0x1;
    const int rc = fenv_create(&bad, 0, 10, 0, 1, 0.25, 1000, 0, FENV_RESET_MT19937, 0, 0);
    if (rc >= 0 || bad != NULL || strlen(fenv_last_error()) == 0) {
        fprintf(stderr, "bad-argument contract violated (rc %d)\n", rc);
        ok = 0;
    }
    ok &= run(5, 1);     /* whole formations per wavefront */
    ok &= run(100, 0);   /* one formation per workgroup, no goal in the observation */
    ok &= run(1500, 1);  /* several agents per thread */
    printf("C ABI: %s\n", ok ? "OK" : "FAILED");
    return ok ? 0 : 1;
}
