/* Host cost of one action chunk of the wrapper stack (csrc/envwrap.c) over the C linear simulator,
 * without Python: 64 envs, hopper dims (Do 11, Da 3, Ta 4), 1 / 2 / 4 / 8 pool threads.
 *   gcc -O3 -march=x86-64-v3 -Iinclude -o /tmp/lowdim_step_bench tools/lowdim_step_bench.c \
 *       -Ldiffusionpolicyoptimization_amd/lib -ldppo_env -Wl,-rpath,$PWD/diffusionpolicyoptimization_amd/lib */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "dppo_env.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
    const int E = argc > 1 ? atoi(argv[1]) : 64, Do = 11, Da = 3, Ta = 4, n = argc > 2 ? atoi(argv[2]) : 20000;
    double A[121], B[33], c[11], goal[11], center[11], scale[11], bound[11];
    float omin[11], omax[11], amin[3], amax[3];
    for (int j = 0; j < Do; ++j) {
        for (int q = 0; q < Do; ++q) A[j * Do + q] = (j == q ? 0.9 : 0.01 * sin(j + 2.0 * q));
        c[j] = 0.01 * j; goal[j] = 0.1; center[j] = 0.0; scale[j] = 0.1; bound[j] = 1e9;
        omin[j] = -2.0f - j; omax[j] = 3.0f + j;
    }
    for (int i = 0; i < Da * Do; ++i) B[i] = 0.02 * cos(i);
    for (int q = 0; q < Da; ++q) { amin[q] = -1.0f; amax[q] = 1.0f; }
    int64_t* seeds = calloc(E, 8);
    for (int i = 0; i < E; ++i) seeds[i] = 42 + i;
    void* sim = dppo_sim_linear_create(E, Do, Da, A, B, c, goal, center, scale, bound, seeds);
    void* env = dppo_lowdim_create(E, Do, Da, 1, Ta, 1000000, 1, (dppo_sim_step_fn)dppo_sim_linear_step_fn(),
                                   (dppo_sim_reset_fn)dppo_sim_linear_reset_fn(), sim, omin, omax, amin, amax);
    float* act = calloc((size_t)E * Ta * Da, 4);
    float* obs = calloc((size_t)E * Do, 4);
    float* fin = calloc((size_t)E * Do, 4);
    double* rew = calloc(E, 8);
    uint8_t *te = calloc(E, 1), *tr = calloc(E, 1), *hf = calloc(E, 1);
    for (int i = 0; i < E * Ta * Da; ++i) act[i] = (float)(0.5 * sin(0.37 * i));
    dppo_lowdim_reset_all(env, obs);
    const int threads[] = {1, 2, 4, 8};
    for (int k = 0; k < 4; ++k) {
        dppo_lowdim_set_threads(env, threads[k], 2000.0);
        for (int r = 0; r < 500; ++r) dppo_lowdim_step(env, act, Ta, rew, te, tr, obs, fin, hf);
        const double t0 = now();
        for (int r = 0; r < n; ++r) dppo_lowdim_step(env, act, Ta, rew, te, tr, obs, fin, hf);
        printf("{\"envs\": %d, \"threads\": %d, \"us_per_chunk\": %.3f}\n", E, threads[k], (now() - t0) / n * 1e6);
    }
    {   /* the simulator alone: 4 sub-steps x E envs */
        int32_t* idx = calloc(E, 4);
        double *a = calloc((size_t)E * Da, 8), *o = calloc((size_t)E * Do, 8), *rw = calloc(E, 8);
        uint8_t* dn = calloc(E, 1);
        int8_t* tl = calloc(E, 1);
        for (int i = 0; i < E; ++i) idx[i] = i;
        const double t0 = now();
        for (int r = 0; r < n; ++r)
            for (int k = 0; k < Ta; ++k) dppo_sim_linear_step(sim, E, idx, a, o, rw, dn, tl);
        printf("{\"envs\": %d, \"simulator_only_us_per_chunk\": %.3f}\n", E, (now() - t0) / n * 1e6);
    }
    dppo_lowdim_destroy(env);
    dppo_sim_linear_destroy(sim);
    return 0;
}
