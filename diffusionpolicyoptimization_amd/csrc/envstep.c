/* envstep.c — batched host stepper for the synthetic locomotion env (env/synthetic.py).
 * One call advances all E envs by one action chunk (MultiStep semantics: act_steps sub-steps,
 * reward summed, stop at termination/truncation) and writes the float32 observation straight into
 * the caller's (pinned) staging buffer, so the next H2D copy needs no host-side repacking.
 * Envs are processed in blocks of EB with the state transposed to [Do][EB] in registers/L1, so
 * every inner loop runs over envs and vectorises (AVX2: 4 doubles). Resets of finished envs are
 * applied by the Python wrapper (rare: once per 250 chunks). */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#define DPPO_ENV_API __attribute__((visibility("default")))
#define EB 16
#define MAXD 64

DPPO_ENV_API int dppo_env_abi(void) { return 3; }

typedef double v4d __attribute__((vector_size(32)));
#define NV (EB / 4)

static inline v4d v4_splat(double x) { return (v4d){x, x, x, x}; }
static inline v4d v4_clamp1(v4d x) {
    return (v4d)_mm256_min_pd(_mm256_max_pd((__m256d)x, _mm256_set1_pd(-1.0)), _mm256_set1_pd(1.0));
}

/* AT = A^T (AT[i*Do + j] = A[j][i]); B [Da][Do]; state [E][Do] f64; actions [E][Ta][Da] f32 */
/* returns the number of envs whose episode ended in this chunk */
DPPO_ENV_API int dppo_env_step(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                                const double* __restrict__ AT, const double* __restrict__ B,
                                const double* __restrict__ c, const double* __restrict__ goal,
                                double* __restrict__ state, int64_t* __restrict__ cnt, const float* __restrict__ actions,
                                double* __restrict__ reward, uint8_t* __restrict__ terminated,
                                uint8_t* __restrict__ truncated, float* __restrict__ obs_out) {
    v4d s[MAXD][NV], ac[MAXD][NV];
    double rsum[EB], alive[EB];
    int64_t ct[EB];
    const int nsub = act_steps < Ta ? act_steps : Ta;
    int n_done = 0;
    for (int e0 = 0; e0 < E; e0 += EB) {
        const int nb = E - e0 < EB ? E - e0 : EB;
        for (int b = 0; b < EB; ++b) {
            const int e = e0 + (b < nb ? b : 0);
            for (int j = 0; j < Do; ++j) s[j][b >> 2][b & 3] = state[(size_t)e * Do + j];
            ct[b] = cnt[e];
            rsum[b] = 0.0;
            alive[b] = b < nb ? 1.0 : 0.0;
        }
        for (int k = 0; k < nsub; ++k) {
            for (int b = 0; b < EB; ++b) {
                const float* a = actions + ((size_t)(e0 + (b < nb ? b : 0)) * Ta + k) * Da;
                for (int i = 0; i < Da; ++i) ac[i][b >> 2][b & 3] = (double)a[i];
            }
            v4d asq[NV], err[NV], acl[MAXD][NV];
            for (int v = 0; v < NV; ++v) { asq[v] = v4_splat(0.0); err[v] = v4_splat(0.0); }
            for (int i = 0; i < Da; ++i)
                for (int v = 0; v < NV; ++v) { asq[v] += ac[i][v] * ac[i][v]; acl[i][v] = v4_clamp1(ac[i][v]); }
            v4d s2[MAXD][NV];
            for (int j = 0; j < Do; ++j) {
                v4d acc[NV];
                for (int v = 0; v < NV; ++v) acc[v] = v4_splat(c[j]);
                for (int i = 0; i < Do; ++i) {
                    const v4d w = v4_splat(AT[(size_t)i * Do + j]);
                    for (int v = 0; v < NV; ++v) acc[v] += w * s[i][v];
                }
                for (int i = 0; i < Da; ++i) {
                    const v4d w = v4_splat(B[(size_t)i * Do + j]);
                    for (int v = 0; v < NV; ++v) acc[v] += w * acl[i][v];
                }
                const v4d gj = v4_splat(goal[j]);
                for (int v = 0; v < NV; ++v) {
                    s2[j][v] = v4_clamp1(acc[v]);
                    const v4d d = s2[j][v] - gj;
                    err[v] += d * d;
                }
            }
            for (int b = 0; b < EB; ++b) {
                if (alive[b] != 0.0) {
                    for (int j = 0; j < Do; ++j) s[j][b >> 2][b & 3] = s2[j][b >> 2][b & 3];
                    ct[b] += 1;
                    rsum[b] += 1.0 - err[b >> 2][b & 3] / Do - 0.01 * asq[b >> 2][b & 3] / Da;
                    if (ct[b] >= max_steps) alive[b] = 0.0;
                }
            }
        }
        for (int b = 0; b < nb; ++b) {
            const int e = e0 + b;
            for (int j = 0; j < Do; ++j) state[(size_t)e * Do + j] = s[j][b >> 2][b & 3];
            cnt[e] = ct[b];
            reward[e] = rsum[b];
            terminated[e] = 0;
            truncated[e] = ct[b] >= max_steps;
            n_done += truncated[e];
            for (int o = 0; o < n_obs_steps; ++o)
                for (int j = 0; j < Do; ++j) obs_out[((size_t)e * n_obs_steps + o) * Do + j] = (float)s[j][b >> 2][b & 3];
        }
    }
    return n_done;
}

static double env_now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* One step of the pipelined rollout (ops.RolloutPipe) with the host's critical path in C: spin
 * until the device's done counter reaches done_target (the sampler wrote this step's actions into
 * the mapped action buffer), step the envs, and — when no episode ended, so no host-side reset
 * still has to rewrite observations — publish go_value to the go counter, releasing the
 * pre-enqueued sampler launch of the next step. go == NULL: never publish (the last step).
 * Returns n_done, with DPPO_ENV_PUBLISHED or'ed in when go was published; -1 host timeout;
 * -2 the device flagged that its own wait for go timed out. */
#define DPPO_ENV_PUBLISHED (1 << 30)
DPPO_ENV_API int dppo_env_step_gated(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                                     const double* AT, const double* B, const double* c, const double* goal,
                                     double* state, int64_t* cnt, const float* actions, double* reward,
                                     uint8_t* terminated, uint8_t* truncated, float* obs_out,
                                     const volatile uint32_t* done, uint32_t done_target, volatile uint32_t* go,
                                     uint32_t go_value, double timeout_s) {
    double t_end = -1.0;
    for (uint32_t spins = 0;; ++spins) {
        const uint32_t v = __atomic_load_n(done, __ATOMIC_ACQUIRE);
        if (v & 0x80000000u) return -2;
        if (v >= done_target) break;
        _mm_pause();
        if ((spins & 1023u) == 1023u) {
            const double now = env_now_s();
            if (t_end < 0.0) t_end = now + timeout_s;
            else if (now > t_end) return -1;
        }
    }
    const int n_done = dppo_env_step(E, Do, Da, act_steps, Ta, max_steps, n_obs_steps, AT, B, c, goal, state, cnt,
                                     actions, reward, terminated, truncated, obs_out);
    if (n_done == 0 && go) {
        __atomic_store_n(go, go_value, __ATOMIC_RELEASE);   /* x86: the obs stores are visible first */
        return DPPO_ENV_PUBLISHED;
    }
    return n_done;
}
