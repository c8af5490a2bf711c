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

#include "dppo_env.h"

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
    v4d s[MAXD][NV], s2[MAXD][NV], acl[MAXD][NV];
    double sbuf[EB];
    const int nsub = act_steps < Ta ? act_steps : Ta;
    const v4d vmax = v4_splat((double)max_steps), one = v4_splat(1.0), zero = v4_splat(0.0);
    const v4d inv_do = v4_splat(1.0 / Do), c_a = v4_splat(0.01 / Da);
    int n_done = 0;
    for (int e0 = 0; e0 < E; e0 += EB) {
        const int nb = E - e0 < EB ? E - e0 : EB;
        v4d ct[NV], rsum[NV], alive[NV];   /* alive: 1.0 / 0.0 per env */
        for (int j = 0; j < Do; ++j) {
            for (int b = 0; b < EB; ++b) sbuf[b] = state[(size_t)(e0 + (b < nb ? b : 0)) * Do + j];
            for (int v = 0; v < NV; ++v) s[j][v] = (v4d){sbuf[4 * v], sbuf[4 * v + 1], sbuf[4 * v + 2], sbuf[4 * v + 3]};
        }
        for (int b = 0; b < EB; ++b) sbuf[b] = (double)cnt[e0 + (b < nb ? b : 0)];
        for (int v = 0; v < NV; ++v) {
            ct[v] = (v4d){sbuf[4 * v], sbuf[4 * v + 1], sbuf[4 * v + 2], sbuf[4 * v + 3]};
            rsum[v] = zero;
            alive[v] = (v4d){4 * v < nb, 4 * v + 1 < nb, 4 * v + 2 < nb, 4 * v + 3 < nb};
        }
        for (int k = 0; k < nsub; ++k) {
            v4d asq[NV], err[NV];
            for (int v = 0; v < NV; ++v) { asq[v] = zero; err[v] = zero; }
            for (int i = 0; i < Da; ++i) {
                for (int b = 0; b < EB; ++b) sbuf[b] = (double)actions[((size_t)(e0 + (b < nb ? b : 0)) * Ta + k) * Da + i];
                for (int v = 0; v < NV; ++v) {
                    const v4d x = (v4d){sbuf[4 * v], sbuf[4 * v + 1], sbuf[4 * v + 2], sbuf[4 * v + 3]};
                    asq[v] += x * x;
                    acl[i][v] = v4_clamp1(x);
                }
            }
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
                    const v4d n = v4_clamp1(acc[v]);
                    const v4d d = n - gj;
                    err[v] += d * d;
                    acc[v] = n;
                }
                /* s[j] is read by later rows j' of this sub-step: keep the new row aside */
                for (int v = 0; v < NV; ++v) s2[j][v] = acc[v];
            }
            for (int v = 0; v < NV; ++v) {
                const __m256d m = _mm256_cmp_pd((__m256d)alive[v], (__m256d)zero, _CMP_NEQ_OQ);
                for (int j = 0; j < Do; ++j) s[j][v] = (v4d)_mm256_blendv_pd((__m256d)s[j][v], (__m256d)s2[j][v], m);
                ct[v] += alive[v];
                rsum[v] += alive[v] * (one - err[v] * inv_do - asq[v] * c_a);
                alive[v] = (v4d)_mm256_and_pd((__m256d)alive[v], _mm256_cmp_pd((__m256d)ct[v], (__m256d)vmax, _CMP_LT_OQ));
            }
        }
        for (int j = 0; j < Do; ++j) {
            for (int v = 0; v < NV; ++v) for (int q = 0; q < 4; ++q) sbuf[4 * v + q] = s[j][v][q];
            for (int b = 0; b < nb; ++b) {
                const int e = e0 + b;
                state[(size_t)e * Do + j] = sbuf[b];
                for (int o = 0; o < n_obs_steps; ++o) obs_out[((size_t)e * n_obs_steps + o) * Do + j] = (float)sbuf[b];
            }
        }
        for (int v = 0; v < NV; ++v)
            for (int q = 0; q < 4; ++q) {
                const int b = 4 * v + q, e = e0 + b;
                if (b >= nb) continue;
                cnt[e] = (int64_t)ct[v][q];
                reward[e] = rsum[v][q];
                terminated[e] = 0;
                truncated[e] = ct[v][q] >= (double)max_steps;
                n_done += truncated[e];
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

/* Write the [E][n] float observation as tagged granules {tag << 32 | fp32 bits} (the tagged
 * rollout protocol, dppo_rollout_enqueue_tagged): each granule is one aligned 8-byte store, so the
 * device never sees a torn value, and a value with the new tag is the new observation. */
DPPO_ENV_API void dppo_env_publish_tagged(int64_t count, const float* obs, uint64_t* obs_tagged, uint32_t tag) {
    const uint64_t hi = (uint64_t)tag << 32;
    for (int64_t i = 0; i < count; ++i) {
        uint32_t bits;
        memcpy(&bits, obs + i, 4);
        __atomic_store_n(obs_tagged + i, hi | bits, __ATOMIC_RELAXED);
    }
}

/* dppo_env_step_gated with the tagged protocol both ways: the envs go in blocks of EB = 16 (the
 * split sampler's env group: each group of a pre-enqueued launch polls only its own 16 envs'
 * observation granules), and for each block in turn: spin until its action granules in act_tagged
 * carry act_tag (the device's stores are the ready flag: no wait for the done counter, whose bit 31
 * still reports a device-side timeout), decode them into `actions` (the float buffer the caller
 * keeps), step the block and, when no episode of the block ended, publish its observation as
 * granules with `tag` at once — so the next launch's first groups run while the host still steps
 * the later blocks. Returns n_done, with DPPO_ENV_PUBLISHED when every block was published (an
 * ended episode leaves its block to the caller, which resets and publishes the whole observation:
 * the early blocks' granules are rewritten with the same tag and values). */
DPPO_ENV_API int dppo_env_step_gated_tagged(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                                            const double* AT, const double* B, const double* c, const double* goal,
                                            double* state, int64_t* cnt, float* actions, double* reward,
                                            uint8_t* terminated, uint8_t* truncated, float* obs_out,
                                            const volatile uint32_t* done, const uint64_t* act_tagged,
                                            uint32_t act_tag, uint64_t* obs_tagged, uint32_t tag, double timeout_s) {
    const int64_t per = (int64_t)Ta * Da, per_obs = (int64_t)n_obs_steps * Do;
    double t_end = -1.0;
    int n_done = 0, all_published = 1;
    for (int e0 = 0; e0 < E; e0 += EB) {
        const int nb = E - e0 < EB ? E - e0 : EB;
        int64_t i = e0 * per;   /* granules before i are known to carry act_tag */
        const int64_t end = (e0 + nb) * per;
        for (uint32_t spins = 0;; ++spins) {
            while (i < end) {
                const uint64_t x = __atomic_load_n(act_tagged + i, __ATOMIC_ACQUIRE);
                if ((uint32_t)(x >> 32) != act_tag) break;
                const uint32_t bits = (uint32_t)x;
                memcpy(actions + i, &bits, 4);
                ++i;
            }
            if (i == end) break;
            if (__atomic_load_n(done, __ATOMIC_ACQUIRE) & 0x80000000u) return -2;
            _mm_pause();
            if ((spins & 1023u) == 1023u) {
                const double now = env_now_s();
                if (t_end < 0.0) t_end = now + timeout_s;
                else if (now > t_end) return -1;
            }
        }
        const int nd = dppo_env_step(nb, Do, Da, act_steps, Ta, max_steps, n_obs_steps, AT, B, c, goal,
                                     state + (size_t)e0 * Do, cnt + e0, actions + (size_t)e0 * per, reward + e0,
                                     terminated + e0, truncated + e0, obs_out + (size_t)e0 * per_obs);
        n_done += nd;
        if (nd == 0 && obs_tagged)
            dppo_env_publish_tagged((int64_t)nb * per_obs, obs_out + (size_t)e0 * per_obs, obs_tagged + (size_t)e0 * per_obs, tag);
        else
            all_published = 0;
    }
    if (all_published && obs_tagged) return n_done | DPPO_ENV_PUBLISHED;
    return n_done;
}
