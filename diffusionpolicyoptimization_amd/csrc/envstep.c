/* envstep.c — batched host stepper for the synthetic locomotion env (env/synthetic.py).
 * One call advances all E envs by one action chunk (MultiStep semantics: act_steps sub-steps,
 * reward summed, stop at termination/truncation) and writes the float32 observation straight into
 * the caller's (pinned) staging buffer, so the next H2D copy needs no host-side repacking.
 * Resets of finished envs are applied by the Python wrapper (rare: once per 250 chunks). */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define DPPO_ENV_API __attribute__((visibility("default")))

static inline double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

DPPO_ENV_API int dppo_env_abi(void) { return 1; }

/* AT = A^T (row i holds column i of A) so the state update vectorises over the output coordinate */
DPPO_ENV_API void dppo_env_step(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                                const double* __restrict__ AT, const double* __restrict__ B,
                                const double* __restrict__ c, const double* __restrict__ goal,
                                double* __restrict__ state, int64_t* __restrict__ cnt, const float* __restrict__ actions,
                                double* __restrict__ reward, uint8_t* __restrict__ terminated,
                                uint8_t* __restrict__ truncated, float* __restrict__ obs_out) {
    double s2[64];
    for (int e = 0; e < E; ++e) {
        double* s = state + (size_t)e * Do;
        double rsum = 0.0;
        uint8_t trunc = 0;
        for (int k = 0; k < act_steps && k < Ta; ++k) {
            const float* a = actions + ((size_t)e * Ta + k) * Da;
            cnt[e] += 1;
            for (int j = 0; j < Do; ++j) s2[j] = c[j];
            for (int i = 0; i < Do; ++i) {
                const double si = s[i];
                const double* ai_row = AT + (size_t)i * Do;
                for (int j = 0; j < Do; ++j) s2[j] += ai_row[j] * si;
            }
            double asq = 0.0;
            for (int i = 0; i < Da; ++i) {
                const double ai = clampd((double)a[i], -1.0, 1.0);
                asq += (double)a[i] * (double)a[i];
                const double* b_row = B + (size_t)i * Do;
                for (int j = 0; j < Do; ++j) s2[j] += ai * b_row[j];
            }
            double err = 0.0;
            for (int j = 0; j < Do; ++j) {
                const double v = clampd(s2[j], -1.0, 1.0);
                s[j] = v;
                const double d = v - goal[j];
                err += d * d;
            }
            rsum += 1.0 - err / Do - 0.01 * asq / Da;
            if (cnt[e] >= max_steps) { trunc = 1; break; }
        }
        reward[e] = rsum;
        terminated[e] = 0;
        truncated[e] = trunc;
        for (int o = 0; o < n_obs_steps; ++o)
            for (int j = 0; j < Do; ++j) obs_out[((size_t)e * n_obs_steps + o) * Do + j] = (float)s[j];
    }
}
