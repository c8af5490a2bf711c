/* envwrap.c — the host env boundary of the reference's gym locomotion stack, batched in C over a
 * simulator callback table, so a real simulator (MuJoCo's C API, or gym envs behind a Python
 * callback) plugs in without the reference's one-process-per-env pipes:
 *
 *   AsyncVectorEnv.step (env/gym_utils/async_vector_env.py:356-456, worker :774-840)
 *     -> MultiStep.step (env/gym_utils/wrapper/multi_step.py:135-192)
 *       -> MujocoLocomotionLowdimWrapper.step (wrapper/mujoco_locomotion_lowdim.py:57-70)
 *         -> the simulator (mujoco_py in the reference; here the dppo_sim callback table)
 *
 * One dppo_lowdim_step call executes one action chunk for all E envs: sub-step k calls sim.step ONCE
 * for the batch of envs still running, with the unnormalised float32 actions (:60-62), normalises
 * the raw observations (:57-58), sums rewards, applies MultiStep's termination / truncation rules
 * and, with reset_within_step, resets the envs whose chunk ended (sim.reset, one batched call).
 * Observations leave as float32 [E][To][Do] straight into the caller's (pinned) staging buffer.
 *
 * Arithmetic follows NumPy's on the reference's dtypes, bit for bit (compiled with
 * -ffp-contract=off): the action map is float32 ((a + 1) / 2 * (max - min) + min, every operand
 * float32); the observation map is float64 with the float32 range (max - min + 1e-6 in float32,
 * NumPy's weak-scalar rule) promoted. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DPPO_ENV_API __attribute__((visibility("default")))

/* The simulator: raw (unnormalised) coordinates, one batched call per sub-step. idx lists the n
 * env indices the call covers (ascending); rows of act / obs / reward / done / time_limit are in
 * idx order. step: act [n][Da] float64 (the float32 unnormalised actions, widened) -> obs [n][Do]
 * float64, reward [n], done [n] (gym's done), time_limit [n] (gym's info["TimeLimit.truncated"]:
 * -1 when the key is absent, else 0 / 1). reset: obs [n][Do]. Return 0, or nonzero to abort the
 * chunk (reported as -1 by dppo_lowdim_step). */
typedef int (*dppo_sim_step_fn)(void* ctx, int n, const int32_t* idx, const double* act, double* obs,
                                double* reward, uint8_t* done, int8_t* time_limit);
typedef int (*dppo_sim_reset_fn)(void* ctx, int n, const int32_t* idx, double* obs);

typedef struct {
    int E, Do, Da, To, act_steps, max_episode_steps, reset_within_step;
    dppo_sim_step_fn step;
    dppo_sim_reset_fn reset;
    void* ctx;
    float *obs_min, *obs_max, *act_min, *act_max;   /* NULL: identity maps (no normalisation file) */
    int64_t* cnt;        /* MultiStep.cnt per env */
    double* hist;        /* [E][To][Do]: the last To normalised observations (MultiStep.obs deque) */
    /* scratch */
    int32_t* idx;
    double *act, *obs, *rew;
    uint8_t* done;
    int8_t* tl;
    uint8_t *term, *trunc, *alive, *last_done;
} LowdimEnv;

DPPO_ENV_API int dppo_lowdim_abi(void) { return 1; }

/* mujoco_locomotion_lowdim.py:57-58, n rows of Do: out = 2 * ((raw - min) / (max - min + 1e-6) - 0.5) */
DPPO_ENV_API void dppo_lowdim_normalize_obs(int64_t n, int Do, const double* raw, const float* mn, const float* mx,
                                            double* out) {
    for (int64_t r = 0; r < n; ++r)
        for (int j = 0; j < Do; ++j) {
            const float rng = (float)(mx[j] - mn[j]) + 1e-6f;      /* float32 array + weak python float */
            const double v = (raw[r * Do + j] - (double)mn[j]) / (double)rng;
            out[r * Do + j] = 2.0 * (v - 0.5);
        }
}

/* mujoco_locomotion_lowdim.py:60-62, float32: a01 = (a + 1) / 2; raw = a01 * (max - min) + min */
DPPO_ENV_API void dppo_lowdim_unnormalize_action(int64_t n, int Da, const float* a, const float* mn, const float* mx,
                                                 float* out) {
    for (int64_t r = 0; r < n; ++r)
        for (int i = 0; i < Da; ++i) {
            const float a01 = (a[r * Da + i] + 1.0f) / 2.0f;
            const float rng = mx[i] - mn[i];
            const float m = a01 * rng;
            out[r * Da + i] = m + mn[i];
        }
}

static void* xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

DPPO_ENV_API void dppo_lowdim_destroy(void* h) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (!e) return;
    free(e->obs_min); free(e->obs_max); free(e->act_min); free(e->act_max);
    free(e->cnt); free(e->hist); free(e->idx); free(e->act); free(e->obs); free(e->rew);
    free(e->done); free(e->tl); free(e->term); free(e->trunc); free(e->alive); free(e->last_done);
    free(e);
}

/* max_episode_steps <= 0: MultiStep(max_episode_steps=None). obs_min/obs_max [Do], act_min/act_max
 * [Da]: the normalization.npz arrays (float32), or NULL for identity maps. */
DPPO_ENV_API void* dppo_lowdim_create(int E, int Do, int Da, int To, int act_steps, int max_episode_steps,
                                      int reset_within_step, dppo_sim_step_fn step, dppo_sim_reset_fn reset, void* ctx,
                                      const float* obs_min, const float* obs_max, const float* act_min,
                                      const float* act_max) {
    if (E < 1 || Do < 1 || Da < 1 || Da > 64 || To < 1 || act_steps < 1 || !step || !reset) return NULL;
    if ((obs_min == NULL) != (obs_max == NULL) || (act_min == NULL) != (act_max == NULL)) return NULL;
    LowdimEnv* e = (LowdimEnv*)xcalloc(1, sizeof(LowdimEnv));
    if (!e) return NULL;
    e->E = E; e->Do = Do; e->Da = Da; e->To = To; e->act_steps = act_steps;
    e->max_episode_steps = max_episode_steps; e->reset_within_step = reset_within_step;
    e->step = step; e->reset = reset; e->ctx = ctx;
    if (obs_min) {
        e->obs_min = (float*)xcalloc(Do, 4); e->obs_max = (float*)xcalloc(Do, 4);
        memcpy(e->obs_min, obs_min, 4 * (size_t)Do); memcpy(e->obs_max, obs_max, 4 * (size_t)Do);
    }
    if (act_min) {
        e->act_min = (float*)xcalloc(Da, 4); e->act_max = (float*)xcalloc(Da, 4);
        memcpy(e->act_min, act_min, 4 * (size_t)Da); memcpy(e->act_max, act_max, 4 * (size_t)Da);
    }
    e->cnt = (int64_t*)xcalloc(E, 8);
    e->hist = (double*)xcalloc((size_t)E * To * Do, 8);
    e->idx = (int32_t*)xcalloc(E, 4);
    e->act = (double*)xcalloc((size_t)E * Da, 8);
    e->obs = (double*)xcalloc((size_t)E * Do, 8);
    e->rew = (double*)xcalloc(E, 8);
    e->done = (uint8_t*)xcalloc(E, 1);
    e->tl = (int8_t*)xcalloc(E, 1);
    e->term = (uint8_t*)xcalloc(E, 1);
    e->trunc = (uint8_t*)xcalloc(E, 1);
    e->alive = (uint8_t*)xcalloc(E, 1);
    e->last_done = (uint8_t*)xcalloc(E, 1);
    if (!e->cnt || !e->hist || !e->idx || !e->act || !e->obs || !e->rew || !e->done || !e->tl || !e->term ||
        !e->trunc || !e->alive || !e->last_done) {
        dppo_lowdim_destroy(e);
        return NULL;
    }
    return e;
}

/* the normalised raw observation of row r of e->obs into env i's history: reset fills every slot
 * (stack_last_n_obs pads with the oldest entry, multi_step.py:68-78), a step shifts it in */
static void hist_put(LowdimEnv* e, int i, int r, int fill) {
    double* h = e->hist + (size_t)i * e->To * e->Do;
    double v[256];
    double* nv = e->Do <= 256 ? v : (double*)malloc(8 * (size_t)e->Do);
    if (e->obs_min) dppo_lowdim_normalize_obs(1, e->Do, e->obs + (size_t)r * e->Do, e->obs_min, e->obs_max, nv);
    else memcpy(nv, e->obs + (size_t)r * e->Do, 8 * (size_t)e->Do);
    if (fill) {
        for (int o = 0; o < e->To; ++o) memcpy(h + (size_t)o * e->Do, nv, 8 * (size_t)e->Do);
    } else {
        memmove(h, h + e->Do, 8 * (size_t)(e->To - 1) * e->Do);
        memcpy(h + (size_t)(e->To - 1) * e->Do, nv, 8 * (size_t)e->Do);
    }
    if (nv != v) free(nv);
}

static void hist_out(const LowdimEnv* e, int i, float* obs_out) {
    const double* h = e->hist + (size_t)i * e->To * e->Do;
    float* o = obs_out + (size_t)i * e->To * e->Do;
    for (int k = 0; k < e->To * e->Do; ++k) o[k] = (float)h[k];
}

/* reset the n envs idx[0..n) (MultiStep.reset, multi_step.py:113-133: cnt = 0, the deque holds the
 * reset observation only) */
static int reset_envs(LowdimEnv* e, int n, const int32_t* idx) {
    if (n == 0) return 0;
    if (e->reset(e->ctx, n, idx, e->obs)) return -1;
    for (int r = 0; r < n; ++r) {
        e->cnt[idx[r]] = 0;
        hist_put(e, idx[r], r, 1);
    }
    return 0;
}

/* AsyncVectorEnv.reset_arg -> MultiStep.reset for every env; obs_out [E][To][Do] float32 */
DPPO_ENV_API int dppo_lowdim_reset_all(void* h, float* obs_out) {
    LowdimEnv* e = (LowdimEnv*)h;
    for (int i = 0; i < e->E; ++i) e->idx[i] = i;
    if (reset_envs(e, e->E, e->idx)) return -1;
    for (int i = 0; i < e->E; ++i) hist_out(e, i, obs_out);
    return 0;
}

DPPO_ENV_API int dppo_lowdim_reset_one(void* h, int env, float* obs_out) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (env < 0 || env >= e->E) return -1;
    int32_t one = env;
    if (reset_envs(e, 1, &one)) return -1;
    hist_out(e, env, obs_out);
    return 0;
}

/* One chunk for all envs (multi_step.py:135-192). actions [E][Ta][Da] float32 (the first
 * min(act_steps, Ta) sub-steps are executed); outputs reward [E] (sum over the executed sub-steps),
 * terminated / truncated [E], obs_out [E][To][Do] (the observation after the chunk, or the reset
 * observation where the chunk ended and reset_within_step is set) and, when final_obs is not NULL,
 * final_obs [E][To][Do] with has_final [E] = 1 for envs that were truncated and reset within the
 * step (info["final_obs"], :177-183). Returns the number of envs whose chunk ended (done), or -1
 * when the simulator reported an error. */
DPPO_ENV_API int dppo_lowdim_step(void* h, const float* actions, int Ta, double* reward, uint8_t* terminated,
                                  uint8_t* truncated, float* obs_out, float* final_obs, uint8_t* has_final) {
    LowdimEnv* e = (LowdimEnv*)h;
    const int E = e->E, Do = e->Do, Da = e->Da, To = e->To;
    const int nsub = e->act_steps < Ta ? e->act_steps : Ta;
    for (int i = 0; i < E; ++i) {
        e->term[i] = e->trunc[i] = 0;
        e->alive[i] = 1;
        e->last_done[i] = 0;
        reward[i] = 0.0;
        if (has_final) has_final[i] = 0;
    }
    for (int k = 0; k < nsub; ++k) {
        /* for act_step, act in enumerate(action): self.cnt += 1; if terminated or truncated: break */
        int n = 0;
        for (int i = 0; i < E; ++i) {
            if (!e->alive[i]) continue;
            e->cnt[i] += 1;
            if (e->term[i] || e->trunc[i]) {
                e->alive[i] = 0;
                continue;
            }
            e->idx[n] = i;
            const float* a = actions + ((size_t)i * Ta + k) * Da;
            float raw[64];
            if (e->act_min) dppo_lowdim_unnormalize_action(1, Da, a, e->act_min, e->act_max, raw);
            else memcpy(raw, a, 4 * (size_t)Da);
            for (int j = 0; j < Da; ++j) e->act[(size_t)n * Da + j] = (double)raw[j];
            ++n;
        }
        if (n == 0) break;
        if (e->step(e->ctx, n, e->idx, e->act, e->obs, e->rew, e->done, e->tl)) return -1;
        for (int r = 0; r < n; ++r) {
            const int i = e->idx[r];
            hist_put(e, i, r, 0);
            reward[i] += e->rew[r];                                /* reward_agg_method = "sum" */
            if (e->tl[r] < 0) {                                    /* no "TimeLimit.truncated" in info */
                if (e->done[r]) e->term[i] = 1;
                else if (e->max_episode_steps > 0 && e->cnt[i] >= e->max_episode_steps) e->trunc[i] = 1;
            } else {
                e->trunc[i] = (uint8_t)(e->tl[r] != 0);
                e->term[i] = e->done[r] ? 1 : 0;
            }
            e->last_done[i] = e->term[i] || e->trunc[i];          /* self.done[-1] */
        }
    }
    /* the returned observation, then reset within the step where the chunk ended (:172-187) */
    int n_done = 0, nr = 0;
    for (int i = 0; i < E; ++i) {
        terminated[i] = e->term[i];
        truncated[i] = e->trunc[i];
        hist_out(e, i, obs_out);
        if (e->last_done[i]) {
            ++n_done;
            if (e->reset_within_step) {
                if (e->trunc[i] && final_obs) {
                    memcpy(final_obs + (size_t)i * To * Do, obs_out + (size_t)i * To * Do, 4 * (size_t)To * Do);
                    has_final[i] = 1;
                }
                e->idx[nr++] = i;
            }
        }
    }
    if (nr) {
        if (reset_envs(e, nr, e->idx)) return -1;
        for (int r = 0; r < nr; ++r) hist_out(e, e->idx[r], obs_out);
    }
    return n_done;
}

DPPO_ENV_API const int64_t* dppo_lowdim_counters(void* h) { return ((LowdimEnv*)h)->cnt; }

/* ---- a reference simulator in C: seeded linear dynamics in RAW coordinates with a terminal set ----
 * Fills the same callback table a MuJoCo C-API stepper would (mj_step per env + the task's reward
 * and termination), so the batched wrapper, the agent and the tests run it end to end on hosts
 * without MuJoCo. raw state s [Do]: s' = A s + B a + c; reward = 1 - mean((s' - goal)^2) - 1e-3 |a|^2;
 * done (terminal, like hopper's unhealthy check) when any |s'_j - center_j| > bound_j. Reset: a seeded hash of
 * (env seed, episode index) around `center`. */
typedef struct {
    int E, Do, Da;
    double *A, *B, *c, *goal, *center, *scale, *bound;   /* A [Do][Do] row-major, B [Da][Do] */
    double* s;          /* [E][Do] */
    int64_t *seed, *episode;
} LinearSim;

DPPO_ENV_API void* dppo_sim_linear_create(int E, int Do, int Da, const double* A, const double* B, const double* c,
                                          const double* goal, const double* center, const double* scale,
                                          const double* bound, const int64_t* seeds) {
    LinearSim* m = (LinearSim*)xcalloc(1, sizeof(LinearSim));
    if (!m) return NULL;
    m->E = E; m->Do = Do; m->Da = Da;
    m->bound = (double*)xcalloc(Do, 8);
    memcpy(m->bound, bound, 8 * (size_t)Do);
    m->A = (double*)xcalloc((size_t)Do * Do, 8); m->B = (double*)xcalloc((size_t)Da * Do, 8);
    m->c = (double*)xcalloc(Do, 8); m->goal = (double*)xcalloc(Do, 8);
    m->center = (double*)xcalloc(Do, 8); m->scale = (double*)xcalloc(Do, 8);
    m->s = (double*)xcalloc((size_t)E * Do, 8);
    m->seed = (int64_t*)xcalloc(E, 8); m->episode = (int64_t*)xcalloc(E, 8);
    memcpy(m->A, A, 8 * (size_t)Do * Do); memcpy(m->B, B, 8 * (size_t)Da * Do);
    memcpy(m->c, c, 8 * (size_t)Do); memcpy(m->goal, goal, 8 * (size_t)Do);
    memcpy(m->center, center, 8 * (size_t)Do); memcpy(m->scale, scale, 8 * (size_t)Do);
    memcpy(m->seed, seeds, 8 * (size_t)E);
    return m;
}

/* VectorEnv.seed([seed + i]) (agent/finetune/train_agent.py:53-56): new env seeds, episode counters
 * restart */
DPPO_ENV_API void dppo_sim_linear_seed(void* p, const int64_t* seeds) {
    LinearSim* m = (LinearSim*)p;
    memcpy(m->seed, seeds, 8 * (size_t)m->E);
    memset(m->episode, 0, 8 * (size_t)m->E);
}

DPPO_ENV_API void dppo_sim_linear_destroy(void* p) {
    LinearSim* m = (LinearSim*)p;
    if (!m) return;
    free(m->A); free(m->B); free(m->c); free(m->goal); free(m->center); free(m->scale); free(m->bound); free(m->s);
    free(m->seed); free(m->episode); free(m);
}

DPPO_ENV_API int dppo_sim_linear_step(void* ctx, int n, const int32_t* idx, const double* act, double* obs,
                                      double* reward, uint8_t* done, int8_t* time_limit) {
    LinearSim* m = (LinearSim*)ctx;
    const int Do = m->Do, Da = m->Da;
    double sn[256];
    if (Do > 256) return 1;
    for (int r = 0; r < n; ++r) {
        double* s = m->s + (size_t)idx[r] * Do;
        const double* a = act + (size_t)r * Da;
        double err = 0.0, asq = 0.0;
        int out = 0;
        for (int j = 0; j < Do; ++j) {
            double v = m->c[j];
            for (int q = 0; q < Do; ++q) v += m->A[(size_t)j * Do + q] * s[q];
            for (int q = 0; q < Da; ++q) v += m->B[(size_t)q * Do + j] * a[q];
            sn[j] = v;
            const double d = v - m->goal[j];
            err += d * d;
            const double dc = v - m->center[j];
            out |= dc > m->bound[j] || dc < -m->bound[j];
        }
        for (int q = 0; q < Da; ++q) asq += a[q] * a[q];
        memcpy(s, sn, 8 * (size_t)Do);
        memcpy(obs + (size_t)r * Do, sn, 8 * (size_t)Do);
        reward[r] = 1.0 - err / Do - 1e-3 * asq;
        done[r] = (uint8_t)out;
        time_limit[r] = -1;
    }
    return 0;
}

DPPO_ENV_API int dppo_sim_linear_reset(void* ctx, int n, const int32_t* idx, double* obs) {
    LinearSim* m = (LinearSim*)ctx;
    const int Do = m->Do;
    for (int r = 0; r < n; ++r) {
        const int i = idx[r];
        double* s = m->s + (size_t)i * Do;
        const uint64_t ep = (uint64_t)m->episode[i]++;
        for (int j = 0; j < Do; ++j) {
            /* splitmix64 of (seed, episode, j) -> U(-1, 1) */
            uint64_t z = (uint64_t)m->seed[i] * 0x9E3779B97F4A7C15ull + ep * 0xBF58476D1CE4E5B9ull + (uint64_t)j * 0x94D049BB133111EBull + 1;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
            s[j] = m->center[j] + m->scale[j] * u;
        }
        memcpy(obs + (size_t)r * Do, s, 8 * (size_t)Do);
    }
    return 0;
}

/* the callback addresses, for bindings that fill the table from C (ctypes: cast to the pointer type) */
DPPO_ENV_API void* dppo_sim_linear_step_fn(void) { return (void*)&dppo_sim_linear_step; }
DPPO_ENV_API void* dppo_sim_linear_reset_fn(void) { return (void*)&dppo_sim_linear_reset; }
