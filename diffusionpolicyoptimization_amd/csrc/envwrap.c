/* envwrap.c — the host env boundary of the reference's gym locomotion stack, batched in C over a
 * simulator callback table and fanned out over a pool of host threads, so a real simulator
 * (MuJoCo's C API, or gym envs behind a Python callback) plugs in without the reference's
 * one-process-per-env pipes:
 *
 *   AsyncVectorEnv.step (env/gym_utils/async_vector_env.py:356-456, worker :774-840)
 *     -> MultiStep.step (env/gym_utils/wrapper/multi_step.py:135-192)
 *       -> MujocoLocomotionLowdimWrapper.step (wrapper/mujoco_locomotion_lowdim.py:57-70)
 *         -> the simulator (mujoco_py in the reference; here the dppo_sim callback table)
 *
 * One dppo_lowdim_step call executes one action chunk for all E envs. The envs are split into
 * contiguous slices, one per pool thread (the reference's worker processes, async_vector_env.py:
 * 189-214, become threads of this process; the caller's thread runs slice 0). Within a slice,
 * sub-step k calls sim.step ONCE for the slice's envs still running, with the unnormalised float32
 * actions (:60-62), normalises the raw observations (:57-58), sums rewards, applies MultiStep's
 * termination / truncation rules and, with reset_within_step, resets the envs whose chunk ended
 * (sim.reset, one batched call per slice). Observations leave as float32 [E][To][Do] straight into
 * the caller's (pinned / mapped) staging buffer. Every env's arithmetic depends on that env alone,
 * so the outputs are bit-identical for any thread count (tests/test_envstack_cpu.py).
 *
 * The gated entries (dppo_lowdim_step_gated_tagged / _gated) are the pipelined rollout's host
 * step (ops.RolloutPipe): each slice thread polls ITS envs' action granules in mapped
 * memory, steps them, and publishes ITS envs' observation granules as soon as they are final, 16
 * envs (one sampler env group) at a time, so the sampler launch for the next chunk (already
 * enqueued, each group polling its own granules) starts group by group while the host still steps.
 *
 * Arithmetic follows NumPy's on the reference's dtypes, bit for bit (compiled with
 * -ffp-contract=off): the action map is float32 ((a + 1) / 2 * (max - min) + min, every operand
 * float32); the observation map is float64 with the float32 range (max - min + 1e-6 in float32,
 * NumPy's weak-scalar rule) promoted. */
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dppo_env.h"

#define DPPO_ENV_API __attribute__((visibility("default")))

/* default solo floor (dppo_lowdim_set_solo_floor): a pool hand-off measured 11-15 us per chunk on
 * the GPU box's host (profiles/r04r_bench_lowdim_t{1,4}_c0.json) */
#define DPPO_SOLO_FLOOR_US 25.0

/* the simulator callback table (dppo_sim_step_fn / dppo_sim_reset_fn) and every entry point are
 * declared in include/dppo_env.h */

struct LowdimEnv;

/* one chunk's arguments, shared by the slice threads */
typedef struct {
    float* actions;                /* [E][Ta][Da]; the gated tagged step decodes into it */
    int Ta;
    double* reward;
    uint8_t *terminated, *truncated;
    float *obs_out, *final_obs;
    uint8_t* has_final;
    /* gated tagged protocol (NULL act_tagged: plain step) */
    const volatile uint32_t* done;
    const uint64_t* act_tagged;
    uint32_t act_tag;
    uint64_t* obs_tagged;          /* NULL: do not publish */
    uint32_t obs_tag;
    double deadline;               /* monotonic seconds */
} Chunk;

typedef struct {
    struct LowdimEnv* env;
    int n;                         /* threads, the caller's included */
    pthread_t* th;
    int* rc;                       /* per-slice result */
    volatile int gen;              /* job generation (bumped under mu) */
    volatile int pending;          /* slices still running */
    volatile int stop;
    int sleepers;
    double spin_s;                 /* how long an idle worker spins before it sleeps */
    pthread_mutex_t mu;
    pthread_cond_t cv;
} Pool;

/* per-env MultiStep flags, one cache line per env: the slice threads write their own envs' flags
 * every sub-step, and packed bytes would put neighbouring slices on one line (false sharing) */
typedef struct {
    uint8_t term, trunc, alive, last_done;
    uint8_t pad[60];
} EnvFlags;

/* one thread's sub-step scratch (the rows of its slice), in allocations of its own */
typedef struct {
    int32_t* idx;
    double *act, *obs, *rew;
    uint8_t* done;
    int8_t* tl;
} Scratch;

typedef struct LowdimEnv {
    int E, Do, Da, To, act_steps, max_episode_steps, reset_within_step;
    dppo_sim_step_fn step;
    dppo_sim_reset_fn reset;
    void* ctx;
    float *obs_min, *obs_max, *act_min, *act_max;   /* NULL: identity maps (no normalisation file) */
    float *obs_rng, *act_rng;   /* (float)(max - min) + 1e-6f and max - min, the maps' float32 ranges */
    int64_t* cnt;        /* MultiStep.cnt per env */
    double* hist;        /* [E][To][Do]: the last To normalised observations (MultiStep.obs deque) */
    EnvFlags* fl;        /* [E] */
    Scratch* scr;        /* [nscr] per pool thread (scr[0]: the caller's, E rows) */
    int nscr;
    Pool* pool;          /* NULL: one thread */
    Chunk chunk;         /* the chunk in flight */
    /* the solo floor (dppo_lowdim_set_solo_floor): a pool steps a chunk on the caller's thread alone
     * while the chunk's estimated stepping work is below the hand-off it would save */
    double solo_floor_s; /* 0: always use the pool */
    double work_est_s;   /* running estimate of one chunk's stepping work, all envs (< 0: none yet) */
    double work0_s;      /* this chunk's stepping work on the caller's thread (waits excluded) */
    int solo;            /* the current mode (hysteresis: enter below the floor, leave above twice it) */
    int64_t solo_chunks;
} LowdimEnv;

DPPO_ENV_API int dppo_lowdim_abi(void) { return 2; }

static double mono_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* mujoco_locomotion_lowdim.py:57-58, one row of Do: out = 2 * ((raw - min) / (max - min + 1e-6) - 0.5),
 * rng[j] = (float)(max - min) + 1e-6f (float32 array + weak python float) */
static inline void norm_obs_row(int Do, const double* raw, const float* mn, const float* rng, double* out) {
    for (int j = 0; j < Do; ++j) {
        const double v = (raw[j] - (double)mn[j]) / (double)rng[j];
        out[j] = 2.0 * (v - 0.5);
    }
}
static inline float obs_rng_of(float mn, float mx) { return (float)(mx - mn) + 1e-6f; }

/* mujoco_locomotion_lowdim.py:60-62, float32: a01 = (a + 1) / 2; raw = a01 * (max - min) + min */
static inline void unnorm_act_row(int Da, const float* a, const float* mn, const float* rng, float* out) {
    for (int i = 0; i < Da; ++i) {
        const float a01 = (a[i] + 1.0f) / 2.0f;
        const float m = a01 * rng[i];
        out[i] = m + mn[i];
    }
}

DPPO_ENV_API void dppo_lowdim_normalize_obs(int64_t n, int Do, const double* raw, const float* mn, const float* mx,
                                            double* out) {
    float stack[256];   /* any Do: wider observations take the range row from the heap */
    float* rng = Do <= 256 ? stack : (float*)malloc(sizeof(float) * (size_t)(Do > 0 ? Do : 1));
    if (!rng) abort();  /* a void entry point: no silent uninitialised output */
    for (int j = 0; j < Do; ++j) rng[j] = obs_rng_of(mn[j], mx[j]);
    for (int64_t r = 0; r < n; ++r) norm_obs_row(Do, raw + r * Do, mn, rng, out + r * Do);
    if (rng != stack) free(rng);
}

DPPO_ENV_API void dppo_lowdim_unnormalize_action(int64_t n, int Da, const float* a, const float* mn, const float* mx,
                                                 float* out) {
    float stack[64];
    float* rng = Da <= 64 ? stack : (float*)malloc(sizeof(float) * (size_t)(Da > 0 ? Da : 1));
    if (!rng) abort();
    for (int i = 0; i < Da; ++i) rng[i] = mx[i] - mn[i];
    for (int64_t r = 0; r < n; ++r) unnorm_act_row(Da, a + r * Da, mn, rng, out + r * Da);
    if (rng != stack) free(rng);
}

static void* xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

static void pool_destroy(Pool* p);

static void scratch_free(LowdimEnv* e) {
    for (int t = 0; t < e->nscr; ++t) {
        Scratch* c = &e->scr[t];
        free(c->idx); free(c->act); free(c->obs); free(c->rew); free(c->done); free(c->tl);
    }
    free(e->scr);
    e->scr = NULL;
    e->nscr = 0;
}

/* n scratch sets of `rows` rows each (64-B aligned allocations: no two threads' scratch shares a line) */
static int scratch_alloc(LowdimEnv* e, int n, int rows) {
    scratch_free(e);
    e->scr = (Scratch*)xcalloc(n, sizeof(Scratch));
    if (!e->scr) return -1;
    e->nscr = n;
    const size_t r64 = ((size_t)rows + 63) & ~(size_t)63;
    for (int t = 0; t < n; ++t) {
        Scratch* c = &e->scr[t];
        c->idx = (int32_t*)aligned_alloc(64, 4 * r64);
        c->act = (double*)aligned_alloc(64, 8 * r64 * e->Da);
        c->obs = (double*)aligned_alloc(64, 8 * r64 * e->Do);
        c->rew = (double*)aligned_alloc(64, 8 * r64);
        c->done = (uint8_t*)aligned_alloc(64, r64);
        c->tl = (int8_t*)aligned_alloc(64, r64);
        if (!c->idx || !c->act || !c->obs || !c->rew || !c->done || !c->tl) return -1;
    }
    return 0;
}

DPPO_ENV_API void dppo_lowdim_destroy(void* h) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (!e) return;
    pool_destroy(e->pool);
    free(e->obs_min); free(e->obs_max); free(e->act_min); free(e->act_max); free(e->obs_rng); free(e->act_rng);
    free(e->cnt); free(e->hist); free(e->fl);
    scratch_free(e);
    free(e);
}

/* max_episode_steps <= 0: MultiStep(max_episode_steps=None). obs_min/obs_max [Do], act_min/act_max
 * [Da]: the normalization.npz arrays (float32), or NULL for identity maps. One thread until
 * dppo_lowdim_set_threads. */
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
    e->solo_floor_s = DPPO_SOLO_FLOOR_US * 1e-6;
    e->work_est_s = -1.0;
    if (obs_min) {
        e->obs_min = (float*)xcalloc(Do, 4); e->obs_max = (float*)xcalloc(Do, 4); e->obs_rng = (float*)xcalloc(Do, 4);
        memcpy(e->obs_min, obs_min, 4 * (size_t)Do); memcpy(e->obs_max, obs_max, 4 * (size_t)Do);
        for (int j = 0; j < Do; ++j) e->obs_rng[j] = obs_rng_of(obs_min[j], obs_max[j]);
    }
    if (act_min) {
        e->act_min = (float*)xcalloc(Da, 4); e->act_max = (float*)xcalloc(Da, 4); e->act_rng = (float*)xcalloc(Da, 4);
        memcpy(e->act_min, act_min, 4 * (size_t)Da); memcpy(e->act_max, act_max, 4 * (size_t)Da);
        for (int i = 0; i < Da; ++i) e->act_rng[i] = act_max[i] - act_min[i];
    }
    e->cnt = (int64_t*)xcalloc(E, 8);
    e->hist = (double*)xcalloc((size_t)E * To * Do, 8);
    e->fl = (EnvFlags*)aligned_alloc(64, sizeof(EnvFlags) * (size_t)E);
    if (!e->cnt || !e->hist || !e->fl || scratch_alloc(e, 1, E)) {
        dppo_lowdim_destroy(e);
        return NULL;
    }
    memset(e->fl, 0, sizeof(EnvFlags) * (size_t)E);
    return e;
}

/* the normalised raw observation `raw` [Do] into env i's history: reset fills every slot
 * (stack_last_n_obs pads with the oldest entry, multi_step.py:68-78), a step shifts it in */
static void hist_put(LowdimEnv* e, int i, const double* raw, int fill) {
    double* h = e->hist + (size_t)i * e->To * e->Do;
    double v[256];
    double* nv = e->Do <= 256 ? v : (double*)malloc(8 * (size_t)e->Do);
    if (e->obs_min) norm_obs_row(e->Do, raw, e->obs_min, e->obs_rng, nv);
    else memcpy(nv, raw, 8 * (size_t)e->Do);
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
 * reset observation only); obs: the n-row scratch the simulator writes */
static int reset_envs(LowdimEnv* e, int n, const int32_t* idx, double* obs) {
    if (n == 0) return 0;
    if (e->reset(e->ctx, n, idx, obs)) return -1;
    for (int r = 0; r < n; ++r) {
        e->cnt[idx[r]] = 0;
        hist_put(e, idx[r], obs + (size_t)r * e->Do, 1);
    }
    return 0;
}

/* ---- the pool: persistent threads, slice t of a chunk = envs [E t / n, E (t + 1) / n) ---- */
static int slice_lo(const LowdimEnv* e, int n, int t) { return (int)((int64_t)e->E * t / n); }

static int run_slice(LowdimEnv* e, int t, int lo, int hi);

typedef struct { Pool* p; int t; } WorkerArg;

static void* worker(void* a) {
    WorkerArg* wa = (WorkerArg*)a;
    Pool* p = wa->p;
    const int t = wa->t;
    free(wa);
    int seen = 0;   /* a new pool starts at generation 0: a chunk dispatched before this thread ran is still seen */
    for (;;) {
        /* spin for a while (a rollout steps every few tens of microseconds), then sleep */
        double t_end = -1.0;
        for (uint32_t spins = 0; __atomic_load_n(&p->gen, __ATOMIC_ACQUIRE) == seen && !p->stop; ++spins) {
            _mm_pause();
            if ((spins & 255u) == 255u) {
                sched_yield();
                const double now = mono_s();
                if (t_end < 0.0) t_end = now + p->spin_s;
                else if (now > t_end) break;
            }
        }
        if (__atomic_load_n(&p->gen, __ATOMIC_ACQUIRE) == seen && !p->stop) {
            pthread_mutex_lock(&p->mu);
            p->sleepers++;
            while (__atomic_load_n(&p->gen, __ATOMIC_ACQUIRE) == seen && !p->stop) pthread_cond_wait(&p->cv, &p->mu);
            p->sleepers--;
            pthread_mutex_unlock(&p->mu);
        }
        if (p->stop) break;
        seen = __atomic_load_n(&p->gen, __ATOMIC_ACQUIRE);
        LowdimEnv* e = p->env;
        p->rc[t] = run_slice(e, t, slice_lo(e, p->n, t), slice_lo(e, p->n, t + 1));
        __atomic_fetch_sub(&p->pending, 1, __ATOMIC_ACQ_REL);
    }
    return NULL;
}

static void pool_destroy(Pool* p) {
    if (!p) return;
    pthread_mutex_lock(&p->mu);
    p->stop = 1;
    pthread_cond_broadcast(&p->cv);
    pthread_mutex_unlock(&p->mu);
    for (int t = 1; t < p->n; ++t) pthread_join(p->th[t], NULL);
    pthread_mutex_destroy(&p->mu);
    pthread_cond_destroy(&p->cv);
    free(p->th); free(p->rc); free(p);
}

/* Threads that step the envs (the caller's included): 1 = step on the caller's thread only;
 * n > E is clamped to E. spin_us: how long an idle pool thread spins for the next chunk before it
 * sleeps (<= 0: 2000 us). Returns the thread count in use, or -1. */
DPPO_ENV_API int dppo_lowdim_set_threads(void* h, int n, double spin_us) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (!e) return -1;
    if (n < 1) n = 1;
    if (n > e->E) n = e->E;
    if (e->pool && e->pool->n == n) {
        e->pool->spin_s = (spin_us > 0 ? spin_us : 2000.0) * 1e-6;
        return n;
    }
    pool_destroy(e->pool);
    e->pool = NULL;
    if (scratch_alloc(e, n, e->E)) return -1;   /* one scratch set per thread (set 0 also serves resets) */
    if (n == 1) return 1;
    Pool* p = (Pool*)xcalloc(1, sizeof(Pool));
    if (!p) return -1;
    p->env = e; p->n = n;
    p->spin_s = (spin_us > 0 ? spin_us : 2000.0) * 1e-6;
    p->th = (pthread_t*)xcalloc(n, sizeof(pthread_t));
    p->rc = (int*)xcalloc(n, sizeof(int));
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->cv, NULL);
    for (int t = 1; t < n; ++t) {
        WorkerArg* wa = (WorkerArg*)malloc(sizeof(WorkerArg));
        wa->p = p; wa->t = t;
        if (pthread_create(&p->th[t], NULL, worker, wa)) {
            free(wa);
            p->n = t;              /* join the ones that started */
            pool_destroy(p);
            return -1;
        }
    }
    e->pool = p;
    return n;
}

/* The solo floor: with a pool, a chunk whose estimated stepping work (a running average of the
 * measured simulator + wrapper time, waits for actions excluded, scaled to all envs) is below
 * floor_us runs on the caller's thread alone; the pool is used again once the estimate exceeds twice
 * the floor. 0 disables (always the pool). Results do not depend on it. */
DPPO_ENV_API int dppo_lowdim_set_solo_floor(void* h, double floor_us) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (!e || floor_us < 0.0) return -1;
    e->solo_floor_s = floor_us * 1e-6;
    e->work_est_s = -1.0;
    e->solo = 0;
    return 0;
}

/* chunks stepped on the caller's thread alone under the solo floor */
DPPO_ENV_API int64_t dppo_lowdim_solo_chunks(void* h) { return ((LowdimEnv*)h)->solo_chunks; }

DPPO_ENV_API int dppo_lowdim_threads(void* h) {
    LowdimEnv* e = (LowdimEnv*)h;
    return e->pool ? e->pool->n : 1;
}

/* run e->chunk on every slice; the caller's thread takes slice 0. Returns the sum of the slices'
 * results, or the most negative one. */
static void note_work(LowdimEnv* e, double chunk_work_s) {
    e->work_est_s = e->work_est_s < 0.0 ? chunk_work_s : e->work_est_s + 0.5 * (chunk_work_s - e->work_est_s);
    if (e->solo) e->solo = e->work_est_s <= 2.0 * e->solo_floor_s;
    else e->solo = e->work_est_s < e->solo_floor_s;
}

static int run_chunk(LowdimEnv* e) {
    Pool* p = e->pool;
    if (!p) return run_slice(e, 0, 0, e->E);
    e->work0_s = 0.0;
    if (e->solo && e->solo_floor_s > 0.0) {
        /* below the floor a pool hand-off (wake, per-slice spins, the join) costs more than the
         * slices it would run in parallel: step every env here, in slice order (bit-identical) */
        const int rc = run_slice(e, 0, 0, e->E);
        e->solo_chunks++;
        note_work(e, e->work0_s);
        return rc;
    }
    __atomic_store_n(&p->pending, p->n - 1, __ATOMIC_RELEASE);
    pthread_mutex_lock(&p->mu);
    __atomic_fetch_add(&p->gen, 1, __ATOMIC_ACQ_REL);
    if (p->sleepers) pthread_cond_broadcast(&p->cv);
    pthread_mutex_unlock(&p->mu);
    p->rc[0] = run_slice(e, 0, 0, slice_lo(e, p->n, 1));
    /* yield now and then: a worker the scheduler placed on this CPU must get to run */
    for (uint32_t spins = 1; __atomic_load_n(&p->pending, __ATOMIC_ACQUIRE) > 0; ++spins) {
        _mm_pause();
        if ((spins & 63u) == 0) sched_yield();
    }
    const int n0 = slice_lo(e, p->n, 1);
    if (e->solo_floor_s > 0.0 && n0 > 0) note_work(e, e->work0_s * e->E / n0);
    int sum = 0, worst = 0;
    for (int t = 0; t < p->n; ++t) {
        if (p->rc[t] < worst) worst = p->rc[t];
        if (p->rc[t] > 0) sum += p->rc[t];
    }
    return worst < 0 ? worst : sum;
}

/* the gated tagged protocol, per slice: wait until env rows [lo, hi)'s action granules carry the
 * tag, decoding them into the float actions. 0, -1 (host timeout), -2 (device flagged a timeout) */
static int slice_wait_actions(LowdimEnv* e, int lo, int hi) {
    const Chunk* c = &e->chunk;
    const int64_t per = (int64_t)c->Ta * e->Da;
    int64_t i = lo * per;
    const int64_t end = hi * per;
    for (uint32_t spins = 0;; ++spins) {
        while (i < end) {
            const uint64_t x = __atomic_load_n(c->act_tagged + i, __ATOMIC_ACQUIRE);
            if ((uint32_t)(x >> 32) != c->act_tag) break;
            const uint32_t bits = (uint32_t)x;
            memcpy(c->actions + i, &bits, 4);
            ++i;
        }
        if (i == end) return 0;
        if (__atomic_load_n(c->done, __ATOMIC_ACQUIRE) & 0x80000000u) return -2;
        _mm_pause();
        if ((spins & 1023u) == 1023u) {
            sched_yield();
            if (mono_s() > c->deadline) return -1;
        }
    }
}

/* One chunk for envs [lo, hi) (multi_step.py:135-192); see dppo_lowdim_step. */
static int run_block(LowdimEnv* e, int t, int lo, int hi) {
    const Chunk* c = &e->chunk;
    const int Do = e->Do, Da = e->Da, To = e->To, Ta = c->Ta;
    if (lo >= hi) return 0;
    if (c->act_tagged) {
        const int w = slice_wait_actions(e, lo, hi);
        if (w) return w;
    }
    const double w0 = t == 0 ? mono_s() : 0.0;
    const Scratch* sc = &e->scr[t];
    int32_t* idx = sc->idx;
    double* act = sc->act;
    double* obs = sc->obs;
    double* rew = sc->rew;
    uint8_t* done = sc->done;
    int8_t* tl = sc->tl;
    EnvFlags* fl = e->fl;
    const int nsub = e->act_steps < Ta ? e->act_steps : Ta;
    for (int i = lo; i < hi; ++i) {
        fl[i].term = fl[i].trunc = 0;
        fl[i].alive = 1;
        fl[i].last_done = 0;
        c->reward[i] = 0.0;
        if (c->has_final) c->has_final[i] = 0;
    }
    for (int k = 0; k < nsub; ++k) {
        /* for act_step, act in enumerate(action): self.cnt += 1; if terminated or truncated: break */
        int n = 0;
        for (int i = lo; i < hi; ++i) {
            if (!fl[i].alive) continue;
            e->cnt[i] += 1;
            if (fl[i].term || fl[i].trunc) {
                fl[i].alive = 0;
                continue;
            }
            idx[n] = i;
            const float* a = c->actions + ((size_t)i * Ta + k) * Da;
            float raw[64];
            if (e->act_min) unnorm_act_row(Da, a, e->act_min, e->act_rng, raw);
            else memcpy(raw, a, 4 * (size_t)Da);
            for (int j = 0; j < Da; ++j) act[(size_t)n * Da + j] = (double)raw[j];
            ++n;
        }
        if (n == 0) break;
        if (e->step(e->ctx, n, idx, act, obs, rew, done, tl)) return -1;
        for (int r = 0; r < n; ++r) {
            const int i = idx[r];
            hist_put(e, i, obs + (size_t)r * Do, 0);
            c->reward[i] += rew[r];                                /* reward_agg_method = "sum" */
            if (tl[r] < 0) {                                       /* no "TimeLimit.truncated" in info */
                if (done[r]) fl[i].term = 1;
                else if (e->max_episode_steps > 0 && e->cnt[i] >= e->max_episode_steps) fl[i].trunc = 1;
            } else {
                fl[i].trunc = (uint8_t)(tl[r] != 0);
                fl[i].term = done[r] ? 1 : 0;
            }
            fl[i].last_done = fl[i].term || fl[i].trunc;          /* self.done[-1] */
        }
    }
    /* the returned observation, then reset within the step where the chunk ended (:172-187) */
    int n_done = 0, nr = 0;
    for (int i = lo; i < hi; ++i) {
        c->terminated[i] = fl[i].term;
        c->truncated[i] = fl[i].trunc;
        hist_out(e, i, c->obs_out);
        if (fl[i].last_done) {
            ++n_done;
            if (e->reset_within_step) {
                if (fl[i].trunc && c->final_obs) {
                    memcpy(c->final_obs + (size_t)i * To * Do, c->obs_out + (size_t)i * To * Do, 4 * (size_t)To * Do);
                    c->has_final[i] = 1;
                }
                idx[nr++] = i;
            }
        }
    }
    if (nr) {
        if (reset_envs(e, nr, idx, obs)) return -1;
        for (int r = 0; r < nr; ++r) hist_out(e, idx[r], c->obs_out);
    }
    if (c->obs_tagged) {   /* publish this slice's observation granules (one aligned 8-byte store each) */
        const uint64_t hi_tag = (uint64_t)c->obs_tag << 32;
        const int64_t per = (int64_t)To * Do;
        for (int64_t q = lo * per; q < hi * per; ++q) {
            uint32_t bits;
            memcpy(&bits, c->obs_out + q, 4);
            __atomic_store_n(c->obs_tagged + q, hi_tag | bits, __ATOMIC_RELEASE);
        }
    }
    if (t == 0) e->work0_s += mono_s() - w0;
    return n_done;
}

/* A slice goes in blocks of ENV_GROUP envs, the split sampler's env group (each group of a
 * pre-enqueued launch polls only its own envs' observation granules): block by block the slice
 * waits for the block's actions, steps it and publishes it, so the device's first groups start
 * while the host still steps later blocks. Envs are independent (per-env seeded resets), so the
 * blocking changes no value. */
#define ENV_GROUP 16
static int run_slice(LowdimEnv* e, int t, int lo, int hi) {
    int n_done = 0;
    for (int b = lo; b < hi; b += ENV_GROUP) {
        const int rc = run_block(e, t, b, b + ENV_GROUP < hi ? b + ENV_GROUP : hi);
        if (rc < 0) return rc;
        n_done += rc;
    }
    return n_done;
}

/* AsyncVectorEnv.reset_arg -> MultiStep.reset for every env; obs_out [E][To][Do] float32 */
DPPO_ENV_API int dppo_lowdim_reset_all(void* h, float* obs_out) {
    LowdimEnv* e = (LowdimEnv*)h;
    for (int i = 0; i < e->E; ++i) e->scr[0].idx[i] = i;
    if (reset_envs(e, e->E, e->scr[0].idx, e->scr[0].obs)) return -1;
    for (int i = 0; i < e->E; ++i) hist_out(e, i, obs_out);
    return 0;
}

DPPO_ENV_API int dppo_lowdim_reset_one(void* h, int env, float* obs_out) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (env < 0 || env >= e->E) return -1;
    int32_t one = env;
    if (reset_envs(e, 1, &one, e->scr[0].obs)) return -1;
    hist_out(e, env, obs_out);
    return 0;
}

static void set_chunk(LowdimEnv* e, float* actions, int Ta, double* reward, uint8_t* terminated, uint8_t* truncated,
                      float* obs_out, float* final_obs, uint8_t* has_final) {
    Chunk* c = &e->chunk;
    memset(c, 0, sizeof(*c));
    c->actions = actions; c->Ta = Ta; c->reward = reward; c->terminated = terminated; c->truncated = truncated;
    c->obs_out = obs_out; c->final_obs = final_obs; c->has_final = final_obs ? has_final : NULL;
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
    if (Ta < 1) return -1;
    set_chunk(e, (float*)actions, Ta, reward, terminated, truncated, obs_out, final_obs, has_final);
    return run_chunk(e);
}

/* dppo_lowdim_step as the pipelined rollout's host step with the tagged protocol both ways
 * (the wrapper-stack counterpart of dppo_env_step_gated_tagged, csrc/envstep.c): every slice
 * thread spins until its envs' action granules act_tagged [E][Ta][Da] carry act_tag (the device's
 * stores are the ready flag; bit 31 of *done reports a device-side timeout), decodes them into
 * `actions`, steps its envs, and — when obs_tagged is not NULL — publishes its envs' observation
 * granules {tag : 32, fp32 bits : 32} of obs_out. The in-wrapper reset is already applied to
 * obs_out, so the observation is always publishable. Returns n_done (| DPPO_ENV_PUBLISHED when
 * published), -1 simulator error or host timeout, -2 the device flagged its own wait timed out. */
DPPO_ENV_API int dppo_lowdim_step_gated_tagged(void* h, float* actions, int Ta, double* reward, uint8_t* terminated,
                                               uint8_t* truncated, float* obs_out, float* final_obs,
                                               uint8_t* has_final, const volatile uint32_t* done,
                                               const uint64_t* act_tagged, uint32_t act_tag, uint64_t* obs_tagged,
                                               uint32_t tag, double timeout_s) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (Ta < 1 || !done || !act_tagged) return -1;
    set_chunk(e, actions, Ta, reward, terminated, truncated, obs_out, final_obs, has_final);
    Chunk* c = &e->chunk;
    c->done = done; c->act_tagged = act_tagged; c->act_tag = act_tag;
    c->obs_tagged = obs_tagged; c->obs_tag = tag;
    c->deadline = mono_s() + timeout_s;
    const int rc = run_chunk(e);
    if (rc < 0) return rc;
    return obs_tagged ? (rc | DPPO_ENV_PUBLISHED) : rc;
}

/* The "go" protocol (dppo_rollout_enqueue): spin until *done >= done_target, step, then store
 * go_value to *go (go NULL: no publish). Same returns as the tagged entry. */
DPPO_ENV_API int dppo_lowdim_step_gated(void* h, float* actions, int Ta, double* reward, uint8_t* terminated,
                                        uint8_t* truncated, float* obs_out, float* final_obs, uint8_t* has_final,
                                        const volatile uint32_t* done, uint32_t done_target, volatile uint32_t* go,
                                        uint32_t go_value, double timeout_s) {
    LowdimEnv* e = (LowdimEnv*)h;
    if (Ta < 1 || !done) return -1;
    const double deadline = mono_s() + timeout_s;
    for (uint32_t spins = 0;; ++spins) {
        const uint32_t v = __atomic_load_n(done, __ATOMIC_ACQUIRE);
        if (v & 0x80000000u) return -2;
        if (v >= done_target) break;
        _mm_pause();
        if ((spins & 1023u) == 1023u && mono_s() > deadline) return -1;
    }
    set_chunk(e, actions, Ta, reward, terminated, truncated, obs_out, final_obs, has_final);
    const int rc = run_chunk(e);
    if (rc < 0) return rc;
    if (go) {
        __atomic_store_n(go, go_value, __ATOMIC_RELEASE);   /* x86: the obs stores are visible first */
        return rc | DPPO_ENV_PUBLISHED;
    }
    return rc;
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
    double *A, *AT, *B, *c, *goal, *center, *scale, *bound;   /* A [Do][Do] row-major, AT = A^T, B [Da][Do] */
    double* s;          /* [E][Do] */
    int64_t *seed, *episode;
    double cost_s;      /* emulated extra work per env sub-step (0: none), dppo_sim_linear_set_cost */
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
    m->AT = (double*)xcalloc((size_t)Do * Do, 8);
    for (int j = 0; j < Do; ++j)
        for (int q = 0; q < Do; ++q) m->AT[(size_t)q * Do + j] = A[(size_t)j * Do + q];
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

/* Measurement knob: busy-wait cost_us per env sub-step inside step, standing in for the work of a
 * physics step (a MuJoCo locomotion step with frame_skip is tens of microseconds on one core), so
 * the pool's fan-out can be measured without a simulator; 0 (the default) turns it off. */
DPPO_ENV_API void dppo_sim_linear_set_cost(void* p, double cost_us) {
    ((LinearSim*)p)->cost_s = cost_us > 0 ? cost_us * 1e-6 : 0.0;
}

DPPO_ENV_API void dppo_sim_linear_destroy(void* p) {
    LinearSim* m = (LinearSim*)p;
    if (!m) return;
    free(m->A); free(m->AT); free(m->B); free(m->c); free(m->goal); free(m->center); free(m->scale); free(m->bound); free(m->s);
    free(m->seed); free(m->episode); free(m);
}

/* Blocks of up to SIM_RB rows are stepped structure-of-arrays (coordinate-major scratch on the stack,
 * so concurrent slices share nothing), with every row's sum still taken term by term in the oracle's
 * order: sn[j] = c[j] + sum_q A[j][q] s[q] + sum_q B[q][j] a[q] (q ascending), err and |a|^2 likewise.
 * The loops over the block's rows are innermost, so they vectorise across envs without reassociating
 * any row's arithmetic (the results are bit-identical to one row at a time). */
#define SIM_RB 32
DPPO_ENV_API int dppo_sim_linear_step(void* ctx, int n, const int32_t* idx, const double* act, double* obs,
                                      double* reward, uint8_t* done, int8_t* time_limit) {
    LinearSim* m = (LinearSim*)ctx;
    const int Do = m->Do, Da = m->Da;
    if (Do > 64 || Da > 64) return 1;
    double xs[64 * SIM_RB], xn[64 * SIM_RB], xa[64 * SIM_RB], err[SIM_RB], asq[SIM_RB];
    int out[SIM_RB];
    for (int r0 = 0; r0 < n; r0 += SIM_RB) {
        const int nb = n - r0 < SIM_RB ? n - r0 : SIM_RB;
        for (int r = 0; r < nb; ++r) {
            const double* s = m->s + (size_t)idx[r0 + r] * Do;
            for (int q = 0; q < Do; ++q) xs[q * SIM_RB + r] = s[q];
            for (int q = 0; q < Da; ++q) xa[q * SIM_RB + r] = act[(size_t)(r0 + r) * Da + q];
            err[r] = 0.0; asq[r] = 0.0; out[r] = 0;
        }
        for (int j = 0; j < Do; ++j) {
            double* o = xn + j * SIM_RB;
            const double cj = m->c[j];
            for (int r = 0; r < nb; ++r) o[r] = cj;
            for (int q = 0; q < Do; ++q) {
                const double aj = m->A[(size_t)j * Do + q];
                const double* x = xs + q * SIM_RB;
                for (int r = 0; r < nb; ++r) o[r] += aj * x[r];
            }
            for (int q = 0; q < Da; ++q) {
                const double bj = m->B[(size_t)q * Do + j];
                const double* x = xa + q * SIM_RB;
                for (int r = 0; r < nb; ++r) o[r] += bj * x[r];
            }
            const double gj = m->goal[j], cen = m->center[j], bd = m->bound[j];
            for (int r = 0; r < nb; ++r) {
                const double d = o[r] - gj;
                err[r] += d * d;
                const double dc = o[r] - cen;
                out[r] |= dc > bd || dc < -bd;
            }
        }
        for (int q = 0; q < Da; ++q) {
            const double* x = xa + q * SIM_RB;
            for (int r = 0; r < nb; ++r) asq[r] += x[r] * x[r];
        }
        for (int r = 0; r < nb; ++r) {
            double* s = m->s + (size_t)idx[r0 + r] * Do;
            double* ob = obs + (size_t)(r0 + r) * Do;
            for (int j = 0; j < Do; ++j) s[j] = ob[j] = xn[j * SIM_RB + r];
            reward[r0 + r] = 1.0 - err[r] / Do - 1e-3 * asq[r];
            done[r0 + r] = (uint8_t)out[r];
            time_limit[r0 + r] = -1;
        }
        if (m->cost_s > 0)
            for (int r = 0; r < nb; ++r) {
                const double t_end = mono_s() + m->cost_s;
                while (mono_s() < t_end) _mm_pause();
            }
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
