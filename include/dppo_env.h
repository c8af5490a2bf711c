/* dppo_env.h — C ABI of libdppo_env.so, the host side of the rollout: the reference's gym
 * locomotion env stack batched in C and stepped by a pool of host threads, the synthetic bench
 * stepper, and the host half of the pipelined (gated) rollout protocol of include/dppo.h.
 *
 * Plain C, host memory only (no HIP types): arrays are caller-owned, row-major, float32 actions /
 * observations and float64 rewards as the reference's wrappers produce them. "Mapped" buffers
 * (done, act_tagged, obs_tagged, go) are the dppo_host_alloc memory the sampler launches of
 * dppo_rollout_enqueue_tagged / dppo_rollout_enqueue read and write.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   AsyncVectorEnv.step / reset_arg      env/gym_utils/async_vector_env.py:356-456 (workers :774-840)
 *   MultiStep.step / reset               env/gym_utils/wrapper/multi_step.py:113-192
 *   MujocoLocomotionLowdimWrapper        env/gym_utils/wrapper/mujoco_locomotion_lowdim.py:39-70
 *   VectorEnv.seed                       agent/finetune/train_agent.py:53-56
 * ctypes binding: diffusionpolicyoptimization_amd/env/lowdim.py and env/synthetic.py; a cgo-style
 * stub is in INTEGRATION.md. */
#ifndef DPPO_ENV_H
#define DPPO_ENV_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPPO_ENV_PUBLISHED (1 << 30)   /* OR'd into a gated step's return when the observation went out */

/* ---- the simulator callback table (the reference's gym / mujoco_py env behind MultiStep) ----
 * Raw (unnormalised) coordinates, one batched call per sub-step for the n env indices idx[0..n)
 * (ascending); rows of act / obs / reward / done / time_limit are in idx order.
 *   step:  act [n][Da] float64 -> obs [n][Do], reward [n], done [n] (gym's done),
 *          time_limit [n] (info["TimeLimit.truncated"]: -1 absent, else 0 / 1)
 *   reset: obs [n][Do]
 * Return 0, or nonzero to abort the chunk. With a pool of more than one thread the callbacks run
 * concurrently on disjoint env sets: the simulator must keep per-env state only. */
typedef int (*dppo_sim_step_fn)(void* ctx, int n, const int32_t* idx, const double* act, double* obs,
                                double* reward, uint8_t* done, int8_t* time_limit);
typedef int (*dppo_sim_reset_fn)(void* ctx, int n, const int32_t* idx, double* obs);

/* ---- the wrapper stack (csrc/envwrap.c) ---- */
int dppo_lowdim_abi(void);   /* 2 */

/* mujoco_locomotion_lowdim.py:57-58 / :60-62, bit-exact with NumPy on the reference's dtypes */
void dppo_lowdim_normalize_obs(int64_t n, int Do, const double* raw, const float* obs_min, const float* obs_max,
                               double* out);
void dppo_lowdim_unnormalize_action(int64_t n, int Da, const float* a, const float* act_min, const float* act_max,
                                    float* out);

/* One MultiStep(MujocoLocomotionLowdimWrapper(sim)) per env for E envs; max_episode_steps <= 0 =
 * None; obs_min/obs_max [Do], act_min/act_max [Da] (normalization.npz, float32) or NULL for
 * identity maps. NULL on invalid shapes. Starts with one thread. */
void* dppo_lowdim_create(int E, int Do, int Da, int To, int act_steps, int max_episode_steps, int reset_within_step,
                         dppo_sim_step_fn step, dppo_sim_reset_fn reset, void* ctx, const float* obs_min,
                         const float* obs_max, const float* act_min, const float* act_max);
void dppo_lowdim_destroy(void* h);

/* Host threads stepping the envs, the caller's included (contiguous env slices, one per thread; the
 * reference's one process per env): n clamped to [1, E]; idle pool threads spin spin_us (<= 0:
 * 2000) before they sleep. Outputs are bit-identical for any n. Returns the count in use, or -1. */
int dppo_lowdim_set_threads(void* h, int n, double spin_us);
int dppo_lowdim_threads(void* h);

/* The solo floor: with n > 1 threads, a chunk whose estimated stepping work (a running average of
 * the measured simulator + wrapper time, waits for actions excluded, scaled to all envs) is below
 * floor_us runs on the caller's thread alone, since the pool's hand-off would cost more than it
 * saves; the pool is used again once the estimate exceeds twice the floor. 0 disables; the default
 * is 25 us. Outputs do not depend on it. 0 or -1. _solo_chunks: chunks stepped alone so far. */
int dppo_lowdim_set_solo_floor(void* h, double floor_us);
int64_t dppo_lowdim_solo_chunks(void* h);

/* AsyncVectorEnv.reset_arg / reset_one_arg: obs_out [E][To][Do] float32. 0 or -1 (simulator error) */
int dppo_lowdim_reset_all(void* h, float* obs_out);
int dppo_lowdim_reset_one(void* h, int env, float* obs_out);

/* One action chunk for every env: actions [E][Ta][Da]; reward [E] (sum), terminated / truncated [E],
 * obs_out [E][To][Do] (after the in-wrapper reset where a chunk ended), final_obs [E][To][Do] +
 * has_final [E] (info["final_obs"]; final_obs may be NULL). Returns the number of envs whose chunk
 * ended, or -1 on a simulator error. */
int dppo_lowdim_step(void* h, const float* actions, int Ta, double* reward, uint8_t* terminated, uint8_t* truncated,
                     float* obs_out, float* final_obs, uint8_t* has_final);

/* The pipelined rollout's host step (tagged protocol both ways): each slice thread spins until its
 * envs' granules of act_tagged [E][Ta][Da] carry act_tag, decodes them into actions, steps, and
 * publishes its envs' observation granules {tag, fp32 bits} into obs_tagged [E][To][Do] (NULL: no
 * publish). Returns n_done | DPPO_ENV_PUBLISHED, -1 (simulator error or timeout_s passed), -2 (bit
 * 31 of *done: the device's own wait timed out). */
int dppo_lowdim_step_gated_tagged(void* h, float* actions, int Ta, double* reward, uint8_t* terminated,
                                  uint8_t* truncated, float* obs_out, float* final_obs, uint8_t* has_final,
                                  const volatile uint32_t* done, const uint64_t* act_tagged, uint32_t act_tag,
                                  uint64_t* obs_tagged, uint32_t tag, double timeout_s);
/* The go-counter protocol: spin until *done >= done_target, step, store go_value to *go (NULL: none). */
int dppo_lowdim_step_gated(void* h, float* actions, int Ta, double* reward, uint8_t* terminated, uint8_t* truncated,
                           float* obs_out, float* final_obs, uint8_t* has_final, const volatile uint32_t* done,
                           uint32_t done_target, volatile uint32_t* go, uint32_t go_value, double timeout_s);

/* MultiStep.cnt of every env ([E], owned by the handle) */
const int64_t* dppo_lowdim_counters(void* h);

/* ---- the C reference simulator (seeded linear dynamics in raw coordinates, terminal set) ---- */
void* dppo_sim_linear_create(int E, int Do, int Da, const double* A, const double* B, const double* c,
                             const double* goal, const double* center, const double* scale, const double* bound,
                             const int64_t* seeds);
void dppo_sim_linear_seed(void* sim, const int64_t* seeds);
void dppo_sim_linear_set_cost(void* sim, double cost_us);   /* measurement: busy work per env sub-step */
void dppo_sim_linear_destroy(void* sim);
/* the C linear simulator's dimensions: obs_dim <= 64 and action_dim <= 64 (dppo_sim_linear_step returns 1
 * past them); the wrapper stack itself takes action_dim <= 64 and any obs_dim */
int dppo_sim_linear_step(void* ctx, int n, const int32_t* idx, const double* act, double* obs, double* reward,
                         uint8_t* done, int8_t* time_limit);
int dppo_sim_linear_reset(void* ctx, int n, const int32_t* idx, double* obs);
void* dppo_sim_linear_step_fn(void);    /* &dppo_sim_linear_step, for bindings that fill the table */
void* dppo_sim_linear_reset_fn(void);

/* ---- the synthetic bench env stepper (csrc/envstep.c; env/synthetic.py is its spec) ---- */
int dppo_env_abi(void);   /* 3 */
int dppo_env_step(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps, const double* AT,
                  const double* B, const double* c, const double* goal, double* state, int64_t* cnt,
                  const float* actions, double* reward, uint8_t* terminated, uint8_t* truncated, float* obs_out);
int dppo_env_step_gated(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                        const double* AT, const double* B, const double* c, const double* goal, double* state,
                        int64_t* cnt, const float* actions, double* reward, uint8_t* terminated, uint8_t* truncated,
                        float* obs_out, const volatile uint32_t* done, uint32_t done_target, volatile uint32_t* go,
                        uint32_t go_value, double timeout_s);
int dppo_env_step_gated_tagged(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
                               const double* AT, const double* B, const double* c, const double* goal, double* state,
                               int64_t* cnt, float* actions, double* reward, uint8_t* terminated, uint8_t* truncated,
                               float* obs_out, const volatile uint32_t* done, const uint64_t* act_tagged,
                               uint32_t act_tag, uint64_t* obs_tagged, uint32_t tag, double timeout_s);
void dppo_env_publish_tagged(int64_t count, const float* obs, uint64_t* obs_tagged, uint32_t tag);

#ifdef __cplusplus
}
#endif
#endif
