/*
 * dppo.h — C ABI of libdppo_hip.so, the MI355X (gfx950) DPPO fine-tuning hot path.
 *
 * The TF reference has no native boundary: its hot path is TF/Keras/TFP ops called from Python.
 * Each entry point below replaces one reference interface (cited file:line, relative to the
 * reference repo root); the Python layer diffusionpolicyoptimization_amd/ (same class names and
 * kwargs as the reference) is the drop-in, and it binds these symbols with ctypes
 * (diffusionpolicyoptimization_amd/_lib.py). INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every pointer argument is DEVICE memory owned by the caller unless it says "host";
 *   - every call is asynchronous on `stream` (a hipStream_t; 0 = null stream) and allocates
 *     nothing; scratch comes from a caller-owned workspace sized by the *_workspace_bytes query;
 *   - return 0 on success, a DPPO_E* code otherwise; dppo_last_error() gives the message
 *     (thread-local); no C++ exception crosses the ABI;
 *   - precision: DPPO_F32 = f32-input MFMA (exact fp32 products, the parity mode),
 *     DPPO_BF16 = bf16 MFMA with fp32 accumulation and an fp32 DDPM/loss epilogue, or
 *     DPPO_F16 = the same with fp16 operands (BASELINE config 5; the backward images carry the
 *     gradient times 4096 for fp16's range, removed exactly in the fp32 weight gradients);
 *   - flat parameter layout (fp32, Keras kernel [in,out] row-major, then bias [out]):
 *       actor : time_w1[TD,2TD] time_b1[2TD] time_w2[2TD,TD] time_b2[TD]
 *               in_w[XD+TD+SD, H] in_b[H] l1_w[H,H] l1_b[H] l2_w[H,H] l2_b[H] out_w[H,XD] out_b[XD]
 *       critic: in_w[SD,HC] in_b[HC] l1_w[HC,HC] l1_b[HC] l2_w[HC,HC] l2_b[HC] out_w[HC,1] out_b[1]
 *     with XD = horizon*action_dim, SD = cond_steps*obs_dim, TD = time_dim.
 */
#ifndef DPPO_H
#define DPPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 13: the actor image (dppo_actor_packed_bytes) holds the row tiles' l2 fold segments; a pack or
 * fused step of an actor image is followed by the fold launch (DPPO_STEP_FUSED_PACK above).
 * ABI 15: dppo_actor_step and DPPO_PPO_TIME_BWD_IN_STEP (ABI 12) are removed: the one-launch actor
 * tail was measured slower than the minibatch's time-MLP backward + the fused step;
 * the actor's one-launch step is dppo_optimizer_step_ex | DPPO_STEP_FUSED_PACK over its range. */
#define DPPO_ABI_VERSION 15

#if defined(__GNUC__)
#define DPPO_API __attribute__((visibility("default")))
#else
#define DPPO_API
#endif

enum { DPPO_OK = 0, DPPO_EINVAL = 1, DPPO_EHIP = 2, DPPO_EUNSUPPORTED = 3 };
enum { DPPO_F32 = 0, DPPO_BF16 = 1, DPPO_F16 = 2 };
enum { DPPO_ADAMW_KERAS = 0, DPPO_ADAMW_TORCH = 1 };
/* ABI 7: OR'd into dppo_optimizer_step's mode. The actor image is packed without the split
 * sampler's tables (W_XS, FOLD/ROUT, TIN, B_OUT2: nothing the PPO row tiles read) and marked stale;
 * the next sampler launch on that image (dppo_sample, dppo_sample_step, dppo_rollout_enqueue*)
 * re-derives them on its own stream first, or dppo_refresh_sampler_tables does it explicitly. The
 * actor parameters must stay allocated and unchanged until then (they are read at the refresh). */
enum { DPPO_STEP_DEFER_SAMPLER_TABLES = 0x100 };
/* ABI 8, OR'd into dppo_optimizer_step's mode: the actor's l2 gradient in grads is in the factored
 * form of DPPO_PPO_L2_DEFERRED; AdamW forms it from pl2, db_out and the actor image's rnd(W_out)
 * (needs actor_params == params and packed_actor). */
enum { DPPO_STEP_L2_FROM_PL2 = 0x200 };
/* ABI 11, OR'd into dppo_optimizer_step's mode. DPPO_STEP_FUSED_PACK: AdamW and the pack in ONE
 * launch when the step packs a single network whose flat parameters are exactly the range: each
 * element's thread stores its updated value into its slots of the images (the values the pack writes).
 * For an actor the launch leaves the split sampler's tables to the next sampler launch (or
 * dppo_refresh_sampler_tables), as after DPPO_STEP_DEFER_SAMPLER_TABLES; a second, small launch on the
 * same stream re-derives the cross-element segments the row tiles read (the l2 fold M = W_l2 W_out,
 * M0 = W_in W_out, the folded out bias and the TEMB table), as it does after every pack of an actor
 * image. The image must have been fully packed once before (its zero padding is not rewritten). Any
 * other combination runs the two launches.
 * DPPO_STEP_CLEAR_GRADS (dppo_optimizer_step_ex only): the step zeroes the range's gradients after
 * reading them, and the byte ranges given to dppo_optimizer_step_ex after every read of the launch
 * (by its last workgroup), so the next minibatch of this range may skip its zeroing launch
 * (DPPO_PPO_PRECLEARED). */
enum { DPPO_STEP_FUSED_PACK = 0x400, DPPO_STEP_CLEAR_GRADS = 0x800 };

/* Model / schedule dimensions (cfg keys of cfg/gym/finetune/hopper-v2/ft_ppo_diffusion_mlp.yaml:18-25,78-110). */
typedef struct dppo_dims {
    int32_t obs_dim;          /* Do */
    int32_t action_dim;       /* Da */
    int32_t horizon_steps;    /* Ta */
    int32_t cond_steps;       /* To */
    int32_t time_dim;         /* TD (16) */
    int32_t actor_hidden;     /* H  (512), multiple of 128 */
    int32_t critic_hidden;    /* HC (256), multiple of 128 */
    int32_t denoising_steps;  /* sampling steps: K (20) for DDPM, ddim_steps S (10) for DDIM */
    int32_t ft_denoising_steps; /* K' (10) */
    int32_t time_stride;      /* diffusion time of sampling row r = r * time_stride: 1 (or 0) for DDPM,
                                 K / S for DDIM (diffusion.py:76-82 uniform discretisation); since ABI 2 */
} dppo_dims;

/* Schedule table, one fp32 row per sampling row r (r = t for DDPM; the DDIM sub-sequence index for
 * DDIM): {c0, c1, c2, c3, logvar, eval_floor, eval_zero, 0} with
 *   x0 = clip(c0 x - c1 eps, -1, 1);  mu = c2 x0 + c3 x;  sigma = exp(logvar / 2)
 * and the eval-mode (deterministic) noise rule sigma = eval_zero ? 0 : clip(sigma, eval_floor, 1e6).
 *   DDPM (model/diffusion/diffusion.py:57-73, diffusion_vpg.py:198-243, 303-315): c0 = sqrt(1/abar_t),
 *     c1 = sqrt(1/abar_t - 1), c2 = mu_coef1, c3 = mu_coef2, logvar = logvar_clipped; eval_floor
 *     1e-3, eval_zero = (t == 0).
 *   DDIM (diffusion.py:76-96, diffusion_vpg.py:184-234, the documented formulas): with abar, abar_prev
 *     of the sub-sequence and eps' = (x - sqrt(abar) x0) / sqrt(1 - abar) after the clip,
 *     mu = sqrt(abar_prev) x0 + d eps', d = sqrt(max(1 - abar_prev - sigma^2, 0)), which is the same
 *     affine form: c2 = sqrt(abar_prev) - d sqrt(abar) / sqrt(1 - abar), c3 = d / sqrt(1 - abar);
 *     c0 = 1 / sqrt(abar), c1 = sqrt(1/abar - 1); logvar = log(sigma^2), sigma = max(eta sqrt((1 - abar_prev)
 *     / (1 - abar) (1 - abar / abar_prev)), 1e-10); eval_floor 0, eval_zero 1; column 7 = s =
 *     sqrt((1 - abar_prev) / (1 - abar) (1 - abar / abar_prev)) (sigma / eta: read only by the
 *     learnable-eta gradient, DPPO_PPO_LEARN_ETA; ABI 9; 0 for DDPM rows). */
#define DPPO_SCHED_COLS 8

DPPO_API int         dppo_abi_version(void);
DPPO_API const char* dppo_last_error(void);

/* ---- parameter packing (replaces Keras variable storage; model/common/mlp.py:95-206) ---- */
DPPO_API size_t dppo_actor_param_count(const dppo_dims* d);
DPPO_API size_t dppo_critic_param_count(const dppo_dims* d);
/* bytes of the packed (MFMA fragment-ordered) device image of one actor / critic */
DPPO_API size_t dppo_actor_packed_bytes(const dppo_dims* d, int precision);
DPPO_API size_t dppo_critic_packed_bytes(const dppo_dims* d, int precision);
/* params: flat fp32 (layout above) -> packed image (forward + transposed fragments) */
DPPO_API int dppo_pack_actor(const dppo_dims* d, int precision, const float* params, void* packed, void* stream);
DPPO_API int dppo_pack_critic(const dppo_dims* d, int precision, const float* params, void* packed, void* stream);

/* ---- a9: diffusion-policy action sampler, VPGDiffusion.call (model/diffusion/diffusion_vpg.py:250-339) ----
 * All K DDPM steps for n_envs rows in ONE launch: DiffusionMLP forward on MFMA + fused DDPM
 * reparameterisation epilogue (diffusion_vpg.py:152-245, 301-320).
 *   cond     [n_envs, To*Do]
 *   x_T      [n_envs, Ta*Da] or NULL -> in-kernel Philox (seed, call_id) stream
 *   noise    [K, n_envs, Ta*Da] raw N(0,1) draws for loop index i (t = K-1-i), or NULL -> Philox
 *   env_offset: global row index of row 0 (Philox counter; multi-GPU shards stay distinct)
 *   final_clip <= 0 means None (cfg default)
 *   actions  [n_envs, Ta*Da]                 (Sample.trajectories)
 *   chains   [n_envs, K'+1, Ta*Da] or NULL   (Sample.chains)                                 */
DPPO_API int dppo_sample(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                const float* sched, const float* cond, int n_envs, const float* x_T, const float* noise,
                uint64_t seed, uint64_t call_id, int env_offset, int deterministic,
                float min_sampling_std, float randn_clip, float final_clip,
                float* actions, float* chains, void* stream);

/* Measurement aid (no reference counterpart): bytes of weight fragments one 16-env sampler tile
 * (one CU) loads per dppo_sample launch with the sampler geometry in use — every denoising step's
 * streamed k-steps plus the resident set, loaded once per actor. bench.py divides it by the launch
 * time for the per-CU load-path figure. Also returns the waves per workgroup. */
DPPO_API int dppo_sampler_stream_bytes(const dppo_dims* d, int precision, int64_t* bytes_per_tile, int* waves);

/* Which sampler layout dppo_sample runs for n_envs envs: *members = 0 for the weight-streaming
 * kernel (one workgroup per 16-env tile), or P > 0 for the split register-resident kernel (P
 * workgroups per 16-env tile, one in-launch partial-sum exchange per denoising step; bf16,
 * actor_hidden 512, horizon*action_dim a multiple of 4, <= 512 envs). The split kernel keeps one
 * 2 MiB exchange buffer per stream, allocated by the library on the first launch on that stream
 * (the one allocation outside a caller workspace). */
DPPO_API int dppo_sampler_layout(const dppo_dims* d, int precision, int n_envs, int* members);

/* How many dppo_sample / dppo_rollout_enqueue* launches of n_envs envs may be in flight at once on
 * the current device (on different streams) without one launch taking CUs another's split-kernel
 * members wait for: floor(CUs / active workgroups) for the split kernel (>= 1), 8 for the
 * weight-streaming kernel. The pipelined rollout (ops.RolloutPipe) uses at most this many streams. */
DPPO_API int dppo_sampler_max_in_flight(const dppo_dims* d, int precision, int n_envs, int* launches);

/* ABI 10: the caller is done sampling on `stream` (a closed rollout pipe): waits for the stream's
 * pending work, then unbinds the exchange buffer the split kernel keeps for it, so a later stream
 * reuses that buffer instead of a new allocation. Slots are also rebound, without a device-wide
 * synchronisation, when more than 16 streams sample. (No reference counterpart: the reference's
 * sampler is a TF call, diffusion_vpg.py:250-339.) */
/* A stream that sampled must be released before its owner destroys it (ops.RolloutPipe.close does);
 * a slot whose stream no longer answers hipStreamQuery is treated as released. */
DPPO_API int dppo_sampler_release_stream(void* stream);

/* Kernel timer (ABI 10, measurement): while enabled, the library brackets the launches of its
 * timed kernels (the sampler, the row tiles, dW, l2_back, time_bwd, AdamW, pack, GAE, the reward
 * scaler's three kernels, ...; dppo_kernel_timing_name(id) names id, NULL past the last) with HIP
 * events on the launch's own stream. dppo_kernel_timing(enable) switches it and clears the window;
 * dppo_kernel_timing_read(n, total_ms[n], launches[n]) waits for the window's launches, returns the
 * summed event time and launch count per id, and clears the window. Off by default: a disabled timer
 * is one flag test per launch. */
DPPO_API int dppo_kernel_timing(int enable);
DPPO_API const char* dppo_kernel_timing_name(int id);
DPPO_API int dppo_kernel_timing_read(int n, double* total_ms, int64_t* launches);

/* The sampler plan for n_envs envs (measurement aid, ABI 6): plan[0] = kernel (0 weight streaming,
 * 1 split with 8 members per 16-env tile, 2 folded split with P members per tile, 3 the pair kernel:
 * P = 2 members running two 16-env tiles half a denoising step apart), plan[1] = members per member
 * set, plan[2] = member sets (2: the base actor's and the fine-tuned actor's steps on separate
 * workgroups), plan[3] = workgroups per launch. */
DPPO_API int dppo_sampler_plan(const dppo_dims* d, int precision, int n_envs, int* plan);

/* One rollout step (agent/finetune/train_ppo_diffusion_agent.py:106-122) in one call:
 * hipMemcpyAsync(cond <- cond_host [host, pinned]), dppo_sample with the Philox noise, hipMemcpyAsync
 * (actions_host [host, pinned] <- actions), then hipStreamSynchronize when synchronize != 0. */
DPPO_API int dppo_sample_step(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                const float* sched, const float* cond_host, float* cond, int n_envs, uint64_t seed,
                uint64_t call_id, int env_offset, int deterministic, float min_sampling_std,
                float randn_clip, float final_clip, float* actions, float* actions_host,
                float* chains, int synchronize, void* stream);

/* Pipelined rollout (the same step, with the launch taken off the host's critical path):
 * the host enqueues step t+1 BEFORE stepping the envs of step t; that launch does everything
 * that does not depend on the observation (noise, time embedding, weights in flight), then waits
 * until *go >= go_value, reads the observation from cond_host, and after writing the actions to
 * actions_host adds 1 per workgroup (ceil(n_envs/16)) to *done. cond_host, actions_host, go and
 * done must come from dppo_host_alloc (mapped, coherent pinned memory). The wait is bounded
 * (~4 s): on timeout the step proceeds and sets bit 31 of *done. */
DPPO_API int dppo_host_alloc(size_t bytes, void** ptr);
DPPO_API int dppo_host_free(void* ptr);
/* ABI 9: n <= 4 copies src_host[i] (dppo_host_alloc memory) -> dst[i] (device), bytes[i] each, in ONE
 * kernel launch on stream that reads the mapped memory over the bus (no copy engine): the rollout's
 * per-step rewards and flags into the update's device buffers (agent :232-263). */
DPPO_API int dppo_copy_from_host(int n, void* const* dst, const void* const* src_host, const size_t* bytes,
                                 void* stream);
DPPO_API int dppo_rollout_enqueue(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                const float* sched, const float* cond_host, float* cond, int n_envs, uint64_t seed,
                uint64_t call_id, int env_offset, int deterministic, float min_sampling_std,
                float randn_clip, float final_clip, float* actions, float* actions_host,
                float* chains, const uint32_t* go, uint32_t go_value, uint32_t* done, void* stream);

/* The same pipelined step with a TAGGED observation (ABI 2): no go counter; the host writes each
 * observation value as an 8-byte granule {tag in the high 32 bits, fp32 bits in the low 32} into
 * obs_tagged ([n_envs][To*Do] uint64, from dppo_host_alloc), and the launch polls its envs'
 * granules until every tag equals `tag` (nonzero, unique among the tags the buffer may hold, e.g.
 * the step count). The observation carries its own ready flag: one PCIe round trip instead of a
 * flag poll followed by a read. The actions come back the same way: actions_tagged ([n_envs][Ta*Da]
 * uint64, from dppo_host_alloc) receives {tag, fp32} granules, so the host can poll the actions
 * themselves instead of waiting for *done (which still counts finished workgroups, and bit 31 still
 * flags a timeout). cond receives the device copy of the observation. */
DPPO_API int dppo_rollout_enqueue_tagged(const dppo_dims* d, int precision, const void* packed_base,
                const void* packed_ft, const float* sched, const uint64_t* obs_tagged, float* cond,
                int n_envs, uint64_t seed, uint64_t call_id, int env_offset, int deterministic,
                float min_sampling_std, float randn_clip, float final_clip, float* actions,
                uint64_t* actions_tagged, float* chains, uint32_t tag, uint32_t* done, void* stream);

/* ---- a10: VPGDiffusion.get_logprobs (diffusion_vpg.py:343-425) + the clip/mean of c_loss
 * (diffusion_ppo.py:50-59) for the old-logprob pass (agent/finetune/train_ppo_diffusion_agent.py:214-229).
 *   cond [n, To*Do], chains [n, K'+1, Ta*Da]
 *   lp_elem [n*K', Ta*Da] or NULL (row = sample*K' + j, t = K'-1-j)
 *   lp_mean [n, K'] or NULL: mean over the first reward_horizon Ta rows of clip(lp, -5, 2)   */
DPPO_API int dppo_logprob(const dppo_dims* d, int precision, const void* packed_ft, const float* sched,
                 const float* cond, const float* chains, int n, float min_logprob_std, int reward_horizon,
                 float* lp_elem, float* lp_mean, void* stream);

/* ---- a6: CriticObs forward (model/common/critic.py:40-54): values [n] ---- */
DPPO_API int dppo_critic_forward(const dppo_dims* d, int precision, const void* packed_critic, const float* cond,
                        int n, float* values, void* stream);

/* ---- a18: RunningRewardScaler.__call__ (util/reward_scaling.py:60-87), in place on device.
 *   reward [S, E] (time-major, fp64), first [S, E] (u8); ret_state [E] fp64 carried across calls;
 *   rms_state [3] fp64 {mean, var, count} (init {0, 1, 1e-4}); reward overwritten with the scaled value;
 *   workspace: dppo_reward_scale_workspace_doubles(S, E) fp64 */
DPPO_API size_t dppo_reward_scale_workspace_doubles(int S, int E);
DPPO_API int dppo_reward_scale(double* reward, const uint8_t* first, double* ret_state, double* rms_state, double* workspace,
                      int S, int E, double gamma, double cliprew, double epsilon, void* stream);
/* same, split for multi-GPU: pass 1 (returns local moments {n, mean, M2} in moments[3]) ... */
DPPO_API int dppo_reward_scale_moments(const double* reward, const uint8_t* first, double* ret_state, double* workspace,
                              double* moments, int S, int E, double gamma, void* stream);
/* ... caller all-reduces/merges moments into rms_state, then pass 2 */
DPPO_API int dppo_reward_scale_apply(double* reward, const double* rms_state, int S, int E, double cliprew,
                            double epsilon, void* stream);
/* ABI 12: RunningRewardScaler(per_env=True) (util/reward_scaling.py:51-66). The reference's
 * RunningMeanStd then has shape (num_envs,) and is updated by ret_rms.update(rets) with rets [E, S]:
 * the moments are taken over axis 0, the ENVS, one (mean, var) pair per time column with batch count
 * E, and NumPy broadcasting joins them to the state (so S must equal the state's length L, or one of
 * the two be 1); transform() divides reward [E, S] by sqrt(var + eps) along its last axis. Kept as
 * written, broadcasting errors included (DPPO_EINVAL "operands could not be broadcast together").
 *   rms_in / rms_out fp64 [1 + 2 L] = {count, mean[L], var[L]} (init {1e-4, 0..., 1...}, L = E);
 *   rms_out has L_out = broadcast(S, L_in) entries and must not alias rms_in;
 *   out [C, E] time-major (C = S, or L_out when S == 1 < L_out: the reference returns [E, L_out]); out
 *   may alias reward when C == S. reward / first / ret_state / workspace as dppo_reward_scale. */
DPPO_API int dppo_reward_scale_per_env(const double* reward, const uint8_t* first, double* ret_state,
                                       const double* rms_in, int L_in, double* rms_out, double* workspace, int S, int E,
                                       double gamma, double cliprew, double epsilon, double* out, void* stream);
/* ... the same split for multi-GPU: the scan and the per-column moments col_moments fp64 [S][2] =
 * {mean_t, var_t} over this rank's envs (the caller merges ranks and updates the state), then the scale */
DPPO_API int dppo_reward_scale_per_env_moments(const double* reward, const uint8_t* first, double* ret_state,
                                               double* workspace, double* col_moments, int S, int E, double gamma,
                                               void* stream);
DPPO_API int dppo_reward_scale_per_env_apply(const double* reward, const double* rms_state, int S, int E, int L,
                                             double cliprew, double epsilon, double* out, void* stream);

/* ---- a19: GAE (train_ppo_diffusion_agent.py:239-263). reward fp64 [S,E], values fp32 [S,E],
 * last_values fp32 [E], terminated u8 [S,E] -> advantages, returns fp32 [S,E] */
DPPO_API int dppo_gae(const double* reward, const float* values, const float* last_values, const uint8_t* terminated,
             int S, int E, double gamma, double lam, double reward_scale_const,
             float* advantages, float* returns, void* stream);

/* ---- a16: episode accounting (train_ppo_diffusion_agent.py:144-167) on the RAW rewards fp64 [S,E]
 * and the episode-start flags first u8 [S+1,E] (row S: the flags after the last step): per env,
 * out fp64 [E][4] = {episodes that start and end inside the rollout (consecutive starts s < en with
 * en - s > 1), sum of their returns, sum of their best rewards max(rew[s:en]) / act_steps, count of
 * best >= success_threshold}; the caller sums the rows in env order. (ABI 14) */
DPPO_API int dppo_episode_sums(const double* reward, const uint8_t* first, int S, int E, int act_steps,
                               double success_threshold, double* out, void* stream);

/* ---- a22: explained-variance moments (train_ppo_diffusion_agent.py:373-377) of y = returns and
 * d = returns - values over n rows: moments fp64[5] = {sum y, sum y^2, sum d, sum d^2, n}, one
 * deterministic workgroup; moments may be device or host-mapped memory (dppo_host_alloc). Summed
 * over ranks they give explained_var = 1 - Var(d) / Var(y). (ABI 5) */
DPPO_API int dppo_value_moments(const float* values, const float* returns, int64_t n, double* moments, void* stream);

/* ---- a12/a13/a20: one PPO minibatch: gather by permutation, PPODiffusion.c_loss forward + gradient
 * of pg_loss + vf_coef*v_loss w.r.t. actor_ft and critic (diffusion_ppo.py:32-132,
 * train_ppo_diffusion_agent.py:287-346).
 * Rollout buffers (sample index n = step*E + env, total = S*E*K'):
 *   obs [S*E, To*Do], chains [S*E, K'+1, Ta*Da], lp_old_mean [S*E, K'] (from dppo_logprob),
 *   advantages / returns [S*E] fp32.
 * Minibatch rows: perm(start .. start+rows-1) with perm = Feistel bijection of [0,total) keyed
 * by (perm_seed, epoch), unravelled to (n, j) = (idx / K', idx % K') (tf.unravel_index);
 * or, when row_index != NULL, idx = row_index[start + r] (host-chosen rows, e.g. c_loss on an
 * explicit batch or a replayed tf.random.shuffle permutation).
 * grads [actor_count + critic_count] fp32 are OVERWRITTEN (actor first). metrics (device, fp64[16]):
 *   {pg_loss, v_loss, approx_kl, clipfrac, ratio_mean, loss, adv_mean, adv_std, ...}.
 * adv_stats: fp64[3] {count, sum, sumsq} of the minibatch advantages, or NULL to compute locally;
 *   a multi-GPU caller computes them with dppo_ppo_adv_stats + all-reduce first. */
typedef struct dppo_ppo_hparams {
    float gamma_denoising, clip_ploss_coef, clip_ploss_coef_base, clip_ploss_coef_rate;
    float min_logprob_std, vf_coef;
    int32_t norm_adv, reward_horizon;
    float loss_scale;       /* multiplies 1/b (= 1/world_size for a DP all-reduce-sum) */
    int32_t global_rows;    /* b used in the 1/b means (rows over all ranks) */
    int32_t flags;          /* ABI 8: DPPO_PPO_* below (0: every gradient materialised) */
    /* ABI 14: the clipped value loss (diffusion_ppo.py:110-116) when clip_vloss_coef > 0:
     * v_loss = 0.5 mean(max((V - R)^2, (V_old + clip(V - V_old, -c, c) - R)^2)) with V_old = old_values[n],
     * the rollout's value pass (device fp32 [S*E]); clip_vloss_coef <= 0 (or old_values NULL): the plain
     * 0.5 mean((V - R)^2) of :118 (every shipped cfg: clip_vloss_coef null) */
    float clip_vloss_coef;
    const float* old_values;
} dppo_ppo_hparams;

/* ABI 8, dppo_ppo_hparams.flags. DPPO_PPO_L2_DEFERRED: the actor's l2 gradient is left in its
 * factored form. The l2 weight region of grads holds pl2 = u2^T dy as [H][XD] (row-major, the rest
 * of the region zero) and the l2 bias region is zero; the true values are pl2 rnd(W_out)^T and
 * db_out rnd(W_out)^T (the block's output feeds only the linear out layer). A following
 * dppo_optimizer_step with DPPO_STEP_L2_FROM_PL2 forms them inside its AdamW launch (one launch
 * fewer per minibatch); dppo_materialize_l2 forms them in place. The factored form is linear, so a
 * data-parallel caller all-reduces it like the other gradients. */
enum { DPPO_PPO_L2_DEFERRED = 1 };
/* ABI 9, dppo_ppo_hparams.flags. DPPO_PPO_LEARN_ETA: a learnable DDIM eta (the original DPPO's
 * EtaFixed; the reference's eta module is absent, so parity is unpinned): the actor's row tiles add
 * d loss / d eta into metrics[8] (fp64), through sigma = eta s and d = sqrt(clip(1 - abar_prev -
 * sigma^2, 0, 1e6)) of each row (schedule column 7 = s). dppo_eta_step applies it. */
enum { DPPO_PPO_LEARN_ETA = 2 };
/* ABI 11, dppo_ppo_hparams.flags. DPPO_PPO_PRECLEARED: the outputs this part would zero first (its
 * gradient range and the ranges dppo_ppo_clear_ranges reports for the same workspace, rows and
 * metrics) are already zero — the previous optimizer step of the range cleared them
 * (DPPO_STEP_CLEAR_GRADS) — so the part skips its zeroing launch. */
enum { DPPO_PPO_PRECLEARED = 4 };

/* ABI 9: the learnable DDIM eta's optimizer step (the original DPPO's EtaFixed trained by its own
 * AdamW every eta_update_interval minibatches, train_ppo_diffusion_agent.py:28-45, 358-359 — the
 * reference's step is commented out and its eta module absent: parity unpinned). eta_state (device
 * fp32[3]) = {logit, m, v}, eta = eta_min + (eta_max - eta_min) (tanh(logit) + 1) / 2. With metrics
 * (device fp64[16], metrics[8] = d loss / d eta of a DPPO_PPO_LEARN_ETA minibatch) and step >= 1 it
 * applies AdamW (mode as dppo_adamw) to the logit; then (also with metrics == NULL: a refresh) it
 * rewrites columns c2, c3, logvar of the ddim_steps rows of sched for the current eta from ddim_base
 * (fp32 [ddim_steps][5] = {abar_prev, sqrt(abar_prev), sqrt(abar), sqrt(1 - abar), s}) and stores
 * eta to eta_out (device or mapped, may be NULL). One launch on stream. */
DPPO_API int dppo_eta_step(float* eta_state, const double* metrics, int64_t step, float lr, float weight_decay,
                           float beta1, float beta2, float eps, int mode, float eta_min, float eta_max,
                           const float* ddim_base, float* sched, int ddim_steps, float* eta_out, void* stream);

DPPO_API size_t dppo_ppo_workspace_bytes(const dppo_dims* d, int precision, int batch_rows);
DPPO_API int dppo_ppo_adv_stats(const float* advantages, int64_t total, int K_ft, uint64_t perm_seed, int epoch,
                       int64_t start, int rows, const int64_t* row_index, double* adv_stats, void* stream);
/* The adv_stats of every minibatch of an update phase in one launch: minibatch m = e * n_batch + b
 * covers permutation positions [b * rows_full, min((b+1) * rows_full, total)) of epoch epoch0 + e;
 * adv_stats receives fp64 [n_epochs * n_batch][3]. Same values as n_epochs * n_batch calls of
 * dppo_ppo_adv_stats (row_index = NULL); a multi-GPU caller all-reduces the whole array once. */
DPPO_API int dppo_ppo_adv_stats_all(const float* advantages, int64_t total, int K_ft, uint64_t perm_seed, int epoch0,
                           int n_epochs, int64_t rows_full, int n_batch, double* adv_stats, void* stream);
DPPO_API int dppo_ppo_minibatch(const dppo_dims* d, int precision, const dppo_ppo_hparams* hp,
                       const void* packed_ft, const void* packed_critic, const float* actor_params,
                       const float* sched, const float* obs, const float* chains, const float* lp_old_mean,
                       const float* advantages, const float* returns, int64_t total, uint64_t perm_seed,
                       int epoch, int64_t start, int rows, const int64_t* row_index, const double* adv_stats,
                       void* workspace, float* grads, double* metrics, void* stream);

/* ---- §8(f) row 3: the pretraining loss DiffusionModel.c_loss -> p_losses / q_sample
 * (model/diffusion/diffusion.py:179-202; predict_epsilon = True), loss and actor gradients.
 * Replaces the TF tape over `self.model.c_loss(**batch)` in agent/pretrain/train_diffusion_agent.py.
 * Row r is sample r: x_start [rows][horizon*action_dim], cond [rows][cond_steps*obs_dim],
 * t [rows] int32 in [0, denoising_steps), noise [rows][horizon*action_dim] (the host draws t and
 * noise, tf.random.uniform / tf.random.normal at diffusion.py:182,187).
 * sched: the DDPM schedule table (denoising_steps rows); qsched [denoising_steps][2] fp32 =
 * {sqrt(alphas_cumprod), sqrt(1 - alphas_cumprod)} (the TF buffers, diffusion.py:62-65).
 * loss = loss_scale * sum((eps - noise)^2) / (global_rows * horizon*action_dim): metrics[0] (fp64,
 * device) receives the local sum of squares; grads [actor_count] fp32 are OVERWRITTEN with
 * d loss / d params. Workspace: dppo_ppo_workspace_bytes(d, precision, rows). Requires
 * time_stride == 1 and denoising_steps <= 64. ---- */
DPPO_API int dppo_pretrain_minibatch(const dppo_dims* d, int precision, const void* packed_actor, const float* actor_params,
                            const float* sched, const float* qsched, const float* x_start, const float* cond,
                            const int32_t* t, const float* noise, int rows, int64_t global_rows, float loss_scale,
                            void* workspace, float* grads, double* metrics, void* stream);

/* One half of dppo_ppo_minibatch on the caller's stream, so a caller can overlap the critic's half
 * of minibatch i+1 with the actor's tail of minibatch i: part 1 = the actor (zeroes the actor
 * gradients and metrics 0, 2..15; row tiles, dW, time-MLP backward; needs adv_stats), part 2 =
 * the critic (zeroes the critic gradients and metric 1; row tiles, dW). Part 1 also splits in two
 * (ABI 6): part 4 = the actor's zeroing + row tiles (its loss metrics are final after it), part 5 =
 * the actor's dW + time-MLP backward, so a data-parallel caller can all-reduce the metrics with the
 * critic's gradients while the actor's dW runs. Same arguments and results as dppo_ppo_minibatch,
 * which runs both halves (the critic on an internal side stream). */
/* ABI 11: the non-gradient byte ranges part (1/4 = actor, 2 = critic, 3 = whole) of a minibatch of
 * batch_rows rows zeroes before it runs (metric slots of `metrics`, workspace accumulators): up to 3,
 * their count in *count. A caller passes them to the preceding dppo_optimizer_step_ex to run that
 * minibatch with DPPO_PPO_PRECLEARED. */
DPPO_API int dppo_ppo_clear_ranges(const dppo_dims* d, int precision, int batch_rows, void* workspace, double* metrics,
                                   int part, void** ptrs, size_t* bytes, int* count);
DPPO_API int dppo_ppo_minibatch_part(const dppo_dims* d, int precision, const dppo_ppo_hparams* hp,
                            const void* packed_ft, const void* packed_critic, const float* actor_params,
                            const float* sched, const float* obs, const float* chains, const float* lp_old_mean,
                            const float* advantages, const float* returns, int64_t total, uint64_t perm_seed,
                            int epoch, int64_t start, int rows, const int64_t* row_index, const double* adv_stats,
                            void* workspace, float* grads, double* metrics, int part, void* stream);

/* Feistel permutation used above, exposed for tests: out[i] = perm(first + i), i < count. */
DPPO_API int dppo_feistel_permute(int64_t first, int64_t count, int64_t n, uint64_t seed, int epoch, int64_t* out,
                         void* stream);

/* ---- a14: optimiser step over a flat fp32 buffer (Keras 3 AdamW semantics by default;
 * train_ppo_agent.py:45-49). step is 1-based. ---- */
DPPO_API int dppo_adamw(float* params, const float* grads, float* m, float* v, int64_t n, int64_t step, float lr,
               float weight_decay, float beta1, float beta2, float eps, int mode, void* stream);

/* Re-derive the packed images of the actor and/or the critic (either pair may be null) in ONE
 * launch; the actor's includes its time tables. = dppo_pack_actor + dppo_pack_critic. */
DPPO_API int dppo_pack_all(const dppo_dims* d, int precision, const float* actor_params, void* packed_actor,
                  const float* critic_params, void* packed_critic, void* stream);

/* One optimiser step after a PPO minibatch as two launches on `stream`
 * (train_ppo_diffusion_agent.py:346 apply_gradients, then the weight images every kernel reads):
 * dppo_adamw over the n elements at params/grads/m/v (a range of the flat [actor | critic]
 * buffer), which also copies n_metrics (<= 256) doubles of `metrics` to `metrics_out` (device or
 * host-mapped memory; the minibatch's metric sums for the host's target_kl check), then
 * dppo_pack_all of the given networks. ABI 5: a nonzero metrics_tag (< 2^53) is stored as the
 * double metrics_out[n_metrics] AFTER the n_metrics sums (system-scope release), so a host polling
 * host-mapped metrics_out for the tag reads complete sums without recording or waiting on an event
 * (metrics_out then holds n_metrics + 1 doubles; pass 0 for no tag). */
/* ABI 8: the actor's l2 gradient of a DPPO_PPO_L2_DEFERRED minibatch, formed in place in grads (the
 * actor range first) from the factored form; workspace = the minibatch's (its pl2 slot is the
 * staging copy). */
DPPO_API int dppo_materialize_l2(const dppo_dims* d, int precision, const void* packed_actor, float* grads,
                                 void* workspace, int batch_rows, void* stream);

/* Enqueue the split-sampler tables of an actor image on `stream` if an optimizer step with
 * DPPO_STEP_DEFER_SAMPLER_TABLES left them stale; a no-op otherwise (ABI 7). */
DPPO_API int dppo_refresh_sampler_tables(const void* packed_actor, void* stream);

DPPO_API int dppo_optimizer_step(const dppo_dims* d, int precision, float* params, const float* grads, float* m,
                        float* v, int64_t n, int64_t step, float lr, float weight_decay, float beta1,
                        float beta2, float eps, int mode, const float* actor_params, void* packed_actor,
                        const float* critic_params, void* packed_critic, const double* metrics,
                        double* metrics_out, int n_metrics, uint64_t metrics_tag, void* stream);
/* ABI 11: dppo_optimizer_step that also zeroes n_clear (<= 4) byte ranges (4-B aligned, sizes multiples
 * of 4) after the launch's last read, and with DPPO_STEP_CLEAR_GRADS the gradients of the range. */
DPPO_API int dppo_optimizer_step_ex(const dppo_dims* d, int precision, float* params, float* grads, float* m,
                           float* v, int64_t n, int64_t step, float lr, float weight_decay, float beta1,
                           float beta2, float eps, int mode, const float* actor_params, void* packed_actor,
                           const float* critic_params, void* packed_critic, const double* metrics,
                           double* metrics_out, int n_metrics, uint64_t metrics_tag, void* const* clear_ptrs,
                           const size_t* clear_bytes, int n_clear, void* stream);


/* ---- ABI 12, §8(e): the data-parallel gradient all-reduce as one kernel over IPC-mapped peer
 * buffers (the reference has no collective: it applies gradients on one device,
 * train_ppo_diffusion_agent.py:345-356, script/run.py:82; RCCL's all_reduce is the default here).
 * Every rank allocates one region of dppo_ipc_region_bytes(capacity) with dppo_ipc_alloc (device
 * memory, zeroed; handle = 64 bytes for hipIpcOpenMemHandle), exchanges the handles out of band
 * (torch.distributed) and opens every peer's with dppo_ipc_open. dppo_ipc_allreduce then sums
 * data[0, n) (fp32, n <= capacity) over the ranks IN PLACE on every rank, in rank order 0..W-1 (so
 * every rank gets the same bits: a sequential fp32 sum): regions[x] = rank x's region as mapped in
 * this process (regions[rank] = the own one), world <= 8, generation = 1, 2, ... the same on every
 * rank for the same call; every rank must make the same calls in the same order, one launch each on
 * its stream. A barrier that waits more than ~2 s sets *fail_host (dppo_host_alloc memory) and the
 * next call returns DPPO_EHIP. */
DPPO_API size_t dppo_ipc_region_bytes(int64_t capacity);
DPPO_API int dppo_ipc_alloc(size_t bytes, void** ptr, void* handle);
DPPO_API int dppo_ipc_open(const void* handle, void** ptr);
DPPO_API int dppo_ipc_close(void* ptr);
DPPO_API int dppo_ipc_free(void* ptr);
DPPO_API int dppo_ipc_allreduce(void* const* regions, int world, int rank, int64_t capacity, float* data, int64_t n,
                                uint64_t generation, uint32_t* fail_host, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DPPO_H */
