"""Whole-iteration restatement of the DPPO fine-tuning loop (float64 NumPy).

TEST INFRASTRUCTURE ONLY — imported by tests/ (and nothing in the product package). It composes
the per-row oracle functions of oracle/dppo_oracle.py into TrainPPODiffusionAgent.run's loop
(reference agent/finetune/train_ppo_diffusion_agent.py:58-377) on the synthetic vector env, so
that the glue the single-kernel tests cannot see is checked against a reference: env resets and
`firsts` (quirk 4), episode accounting, the reward scaler's state carried across iterations, the
value / old-log-prob passes, GAE, the minibatch index math, c_loss + one Keras AdamW over
[actor_ft | critic], and the target_kl stop.

Where the TF reference draws from TF's RNG (the sampler's tf.random.normal, diffusion_vpg.py:
280,319; the minibatch tf.random.shuffle, agent :287) this restatement uses the build's own
counter streams (oracle/philox.py: Philox normals keyed by (seed, call_id, env row, slot), the
keyed Feistel permutation keyed by (perm_seed, epoch + 1000 * itr)), as the build documents
(DESIGN.md §4). Everything else follows the cited reference lines.
"""
import numpy as np

from . import dppo_oracle as O
from . import philox as PX


# ----------------------------------------------------------------------------------------------
# the synthetic locomotion env behind the reference's MultiStep wrapper
# (env/gym_utils/wrapper/multi_step.py:135-192, reset_within_step=True, reward_agg "sum")
# ----------------------------------------------------------------------------------------------
class SyntheticVecEnvOracle:
    """Seeded linear dynamics clipped to [-1, 1], reward 1 - mean((s - goal)^2) - 0.01 mean(a^2),
    truncation at max_episode_steps sub-steps (no terminal states). Same constants as the build's
    synthetic env (family_seed -> A, B, c, goal; (env seed, episode, coordinate) -> initial state)."""

    def __init__(self, seeds, obs_dim, action_dim, act_steps, max_episode_steps, family_seed=0):
        self.seeds = np.asarray(seeds, np.int64)
        E = len(self.seeds)
        self.E, self.obs_dim, self.action_dim = E, obs_dim, action_dim
        self.act_steps, self.max_episode_steps = act_steps, max_episode_steps
        rng = np.random.default_rng(10_000 + family_seed)
        q, _ = np.linalg.qr(rng.normal(size=(obs_dim, obs_dim)))
        self.A = 0.97 * q
        self.B = rng.normal(0, 0.3, size=(action_dim, obs_dim))
        self.c = rng.normal(0, 0.02, size=obs_dim)
        self.goal = rng.uniform(-0.5, 0.5, size=obs_dim)
        self.state = np.zeros((E, obs_dim))
        self.cnt = np.zeros(E, np.int64)
        self.episode = np.zeros(E, np.int64)

    def _initial(self, idx):
        sd = self.seeds[idx].astype(np.float64)[:, None]
        ep = self.episode[idx].astype(np.float64)[:, None]
        j = np.arange(self.obs_dim, dtype=np.float64)[None, :]
        h = np.sin(sd * 12.9898 + ep * 78.233 + j * 37.719 + 0.5) * 43758.5453
        return (h - np.floor(h) - 0.5) * 0.2

    def reset_all(self):
        idx = np.arange(self.E)
        self.state[:] = self._initial(idx)
        self.cnt[:] = 0
        return self.state.copy()

    def step(self, actions):
        """actions [E, act_steps, Da] -> (obs [E, Do], reward [E], terminated [E], truncated [E])."""
        E = self.E
        reward = np.zeros(E)
        truncated = np.zeros(E, bool)
        alive = np.ones(E, bool)
        for k in range(actions.shape[1]):                              # multi_step.py:146-170
            self.cnt[alive] += 1
            a = np.clip(actions[:, k], -1, 1)
            s = np.clip(self.state @ self.A.T + a @ self.B + self.c, -1.0, 1.0)
            self.state = np.where(alive[:, None], s, self.state)
            r = 1.0 - np.mean((self.state - self.goal) ** 2, axis=1) - 0.01 * np.mean(actions[:, k] ** 2, axis=1)
            reward += np.where(alive, r, 0.0)
            truncated |= alive & (self.cnt >= self.max_episode_steps)
            alive &= ~truncated
        terminated = np.zeros(E, bool)
        done = terminated | truncated
        if done.any():                                                 # reset_within_step (:177-187)
            idx = np.nonzero(done)[0]
            self.episode[idx] += 1
            self.state[idx] = self._initial(idx)
            self.cnt[idx] = 0
        return self.state.copy(), reward, terminated, truncated


# ----------------------------------------------------------------------------------------------
# the fine-tuning loop
# ----------------------------------------------------------------------------------------------
def _flat(spec, d):
    return np.concatenate([np.asarray(d[n], np.float64).reshape(-1) for n, _ in spec])


def _unflat(spec, flat):
    out, o = {}, 0
    for n, s in spec:
        k = int(np.prod(s))
        out[n] = flat[o:o + k].reshape(s)
        o += k
    return out


class PPODiffusionLoopOracle:
    """TrainPPODiffusionAgent.run (agent :58-377) with PPODiffusion / VPGDiffusion on the oracle
    functions. actor_spec / critic_spec: [(name, shape)] of the flat [actor_ft | critic] layout
    (include/dppo.h); base / ft / critic: parameter dicts (f64). Noise, permutation and env seeds
    are inputs (see the module docstring)."""

    def __init__(self, base, ft, critic, actor_spec, critic_spec, sched, env, *, seed, perm_seed,
                 n_steps, ft_steps, act_steps, horizon_steps, action_dim, val_freq, batch_size,
                 update_epochs, target_kl, gamma=0.99, gae_lambda=0.95, reward_scale_running=True,
                 reward_scale_const=1.0, reset_at_iteration=False, force_train=False, lr=1e-4,
                 weight_decay=0.004, min_sampling_std=0.1, randn_clip=3.0, min_logprob_std=0.1,
                 gamma_denoising=0.99, clip_ploss_coef=0.01, clip_ploss_coef_base=0.01,
                 clip_ploss_coef_rate=3.0, vf_coef=0.5, success_threshold=3.0, env_offset=0,
                 n_critic_warmup_itr=0, ft_denoising_steps_d=0, ft_denoising_steps_t=0):
        self.base = {k: np.asarray(v, np.float64) for k, v in base.items()}
        self.actor_spec, self.critic_spec = actor_spec, critic_spec
        self.theta = np.concatenate([_flat(actor_spec, ft), _flat(critic_spec, critic)])
        self.n_actor = int(sum(int(np.prod(s)) for _, s in actor_spec))
        self.m = np.zeros_like(self.theta)
        self.v = np.zeros_like(self.theta)
        self.opt_steps = 0
        self.sched, self.env = sched, env
        self.seed, self.perm_seed, self.env_offset = seed, perm_seed, env_offset
        self.S, self.kf, self.act_steps, self.horizon, self.da = n_steps, ft_steps, act_steps, horizon_steps, action_dim
        self.val_freq, self.batch_size, self.update_epochs, self.target_kl = val_freq, batch_size, update_epochs, target_kl
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.reward_scaler = O.RunningRewardScalerOracle(env.E) if reward_scale_running else None
        self.reward_scale_const = reward_scale_const
        self.reset_at_iteration, self.force_train = reset_at_iteration, force_train
        self.lr, self.wd = lr, weight_decay
        self.min_sampling_std, self.randn_clip, self.min_logprob_std = min_sampling_std, randn_clip, min_logprob_std
        self.closs_kw = dict(gamma_denoising=gamma_denoising, clip_ploss_coef=clip_ploss_coef,
                             clip_ploss_coef_base=clip_ploss_coef_base, clip_ploss_coef_rate=clip_ploss_coef_rate,
                             min_logprob_std=min_logprob_std, vf_coef=vf_coef, reward_horizon=act_steps)
        self.success_threshold = success_threshold
        self.n_critic_warmup_itr = n_critic_warmup_itr
        self.ft_steps_d, self.ft_steps_t, self.ft_steps_cnt = ft_denoising_steps_d, ft_denoising_steps_t, 0
        self.call_id = 0
        self.itr = 0
        self.prev_obs = None
        self.done_venv = np.zeros(env.E, bool)
        self.n_updates = 0

    @property
    def ft(self):
        return _unflat(self.actor_spec, self.theta[:self.n_actor])

    @property
    def critic(self):
        return _unflat(self.critic_spec, self.theta[self.n_actor:])

    # one call of model(cond, deterministic) (diffusion_vpg.py:250-339) with the build's Philox draws
    def _sample(self, obs32, deterministic):
        E, K, xd = self.env.E, len(self.sched["ddpm_logvar_clipped"]), self.horizon * self.da
        x_T = PX.sampler_normals(self.seed, self.call_id, self.env_offset, E, xd, K)
        z = np.stack([PX.sampler_normals(self.seed, self.call_id, self.env_offset, E, xd, i) for i in range(K)])
        self.call_id += 1
        sh = (E, self.horizon, self.da)
        traj, chain = O.sample(self.base, self.ft, self.sched, obs32[:, None, :], x_T.reshape(sh),
                               z.reshape((K,) + sh), self.kf, deterministic=deterministic,
                               min_std=self.min_sampling_std, randn_clip=self.randn_clip)
        return traj, chain

    def iteration(self):
        """One pass of the while-loop body (agent :58-377). Returns a dict of what it produced."""
        S, E, kf = self.S, self.env.E, self.kf
        eval_mode = self.itr % self.val_freq == 0 and not self.force_train          # :68
        last_itr_eval = eval_mode                                                    # :70 (quirk 4)
        firsts = np.zeros((S + 1, E))
        if self.reset_at_iteration or eval_mode or last_itr_eval or self.prev_obs is None:   # :74-77
            self.prev_obs = self.env.reset_all()
            firsts[0] = 1
        else:
            firsts[0] = self.done_venv                                               # :79
        obs_traj = np.zeros((S, E, self.env.obs_dim))
        chains = np.zeros((S, E, kf + 1, self.horizon, self.da))
        rewards = np.zeros((S, E))
        terms = np.zeros((S, E))
        for step in range(S):                                                        # :106-141
            o32 = self.prev_obs.astype(np.float32).astype(np.float64)                # tf.float32 cond (:111-113)
            traj, chain = self._sample(o32, eval_mode)
            # the env receives the fp32 actions (np.array of the fp32 sample, :124)
            act = traj[:, :self.act_steps].astype(np.float32).astype(np.float64)
            obs, r, term, trunc = self.env.step(act)
            self.done_venv = term | trunc
            obs_traj[step] = o32
            chains[step] = chain
            rewards[step] = r
            terms[step] = term
            firsts[step + 1] = self.done_venv
            self.prev_obs = obs
        out = dict(eval=eval_mode, firsts=firsts, rewards=rewards.copy(), chains=chains, obs=obs_traj,
                   episodes=O.episode_stats(firsts, rewards, self.act_steps, self.success_threshold))  # :144-183
        if not eval_mode:
            out.update(self._update(obs_traj, chains, rewards, terms, firsts))
        self._anneal()                                                               # :399
        self.itr += 1
        return out

    def _anneal(self):
        """VPGDiffusion.step (diffusion_vpg.py:114-142): every ft_denoising_steps_t calls, K' drops by
        ft_denoising_steps_d (floor 0) and the frozen base actor becomes a copy of actor_ft
        (`self.actor = self.actor_ft; self.actor_ft = deepcopy(self.actor)`); actor_ft and its
        optimiser state carry on."""
        self.ft_steps_cnt += 1
        if self.ft_steps_d > 0 and self.ft_steps_t > 0 and self.ft_steps_cnt % self.ft_steps_t == 0:
            self.kf = max(0, self.kf - self.ft_steps_d)
            self.base = self.ft

    def _update(self, obs_traj, chains, rewards, terms, firsts):
        S, E, kf = self.S, self.env.E, self.kf
        N = S * E
        obs_k = obs_traj.reshape(N, 1, -1)
        chains_k = chains.reshape(N, kf + 1, self.horizon, self.da)
        critic = self.critic
        values = O.critic_forward(critic, obs_k)[0][:, 0].reshape(S, E)              # :191-208
        lp = O.get_logprobs(self.ft, self.sched, obs_k, chains_k, kf, self.min_logprob_std)   # :209-229
        H = min(self.act_steps, self.horizon)
        lp_old = np.clip(lp, -5, 2)[:, :H].mean(axis=(1, 2)).reshape(N, kf)          # c_loss :50-59
        if self.reward_scaler is not None:                                           # :232-236
            rewards = self.reward_scaler(rewards.T, firsts[:-1].T).T
        last_obs = self.prev_obs.astype(np.float32).astype(np.float64)
        last_values = O.critic_forward(critic, last_obs[:, None, :])[0][:, 0]        # :252
        adv, ret = O.gae(rewards, values, last_values, terms, self.gamma, self.gae_lambda,
                         self.reward_scale_const)                                    # :239-263
        adv_k, ret_k, val_k = adv.reshape(-1), ret.reshape(-1), values.reshape(-1)
        total = N * kf                                                               # :282
        num_batch = max(1, total // self.batch_size)                                 # :288
        metrics_log = []
        for update_epoch in range(self.update_epochs):                               # :284
            perm = PX.feistel_permute(np.arange(total), total, self.perm_seed, update_epoch + 1000 * self.itr)
            for batch in range(num_batch):                                           # :289
                inds = perm[batch * self.batch_size:(batch + 1) * self.batch_size]   # :290-292
                bi, di = inds // kf, inds % kf                                       # :293-296
                met, ga, gc = O.c_loss(self.ft, critic, self.sched, obs_k[bi], chains_k[bi, di], chains_k[bi, di + 1],
                                       di, ret_k[bi], val_k[bi], adv_k[bi], lp_old[bi, di], kf, **self.closs_kw)
                g = np.concatenate([_flat(self.actor_spec, ga), _flat(self.critic_spec, gc)])
                if self.itr >= self.n_critic_warmup_itr:                             # :348-356
                    self.opt_steps += 1
                    self.theta, self.m, self.v = O.keras_adamw_step(self.theta, g, self.m, self.v, self.opt_steps,
                                                                    lr=self.lr, wd=self.wd)
                critic = self.critic
                self.n_updates += 1
                metrics_log.append(met)
                if self.target_kl is not None and met["approx_kl"] > self.target_kl:   # :366-368
                    break                                                            # the batch loop only
        return dict(values=values, lp_old=lp_old, adv=adv, ret=ret, metrics=metrics_log,
                    explained_var=O.explained_variance(val_k, ret_k))
