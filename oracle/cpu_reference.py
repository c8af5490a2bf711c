"""CPU baseline: an fp32 torch-CPU restatement of one DPPO fine-tuning iteration.

TEST / MEASUREMENT INFRASTRUCTURE ONLY — used by bench.py's cpu_baseline leg (and its CPU test),
never by the product package. TF-CPU (the reference's own runtime) cannot be installed here or
on the GPU box (no network), so SURVEY.md §8(d) names this as the CPU reference: the same
algorithm in fp32 on the host's cores, with autograd for the PPO gradient as TF's GradientTape
gives the reference (agent/finetune/train_ppo_diffusion_agent.py:314-356). It runs the WHOLE
iteration of the benchmark workload, not an extrapolation:
  * rollout: S chunks of `model(cond)` (diffusion_vpg.py:250-339: K DDPM steps through the
    DiffusionMLP, base actor for t >= K', fine-tuned below) + the synthetic env step;
  * value and old-log-prob passes (agent :191-229), running reward scaler (util/reward_scaling.py),
    GAE (agent :239-263) in float64 NumPy as the reference does;
  * update_epochs x (S*E*K' // b) minibatches of c_loss (diffusion_ppo.py:32-132) + autograd +
    Keras-3 AdamW (decoupled decay 0.004, eps 1e-7) over [actor_ft | critic].
Like the reference, the wasted base-actor forwards of quirk 1 are skipped (algorithmic work only).
"""
import math
import time

import numpy as np
import torch

from . import dppo_oracle as O
from .iteration import SyntheticVecEnvOracle


def _glorot(g, fi, fo):
    lim = math.sqrt(6.0 / (fi + fo))
    return (torch.rand(fi, fo, generator=g) * 2 - 1) * lim


class TorchCPUDPPO:
    def __init__(self, obs_dim=11, action_dim=3, horizon=4, K=20, KF=10, hidden=512, critic_hidden=256, time_dim=16,
                 seed=0):
        g = torch.Generator().manual_seed(seed)
        self.Do, self.Da, self.Ta, self.K, self.KF, self.TD = obs_dim, action_dim, horizon, K, KF, time_dim
        self.XD = horizon * action_dim
        ind = self.XD + time_dim + obs_dim

        def actor():
            return {"tw1": _glorot(g, time_dim, 2 * time_dim), "tb1": torch.zeros(2 * time_dim),
                    "tw2": _glorot(g, 2 * time_dim, time_dim), "tb2": torch.zeros(time_dim),
                    "in_w": _glorot(g, ind, hidden), "in_b": torch.zeros(hidden),
                    "l1_w": _glorot(g, hidden, hidden), "l1_b": torch.zeros(hidden),
                    "l2_w": _glorot(g, hidden, hidden), "l2_b": torch.zeros(hidden),
                    "out_w": _glorot(g, hidden, self.XD), "out_b": torch.zeros(self.XD)}
        self.base = actor()
        self.ft = {k: v.clone().requires_grad_(True) for k, v in self.base.items()}
        self.critic = {"in_w": _glorot(g, obs_dim, critic_hidden), "in_b": torch.zeros(critic_hidden),
                       "l1_w": _glorot(g, critic_hidden, critic_hidden), "l1_b": torch.zeros(critic_hidden),
                       "l2_w": _glorot(g, critic_hidden, critic_hidden), "l2_b": torch.zeros(critic_hidden),
                       "out_w": _glorot(g, critic_hidden, 1), "out_b": torch.zeros(1)}
        for v in self.critic.values():
            v.requires_grad_(True)
        self.train_vars = list(self.ft.values()) + list(self.critic.values())
        self.m = [torch.zeros_like(p) for p in self.train_vars]
        self.v = [torch.zeros_like(p) for p in self.train_vars]
        self.opt_step = 0
        s = O.ddpm_schedule(K)
        self.sched = {k: torch.tensor(np.asarray(v, np.float32)) for k, v in s.items()}
        half = time_dim // 2
        self.freqs = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000) / (half - 1)))
        self.gen = torch.Generator().manual_seed(seed + 1)

    # ---- networks (mlp_diffusion.py:38-90, mlp.py:95-206, critic.py:15-54) ----
    def _temb(self, p, t):
        e = t.float()[:, None] * self.freqs[None, :]
        e = torch.cat([e.sin(), e.cos()], dim=-1)
        a = torch.addmm(p["tb1"], e, p["tw1"])
        return torch.addmm(p["tb2"], a * torch.tanh(torch.nn.functional.softplus(a)), p["tw2"])

    @staticmethod
    def _resmlp(p, x, act):
        h1 = torch.addmm(p["in_b"], x, p["in_w"])
        h2 = torch.addmm(p["l1_b"], act(h1), p["l1_w"])
        h3 = torch.addmm(p["l2_b"], act(h2), p["l2_w"]) + h1
        return torch.addmm(p["out_b"], h3, p["out_w"])

    def eps(self, p, x, t, state):
        inp = torch.cat([x, self._temb(p, t), state], dim=-1)
        return self._resmlp(p, inp, torch.relu)

    def value(self, state):
        return self._resmlp(self.critic, state, torch.nn.functional.mish)[:, 0]

    def _pmv(self, e, x, t):
        s = self.sched
        xr = (s["sqrt_recip_alphas_cumprod"][t][:, None] * x - s["sqrt_recipm1_alphas_cumprod"][t][:, None] * e).clamp(-1, 1)
        mu = s["ddpm_mu_coef1"][t][:, None] * xr + s["ddpm_mu_coef2"][t][:, None] * x
        return mu, s["ddpm_logvar_clipped"][t]

    # ---- sampler (diffusion_vpg.py:250-339), train mode ----
    @torch.no_grad()
    def sample(self, state, min_std=0.1, randn_clip=3.0):
        E = state.shape[0]
        x = torch.randn(E, self.XD, generator=self.gen)
        chain = []
        for i in range(self.K):
            t = self.K - 1 - i
            tb = torch.full((E,), t, dtype=torch.long)
            e = self.eps(self.ft if t < self.KF else self.base, x, tb, state)
            mu, logvar = self._pmv(e, x, tb)
            std = torch.exp(0.5 * logvar).clamp(min_std, 1e6)[:, None]
            x = mu + std * torch.randn(E, self.XD, generator=self.gen).clamp(-randn_clip, randn_clip)
            if t <= self.KF:
                chain.append(x)
        return x, torch.stack(chain, dim=1)

    def _logprob_rows(self, state, prev, nxt, t, min_std=0.1):
        e = self.eps(self.ft, prev, t, state)
        mu, logvar = self._pmv(e, prev, t)
        std = torch.exp(0.5 * logvar).clamp(min_std, 1e6)[:, None]
        lp = -0.5 * ((nxt - mu) / std) ** 2 - torch.log(std) - 0.5 * math.log(2 * math.pi)
        return lp.clamp(-5, 2).mean(dim=1)                                 # diffusion_ppo.py:50-59

    def _keras_adamw(self, grads, lr=1e-4, wd=0.004, b1=0.9, b2=0.999, eps=1e-7):
        self.opt_step += 1
        alpha = lr * math.sqrt(1 - b2 ** self.opt_step) / (1 - b1 ** self.opt_step)
        with torch.no_grad():
            for p, g, m, v in zip(self.train_vars, grads, self.m, self.v):
                p.mul_(1 - wd * lr)
                m.add_((g - m) * (1 - b1))
                v.add_((g * g - v) * (1 - b2))
                p.sub_(alpha * m / (v.sqrt() + eps))

    # ---- one fine-tuning iteration (agent :58-377) ----
    def iteration(self, env, S, batch_size, update_epochs=5, gamma=0.99, lam=0.95, scaler=None, obs=None,
                  max_minibatches=None):
        """Returns (timings dict, next obs). max_minibatches bounds the update (1-thread sample)."""
        E, kf = env.E, self.KF
        t0 = time.perf_counter()
        if obs is None:
            obs = env.reset_all()
        obs_traj = np.zeros((S, E, self.Do), np.float32)
        chains = torch.zeros(S, E, kf + 1, self.XD)
        rewards, terms, firsts = np.zeros((S, E)), np.zeros((S, E)), np.zeros((S + 1, E))
        for step in range(S):
            o = torch.from_numpy(obs.astype(np.float32))
            traj, chain = self.sample(o)
            obs_traj[step] = o.numpy()
            chains[step] = chain
            obs, r, term, trunc = env.step(traj.view(E, self.Ta, self.Da).double().numpy())
            rewards[step], terms[step], firsts[step + 1] = r, term, term | trunc
        t1 = time.perf_counter()
        N = S * E
        obs_k = torch.from_numpy(obs_traj.reshape(N, self.Do))
        ch_k = chains.view(N, kf + 1, self.XD)
        with torch.no_grad():
            values = self.value(obs_k).double().numpy().reshape(S, E)
            lp_old = torch.empty(N, kf)
            for j in range(kf):
                t = torch.full((N,), kf - 1 - j, dtype=torch.long)
                lp_old[:, j] = self._logprob_rows(obs_k, ch_k[:, j], ch_k[:, j + 1], t)
            last_v = self.value(torch.from_numpy(obs.astype(np.float32))).double().numpy()
        if scaler is not None:
            rewards = scaler(rewards.T, firsts[:-1].T).T
        adv, ret = O.gae(rewards, values, last_v, terms, gamma, lam)
        adv_k = torch.from_numpy(adv.reshape(-1).astype(np.float32))
        ret_k = torch.from_numpy(ret.reshape(-1).astype(np.float32))
        t2 = time.perf_counter()
        total = N * kf
        num_batch = max(1, total // batch_size)
        done = 0
        for _ in range(update_epochs):
            perm = torch.randperm(total, generator=self.gen)
            for b in range(num_batch):
                if max_minibatches is not None and done >= max_minibatches:
                    break
                inds = perm[b * batch_size:(b + 1) * batch_size]
                bi, di = inds // kf, inds % kf
                st = obs_k[bi]
                new = self._logprob_rows(st, ch_k[bi, di], ch_k[bi, di + 1], (kf - 1 - di))
                a = adv_k[bi]
                a = (a - a.mean()) / (a.std(unbiased=False) + 1e-8)
                a = a * 0.99 ** (kf - di.float() - 1)
                logr = new - lp_old[bi, di]
                r = logr.exp()
                pg = torch.max(-a * r, -a * r.clamp(0.99, 1.01)).mean()
                v_loss = 0.5 * ((self.value(st) - ret_k[bi]) ** 2).mean()
                loss = pg + 0.5 * v_loss
                grads = torch.autograd.grad(loss, self.train_vars)
                self._keras_adamw(grads)
                _ = float(((r - 1) - logr).detach().mean())                    # approx_kl, read per minibatch
                done += 1
        t3 = time.perf_counter()
        return dict(rollout_s=t1 - t0, passes_s=t2 - t1, update_s=t3 - t2, minibatches=done,
                    minibatches_full=update_epochs * num_batch), obs


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores():
    try:
        seen = set()
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":")[1].strip()
                    seen.add((phys, core))
        return len(seen) or None
    except OSError:
        return None


def time_iteration(n_envs, S, batch_size, update_epochs=5, threads=None, obs_dim=11, action_dim=3, seed=0,
                   max_minibatches=None, warm_steps=2):
    """One full iteration of the workload on `threads` CPU threads (default: torch's). Returns
    (seconds, breakdown). A short warm-up (warm_steps rollout chunks, one small minibatch) runs
    first so allocator / thread-pool start-up is not timed."""
    if threads:
        torch.set_num_threads(int(threads))
    m = TorchCPUDPPO(obs_dim=obs_dim, action_dim=action_dim, seed=seed)
    env = SyntheticVecEnvOracle(np.arange(n_envs) + seed, obs_dim, action_dim, 4, 1000)
    m.iteration(env, warm_steps, min(batch_size, warm_steps * n_envs * 10), update_epochs=1, max_minibatches=1)
    scaler = O.RunningRewardScalerOracle(n_envs)
    t0 = time.perf_counter()
    br, _ = m.iteration(env, S, batch_size, update_epochs, scaler=scaler, max_minibatches=max_minibatches)
    return time.perf_counter() - t0, br
