"""PPODiffusion (reference model/diffusion/diffusion_ppo.py:7-132).

c_loss keeps the reference signature and 8-tuple return; its forward AND the gradient of
pg_loss + vf_coef * v_loss (train_ppo_diffusion_agent.py:340) w.r.t. [actor_ft | critic] are one
fused HIP pass (dppo_ppo_minibatch), left in `self.grads` for the optimiser. The agent uses
`minibatch()`, the same pass gathering rows straight from the HBM-resident rollout buffers."""
import numpy as np
import torch

from ... import _lib, ops
from .diffusion_vpg import VPGDiffusion, _as_state

# metrics slots written by the kernels (sums over rows; see update.hip)
M_PG, M_VLOSS, M_KL, M_CLIPFRAC, M_RATIO = 0, 1, 2, 3, 4
M_DETA = 8   # learn_eta: d loss / d eta (DPPO_PPO_LEARN_ETA)


class PPODiffusion(VPGDiffusion):
    def __init__(self, gamma_denoising, clip_ploss_coef, clip_ploss_coef_base=1e-3, clip_ploss_coef_rate=3,
                 clip_vloss_coef=None, clip_advantage_lower_quantile=0, clip_advantage_upper_quantile=1, norm_adv=True,
                 vf_coef=0.5, **kwargs):
        super().__init__(**kwargs)
        self.gamma_denoising = gamma_denoising
        self.clip_ploss_coef = clip_ploss_coef
        self.clip_ploss_coef_base = clip_ploss_coef_base
        self.clip_ploss_coef_rate = clip_ploss_coef_rate
        self.clip_vloss_coef = clip_vloss_coef
        self.clip_advantage_lower_quantile = clip_advantage_lower_quantile  # unused, as in the reference (:77-80)
        self.clip_advantage_upper_quantile = clip_advantage_upper_quantile
        self.norm_adv = norm_adv
        self.vf_coef = vf_coef
        self.metrics = torch.zeros(16, dtype=torch.float64, device=self.device)
        self._ws = {}

    def hparams(self, global_rows, reward_horizon=4, loss_scale=1.0, l2_deferred=False, old_values=None):
        """old_values: the rollout's value pass (fp32 [S*E] by sample), read by the clipped value loss when
        clip_vloss_coef is set (diffusion_ppo.py:110-116)."""
        return ops.ppo_hparams(self.gamma_denoising, self.clip_ploss_coef, self.clip_ploss_coef_base,
                               self.clip_ploss_coef_rate, self.min_logprob_denoising_std, self.vf_coef, self.norm_adv,
                               reward_horizon, loss_scale, global_rows, l2_deferred=l2_deferred,
                               learn_eta=self.learn_eta, clip_vloss_coef=self.clip_vloss_coef,
                               old_values=old_values if self.clip_vloss_coef is not None else None)

    def workspace(self, rows):
        ws = self._ws.get(rows)
        if ws is None:
            ws = self._ws[rows] = ops.ppo_workspace(self.dims, self.precision, rows, self.device)
        return ws

    def minibatch(self, obs, chains, lp_old_mean, advantages, returns, perm_seed, epoch, start, rows,
                  global_rows=None, reward_horizon=4, loss_scale=1.0, adv_stats=None, row_index=None, part=None,
                  metrics=None, old_values=None):
        """One fused PPO minibatch over HBM rollout buffers (obs [N,SD], chains [N,K'+1,XD],
        lp_old_mean [N,K'], advantages/returns [N]); writes self.grads and self.metrics (sums).
        part = 1 / 2 runs only the actor / critic half on the current stream (metrics: an
        alternative fp64[16] buffer)."""
        hp = self.hparams(global_rows or rows, reward_horizon, loss_scale, old_values=old_values)
        ops.ppo_minibatch(self.dims, self.precision, hp, self.packed_ft, self.packed_critic, self.actor_ft_params,
                          self.sched, obs, chains, lp_old_mean, advantages, returns, perm_seed, epoch, start, rows,
                          self.workspace(rows), self.grads, self.metrics if metrics is None else metrics,
                          adv_stats=adv_stats, row_index=row_index, part=part)

    def bind_minibatch(self, obs, chains, lp_old_mean, advantages, returns, perm_seed, max_rows, reward_horizon=4,
                       loss_scale=1.0, l2_deferred=False, old_values=None):
        """minibatch() over fixed rollout buffers for a whole update phase, its arguments validated
        and marshalled once (ops.BoundMinibatch): returns f(epoch, start, rows, global_rows=None,
        adv_stats=None, part=None, metrics=None). Every minibatch uses the max_rows workspace.
        l2_deferred: the actor's l2 gradient stays factored for an optimizer step with l2_from_pl2."""
        bound = ops.BoundMinibatch(self.dims, self.precision, self.packed_ft, self.packed_critic, self.actor_ft_params,
                                   self.sched, obs, chains, lp_old_mean, advantages, returns, perm_seed,
                                   self.workspace(max_rows), self.grads, max_rows)
        hps = {}

        def run(epoch, start, rows, global_rows=None, adv_stats=None, part=None, metrics=None, stream=None,
                precleared=False):
            # precleared (ABI 11, DPPO_PPO_PRECLEARED): the optimizer step before this call already
            # zeroed what the part would zero first (its gradients and ops.ClearRanges for these rows)
            g = int(global_rows or rows)
            hp = hps.get((g, precleared))
            if hp is None:
                hp = hps[(g, precleared)] = self.hparams(g, reward_horizon, loss_scale, l2_deferred=l2_deferred,
                                                         old_values=old_values)
                if precleared:
                    hp.flags |= _lib.DPPO_PPO_PRECLEARED
            bound(hp, epoch, start, rows, self.metrics if metrics is None else metrics, adv_stats=adv_stats, part=part,
                  stream=stream)
        return run

    def bc_loss(self, obs, *, x_T=None, noise=None):
        """The behaviour-cloning term of c_loss (diffusion_ppo.py:63-71): chains of the frozen base policy
        for these observations (every denoising step on the base actor, use_base_policy=True), their
        log-probs under actor_ft (:343-425) clipped to [-5, 2], negated mean over every element. The agent
        reports it but leaves it out of the loss (train_ppo_diffusion_agent.py:340-342), so it has no
        gradient here. Its Philox draws use a call counter of their own (high call ids), so the rollout's
        noise does not depend on use_bc_loss; x_T / noise inject the draws (tests)."""
        state = _as_state(obs, self.device, self.dims.sd)
        n = state.shape[0]
        calls = getattr(self, "_bc_calls", 0)
        _, ch = ops.sample(self.dims, self.precision, self.packed_base, self.packed_base, self.sched_for(False), state,
                           x_T=x_T, noise=noise, seed=self.seed, call_id=(1 << 40) + calls,
                           env_offset=self._env_offset, deterministic=False,
                           min_sampling_std=self.get_min_sampling_denoising_std(), randn_clip=self.randn_clip_value,
                           final_clip=self.final_action_clip_value, want_chains=True)
        self._bc_calls = calls + 1
        lp = self.get_logprobs(state, ch.view(n, self.ft_denoising_steps + 1, self.dims.xd))
        return -float(lp.clamp(-5, 2).mean())

    def c_loss(self, obs, chains_prev, chains_next, denoising_inds, returns, oldvalues, advantages, oldlogprobs,
               use_bc_loss=False, reward_horizon=4):
        """diffusion_ppo.py:32-132 on an explicit batch. Returns (pg_loss, entropy_loss, v_loss, clipfrac,
        approx_kl, ratio, bc_loss, eta) as floats; gradients are left in self.grads (of pg_loss +
        vf_coef v_loss: the agent's loss, train_ppo_diffusion_agent.py:340-342; bc_loss is reported only)."""
        bc = self.bc_loss(obs) if use_bc_loss else 0.0   # :63-71
        dev = self.device
        state = _as_state(obs, dev, self.dims.sd)
        b = state.shape[0]
        kf, xd = self.ft_denoising_steps, self.dims.xd
        j = torch.as_tensor(denoising_inds, device=dev).long().reshape(b)
        r = torch.arange(b, device=dev)
        ch = torch.zeros(b, kf + 1, xd, dtype=torch.float32, device=dev)
        ch[r, j] = torch.as_tensor(chains_prev, device=dev, dtype=torch.float32).reshape(b, xd)
        ch[r, j + 1] = torch.as_tensor(chains_next, device=dev, dtype=torch.float32).reshape(b, xd)
        old = torch.as_tensor(oldlogprobs, device=dev, dtype=torch.float32)
        if old.dim() == 3:  # per element [b, Ta, Da]: clip to [-5, 2] and mean over the horizon (:50-59)
            old = old.clamp(-5, 2)[:, :reward_horizon].mean(dim=(1, 2))
        lp_old = torch.zeros(b, kf, dtype=torch.float32, device=dev)
        lp_old[r, j] = old.reshape(b)
        adv = torch.as_tensor(advantages, device=dev, dtype=torch.float32).reshape(b).contiguous()
        ret = torch.as_tensor(returns, device=dev, dtype=torch.float32).reshape(b).contiguous()
        row_index = (r * kf + j).contiguous()
        oldv = None
        if self.clip_vloss_coef is not None:   # :110-116: sample n = row r of this batch
            oldv = torch.as_tensor(oldvalues, device=dev, dtype=torch.float32).reshape(b).contiguous()
        self.minibatch(state, ch, lp_old, adv, ret, 0, 0, 0, b, reward_horizon=reward_horizon, row_index=row_index,
                       old_values=oldv)
        m = (self.metrics[:5] / b).cpu().numpy()
        eta = self.current_eta()
        # entropy_loss = -mean(eta), the last element mean(eta) (diffusion_ppo.py:49, 131); with
        # learn_eta, d loss / d eta is left in self.metrics[M_DETA]
        return (float(m[M_PG]), -eta, float(m[M_VLOSS]), float(m[M_CLIPFRAC]), float(m[M_KL]), float(m[M_RATIO]),
                bc, eta)
