"""VPGDiffusion (reference model/diffusion/diffusion_vpg.py:27-481) on MI355X.

State lives in HBM as flat fp32 buffers in the Keras layout (include/dppo.h):
  base_params   frozen pretrained actor                       (diffusion_vpg.py:100-102)
  train_params  [actor_ft | critic], the variables the single AdamW updates (quirk 2)
plus their packed MFMA fragment images (bf16 or fp32) that the kernels read. Every forward runs
in a fused HIP kernel: the K-step sampler (dppo_sample), the chain log-prob pass (dppo_logprob),
the critic value pass (dppo_critic_forward); the PPO loss/gradient is PPODiffusion.c_loss."""
import copy
import logging
import os

import numpy as np
import torch

from ... import ops
from ...util import keras_weights
from .diffusion import DiffusionModel, Sample

log = logging.getLogger(__name__)


def _as_state(cond, device, sd):
    x = cond["state"] if isinstance(cond, dict) else cond
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(np.asarray(x, np.float32))
    x = x.to(device=device, dtype=torch.float32)
    return x.reshape(x.shape[0], sd).contiguous()


class VPGDiffusion(DiffusionModel):
    def __init__(self, actor, critic, ft_denoising_steps, ft_denoising_steps_d=0, ft_denoising_steps_t=0,
                 network_path=None, min_sampling_denoising_std=0.1, min_logprob_denoising_std=0.1, eta=None,
                 learn_eta=False, **kwargs):
        eta_cfg = self._eta_config(eta)
        super().__init__(network=actor, network_path=network_path, ddim_eta=eta_cfg["base_eta"], **kwargs)
        # "Cannot learn eta with DDPM." (diffusion_vpg.py:52)
        assert not (learn_eta and not self.use_ddim), "Cannot learn eta with DDPM."
        assert ft_denoising_steps <= self.sampling_steps
        self.ft_denoising_steps = int(ft_denoising_steps)
        self.ft_denoising_steps_d = ft_denoising_steps_d
        self.ft_denoising_steps_t = ft_denoising_steps_t
        self.ft_denoising_steps_cnt = 0
        self.min_sampling_denoising_std = min_sampling_denoising_std
        self.min_logprob_denoising_std = min_logprob_denoising_std
        self.learn_eta = bool(learn_eta)
        if self.learn_eta:
            self._init_learnable_eta(eta_cfg)
        self.actor = actor
        self.critic = critic
        critic._owner = self
        cond_steps = actor.cond_dim // self.obs_dim
        self.dims = ops.ModelDims(obs_dim=self.obs_dim, action_dim=self.action_dim,
                                  horizon_steps=self.horizon_steps, cond_steps=cond_steps, time_dim=actor.time_dim,
                                  actor_hidden=actor.hidden, critic_hidden=critic.hidden,
                                  denoising_steps=self.sampling_steps, ft_denoising_steps=self.ft_denoising_steps,
                                  time_stride=self.time_stride)
        self.actor_spec = ops.actor_param_spec(self.dims)
        self.critic_spec = ops.critic_param_spec(self.dims)
        self.n_actor = ops.spec_count(self.actor_spec)
        self.n_critic = ops.spec_count(self.critic_spec)
        rng = np.random.default_rng(self.seed)
        base = self._load_actor(network_path, rng)
        critic_p = critic.init_params(np.random.default_rng(self.seed + 1))  # fresh critic (:109-110)
        dev = self.device
        self.base_params = torch.tensor(ops.flatten_params(self.actor_spec, base), device=dev)
        self.train_params = torch.empty(self.n_actor + self.n_critic, dtype=torch.float32, device=dev)
        self.train_params[:self.n_actor].copy_(self.base_params)  # actor_ft = deepcopy(actor) (:95-97)
        self.train_params[self.n_actor:].copy_(torch.tensor(ops.flatten_params(self.critic_spec, critic_p)))
        # gradients + an 8-float tail: the data-parallel agent reduces the minibatch metrics in the
        # same all-reduce as the gradients (one collective per minibatch)
        self.grads_ext = torch.zeros(self.train_params.numel() + 8, dtype=torch.float32, device=dev)
        self.grads = self.grads_ext[:self.train_params.numel()]
        self.packed_base = ops.pack_actor(self.dims, self.base_params, self.precision)
        self.packed_ft = torch.empty_like(self.packed_base)
        self.packed_critic = torch.empty(ops.critic_packed_bytes(self.dims, self.precision), dtype=torch.uint8,
                                         device=dev)
        self.repack()
        self._call_id = 0
        self._env_offset = 0
        log.info("Number of finetuned parameters: %d (actor_ft) + %d (critic)", self.n_actor, self.n_critic)

    @staticmethod
    def _eta_config(eta):
        """eta of the DDIM mean/variance: a number, or an EtaFixed-style config {base_eta, min_eta,
        max_eta} (the original DPPO's model.diffusion.eta.EtaFixed; defaults 1 / 0.1 / 1)."""
        if eta is None:
            return dict(base_eta=1.0, min_eta=0.1, max_eta=1.0)
        if isinstance(eta, (int, float)):
            return dict(base_eta=float(eta), min_eta=0.1, max_eta=1.0)
        if hasattr(eta, "get") and eta.get("base_eta") is not None:
            return dict(base_eta=float(eta.get("base_eta")), min_eta=float(eta.get("min_eta", 0.1)),
                        max_eta=float(eta.get("max_eta", 1.0)))
        raise ValueError(f"eta must be a number or an EtaFixed config with base_eta, got {eta!r}")

    def _init_learnable_eta(self, cfg):
        """learn_eta (§8(f) row 4, PARITY UNPINNED: the reference's eta module, model/diffusion/eta.py
        of the original DPPO, is absent and its eta step is commented out): EtaFixed's one scalar,
        eta = min + (max - min) (tanh(logit) + 1) / 2, logit initialised at base_eta. The device state
        {logit, m, v} is stepped by dppo_eta_step, which also re-derives the DDIM rows of self.sched
        (train-mode sampling and every log-prob), so the table always holds the current eta."""
        lo, hi, base = cfg["min_eta"], cfg["max_eta"], cfg["base_eta"]
        if not lo < base < hi:
            raise ValueError(f"learn_eta: base_eta {base} must lie strictly inside (min_eta {lo}, max_eta {hi})")
        self.eta_min, self.eta_max = lo, hi
        logit = float(np.arctanh(2.0 * (base - lo) / (hi - lo) - 1.0))
        dev = self.device
        self.eta_state = torch.tensor([logit, 0.0, 0.0], dtype=torch.float32, device=dev)
        self.eta_value = torch.zeros(1, dtype=torch.float32, device=dev)
        dd = {k: getattr(self, k) for k in ("ddim_alphas_prev", "ddim_sqrt_alphas_prev", "ddim_sqrt_alphas",
                                            "ddim_sqrt_1m_alphas", "ddim_sfac")}
        self.eta_base = torch.tensor(ops.ddim_eta_base(dd), device=dev)
        self.eta_step_count = 0
        self.refresh_eta()

    def refresh_eta(self):
        """Re-derive the eta columns of the train-mode DDIM table from the current logit (no step)."""
        ops.eta_step(self.eta_state, None, 0, 0.0, 0.0, self.eta_min, self.eta_max, self.eta_base, self.sched,
                     eta_out=self.eta_value)

    def eta_optimizer_step(self, metrics, lr, weight_decay, beta1=0.9, beta2=0.999, eps=1e-7):
        """One AdamW step of the eta logit from metrics[8] (d loss / d eta of a learn_eta minibatch,
        the gradient the reference's eta_optimizer would apply, agent :358-359)."""
        self.eta_step_count += 1
        ops.eta_step(self.eta_state, metrics, self.eta_step_count, lr, weight_decay, self.eta_min, self.eta_max,
                     self.eta_base, self.sched, eta_out=self.eta_value, beta1=beta1, beta2=beta2, eps=eps)

    def current_eta(self):
        """eta of the train-mode DDIM rows (c_loss's `eta` metric, diffusion_ppo.py:131)."""
        if self.learn_eta:
            return float(self.eta_value.item())
        return self.ddim_eta if self.use_ddim else 1.0

    # ------------------------------------------------------------------ parameters
    @property
    def actor_ft_params(self):
        return self.train_params[:self.n_actor]

    @property
    def critic_params(self):
        return self.train_params[self.n_actor:]

    @property
    def trainable_variables(self):
        return [self.train_params]

    def repack(self, part=None):
        """Re-derive the packed fragment images of actor_ft (part 1) and/or critic (part 2) after an
        optimiser step."""
        if part is None:               # both images in one launch
            ops.pack_all(self.dims, self.precision, self.actor_ft_params, self.packed_ft, self.critic_params,
                         self.packed_critic)
        elif part == 1:
            ops.pack_actor(self.dims, self.actor_ft_params, self.precision, out=self.packed_ft)
        elif part == 2:
            ops.pack_critic(self.dims, self.critic_params, self.precision, out=self.packed_critic)

    def _load_actor(self, path, rng):
        # network_path: null is the only way to ask for synthetic weights; a path that does not
        # exist fails here as the reference's load_weights does (diffusion_vpg.py:91-97), instead of
        # silently fine-tuning a random actor
        if path is None:
            log.info("base policy: seeded glorot_uniform actor (synthetic weights, network_path: null)")
            return self.network.init_params(rng)
        path = str(path)
        if not os.path.exists(path):
            raise FileNotFoundError(f"base policy checkpoint {path!r} does not exist (set network_path / "
                                    "base_policy_path to null for seeded synthetic weights)")
        if path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as f:
                keys = [k for k in f.files]
                pref = "actor." if any(k.startswith("actor.") for k in keys) else ""
                return {n: np.asarray(f[pref + n], np.float32).reshape(s) for n, s in self.actor_spec}
        if path.endswith(".h5"):          # Keras-3 weights of a DiffusionMLP (pretrain checkpoint)
            return keras_weights.load_actor(path, self.actor_spec)
        raise ValueError(f"unsupported checkpoint format: {path}")

    def _eta_checkpoint(self):
        """The learnable eta's state for a checkpoint: {logit, m, v, step} (None without learn_eta).
        The original DPPO saves the eta module's logit with the model; m, v and the step count make
        a resumed run continue the eta optimizer exactly."""
        if not self.learn_eta:
            return None
        logit, m, v = (float(x) for x in self.eta_state.detach().cpu().numpy())
        return {"logit": logit, "m": m, "v": v, "step": int(self.eta_step_count)}

    def _restore_eta(self, eta):
        if eta is None or not self.learn_eta:
            return
        self.eta_state.copy_(torch.tensor([eta["logit"], eta["m"], eta["v"]], dtype=torch.float32))
        self.eta_step_count = int(eta["step"])
        self.refresh_eta()     # the train-mode DDIM table follows the restored logit

    def save_weights(self, path):
        """PPODiffusion.save_weights: a Keras-3 weights file for *.h5 (actor/, actor_ft/, critic/;
        agent/finetune/train_agent.py:127-133), else .npz with actor./actor_ft./critic. keys. A
        learn_eta model also saves its eta (eta/ group, or eta.state / eta.step keys)."""
        eta = self._eta_checkpoint()
        if str(path).endswith(".h5"):
            sp = lambda spec, flat: ops.unflatten_params(spec, flat.detach().cpu().numpy())
            keras_weights.save_ppo_model(str(path), sp(self.actor_spec, self.base_params),
                                         sp(self.actor_spec, self.actor_ft_params),
                                         sp(self.critic_spec, self.critic_params), eta=eta)
            return
        d = {}
        for prefix, flat, spec in (("actor.", self.base_params, self.actor_spec),
                                   ("actor_ft.", self.actor_ft_params, self.actor_spec),
                                   ("critic.", self.critic_params, self.critic_spec)):
            for n, v in ops.unflatten_params(spec, flat.detach().cpu().numpy()).items():
                d[prefix + n] = v
        if eta is not None:
            d["eta.state"] = np.array([eta["logit"], eta["m"], eta["v"]], np.float32)
            d["eta.step"] = np.array(eta["step"], np.int64)
        np.savez(path, **d)

    def load_weights(self, path):
        if str(path).endswith(".h5"):
            w = keras_weights.load_ppo_model(str(path), self.actor_spec, self.critic_spec)
            for key, flat, spec in (("actor", self.base_params, self.actor_spec),
                                    ("actor_ft", self.actor_ft_params, self.actor_spec),
                                    ("critic", self.critic_params, self.critic_spec)):
                flat.copy_(torch.tensor(ops.flatten_params(spec, w[key])))
            ops.pack_actor(self.dims, self.base_params, self.precision, out=self.packed_base)
            self.repack()
            self._restore_eta(w.get("eta"))
            return
        eta = None
        with np.load(path, allow_pickle=False) as f:
            for prefix, flat, spec in (("actor.", self.base_params, self.actor_spec),
                                       ("actor_ft.", self.actor_ft_params, self.actor_spec),
                                       ("critic.", self.critic_params, self.critic_spec)):
                if all(prefix + n in f.files for n, _ in spec):
                    flat.copy_(torch.tensor(ops.flatten_params(spec, {n: f[prefix + n] for n, _ in spec})))
            if "eta.state" in f.files:
                st = f["eta.state"]
                eta = {"logit": float(st[0]), "m": float(st[1]), "v": float(st[2]),
                       "step": int(f["eta.step"]) if "eta.step" in f.files else 0}
        ops.pack_actor(self.dims, self.base_params, self.precision, out=self.packed_base)
        self.repack()
        self._restore_eta(eta)

    # ------------------------------------------------------------------ annealing (diffusion_vpg.py:114-148)
    def step(self):
        if not isinstance(self.min_sampling_denoising_std, float):
            self.min_sampling_denoising_std.step()
        self.ft_denoising_steps_cnt += 1
        if (self.ft_denoising_steps_d > 0 and self.ft_denoising_steps_t > 0
                and self.ft_denoising_steps_cnt % self.ft_denoising_steps_t == 0):
            self.ft_denoising_steps = max(0, self.ft_denoising_steps - self.ft_denoising_steps_d)
            self.base_params.copy_(self.actor_ft_params)
            self.dims = ops.ModelDims(**{**self.dims.__dict__, "ft_denoising_steps": self.ft_denoising_steps})
            ops.pack_actor(self.dims, self.base_params, self.precision, out=self.packed_base)
            if hasattr(self, "_ws"):
                self._ws.clear()     # PPO workspaces are sized for the old K'
            # the agent re-sizes its K'-shaped rollout buffers before the next iteration
            # (TrainPPODiffusionAgent._fit_buffers_to_model; reference agent :87-95)
            log.info("Finished annealing fine-tuning denoising steps to %d", self.ft_denoising_steps)

    def get_min_sampling_denoising_std(self):
        if isinstance(self.min_sampling_denoising_std, float):
            return self.min_sampling_denoising_std
        return self.min_sampling_denoising_std()

    # ------------------------------------------------------------------ sampler (diffusion_vpg.py:250-339)
    def set_rng(self, seed, env_offset=0):
        """Philox stream of the in-kernel noise: (seed, call counter, global env row)."""
        self.seed = int(seed)
        self._env_offset = int(env_offset)

    def __call__(self, cond, deterministic=False, return_chain=True, use_base_policy=False, *, x_T=None, noise=None,
                 actions_out=None, chains_out=None):
        state = _as_state(cond, self.device, self.dims.sd)
        E = state.shape[0]
        packed_ft = self.packed_base if use_base_policy else self.packed_ft
        acts, chains = ops.sample(
            self.dims, self.precision, self.packed_base, packed_ft, self.sched_for(deterministic), state, x_T=x_T,
            noise=noise,
            seed=self.seed, call_id=self._call_id, env_offset=self._env_offset, deterministic=deterministic,
            min_sampling_std=self.get_min_sampling_denoising_std(), randn_clip=self.randn_clip_value,
            final_clip=self.final_action_clip_value, actions=actions_out, chains=chains_out,
            want_chains=return_chain)
        self._call_id += 1
        traj = acts.view(E, self.horizon_steps, self.action_dim)
        ch = chains.view(E, self.ft_denoising_steps + 1, self.horizon_steps, self.action_dim) if chains is not None else None
        return Sample(traj, ch)

    def bind_rollout(self, cond_host, obs_traj, actions, actions_host, chains_traj):
        """A pre-bound rollout step: step(i, deterministic) copies the pinned observation
        cond_host [E, SD] into obs_traj[i], samples into actions / chains_traj[i] and copies the
        actions into pinned actions_host, then waits for the stream — one FFI call per env step
        (dppo_sample_step). Same Philox stream and call counter as __call__."""
        return ops.SampleStepper(self, cond_host, obs_traj, actions, actions_host, chains_traj)

    # ------------------------------------------------------------------ log-probs (diffusion_vpg.py:343-481)
    def get_logprobs(self, cond, chains, get_ent=False, use_base_policy=False, reduced=False):
        """-> [n*K', Ta, Da] (row = sample*K' + j, t = K'-1-j). reduced=True instead returns the
        clipped mean c_loss uses, [n, K'] (diffusion_ppo.py:50-59)."""
        state = _as_state(cond, self.device, self.dims.sd)
        n = state.shape[0]
        kf = self.ft_denoising_steps
        ch = torch.as_tensor(chains, device=self.device, dtype=torch.float32).reshape(n, kf + 1, self.dims.xd)
        packed = self.packed_base if use_base_policy else self.packed_ft
        lpe, lpm = ops.logprob(self.dims, self.precision, packed, self.sched, state, ch.contiguous(),
                               min_logprob_std=self.min_logprob_denoising_std, want_elem=not reduced,
                               want_mean=reduced)
        if reduced:
            return lpm
        lpe = lpe.view(n * kf, self.horizon_steps, self.action_dim)
        if get_ent:
            return lpe, torch.ones_like(lpe)
        return lpe

    def get_logprobs_subsample(self, cond, chains_prev, chains_next, denoising_inds, get_ent=False,
                               use_base_policy=False):
        """Per-row denoising index j (t = K'-1-j): evaluated by placing each (prev, next) pair at
        chain slots (j, j+1) of a one-sample chain and reading row j of the chain log-probs."""
        state = _as_state(cond, self.device, self.dims.sd)
        b = state.shape[0]
        kf, xd = self.ft_denoising_steps, self.dims.xd
        j = torch.as_tensor(denoising_inds, device=self.device).long().reshape(b)
        ch = torch.zeros(b, kf + 1, xd, dtype=torch.float32, device=self.device)
        r = torch.arange(b, device=self.device)
        ch[r, j] = torch.as_tensor(chains_prev, device=self.device, dtype=torch.float32).reshape(b, xd)
        ch[r, j + 1] = torch.as_tensor(chains_next, device=self.device, dtype=torch.float32).reshape(b, xd)
        lpe = self.get_logprobs(state, ch, use_base_policy=use_base_policy).view(b, kf, self.horizon_steps,
                                                                                 self.action_dim)
        out = lpe[r, j]
        if get_ent:
            return out, torch.ones_like(out)
        return out

    # ------------------------------------------------------------------ critic (critic.py:40-54)
    def critic_values(self, cond):
        state = _as_state(cond, self.device, self.dims.sd)
        return ops.critic_forward(self.dims, self.precision, self.packed_critic, state)
