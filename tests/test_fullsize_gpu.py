"""Full-size per-GPU shards of BASELINE configs 2-5 through the agent on the HIP path: one train
iteration at the config's own size (reference agent/finetune/train_ppo_diffusion_agent.py:58-377,
model/diffusion/diffusion_ppo.py:32-132), checked by properties and against the oracle on sampled
rows.

  * config 2 (the benchmarked workload: hopper, 64 envs x 500 chunks, bf16 denoiser, 5 epochs x 6
    minibatches of 50,000 rows = 30 applied);
  * config 3 / 4 (walker2d / halfcheetah dims: Do 17, Da 6, XD = 24; the per-GPU shard of the
    8-GPU halfcheetah run is the same 256 envs): 256 envs x 500 chunks, bf16 denoiser;
  * config 5 (hopper DDIM, 10 rows over K = 20, fp16; the per-GPU shard of the 4096-env run):
    512 envs x 500 chunks.

Checks:
  * every minibatch of every epoch applied: n_updates = update_epochs x floor(S E K' / b)
    (target_kl lifted so no early stop can hide a skipped minibatch), parameters finite and moved;
  * the value pass and the old-log-prob pass (agent :191-229) on 256 sampled rollout samples
    against the oracle (rounding operands as the kernels do) with the pre-update parameters;
  * the reward scaler + GAE (agent :232-263) over ALL S x E entries against the oracle given the
    GPU's own values and the raw rewards (fp64 scans: the advantages match to fp32 storage);
  * explained variance (agent :373-377) against the oracle's formula on the same values/returns.
"""
import os

import numpy as np
import pytest

from oracle import dppo_oracle as O
from tests.helpers import to_f64

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [("hopper-v2", "ft_ppo_diffusion_mlp_64env", "bf16", 64, O.round_bf16),
         ("walker2d-v2", "ft_ppo_diffusion_mlp", "bf16", 256, O.round_bf16),
         ("hopper-v2", "ft_ppo_diffusion_mlp_ddim", "fp16", 512, O.round_fp16)]


@pytest.mark.parametrize("sub,name,precision,E,rnd", CASES,
                         ids=["hopper-config2-64env-bf16", "walker-config3-4-256env-bf16", "ddim-config5-512env-fp16"])
def test_full_size_train_iteration(cuda, tmp_path, sub, name, precision, E, rnd):
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune", sub), name,
                      ["train.force_train=True", "train.n_train_itr=2", "train.target_kl=1000000000.0",
                       f"logdir={tmp_path}", "train.save_checkpoints=false", "train.save_results=false"])
    a = get_class(cfg._target_)(cfg)
    m = a.model
    d = m.dims
    assert m.precision == precision and a.n_envs == E and a.n_steps == 500
    S, kf, na = a.n_steps, m.ft_denoising_steps, m.n_actor
    p0 = m.train_params.cpu().numpy()
    res = a.iteration()
    torch.cuda.synchronize()
    p1 = m.train_params.cpu().numpy()

    n_mb = a.update_epochs * max(1, S * E * kf // a.batch_size)
    assert a.timing["n_updates"] == n_mb, (a.timing["n_updates"], n_mb)
    assert np.isfinite(p1).all() and np.abs(p1 - p0).max() > 0
    for k in ("pg_loss", "v_loss", "approx_kl", "explained_var"):
        assert np.isfinite(res[k]), (k, res[k])

    # value / old-log-prob passes on sampled samples, pre-update parameters
    ft0 = to_f64(ops.unflatten_params(m.actor_spec, p0[:na]))
    critic0 = to_f64(ops.unflatten_params(m.critic_spec, p0[na:]))
    if d.time_stride > 1:
        sched = O.ddim_schedule(d.denoising_steps * d.time_stride, d.denoising_steps, m.ddim_eta)
    else:
        sched = O.ddpm_schedule(d.denoising_steps)
    pick = np.random.default_rng(7).choice(S * E, 256, replace=False)
    obs = a.obs_traj.view(S * E, -1).cpu().numpy()[pick].astype(np.float64)
    chains = a.chains_traj.view(S * E, kf + 1, -1).cpu().numpy()[pick].astype(np.float64)
    v_ref = O.critic_forward(critic0, obs.reshape(-1, 1, d.sd), rnd=rnd)[0][:, 0]
    v_got = a.values.cpu().numpy()[pick]
    assert np.abs(v_got - v_ref).max() <= 2e-3 * max(1.0, np.abs(v_ref).max()), np.abs(v_got - v_ref).max()
    lp = O.get_logprobs(ft0, sched, obs.reshape(-1, 1, d.sd), chains.reshape(-1, kf + 1, d.horizon_steps, d.action_dim),
                        kf, m.min_logprob_denoising_std, rnd=rnd)
    lp_ref = np.clip(lp, -5, 2)[:, :a.reward_horizon].mean(axis=(1, 2)).reshape(-1, kf)
    lp_got = a.lp_old.cpu().numpy()[pick]
    assert np.abs(lp_got - lp_ref).max() <= 2e-3, np.abs(lp_got - lp_ref).max()

    # reward scaler + GAE over the whole rollout, from the GPU's values and the raw rewards
    values = a.values.view(S, E).cpu().numpy().astype(np.float64)
    rewards = a.reward_pin.numpy().astype(np.float64)
    firsts = a.firsts[:-1]
    scaled = O.RunningRewardScalerOracle(E)(rewards.T, firsts.T).T
    adv_ref, ret_ref = O.gae(scaled, values, a.last_values.cpu().numpy().astype(np.float64), a.term_pin.numpy(),
                             a.gamma, a.gae_lambda, a.reward_scale_const)
    adv, ret = a.adv.cpu().numpy(), a.ret.cpu().numpy()
    assert np.abs(adv - adv_ref).max() <= 1e-5 * np.abs(adv_ref).max(), np.abs(adv - adv_ref).max()
    assert np.abs(ret - ret_ref).max() <= 1e-5 * np.abs(ret_ref).max(), np.abs(ret - ret_ref).max()
    ev_ref = O.explained_variance(values.reshape(-1), ret_ref.reshape(-1))
    assert abs(res["explained_var"] - ev_ref) <= 1e-4 * max(1.0, abs(ev_ref)), (res["explained_var"], ev_ref)
