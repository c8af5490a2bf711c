"""Rank bodies for tests/test_dist_cpu.py (gloo, world_size 2 / 4 / 8). Kept in their own module so the
spawned processes import them without re-running the test module. Each body asserts against the
single-process oracle on the full (un-sharded) data; mp.spawn re-raises a failure in the parent."""
import os

import numpy as np
import torch
import torch.distributed as dist

from oracle import dppo_oracle as O


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _flat(g):
    return np.concatenate([np.asarray(g[k], np.float64).ravel() for k in sorted(g)])


def reward_rms(rank, world, port):
    """Reward-RMS over env shards == the oracle scaler on the whole env batch, two calls in a row
    (return state carries over)."""
    from diffusionpolicyoptimization_amd.util import dist as D
    _init(rank, world, port)
    rng = np.random.default_rng(7)
    S, E = 37, 16
    n_loc, off = D.shard_envs(E, world, rank)
    ref = O.RunningRewardScalerOracle(E)
    rms = (0.0, 1.0, 1e-4)
    ret_loc = np.zeros(n_loc)
    for call in range(2):
        reward = rng.normal(0.3, 1.5, (S, E))
        first = (rng.random((S, E)) < 0.05).astype(np.float64)
        want = ref(reward.T, first.T)                       # [E, S]
        rets = np.zeros((S, n_loc))
        prev = ret_loc
        for t in range(S):
            prev = rets[t] = reward[t, off:off + n_loc] + (1 - first[t, off:off + n_loc]) * 0.99 * prev
        ret_loc = rets[-1]
        x = rets.ravel()
        local = torch.tensor([x.size, x.mean(), ((x - x.mean()) ** 2).sum()], dtype=torch.float64)
        n, mean, m2 = D.gather_moments(local)
        rms = D.rms_update(rms, n, mean, m2)
        np.testing.assert_allclose([rms[0], rms[1], rms[2]], [ref.mean, ref.var, ref.count], rtol=1e-12)
        got = np.clip(reward[:, off:off + n_loc] / np.sqrt(rms[1] + 1e-8), -10, 10)
        np.testing.assert_allclose(got.T, want[off:off + n_loc], rtol=1e-12)
    dist.destroy_process_group()


def dp_gradient(rank, world, port):
    """Per-shard PPO gradients with global advantage moments and 1/B_global scaling, summed over
    ranks, == the full-minibatch oracle gradient (and metrics)."""
    from diffusionpolicyoptimization_amd.util import dist as D
    _init(rank, world, port)
    rng = np.random.default_rng(11)
    Do, Ta, Da, K, kf = 11, 4, 3, 20, 10
    base = {k: np.asarray(v, np.float64) for k, v in O.init_actor(rng, Do, Da, Ta, bias_scale=0.05).items()}
    critic = {k: np.asarray(v, np.float64) for k, v in O.init_critic(rng, Do, bias_scale=0.05).items()}
    sched = O.ddpm_schedule(K)
    B = 24
    obs = rng.uniform(-1, 1, (B, 1, Do))
    cp = rng.normal(0, .5, (B, Ta, Da))
    cn = cp + rng.normal(0, .05, (B, Ta, Da))
    j = rng.integers(0, kf, B)
    ret = rng.normal(size=B)
    adv = rng.normal(0.2, 1.3, B)
    # old log-probs near the new ones so both clip branches occur
    oldlp = rng.normal(0, 0.02, B) + _row_logprob(base, sched, obs, cp, cn, j, kf)
    full_m, full_a, full_c = O.c_loss(base, critic, sched, obs, cp, cn, j, ret, None, adv, oldlp, kf)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    a_loc = adv[sl]
    st = D.allreduce_sum_(torch.tensor([a_loc.size, a_loc.sum(), (a_loc ** 2).sum()], dtype=torch.float64))
    am, asd = D.adv_norm_from_stats(st)
    m, ga, gc = O.c_loss(base, critic, sched, obs[sl], cp[sl], cn[sl], j[sl], ret[sl], None, a_loc, oldlp[sl], kf,
                         adv_mean_std=(am, asd), denom=B)
    g = D.allreduce_sum_(torch.tensor(np.concatenate([_flat(ga), _flat(gc)])))
    want = np.concatenate([_flat(full_a), _flat(full_c)])
    np.testing.assert_allclose(g.numpy(), want, rtol=1e-9, atol=1e-12 * np.abs(want).max())
    keys = ("pg_loss", "v_loss", "approx_kl", "clipfrac", "ratio")
    mt = D.allreduce_sum_(torch.tensor([m[k] for k in keys], dtype=torch.float64))
    np.testing.assert_allclose(mt.numpy(), [full_m[k] for k in keys], rtol=1e-9, atol=1e-14)
    assert 0 < full_m["clipfrac"] < 1, "test data should exercise both clip branches"
    dist.destroy_process_group()


def _row_logprob(p, sched, obs, cp, cn, j, kf, horizon=4):
    t = kf - 1 - np.asarray(j)
    eps, _ = O.diffusion_mlp_forward(p, cp, t, obs)
    mu, logvar, _ = O.p_mean_var(sched, eps, cp, t)
    std = np.clip(np.exp(0.5 * logvar), 0.1, 1e6)
    return np.clip(O.gaussian_logprob(cn, mu, std), -5, 2)[:, :horizon].mean(axis=(1, 2))


def episodes_and_ev(rank, world, port):
    """Episode statistics and explained variance summed over env shards == the oracle on all envs."""
    from diffusionpolicyoptimization_amd.agent.finetune.train_ppo_diffusion_agent import (episode_stats_from_sums,
                                                                                          episode_sums)
    from diffusionpolicyoptimization_amd.util import dist as D
    _init(rank, world, port)
    rng = np.random.default_rng(3)
    S, E, act_steps = 60, 16, 4
    firsts = (rng.random((S + 1, E)) < 0.08).astype(np.float64)
    firsts[0] = 1
    rew = rng.normal(1.0, 2.0, (S, E))
    n_loc, off = D.shard_envs(E, world, rank)
    sums = D.allreduce_sum_(torch.tensor(episode_sums(firsts[:, off:off + n_loc], rew[:, off:off + n_loc],
                                                      act_steps, 3.0), dtype=torch.float64))
    got = episode_stats_from_sums(sums.tolist())
    want = O.episode_stats(firsts, rew, act_steps, 3.0)
    assert got["num_episode_finished"] == want["num_episode_finished"] > 0
    for k in ("avg_episode_reward", "avg_best_reward", "success_rate"):
        np.testing.assert_allclose(got[k], want[k], rtol=1e-12)
    vals = rng.normal(size=(S, E))
    rets = vals + rng.normal(0, 0.4, (S, E))
    ev = D.explained_variance(torch.tensor(vals[:, off:off + n_loc]).reshape(-1),
                              torch.tensor(rets[:, off:off + n_loc]).reshape(-1))
    np.testing.assert_allclose(ev, O.explained_variance(vals.ravel(), rets.ravel()), rtol=1e-10)
    # the agent's path: per-rank moments (what dppo_value_moments stores) summed over ranks
    y, d = rets[:, off:off + n_loc].ravel(), (rets - vals)[:, off:off + n_loc].ravel()
    mom = [y.sum(), (y * y).sum(), d.sum(), (d * d).sum(), float(y.size)]
    ev2 = D.explained_variance_from_moments(mom, torch.device("cpu"), group=dist.group.WORLD)
    np.testing.assert_allclose(ev2, O.explained_variance(vals.ravel(), rets.ravel()), rtol=1e-10)
    dist.destroy_process_group()
