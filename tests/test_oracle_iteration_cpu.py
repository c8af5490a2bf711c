"""CPU checks of the whole-iteration oracle (oracle/iteration.py) and the CPU baseline
(oracle/cpu_reference.py): the loop semantics the GPU parity test relies on."""
import numpy as np

from oracle import dppo_oracle as O
from oracle.iteration import PPODiffusionLoopOracle, SyntheticVecEnvOracle
from tests.helpers import HOPPER, make_models


def _spec(d):
    td, h, xd = d["time_dim"], d["actor_hidden"], d["horizon_steps"] * d["action_dim"]
    ain = xd + td + d["obs_dim"]
    a = [("time_w1", (td, 2 * td)), ("time_b1", (2 * td,)), ("time_w2", (2 * td, td)), ("time_b2", (td,)),
         ("in_w", (ain, h)), ("in_b", (h,)), ("l1_w", (h, h)), ("l1_b", (h,)), ("l2_w", (h, h)), ("l2_b", (h,)),
         ("out_w", (h, xd)), ("out_b", (xd,))]
    hc = d["critic_hidden"]
    c = [("in_w", (d["obs_dim"], hc)), ("in_b", (hc,)), ("l1_w", (hc, hc)), ("l1_b", (hc,)), ("l2_w", (hc, hc)),
         ("l2_b", (hc,)), ("out_w", (hc, 1)), ("out_b", (1,))]
    return a, c


def _loop(target_kl=1.0, val_freq=3, S=12, E=2, max_ep=24, batch=60):
    base, ft, critic = make_models(seed=1)
    a_spec, c_spec = _spec(HOPPER)
    env = SyntheticVecEnvOracle(np.arange(E) + 42, 11, 3, 4, max_ep)
    return PPODiffusionLoopOracle(base, ft, critic, a_spec, c_spec, O.ddpm_schedule(20), env, seed=42, perm_seed=7,
                                  n_steps=S, ft_steps=10, act_steps=4, horizon_steps=4, action_dim=3,
                                  val_freq=val_freq, batch_size=batch, update_epochs=2, target_kl=target_kl)


def test_oracle_loop_resets_only_on_eval_and_counts_episodes():
    orc = _loop()
    outs = [orc.iteration() for _ in range(4)]
    assert [o["eval"] for o in outs] == [True, False, False, True]
    # eval iterations reset (firsts[0] = 1); train iterations continue (quirk 4)
    assert (outs[0]["firsts"][0] == 1).all() and (outs[3]["firsts"][0] == 1).all()
    for i in (1, 2):
        np.testing.assert_array_equal(outs[i]["firsts"][0], outs[i - 1]["firsts"][-1])
    # 6-chunk episodes in 12-step iterations: episodes complete inside each iteration
    assert outs[0]["episodes"]["num_episode_finished"] > 0
    # a train iteration changes the parameters; an eval one does not
    th = orc.theta.copy()
    orc.iteration()      # itr 4: train
    assert np.abs(orc.theta - th).max() > 0


def test_oracle_loop_kl_stop_applies_one_minibatch_per_epoch():
    orc = _loop(target_kl=-1.0)
    orc.iteration()
    orc.iteration()
    assert orc.n_updates == 2            # update_epochs = 2, each epoch stops after its first minibatch


def test_cpu_reference_runs_an_iteration():
    from oracle import cpu_reference as C
    t, br = C.time_iteration(4, 3, 60, update_epochs=1, threads=2, warm_steps=1)
    assert t > 0 and br["minibatches"] == 2 and br["minibatches_full"] == 2
    assert C.cpu_model() and (C.physical_cores() or 1) >= 1
