"""End-to-end agent on the GPU: a few iterations of the debug cfg through the drop-in surface."""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_agent_iterations(cuda, precision, tmp_path):
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      [f"model.precision={precision}", "train.n_steps=20", "train.batch_size=200",
                       "train.n_train_itr=3", "train.val_freq=2", f"logdir={tmp_path}"])
    agent = get_class(cfg._target_)(cfg)
    res = agent.run()
    assert [r["eval"] for r in res] == [True, False, True]
    tr = res[1]
    for k in ("pg_loss", "v_loss", "approx_kl", "explained_var"):
        assert math.isfinite(tr[k]), (k, tr[k])
    assert agent.timing["n_updates"] == 5 * ((20 * 4 * 10) // 200)
    assert agent.actor_optimizer.iterations == agent.timing["n_updates"]
    p = agent.model.train_params.cpu().numpy()
    assert np.isfinite(p).all()
    # agent/finetune/train_agent.py:127-133: a Keras-3 weights file per save, readable back
    ck = os.path.join(tmp_path, "checkpoint", "state_0.weights.h5")
    assert os.path.exists(ck)
    from diffusionpolicyoptimization_amd.util import keras_weights
    w = keras_weights.load_ppo_model(ck, agent.model.actor_spec, agent.model.critic_spec)
    assert set(w) == {"actor", "actor_ft", "critic"}


def test_target_kl_stops_each_epoch_like_the_reference(cuda, tmp_path):
    """The target_kl early stop (agent :366-370): the minibatch whose approx_kl exceeds target_kl
    IS applied and its `break` leaves only that epoch's batch loop (the outer `if flag_break:
    break` is never reached and flag_break is reset per epoch, :284-286), so every epoch still
    applies its first minibatch. The check runs one minibatch behind here; a stop carried over from
    the previous epoch's last minibatch must not drop the next epoch's first one. With
    target_kl = -1 every approx_kl (>= 0) stops: exactly one AdamW step per epoch."""
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      ["model.precision=fp32", "train.n_steps=20", "train.batch_size=200", "train.n_train_itr=2",
                       "train.val_freq=100", "train.target_kl=-1.0", f"logdir={tmp_path}"])
    a = get_class(cfg._target_)(cfg)
    a.run()
    assert a.timing["n_updates"] == a.update_epochs, a.timing["n_updates"]
    assert a.actor_optimizer.iterations == a.update_epochs
    assert np.isfinite(a.model.train_params.cpu().numpy()).all()
    # num_batch = 1: the stop (by the single minibatch of each epoch) is always carried into the
    # next epoch, which must still apply its minibatch
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      ["model.precision=fp32", "train.n_steps=20", "train.batch_size=800", "train.n_train_itr=2",
                       "train.val_freq=100", "train.target_kl=-1.0", f"logdir={tmp_path}/b"])
    a = get_class(cfg._target_)(cfg)
    a.run()
    assert a.timing["n_updates"] == a.update_epochs, a.timing["n_updates"]


def test_envs_reset_only_on_eval_iterations(cuda, tmp_path):
    """the reference assigns last_itr_eval = eval_mode just before testing it
    (agent :70-74), so with reset_at_iteration False the envs are reset only on eval iterations:
    the train iteration right after an eval continues from the eval's env state, with
    firsts[0] = the eval's last done flags."""
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      ["model.precision=fp32", "train.n_steps=20", "train.batch_size=200", "train.n_train_itr=4",
                       "train.val_freq=3", "env.reset_at_iteration=false", "env.max_episode_steps=44",
                       f"logdir={tmp_path}"])
    a = get_class(cfg._target_)(cfg)
    resets = []
    orig = a.reset_env_all

    def counting(*args, **kw):
        resets.append(a.itr)
        return orig(*args, **kw)
    a.reset_env_all = counting
    firsts0, done_before = [], []
    for _ in range(4):
        done_before.append(a.done_venv.copy())
        a.iteration()
        firsts0.append(a.firsts[0].copy())
    assert [r["eval"] for r in a.run_results] == [True, False, False, True]
    assert resets == [0, 3], resets
    # itr 1 and 2 continue: firsts[0] = the previous iteration's final done flags (episodes of
    # 11 chunks end inside a 20-step rollout, so some envs are mid-episode and some just reset)
    for i in (1, 2):
        np.testing.assert_array_equal(firsts0[i], done_before[i].astype(np.float64))
    np.testing.assert_array_equal(firsts0[3], np.ones(a.n_envs))


def test_bound_rollout_step_matches_model_call(cuda):
    """dppo_sample_step (H2D + sampler + D2H in one call) == model(...) on the same Philox draws."""
    import torch

    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      ["model.precision=bf16"])
    model = instantiate(cfg.model, device=cuda, seed=3)
    d = model.dims
    S, E = 3, 40
    obs_pin = torch.empty(E, d.sd, dtype=torch.float32).pin_memory()
    act_pin = torch.empty(E, d.xd, dtype=torch.float32).pin_memory()
    obs_traj = torch.zeros(S, E, d.sd, device=cuda)
    chains = torch.zeros(S, E, d.ft_denoising_steps + 1, d.xd, device=cuda)
    act = torch.empty(E, d.xd, device=cuda)
    step = model.bind_rollout(obs_pin, obs_traj, act, act_pin, chains)
    rng = np.random.default_rng(0)
    for i in range(S):
        o = rng.uniform(-1, 1, (E, d.sd)).astype(np.float32)
        obs_pin.numpy()[:] = o
        cid = model._call_id
        step(i, deterministic=(i == 2))
        got_a = act_pin.numpy().copy()
        model._call_id = cid
        ref = model(torch.tensor(o, device=cuda), deterministic=(i == 2), return_chain=True)
        torch.cuda.synchronize()
        assert model._call_id == cid + 1
        np.testing.assert_array_equal(obs_traj[i].cpu().numpy(), o)
        np.testing.assert_array_equal(got_a, ref.trajectories.reshape(E, -1).cpu().numpy())
        np.testing.assert_array_equal(chains[i].cpu().numpy(), ref.chains.reshape(E, -1, d.xd).cpu().numpy())
    with pytest.raises(IndexError):
        step(S)


@pytest.mark.parametrize("protocol,precision,E", [("tagged", "bf16", 40), ("go", "bf16", 40), ("tagged", "fp32", 40),
                                                  ("tagged", "bf16", 512)])
def test_pipelined_rollout_matches_model_call(cuda, protocol, precision, E, monkeypatch):
    """Pre-enqueued launches fed by the host == model(...), for both observation protocols:
    dppo_rollout_enqueue_tagged (the launch polls tagged observation granules) and
    dppo_rollout_enqueue (a go counter, then the float buffer). At 512 envs the split sampler's
    256 active workgroups fill the device, so the pipe must keep ONE launch in flight (two would
    take CUs each other's members wait for): the co-residency guard of ops.RolloutPipe."""
    import torch

    monkeypatch.setenv("DPPO_ROLLOUT_PROTOCOL", protocol)
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      [f"model.precision={precision}"])
    model = instantiate(cfg.model, device=cuda, seed=5)
    d = model.dims
    S = 4
    obs_traj = torch.zeros(S, E, d.sd, device=cuda)
    chains = torch.zeros(S, E, d.ft_denoising_steps + 1, d.xd, device=cuda)
    act = torch.empty(E, d.xd, device=cuda)
    pipe = ops.RolloutPipe(model, obs_traj, act, chains)
    assert pipe.protocol == protocol
    members = ops.sampler_layout(d, precision, E)
    if members:
        cus = torch.cuda.get_device_properties(cuda).multi_processor_count
        assert len(pipe._tstreams) == min(2, max(1, cus // (members * ((E + 15) // 16))))
    rng = np.random.default_rng(2)
    obs = [rng.uniform(-1, 1, (E, d.sd)).astype(np.float32) for _ in range(S)]
    cid0 = model._call_id
    pipe.obs.numpy()[:] = obs[0]
    pipe.begin()
    pipe.enqueue(0)
    pipe.publish()
    got = []
    for i in range(S):
        if i + 1 < S:
            pipe.enqueue(i + 1)
        pipe.wait()
        got.append(pipe.act.numpy().copy())
        if i + 1 < S:
            pipe.obs.numpy()[:] = obs[i + 1]
            pipe.publish()
    pipe.end()
    torch.cuda.synchronize()
    model._call_id = cid0
    for i in range(S):
        ref = model(torch.tensor(obs[i], device=cuda), return_chain=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(obs_traj[i].cpu().numpy(), obs[i])
        np.testing.assert_array_equal(got[i], ref.trajectories.reshape(E, -1).cpu().numpy())
        np.testing.assert_array_equal(chains[i].cpu().numpy(), ref.chains.reshape(E, -1, d.xd).cpu().numpy())
    pipe.close()


@pytest.mark.parametrize("protocol,threads", [("tagged", 1), ("tagged", 4), ("go", 3)])
def test_pipelined_rollout_matches_model_call_lowdim(cuda, protocol, threads, monkeypatch):
    """The pipelined rollout over the reference's wrapper stack (env/lowdim.py): the gated host step
    dppo_lowdim_step_gated_tagged (slice threads poll their envs' action granules, step, publish
    their observation granules) or dppo_lowdim_step_gated (go counter) drives pre-enqueued sampler
    launches; actions, observations and rewards equal an unpipelined replay (model(obs) -> plain
    one-thread env step) bit for bit, with terminal states and in-wrapper resets inside the run."""
    import torch

    monkeypatch.setenv("DPPO_ROLLOUT_PROTOCOL", protocol)
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.env.lowdim import LinearSimulator, LowdimVecEnv, load_normalization
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp", ["model.precision=bf16"])
    model = instantiate(cfg.model, device=cuda, seed=9)
    d = model.dims
    S, E = 24, 40
    norm = load_normalization(os.path.join(ROOT, "tests", "golden", "hopper_medium_v2_normalization.npz"))

    def make(th):
        sim = LinearSimulator(E, d.obs_dim, d.action_dim, family_seed=1, norm=norm, bound_frac=0.6)
        sim.seed([100 + i for i in range(E)])
        return LowdimVecEnv(sim, E, d.obs_dim, d.action_dim, act_steps=4, n_obs_steps=1, max_episode_steps=40,
                            normalization=norm, num_threads=th)
    venv, ref_env = make(threads), make(1)
    assert venv.num_threads == threads
    obs_traj = torch.zeros(S, E, d.sd, device=cuda)
    chains = torch.zeros(S, E, d.ft_denoising_steps + 1, d.xd, device=cuda)
    act = torch.empty(E, d.xd, device=cuda)
    pipe = ops.RolloutPipe(model, obs_traj, act, chains)
    obs_np = pipe.obs.numpy().reshape(E, 1, d.obs_dim)
    act_view = pipe.act.numpy().reshape(E, 4, d.action_dim)
    obs_np[:] = venv.reset_arg()["state"]
    obs0 = obs_np.copy()
    cid0 = model._call_id
    got_a, got_o, got_r, n_done = [], [], [], 0
    pipe.begin()
    pipe.enqueue(0)
    pipe.publish()
    for i in range(S):
        more = i + 1 < S
        if more:
            pipe.enqueue(i + 1)
        _, r, term, trunc, _ = venv.step(act_view, obs_out=obs_np, gate=pipe.gate(publish=more))
        assert venv.published == more
        if more:
            pipe.published_by_gate()
        got_a.append(act_view.copy())
        got_o.append(obs_np.copy())
        got_r.append(r)
        n_done += int((term | trunc).sum())
    pipe.end()
    torch.cuda.synchronize()
    assert n_done > 0
    model._call_id = cid0
    o = ref_env.reset_arg()["state"]
    np.testing.assert_array_equal(o, obs0)
    for i in range(S):
        np.testing.assert_array_equal(obs_traj[i].cpu().numpy(), o.reshape(E, -1))
        ref = model(torch.tensor(o.reshape(E, -1), device=cuda), return_chain=True)
        a = ref.trajectories.reshape(E, 4, d.action_dim).cpu().numpy()
        # (go protocol: the launch writes its actions into the float buffer itself, and launch i + 1,
        # released by the step's publish, may overwrite it before the test's copy; the observations
        # and rewards below are the actions' downstream check there)
        if protocol == "tagged":
            np.testing.assert_array_equal(got_a[i], a)
        ob, r, _, _, _ = ref_env.step(a)
        o = ob["state"].copy()
        np.testing.assert_array_equal(got_o[i], o)
        np.testing.assert_array_equal(got_r[i], r)
    pipe.close()


@pytest.mark.parametrize("overrides", ["", "train.dp_scale_batch=true"], ids=["reference-batch", "scaled-batch"])
def test_data_parallel_agent_two_ranks_share_one_gpu(tmp_path, overrides):
    """2 ranks (gloo, both on cuda:0) run the DP agent; replicas must stay bit-identical, with the
    reference's global minibatch (default) or batch_size rows per rank (dp_scale_batch)."""
    import socket
    import subprocess
    import sys
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DPPO_DIST_BACKEND="gloo", DPPO_SINGLE_DEVICE="1", DPPO_SMOKE_OVERRIDES=overrides)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "tools", "dist_smoke.py")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "replicas_identical=True" in out.stdout


def test_rccl_runs_the_update_bucket_pattern(cuda):
    """RCCL ("nccl") on the one-GPU box: a world-size-1 process group all-reduces the agent's two
    gradient buckets from the two streams the split update issues them on (tools/rccl_probe.py);
    the results are the inputs (a sum over one rank). Multi-rank RCCL needs more than one GPU."""
    import json
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "tools", "rccl_probe.py")],
                         env=dict(os.environ), capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["backend"] == "nccl" and res["world"] == 1 and res["result_ok"], res


def test_data_parallel_update_equals_single_rank_on_the_union(cuda, tmp_path):
    """SURVEY §8(e) on the HIP path: 2 ranks (gloo, both on cuda:0), reference batch semantics
    (dp_scale_batch = false: the GLOBAL minibatch is batch_size rows, batch_size / 2 drawn by each
    rank from its own shard). Against ONE rank running the same cfg over all 8 envs:
      * the two rollout shards are exactly the single rank's rollout (per-global-env seeds and
        Philox rows), and the advantages / returns (reward-RMS moments Chan-merged over ranks) match;
      * the all-reduced gradient of minibatch 0 equals the single rank's gradient over the union of
        the two ranks' rows (same global 1/batch_size scaling and global advantage moments), up to
        fp summation order."""
    import socket
    import subprocess
    import sys

    import torch

    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dp_equiv import OVERRIDES
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DPPO_DIST_BACKEND="gloo", DPPO_SINGLE_DEVICE="1", DPPO_EQUIV_DIR=str(tmp_path))
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "tools", "dp_equiv.py")], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(2)]
    assert int(r[0]["world"]) == 2 and int(r[0]["rows"]) == 200 and int(r[1]["env_offset"]) == 4
    np.testing.assert_array_equal(r[0]["grads"], r[1]["grads"])        # replicas see one gradient

    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      OVERRIDES + [f"logdir={tmp_path}/single"])
    a = get_class(cfg._target_)(cfg)
    m = a.model
    np.testing.assert_array_equal(m.train_params.cpu().numpy(), r[0]["params"])
    got = {}

    def hook(epoch, batch, start, rows):
        if (epoch, batch) != (0, 0):
            return
        S, E, kf = a.n_steps, a.n_envs, m.ft_denoising_steps
        El = int(r[0]["n_envs"])
        # the shards, side by side, are the single rank's rollout
        for name, buf in (("obs", a.obs_traj), ("chains", a.chains_traj)):
            np.testing.assert_array_equal(np.concatenate([r[0][name], r[1][name]], axis=1), buf.cpu().numpy())
        adv = np.concatenate([r[0]["adv"], r[1]["adv"]], axis=1)
        np.testing.assert_allclose(adv, a.adv.cpu().numpy(), rtol=0, atol=1e-5 * np.abs(adv).max())
        # the union of the ranks' rows in the single rank's sample numbering
        idx = []
        for i in range(2):
            loc = ops.feistel_permute(0, int(r[i]["rows"]), S * El * kf, int(r[i]["perm_seed"]), int(r[i]["epoch"]),
                                      a.device).cpu().numpy()
            n_loc, j = loc // kf, loc % kf
            n_glob = (n_loc // El) * E + i * El + n_loc % El
            idx.append(n_glob * kf + j)
        idx = torch.tensor(np.concatenate(idx), device=a.device)
        N = S * E
        m.minibatch(a.obs_traj.view(N, -1), a.chains_traj.view(N, kf + 1, -1), a.lp_old, a.adv.view(-1),
                    a.ret.view(-1), 0, 0, 0, idx.numel(), global_rows=a.batch_size, row_index=idx)
        torch.cuda.synchronize()
        got["grads"] = m.grads.cpu().numpy().copy()
        got["metrics"] = m.metrics[:5].cpu().numpy().copy()
        raise StopIteration
    a.minibatch_hook = hook
    with pytest.raises(StopIteration):
        a.iteration(force_train=True)
    g1, g2 = got["grads"], r[0]["grads"]
    err = np.abs(g1 - g2).max() / np.abs(g1).max()
    assert err < 1e-4, err
    np.testing.assert_allclose(got["metrics"], r[0]["metrics"], rtol=1e-4, atol=1e-7)


def test_pretrain_agent_trains(cuda, tmp_path):
    """§8(f) row 3 end to end: TrainDiffusionAgent (agent/pretrain/train_diffusion_agent.py) on a
    synthetic stitched dataset: the diffusion loss falls over epochs, EMA and checkpoints are
    written, and DiffusionModel.p_losses on the loaded checkpoint reproduces the loss of the model."""
    import torch

    from diffusionpolicyoptimization_amd.agent.dataset.sequence import synthetic_dataset
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config, instantiate
    data = synthetic_dataset(str(tmp_path / "train.npz"), n_episodes=6, episode_len=160, seed=1)
    cfg = load_config(os.path.join(ROOT, "cfg/gym/pretrain/hopper-medium-v2"), "pre_diffusion_mlp",
                      [f"train_dataset_path={data}", f"logdir={tmp_path}/log", "train.n_epochs=4",
                       "train.batch_size=256", "train.epoch_start_ema=2", "train.update_ema_freq=1",
                       "train.save_model_freq=2", "train.learning_rate=1e-3"])
    agent = get_class(cfg._target_)(cfg)
    b = next(agent.dataset_train.batches(512))
    t = torch.randint(0, 20, (512,), device=cuda, dtype=torch.int32)
    z = torch.randn(512, 12, device=cuda)
    first = float(agent.model.p_losses(b["actions"], b["conditions"], t, z))
    last_epoch = agent.run()
    last = float(agent.model.p_losses(b["actions"], b["conditions"], t, z))
    assert np.isfinite(last_epoch) and np.isfinite(first) and last < 0.8 * first, (first, last)
    ck = os.path.join(agent.checkpoint_dir, "state_4.weights.h5")   # network.save_weights layout
    assert os.path.exists(ck) and os.path.exists(ck.replace("state_", "ema_state_"))
    assert not torch.equal(agent.ema_params, agent.model.params)
    m2 = instantiate(cfg.model, network_path=ck)
    m2._pretrain_init()
    torch.testing.assert_close(m2.params, agent.model.params)
    assert float(m2.p_losses(b["actions"], b["conditions"], t, z)) == last


def test_split_update_matches_fused(cuda, tmp_path, monkeypatch):
    """The single-GPU split update (critic half on a side stream, actor half on the main stream,
    AdamW by ranges) gives the same training as the fused minibatch, up to float-atomic order in
    the dW sums (amplified only where Adam divides a near-zero gradient by its near-zero norm)."""
    import torch

    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DPPO_SPLIT_UPDATE", flag)
        cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                          ["model.precision=fp32", "train.n_steps=20", "train.batch_size=200", "train.n_train_itr=2",
                           "train.val_freq=100", f"logdir={tmp_path}/{flag}"])
        a = get_class(cfg._target_)(cfg)
        res = a.run()
        torch.cuda.synchronize()
        out[flag] = (a.model.train_params.cpu().numpy().copy(), res[-1], a.timing["n_updates"])
    p1, r1, n1 = out["1"]
    p0, r0, n0 = out["0"]
    assert n1 == n0
    d = np.abs(p1 - p0)
    assert np.median(d) < 1e-6 and d.max() < 5e-3, (float(np.median(d)), float(d.max()))
    for k in ("pg_loss", "v_loss"):
        assert abs(r1[k] - r0[k]) <= 1e-3 * (abs(r0[k]) + 1e-3), (k, r1[k], r0[k])


@pytest.mark.parametrize("cfg_name", ["ft_ppo_diffusion_mlp", "ft_ppo_diffusion_mlp_ddim_learn_eta"])
def test_split_dp_update_matches_fused_dp(cuda, tmp_path, monkeypatch, cfg_name):
    """the split update under data parallelism (parts 2 / 4 / 5, two gradient buckets
    all-reduced from two streams: critic + metrics + d loss / d eta on the side stream during the
    actor's dW, then the actor's) against the fused data-parallel path (one collective per
    minibatch). One process plays rank 0 of W = 2 with an all-reduce that sums two identical
    replicas (x 2, issued on the stream the agent calls it from), so both paths run every stream
    ordering and bucket boundary of the real DP update; gradients, metrics, the KL / eta steps and
    the parameters must agree up to the float-atomic order the single-GPU split test allows."""
    import torch

    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DPPO_SPLIT_UPDATE", flag)
        extra = ["env.n_envs=8", "train.n_critic_warmup_itr=0", "train.eta_lr=1e-2"] if "eta" in cfg_name else []
        cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), cfg_name,
                          ["model.precision=fp32", "train.n_steps=20", "train.batch_size=200", "train.n_train_itr=2",
                           "train.val_freq=100", f"logdir={tmp_path}/{flag}"] + extra)
        a = get_class(cfg._target_)(cfg)
        a.world_size = 2                          # rank 0 of 2; every reduction goes through _allreduce
        calls = []

        def replica_sum(t, calls=calls):
            calls.append(t.numel())
            return t.mul_(2.0)
        a._allreduce = replica_sum
        res = a.run()
        torch.cuda.synchronize()
        m = a.model
        out[flag] = (m.train_params.cpu().numpy().copy(), res[-1], a.timing["n_updates"], calls,
                     m.current_eta(), getattr(m, "eta_step_count", 0))
    p1, r1, n1, c1, e1, s1 = out["1"]
    p0, r0, n0, c0, e0, s0 = out["0"]
    assert n1 == n0 > 0 and s1 == s0
    na = m.n_actor
    # the split path all-reduces two buckets per minibatch (critic + metrics, then the actor), the
    # fused one one bucket; both once for the advantage-moment table and the episode sums
    assert sorted(set(c1)) != sorted(set(c0)) and na in c1 and m.grads_ext.numel() in c0
    d = np.abs(p1 - p0)
    assert np.median(d) < 1e-6 and d.max() < 5e-3, (float(np.median(d)), float(d.max()))
    for k in ("pg_loss", "v_loss", "approx_kl", "clipfrac"):
        assert abs(r1[k] - r0[k]) <= 1e-3 * (abs(r0[k]) + 1e-3), (k, r1[k], r0[k])
    assert abs(e1 - e0) <= 1e-5 * abs(e0), (e1, e0)


@pytest.mark.parametrize("protocol", ["tagged", "go"])
def test_pipelined_rollout_unpublished_observation_times_out(cuda, protocol, monkeypatch):
    """A launch whose observation never comes (the host died or stalled) gives up after its
    bounded device-side wait (~4 s), flags bit 31 of the done counter and still finishes, so no
    wave is left spinning; RolloutPipe.wait raises instead of returning stale actions."""
    import torch

    monkeypatch.setenv("DPPO_ROLLOUT_PROTOCOL", protocol)
    from diffusionpolicyoptimization_amd import _lib, ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      ["model.precision=bf16"])
    model = instantiate(cfg.model, device=cuda, seed=5)
    d = model.dims
    E = 40
    obs_traj = torch.zeros(1, E, d.sd, device=cuda)
    chains = torch.zeros(1, E, d.ft_denoising_steps + 1, d.xd, device=cuda)
    act = torch.empty(E, d.xd, device=cuda)
    pipe = ops.RolloutPipe(model, obs_traj, act, chains)
    pipe.begin()
    pipe.enqueue(0)                      # never published
    with pytest.raises(_lib.DppoError, match="timed out"):
        pipe.wait(timeout_s=30.0)
    pipe.end()
    torch.cuda.synchronize()             # the launch drained
    assert int(pipe._done[0]) & 0x80000000
    pipe.close()


def test_keras_checkpoints_round_trip_through_the_model(cuda, tmp_path):
    """§8(f) row 2 end to end: PPODiffusion.save_weights -> state_*.weights.h5 (actor/, actor_ft/,
    critic/) -> load_weights into a fresh model; a pretrain-style network file (DiffusionMLP at the
    root) as network_path loads into BOTH actors (diffusion_vpg.py:85-97); a missing path raises."""
    import torch

    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util import keras_weights
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp", ["model.precision=bf16"])
    m = instantiate(cfg.model, device=cuda, seed=3)
    m.train_params.add_(torch.randn_like(m.train_params) * 1e-3)
    m.repack()
    p = str(tmp_path / "state_7.weights.h5")
    m.save_weights(p)
    m2 = instantiate(cfg.model, device=cuda, seed=4)
    m2.load_weights(p)
    assert torch.equal(m2.base_params, m.base_params) and torch.equal(m2.train_params, m.train_params)
    # the repacked images serve the same policy (image padding bytes are not compared)
    cond = torch.rand(16, m.dims.sd, device=cuda) * 2 - 1
    m._call_id = m2._call_id = 0
    m2.seed = m.seed
    assert torch.equal(m(cond).trajectories, m2(cond).trajectories)
    assert torch.equal(m.critic_values(cond), m2.critic_values(cond))
    net = str(tmp_path / "state_785.weights.h5")
    keras_weights.save_actor(net, ops.unflatten_params(m.actor_spec, m.actor_ft_params.cpu().numpy()))
    m3 = instantiate(cfg.model, device=cuda, network_path=net)
    assert torch.equal(m3.base_params, m.actor_ft_params) and torch.equal(m3.actor_ft_params, m.actor_ft_params)
    with pytest.raises(FileNotFoundError):
        instantiate(cfg.model, device=cuda, network_path=str(tmp_path / "missing.weights.h5"))


def test_learn_eta_agent_iterations(cuda, tmp_path):
    """§8(f) row 4 (parity unpinned): the DDIM agent with a learnable eta runs train iterations; the
    eta logit moves by its AdamW (one step per minibatch, eta_update_interval 1), eta stays inside
    (min_eta, max_eta), the train-mode DDIM table holds the current eta's rows (ddim_buffers at that
    eta), the eval table keeps eta = 0, and c_loss's eta metric reports it."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddim_buffers
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_ddim_learn_eta",
                      ["model.precision=fp32", "env.n_envs=8", "train.n_steps=20", "train.batch_size=200",
                       "train.n_train_itr=2", "train.val_freq=100", "train.n_critic_warmup_itr=0",
                       "train.eta_lr=1e-2", f"logdir={tmp_path}"])
    agent = get_class(cfg._target_)(cfg)
    m = agent.model
    assert m.learn_eta
    logit0 = float(m.eta_state[0].item())
    eta0 = m.current_eta()
    assert abs(eta0 - 0.5) < 1e-6
    res = agent.run()
    n_mb = agent.timing["n_updates"]
    assert n_mb > 0 and m.eta_step_count == n_mb
    eta1 = m.current_eta()
    assert float(m.eta_state[0].item()) != logit0 and 0.1 < eta1 < 1.0
    assert all(math.isfinite(r["pg_loss"]) for r in res if not r["eval"])
    ref = ops.sched_table(ddim_buffers(20, 10, np.float32(eta1)))
    np.testing.assert_allclose(m.sched.cpu().numpy()[:, 2:5], ref[:, 2:5], rtol=3e-7, atol=1e-7)
    ev = ops.sched_table(ddim_buffers(20, 10, 0.0))
    np.testing.assert_array_equal(m.sched_eval.cpu().numpy(), ev)
    assert np.isfinite(m.train_params.cpu().numpy()).all()
    # the eta state is part of the checkpoint (h5 and npz); a fresh model restores
    # logit, moments and step count, and its train-mode DDIM table follows the restored eta
    from diffusionpolicyoptimization_amd.util.config import instantiate
    for ext in ("weights.h5", "npz"):
        path = str(tmp_path / f"eta_ckpt.{ext}")
        m.save_weights(path)
        m2 = instantiate(cfg.model, device=cuda)
        assert abs(m2.current_eta() - 0.5) < 1e-6
        m2.load_weights(path)
        assert torch.equal(m2.eta_state, m.eta_state) and m2.eta_step_count == m.eta_step_count
        assert m2.current_eta() == m.current_eta()
        np.testing.assert_array_equal(m2.sched.cpu().numpy(), m.sched.cpu().numpy())
        assert torch.equal(m2.train_params, m.train_params)


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("bf16", 2e-3)])
def test_bc_loss_matches_oracle(cuda, precision, tol, tmp_path):
    """c_loss's behaviour-cloning term (diffusion_ppo.py:63-71; use_bc_loss, off in every cfg): base-policy
    chains for the batch's observations (every step on the base actor), their clipped actor_ft log-probs,
    negated mean — PPODiffusion.bc_loss with injected draws against the oracle's composition of its
    sampler and log-probs (bf16: the oracle rounding operands at the kernels' points). Then the agent's
    report: use_bc_loss=True puts a finite value in the update's info; the term's Philox draws leave the
    model's call counter (the rollout's stream) where it was."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import get_class, instantiate, load_config
    from helpers import to_f64
    from oracle import dppo_oracle as O
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      [f"model.precision={precision}"])
    m = instantiate(cfg.model, device=cuda, seed=3)
    d = m.dims
    E, K, kf = 37, d.denoising_steps, m.ft_denoising_steps
    rng = np.random.default_rng(8)
    state = rng.uniform(-1, 1, (E, d.cond_steps, d.obs_dim)).astype(np.float32)
    xT = rng.standard_normal((E, d.horizon_steps, d.action_dim)).astype(np.float32)
    z = rng.standard_normal((K, E, d.horizon_steps, d.action_dim)).astype(np.float32)
    calls = m._call_id
    bc = m.bc_loss(torch.tensor(state.reshape(E, -1), device=cuda), x_T=torch.tensor(xT.reshape(E, -1), device=cuda),
                   noise=torch.tensor(z.reshape(K, E, -1), device=cuda))
    assert m._call_id == calls
    na = m.n_actor
    base = ops.unflatten_params(m.actor_spec, m.base_params.cpu().numpy())
    ft = ops.unflatten_params(m.actor_spec, m.train_params.cpu().numpy()[:na])
    rnd = {"fp32": None, "bf16": O.round_bf16}[precision]
    ref = O.bc_loss(to_f64(base), to_f64(ft), O.ddpm_schedule(K), state.astype(np.float64), xT.astype(np.float64),
                    z.astype(np.float64), kf, min_std=m.get_min_sampling_denoising_std(), randn_clip=m.randn_clip_value,
                    min_logprob_std=m.min_logprob_denoising_std, rnd=rnd)
    assert abs(bc - ref) <= tol * max(1.0, abs(ref)), (bc, ref)
    if precision == "fp32":
        cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                          ["train.n_steps=8", "train.batch_size=160", "+train.use_bc_loss=true", f"logdir={tmp_path}",
                           "train.save_checkpoints=false"])
        agent = get_class(cfg._target_)(cfg)
        info = agent.iteration(force_train=True)
        assert math.isfinite(info["bc_loss"]) and info["bc_loss"] != 0.0, info["bc_loss"]
