"""TrainPPODiffusionAgent (reference agent/finetune/train_ppo_diffusion_agent.py:22-468) on MI355X.

One iteration = rollout + (train iterations only) value/log-prob pass, reward scaling, GAE and
the PPO epochs. Differences from the reference are only where data lives and what runs it:
  * rollout buffers (obs [S,E,SD], chains [S,E,K'+1,XD]) stay in HBM; per env step the host
    moves only obs (H2D, pinned) and actions (D2H, pinned); chains never leave the device;
  * sampler / critic / log-prob / reward scaler / GAE / PPO loss+grad / AdamW are HIP kernels;
  * data parallel: each rank owns n_envs/world envs, draws its share of every minibatch from its
    own rollout, and the gradient, the minibatch advantage moments, the reward-RMS moments and
    the metrics are summed with torch.distributed (RCCL) so all replicas take identical steps.
Semantics kept on purpose: eval at itr % val_freq == 0 with env reset only
then (4), population-std advantage normalisation per minibatch (3), one optimiser (2)."""
import logging
import os
import pickle
import time

import numpy as np
import torch
import torch.distributed as dist

from ... import ops
from ...util.dist import allreduce_sum_, explained_variance_from_moments
from ...util.scheduler import CosineAnnealingWarmupRestarts
from ...util.timer import Timer
from .train_ppo_agent import TrainPPOAgent

log = logging.getLogger(__name__)


def episode_sums(firsts, rew, act_steps, success_threshold):
    """Per-rank episode sums (n_finished, sum of returns, sum of best rewards, n_success) over
    the episodes that start and end inside the rollout (agent :144-167). firsts [S+1,E], rew [S,E].

    Vectorised over envs (the per-env loop of the reference took ~0.4 ms at 64 envs and ~3 ms at
    512, host time that the update loop, at most one minibatch ahead of the GPU, turned into GPU
    idle time): the episodes are the consecutive pairs of episode starts of one env, env-major as
    the reference visits them; returns and best rewards are add / max reductions over each
    episode's rewards (np.add.reduceat / np.maximum.reduceat over the env-major flattened rewards)."""
    firsts = np.asarray(firsts)
    rew = np.asarray(rew, dtype=np.float64)
    S, E = rew.shape
    e_i, t_i = np.nonzero(firsts.T == 1)            # env-major, t ascending within an env
    same = e_i[1:] == e_i[:-1]
    s, en, e = t_i[:-1][same], t_i[1:][same], e_i[:-1][same]
    keep = en - s > 1
    s, en, e = s[keep], en[keep], e[keep]
    if s.size == 0:
        return [0.0, 0.0, 0.0, 0.0]
    flat = np.concatenate([rew.T.reshape(-1), np.zeros(1)])   # a pad element: an end index may be E*S
    idx = np.empty(2 * s.size, dtype=np.int64)
    idx[0::2] = e * S + s
    idx[1::2] = e * S + en
    ret = np.add.reduceat(flat, idx)[0::2]
    b = np.maximum.reduceat(flat, idx)[0::2] / act_steps
    tot = 0.0
    for x in ret.tolist():      # the reference's running sum, in its order
        tot += x
    best = 0.0
    for x in b.tolist():
        best += x
    return [float(s.size), tot, best, float(np.count_nonzero(b >= success_threshold))]


def episode_stats_from_sums(sums):
    n_ep, tot, best, succ = sums
    if n_ep == 0:
        return dict(num_episode_finished=0, avg_episode_reward=0.0, avg_best_reward=0.0, success_rate=0.0)
    return dict(num_episode_finished=int(n_ep), avg_episode_reward=tot / n_ep, avg_best_reward=best / n_ep,
                success_rate=succ / n_ep)


class TrainPPODiffusionAgent(TrainPPOAgent):
    def __init__(self, cfg):
        super().__init__(cfg)
        self.reward_horizon = cfg.get("reward_horizon", self.act_steps)
        self.learn_eta = self.model.learn_eta
        if self.learn_eta:
            # the eta AdamW of agent :28-45 (Keras defaults, its own cosine-warmup schedule evaluated at
            # the eta optimizer's step count), stepped every eta_update_interval minibatches as the
            # commented-out :358-359 (the original DPPO's schedule); PARITY UNPINNED
            el = cfg.train.eta_lr_scheduler
            self.eta_update_interval = int(cfg.train.eta_update_interval)
            self.eta_lr_scheduler = CosineAnnealingWarmupRestarts(
                first_cycle_steps=el.first_cycle_steps, cycle_mult=1.0, max_lr=cfg.train.eta_lr, min_lr=el.min_lr,
                warmup_steps=el.warmup_steps, gamma=1.0)
            self.eta_weight_decay = float(cfg.train.get("eta_weight_decay", 0.004))
        self.perm_seed = int(cfg.train.get("perm_seed", self.seed * 1_000_003 + 17)) + 7919 * self.rank
        self.timing = {"rollout_s": 0.0, "update_s": 0.0, "n_updates": 0, "env_steps": 0, "iters": 0}
        self.emulate_world = max(1, int(cfg.train.get("emulate_world", 1)))
        if self.emulate_world > 1 and self.world_size > 1:
            raise ValueError("train.emulate_world is a single-process measurement mode")
        self.sampler_events = None    # optional list of (start, end) torch.cuda.Event pairs
        self.update_events = None
        self.host_profile = None      # optional dict: host seconds per update-loop phase (tools)
        self._passes_enqueued = False
        # test hook: called as minibatch_hook(epoch, batch, start, rows) after a minibatch's
        # gradients (all-reduced under data parallelism) are in self.model.grads
        self.minibatch_hook = None
        self._alloc_buffers()
        self.done_venv = np.zeros(self.n_envs, dtype=bool)
        self.last_itr_eval = False
        self.cnt_train_step = 0
        self.run_results = []
        self.prev_obs_venv = None
        self.last_info = {}
        self._stepper = None

    # ------------------------------------------------------------------ buffers
    def _alloc_buffers(self):
        S, E, d = self.n_steps, self.n_envs, self.model.dims
        dev = self.device
        self._buf_kf = d.ft_denoising_steps
        self.obs_traj = torch.empty(S, E, d.sd, dtype=torch.float32, device=dev)
        self.chains_traj = torch.empty(S, E, d.ft_denoising_steps + 1, d.xd, dtype=torch.float32, device=dev)
        self.act_dev = torch.empty(E, d.xd, dtype=torch.float32, device=dev)
        self.pipe = None
        if self.cfg.train.get("pipelined_rollout", True):
            # observation / action staging in coherent mapped memory, launches pre-enqueued
            self.pipe = ops.RolloutPipe(self.model, self.obs_traj, self.act_dev, self.chains_traj)
            self.obs_pin = self.pipe.obs.view(E, self.n_cond_step, self.obs_dim)
            self.act_pin = self.pipe.act
        else:
            self.obs_pin = torch.empty(E, self.n_cond_step, self.obs_dim, dtype=torch.float32).pin_memory()
            self.act_pin = torch.empty(E, d.xd, dtype=torch.float32).pin_memory()
        # per-step rewards and flags in coherent mapped memory: the host writes them during the rollout
        # and the update moves all three to the device in one kernel (ops.copy_from_host)
        self._reward_map = ops.MappedArray((S, E), np.float64)
        self._term_map = ops.MappedArray((S, E), np.uint8)
        # firsts with row S (the flags after the last step): the episode accounting reads all S + 1 rows,
        # the reward scaler the first S
        self._first_map = ops.MappedArray((S + 1, E), np.uint8)
        self.reward_pin = self._reward_map.tensor
        self.term_pin = self._term_map.tensor
        self.first_pin = self._first_map.tensor
        self.firsts = np.zeros((S + 1, E))
        self.reward_dev = torch.empty(S, E, dtype=torch.float64, device=dev)
        self.last_obs_dev = torch.empty(E, d.sd, dtype=torch.float32, device=dev)
        self.first_all_dev = torch.empty(S + 1, E, dtype=torch.uint8, device=dev)
        self.first_dev = self.first_all_dev[:S]
        self.episode_dev = torch.empty(E, 4, dtype=torch.float64, device=dev)
        self.term_dev = torch.empty(S, E, dtype=torch.uint8, device=dev)
        self.values = torch.empty(S * E, dtype=torch.float32, device=dev)
        self.last_values = torch.empty(E, dtype=torch.float32, device=dev)
        self.lp_old = torch.empty(S * E, d.ft_denoising_steps, dtype=torch.float32, device=dev)
        self.adv = torch.empty(S, E, dtype=torch.float32, device=dev)
        self.ret = torch.empty(S, E, dtype=torch.float32, device=dev)
        self.adv_stats = torch.zeros(3, dtype=torch.float64, device=dev)

    def _fit_buffers_to_model(self):
        """The K'-shaped buffers (chains_traj [S,E,K'+1,XD], lp_old [S*E,K'], the rollout pipe bound
        to them) follow model.ft_denoising_steps, which annealing (model.step(), diffusion_vpg.py:
        114-142, ft_denoising_steps_d / _t) lowers between iterations. The reference allocates its
        chains_trajs from model.ft_denoising_steps every iteration (agent :87-95); here they are
        re-sized only when K' changed. The env state (the last observation in the staging buffer)
        carries over."""
        kf = self.model.ft_denoising_steps
        if kf == self._buf_kf:
            return
        if kf < 1:
            raise ValueError("ft_denoising_steps annealed to 0: no fine-tuned denoising step is left to update")
        obs = self.obs_pin.numpy().copy()
        if self.pipe is not None:
            self.pipe.close()
        # the old mapped reward / flag buffers are freed with their last view (ops.MappedArray):
        # no device copy from them may still be pending
        torch.cuda.synchronize(self.device)
        self._alloc_buffers()
        self.obs_pin.numpy()[:] = obs
        if self.prev_obs_venv is not None:
            self.prev_obs_venv = {"state": self.obs_pin.numpy()}
        self._stepper = None
        self._passes_enqueued = False
        log.info("rollout buffers re-sized for ft_denoising_steps = %d", kf)

    def _logprob_range(self, s0, s1):
        """The old-log-prob pass (:209-229) over rollout steps [s0, s1) on the current stream."""
        E, m = self.n_envs, self.model
        kf = m.ft_denoising_steps
        a, b = s0 * E, s1 * E
        ops.logprob(m.dims, m.precision, m.packed_ft, m.sched, self.obs_traj.view(-1, m.dims.sd)[a:b],
                    self.chains_traj.view(-1, kf + 1, m.dims.xd)[a:b], min_logprob_std=m.min_logprob_denoising_std,
                    reward_horizon=self.reward_horizon, want_elem=False, lp_mean=self.lp_old[a:b])

    def _enqueue_passes(self, from_step=0):
        """The value and old-log-prob passes over the rollout (:191-229): one fused launch each,
        no num_split needed. Steps before from_step already had their log-probs computed during
        the rollout (pass stream, see rollout())."""
        S, E, m = self.n_steps, self.n_envs, self.model
        N = S * E
        ops.critic_forward(m.dims, m.precision, m.packed_critic, self.obs_traj.view(N, -1), values=self.values)
        if from_step < S:
            self._logprob_range(from_step, S)
        if getattr(self, "_pass_stream", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._pass_stream)
        self._passes_enqueued = True

    def _allreduce(self, t):
        return allreduce_sum_(t)

    def _bucket_allreduce(self, name, t):
        """The per-minibatch gradient buckets (fp32, grads_ext slices): torch.distributed (RCCL,
        the default) or, with train.allreduce = ipc (env DPPO_ALLREDUCE), dppo_ipc_allreduce over
        IPC-mapped peer regions (util/ipc.py; one group per bucket, since the two buckets run on two
        streams), on the current stream."""
        groups = getattr(self, "_ipc_groups", None)
        if groups is None:
            return self._allreduce(t)
        return groups[name](t)

    def _ipc_setup(self, split):
        """Collective (every rank, same point of the update): the IPC groups of the gradient buckets."""
        mode = os.environ.get("DPPO_ALLREDUCE") or str(self.cfg.train.get("allreduce", "rccl"))
        if mode != "ipc" or self.world_size == 1 or getattr(self, "_ipc_groups", None) is not None:
            return
        from ...util.ipc import IpcAllReduce
        m = self.model
        na, ne = m.n_actor, m.grads_ext.numel()
        # only the buckets the update issues: the split update's two (actor, critic + metrics), or the
        # single "all" bucket of the unsplit path (max_grad_norm or DPPO_SPLIT_UPDATE=0)
        if split:
            self._ipc_groups = {"actor": IpcAllReduce(na, device=self.device),
                                "critic": IpcAllReduce(ne - na, device=self.device)}
        else:
            self._ipc_groups = {"all": IpcAllReduce(ne, device=self.device)}

    def close_collectives(self):
        """Collective (every rank): unmap and free the IPC groups (run() calls it after the last
        iteration)."""
        for g in (getattr(self, "_ipc_groups", None) or {}).values():
            g.close()
        self._ipc_groups = None

    # ------------------------------------------------------------------ rollout (agent :58-141)
    def rollout(self, eval_mode, defer_stats=False):
        """One rollout of S chunks; returns the episode statistics, or None with defer_stats (the
        train iteration computes them on the host while the update's first kernels run)."""
        S, E = self.n_steps, self.n_envs
        self._ep_local = None
        self._ep_dev_valid = False
        # quirk 4: the reference assigns last_itr_eval = eval_mode right before it tests it (agent
        # :70-74), so its "right after eval mode" clause never fires: envs are reset only when
        # reset_at_iteration is set or on eval iterations, and the train iteration after an eval
        # continues from the eval's env state with firsts[0] = done_venv. (The first iteration has
        # no env state yet; the reference's itr 0 is always an eval, :68.)
        self.last_itr_eval = eval_mode
        if self.reset_at_iteration or eval_mode or self.last_itr_eval or self.prev_obs_venv is None:
            obs = self.reset_env_all()
            self.obs_pin.numpy()[:] = obs["state"]
            self.firsts[0] = 1
        else:
            self.firsts[0] = self.done_venv  # envs that finished were already reset in-wrapper
        obs_np = self.obs_pin.numpy()
        act_view = self.act_pin.numpy().reshape(E, self.horizon_steps, self.action_dim)[:, :self.act_steps]
        stream = torch.cuda.current_stream(self.device)
        rew_np, term_np = self.reward_pin.numpy(), self.term_pin.numpy()

        def bookkeeping(step, reward, terminated, truncated):
            done = terminated | truncated
            rew_np[step] = reward
            term_np[step] = terminated
            self.firsts[step + 1] = done
            self.done_venv = done
            if not eval_mode:
                self.cnt_train_step += self.n_envs_global * self.act_steps

        if self.pipe is not None:
            # step t+1's launch is enqueued before the envs of step t are stepped; it waits on
            # the device for the observation the host publishes after the env step
            pipe = self.pipe
            early = defer_stats      # a train iteration: its value / old-log-prob passes follow the rollout
            # The old-log-prob pass of finished chunks runs DURING the rollout: actor_ft is frozen
            # until the update, chunk t's chains and observation are final once launch t is done, and
            # the sampler holds a few CUs only. Every G steps one log-prob launch over the last G
            # chunks (G x E x K' rows) goes to a pass stream behind the events of the two latest
            # launches, onto the idle CUs (DPPO_PASS_CHUNK = G; 0 = after the rollout).
            G = int(os.environ.get("DPPO_PASS_CHUNK", "10")) if early else 0
            if G > 0 and getattr(self, "_pass_stream", None) is None:
                self._pass_stream = torch.cuda.Stream(device=self.device)
            done_lp = 0
            # completion events of the launches, a ring re-recorded per step (only the two latest
            # launches <= last are ever waited on); created once per agent
            if G > 0 and getattr(self, "_launch_evs", None) is None:
                self._launch_evs = [torch.cuda.Event() for _ in range(4)]
            evs = self._launch_evs if G > 0 else None

            def overlap_passes(last):
                # launches 0..last are enqueued: log-probs of steps [done_lp, last] once they finish
                nonlocal done_lp
                if G <= 0 or last + 1 - done_lp < G:
                    return
                ps = self._pass_stream
                for i in range(max(0, last - 1), last + 1):   # the two streams' latest launches <= last
                    ps.wait_event(evs[i % 4])
                with torch.cuda.stream(ps):
                    self._logprob_range(done_lp, last + 1)
                done_lp = last + 1

            def last_enqueued():
                # right behind the last sampler launch, so the GPU runs the passes while the host
                # does the last env step and the rollout's bookkeeping (they read only obs / chains)
                pipe.end()
                self._enqueue_passes(done_lp)

            pipe.begin()
            if G > 0:
                self._pass_stream.wait_stream(stream)       # the weights the log-probs read
            pipe.enqueue(0, eval_mode)
            if G > 0:
                pipe.launch_event(evs[0])
            if early and S == 1:
                last_enqueued()
            pipe.publish()
            # wait + step + publish in C (the tagged stepper decodes the actions into act_view itself,
            # so it needs the whole [E, horizon, Da] buffer: act_steps == horizon_steps)
            gated = getattr(self.venv, "native", None) is not None and act_view.flags.c_contiguous
            for step in range(S):
                more = step + 1 < S
                if more:
                    pipe.enqueue(step + 1, eval_mode)
                    if G > 0:
                        pipe.launch_event(evs[(step + 1) % 4])
                        if step + 2 < S:
                            overlap_passes(step)           # launch `step` finished before launch step+1 can
                    if early and step + 2 == S:
                        last_enqueued()
                if gated:
                    _, reward, terminated, truncated, _ = self.venv.step(act_view, obs_out=obs_np,
                                                                         gate=pipe.gate(publish=more))
                    if more:
                        pipe.published_by_gate() if self.venv.published else pipe.publish()
                else:
                    pipe.wait()
                    _, reward, terminated, truncated, _ = self.venv.step(act_view, obs_out=obs_np)
                    if more:
                        pipe.publish()
                bookkeeping(step, reward, terminated, truncated)
            if not early:
                pipe.end()
                stream.synchronize()
            # (a train iteration goes on enqueueing its update behind the passes: no host sync here)
        else:
            if self._stepper is None:
                self._stepper = self.model.bind_rollout(self.obs_pin, self.obs_traj, self.act_dev, self.act_pin,
                                                        self.chains_traj)
            sample_step = self._stepper
            for step in range(S):
                if self.sampler_events is not None:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev0.record(stream)
                # H2D obs -> obs_traj[step], K-step sampler -> chains_traj[step], D2H actions, stream wait
                sample_step(step, eval_mode)
                if self.sampler_events is not None:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(stream)
                    self.sampler_events.append((ev0, ev1))
                _, reward, terminated, truncated, _ = self.venv.step(act_view, obs_out=obs_np)
                bookkeeping(step, reward, terminated, truncated)
        self.prev_obs_venv = {"state": obs_np}
        return None if defer_stats else self.episode_stats()

    def _episode_sums_local(self):
        """This rank's episode sums: the update's dppo_episode_sums rows summed in env order (the
        reference's visit order), or the host restatement when no update ran on this rollout."""
        if getattr(self, "_ep_local", None) is None:
            if getattr(self, "_ep_dev_valid", False):
                rows = self.episode_dev.cpu().numpy()
                acc = [0.0, 0.0, 0.0, 0.0]
                for r in rows.tolist():
                    for c in range(4):
                        acc[c] += r[c]
                self._ep_local = acc
            else:
                self._ep_local = episode_sums(self.firsts, self.reward_pin.numpy(), self.act_steps,
                                              self.best_reward_threshold_for_success)
        return self._ep_local

    def episode_stats(self):
        """agent :144-183; sums over ranks so every rank logs the global statistics."""
        sums = list(self._episode_sums_local())
        if self.world_size > 1:
            t = torch.tensor(sums, dtype=torch.float64, device=self.device)
            self._allreduce(t)
            sums = t.tolist()
        return episode_stats_from_sums(sums)

    # ------------------------------------------------------------------ update (agent :186-377)
    def update(self):
        S, E, m = self.n_steps, self.n_envs, self.model
        kf = m.ft_denoising_steps
        N = S * E
        obs_flat = self.obs_traj.view(N, -1)
        chains_flat = self.chains_traj.view(N, kf + 1, -1)
        if not self._passes_enqueued:
            self._enqueue_passes()
        self._passes_enqueued = False
        np.copyto(self.first_pin.numpy(), self.firsts, casting="unsafe")
        copies = [(self.reward_dev, self._reward_map), (self.term_dev, self._term_map),
                  (self.first_all_dev, self._first_map)]
        if self.pipe is not None:           # the last observation, for the bootstrap values (:239-246)
            last_obs = self.last_obs_dev
            copies.append((last_obs, self.pipe.obs_mapped))
        ops.copy_from_host(copies)
        # the episode accounting (:144-167) on the raw rewards, before the scaler rewrites them in place;
        # read after the update's final synchronize (_episode_sums_local)
        ops.episode_sums(self.reward_dev, self.first_all_dev, self.act_steps, self.best_reward_threshold_for_success,
                         self.episode_dev)
        self._ep_local = None
        self._ep_dev_valid = True
        if self.reward_scale_running:                                                  # :232-236
            self.running_reward_scaler.scale_(self.reward_dev, self.first_dev,
                                              group=dist.group.WORLD if self.world_size > 1 else None)
        if self.pipe is None:
            last_obs = self.obs_pin.view(E, -1).to(self.device, non_blocking=True)
        ops.critic_forward(m.dims, m.precision, m.packed_critic, last_obs, values=self.last_values)
        ops.gae(self.reward_dev, self.values.view(S, E), self.last_values, self.term_dev, self.gamma, self.gae_lambda,
                self.reward_scale_const, adv=self.adv, ret=self.ret)                       # :239-263
        adv_flat, ret_flat = self.adv.view(-1), self.ret.view(-1)
        # explained-variance moments of the pre-update values and returns (:373-377), read after the
        # epochs from host-mapped memory (no torch reductions or host syncs at the end of the update)
        if getattr(self, "_ev_map", None) is None:
            self._ev_map = ops.MappedDoubles(5)
        ops.value_moments(self.values, ret_flat, self._ev_map.address)

        total_local = N * kf
        # W: the data-parallel width the minibatch arithmetic follows. train.emulate_world = W' > 1
        # on ONE process is a measurement mode (bench.py --emulate-ranks): this rank runs exactly one
        # rank's share of the W'-rank update (W' x the minibatches, batch_size / W' rows each, the
        # gradient scaled by 1 / batch_size) with every collective skipped
        W = self.world_size if self.world_size > 1 else self.emulate_world
        total_global = total_local * W
        # Data parallel: by default the global minibatch is the reference's
        # batch_size rows, batch_size / world drawn by each rank from its own shard (each rank's
        # keyed permutation of its rows), so the update is the reference's PPO over the union of
        # the shards (world x more minibatches than one rank over its own envs). With
        # train.dp_scale_batch = true every rank runs a full batch_size minibatch of its own and
        # the gradients are averaged: the reference run with batch_size x world.
        eff_batch = self.batch_size * (W if self.dp_scale_batch else 1)
        num_batch = max(1, total_global // eff_batch)                                     # :288
        rows_local_full = eff_batch // W
        clipfracs, info = [], {}
        caller = torch.cuda.current_stream(self.device)
        # the epochs run on the caller's stream (a high-priority stream for the actor's half, r03, was
        # measured slower: update 15.0 vs 14.8 ms per iteration, tools/ab_env.sh)
        with torch.cuda.stream(caller):
            stream = torch.cuda.current_stream(self.device)
            # The target_kl check (:366-370) reads each minibatch's approx_kl on the host. It runs one
            # minibatch behind: minibatch i's gradients are enqueued before the host waits for i-1's
            # metrics (an event right after i-1's kernels, the metrics copied to pinned memory), so the
            # GPU never idles on that read. Only the AdamW step of i waits for the verdict. In the
            # reference the minibatch that exceeds target_kl IS applied and its `break` leaves only the
            # batch loop of that epoch (`if flag_break: break` sits inside the batch loop and is never
            # reached; flag_break is reset per epoch, :284-286,366-370), so the next epoch still runs.
            # Here: a stop by minibatch i-1 of the SAME epoch drops i's gradients (the reference never
            # computes them) and ends the epoch; a stop by the previous epoch's last minibatch ended an
            # epoch that was over anyway, so i (the new epoch's first) is applied.
            # Each minibatch's metric sums land in mapped host memory, copied by its optimiser-step
            # launch (dppo_optimizer_step) or, before the critic warm-up ends, by a plain copy; one event
            # per slot marks them readable.
            # With the optimiser step applied (after the critic warm-up) the launch stores a tag after the
            # sums and the host polls it (ABI 5): no event record or cross-stream wait on the minibatch
            # chain. In the split update the critic's step copies its own v_loss (metric 1) with the
            # same tag, so the main stream never waits for the side stream inside the epochs.
            if not hasattr(self, "_met_map"):
                self._met_map = [ops.MappedDoubles(8) for _ in range(2)]
                self._cmet_map = [ops.MappedDoubles(8) for _ in range(2)]
                self._ev_m = [torch.cuda.Event() for _ in range(2)]
                self._mb_tag = 0
            pending = None
            last_mb = None   # (epoch key, start, rows) of the last minibatch run (the bc_loss report)
            eta_now = m.current_eta()   # c_loss's eta metric (diffusion_ppo.py:131), as of the update's start

            def finish(p):
                slot, ev, grows, _, tag, ctag = p
                if tag:
                    self._met_map[slot].wait_tag(5, tag)
                    met = self._met_map[slot].array[:5].copy()
                    if ctag:
                        self._cmet_map[slot].wait_tag(1, ctag)
                        met[1] = self._cmet_map[slot].array[0]
                    met /= grows
                else:
                    ev.synchronize()
                    met = self._met_map[slot].array[:5] / grows
                self.timing["n_updates"] += 1
                inf = dict(pg_loss=float(met[0]), v_loss=float(met[1]), approx_kl=float(met[2]),
                           clipfrac=float(met[3]), ratio=float(met[4]), bc_loss=0.0, eta=eta_now,
                           entropy_loss=-eta_now, loss=float(met[0] + self.vf_coef * met[1]))
                clipfracs.append(inf["clipfrac"])
                return inf, self.target_kl is not None and inf["approx_kl"] > self.target_kl

            dp = self.world_size > 1
            split = self.max_grad_norm is None and os.environ.get("DPPO_SPLIT_UPDATE", "1") != "0"
            if dp:
                self._ipc_setup(split)
            # every minibatch's advantage moments (norm_adv, diffusion_ppo.py:74-75) in one launch, and
            # on several GPUs one all-reduce of the whole table instead of one per minibatch
            n_mb = self.update_epochs * num_batch
            if getattr(self, "_adv_all", None) is None or self._adv_all.shape[0] != n_mb:
                self._adv_all = torch.zeros(n_mb, 3, dtype=torch.float64, device=self.device)
            ops.ppo_adv_stats_all(adv_flat, total_local, kf, self.perm_seed, 1000 * self.itr, self.update_epochs,
                                  rows_local_full, num_batch, self._adv_all)
            if dp:
                self._allreduce(self._adv_all)
            # Split update: the critic's half of each minibatch (row tiles, dW, its AdamW range,
            # repack) runs on a side stream and the actor's on the main stream, so the critic of
            # minibatch i+1 fills the CUs the actor leaves idle in its dW / small-kernel tail of i.
            # Metrics alternate between two device buffers; the main stream joins the critic's half
            # before copying a minibatch's metrics.
            # Under data parallelism the gradients go out in two buckets, each as soon as it is final:
            # the critic's gradients + the minibatch's metric sums on the side stream once the actor's
            # row tiles have produced their loss metrics (overlapping the actor's dW), then the actor's
            # gradients on the main stream (overlapping the critic's optimiser step and repack).
            if split:
                if getattr(self, "_side", None) is None:
                    self._side = torch.cuda.Stream(device=self.device)
                    self._met_dev = [torch.zeros(16, dtype=torch.float64, device=self.device) for _ in range(2)]
                    self._ev_rows = torch.cuda.Event()
                    self._ev_met = torch.cuda.Event()
                side = self._side
                side.wait_stream(stream)
                na = m.n_actor
            # the per-update arguments of the minibatch and optimizer calls, validated and marshalled
            # once (host enqueue time per minibatch: an 8-GPU rank runs 255 small ones per iteration)
            # Both halves' optimizer steps are ONE launch each (ABI 11, DPPO_STEP_FUSED_PACK): AdamW, the
            # weight image (the actor's: actor_tile_step_kernel, then its row tiles' fold launch) and the
            # zeroing of what the next minibatch's half would zero first (DPPO_STEP_CLEAR_GRADS +
            # ops.ClearRanges; the next half runs DPPO_PPO_PRECLEARED). The actor's time-MLP backward and
            # W_out / l2 gradients stay one launch in the minibatch (time_l2_bwd). Measured slower and
            # removed: the actor's whole tail in one launch (r06, profiles/r06de_actor_tail_ab.txt; r05g
            # workgroup-0 form, profiles/r05g_step_ab.txt), the l2 gradient left factored for the step
            # (profiles/r05r_l2_defer_ab.txt), the critic's half held behind the actor's step, and the
            # AdamW + pack launch pair. Not with a test hook reading the gradients (zero after the step).
            fuse = split and self.minibatch_hook is None
            # the actor's image skips the split sampler's tables (fold, TIN, W_XS, B_OUT2), which no PPO
            # kernel reads: the next rollout's first sampler launch re-derives them once
            defer = True
            opt = self.actor_optimizer
            ng_all = m.grads.numel()
            # the bound calls are reused across updates while every buffer they captured is the same
            # (~0.2 ms of host marshalling per update, with the device idle behind it)
            ptrs = lambda *ts: tuple((t.data_ptr(), tuple(t.shape)) for t in ts)
            bkey = (ptrs(obs_flat, chains_flat, self.lp_old, adv_flat, ret_flat, m.grads, m.train_params,
                         m.packed_ft, m.packed_critic, m.sched, m.workspace(rows_local_full), opt.m, opt.v),
                    self.perm_seed, rows_local_full, self.reward_horizon, split,
                    self.max_grad_norm is None, m.dims.ft_denoising_steps, m.precision, fuse)
            if getattr(self, "_bound_key", None) != bkey:
                bound = {"run_mb": m.bind_minibatch(obs_flat, chains_flat, self.lp_old, adv_flat, ret_flat,
                                                    self.perm_seed, rows_local_full, reward_horizon=self.reward_horizon,
                                                    old_values=self.values)}   # the clipped v_loss's (:110-116)
                if split:
                    bound["actor"] = opt.bind_range(m.grads, 0, na, m.dims, m.precision,
                                                    packs={"actor": (m.actor_ft_params, m.packed_ft)},
                                                    defer_sampler_tables=defer, fused_pack=fuse, clear_grads=fuse)
                    bound["critic"] = opt.bind_range(m.grads, na, ng_all, m.dims, m.precision,
                                                     packs={"critic": (m.critic_params, m.packed_critic)},
                                                     fused_pack=fuse, clear_grads=fuse)
                    if fuse:   # what each half of a full minibatch zeroes, per metrics buffer
                        ws_full = m.workspace(rows_local_full)
                        bound["clear"] = [(ops.ClearRanges(m.dims, m.precision, rows_local_full, ws_full, t, 1),
                                           ops.ClearRanges(m.dims, m.precision, rows_local_full, ws_full, t, 2))
                                          for t in self._met_dev] if fuse else None
                elif self.max_grad_norm is None:
                    bound["all"] = opt.bind_range(m.grads, 0, ng_all, m.dims, m.precision,
                                                  packs={"actor": (m.actor_ft_params, m.packed_ft),
                                                         "critic": (m.critic_params, m.packed_critic)},
                                                  defer_sampler_tables=defer)
                self._bound_key, self._bound = bkey, bound
            run_mb = self._bound["run_mb"]
            step_actor, step_critic = self._bound.get("actor"), self._bound.get("critic")
            step_all = self._bound.get("all")
            clear_next = self._bound.get("clear")
            cleared = False   # the previous optimizer step zeroed this minibatch's accumulators
            # raw device addresses and stream handles, computed once: per minibatch the host passes
            # ints instead of slicing tensors and entering stream contexts (~tens of us per minibatch,
            # which an 8-GPU rank's 255 small minibatches per iteration wait on)
            adv_base = self._adv_all.data_ptr()
            st_main = stream.cuda_stream
            st_side = side.cuda_stream if split else None
            met_ptrs = [t.data_ptr() for t in self._met_dev] if split else None
            k = 0
            for update_epoch in range(self.update_epochs):
                for batch in range(num_batch):
                    start = batch * rows_local_full
                    rows = min(rows_local_full, total_local - start)
                    if rows <= 0:
                        break
                    global_rows = rows * W
                    stats = adv_base + 24 * (update_epoch * num_batch + batch)   # fp64[3] row
                    hp_ = self.host_profile
                    if hp_ is not None:
                        t_h0 = time.perf_counter()
                    if self.update_events is not None:
                        ev0 = torch.cuda.Event(enable_timing=True)
                        ev0.record(stream)
                    mb_args = (update_epoch + 1000 * self.itr, start, rows)
                    prev_mb, last_mb = last_mb, mb_args
                    pre = cleared and rows == rows_local_full
                    mb_kw = dict(global_rows=global_rows, adv_stats=stats)
                    met = m.metrics
                    tagged = self.itr >= self.n_critic_warmup_itr
                    if split:
                        met = self._met_dev[k % 2]
                        met_p = met_ptrs[k % 2]
                        run_mb(*mb_args, **mb_kw, part=2, metrics=met_p, stream=st_side, precleared=pre)
                        if not tagged and not dp:
                            ev_c = torch.cuda.Event()
                            ev_c.record(side)
                        if dp:
                            ng = m.grads.numel()
                            run_mb(*mb_args, **mb_kw, part=4, metrics=met,   # actor row tiles
                                   precleared=pre)
                            self._ev_rows.record(stream)
                            with torch.cuda.stream(side):          # bucket 1: critic gradients + metrics
                                side.wait_event(self._ev_rows)
                                m.grads_ext[ng:ng + 5].copy_(met[:5])
                                m.grads_ext[ng + 5:ng + 6].copy_(met[8:9])   # learn_eta: d loss / d eta
                                self._bucket_allreduce("critic", m.grads_ext[na:])
                                met[:5].copy_(m.grads_ext[ng:ng + 5])
                                met[8:9].copy_(m.grads_ext[ng + 5:ng + 6])
                                self._ev_met.record(side)
                            run_mb(*mb_args, **mb_kw, part=5, metrics=met)   # actor dW + time MLP
                            self._bucket_allreduce("actor", m.grads_ext[:na])      # bucket 2: actor gradients
                            stream.wait_event(self._ev_met)
                        else:
                            run_mb(*mb_args, **mb_kw, part=1, metrics=met_p, stream=st_main, precleared=pre)
                            if not tagged:
                                stream.wait_event(ev_c)
                    else:
                        run_mb(*mb_args, **mb_kw)
                        if dp:                             # one collective: gradients + metric sums
                            ng = m.grads.numel()
                            m.grads_ext[ng:ng + 5].copy_(m.metrics[:5])
                            m.grads_ext[ng + 5:ng + 6].copy_(m.metrics[8:9])
                            self._bucket_allreduce("all", m.grads_ext)
                            m.metrics[:5].copy_(m.grads_ext[ng:ng + 5])
                            m.metrics[8:9].copy_(m.grads_ext[ng + 5:ng + 6])
                    if self.minibatch_hook is not None:
                        if split:
                            stream.wait_stream(side)
                            m.metrics[:5].copy_(met[:5])   # the hook reads model.metrics
                        self.minibatch_hook(update_epoch, batch, start, rows)
                    if hp_ is not None:
                        t_h1 = time.perf_counter()
                    slot = k % 2
                    if pending is not None:
                        info, stop = finish(pending)
                        same_epoch = pending[3] == update_epoch
                        pending = None
                        if stop and same_epoch:                                    # :366-368
                            cleared = False   # this minibatch's sums stay; no step clears them
                            last_mb = prev_mb   # the reference never computes this one
                            break
                    # the optimiser step (agent :346): AdamW, the metric sums to the host and the weight
                    # images re-derived, one dppo_optimizer_step per stream (two launches each). The actor
                    # image skips the split sampler's tables (fold, TIN, W_XS, B_OUT2), which no PPO kernel
                    # reads: the next rollout's first sampler launch re-derives them once
                    # (DPPO_STEP_DEFER_SAMPLER_TABLES)
                    if hp_ is not None:
                        t_h2 = time.perf_counter()
                    ng = m.grads.numel()
                    met_out = self._met_map[slot]
                    tag = ctag = 0
                    if tagged:
                        lr = opt.begin_step()
                        self._mb_tag += 1
                        tag = self._mb_tag
                        if split:
                            ctag = tag
                            ca, cc = clear_next[(k + 1) % 2] if fuse else (None, None)
                            step_actor(lr, metrics=met_p, metrics_out=met_out.address, n_metrics=5, metrics_tag=tag,
                                       stream=st_main, clear=ca)
                            step_critic(lr, metrics=met_p + 8, metrics_out=self._cmet_map[slot].address,   # met[1]
                                        n_metrics=1, metrics_tag=ctag, stream=st_side, clear=cc)
                            cleared = fuse
                        elif self.max_grad_norm is not None:
                            self._clip_by_norm_per_tensor()
                            opt.apply_range(m.grads, 0, ng, lr, m.dims, m.precision,
                                            packs={"actor": (m.actor_ft_params, m.packed_ft),
                                                   "critic": (m.critic_params, m.packed_critic)},
                                            metrics=met, metrics_out=met_out.address, n_metrics=5, metrics_tag=tag,
                                            defer_sampler_tables=defer)
                        else:
                            step_all(lr, metrics=met, metrics_out=met_out.address, n_metrics=5, metrics_tag=tag)
                        if self.learn_eta and batch % self.eta_update_interval == 0:   # :358-359
                            m.eta_optimizer_step(met, self.eta_lr_scheduler(m.eta_step_count), self.eta_weight_decay)
                    else:
                        torch.from_numpy(met_out.array[:5]).copy_(met[:5])
                        cleared = False
                    if self.update_events is not None:
                        ev1 = torch.cuda.Event(enable_timing=True)
                        ev1.record(stream)
                        self.update_events.append((ev0, ev1))
                    ev_m = None
                    if not tag:
                        ev_m = self._ev_m[slot]
                        ev_m.record(stream)
                    pending = (slot, ev_m, global_rows, update_epoch, tag, ctag)
                    k += 1
                    if hp_ is not None:   # host seconds: enqueue grads, wait for the previous metrics, enqueue step
                        t_h3 = time.perf_counter()
                        for key, dt in (("enqueue_grads", t_h1 - t_h0), ("wait_metrics", t_h2 - t_h1),
                                        ("enqueue_step", t_h3 - t_h2)):
                            hp_[key] = hp_.get(key, 0.0) + dt
                        hp_["minibatches"] = hp_.get("minibatches", 0) + 1
            if pending is not None:
                info, _ = finish(pending)
            if split:
                stream.wait_stream(side)
        stream = caller
        # explained variance (:373-377) from the moments value_moments stored before the epochs
        stream.synchronize()
        for g in (getattr(self, "_ipc_groups", None) or {}).values():
            g.check()   # a barrier timeout in any bucket all-reduce of this update
        if self.use_bc_loss and last_mb is not None:
            info["bc_loss"] = self._bc_loss_report(last_mb, obs_flat, total_local, kf)
        info["explained_var"] = explained_variance_from_moments(
            self._ev_map.array.copy(), self.device, group=dist.group.WORLD if self.world_size > 1 else None)
        info["clipfrac"] = float(np.mean(clipfracs)) if clipfracs else 0.0
        return info

    def _bc_loss_report(self, mb, obs_flat, total_local, kf):
        """c_loss's bc_loss (diffusion_ppo.py:63-71) of the update's last minibatch, the value the reference
        logs (train_ppo_diffusion_agent.py:441, 450): base-policy chains for that minibatch's observations
        and their clipped actor_ft log-probs (PPODiffusion.bc_loss). The reference evaluates it on every
        minibatch, but it is not in the loss (:340-342) and only the last value is observable, so only that
        one is computed. Under data parallelism the mean is over the union of the ranks' rows."""
        epoch_key, start, rows = mb
        idx = ops.feistel_permute(start, rows, total_local, self.perm_seed, epoch_key, self.device)
        idx = idx[idx >= 0]
        m = self.model
        n_el = float(idx.numel() * kf * m.dims.xd)
        s = -m.bc_loss(obs_flat[idx // kf]) * n_el if idx.numel() else 0.0   # sum of the clipped log-probs
        if self.world_size > 1:
            t = torch.tensor([s, n_el], dtype=torch.float64, device=self.device)
            self._allreduce(t)
            s, n_el = float(t[0]), float(t[1])
        return -s / max(n_el, 1.0)

    def _clip_by_norm_per_tensor(self):
        """Else-branch of agent :349-353: tf.clip_by_norm(grad, 1.0) per variable."""
        g = self.model.grads
        o = 0
        for spec in (self.model.actor_spec, self.model.critic_spec):
            for _, shape in spec:
                k = int(np.prod(shape))
                seg = g[o:o + k]
                nrm = torch.linalg.vector_norm(seg)
                seg.mul_(torch.clamp(1.0 / torch.clamp(nrm, min=1e-30), max=1.0))
                o += k

    # ------------------------------------------------------------------ one iteration / the loop
    def iteration(self, force_train=None):
        timer = Timer()
        ft = self.force_train if force_train is None else force_train
        eval_mode = self.itr % self.val_freq == 0 and not ft
        torch.cuda.synchronize(self.device)
        self._fit_buffers_to_model()
        t0 = Timer()
        stats = self.rollout(eval_mode, defer_stats=not eval_mode)
        if eval_mode:
            torch.cuda.synchronize(self.device)
        t_roll = t0()   # train iterations: host time to the last env step (the passes run behind it)
        info = {}
        if not eval_mode:
            info = self.update()
            torch.cuda.synchronize(self.device)
            stats = self.episode_stats()
        t_upd = t0()
        self.timing["rollout_s"] += t_roll
        self.timing["update_s"] += t_upd
        self.timing["iters"] += 1
        if not eval_mode:
            self.timing["env_steps"] += self.n_envs_global * self.act_steps * self.n_steps
        self.model.step()
        if self.itr % self.save_model_freq == 0 or self.itr == self.n_train_itr - 1:
            if self.cfg.train.get("save_checkpoints", True):
                self.save_model()
        res = {"itr": self.itr, "step": self.cnt_train_step, "time": timer(), "eval": eval_mode, **stats, **info}
        self.run_results.append(res)
        if self.rank == 0 and self.itr % self.log_freq == 0:
            if eval_mode:
                log.info("eval: success rate %8.4f | avg episode reward %8.4f | avg best reward %8.4f",
                         stats["success_rate"], stats["avg_episode_reward"], stats["avg_best_reward"])
            else:
                log.info("%d: step %8d | loss %8.4f | pg loss %8.4f | value loss %8.4f | reward %8.4f | t:%8.4f",
                         self.itr, self.cnt_train_step, info["loss"], info["pg_loss"], info["v_loss"],
                         stats["avg_episode_reward"], res["time"])
        self.last_info = res
        self.itr += 1
        return res

    def run(self):
        results = self._run_loop()
        if self.world_size > 1:
            self.close_collectives()   # collective: only on the normal exit every rank reaches
        return results

    def _run_loop(self):
        while self.itr < self.n_train_itr:
            self.iteration()
            if self.rank == 0 and self.cfg.train.get("save_results", True):
                os.makedirs(os.path.dirname(self.result_path) or ".", exist_ok=True)
                with open(self.result_path, "wb") as f:
                    pickle.dump(self.run_results, f)
        return self.run_results
