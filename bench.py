"""Benchmark: DPPO fine-tuning throughput on MI355X (BASELINE.json metric).

A bench "step" = one full fine-tuning iteration of the hot path on synthetic data: a rollout of
S chunks over E envs (the 20-step DDPM sampler per chunk + host env step + pinned H2D/D2H), the
value and old-log-prob passes, reward scaling, GAE and the PPO epochs (5 x minibatches of
50,000 rows, fused loss+gradient, AdamW). Workload = BASELINE config 2: hopper-v2, 64 envs per GPU,
S = 500, K = 20 DDPM steps (K' = 10), bf16 denoiser. value = whole-job env-steps/s over the full
iteration (rollout + update), summed over ranks (weak scaling: 64 envs per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "env-steps/sec + PPO-updates/sec, hopper-v2 64 envs 20 DDPM steps, 1/2/4/8 GPU"
PEAK = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}  # dense TFLOP/s, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0


def sampler_flops_per_env(d):
    """Algorithmic FLOPs of one K-step sample for one env: K x 2 x MACs of the
    four Dense layers of the needed actor (time MLP excluded, ~0.2%)."""
    h = d.actor_hidden
    macs = d.actor_in * h + 2 * h * h + h * d.xd
    return d.denoising_steps * 2 * macs


CU_LOAD_PEAK_GBS = 64 * 2.4   # per-CU vector-memory (TA) path: 64 B/clk at the 2.4 GHz max clock

# Latency floor of one denoising step of the split sampler (csrc/sampler_split.hip, P = 2 members
# per 16-env group, the default; l2 folded into the out-Dense), the figure its per-step time is
# compared with: one in-launch exchange of partial sums between the P workgroups of a group
# (tools/xchg_probe2.hip: 0.59 us per step at P = 2, 0.98 at 4, with the members on one XCD, sc0
# granules, nothing else in the step) + the step's MFMA issue on one SIMD (2 waves x n
# v_mfma_f32_16x16x32_bf16 x 16 cycles at 2.4 GHz; n per wave = in-Dense 4 + residual 4/P + l1
# 64/P + fold 4/P: P = 2: 4 + 2 + 32 + 2 = 40, P = 4: 4 + 1 + 16 + 1 = 22; r01 8-member kernel 28).
# Everything else in a step (LDS round trips, barriers, VALU epilogues, the DDPM update) is latency
# this floor does not count. fp32 (v_mfma_f32_16x16x4_f32: 4 issues of 32 cycles per 16-wide k-step;
# the in-Dense's state k-step is formed once per launch, so one k-step per step): P = 8 members of 4
# waves, one wave per SIMD issuing in-Dense 8 tiles x 4 + residual 4 + l1 32 k x 4 + fold 4 = 168;
# P = 4 of 8 waves, 2 per SIMD x (16 + 4 + 128 + 4).
SPLIT_DEFAULT_P = 2
SPLIT_MFMA_US_F32 = {8: 168 * 32 / 2.4e3, 4: 2 * 152 * 32 / 2.4e3}
SPLIT_XCHG_US = {2: 0.59, 4: 0.98, 8: 1.55}
SPLIT_MFMA_US = {2: 2 * 40 * 16 / 2.4e3, 4: 2 * 22 * 16 / 2.4e3, 8: 2 * 28 * 16 / 2.4e3}


def sampler_layout(d, precision, envs):
    """Workgroups per 16-env group of the sampler the library runs (0 = weight-streaming kernel)."""
    from diffusionpolicyoptimization_amd import ops
    return ops.sampler_layout(d, precision, envs)


def sampler_stream_bytes_per_tile(d, precision):
    """Weight bytes ONE 16-row sampler tile (one CU) loads per launch (the library reports it for
    the sampler geometry in use: streamed k-steps every denoising step + the resident set once
    per actor; include/dppo.h dppo_sampler_stream_bytes)."""
    import ctypes

    from diffusionpolicyoptimization_amd import _lib
    out, waves = ctypes.c_int64(), ctypes.c_int()
    _lib.call("dppo_sampler_stream_bytes", ctypes.byref(d.c()), _lib.PRECISION[precision],
              ctypes.byref(out), ctypes.byref(waves))
    return out.value


def cpu_baseline(cfg, n_envs, S, bs):
    """CPU baseline (kind "port"): oracle/cpu_reference.py, an fp32 torch-CPU restatement of the
    whole iteration (rollout through the synthetic env, value / log-prob passes, reward scaling,
    GAE, update_epochs x minibatches with autograd + Keras AdamW), timed for ONE FULL iteration of
    this workload on torch's thread pool (the host's CPU share), plus a 1-thread figure from a
    bounded sample (the rollout chunks one full minibatch needs, that minibatch, the passes over
    those chunks) scaled to the iteration. TF-CPU itself cannot be installed (no network)."""
    import torch

    from oracle import cpu_reference as C
    threads = torch.get_num_threads()
    omp = os.environ.get("OMP_NUM_THREADS")
    kw = dict(obs_dim=cfg.obs_dim, action_dim=cfg.action_dim)
    upd = int(cfg.train.update_epochs)
    t_full, br = C.time_iteration(n_envs, S, bs, upd, **kw)
    n_mb = br["minibatches"]
    # 1 thread: enough chunks for one full minibatch of bs rows (S*E*K' >= bs) + that minibatch,
    # scaled to the iteration
    s1 = min(S, max(10, -(-bs // (n_envs * cfg.ft_denoising_steps))))
    t1, b1 = C.time_iteration(n_envs, s1, bs, upd, threads=1, max_minibatches=1, **kw)
    torch.set_num_threads(threads)
    t1_iter = (b1["rollout_s"] + b1["passes_s"]) * S / s1 + b1["update_s"] / max(1, b1["minibatches"]) * n_mb
    env_steps = n_envs * cfg.act_steps * S
    return {"value": env_steps / t_full, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "threads": threads, "physical_cores": C.physical_cores(), "cpu_model": C.cpu_model(),
            "value_1thread": env_steps / t1_iter,
            "ppo_updates_per_sec": n_mb / br["update_s"] if br["update_s"] > 0 else None,
            "seconds_per_iter": t_full, "breakdown_s": {k: br[k] for k in ("rollout_s", "passes_s", "update_s")},
            "cores_note": (f"{threads} threads = torch's pool, which follows OMP_NUM_THREADS={omp}: the CPU share the GPU "
                           "box gives one GPU's job (the harness sets it to 16 per GPU and its process guard limits "
                           "the job's CPU use; nproc / os.cpu_count() show the whole host, "
                           f"{C.physical_cores()} physical cores, shared with the other GPUs' jobs)"),
            "sample": (f"oracle/cpu_reference.py (fp32 torch-CPU, autograd) timed on ONE full iteration: {n_envs} "
                       f"envs x {S} chunks, K={cfg.denoising_steps}, {n_mb} minibatches of {bs} rows, "
                       f"{threads} threads, {t_full:.1f} s; value_1thread from {s1} chunks + 1 full minibatch "
                       f"on 1 thread scaled to the iteration ({t1_iter:.0f} s/iter)")}


# per-kernel figures (north_star: "achieved HBM GB/s on the DDPM/GAE kernels and MFMA utilisation
# on the denoiser GEMMs"), computed from ALGORITHMIC bytes / FLOPs (with the dtypes
# the kernels actually move) over per-kernel launch times. The figures are measured LIVE in this
# run: the library's kernel timer (dppo_kernel_timing, HIP events around each launch on its own
# stream) over one instrumented iteration. The committed rocprofv3 whole-iteration trace of the
# same workload is reported beside them as a cross-check.
KERNEL_STATS_CSV = os.path.join(ROOT, "profiles", "r06end_iteration_kernel_stats.csv")


def kernel_times_live(agent):
    """One untimed iteration with the library's kernel timer on: {kernel: (total_ms, launches)}."""
    import ctypes

    import numpy as np
    from diffusionpolicyoptimization_amd import _lib
    lib = _lib.load()
    names = []
    while True:
        nm = lib.dppo_kernel_timing_name(len(names))
        if not nm:
            break
        names.append(nm.decode())
    _lib.call("dppo_kernel_timing", 1)
    try:
        agent.iteration(force_train=True)
        tot = np.zeros(len(names))
        cnt = np.zeros(len(names), np.int64)
        _lib.call("dppo_kernel_timing_read", len(names), ctypes.c_void_p(tot.ctypes.data), ctypes.c_void_p(cnt.ctypes.data))
    finally:
        _lib.call("dppo_kernel_timing", 0)
    return {n: (float(t), int(c)) for n, t, c in zip(names, tot, cnt) if c > 0}


def kernel_stats_csv(path=KERNEL_STATS_CSV):
    """{base kernel name: (total_ms, launches)} of a committed rocprofv3 --stats CSV (the cross-check)."""
    import csv
    if not os.path.exists(path):
        return None
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Name"]
            k = k[5:] if k.startswith("void ") else k
            base = k.split("<")[0].split("(")[0].split("::")[-1]
            if "pack_all_kernel" in base or base == "rt_fold_kernel":   # the live timer's KT_PACK_ALL scope
                base = "pack_all_kernel"
            elif base == "time_l2_bwd_kernel":
                base = "time_bwd_kernel"
            elif "actor_tile_step_kernel" in k or "actor_step_kernel" in k:
                base = "adamw_kernel"
            elif base.startswith("actor_rowtile_kernel"):
                base = "actor_rowtile_train" if "true" in k else "actor_rowtile_logprob"
            elif base.startswith("critic_rowtile_kernel"):
                base = "critic_rowtile_train" if "true" in k else "critic_rowtile_forward"
            elif base == "adv_stats_all_kernel":
                base = "adv_stats_kernel"
            elif "adamw_fused_kernel" in base:   # (rocprof leaves this template's name mangled)
                base = "adamw_kernel"
            tot, calls = float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])
            t0, c0 = out.get(base, (0.0, 0))
            out[base] = (t0 + tot, c0 + calls)
    return out


def kernel_figures(d, S, E, batch, n_mb, precision, times, source, iters=1):
    """times: {kernel: (total_ms, launches)} over `iters` iterations with n_mb minibatches of `batch` rows."""
    out = {"source": source, "hbm_peak_GBs": HBM_PEAK_GBS, "minibatches": n_mb}
    N = S * E
    na = d.actor_in * d.actor_hidden + 2 * d.actor_hidden ** 2 + d.actor_hidden * d.xd  # actor weights (MACs/row)
    n_par = None
    try:
        from diffusionpolicyoptimization_amd import ops
        n_par = ops.spec_count(ops.actor_param_spec(d)) + ops.spec_count(ops.critic_param_spec(d))
    except Exception:
        pass
    hbm = {
        # reward f64 + values f32 + terminated u8 in, advantages + returns f32 out; + last values
        "gae_kernel": (21 * N + 4 * E, "21 B per (t, e): r f64, V f32, term u8 in; A, R f32 out"),
        # forward scan: r f64 + first u8 in, rets f64 out; moments: rets f64 in; apply: r f64 in + out
        "rets_kernel": (17 * N, "17 B per (t, e)"),
        "moments_kernel": (8 * N, "8 B per (t, e)"),
        "scale_apply_kernel": (16 * N, "16 B per (t, e)"),
    }
    for name, (nbytes, note) in hbm.items():
        if name in times:
            tot, calls = times[name]
            avg = tot / calls * 1e6          # ns
            out[name] = {"bytes_per_launch": nbytes, "launches": calls, "avg_us": avg / 1e3,
                         "achieved_GBs": nbytes / avg, "frac": nbytes / avg / HBM_PEAK_GBS, "note": note}
    if "adamw_kernel" in times and n_par:
        tot, calls = times["adamw_kernel"]
        per_mb = 28 * n_par            # p, g, m, v in; p, m, v out (fp32) over actor_ft + critic
        ns = tot * 1e6 / n_mb
        out["adamw_kernel"] = {"bytes_per_minibatch": per_mb, "launches_per_minibatch": calls / n_mb,
                               "us_per_minibatch": ns / 1e3, "achieved_GBs": per_mb / ns, "frac": per_mb / ns / HBM_PEAK_GBS,
                               "note": "28 B per parameter, actor and critic ranges summed (two launches under "
                                       "the split update, on two streams; since ABI 11 each also stores its "
                                       "network's image slots and zeroes the next minibatch's accumulators, "
                                       "replacing the pack and zero launches); durations include sharing the CUs"}
    peak = PEAK["bf16" if precision in ("bf16", "fp16") else "fp32"]
    if "actor_rowtile_train" in times:
        tot, calls = times["actor_rowtile_train"]
        fl = 2 * 2 * na * batch            # forward + backward-dX of the actor, per minibatch
        ns = tot * 1e6 / n_mb
        out["actor_rowtile_train"] = {"flops_per_minibatch": fl, "launches": calls, "us_per_minibatch": ns / 1e3,
                                      "achieved_TFLOPs": fl / ns / 1e3, "frac": fl / ns / 1e3 / peak,
                                      "note": "algorithmic FLOPs of the reference network (its l2 layer included); "
                                              "since r05 the kernel folds l2 into the out-Dense (DESIGN §3) and "
                                              "computes about half of them"}
    dw = [times[k] for k in ("dw_kernel_actor", "dw_kernel_critic", "dw_kernel") if k in times]
    if dw:
        tot = sum(t for t, _ in dw)
        hc = d.critic_hidden
        nc = d.sd * hc + 2 * hc * hc + hc
        fl = 2 * (na + nc) * batch         # actor + critic weight gradients over the minibatch rows
        ns = tot * 1e6 / n_mb
        out["dw_kernel"] = {"flops_per_minibatch": fl, "us_per_minibatch": ns / 1e3,
                            "achieved_TFLOPs": fl / ns / 1e3, "frac": fl / ns / 1e3 / peak,
                            "note": "actor + critic launches summed; algorithmic FLOPs as the reference computes "
                                    "them (every row for the critic, which runs on distinct samples only; l2's "
                                    "H x H weight gradient, which the kernels form as (u2^T dy) W_out^T)"}
        for k in ("dw_kernel_actor", "dw_kernel_critic"):
            if k in times:
                out["dw_kernel"][k.replace("dw_kernel_", "") + "_us_per_minibatch"] = times[k][0] * 1e3 / n_mb
    if "actor_rowtile_logprob" in times:
        tot, calls = times["actor_rowtile_logprob"]
        fl = 2 * na * N * d.ft_denoising_steps * iters   # the old-log-prob pass over S*E*K' rows per iteration
        out["actor_rowtile_logprob"] = {"flops_per_iteration": fl, "launches": calls, "avg_us": tot * 1e3 / calls,
                                        "achieved_TFLOPs": fl / (tot * 1e9), "frac": fl / (tot * 1e9) / peak,
                                        "note": "launched in chunks during the rollout (every 10 env steps, beside "
                                                "the sampler), so the FLOPs are summed over the iteration's launches"}
    for k in ("time_bwd_kernel", "l2_back_kernel", "pack_all_kernel", "zero_kernel", "crit_rows_kernel",
              "critic_rowtile_train", "critic_rowtile_forward", "adv_stats_kernel"):
        if k in times:
            tot, calls = times[k]
            out.setdefault("latency_kernels_us", {})[k] = {"launches": calls, "avg_us": tot * 1e3 / calls}
    if "sampler" in times:
        tot, calls = times["sampler"]
        out["sampler_in_rollout"] = {"launches": calls, "avg_us": tot * 1e3 / calls,
                                     "note": "pipelined launches: each includes its wait for the host's observation"}
    return out


def sampler_burst_ms(agent, n=30):
    """Average sampler launch duration with HIP events on the launch stream, over n launches
    enqueued back to back on the rollout's own buffers (same workload as the timed region). The
    per-step events inside the rollout also contain the host's enqueue gap after the event record
    (the stream is idle between env steps), so they overstate the kernel; this burst measures the
    kernel itself and is what rocprofv3's per-kernel average reports."""
    import torch
    m = agent.model
    stream = torch.cuda.current_stream(agent.device)
    args = dict(deterministic=False, return_chain=True, actions_out=agent.act_dev, chains_out=agent.chains_traj[0])
    m(agent.obs_traj[0], **args)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(agent.device)
    ev0.record(stream)
    for _ in range(n):
        m(agent.obs_traj[0], **args)
    ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / n, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config-dir", default=os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"))
    ap.add_argument("--config-name", default="ft_ppo_diffusion_mlp_64env")
    ap.add_argument("--envs-per-gpu", type=int, default=64)
    ap.add_argument("--n-steps", type=int, default=None, help="override S (chunks per rollout)")
    ap.add_argument("--precision", default=None)
    ap.add_argument("--batch-size", type=int, default=None, help="override train.batch_size (measurement)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="measurement mode: run ONE rank's share of an N-rank job on this GPU (the reference's "
                         "global minibatch split N ways: N x the minibatches of batch_size / N rows), every "
                         "collective skipped; value = N x this rank's env steps / its time (a bound on the "
                         "N-GPU number without collective time)")
    ap.add_argument("--env", choices=["synthetic", "lowdim"], default="synthetic",
                    help="synthetic: the AVX2 synthetic stepper (the headline workload); lowdim: the reference's "
                         "MultiStep + lowdim wrapper stack (csrc/envwrap.c) on the hopper normalization.npz over the "
                         "C linear simulator, pipelined through the gated thread-pool step")
    ap.add_argument("--env-threads", type=int, default=None, help="lowdim: host threads stepping the envs")
    ap.add_argument("--sim-cost-us", type=float, default=0.0,
                    help="lowdim: emulated physics work per env sub-step of the C simulator (measurement knob)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    world = int(os.environ.get("WORLD_SIZE", "1"))
    over = [f"env.n_envs={args.envs_per_gpu * world}", "train.force_train=True", "train.save_checkpoints=False",
            "train.save_results=False", "train.n_train_itr=1000000", "logdir=/tmp/dppo_bench"]
    if args.n_steps:
        over.append(f"train.n_steps={args.n_steps}")
    if args.precision:
        over.append(f"model.precision={args.precision}")
    if args.batch_size:
        over.append(f"train.batch_size={args.batch_size}")
    if args.env == "lowdim":
        npz = os.path.join(ROOT, "tests", "golden", "hopper_medium_v2_normalization.npz")
        over += ["env.synthetic=lowdim", f"+env.wrappers.mujoco_locomotion_lowdim.normalization_path={npz}",
                 f"+env.sim_cost_us={args.sim_cost_us}"]
        if args.env_threads:
            over.append(f"+env.num_threads={args.env_threads}")
    emu = max(1, args.emulate_ranks)
    if emu > 1:
        if world > 1:
            raise SystemExit("--emulate-ranks runs one process")
        over.append(f"train.emulate_world={emu}")
    cfg = load_config(args.config_dir, args.config_name, over)
    agent = get_class(cfg._target_)(cfg)
    rank = agent.rank
    dev = agent.device
    d = agent.model.dims

    for _ in range(args.warmup):
        agent.iteration(force_train=True)
    # the timed region carries no per-minibatch HIP timing events (their records sit on the
    # minibatch chain); ppo_minibatch_avg_ms comes from one instrumented iteration after it
    agent.sampler_events, agent.update_events = None, None
    agent.timing.update(rollout_s=0.0, update_s=0.0, n_updates=0, env_steps=0, iters=0)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.iteration(force_train=True)
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, agent.timing["rollout_s"], agent.timing["update_s"]], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, t_roll, t_upd = t.tolist()
    n_updates = agent.timing["n_updates"]

    agent.sampler_events, agent.update_events = [], []   # instrumented, untimed
    agent.host_profile = {}
    agent.iteration(force_train=True)
    barrier()
    hp = agent.host_profile
    host_us = {k: 1e6 * v / max(1, hp.get("minibatches", 0)) for k, v in hp.items() if k != "minibatches"}
    loop_samp_ms = sum(a.elapsed_time(b) for a, b in agent.sampler_events) / max(1, len(agent.sampler_events))
    samp_ms, n_burst = sampler_burst_ms(agent)
    upd_ms = sum(a.elapsed_time(b) for a, b in agent.update_events) / max(1, len(agent.update_events))
    env_steps = agent.n_envs_global * cfg.act_steps * cfg.train.n_steps * args.steps * emu
    flops = sampler_flops_per_env(d) * agent.n_envs
    prec = agent.model.precision
    members = sampler_layout(d, prec, agent.n_envs)
    from diffusionpolicyoptimization_amd import ops as _ops
    plan = _ops.sampler_plan(d, prec, agent.n_envs)
    kname = {0: "sample_kernel", 2: "sample_split4_kernel"}[plan["kernel"]]
    achieved = flops / (samp_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if kname + "<" in tj.get("kernel", "") and tj.get("precision") == prec and tj.get("envs") == agent.n_envs:
            traffic = tj.get("hbm_bytes_per_launch")
    if members:
        P = plan["members"] or SPLIT_DEFAULT_P
        step_us = samp_ms * 1e3 / d.denoising_steps
        floor_us = SPLIT_XCHG_US[P] + (SPLIT_MFMA_US_F32 if prec == "fp32" else SPLIT_MFMA_US)[P]
        bound = {"kind": "latency", "kernel": kname, "workgroups_per_16_envs": members, "members_per_set": P,
                 "sampler_plan": plan,
                 "us_per_denoising_step": step_us, "floor_us_per_step": floor_us, "frac": floor_us / step_us,
                 "note": (f"each 16-env group runs on {P} CUs with 1/{P} of an actor resident in registers and "
                          "LDS (the base and fine-tuned actors' steps on two such member sets when "
                          "workgroups_per_16_envs is twice members_per_set); a denoising step is a dependent "
                          "chain of small GEMMs (M = 16 envs; l2 folded into the out-Dense) and one cross-CU "
                          "partial-sum exchange, so its floor "
                          "is that exchange (tools/xchg_probe2.hip) plus the step's MFMA issue, not bytes or "
                          "FLOPs; see DESIGN.md")}
    else:
        stream_b = sampler_stream_bytes_per_tile(d, prec)
        bound = {"kind": "load_path", "kernel": kname, "bytes_per_cu_per_launch": stream_b,
                 "achieved_GBs_per_cu": stream_b / (samp_ms * 1e-3) / 1e9, "peak_GBs_per_cu": CU_LOAD_PEAK_GBS,
                 "frac": stream_b / (samp_ms * 1e-3) / 1e9 / CU_LOAD_PEAK_GBS,
                 "note": "each 16-row tile streams its actor's weights from L2 into one CU every denoising step"}
    out = {
        "metric": METRIC, "value": env_steps / elapsed, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": prec, "data": "synthetic",
        "config": {"workload": (f"{cfg.env_name} DPPO fine-tune iteration: {agent.n_envs} envs/GPU x "
                                f"{cfg.train.n_steps} chunks (Ta={cfg.horizon_steps}), K={d.denoising_steps} DDPM "
                                f"steps (K'={d.ft_denoising_steps}), {cfg.train.update_epochs} PPO epochs x "
                                f"minibatch {cfg.train.batch_size}, {prec} denoiser, " + (
                                    "synthetic linear env" if args.env == "synthetic" else
                                    f"reference wrapper stack (MultiStep + MujocoLocomotionLowdimWrapper in C, "
                                    f"{agent.venv.num_threads} host threads) over the C linear simulator"
                                    + (f" with {args.sim_cost_us} us emulated work per env sub-step"
                                       if args.sim_cost_us else ""))),
                   "env": args.env,
                   "global_envs": agent.n_envs_global, "chunks_per_rollout": cfg.train.n_steps,
                   "parallelism": f"dp{world} (env shards + RCCL grad all-reduce)" if world > 1 else "single GPU",
                   "batch_semantics": (f"per-rank minibatch {cfg.train.batch_size} (global {cfg.train.batch_size * world}, "
                                       "train.dp_scale_batch=true)" if agent.dp_scale_batch and world > 1 else
                                       f"global minibatch {cfg.train.batch_size} rows = the reference's "
                                       f"({cfg.train.batch_size // world} per rank)")},
        "ppo_updates_per_sec": n_updates / elapsed,
        "rollout_env_steps_per_sec": env_steps / t_roll if t_roll > 0 else None,
        "rollout_s_per_iter": t_roll / args.steps, "update_s_per_iter": t_upd / args.steps,
        "sampler_bound": bound,
        "roofline": {"bound": "mfma", "kernel": kname + " (K-step DDPM sampler, all layers fused)",
                     "achieved": achieved, "peak": PEAK[prec], "unit": "TFLOP/s",
                     "frac": achieved / PEAK[prec], "traffic": traffic,
                     "avg_launch_ms": samp_ms, "flops_per_launch": flops, "burst_launches": n_burst,
                     "in_loop_event_ms": loop_samp_ms if agent.sampler_events else None,
                     "note": ("M = envs/GPU rows per GEMM: at 64 envs the sampler is a dependent chain of "
                              "K x 3 small GEMMs (in-Dense, l1, the folded l2 + out-Dense), far below MFMA peak by "
                              "construction; sampler_bound gives "
                              "the figure that bounds it")},
        "ppo_minibatch_avg_ms": upd_ms,
        "host_us_per_minibatch": host_us,
    }
    n_mb_iter = n_updates / max(1, args.steps)
    if emu == 1:
        mb_before = agent.timing["n_updates"]
        live = kernel_times_live(agent)
        n_mb_live = agent.timing["n_updates"] - mb_before
        figs = kernel_figures(d, cfg.train.n_steps, agent.n_envs, cfg.train.batch_size, n_mb_live or 1, prec, live,
                              "live: dppo_kernel_timing (HIP events around each launch) over one untimed iteration")
        prof = kernel_stats_csv()
        if prof:
            n_mb_prof = prof.get("actor_rowtile_train", (0, n_mb_live))[1] or n_mb_live
            cross = kernel_figures(d, cfg.train.n_steps, agent.n_envs, cfg.train.batch_size, n_mb_prof, prec, prof,
                                   os.path.relpath(KERNEL_STATS_CSV, ROOT),
                                   iters=max(1, round(n_mb_prof / max(1, n_mb_live))))
            figs["profile_crosscheck"] = {k: v for k, v in cross.items() if k != "hbm_peak_GBs"}
        out["kernels"] = figs
    if emu > 1:
        out["emulated_ranks"] = emu
        out["scaling"] = "weak (emulated)"
        out["config"]["parallelism"] = f"ONE rank of dp{emu} emulated on 1 GPU (collectives skipped)"
        out["config"]["batch_semantics"] = (f"global minibatch {cfg.train.batch_size} rows = the reference's "
                                            f"({cfg.train.batch_size // emu} per rank, {int(n_mb_iter)} minibatches "
                                            "per rank per iteration)")
        out["note"] = (f"value = {emu} x this rank's env steps / its wall time: the {emu}-GPU throughput this "
                       "rank's compute allows, all-reduce time excluded (an upper bound on the real run)")
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, agent.n_envs, cfg.train.n_steps, cfg.train.batch_size)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
