"""Data-parallel pieces of the DPPO iteration, as small functions over torch
tensors so the same code runs on RCCL ("nccl") across GPUs and on gloo in the CPU tests.

Decomposition used by the agent, per PPO minibatch of B global rows over W ranks:
  * every rank draws B/W rows from its OWN rollout shard (env batch split evenly);
  * the advantage moments {n, sum, sumsq} are summed over ranks, so norm_adv uses the global
    minibatch mean / population std (diffusion_ppo.py:74-75);
  * each rank's gradient is scaled by 1/B (not 1/(B/W)) and the gradients are SUMMED, which is
    exactly the gradient of the mean loss over the global minibatch;
  * reward-RMS moments {n, mean, M2} are merged with Chan's rule (identical on every rank);
  * metrics are sums over rows, summed over ranks and divided by B on the host."""
import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _host_staged(t, group=None):
    """gloo reduces host tensors; RCCL ("nccl") device tensors."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def allreduce_sum_(t, group=None):
    if world() > 1:
        if _host_staged(t, group):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def broadcast_(t, src=0, group=None):
    if world() > 1:
        if _host_staged(t, group):
            h = t.cpu()
            dist.broadcast(h, src=src, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src, group=group)
    return t


def shard_envs(n_global, world_size, rank):
    """Contiguous env shard of `rank`: (n_local, first global env index)."""
    if n_global % world_size:
        raise ValueError(f"n_envs={n_global} must divide evenly over {world_size} ranks")
    n = n_global // world_size
    return n, rank * n


def chan_merge(triples):
    """Merge (n, mean, M2) triples in the given order (Chan et al.), in float64."""
    n, mean, m2 = 0.0, 0.0, 0.0
    for gn, gm, g2 in triples:
        gn, gm, g2 = float(gn), float(gm), float(g2)
        if gn == 0:
            continue
        tot = n + gn
        delta = gm - mean
        mean = mean + delta * gn / tot
        m2 = m2 + g2 + delta * delta * n * gn / tot
        n = tot
    return n, mean, m2


def gather_moments(local, group=None):
    """All-gather a local (n, mean, M2) fp64 tensor and merge in rank order."""
    if world() == 1:
        return tuple(float(x) for x in local.cpu())
    if _host_staged(local, group):
        local = local.cpu()
    parts = [torch.zeros_like(local) for _ in range(world())]
    dist.all_gather(parts, local, group=group)
    return chan_merge([tuple(p.cpu().tolist()) for p in parts])


def rms_update(rms, n, mean, m2):
    """RunningMeanStd.update_from_moments (util/reward_scaling.py:29-39) with batch var = M2/n.
    rms = (mean, var, count) -> new tuple."""
    r_mean, r_var, r_count = (float(x) for x in rms)
    bv = m2 / n
    delta = mean - r_mean
    tot = r_count + n
    new_mean = r_mean + delta * n / tot
    M2 = r_var * r_count + bv * n + delta * delta * r_count * n / tot
    return new_mean, M2 / (tot - 1), tot


def adv_norm_from_stats(stats):
    """(count, sum, sumsq) -> (mean, population std) as the kernels use them."""
    c, s, s2 = (float(x) for x in stats)
    mean = s / c
    var = max(s2 / c - mean * mean, 0.0)
    return mean, var ** 0.5


def explained_variance(y_pred, y_true, group=None):
    """1 - Var(y - y_pred) / Var(y) over the rows of all ranks (agent :373-377), from summed
    fp64 moments; nan when Var(y) == 0."""
    y_pred, y_true = y_pred.double(), y_true.double()
    d = y_true - y_pred
    n = torch.tensor(float(y_true.numel()), dtype=torch.float64, device=y_true.device)
    mom = allreduce_sum_(torch.stack([y_true.sum(), (y_true * y_true).sum(), d.sum(), (d * d).sum(), n]), group)
    n = mom[4]
    var_y = float(mom[1] / n - (mom[0] / n) ** 2)
    var_d = float(mom[3] / n - (mom[2] / n) ** 2)
    return float("nan") if var_y == 0 else 1.0 - var_d / var_y


def explained_variance_from_moments(mom, device, group=None):
    """explained_variance from the per-rank moments {sum y, sum y^2, sum d, sum d^2, n} (fp64, as
    dppo_value_moments stores them), summed over ranks when a group is given."""
    import numpy as np
    mom = np.asarray(mom, dtype=np.float64)
    if group is not None:
        t = allreduce_sum_(torch.tensor(mom, dtype=torch.float64, device=device), group)
        mom = t.cpu().numpy()
    n = mom[4]
    var_y = float(mom[1] / n - (mom[0] / n) ** 2)
    var_d = float(mom[3] / n - (mom[2] / n) ** 2)
    return float("nan") if var_y == 0 else 1.0 - var_d / var_y
