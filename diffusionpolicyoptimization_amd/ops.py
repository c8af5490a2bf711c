"""Thin torch-tensor wrappers over the C ABI (include/dppo.h).

Tensors are device tensors owned by the caller; every op is enqueued on the current torch
stream of the tensor's device. Shapes/dtypes are checked here before any launch so that a bad
call can never reach a kernel with mismatched extents.
"""
import ctypes
import functools
import os
import math
import time
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import ptr, stream_handle


@dataclass(frozen=True)
class ModelDims:
    obs_dim: int = 11
    action_dim: int = 3
    horizon_steps: int = 4
    cond_steps: int = 1
    time_dim: int = 16
    actor_hidden: int = 512
    critic_hidden: int = 256
    denoising_steps: int = 20       # sampling steps (DDIM: ddim_steps)
    ft_denoising_steps: int = 10
    time_stride: int = 1            # diffusion time of sampling row r is r * time_stride (DDIM: K / S)

    @property
    def xd(self):
        return self.horizon_steps * self.action_dim

    @property
    def sd(self):
        return self.cond_steps * self.obs_dim

    @property
    def actor_in(self):
        return self.xd + self.time_dim + self.sd

    def c(self):
        return _lib.DppoDims(self.obs_dim, self.action_dim, self.horizon_steps, self.cond_steps, self.time_dim,
                             self.actor_hidden, self.critic_hidden, self.denoising_steps, self.ft_denoising_steps,
                             self.time_stride)


def actor_param_spec(d: ModelDims):
    """Flat fp32 layout of include/dppo.h (Keras kernels [in,out])."""
    td, h, xd = d.time_dim, d.actor_hidden, d.xd
    return [("time_w1", (td, 2 * td)), ("time_b1", (2 * td,)), ("time_w2", (2 * td, td)), ("time_b2", (td,)),
            ("in_w", (d.actor_in, h)), ("in_b", (h,)), ("l1_w", (h, h)), ("l1_b", (h,)),
            ("l2_w", (h, h)), ("l2_b", (h,)), ("out_w", (h, xd)), ("out_b", (xd,))]


def critic_param_spec(d: ModelDims):
    h = d.critic_hidden
    return [("in_w", (d.sd, h)), ("in_b", (h,)), ("l1_w", (h, h)), ("l1_b", (h,)),
            ("l2_w", (h, h)), ("l2_b", (h,)), ("out_w", (h, 1)), ("out_b", (1,))]


def spec_count(spec):
    return int(sum(int(np.prod(s)) for _, s in spec))


# Per-dims constants of the hot host paths, computed once: the update loop calls the minibatch,
# optimiser and repack wrappers ~10x per PPO minibatch, and at the per-rank minibatch of an 8-GPU
# run (6,250 rows) their Python cost, not the GPU, set the pace.
@functools.lru_cache(maxsize=None)
def _dims_c(d):
    return d.c()


@functools.lru_cache(maxsize=None)
def _n_params(d):
    return spec_count(actor_param_spec(d)), spec_count(critic_param_spec(d))


@functools.lru_cache(maxsize=None)
def _packed_bytes(d, prec):
    return (int(_lib.query("dppo_actor_packed_bytes", ctypes.byref(_dims_c(d)), prec)),
            int(_lib.query("dppo_critic_packed_bytes", ctypes.byref(_dims_c(d)), prec)))


@functools.lru_cache(maxsize=None)
def _workspace_bytes(d, prec, rows):
    return int(_lib.query("dppo_ppo_workspace_bytes", ctypes.byref(_dims_c(d)), prec, int(rows)))


def flatten_params(spec, params):
    return np.concatenate([np.asarray(params[n], np.float32).reshape(-1) for n, _ in spec])


def unflatten_params(spec, flat):
    out, o = {}, 0
    flat = np.asarray(flat)
    for n, s in spec:
        k = int(np.prod(s))
        out[n] = flat[o:o + k].reshape(s)
        o += k
    return out


def _check(t, shape, dtype, name):
    if t is None:
        return
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def _prec(precision):
    return _lib.PRECISION[precision] if isinstance(precision, str) else int(precision)


# ------------------------------------------------------------------------------------------------
# packing
# ------------------------------------------------------------------------------------------------
def actor_packed_bytes(d: ModelDims, precision):
    return int(_lib.query("dppo_actor_packed_bytes", ctypes.byref(d.c()), _prec(precision)))


def pack_all(d: ModelDims, precision, actor_params=None, packed_actor=None, critic_params=None, packed_critic=None):
    """Both images (either pair may be None) in one launch (dppo_pack_all)."""
    p = _prec(precision)
    na, nc = _n_params(d)
    ab, cb = _packed_bytes(d, p)
    _check(actor_params, (na,), torch.float32, "actor params")
    _check(packed_actor, (ab,), torch.uint8, "packed actor")
    _check(critic_params, (nc,), torch.float32, "critic params")
    _check(packed_critic, (cb,), torch.uint8, "packed critic")
    t = actor_params if actor_params is not None else critic_params
    _lib.call("dppo_pack_all", ctypes.byref(_dims_c(d)), p, ptr(actor_params), ptr(packed_actor), ptr(critic_params),
              ptr(packed_critic), stream_handle(t.device))


def optimizer_step(d: ModelDims, precision, params, grads, m, v, step, lr, weight_decay, beta1, beta2, eps, mode,
                   actor_params=None, packed_actor=None, critic_params=None, packed_critic=None, metrics=None,
                   metrics_out=None, n_metrics=0, metrics_tag=0, defer_sampler_tables=False):
    """AdamW over params/grads/m/v (equal-length flat ranges), the metric sums copied to
    metrics_out (a device tensor or a dppo_host_alloc address), then the given images re-derived:
    two launches on the current stream (dppo_optimizer_step). A nonzero metrics_tag is stored as
    metrics_out[n_metrics] after the sums (the host polls it instead of an event).
    defer_sampler_tables: the actor image's split-sampler tables are left stale and re-derived by
    the next sampler launch on it (DPPO_STEP_DEFER_SAMPLER_TABLES; the PPO kernels never read them)."""
    n = params.numel()
    for t, nm in ((grads, "grads"), (m, "m"), (v, "v")):
        if t.numel() != n:
            raise ValueError(f"{nm}: expected {n} elements")
    p = _prec(precision)
    mo = metrics_out if isinstance(metrics_out, int) else (metrics_out.data_ptr() if metrics_out is not None else None)
    _lib.call("dppo_optimizer_step", ctypes.byref(_dims_c(d)), p, ptr(params), ptr(grads), ptr(m), ptr(v), int(n),
              int(step), float(lr), float(weight_decay), float(beta1), float(beta2), float(eps),
              (_lib.DPPO_ADAMW_KERAS if mode == "keras" else _lib.DPPO_ADAMW_TORCH) |
              (_lib.DPPO_STEP_DEFER_SAMPLER_TABLES if defer_sampler_tables else 0), ptr(actor_params), ptr(packed_actor),
              ptr(critic_params), ptr(packed_critic), ptr(metrics), ctypes.c_void_p(mo) if mo else None,
              int(n_metrics), ctypes.c_uint64(int(metrics_tag)), stream_handle(params.device))


def refresh_sampler_tables(packed_actor):
    """Re-derive an actor image's split-sampler tables on the current stream if an optimizer step
    deferred them (no-op otherwise); sampler launches do this themselves (dppo_refresh_sampler_tables)."""
    _lib.call("dppo_refresh_sampler_tables", ptr(packed_actor), stream_handle(packed_actor.device))


def episode_sums(reward, firsts, act_steps, success_threshold, out):
    """a16 (train_ppo_diffusion_agent.py:144-167) on the device: reward fp64 [S,E] (raw), firsts u8
    [S+1,E] -> out fp64 [E,4] rows {episodes, sum of returns, sum of best rewards, successes} per env
    (dppo_episode_sums); sum the rows in env order."""
    S, E = reward.shape
    if reward.dtype != torch.float64 or firsts.dtype != torch.uint8 or tuple(firsts.shape) != (S + 1, E):
        raise ValueError("episode_sums: reward fp64 [S,E] and firsts u8 [S+1,E] expected")
    if out.dtype != torch.float64 or tuple(out.shape) != (E, 4) or not (reward.is_contiguous() and firsts.is_contiguous()
                                                                          and out.is_contiguous()):
        raise ValueError("episode_sums: out fp64 [E,4], all contiguous")
    _lib.call("dppo_episode_sums", ptr(reward), ptr(firsts), int(S), int(E), int(act_steps), float(success_threshold),
              ptr(out), stream_handle(reward.device))
    return out


def value_moments(values, returns, out_address):
    """{sum y, sum y^2, sum d, sum d^2, n} of y = returns, d = returns - values (fp64) into 5 doubles
    at out_address (host-mapped, dppo_host_alloc) or a device tensor (dppo_value_moments)."""
    n = values.numel()
    if returns.numel() != n:
        raise ValueError("values / returns: length mismatch")
    out = out_address if isinstance(out_address, int) else out_address.data_ptr()
    _lib.call("dppo_value_moments", ptr(values), ptr(returns), int(n), ctypes.c_void_p(out), stream_handle(values.device))


class _HostBlock:
    """Owner of one dppo_host_alloc block: freed (dppo_host_free) when the last view of it is gone.
    The ctypes array every NumPy / torch view is built on holds it, so no view outlives the memory."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        _lib.call("dppo_host_alloc", ctypes.c_size_t(nbytes), ctypes.byref(p))
        self.address, self.nbytes = p.value, nbytes

    def view(self):
        buf = (ctypes.c_uint8 * self.nbytes).from_address(self.address)
        buf.owner = self
        return np.ctypeslib.as_array(buf)

    def __del__(self):
        if getattr(self, "address", None) and _lib._lib is not None:
            _lib.query("dppo_host_free", ctypes.c_void_p(self.address))
            self.address = None


class MappedArray:
    """A NumPy array (and a torch CPU view of it) over coherent mapped pinned memory
    (dppo_host_alloc): the host writes it, copy_from_host moves it to the device in one kernel.
    The memory is freed when the MappedArray and every array / tensor view of it are gone; a
    pending device copy from it must be complete by then (the owner synchronises first)."""

    def __init__(self, shape, dtype):
        nbytes = int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize
        block = _HostBlock(max(1, nbytes))
        self.address = block.address
        self.array = block.view()[:nbytes].view(dtype).reshape(shape)
        self.array[...] = 0
        self.tensor = torch.from_numpy(self.array)


class MappedRef:
    """address + size of a dppo_host_alloc buffer owned elsewhere (copy_from_host source)."""

    def __init__(self, address, nbytes):
        self.address, self.nbytes = address, nbytes


def copy_from_host(pairs, stream=None):
    """[(device tensor, MappedArray | MappedRef)] -> one dppo_copy_from_host launch on the current
    stream."""
    if not pairs:
        return
    if len(pairs) > 4:
        raise ValueError("copy_from_host: at most 4 ranges per launch")
    n = len(pairs)
    dst = (ctypes.c_void_p * n)(*[t.data_ptr() for t, _ in pairs])
    src = (ctypes.c_void_p * n)(*[m.address for _, m in pairs])
    nb = (ctypes.c_size_t * n)()
    for i, (t, m) in enumerate(pairs):
        n_src = m.nbytes if isinstance(m, MappedRef) else m.array.nbytes
        if not t.is_cuda or not t.is_contiguous() or t.numel() * t.element_size() != n_src:
            raise ValueError("copy_from_host: destination must be a contiguous device tensor of the source's size")
        nb[i] = n_src
    _lib.call("dppo_copy_from_host", n, dst, src, nb, stream_handle(pairs[0][0].device) if stream is None else stream)


class MappedDoubles:
    """n doubles of coherent mapped pinned memory (dppo_host_alloc) the device stores into and the
    host reads as a numpy array (the PPO metric sums of dppo_optimizer_step)."""

    def __init__(self, n):
        p = ctypes.c_void_p()
        _lib.call("dppo_host_alloc", ctypes.c_size_t(8 * n), ctypes.byref(p))
        self.address = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_double * n).from_address(self.address))
        self.array[:] = 0.0

    def wait_tag(self, index, tag, timeout_s=30.0):
        """Spin until array[index] == tag (a tag the device stores after the data it guards)."""
        a = self.array
        if a[index] == tag:
            return
        t_end = time.perf_counter() + timeout_s
        while a[index] != tag:
            if time.perf_counter() > t_end:
                raise _lib.DppoError(f"mapped tag {tag} not seen within {timeout_s} s (found {a[index]})")

    def __del__(self):
        if getattr(self, "address", None) and _lib._lib is not None:
            _lib.query("dppo_host_free", ctypes.c_void_p(self.address))
            self.address = None


def critic_packed_bytes(d: ModelDims, precision):
    return int(_lib.query("dppo_critic_packed_bytes", ctypes.byref(d.c()), _prec(precision)))


def pack_actor(d: ModelDims, params_flat, precision, out=None):
    p = _prec(precision)
    _check(params_flat, (_n_params(d)[0],), torch.float32, "actor params")
    if out is None:
        out = torch.empty(_packed_bytes(d, p)[0], dtype=torch.uint8, device=params_flat.device)
    else:
        _check(out, (_packed_bytes(d, p)[0],), torch.uint8, "packed actor")
    _lib.call("dppo_pack_actor", ctypes.byref(_dims_c(d)), p, ptr(params_flat), ptr(out),
              stream_handle(params_flat.device))
    return out


def pack_critic(d: ModelDims, params_flat, precision, out=None):
    p = _prec(precision)
    _check(params_flat, (_n_params(d)[1],), torch.float32, "critic params")
    if out is None:
        out = torch.empty(_packed_bytes(d, p)[1], dtype=torch.uint8, device=params_flat.device)
    else:
        _check(out, (_packed_bytes(d, p)[1],), torch.uint8, "packed critic")
    _lib.call("dppo_pack_critic", ctypes.byref(_dims_c(d)), p, ptr(params_flat), ptr(out),
              stream_handle(params_flat.device))
    return out


# ------------------------------------------------------------------------------------------------
# sampler / logprob / critic
# ------------------------------------------------------------------------------------------------
def sample(d: ModelDims, precision, packed_base, packed_ft, sched, cond, x_T=None, noise=None, seed=0, call_id=0,
           env_offset=0, deterministic=False, min_sampling_std=0.1, randn_clip=3.0, final_clip=None,
           actions=None, chains=None, want_chains=True):
    E = cond.shape[0]
    dev = cond.device
    _check(cond, (E, d.sd), torch.float32, "cond")
    _check(sched, (d.denoising_steps, _lib.SCHED_COLS), torch.float32, "sched")
    _check(x_T, (E, d.xd), torch.float32, "x_T")
    _check(noise, (d.denoising_steps, E, d.xd), torch.float32, "noise")
    _check(packed_base, (actor_packed_bytes(d, precision),), torch.uint8, "packed_base")
    _check(packed_ft, (actor_packed_bytes(d, precision),), torch.uint8, "packed_ft")
    if actions is None:
        actions = torch.empty(E, d.xd, dtype=torch.float32, device=dev)
    if chains is None and want_chains:
        chains = torch.empty(E, d.ft_denoising_steps + 1, d.xd, dtype=torch.float32, device=dev)
    _check(actions, (E, d.xd), torch.float32, "actions")
    _check(chains, (E, d.ft_denoising_steps + 1, d.xd), torch.float32, "chains")
    _lib.call("dppo_sample", ctypes.byref(d.c()), _prec(precision), ptr(packed_base), ptr(packed_ft), ptr(sched),
              ptr(cond), E, ptr(x_T), ptr(noise), ctypes.c_uint64(seed & (2 ** 64 - 1)), ctypes.c_uint64(call_id),
              int(env_offset), int(bool(deterministic)), float(min_sampling_std), float(randn_clip),
              float(final_clip) if final_clip is not None else 0.0, ptr(actions), ptr(chains), stream_handle(dev))
    return actions, chains


def sampler_layout(d: ModelDims, precision, n_envs):
    """Workgroups per 16-env tile of the sampler dppo_sample runs for n_envs envs: 0 = the
    weight-streaming kernel, P > 0 = the split register-resident kernel (include/dppo.h)."""
    m = ctypes.c_int()
    _lib.call("dppo_sampler_layout", ctypes.byref(d.c()), _prec(precision), int(n_envs), ctypes.byref(m))
    return m.value


def sampler_max_in_flight(d: ModelDims, precision, n_envs):
    """Sampler launches of n_envs envs that may be in flight together (include/dppo.h), divided
    among the ranks that share this GPU (DPPO_SINGLE_DEVICE rehearsals: every rank's launches need
    their co-resident workgroups at once)."""
    m = ctypes.c_int()
    _lib.call("dppo_sampler_max_in_flight", ctypes.byref(d.c()), _prec(precision), int(n_envs), ctypes.byref(m))
    sharing = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))) \
        if os.environ.get("DPPO_SINGLE_DEVICE") else 1
    return max(1, m.value // max(1, sharing))


def sampler_plan(d: ModelDims, precision, n_envs):
    """The sampler the library runs for n_envs envs (dppo_sampler_plan): dict(kernel, members,
    sets, workgroups); kernel: 0 weight streaming, 2 folded split (one 16-env tile per member
    set; kernel ids 1 and 3, the r01 P = 8 and r03 pair kernels, were measured slower and removed)."""
    out = (ctypes.c_int * 4)()
    _lib.call("dppo_sampler_plan", ctypes.byref(d.c()), _prec(precision), int(n_envs), out)
    return dict(kernel=out[0], members=out[1], sets=out[2], workgroups=out[3])


class SampleStepper:
    """dppo_sample_step with every argument but the step index, call counter and mode bound once
    (the rollout's buffers never move), so a rollout step costs one ctypes call."""

    def __init__(self, model, cond_host, obs_traj, actions, actions_host, chains_traj):
        d = model.dims
        S, E = obs_traj.shape[0], obs_traj.shape[1]
        _check(obs_traj, (S, E, d.sd), torch.float32, "obs_traj")
        _check(chains_traj, (S, E, d.ft_denoising_steps + 1, d.xd), torch.float32, "chains_traj")
        _check(actions, (E, d.xd), torch.float32, "actions")
        if cond_host.is_cuda or actions_host.is_cuda or not (cond_host.is_pinned() and actions_host.is_pinned()):
            raise ValueError("cond_host / actions_host must be pinned host tensors")
        if cond_host.numel() != E * d.sd or actions_host.numel() != E * d.xd:
            raise ValueError("cond_host / actions_host sizes do not match the rollout")
        self.model, self.S, self.E = model, S, E
        self._fn = _lib.load().dppo_sample_step
        self._dims = d.c()
        self._keep = (cond_host, obs_traj, actions, actions_host, chains_traj)
        self._obs0, self._obs_step = obs_traj.data_ptr(), E * d.sd * 4
        self._ch0, self._ch_step = chains_traj.data_ptr(), E * (d.ft_denoising_steps + 1) * d.xd * 4
        self._fixed = (ptr(cond_host), ptr(actions), ptr(actions_host))
        # consecutive launches alternate over DPPO_ROLLOUT_STREAMS streams (default 2): launch t+1 is
        # dispatched, and runs its observation-independent prologue (resident weights, noise), while
        # launch t still runs, instead of after it retires. begin() / end() order them against the
        # caller's stream around a rollout. Two launches in flight must both fit on the device (the
        # split sampler's members wait for each other inside a launch): above that size, one stream.
        nst = max(1, int(os.environ.get("DPPO_ROLLOUT_STREAMS", "2")))
        nst = min(nst, sampler_max_in_flight(d, model.precision, E))
        dev = obs_traj.device
        self._tstreams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(nst - 1)]
        self._handles = [ctypes.c_void_p(st.cuda_stream) for st in self._tstreams]
        self._stream = self._handles[0]

    def __call__(self, i, deterministic=False):
        if not 0 <= i < self.S:
            raise IndexError(f"rollout step {i} outside [0, {self.S})")
        m = self.model
        fc = m.final_action_clip_value
        cond_host, actions, actions_host = self._fixed
        rc = self._fn(ctypes.byref(self._dims), _prec(m.precision), ptr(m.packed_base), ptr(m.packed_ft), ptr(m.sched_for(deterministic)),
                      cond_host, ctypes.c_void_p(self._obs0 + i * self._obs_step), self.E,
                      ctypes.c_uint64(m.seed & (2 ** 64 - 1)), ctypes.c_uint64(m._call_id), m._env_offset,
                      int(bool(deterministic)), float(m.get_min_sampling_denoising_std()), float(m.randn_clip_value),
                      float(fc) if fc is not None else 0.0, actions, actions_host,
                      ctypes.c_void_p(self._ch0 + i * self._ch_step), 1, self._stream)
        if rc:
            raise _lib.DppoError(f"dppo_sample_step failed ({rc}): {_lib.load().dppo_last_error().decode()}")
        m._call_id += 1


class RolloutPipe:
    """Pipelined rollout steps (dppo_rollout_enqueue). The observation and action staging buffers
    and two step counters live in coherent mapped pinned memory (dppo_host_alloc); the launch of
    step t+1 is enqueued BEFORE the host steps the envs of step t and waits on the `go` counter, so
    the launch latency overlaps host work and the host learns that step t is done by polling the
    `done` counter instead of a stream synchronisation.
        pipe.enqueue(i, det)   step i's launch (waits until its observation is published)
        pipe.publish()         the observation buffer holds the next step's input
        pipe.wait()            block until the oldest unfinished step has written its actions
    obs / act are torch views over the staging memory ([E, SD] / [E, XD] float32)."""

    def __init__(self, model, obs_traj, actions, chains_traj):
        d = model.dims
        S, E = obs_traj.shape[0], obs_traj.shape[1]
        _check(obs_traj, (S, E, d.sd), torch.float32, "obs_traj")
        _check(chains_traj, (S, E, d.ft_denoising_steps + 1, d.xd), torch.float32, "chains_traj")
        _check(actions, (E, d.xd), torch.float32, "actions")
        lib = _lib.load()
        self._lib, self.model, self.S, self.E = lib, model, S, E
        self._bufs = []

        def alloc(nbytes):
            p = ctypes.c_void_p()
            _lib.call("dppo_host_alloc", ctypes.c_size_t(nbytes), ctypes.byref(p))
            self._bufs.append(p.value)
            return p.value
        po, pa, pc = alloc(4 * E * d.sd), alloc(4 * E * d.xd), alloc(256)
        # the observation protocol: "tagged" (default: the observation is published as tagged
        # granules the launch polls itself, dppo_rollout_enqueue_tagged) or "go" (a go counter, then
        # the launch reads the float buffer); DPPO_ROLLOUT_PROTOCOL=go selects the latter
        self.protocol = os.environ.get("DPPO_ROLLOUT_PROTOCOL", "tagged")
        if self.protocol not in ("tagged", "go"):
            raise ValueError(f"DPPO_ROLLOUT_PROTOCOL must be 'tagged' or 'go', got {self.protocol!r}")
        pt = alloc(8 * E * d.sd)
        self._obs_tag = np.ctypeslib.as_array((ctypes.c_uint64 * (E * d.sd)).from_address(pt))
        pat = alloc(8 * E * d.xd)   # tagged actions (tagged protocol): the host polls the actions themselves
        self._act_tag = np.ctypeslib.as_array((ctypes.c_uint64 * (E * d.xd)).from_address(pat))
        self.obs = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_float * (E * d.sd)).from_address(po))).view(E, d.sd)
        self.obs_mapped = MappedRef(po, 4 * E * d.sd)   # for copy_from_host
        self.act = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_float * (E * d.xd)).from_address(pa))).view(E, d.xd)
        ctr = np.ctypeslib.as_array((ctypes.c_uint32 * 64).from_address(pc))
        self._go, self._done = ctr[0:1], ctr[16:17]          # separate 64-B lines
        self._p = dict(obs=ctypes.c_void_p(po), act=ctypes.c_void_p(pa), go=ctypes.c_void_p(pc),
                       done=ctypes.c_void_p(pc + 64), obs_tag=ctypes.c_void_p(pt), act_tag=ctypes.c_void_p(pat))
        self._fn = lib.dppo_rollout_enqueue_tagged if self.protocol == "tagged" else lib.dppo_rollout_enqueue
        self._dims = d.c()
        self._keep = (obs_traj, actions, chains_traj)
        self._obs0, self._obs_step = obs_traj.data_ptr(), E * d.sd * 4
        self._ch0, self._ch_step = chains_traj.data_ptr(), E * (d.ft_denoising_steps + 1) * d.xd * 4
        self._actions = ptr(actions)
        # consecutive launches alternate over DPPO_ROLLOUT_STREAMS streams (default 2): launch t+1 is
        # dispatched, and runs its observation-independent prologue (resident weights, noise), while
        # launch t still runs, instead of after it retires. begin() / end() order them against the
        # caller's stream around a rollout. Two launches in flight must both fit on the device (the
        # split sampler's members wait for each other inside a launch): above that size, one stream.
        nst = max(1, int(os.environ.get("DPPO_ROLLOUT_STREAMS", "2")))
        nst = min(nst, sampler_max_in_flight(d, model.precision, E))
        dev = obs_traj.device
        self._tstreams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(nst - 1)]
        self._handles = [ctypes.c_void_p(st.cuda_stream) for st in self._tstreams]
        self._stream = self._handles[0]
        self.nwg = (E + 15) // 16
        self.enqueued = 0      # steps launched so far (step s waits for go >= s + 1)
        self.published = 0
        self.finished = 0

    def enqueue(self, i, deterministic=False):
        if not 0 <= i < self.S:
            raise IndexError(f"rollout step {i} outside [0, {self.S})")
        m = self.model
        fc = m.final_action_clip_value
        p = self._p
        self._stream = self._handles[self.enqueued % len(self._handles)]
        self.enqueued += 1
        common = (ctypes.byref(self._dims), _prec(m.precision), ptr(m.packed_base), ptr(m.packed_ft),
                  ptr(m.sched_for(deterministic)))
        tail = (self.E, ctypes.c_uint64(m.seed & (2 ** 64 - 1)), ctypes.c_uint64(m._call_id), m._env_offset,
                int(bool(deterministic)), float(m.get_min_sampling_denoising_std()), float(m.randn_clip_value),
                float(fc) if fc is not None else 0.0, self._actions, p["act"],
                ctypes.c_void_p(self._ch0 + i * self._ch_step))
        obs_dev = ctypes.c_void_p(self._obs0 + i * self._obs_step)
        if self.protocol == "tagged":   # step s waits for granules tagged s + 1 (= its publish count)
            tail_t = tail[:-2] + (p["act_tag"],) + tail[-1:]          # tagged actions replace actions_host
            rc = self._fn(*common, p["obs_tag"], obs_dev, *tail_t, ctypes.c_uint32(self.enqueued), p["done"],
                          self._stream)
        else:
            rc = self._fn(*common, p["obs"], obs_dev, *tail, p["go"], ctypes.c_uint32(self.enqueued), p["done"],
                          self._stream)
        if rc:
            raise _lib.DppoError(f"dppo_rollout_enqueue failed ({rc}): {self._lib.dppo_last_error().decode()}")
        m._call_id += 1

    def launch_event(self, ev=None):
        """An event recorded on the stream of the most recent launch (its completion); ev: an
        event to re-record (a caller's ring: creating and destroying one per step cost ~3 us of
        host time each, ~1.5 ms per 500-step rollout when the list was freed)."""
        if ev is None:
            ev = torch.cuda.Event()
        ev.record(self._tstreams[(self.enqueued - 1) % len(self._tstreams)])
        return ev

    def begin(self):
        """Before a rollout: split-sampler tables an optimizer step deferred are re-derived on the
        caller's stream, then the launch streams wait for it (updated weights and tables). A launch
        reads its resident tables in its prologue, before its observation wait, so the refresh must
        precede every stream, not only the first launch's."""
        with torch.cuda.stream(self._tstreams[0]):
            refresh_sampler_tables(self.model.packed_ft)
            refresh_sampler_tables(self.model.packed_base)
        for st in self._tstreams[1:]:
            st.wait_stream(self._tstreams[0])

    def end(self):
        """After a rollout: the caller's stream waits for every launch stream."""
        for st in self._tstreams[1:]:
            self._tstreams[0].wait_stream(st)

    def publish(self):
        self.published += 1
        if self.protocol == "tagged":         # one aligned 8-byte store per value: never torn
            bits = self.obs.numpy().reshape(-1).view(np.uint32).astype(np.uint64)
            self._obs_tag[:] = (np.uint64(self.published) << np.uint64(32)) | bits
        else:
            self._go[0] = self.published      # x86 stores are ordered: the observation is visible first

    def gate(self, publish, timeout_s=30.0):
        """Arguments of a gated env step (env.step(..., gate=...)): the native stepper waits for
        this step's done count itself and, if publish, releases the next launch. Call
        published() after a step that did publish, publish() after one that did not."""
        self.finished += 1
        if self.protocol == "tagged":   # the finished launch's actions carry its tag (= finished)
            pub = (self._p["obs_tag"], self.published + 1) if publish else (None, 0)
            return ("tagged", self._p["done"], self._p["act_tag"], ctypes.c_uint32(self.finished), pub[0],
                    ctypes.c_uint32(pub[1]), ctypes.c_double(timeout_s))
        pub = (self._p["go"], self.published + 1) if publish else (None, 0)
        return ("go", self._p["done"], ctypes.c_uint32(self.finished * self.nwg), pub[0],
                ctypes.c_uint32(pub[1]), ctypes.c_double(timeout_s))

    def published_by_gate(self):
        self.published += 1

    def wait(self, timeout_s=30.0):
        import time
        self.finished += 1
        target = self.finished * self.nwg
        done = self._done
        tagged = self.protocol == "tagged"
        t0 = None
        while True:
            v = int(done[0])
            if v & 0x80000000:
                raise _lib.DppoError("rollout step timed out waiting for its observation")
            if tagged:   # the launch stores its actions as {tag, bits} granules (no host float copy)
                x = self._act_tag.copy()
                if ((x >> np.uint64(32)) == np.uint64(self.finished)).all():
                    self.act.numpy().reshape(-1).view(np.uint32)[:] = (x & np.uint64(0xFFFFFFFF)).astype(np.uint32)
                    return
            elif v >= target:
                return
            if t0 is None:
                t0 = time.perf_counter()
            elif time.perf_counter() - t0 > timeout_s:
                raise _lib.DppoError(f"rollout step {self.finished - 1} did not finish within {timeout_s} s")

    def close(self):
        for st in self._tstreams:
            st.synchronize()
        for h in self._handles:     # the split sampler's exchange buffers of these streams go back to the pool
            _lib.call("dppo_sampler_release_stream", h)
        for b in self._bufs:
            self._lib.dppo_host_free(ctypes.c_void_p(b))
        self._bufs = []

    def __del__(self):
        try:
            if self._bufs:
                self.close()
        except Exception:
            pass


def logprob(d: ModelDims, precision, packed_ft, sched, cond, chains, min_logprob_std=0.1, reward_horizon=None,
            want_elem=True, want_mean=True, lp_elem=None, lp_mean=None):
    n = cond.shape[0]
    dev = cond.device
    kf = d.ft_denoising_steps
    _check(cond, (n, d.sd), torch.float32, "cond")
    _check(chains, (n, kf + 1, d.xd), torch.float32, "chains")
    _check(sched, (d.denoising_steps, _lib.SCHED_COLS), torch.float32, "sched")
    _check(packed_ft, (actor_packed_bytes(d, precision),), torch.uint8, "packed_ft")
    if want_elem and lp_elem is None:
        lp_elem = torch.empty(n * kf, d.xd, dtype=torch.float32, device=dev)
    if want_mean and lp_mean is None:
        lp_mean = torch.empty(n, kf, dtype=torch.float32, device=dev)
    _check(lp_elem, (n * kf, d.xd), torch.float32, "lp_elem")
    _check(lp_mean, (n, kf), torch.float32, "lp_mean")
    rh = d.horizon_steps if reward_horizon is None else int(reward_horizon)
    _lib.call("dppo_logprob", ctypes.byref(d.c()), _prec(precision), ptr(packed_ft), ptr(sched), ptr(cond),
              ptr(chains), n, float(min_logprob_std), rh, ptr(lp_elem), ptr(lp_mean), stream_handle(dev))
    return lp_elem, lp_mean


def critic_forward(d: ModelDims, precision, packed_critic, cond, values=None):
    n = cond.shape[0]
    _check(cond, (n, d.sd), torch.float32, "cond")
    _check(packed_critic, (critic_packed_bytes(d, precision),), torch.uint8, "packed_critic")
    if values is None:
        values = torch.empty(n, dtype=torch.float32, device=cond.device)
    _check(values, (n,), torch.float32, "values")
    _lib.call("dppo_critic_forward", ctypes.byref(d.c()), _prec(precision), ptr(packed_critic), ptr(cond), n,
              ptr(values), stream_handle(cond.device))
    return values


# ------------------------------------------------------------------------------------------------
# scans
# ------------------------------------------------------------------------------------------------
def gae(reward, values, last_values, terminated, gamma=0.99, lam=0.95, reward_scale_const=1.0, adv=None, ret=None):
    S, E = reward.shape
    _check(reward, (S, E), torch.float64, "reward")
    _check(values, (S, E), torch.float32, "values")
    _check(last_values, (E,), torch.float32, "last_values")
    _check(terminated, (S, E), torch.uint8, "terminated")
    if adv is None:
        adv = torch.empty(S, E, dtype=torch.float32, device=reward.device)
    if ret is None:
        ret = torch.empty(S, E, dtype=torch.float32, device=reward.device)
    _lib.call("dppo_gae", ptr(reward), ptr(values), ptr(last_values), ptr(terminated), S, E, float(gamma), float(lam),
              float(reward_scale_const), ptr(adv), ptr(ret), stream_handle(reward.device))
    return adv, ret


def reward_scale_workspace(S, E, device):
    n = int(_lib.query("dppo_reward_scale_workspace_doubles", S, E))
    return torch.empty(n, dtype=torch.float64, device=device)


def reward_scale(reward, first, ret_state, rms_state, workspace=None, gamma=0.99, cliprew=10.0, epsilon=1e-8):
    """In place: reward [S,E] fp64 is replaced by the scaled reward (RunningRewardScaler.__call__)."""
    S, E = reward.shape
    _check(reward, (S, E), torch.float64, "reward")
    _check(first, (S, E), torch.uint8, "first")
    _check(ret_state, (E,), torch.float64, "ret_state")
    _check(rms_state, (3,), torch.float64, "rms_state")
    if workspace is None:
        workspace = reward_scale_workspace(S, E, reward.device)
    _lib.call("dppo_reward_scale", ptr(reward), ptr(first), ptr(ret_state), ptr(rms_state), ptr(workspace), S, E,
              float(gamma), float(cliprew), float(epsilon), stream_handle(reward.device))
    return reward


def reward_scale_moments(reward, first, ret_state, moments, workspace, gamma=0.99):
    S, E = reward.shape
    _lib.call("dppo_reward_scale_moments", ptr(reward), ptr(first), ptr(ret_state), ptr(workspace), ptr(moments), S, E,
              float(gamma), stream_handle(reward.device))
    return moments


def reward_scale_apply(reward, rms_state, cliprew=10.0, epsilon=1e-8):
    S, E = reward.shape
    _lib.call("dppo_reward_scale_apply", ptr(reward), ptr(rms_state), S, E, float(cliprew), float(epsilon),
              stream_handle(reward.device))
    return reward


def _bcast_len(S, L):
    if S == L or S == 1:
        return L
    if L == 1:
        return S
    raise ValueError(f"operands could not be broadcast together with shapes ({S},) ({L},)")


def reward_scale_per_env(reward, first, ret_state, rms_in, L_in, rms_out, workspace, out, gamma=0.99, cliprew=10.0,
                         epsilon=1e-8):
    """RunningRewardScaler(per_env=True).__call__ (reference util/reward_scaling.py:51-66), time-major:
    reward / first [S,E], rms_in / rms_out fp64 [1 + 2 L] = {count, mean[L], var[L]} (distinct buffers),
    out [C, E] (C = S, or the new state length when S == 1). Returns the new state length."""
    S, E = reward.shape
    _check(reward, (S, E), torch.float64, "reward")
    _check(first, (S, E), torch.uint8, "first")
    _check(ret_state, (E,), torch.float64, "ret_state")
    Lo = _bcast_len(S, L_in)
    C = S if (S > 1 or Lo == 1) else Lo
    _check(out, (C, E), torch.float64, "out")
    if rms_in.numel() < 1 + 2 * L_in or rms_out.numel() < 1 + 2 * Lo:
        raise ValueError("rms state buffers too small")
    _lib.call("dppo_reward_scale_per_env", ptr(reward), ptr(first), ptr(ret_state), ptr(rms_in), int(L_in), ptr(rms_out),
              ptr(workspace), S, E, float(gamma), float(cliprew), float(epsilon), ptr(out), stream_handle(reward.device))
    return Lo


def reward_scale_per_env_moments(reward, first, ret_state, workspace, col_moments, gamma=0.99):
    S, E = reward.shape
    _check(col_moments, (S, 2), torch.float64, "col_moments")
    _lib.call("dppo_reward_scale_per_env_moments", ptr(reward), ptr(first), ptr(ret_state), ptr(workspace),
              ptr(col_moments), S, E, float(gamma), stream_handle(reward.device))
    return col_moments


def reward_scale_per_env_apply(reward, rms_state, L, out, cliprew=10.0, epsilon=1e-8):
    S, E = reward.shape
    _lib.call("dppo_reward_scale_per_env_apply", ptr(reward), ptr(rms_state), S, E, int(L), float(cliprew),
              float(epsilon), ptr(out), stream_handle(reward.device))
    return out


# ------------------------------------------------------------------------------------------------
# update
# ------------------------------------------------------------------------------------------------
def feistel_permute(first, count, n, seed, epoch, device):
    out = torch.empty(count, dtype=torch.int64, device=device)
    _lib.call("dppo_feistel_permute", int(first), int(count), int(n), ctypes.c_uint64(seed), int(epoch), ptr(out),
              stream_handle(device))
    return out


def ppo_workspace(d: ModelDims, precision, rows, device):
    nbytes = int(_lib.query("dppo_ppo_workspace_bytes", ctypes.byref(d.c()), _prec(precision), int(rows)))
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def ppo_adv_stats(advantages, total, kf, perm_seed, epoch, start, rows, out, row_index=None):
    _lib.call("dppo_ppo_adv_stats", ptr(advantages), int(total), int(kf), ctypes.c_uint64(perm_seed), int(epoch),
              int(start), int(rows), ptr(row_index), ptr(out), stream_handle(advantages.device))
    return out


def ppo_adv_stats_all(advantages, total, kf, perm_seed, epoch0, n_epochs, rows_full, n_batch, out):
    """out fp64 [n_epochs * n_batch, 3]: every minibatch's advantage moments in one launch."""
    _check(out, (n_epochs * n_batch, 3), torch.float64, "out")
    _lib.call("dppo_ppo_adv_stats_all", ptr(advantages), int(total), int(kf), ctypes.c_uint64(perm_seed), int(epoch0),
              int(n_epochs), int(rows_full), int(n_batch), ptr(out), stream_handle(advantages.device))
    return out


def ppo_hparams(gamma_denoising=0.99, clip_ploss_coef=0.01, clip_ploss_coef_base=0.01, clip_ploss_coef_rate=3.0,
                min_logprob_std=0.1, vf_coef=0.5, norm_adv=True, reward_horizon=4, loss_scale=1.0, global_rows=1,
                l2_deferred=False, learn_eta=False, clip_vloss_coef=None, old_values=None):
    """l2_deferred (ABI 8, DPPO_PPO_L2_DEFERRED): the actor's l2 gradient is left factored in grads
    for an optimizer step with l2_from_pl2 (or materialize_l2). learn_eta (ABI 9,
    DPPO_PPO_LEARN_ETA): the row tiles add d loss / d eta of a DDIM schedule into metrics[8].
    clip_vloss_coef (ABI 14, diffusion_ppo.py:110-116): the clipped value loss against old_values, the
    rollout's value pass (device fp32 [S*E], indexed by sample; the caller keeps it alive)."""
    flags = (_lib.DPPO_PPO_L2_DEFERRED if l2_deferred else 0) | (_lib.DPPO_PPO_LEARN_ETA if learn_eta else 0)
    clip = clip_vloss_coef is not None
    if clip and (old_values is None or old_values.dtype != torch.float32 or not old_values.is_cuda):
        raise ValueError("clip_vloss_coef needs the rollout's old values (fp32 device tensor)")
    if clip and not float(clip_vloss_coef) > 0:
        raise ValueError("clip_vloss_coef must be > 0")
    return _lib.DppoPpoHparams(float(gamma_denoising), float(clip_ploss_coef), float(clip_ploss_coef_base),
                               float(clip_ploss_coef_rate), float(min_logprob_std), float(vf_coef), int(bool(norm_adv)),
                               int(reward_horizon), float(loss_scale), int(global_rows), flags,
                               float(clip_vloss_coef) if clip else 0.0, old_values.data_ptr() if clip else None)


def ddim_eta_base(schedule):
    """fp32 [S][5] eta-independent rows of a DDIM schedule (ddim_buffers) for dppo_eta_step:
    {abar_prev, sqrt(abar_prev), sqrt(abar), sqrt(1 - abar), s = sigma / eta}."""
    return np.stack([schedule["ddim_alphas_prev"], schedule["ddim_sqrt_alphas_prev"], schedule["ddim_sqrt_alphas"],
                     schedule["ddim_sqrt_1m_alphas"], schedule["ddim_sfac"]], axis=1).astype(np.float32)


def eta_step(eta_state, metrics, step, lr, weight_decay, eta_min, eta_max, ddim_base, sched, eta_out=None,
             beta1=0.9, beta2=0.999, eps=1e-7, mode=0):
    """dppo_eta_step on the current stream: AdamW on the eta logit from metrics[8] (metrics=None:
    only re-derive the schedule's eta columns), then the DDIM rows of sched for the new eta."""
    _check(eta_state, (3,), torch.float32, "eta_state")
    _check(sched, (sched.shape[0], _lib.SCHED_COLS), torch.float32, "sched")
    _check(ddim_base, (sched.shape[0], 5), torch.float32, "ddim_base")
    if metrics is not None:
        _check(metrics, (16,), torch.float64, "metrics")
    _lib.call("dppo_eta_step", ptr(eta_state), ptr(metrics), int(step), float(lr), float(weight_decay), float(beta1),
              float(beta2), float(eps), int(mode), float(eta_min), float(eta_max), ptr(ddim_base), ptr(sched),
              int(sched.shape[0]), ptr(eta_out), stream_handle(eta_state.device))


def materialize_l2(d: ModelDims, precision, packed_actor, grads, workspace, batch_rows):
    """The actor's l2 gradient of an l2_deferred minibatch formed in place (dppo_materialize_l2)."""
    _lib.call("dppo_materialize_l2", ctypes.byref(_dims_c(d)), _prec(precision), ptr(packed_actor), ptr(grads),
              ptr(workspace), int(batch_rows), stream_handle(grads.device))


def ppo_minibatch(d: ModelDims, precision, hp, packed_ft, packed_critic, actor_params, sched, obs, chains, lp_old_mean,
                  advantages, returns, perm_seed, epoch, start, rows, workspace, grads, metrics, adv_stats=None,
                  row_index=None, part=None):
    n = obs.shape[0]
    kf = d.ft_denoising_steps
    _check(obs, (n, d.sd), torch.float32, "obs")
    _check(chains, (n, kf + 1, d.xd), torch.float32, "chains")
    _check(lp_old_mean, (n, kf), torch.float32, "lp_old_mean")
    _check(advantages, (n,), torch.float32, "advantages")
    _check(returns, (n,), torch.float32, "returns")
    na, nc = _n_params(d)
    _check(actor_params, (na,), torch.float32, "actor_params")
    _check(grads, (na + nc,), torch.float32, "grads")
    _check(metrics, (16,), torch.float64, "metrics")
    if row_index is not None:
        _check(row_index, (row_index.numel(),), torch.int64, "row_index")
        if row_index.numel() < start + rows:
            raise ValueError("row_index shorter than start + rows")
    need = _workspace_bytes(d, _prec(precision), int(rows))
    if workspace.numel() < need:
        raise ValueError(f"workspace too small: {workspace.numel()} < {need}")
    args = (ctypes.byref(_dims_c(d)), _prec(precision), ctypes.byref(hp), ptr(packed_ft), ptr(packed_critic),
            ptr(actor_params), ptr(sched), ptr(obs), ptr(chains), ptr(lp_old_mean), ptr(advantages), ptr(returns),
            int(n * kf), ctypes.c_uint64(perm_seed), int(epoch), int(start), int(rows), ptr(row_index), ptr(adv_stats),
            ptr(workspace), ptr(grads), ptr(metrics))
    if part is None:
        _lib.call("dppo_ppo_minibatch", *args, stream_handle(obs.device))
    else:   # 1 = actor half, 2 = critic half, on the current stream (dppo_ppo_minibatch_part)
        _lib.call("dppo_ppo_minibatch_part", *args, int(part), stream_handle(obs.device))


class BoundMinibatch:
    """ppo_minibatch with the arguments that stay fixed over an update phase (rollout buffers,
    weights and images, workspace, gradients) validated and marshalled once; a call passes what
    changes per minibatch. The host's enqueue time per minibatch matters where minibatches are
    small (an 8-GPU rank's 6,250 rows: ~0.13 ms of GPU time each)."""

    def __init__(self, d: ModelDims, precision, packed_ft, packed_critic, actor_params, sched, obs, chains,
                 lp_old_mean, advantages, returns, perm_seed, workspace, grads, max_rows):
        n = obs.shape[0]
        kf = d.ft_denoising_steps
        _check(obs, (n, d.sd), torch.float32, "obs")
        _check(chains, (n, kf + 1, d.xd), torch.float32, "chains")
        _check(lp_old_mean, (n, kf), torch.float32, "lp_old_mean")
        _check(advantages, (n,), torch.float32, "advantages")
        _check(returns, (n,), torch.float32, "returns")
        na, nc = _n_params(d)
        _check(actor_params, (na,), torch.float32, "actor_params")
        _check(grads, (na + nc,), torch.float32, "grads")
        need = _workspace_bytes(d, _prec(precision), int(max_rows))
        if workspace.numel() < need:
            raise ValueError(f"workspace too small: {workspace.numel()} < {need}")
        self.max_rows = int(max_rows)
        self._lib = _lib.load()
        self._dims = _dims_c(d)
        self._prec = _prec(precision)
        self._mid = (ptr(packed_ft), ptr(packed_critic), ptr(actor_params), ptr(sched), ptr(obs), ptr(chains),
                     ptr(lp_old_mean), ptr(advantages), ptr(returns), int(n * kf), ctypes.c_uint64(int(perm_seed)))
        self._tail = (ptr(workspace), ptr(grads))
        self._dev = obs.device
        self._keep = (packed_ft, packed_critic, actor_params, sched, obs, chains, lp_old_mean, advantages, returns,
                      workspace, grads)   # the pointers above stay valid while this object lives

    def __call__(self, hp, epoch, start, rows, metrics, adv_stats=None, part=None, stream=None):
        """metrics / adv_stats: device tensors, or device addresses (ints) of fp64[16] / fp64[3]
        (the update loop passes precomputed addresses); stream: a raw stream handle (default: the
        current stream)."""
        if not 0 < rows <= self.max_rows:
            raise ValueError(f"rows {rows} outside (0, {self.max_rows}]")
        if isinstance(metrics, torch.Tensor):
            if metrics.dtype != torch.float64 or metrics.numel() < 16:
                raise ValueError("metrics: expected fp64[16]")
            metrics = metrics.data_ptr()
        if isinstance(adv_stats, torch.Tensor):
            adv_stats = adv_stats.data_ptr()
        args = (ctypes.byref(self._dims), self._prec, ctypes.byref(hp)) + self._mid + (
            int(epoch), int(start), int(rows), None, adv_stats) + self._tail + (metrics,)
        st = stream_handle(self._dev) if stream is None else stream
        if part is None:
            rc = self._lib.dppo_ppo_minibatch(*args, st)
        else:
            rc = self._lib.dppo_ppo_minibatch_part(*args, int(part), st)
        if rc != 0:
            raise _lib.DppoError(f"dppo_ppo_minibatch failed ({rc}): {self._lib.dppo_last_error().decode()}")


class BoundOptimizerStep:
    """optimizer_step over a fixed range and fixed images, validated and marshalled once; a call
    passes the step, learning rate, metric source and tag (see BoundMinibatch)."""

    def __init__(self, d: ModelDims, precision, params, grads, m, v, weight_decay, beta1, beta2, eps, mode,
                 actor_params=None, packed_actor=None, critic_params=None, packed_critic=None,
                 defer_sampler_tables=False, l2_from_pl2=False, fused_pack=False, clear_grads=False):
        """fused_pack (ABI 11, DPPO_STEP_FUSED_PACK): AdamW and the image in one launch where the
        library can (one network whose parameters are the range); clear_grads (DPPO_STEP_CLEAR_GRADS):
        the step zeroes the range's gradients and the `clear` ranges of each call after reading them."""
        n = params.numel()
        for t, nm in ((grads, "grads"), (m, "m"), (v, "v")):
            if t.numel() != n:
                raise ValueError(f"{nm}: expected {n} elements")
        self._lib = _lib.load()
        self._dims = _dims_c(d)
        mode_i = ((_lib.DPPO_ADAMW_KERAS if mode == "keras" else _lib.DPPO_ADAMW_TORCH) |
                  (_lib.DPPO_STEP_DEFER_SAMPLER_TABLES if defer_sampler_tables else 0) |
                  (_lib.DPPO_STEP_L2_FROM_PL2 if l2_from_pl2 else 0) |
                  (_lib.DPPO_STEP_FUSED_PACK if fused_pack else 0) |
                  (_lib.DPPO_STEP_CLEAR_GRADS if clear_grads else 0))
        self._head = (ctypes.byref(self._dims), _prec(precision), ptr(params), ptr(grads), ptr(m), ptr(v), int(n))
        self._hp = (float(weight_decay), float(beta1), float(beta2), float(eps), mode_i, ptr(actor_params),
                    ptr(packed_actor), ptr(critic_params), ptr(packed_critic))
        self._dev = params.device
        self._keep = (params, grads, m, v, actor_params, packed_actor, critic_params, packed_critic)

    def __call__(self, step, lr, metrics=None, metrics_out=None, n_metrics=0, metrics_tag=0, stream=None, clear=None):
        """metrics_out: a device tensor or a dppo_host_alloc address (as optimizer_step); metrics: a
        device tensor or address; stream: a raw stream handle (default: the current stream); clear: a
        ClearRanges (byte ranges zeroed after the step's last read, dppo_optimizer_step_ex)."""
        mo = metrics_out if isinstance(metrics_out, int) else (metrics_out.data_ptr() if metrics_out is not None else None)
        mi = metrics if isinstance(metrics, int) else ptr(metrics)
        cp, cb, cn = (None, None, 0) if clear is None else clear.args
        rc = self._lib.dppo_optimizer_step_ex(*self._head, int(step), float(lr), *self._hp, mi,
                                              ctypes.c_void_p(mo) if mo else None, int(n_metrics),
                                              ctypes.c_uint64(int(metrics_tag)), cp, cb, cn,
                                              stream_handle(self._dev) if stream is None else stream)
        if rc != 0:
            raise _lib.DppoError(f"dppo_optimizer_step failed ({rc}): {self._lib.dppo_last_error().decode()}")


class ClearRanges:
    """The non-gradient byte ranges a minibatch part zeroes first (dppo_ppo_clear_ranges: metric slots
    of `metrics`, the workspace's accumulators for `rows`), marshalled for dppo_optimizer_step_ex, so
    the optimizer step before that minibatch clears them and the minibatch runs with
    DPPO_PPO_PRECLEARED. metrics: a device address or fp64[16] tensor; workspace: the uint8 tensor."""

    def __init__(self, d: ModelDims, precision, rows, workspace, metrics, part):
        lib = _lib.load()
        self._ptrs = (ctypes.c_void_p * 4)()
        self._bytes = (ctypes.c_size_t * 4)()
        cnt = ctypes.c_int(0)
        mptr = metrics if isinstance(metrics, int) else metrics.data_ptr()
        rc = lib.dppo_ppo_clear_ranges(ctypes.byref(_dims_c(d)), _prec(precision), int(rows), ptr(workspace),
                                       ctypes.c_void_p(mptr), int(part), self._ptrs, self._bytes, ctypes.byref(cnt))
        if rc != 0:
            raise _lib.DppoError(f"dppo_ppo_clear_ranges failed ({rc}): {lib.dppo_last_error().decode()}")
        self.count = cnt.value
        self.args = (self._ptrs, self._bytes, self.count)
        self._keep = (workspace, metrics)

    def ranges(self):
        return [(int(self._ptrs[i]), int(self._bytes[i])) for i in range(self.count)]


def q_sched_table(schedule):
    """[K][2] fp32 {sqrt(alphas_cumprod), sqrt(1 - alphas_cumprod)}: the q_sample buffers of
    diffusion.py:62-65 (computed in fp32 like the TF buffers)."""
    ac = np.asarray(schedule["alphas_cumprod"], np.float32)
    return np.stack([np.sqrt(ac), np.sqrt(np.float32(1.0) - ac)], axis=1).astype(np.float32)


def pretrain_minibatch(d: ModelDims, precision, packed_actor, actor_params, sched, qsched, x_start, cond, t, noise,
                       workspace, grads, metrics, global_rows=None, loss_scale=1.0):
    """p_losses (diffusion.py:186-194) and its actor gradient for one batch; see include/dppo.h.
    Returns the loss as a device scalar (metrics[0] / (global_rows * xd) * loss_scale)."""
    n = x_start.shape[0]
    g = n if global_rows is None else int(global_rows)
    _check(x_start, (n, d.xd), torch.float32, "x_start")
    _check(cond, (n, d.sd), torch.float32, "cond")
    _check(t, (n,), torch.int32, "t")
    _check(noise, (n, d.xd), torch.float32, "noise")
    _check(qsched, (d.denoising_steps, 2), torch.float32, "qsched")
    na = spec_count(actor_param_spec(d))
    _check(actor_params, (na,), torch.float32, "actor_params")
    if grads.numel() < na:
        raise ValueError("grads: needs at least the actor parameter count")
    _check(metrics, (16,), torch.float64, "metrics")
    need = int(_lib.query("dppo_ppo_workspace_bytes", ctypes.byref(d.c()), _prec(precision), int(n)))
    if workspace.numel() < need:
        raise ValueError(f"workspace too small: {workspace.numel()} < {need}")
    _lib.call("dppo_pretrain_minibatch", ctypes.byref(d.c()), _prec(precision), ptr(packed_actor), ptr(actor_params),
              ptr(sched), ptr(qsched), ptr(x_start), ptr(cond), ptr(t), ptr(noise), int(n), int(g), float(loss_scale),
              ptr(workspace), ptr(grads), ptr(metrics), stream_handle(x_start.device))
    return metrics[0] * (float(loss_scale) / (g * d.xd))


def adamw(params, grads, m, v, step, lr, weight_decay=0.004, beta1=0.9, beta2=0.999, eps=1e-7, mode="keras"):
    n = params.numel()
    for t, nm in ((grads, "grads"), (m, "m"), (v, "v")):
        _check(t, (n,), torch.float32, nm)
    _lib.call("dppo_adamw", ptr(params), ptr(grads), ptr(m), ptr(v), int(n), int(step), float(lr), float(weight_decay),
              float(beta1), float(beta2), float(eps),
              _lib.DPPO_ADAMW_KERAS if mode == "keras" else _lib.DPPO_ADAMW_TORCH, stream_handle(params.device))


def sched_table(schedule):
    """[rows][8] fp32 table (include/dppo.h) from the fp32 DDPM buffers, or from the DDIM
    sub-sequence coefficients (model/diffusion/sampling.py: ddpm_buffers / ddim_buffers)."""
    if "ddim_c0" in schedule:
        tab = np.zeros((len(schedule["ddim_c0"]), _lib.SCHED_COLS), np.float32)
        for j, k in enumerate(("ddim_c0", "ddim_c1", "ddim_c2", "ddim_c3", "ddim_logvar")):
            tab[:, j] = schedule[k]
        tab[:, 5] = 0.0                      # eval: no noise on any DDIM row (diffusion_vpg.py:303-306)
        tab[:, 6] = 1.0
        tab[:, 7] = schedule["ddim_sfac"]    # sigma / eta: the learnable-eta gradient's row factor
        return tab
    K = len(schedule["betas"])
    tab = np.zeros((K, _lib.SCHED_COLS), np.float32)
    tab[:, 0] = schedule["sqrt_recip_alphas_cumprod"]
    tab[:, 1] = schedule["sqrt_recipm1_alphas_cumprod"]
    tab[:, 2] = schedule["ddpm_mu_coef1"]
    tab[:, 3] = schedule["ddpm_mu_coef2"]
    tab[:, 4] = schedule["ddpm_logvar_clipped"]
    tab[:, 5] = 1e-3                         # eval: t > 0 clips at 1e-3, t = 0 has no noise (:308-312)
    tab[0, 6] = 1.0
    return tab


def adam_alpha(lr, beta1, beta2, step):
    return lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
