"""RunningRewardScaler (reference util/reward_scaling.py:42-87) on the device.

The scan (discounted running return), the moment reduction and the rescale run in one fp64 HIP
pass set (dppo_reward_scale*). The reference API — __call__(reward [E,S], first [E,S]) on NumPy
arrays — is kept; the agent uses the time-major device form scale_() without host round trips.
Multi-GPU: the per-rank moments are merged with an all-reduce before the update (Chan's rule), so
every rank applies the same global statistics.

per_env=True (reward_scaling.py:51-66) is kept as the reference writes it: the RunningMeanStd has
shape (num_envs,) but `ret_rms.update(rets)` reduces rets [E, S] over axis 0 — the envs — so each
TIME COLUMN gives one (mean, var) pair with batch count E, joined to the state by NumPy broadcasting
(S must equal the state's length, or one of them be 1: anything else raises NumPy's
"operands could not be broadcast together", here a ValueError), and transform() divides reward
[E, S] column-wise. dppo_reward_scale_per_env runs it on the device."""
import numpy as np
import torch

from .. import ops
from . import dist as dist_util


class RunningRewardScaler:
    def __init__(self, num_envs, cliprew=10.0, gamma=0.99, epsilon=1e-8, per_env=False, device=None):
        self.num_envs, self.cliprew, self.gamma, self.epsilon = num_envs, cliprew, gamma, epsilon
        self.per_env = bool(per_env)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ret = torch.zeros(num_envs, dtype=torch.float64, device=self.device)
        if self.per_env:
            # {count, mean[L], var[L]} (RunningMeanStd(shape=(num_envs,)): mean 0, var 1, count 1e-4)
            self._L = num_envs
            self._pe = [self._pe_state(num_envs, num_envs), None]
            self.rms = None
        else:
            self.rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=self.device)  # mean, var, count
        self._ws = None

    def _pe_state(self, L, cap):
        t = torch.zeros(1 + 2 * cap, dtype=torch.float64, device=self.device)
        t[0] = 1e-4
        t[1 + L:1 + 2 * L] = 1.0
        return t

    def _workspace(self, S, E):
        if self._ws is None or self._ws[0] != (S, E):
            self._ws = ((S, E), ops.reward_scale_workspace(S, E, self.device))
        return self._ws[1]

    # ---------------------------------------------------------------- per_env = True
    def _per_env_scale(self, reward_se, first_se, group, out=None):
        S, E = reward_se.shape
        ws = self._workspace(S, E)
        Lo = ops._bcast_len(S, self._L)
        C = S if (S > 1 or Lo == 1) else Lo
        if out is None:
            out = reward_se if C == S else torch.empty(C, E, dtype=torch.float64, device=self.device)
        rin = self._pe[0]
        if self._pe[1] is None or self._pe[1].numel() < 1 + 2 * Lo:
            self._pe[1] = torch.zeros(1 + 2 * max(Lo, self._L), dtype=torch.float64, device=self.device)
        rout = self._pe[1]
        if group is None or not torch.distributed.is_initialized() or torch.distributed.get_world_size(group) == 1:
            self._L = ops.reward_scale_per_env(reward_se, first_se, self.ret, rin, self._L, rout, ws, out, self.gamma,
                                               self.cliprew, self.epsilon)
        else:
            # per time column (n = this rank's envs, mean, M2) merged over ranks in rank order (Chan),
            # then the reference's update_from_moments with NumPy broadcasting, on the host
            colm = torch.zeros(S, 2, dtype=torch.float64, device=self.device)
            ops.reward_scale_per_env_moments(reward_se, first_se, self.ret, ws, colm, self.gamma)
            loc = torch.stack([torch.full((S,), float(E), dtype=torch.float64, device=self.device),
                               colm[:, 0], colm[:, 1] * E], 1)
            W = torch.distributed.get_world_size(group)
            src = loc.cpu() if dist_util._host_staged(loc, group) else loc
            parts = [torch.zeros_like(src) for _ in range(W)]
            torch.distributed.all_gather(parts, src, group=group)
            parts = [p.cpu().numpy() for p in parts]
            n = np.zeros(S)
            bm = np.zeros(S)
            bv = np.zeros(S)
            for t in range(S):
                nt, mt, m2 = dist_util.chan_merge([tuple(p[t]) for p in parts])
                n[t], bm[t], bv[t] = nt, mt, m2 / nt
            st = rin.cpu().numpy()
            L = self._L
            count, mean, var = st[0], st[1:1 + L], st[1 + L:1 + 2 * L]
            bc = n[0]
            delta = bm - mean                                       # broadcasting as reward_scaling.py:30-39
            tot = count + bc
            new_mean = mean + delta * bc / tot
            M2 = var * count + bv * bc + delta ** 2 * count * bc / tot
            new_var = M2 / (tot - 1)
            Lo = new_mean.shape[0]
            rout[0] = tot
            rout[1:1 + Lo] = torch.from_numpy(np.ascontiguousarray(new_mean))
            rout[1 + Lo:1 + 2 * Lo] = torch.from_numpy(np.ascontiguousarray(new_var))
            ops.reward_scale_per_env_apply(reward_se, rout, Lo, out, self.cliprew, self.epsilon)
            self._L = Lo
        self._pe = [rout, rin]
        return out

    def scale_(self, reward_se, first_se, group=None):
        """In place on time-major device tensors reward [S,E] fp64, first [S,E] u8."""
        S, E = reward_se.shape
        if self.per_env:
            if S == 1 and ops._bcast_len(S, self._L) > 1:
                raise ValueError("per_env with one time column broadcasts the reward to [E, num_envs]: use __call__")
            return self._per_env_scale(reward_se, first_se, group)
        ws = self._workspace(S, E)
        if group is None or not torch.distributed.is_initialized() or torch.distributed.get_world_size(group) == 1:
            ops.reward_scale(reward_se, first_se, self.ret, self.rms, ws, self.gamma, self.cliprew, self.epsilon)
            return reward_se
        moments = torch.zeros(3, dtype=torch.float64, device=self.device)
        ops.reward_scale_moments(reward_se, first_se, self.ret, moments, ws, self.gamma)
        n, mean, m2 = dist_util.gather_moments(moments, group)
        self.rms.copy_(torch.tensor(dist_util.rms_update(self.rms.cpu().tolist(), n, mean, m2), dtype=torch.float64))
        ops.reward_scale_apply(reward_se, self.rms, self.cliprew, self.epsilon)
        return reward_se

    def __call__(self, reward, first):
        """Reference signature: reward, first [E, S] NumPy -> scaled [E, S] NumPy (per_env with S == 1
        and a state longer than 1 returns the reference's broadcast [E, L])."""
        r = torch.tensor(np.ascontiguousarray(np.asarray(reward, np.float64).T), device=self.device)
        f = torch.tensor(np.ascontiguousarray(np.asarray(first).T).astype(np.uint8), device=self.device)
        if self.per_env:
            return self._per_env_scale(r, f, None).cpu().numpy().T
        self.scale_(r, f)
        return r.cpu().numpy().T

    @property
    def ret_rms(self):
        class _RMS:
            pass
        o = _RMS()
        if self.per_env:
            v = self._pe[0].cpu().numpy()
            L = self._L
            o.mean, o.var, o.count = v[1:1 + L].copy(), v[1 + L:1 + 2 * L].copy(), float(v[0])
            return o
        v = self.rms.cpu().numpy()
        o.mean, o.var, o.count = float(v[0]), float(v[1]), float(v[2])
        return o
