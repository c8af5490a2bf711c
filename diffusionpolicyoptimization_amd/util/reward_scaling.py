"""RunningRewardScaler (reference util/reward_scaling.py:42-87) on the device.

The scan (discounted running return), the moment reduction and the rescale run in one fp64 HIP
pass set (dppo_reward_scale*). The reference API — __call__(reward [E,S], first [E,S]) on NumPy
arrays — is kept; the agent uses the time-major device form scale_() without host round trips.
Multi-GPU: the per-rank moments are merged with an all-reduce before the update (Chan's rule), so
every rank applies the same global statistics."""
import numpy as np
import torch

from .. import ops
from . import dist as dist_util


class RunningRewardScaler:
    def __init__(self, num_envs, cliprew=10.0, gamma=0.99, epsilon=1e-8, per_env=False, device=None):
        if per_env:
            raise NotImplementedError("per_env=True is not used by any fine-tune cfg and is not implemented")
        self.num_envs, self.cliprew, self.gamma, self.epsilon = num_envs, cliprew, gamma, epsilon
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ret = torch.zeros(num_envs, dtype=torch.float64, device=self.device)
        self.rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=self.device)  # mean, var, count
        self._ws = None

    def _workspace(self, S, E):
        if self._ws is None or self._ws[0] != (S, E):
            self._ws = ((S, E), ops.reward_scale_workspace(S, E, self.device))
        return self._ws[1]

    def scale_(self, reward_se, first_se, group=None):
        """In place on time-major device tensors reward [S,E] fp64, first [S,E] u8."""
        S, E = reward_se.shape
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
        """Reference signature: reward, first [E, S] NumPy -> scaled [E, S] NumPy."""
        r = torch.tensor(np.ascontiguousarray(np.asarray(reward, np.float64).T), device=self.device)
        f = torch.tensor(np.ascontiguousarray(np.asarray(first).T).astype(np.uint8), device=self.device)
        self.scale_(r, f)
        return r.cpu().numpy().T

    @property
    def ret_rms(self):
        class _RMS:
            pass
        v = self.rms.cpu().numpy()
        o = _RMS()
        o.mean, o.var, o.count = float(v[0]), float(v[1]), float(v[2])
        return o
