"""StitchedSequenceDataset (reference agent/dataset/sequence.py:25-176): stitched trajectories of
states / actions with a 1-D traj_lengths array, sampled as (horizon_steps actions, cond_steps states)
windows that never cross an episode boundary. The arrays live on the device; a batch is gathered
there by index arithmetic (no per-sample host loop)."""
import logging

import numpy as np
import torch

log = logging.getLogger(__name__)


def make_indices(traj_lengths, horizon_steps):
    """sequence.py:135-148: for every episode, starts i in [begin, begin + len - horizon] paired
    with the number of steps before i inside the episode. Returns int64 [n, 2]."""
    out = []
    begin = 0
    for L in np.asarray(traj_lengths, np.int64):
        n = int(L) - horizon_steps + 1
        if n > 0:
            s = np.arange(begin, begin + n, dtype=np.int64)
            out.append(np.stack([s, s - begin], axis=1))
        begin += int(L)
    return np.concatenate(out) if out else np.zeros((0, 2), np.int64)


class StitchedSequenceDataset:
    def __init__(self, dataset_path, horizon_steps=64, cond_steps=1, img_cond_steps=1, max_n_episodes=10000,
                 use_img=False, device="cuda:0"):
        if use_img:
            raise NotImplementedError("image observations are outside the gym state-only hot path")
        if not str(dataset_path).endswith(".npz"):
            raise ValueError(f"unsupported dataset format {dataset_path}: .npz only (pickle files are not loaded)")
        self.horizon_steps, self.cond_steps = int(horizon_steps), int(cond_steps)
        self.device = torch.device(device if str(device).startswith(("cuda", "cpu")) else "cuda:0")
        with np.load(dataset_path, allow_pickle=False) as f:
            traj_lengths = np.asarray(f["traj_lengths"][:max_n_episodes])
            total = int(traj_lengths.sum())
            states = np.asarray(f["states"][:total], np.float32)
            actions = np.asarray(f["actions"][:total], np.float32)
        self.indices = make_indices(traj_lengths, self.horizon_steps)
        self.states = torch.tensor(states, device=self.device)
        self.actions = torch.tensor(actions, device=self.device)
        self._idx = torch.tensor(self.indices, device=self.device)
        log.info("Loaded dataset from %s: %d episodes, %d windows", dataset_path, len(traj_lengths), len(self))

    def __len__(self):
        return len(self.indices)

    def gather(self, which):
        """Windows `which` (device int64 [B]) -> {"actions": [B, Ta, Da], "conditions": {"state": [B, To, Do]}}.
        States before the episode start repeat its first state (sequence.py:100-107)."""
        ix = self._idx[which]
        start, before = ix[:, 0], ix[:, 1]
        ta = torch.arange(self.horizon_steps, device=self.device)
        actions = self.actions[start[:, None] + ta[None, :]]
        back = torch.arange(self.cond_steps - 1, -1, -1, device=self.device)      # oldest first
        rows = start[:, None] - torch.minimum(back[None, :], before[:, None])
        return {"actions": actions, "conditions": {"state": self.states[rows]}}

    def __getitem__(self, idx):
        b = self.gather(torch.tensor([int(idx)], device=self.device))
        return {"actions": b["actions"][0], "conditions": {"state": b["conditions"]["state"][0]}}

    def batches(self, batch_size):
        """Consecutive windows in index order, as the reference's unshuffled tf.data pipeline
        (agent/pretrain/train_agent.py:104-107); the last batch may be short."""
        n = len(self)
        for b0 in range(0, n, batch_size):
            yield self.gather(torch.arange(b0, min(n, b0 + batch_size), device=self.device))


def synthetic_dataset(path, n_episodes=8, episode_len=200, obs_dim=11, action_dim=3, seed=0):
    """A small stitched dataset with the reference's npz keys (for tests and demos: the D4RL-derived
    train.npz is not shipped)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(episode_len // 2, episode_len + 1, n_episodes)
    T = int(lens.sum())
    states = rng.uniform(-1, 1, (T, obs_dim)).astype(np.float32)
    actions = np.tanh(states[:, :action_dim] + 0.1 * rng.standard_normal((T, action_dim))).astype(np.float32)
    np.savez(path, states=states, actions=actions, traj_lengths=lens)
    return path
