"""Pretraining host logic without a GPU: StitchedSequenceDataset windows against a direct
restatement of the reference's make_indices / __getitem__ (agent/dataset/sequence.py:89-148), and
the CosineDecayRestarts schedule (agent/pretrain/train_agent.py:117-123)."""
import math

import numpy as np

from diffusionpolicyoptimization_amd.agent.dataset.sequence import (StitchedSequenceDataset, make_indices,
                                                                    synthetic_dataset)
from diffusionpolicyoptimization_amd.util.scheduler import CosineDecayRestarts


def _ref_indices(traj_lengths, horizon):
    out, cur = [], 0
    for L in traj_lengths:
        max_start = cur + L - horizon
        out += [(i, i - cur) for i in range(cur, max_start + 1)]
        cur += L
    return out


def test_indices_match_reference_loop():
    lens = [7, 3, 4, 12, 5]
    for h in (1, 4, 5):
        assert [tuple(x) for x in make_indices(lens, h)] == _ref_indices(lens, h)


def test_windows_match_reference_getitem(tmp_path):
    path = synthetic_dataset(str(tmp_path / "train.npz"), n_episodes=5, episode_len=12, seed=3)
    with np.load(path) as f:
        states, actions, lens = f["states"], f["actions"], f["traj_lengths"]
    H, To = 4, 3
    ds = StitchedSequenceDataset(path, horizon_steps=H, cond_steps=To, device="cpu")
    idx = _ref_indices(list(lens), H)
    assert len(ds) == len(idx)
    for k in range(0, len(idx), 3):
        start, nbs = idx[k]
        st = states[start - nbs:start + 1]
        ref_s = np.stack([st[max(nbs - t, 0)] for t in reversed(range(To))])
        got = ds[k]
        np.testing.assert_array_equal(got["actions"].numpy(), actions[start:start + H])
        np.testing.assert_array_equal(got["conditions"]["state"].numpy(), ref_s)
    b = list(ds.batches(16))
    assert sum(x["actions"].shape[0] for x in b) == len(ds)


def test_cosine_decay_restarts():
    s = CosineDecayRestarts(1e-3, 3000, t_mul=1.0, m_mul=1.0, alpha=0.1)
    assert abs(s(0) - 1e-3) < 1e-15
    assert abs(s(1500) - 1e-3 * (0.9 * 0.5 + 0.1)) < 1e-12
    assert abs(s(3000) - 1e-3) < 1e-15                  # restart
    assert abs(s(2999) - 1e-3 * (0.9 * 0.5 * (1 + math.cos(math.pi * 2999 / 3000)) + 0.1)) < 1e-12
    s2 = CosineDecayRestarts(1.0, 10, t_mul=2.0, m_mul=0.5, alpha=0.0)
    assert abs(s2(10) - 0.5) < 1e-12                     # second cycle starts at m_mul
    assert abs(s2(20) - 0.5 * 0.5 * (1 + math.cos(math.pi * 0.5))) < 1e-12
