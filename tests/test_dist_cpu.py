"""Data-parallel decomposition on world_size 2, 4 and 8 with gloo on the CPU: every
cross-rank reduction the agent performs gives the single-process oracle's answer on the whole
batch. The same util/dist.py functions run over RCCL on GPUs."""
import socket

import pytest
import torch.multiprocessing as mp

from diffusionpolicyoptimization_amd.util import dist as D
from tests import dist_workers as W


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, world=2):
    mp.spawn(fn, args=(world, _port()), nprocs=world, join=True)


def test_shard_envs():
    assert [D.shard_envs(64, 4, r) for r in range(4)] == [(16, 0), (16, 16), (16, 32), (16, 48)]
    with pytest.raises(ValueError):
        D.shard_envs(10, 4, 0)


def test_chan_merge_matches_concatenation():
    import numpy as np
    rng = np.random.default_rng(0)
    parts = [rng.normal(i, 1 + i, 100 + 37 * i) for i in range(4)]
    trip = [(p.size, p.mean(), ((p - p.mean()) ** 2).sum()) for p in parts]
    n, mean, m2 = D.chan_merge(trip)
    x = np.concatenate(parts)
    assert n == x.size
    np.testing.assert_allclose([mean, m2], [x.mean(), ((x - x.mean()) ** 2).sum()], rtol=1e-12)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_reward_rms(world):
    """The rank-order Chan merge of the reward-RMS moments at 2 / 4 / 8 ranks."""
    _spawn(W.reward_rms, world)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gradient(world):
    """The advantage-moment table and the summed 1/B-scaled gradients at 2 / 4 / 8 ranks."""
    _spawn(W.dp_gradient, world)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_episode_stats_and_explained_variance(world):
    _spawn(W.episodes_and_ev, world)
