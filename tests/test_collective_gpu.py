"""The IPC gradient all-reduce (csrc/collective.hip, util/ipc.py) with 2 and 4
processes sharing cuda:0 (same-device IPC: RCCL cannot place two ranks on one GPU, and this pool
gives one GPU per box). The sum over ranks must be the same bits on every rank and equal to a
sequential float32 sum in rank order; the data-parallel agent on it must match one rank over the
union of the shards, and every rank must end the iteration with bit-identical parameters."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(script, world, env_extra, timeout=240):
    env = dict(os.environ, DPPO_SINGLE_DEVICE="1", **env_extra)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tools", script)],
                         env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_allreduce_is_the_rank_order_sum_on_every_rank(cuda, tmp_path, world):
    _run("ipc_check.py", world, {"DPPO_IPC_DIR": str(tmp_path)})
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    k = 0
    while f"x{k}" in r[0]:
        for v in ("x", "y"):
            want = r[0][f"{v}{k}"].copy()
            for i in range(1, world):                 # sequential fp32 sum in rank order
                want = (want + r[i][f"{v}{k}"]).astype(np.float32)
            for i in range(world):
                np.testing.assert_array_equal(r[i][f"s{v}{k}"], want)
        k += 1
    assert k == 10


def test_data_parallel_update_over_ipc(cuda, tmp_path):
    """tools/dp_equiv.py (2 ranks, the reference-batch DP agent) with the gradient buckets summed by
    dppo_ipc_allreduce instead of gloo: the replicas see one gradient, which equals the single
    rank's over the union of their rows (test_data_parallel_update_equals_single_rank_on_the_union
    checks the same with gloo), and end the iteration with bit-identical parameters."""
    _run("dp_equiv.py", 2, {"DPPO_DIST_BACKEND": "gloo", "DPPO_EQUIV_DIR": str(tmp_path), "DPPO_ALLREDUCE": "ipc"},
         timeout=300)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(2)]
    np.testing.assert_array_equal(r[0]["grads"], r[1]["grads"])
    np.testing.assert_array_equal(np.load(tmp_path / "rank0_params_end.npy"), np.load(tmp_path / "rank1_params_end.npy"))
    # against the same run over gloo (the bucket sums of two ranks are a + b either way)
    g_dir = tmp_path / "gloo"
    g_dir.mkdir()
    _run("dp_equiv.py", 2, {"DPPO_DIST_BACKEND": "gloo", "DPPO_EQUIV_DIR": str(g_dir)}, timeout=300)
    rg = dict(np.load(g_dir / "rank0.npz"))
    scale = np.abs(rg["grads"]).max()
    # the minibatch's own gradients differ by float-atomic order between the two runs
    assert np.abs(r[0]["grads"] - rg["grads"]).max() <= 1e-5 * scale
    np.testing.assert_allclose(r[0]["metrics"], rg["metrics"], rtol=1e-5, atol=1e-8)
