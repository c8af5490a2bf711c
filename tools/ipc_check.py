"""IPC all-reduce check (tests/test_collective_gpu.py): W ranks under torch.distributed.run, all on
cuda:0 (DPPO_SINGLE_DEVICE rehearsal: same-device IPC), gloo for the handle exchange. Each rank
sums seeded per-rank data with util/ipc.IpcAllReduce — several sizes, consecutive calls (the slot
alternation), and two groups on two streams at once (the agent's two buckets) — and saves its
inputs and results to $DPPO_IPC_DIR/rank<r>.npz.
    DPPO_IPC_DIR=/tmp/ipc python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29513 tools/ipc_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = (1, 7, 1000, 135_000, 687_941)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from diffusionpolicyoptimization_amd.util.ipc import IpcAllReduce
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    g1 = IpcAllReduce(max(SIZES), device=dev)
    g2 = IpcAllReduce(200_000, device=dev)
    side = torch.cuda.Stream(device=dev)
    out = {}
    rng = np.random.default_rng(100 + rank)
    for k, n in enumerate(SIZES * 2):                 # every size twice: both slots
        x = rng.normal(0, 1 + rank, n).astype(np.float32)
        y = rng.normal(0, 1, min(n, 200_000)).astype(np.float32)
        tx, ty = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        g1(tx)                                        # main stream
        with torch.cuda.stream(side):                 # the other group, concurrently
            g2(ty)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        out[f"x{k}"], out[f"y{k}"] = x, y
        out[f"sx{k}"], out[f"sy{k}"] = tx.cpu().numpy(), ty.cpu().numpy()
    np.savez(os.path.join(os.environ["DPPO_IPC_DIR"], f"rank{rank}.npz"), world=world, **out)
    g1.close()
    g2.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
