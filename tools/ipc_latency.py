"""Per-call latency of the IPC gradient all-reduce (util/ipc.IpcAllReduce, csrc/collective.hip) at the
update's bucket sizes — the critic bucket + metrics (134,913 + 6 floats, 0.54 MB) and the actor bucket
(553,020 floats, 2.2 MB) — with W processes sharing cuda:0 (same-device IPC: this pool's rehearsal; NOT
an xGMI figure). Each rank times `reps` back-to-back calls on its stream with HIP events; rank 0 writes
the max over ranks of the mean per-call time to $DPPO_IPC_OUT (JSON).
    DPPO_IPC_OUT=gpurun_out/ipc_w2.json python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29515 tools/ipc_latency.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = {"critic_bucket_0.54MB": 134_919, "actor_bucket_2.2MB": 553_020}


def main():
    import torch
    import torch.distributed as dist

    from diffusionpolicyoptimization_amd.util.ipc import IpcAllReduce
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    reps = int(os.environ.get("DPPO_IPC_REPS", "200"))
    res = {}
    for name, n in SIZES.items():
        g = IpcAllReduce(n, device=dev)
        t = torch.randn(n, device=dev)
        for _ in range(20):
            g(t)
        torch.cuda.synchronize(dev)
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g(t)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        g.check()
        all_us = [None] * world
        dist.all_gather_object(all_us, us)
        res[name] = {"floats": n, "us_per_call_max_over_ranks": max(all_us), "us_per_call_per_rank": all_us}
        g.close()
    if rank == 0:
        out = {"world": world, "device": "one MI355X shared by all ranks (same-device IPC; not xGMI)",
               "reps": reps, **res}
        with open(os.environ.get("DPPO_IPC_OUT", "ipc_latency.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
