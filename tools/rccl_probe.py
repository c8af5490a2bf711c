"""RCCL ("nccl" backend) on this pool's one-GPU boxes: a world-size-1 process group over RCCL,
the agent's two gradient buckets (critic + metric sums on a side stream, then the actor's on the
main stream: agent :_update split path) all-reduced from the streams the agent issues them on, the
results checked (a sum over one rank is the input) and the per-call time printed. What this shows
is that RCCL initialises and runs under the box's environment (HSA_ENABLE_IPC_MODE_LEGACY=0) with
the stream pattern of the update; one rank moves no bytes, so the times are call overheads, not
bandwidth. Launch: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 ..."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusionpolicyoptimization_amd import ops  # noqa: E402

dist.init_process_group("nccl")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
d = ops.ModelDims()
na, nc = ops.spec_count(ops.actor_param_spec(d)), ops.spec_count(ops.critic_param_spec(d))
grads_ext = torch.randn(na + nc + 6, device=dev)
ref = grads_ext.clone()
side = torch.cuda.Stream(device=dev)
main = torch.cuda.current_stream(dev)
ev = torch.cuda.Event()


def bucket_pair():
    side.wait_stream(main)
    with torch.cuda.stream(side):               # bucket 1: critic gradients + metric sums
        dist.all_reduce(grads_ext[na:])
        ev.record(side)
    dist.all_reduce(grads_ext[:na])             # bucket 2: the actor's gradients
    main.wait_event(ev)


for _ in range(5):
    bucket_pair()
torch.cuda.synchronize()
ok = torch.equal(grads_ext, ref * world)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 100
e0.record()
for _ in range(reps):
    bucket_pair()
e1.record()
torch.cuda.synchronize()
out = {"backend": dist.get_backend(), "world": world, "rank": rank, "actor_bucket_bytes": 4 * na,
       "critic_bucket_bytes": 4 * (nc + 6), "result_ok": bool(ok),
       "us_per_bucket_pair": e0.elapsed_time(e1) / reps * 1e3,
       "note": "world size 1: RCCL init + the update's two-stream bucket pattern; no bytes cross a link"}
if rank == 0:
    print(json.dumps(out))
dist.destroy_process_group()
