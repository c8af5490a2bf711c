"""The gradient all-reduce over IPC-mapped peer buffers (csrc/collective.hip, include/dppo.h ABI 12).

SURVEY.md §8(e) puts one all-reduce of the gradient buckets in every PPO minibatch of the
data-parallel update (the reference has none: it applies gradients on one device,
train_ppo_diffusion_agent.py:345-356). RCCL's all_reduce (torch.distributed, backend "nccl") is
the default; `train.allreduce: ipc` replaces it for the fp32 gradient buckets by
dppo_ipc_allreduce: one kernel per call that sums the ranks' data in rank order (the same bits on
every rank) through each peer's region, mapped once with hipIpcOpenMemHandle. One IpcAllReduce
per bucket / stream (calls of one group are ordered; two groups may run concurrently).

Exercised on this pool with 2 and 4 processes sharing one GPU (tests/test_collective_gpu.py);
unmeasured on xGMI."""
import ctypes

import torch
import torch.distributed as dist

from .. import _lib


class IpcAllReduce:
    """Collective constructor: every rank of `group` creates one with the same capacity (fp32
    elements). __call__(t) sums the fp32 CUDA tensor t (contiguous, t.numel() <= capacity) over the
    ranks in place, on `stream` (a raw handle) or the current stream."""

    def __init__(self, capacity, group=None, device=None):
        self.lib = _lib.load()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("dppo_ipc_allreduce supports at most 8 ranks")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.capacity = int(capacity)
        nbytes = int(self.lib.dppo_ipc_region_bytes(self.capacity))
        self._own = ctypes.c_void_p()
        handle = ctypes.create_string_buffer(64)
        with torch.cuda.device(self.device):
            _lib.call("dppo_ipc_alloc", nbytes, ctypes.byref(self._own), handle)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle.raw), group=group)
        self._peers = []
        regions = (ctypes.c_void_p * self.world)()
        for x, h in enumerate(handles):
            if x == self.rank:
                regions[x] = self._own.value
                continue
            p = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                _lib.call("dppo_ipc_open", ctypes.create_string_buffer(h, 64), ctypes.byref(p))
            self._peers.append(p)
            regions[x] = p.value
        self._regions = regions
        fail = ctypes.c_void_p()
        _lib.call("dppo_host_alloc", 4, ctypes.byref(fail))
        self._fail = fail
        self.generation = 0
        # every rank has mapped every peer before any kernel can signal into it
        dist.barrier(group=group)

    def check(self):
        """Raise if any call of this group since the last check timed out in its barrier (a peer did not
        arrive; the kernel's abort word made every workgroup of every rank leave): the reduced buckets
        of that update are not valid. The agent calls it after every update's final synchronize."""
        if self._fail is not None and ctypes.c_uint32.from_address(self._fail.value).value:
            raise _lib.DppoError("dppo_ipc_allreduce: a barrier timed out during this update (a peer did not "
                                 "arrive); the group's results are not valid")

    def __call__(self, t, stream=None):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("IpcAllReduce: expected a contiguous fp32 CUDA tensor")
        n = t.numel()
        if n > self.capacity:
            raise ValueError(f"IpcAllReduce: {n} elements > capacity {self.capacity}")
        self.generation += 1
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        rc = self.lib.dppo_ipc_allreduce(self._regions, self.world, self.rank, self.capacity,
                                         ctypes.c_void_p(t.data_ptr()), n, ctypes.c_uint64(self.generation),
                                         self._fail, ctypes.c_void_p(st))
        if rc != 0:
            raise _lib.DppoError(f"dppo_ipc_allreduce failed ({rc}): {self.lib.dppo_last_error().decode()}")
        return t

    def close(self):
        """Collective: waits for the device, then unmaps the peers and frees the own region."""
        if self._own is None:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)      # no peer still reads or writes the own region
        for p in self._peers:
            self.lib.dppo_ipc_close(p)
        self._peers = []
        dist.barrier(group=self.group)
        self.lib.dppo_ipc_free(self._own)
        self.lib.dppo_host_free(self._fail)
        self._own = None
        self._fail = None
