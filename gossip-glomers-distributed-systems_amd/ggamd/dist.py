"""Sharded rounds: one engine per GPU (rank), vertex-range shards, one
all-gather of boundary state per round through torch.distributed.

The reference has no equivalent (each Maelstrom node is its own process and
every gossip hop crosses a pipe); here the per-round exchange replaces the
network delivery of every forward/push/read crossing a shard boundary
(SURVEY.md §8e). A round on every rank is

    gg_dist_round_begin   -> the rank's kernels for its own nodes
    all_gather            -> frontier (always), fired bitmap (always) and seen
                             (rounds whose successor may read remote sets) slices
    gg_dist_round_end     -> this rank's counters; all_reduce sums them

On GPUs the backend is "nccl" (= RCCL over xGMI on ROCm) and the gather is
in place on the engine's own device buffers; on CPU (tests) it is gloo over
host buffers of the CPU oracle engine.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from .engine import COUNT_FIELDS, Engine

M64 = (1 << 64) - 1


class _CudaBuf:
    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3, "strides": None}


def _view(ptr: int, nbytes: int, device: torch.device) -> torch.Tensor:
    if device.type == "cuda":
        return torch.as_tensor(_CudaBuf(ptr, nbytes), device=device)
    arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr))
    return torch.from_numpy(arr)


class ShardedRunner:
    def __init__(self, eng: Engine, device: torch.device, group=None):
        self.eng = eng
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert self.world == eng.world and self.rank == eng.rank
        self.inplace = dist.get_backend(group) == "nccl"

    def _gather(self, ptr: int, slice_bytes: int):
        full = _view(ptr, slice_bytes * self.world, self.device)
        own = full[self.rank * slice_bytes:(self.rank + 1) * slice_bytes]
        if self.inplace:
            dist.all_gather_into_tensor(full, own, group=self.group)
        else:
            parts = [full[p * slice_bytes:(p + 1) * slice_bytes] for p in range(self.world)]
            dist.all_gather(parts, own.clone(), group=self.group)

    def round(self) -> dict:
        x = self.eng.dist_round_begin()
        self._gather(x.frontier, x.frontier_bytes)
        self._gather(x.fired, x.fired_bytes)
        if x.flags_bytes:
            self._gather(x.flags, x.flags_bytes)
        if x.need_seen:
            self._gather(x.seen, x.seen_bytes)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        return self.eng.dist_round_end()

    def step(self, n_rounds: int, reduce: bool = True) -> list[dict]:
        local = [self.round() for _ in range(n_rounds)]
        return self.reduce(local) if reduce else local

    def reduce(self, local: list[dict]) -> list[dict]:
        """Sum the per-rank counters of each round (seen_hash mod 2^64)."""
        if not local:
            return []
        vals = np.array([[s[f] for f in COUNT_FIELDS] for s in local], dtype=np.uint64)
        t = torch.from_numpy(vals.view(np.int64).copy())
        ms = torch.tensor([s["kernel_ms"] for s in local], dtype=torch.float64)
        if self.inplace:
            t = t.to(self.device)
            ms = ms.to(self.device)
        dist.all_reduce(t, group=self.group)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX, group=self.group)
        tot = t.cpu().numpy().view(np.uint64)
        out = []
        for k, s in enumerate(local):
            d = {"round": s["round"], "kernel_ms": float(ms[k]),
                 "work_rows": s["work_rows"], "work_gathers": s["work_gathers"]}
            for j, f in enumerate(COUNT_FIELDS):
                d[f] = int(tot[k, j]) & M64
            out.append(d)
        return out
