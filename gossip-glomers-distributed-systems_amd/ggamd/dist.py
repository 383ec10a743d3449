"""Sharded rounds: one engine per GPU (rank), locality-ordered vertex ranges,
one all-to-all-v of packed ghost payloads per round through torch.distributed.

The reference has no equivalent (each Maelstrom node is its own process and
every gossip hop crosses a pipe); here the per-round exchange replaces the
network delivery of every forward/push/read/read_ok crossing a shard boundary
(SURVEY.md §8e). A round on every rank is

    gg_dist_round_begin   -> the rank's kernels for its owned nodes, then a pack
                             kernel: for each other rank q, the owned nodes q
                             holds as ghosts (F row, flags, sync-fired bit, and
                             the set row in sync rounds)
    all_to_all_single     -> per-peer byte counts from the engine
    gg_dist_round_end     -> unpack kernel into this rank's ghost rows

On GPUs the backend is "nccl" (= RCCL over xGMI on ROCm). By default `step`
hands the exchange to the engine: rank 0 makes an RCCL unique id, torch
broadcasts it, every engine opens its own communicator (gg_dist_comm_init) and
gg_dist_step(n) runs n rounds with grouped ncclSend/ncclRecv of the non-empty
segments on the engine stream, with no Python and no cross-stream event hop per
round. GG_DIST_TRANSPORT=torch (or transport="torch") keeps the per-round
all_to_all_single through torch instead, enqueued on the engine's own HIP stream
(torch.cuda.ExternalStream). Either way a multi-round step runs without host
synchronisation and the per-round counters are collected once at the end
(gg_dist_flush) and summed over ranks with one all_reduce. With "gloo" (CPU tests, or several ranks sharing one GPU in the GPU
tests) the payloads are staged through host memory.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist

from .engine import COUNT_FIELDS, Engine

M64 = (1 << 64) - 1


class _CudaBuf:
    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3, "strides": None}


def _view(ptr: int, nbytes: int, on_device: bool, device: torch.device) -> torch.Tensor:
    if nbytes == 0 or not ptr:
        return torch.empty(0, dtype=torch.uint8, device=device if on_device else "cpu")
    if on_device:
        return torch.as_tensor(_CudaBuf(ptr, nbytes), device=device)
    arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr))
    return torch.from_numpy(arr)


class ShardedRunner:
    def __init__(self, eng: Engine, device: torch.device, group=None, transport: str | None = None):
        self.eng = eng
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert self.world == eng.world and self.rank == eng.rank
        self.nccl = dist.get_backend(group) == "nccl"
        self._views = {}   # (ptr, bytes, on_device) -> tensor view of engine memory
        self._streams = {}  # stream ptr -> torch.cuda.ExternalStream
        want = transport or os.environ.get("GG_DIST_TRANSPORT", "engine")
        if want not in ("engine", "torch"):
            raise ValueError(f"transport {want!r}: 'engine' or 'torch'")
        self.engine_comm = self.nccl and want == "engine" and self._init_engine_comm()
        self.transport = "engine RCCL send/recv" if self.engine_comm else (
            "torch all_to_all_single" if self.nccl else "gloo via host")

    def _init_engine_comm(self) -> bool:
        """Open the engine's own RCCL communicator if every rank can (agreed by
        an all_reduce first, so no rank waits in a collective init alone)."""
        ok, why = self.eng.dist_comm_available()
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 0:
            return False
        uid = torch.zeros(128, dtype=torch.uint8, device=self.device)
        if self.rank == 0:
            uid.copy_(torch.frombuffer(bytearray(self.eng.dist_comm_id()), dtype=torch.uint8))
        src = 0 if self.group is None else dist.get_global_rank(self.group, 0)
        dist.broadcast(uid, src=src, group=self.group)
        self.eng.dist_comm_init(uid.cpu().numpy().tobytes())
        return True

    def _view(self, ptr, nbytes, on_dev):
        key = (ptr, nbytes, on_dev)
        v = self._views.get(key)
        if v is None:
            v = self._views[key] = _view(ptr, nbytes, on_dev, self.device)
        return v

    def _stream(self, ptr):
        if not ptr:
            return None
        s = self._streams.get(ptr)
        if s is None:
            s = self._streams[ptr] = torch.cuda.ExternalStream(ptr, device=self.device)
        return s

    def round(self, wait: bool = False) -> dict | None:
        """One sharded round with the exchange through torch.distributed: every
        rank first tells every rank how many bytes it sends it (an all_to_all of
        the sizes: the engine's segments carry only what the peer reads next
        round), then the segments move point-to-point into the
        receivers' fixed segment offsets."""
        x = self.eng.dist_round_begin()
        W = self.world
        on_dev = bool(x.on_device)
        ss = [int(x.send_bytes[i]) for i in range(W)]
        soff = [int(x.send_off[i]) for i in range(W)]
        roff = [int(x.recv_off[i]) for i in range(W)]
        ext = self._stream(x.stream)
        size_dev = self.device if self.nccl else torch.device("cpu")
        st = torch.tensor(ss, dtype=torch.int64, device=size_dev)
        rt = torch.empty_like(st)
        if self.nccl and ext is not None:
            # torch orders the collective only with the current stream (ext): the
            # read of its result must be issued on ext as well, not on the default stream
            with torch.cuda.stream(ext):
                dist.all_to_all_single(rt, st, group=self.group)
                rs = rt.cpu().tolist()
        else:
            dist.all_to_all_single(rt, st, group=self.group)
            rs = rt.cpu().tolist()
        for i in range(W):
            x.recv_bytes[i] = rs[i]
        if not any(ss) and not any(rs):
            return self.eng.dist_round_end(wait=wait)
        send = self._view(x.send, x.send_total, on_dev)
        recv = self._view(x.recv, x.recv_total, on_dev)
        stage = on_dev and not self.nccl  # gloo with device buffers (ranks sharing one GPU): via host
        if stage:
            if ext is not None:
                ext.synchronize()
            send_b, recv_b = send.cpu(), torch.empty(recv.numel(), dtype=torch.uint8)
        else:
            send_b, recv_b = send, recv
        glob = (lambda r: r) if self.group is None else (lambda r: dist.get_global_rank(self.group, r))
        ops = []
        for q in range(W):
            if ss[q]:
                ops.append(dist.P2POp(dist.isend, send_b[soff[q]:soff[q] + ss[q]], glob(q), self.group))
            if rs[q]:
                ops.append(dist.P2POp(dist.irecv, recv_b[roff[q]:roff[q] + rs[q]], glob(q), self.group))
        if self.nccl and ext is not None:
            with torch.cuda.stream(ext):
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
        else:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if stage:
            if ext is not None:
                with torch.cuda.stream(ext):
                    recv.copy_(recv_b)
            else:
                recv.copy_(recv_b)
        return self.eng.dist_round_end(wait=wait)

    def step(self, n_rounds: int, reduce: bool = True) -> list[dict]:
        if self.engine_comm:
            self.eng.dist_step(n_rounds)
        else:
            for _ in range(n_rounds):
                self.round(wait=False)
        local = self.eng.dist_flush()
        return self.reduce(local) if reduce else local

    def reduce(self, local: list[dict]) -> list[dict]:
        """Sum the per-rank counters of each round (seen_hash mod 2^64)."""
        if not local:
            return []
        vals = np.array([[s[f] for f in COUNT_FIELDS] for s in local], dtype=np.uint64)
        t = torch.from_numpy(vals.view(np.int64).copy())
        ms = torch.tensor([s["kernel_ms"] for s in local], dtype=torch.float64)
        if self.nccl:
            t = t.to(self.device)
            ms = ms.to(self.device)
        dist.all_reduce(t, group=self.group)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX, group=self.group)
        tot = t.cpu().numpy().view(np.uint64)
        ms = ms.cpu()
        out = []
        for k, s in enumerate(local):
            d = dict(s)
            d["kernel_ms"] = float(ms[k])
            for j, f in enumerate(COUNT_FIELDS):
                d[f] = int(tot[k, j]) & M64
            out.append(d)
        return out
