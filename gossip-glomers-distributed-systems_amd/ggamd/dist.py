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
hands the exchange to the engine: part 0 of every lane group makes an RCCL
unique id, torch hands the ids round, every engine opens a communicator over
its lane group's parts (gg_dist_comm_init) and gg_dist_step(n) runs n rounds
with grouped ncclSend/ncclRecv of the non-empty segments on the engine stream,
with no Python and no cross-stream event hop per round. With "gloo"
transport="engine" runs the same gg_dist_step sequencing (size handshake,
peers, offsets) over `HostTransport`, gg_transport callbacks that move each
group through host memory with torch.distributed point-to-point ops: the test
harness for the engine's own exchange on ranks that share one GPU.

GG_DIST_TRANSPORT=torch (or transport="torch") keeps the per-round
all_to_all_single through torch instead, enqueued on the engine's own HIP stream
(torch.cuda.ExternalStream); with "gloo" (CPU tests, or several ranks sharing
one GPU in the GPU tests) that path stages the payloads through host memory.
Either way the per-round counters are collected once at the end (gg_dist_flush)
and summed over ranks with one all_reduce.
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


class HostTransport:
    """gg_transport over torch.distributed (gloo), staged through host memory.

    The engine calls group_start, send/recv per peer part, group_end at the
    points where it would issue its RCCL group; group_end synchronises the
    engine stream, copies the send buffers out, runs the point-to-point ops
    with the peers' global ranks, and writes the receive buffers back before
    returning (gossip.h: stream semantics of a host-staged transport)."""

    def __init__(self, eng: Engine, device: torch.device, group=None, rank_of: list[int] | None = None):
        from .engine import XPORT_START, XPORT_XFER, GGTransport
        self.device, self.group = device, group
        P = eng.parts
        lgrp = eng.rank // P
        glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
        # the process rank of each part of this engine's lane group (default: one engine per process)
        self._rank_of = rank_of or [glob(lgrp * P + q) for q in range(P)]
        self.ops = []
        self.error = None
        self.groups = 0
        self._cbs = (XPORT_START(self._start), XPORT_XFER(self._send), XPORT_XFER(self._recv), XPORT_START(self._end))
        self.struct = GGTransport(None, *self._cbs)
        eng.dist_transport_init(self.struct)

    def _start(self, _user):
        self.ops = []
        return 0

    def _send(self, _user, buf, nbytes, part, stream):
        self.ops.append(("send", buf, nbytes, part, stream))
        return 0

    def _recv(self, _user, buf, nbytes, part, stream):
        self.ops.append(("recv", buf, nbytes, part, stream))
        return 0

    def _end(self, _user):
        try:
            self.groups += 1
            if not self.ops:
                return 0
            torch.cuda.ExternalStream(self.ops[0][4], device=self.device).synchronize()
            p2p, back = [], []
            for kind, buf, n, part, _ in self.ops:
                dv = _view(buf, n, True, self.device)
                if kind == "send":
                    p2p.append(dist.P2POp(dist.isend, dv.cpu(), self._rank_of[part], self.group))
                else:
                    hb = torch.empty(n, dtype=torch.uint8)
                    p2p.append(dist.P2POp(dist.irecv, hb, self._rank_of[part], self.group))
                    back.append((dv, hb))
            for w in dist.batch_isend_irecv(p2p):
                w.wait()
            for dv, hb in back:
                dv.copy_(hb)
            torch.cuda.synchronize(self.device)
            return 0
        except BaseException as exc:  # noqa: BLE001  (reported by the engine as GG_EIO)
            self.error = exc
            return 1


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
        if want not in ("engine", "torch", "ipc"):
            raise ValueError(f"transport {want!r}: 'engine', 'torch' or 'ipc'")
        self.host_xport = None
        if want == "ipc" and eng.parts > 1:
            # device-driven exchange: the parts map each other's windows once; the
            # rounds need no collective and no host wait (gossip.h gg_dist_ipc_*)
            self.engine_comm = True
            _ipc_connect([eng], self.group, self.rank, self.world, eng.parts)
        elif self.nccl:
            self.engine_comm = want == "engine" and self._init_engine_comm()
        else:  # gloo: the engine's own sequencing only when asked (transport="engine")
            self.engine_comm = transport == "engine" and eng.parts > 1
            if self.engine_comm:
                self.host_xport = HostTransport(eng, device, group)
        if eng.parts == 1 and self.nccl:
            self.engine_comm = True  # lane groups only: nothing to exchange, gg_dist_step runs the rounds
        if self.engine_comm:
            self.transport = "none (lane groups only)" if eng.parts == 1 else (
                "device-driven: IPC-mapped peer windows, kernel flag hand-over" if want == "ipc" else
                "engine RCCL send/recv" if self.nccl else "engine sequencing, gloo host transport")
        else:
            self.transport = "torch all_to_all_single" if self.nccl else "gloo via host"

    def close(self) -> None:
        """Collective: drop the device-driven exchange's peer mappings on every rank
        before any rank closes its engine (see _ipc_teardown)."""
        if self.transport.startswith("device-driven"):
            _ipc_teardown([self.eng], self.group)
            self.transport = "closed"

    def _init_engine_comm(self) -> bool:
        """Open the engine's own RCCL communicator (over its lane group's parts)
        if every rank can (agreed by an all_reduce first, so no rank waits in a
        collective init alone). Part 0 of each lane group makes the group's id;
        one all_gather hands every rank its group's id."""
        if self.eng.parts == 1:
            return False
        ok, why = self.eng.dist_comm_available()
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 0:
            return False
        P = self.eng.parts
        uid = torch.zeros(128, dtype=torch.uint8, device=self.device)
        if self.rank % P == 0:
            uid.copy_(torch.frombuffer(bytearray(self.eng.dist_comm_id()), dtype=torch.uint8))
        ids = [torch.empty_like(uid) for _ in range(self.world)]
        dist.all_gather(ids, uid, group=self.group)
        self.eng.dist_comm_init(ids[self.rank // P * P].cpu().numpy().tobytes())
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
        self.exchange(x)
        return self.eng.dist_round_end(wait=wait)

    def exchange(self, x) -> None:
        """The exchange of a begun round (gg_dist_round_begin's gg_exchange)."""
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
            return
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

    def step(self, n_rounds: int, reduce: bool = True) -> list[dict]:
        if self.engine_comm:
            try:
                self.eng.dist_step(n_rounds)
            except Exception:
                if self.host_xport is not None and self.host_xport.error is not None:
                    raise self.host_xport.error
                raise
        else:
            for _ in range(n_rounds):
                self.round(wait=False)
        local = self.eng.dist_flush()
        return self.reduce(local) if reduce else local

    @property
    def can_run_episodes(self) -> bool:
        """gg_dist_run_episodes applies: the device-driven exchange, or lane groups only."""
        return self.engine_comm and (self.transport.startswith("device-driven") or self.eng.parts == 1)

    def run_episodes(self, n_rounds: int, episodes: int) -> list[list[dict]]:
        """Right after reset() and the broadcasts on this rank (every rank calls
        it alike): `episodes` episodes of n_rounds rounds back to back on the
        device, one host wait; this rank's stats per episode (not reduced)."""
        return self.eng.dist_run_episodes(n_rounds, episodes)

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


def _ipc_connect(engines: list[Engine], group, rank: int, world: int, P: int) -> None:
    """Every process exports its engines' windows (one blob each, engines in
    lane-group order), one all_gather of the blobs, and each engine imports the
    P blobs of its own lane group in part order."""
    import time

    from .engine import IPC_BLOB_BYTES
    dbg = os.environ.get("GG_IPC_DEBUG")
    t0 = time.perf_counter()
    err = None
    if dbg:
        print(f"_ipc_connect rank {rank}: exporting", flush=True)
    try:
        mine = b"".join(e.dist_ipc_export() for e in engines)
    except Exception as exc:  # still join the all_gather (zero blobs: every importer refuses them)
        err = exc
        mine = bytes(IPC_BLOB_BYTES * len(engines))
    t = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
    if dist.get_backend(group) == "nccl":
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    got = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(got, t, group=group)
    allb = [g.cpu().numpy().tobytes() for g in got]  # allb[r][h * BLOB:]: engine h of rank r
    if dbg:
        print(f"_ipc_connect rank {rank}: exported and gathered in {time.perf_counter() - t0:.3f} s", flush=True)
    if err is not None:
        raise err
    B = IPC_BLOB_BYTES
    # the ranks map their peers' windows one rank at a time (a barrier between
    # turns; GG_IPC_SERIAL_IMPORT=0: all at once), so a mapping that does not
    # return names its rank. The stall this was first tried against (C4 2^24 on 2
    # ranks) was the windows' size, not concurrency: the engine now allocates
    # windows above 1 GiB in whole GiB
    serial = os.environ.get("GG_IPC_SERIAL_IMPORT", "1") != "0"
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    ierr = None
    for turn in range(world if serial else 1):
        if not serial or turn == rank:
            try:
                for h, e in enumerate(engines):
                    g = rank // P  # the process's lane group index (rank = group * P + part)
                    blobs = b"".join(allb[g * P + q][h * B:(h + 1) * B] for q in range(P))
                    e.dist_ipc_import(blobs)
            except Exception as exc:  # noqa: BLE001 — every rank still takes part in every turn
                ierr = exc
        if serial:
            dist.all_reduce(torch.zeros(1, dtype=torch.int32, device=dev), group=group)
    if dbg:
        print(f"_ipc_connect rank {rank}: imported ({'in turn' if serial else 'at once'}) in "
              f"{time.perf_counter() - t0:.3f} s", flush=True)
    if ierr is not None:
        raise ierr


def _ipc_teardown(engines: list[Engine], group) -> None:
    """Collective: every rank leaves the exchange (gg_dist_ipc_close: its stream
    drained, its peers' windows no longer used), then one all_reduce, so that no
    engine is destroyed — its window going back to the process's pool, to be
    zeroed and exported by a later engine — while a peer may still write into it.
    A rank whose call failed still joins the collective."""
    err = None
    dbg = os.environ.get("GG_IPC_DEBUG")
    for e in engines:
        try:
            e.dist_ipc_close()
        except Exception as exc:  # noqa: BLE001
            err = err or exc
    if dbg:
        print(f"_ipc_teardown rank {dist.get_rank(group)}: left the exchange ({err!r})", flush=True)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    dist.all_reduce(flag, group=group)
    if dbg:
        print(f"_ipc_teardown rank {dist.get_rank(group)}: barrier passed", flush=True)
    if err is not None:
        raise err


def _sum_rounds(a: list[dict], b: list[dict]) -> list[dict]:
    """Per-round counters of two engines over disjoint lanes, summed (seen_hash mod 2^64)."""
    out = []
    for x, y in zip(a, b):
        d = dict(x)
        for f in COUNT_FIELDS:
            d[f] = (x[f] + y[f]) & M64
        d["kernel_ms"] = max(x["kernel_ms"], y["kernel_ms"])
        d["sent_bytes"] = x["sent_bytes"] + y["sent_bytes"]
        out.append(d)
    return out


class HalvesRunner:
    """Two engines per GPU, each half of this process's message lanes, so one
    half's exchange overlaps the other half's kernels.

    Process p = g * P + q of a job with L lane groups x P vertex parts holds
    engines (2g, q) and (2g + 1, q) of a 2L x P engine grid (gg_config
    lane_groups = 2L, world = 2N): the same vertex range, lanes split in two.
    Lane groups never interact, so the job's results are those of the L x P
    job. Each engine has its own HIP stream and its own exchange (an RCCL
    communicator over its lane group's P parts, or HostTransport over gloo), and
    a round is enqueued half by half: while half A's payload moves, half B's
    kernels run, and the reverse for A's next round. On a graph where every
    node has remote neighbours (R-MAT, random long links) this is the overlap
    that interior-first ordering cannot give: there are no interior nodes."""

    def __init__(self, engines: list[Engine], device: torch.device, group=None, transport: str | None = None):
        assert len(engines) == 2
        self.engs = engines
        self.device, self.group = device, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        P = engines[0].parts
        self.P = P
        g, q = divmod(self.rank, P)
        for h, e in enumerate(engines):
            assert e.world == 2 * self.world and e.rank == (2 * g + h) * P + q and e.parts == P
        self.nccl = dist.get_backend(group) == "nccl"
        glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
        self.xports = []
        want = transport or os.environ.get("GG_DIST_TRANSPORT", "engine")
        if P == 1:
            self.transport = "none (lane groups only)"
        elif want == "ipc":
            _ipc_connect(engines, group, self.rank, self.world, P)
            self.transport = "device-driven: IPC-mapped peer windows, two lane halves per GPU"
        elif self.nccl:
            ok = all(e.dist_comm_available()[0] for e in engines)
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            if int(flag.item()) == 0:
                raise RuntimeError("RCCL entry points unavailable on some rank")
            uid = torch.zeros(2, 128, dtype=torch.uint8, device=device)
            if q == 0:
                for h, e in enumerate(engines):
                    uid[h].copy_(torch.frombuffer(bytearray(e.dist_comm_id()), dtype=torch.uint8))
            ids = [torch.empty_like(uid) for _ in range(self.world)]
            dist.all_gather(ids, uid, group=group)
            for h, e in enumerate(engines):
                e.dist_comm_init(ids[g * P][h].cpu().numpy().tobytes())
            self.transport = "engine RCCL send/recv, two lane halves per GPU"
        else:
            for e in engines:
                self.xports.append(HostTransport(e, device, group, rank_of=[glob(g * P + x) for x in range(P)]))
            self.transport = "engine sequencing, gloo host transport, two lane halves per GPU"

    def close(self) -> None:
        """Collective: drop both halves' peer mappings on every rank before any
        rank closes its engines (see _ipc_teardown)."""
        if self.transport.startswith("device-driven"):
            _ipc_teardown(self.engs, self.group)
            self.transport = "closed"

    def step(self, n_rounds: int, reduce: bool = True) -> list[dict]:
        if self.transport.startswith("device-driven"):
            # both halves' rounds are enqueued at once on their own streams; the
            # kernels' flags order each half's rounds with its peers, and the two
            # streams overlap one half's exchange with the other half's kernels
            for e in self.engs:
                e.dist_step(n_rounds)
        else:
            for _ in range(n_rounds):
                for e in self.engs:  # half A's round, then half B's: B's kernels run during A's exchange
                    e.dist_step(1)
        local = _sum_rounds(self.engs[0].dist_flush(), self.engs[1].dist_flush())
        return ShardedRunner.reduce(self, local) if reduce else local
