"""ctypes binding of the engine C ABI (include/gossip.h).

`Engine` drives any library exporting the gossip.h symbols. The product is
``libgossip_hip.so`` (HIP kernels for gfx950, built in-tree by ``make``);
tests may hand in the CPU oracle library explicitly. `Engine()` without a
library path loads the HIP library and raises if it is missing — there is no
silent CPU fallback on the product path.

The handler surface mirrors the reference node (``broadcast/main.go:22-40``):
``topology`` (HandleTopology), ``broadcast`` (client HandleBroadcast), ``read``
(HandleRead) and ``step`` (the passing of lockstep 100 ms rounds, during which
every node-to-node broadcast, broadcast_ok, read and read_ok happens).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP_LIB = os.environ.get("GG_HIP_LIB") or os.path.join(PKG_DIR, "libgossip_hip.so")
HOST_LIB = os.path.join(PKG_DIR, "libgossip_host.so")

GG_TRACK_DELIVERY = 1
ERRNO = {-5: "EIO", -12: "ENOMEM", -22: "EINVAL", -28: "ENOSPC", -38: "ENOSYS"}


class GGConfig(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint64),
        ("n_lanes", C.c_uint32),
        ("flags", C.c_uint32),
        ("seed", C.c_uint64),
        ("sync_base_ticks", C.c_uint32),
        ("sync_jitter_ticks", C.c_uint32),
        ("enable_sync", C.c_int32),
        ("device", C.c_int32),
        ("rank", C.c_uint32),
        ("world", C.c_uint32),
        ("lane_groups", C.c_uint32),
        ("batch_ticks", C.c_uint32),
    ]


class GGRoundStats(C.Structure):
    _fields_ = [
        ("round", C.c_int64),
        ("new_bits", C.c_uint64),
        ("fwd_sent", C.c_uint64),
        ("fwd_delivered", C.c_uint64),
        ("pushes", C.c_uint64),
        ("push_delivered", C.c_uint64),
        ("acks", C.c_uint64),
        ("reads", C.c_uint64),
        ("read_oks", C.c_uint64),
        ("dropped", C.c_uint64),
        ("syncs_fired", C.c_uint64),
        ("seen_hash", C.c_uint64),
        ("kernel_ms", C.c_double),
        ("work_rows", C.c_uint64),
        ("work_gathers", C.c_uint64),
        ("prep_ms", C.c_double),
        ("expand_ms", C.c_double),
        ("stream_ms", C.c_double),
        ("prep_bytes", C.c_uint64),
        ("expand_bytes", C.c_uint64),
        ("stream_bytes", C.c_uint64),
        ("sent_bytes", C.c_uint64),
        ("path", C.c_uint64),
    ]


class GGExchange(C.Structure):
    _fields_ = [
        ("send", C.c_void_p),
        ("recv", C.c_void_p),
        ("send_bytes", C.POINTER(C.c_uint64)),
        ("recv_bytes", C.POINTER(C.c_uint64)),
        ("send_off", C.POINTER(C.c_uint64)),
        ("recv_off", C.POINTER(C.c_uint64)),
        ("send_total", C.c_uint64),
        ("recv_total", C.c_uint64),
        ("on_device", C.c_int32),
        ("exact", C.c_int32),
        ("stream", C.c_void_p),
    ]


XPORT_START = C.CFUNCTYPE(C.c_int, C.c_void_p)
XPORT_XFER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p)


class GGTransport(C.Structure):  # include/gossip.h gg_transport
    _fields_ = [
        ("user", C.c_void_p),
        ("group_start", XPORT_START),
        ("send", XPORT_XFER),
        ("recv", XPORT_XFER),
        ("group_end", XPORT_START),
    ]


class GGGenSpec(C.Structure):  # include/gossip_gen.h
    _fields_ = [
        ("kind", C.c_uint32),
        ("k", C.c_uint32),
        ("n", C.c_uint64),
        ("a", C.c_double),
        ("b", C.c_double),
        ("c", C.c_double),
        ("seed", C.c_uint64),
    ]


GEN_KINDS = {"tree": 1, "random_regular": 2, "rmat": 3, "grid_links": 4}
GEN_SYMBOLS = ["gg_topology_generate", "gg_topology_export"]  # HIP library only

STAT_FIELDS = [f for f, _ in GGRoundStats._fields_]
DIAG_FIELDS = ("round", "kernel_ms", "work_rows", "work_gathers", "prep_ms", "expand_ms", "stream_ms",
               "prep_bytes", "expand_bytes", "stream_bytes", "sent_bytes", "path")
# gg_round_stats.path bits (gossip.h GG_PATH_*)
IPC_BLOB_BYTES = 1024  # gossip.h GG_IPC_BLOB_BYTES
PATH_STREAM, PATH_DB, PATH_SYNC_STREAM, PATH_TILES, PATH_MASKED, PATH_BATCHED, PATH_NO_PREP = 1, 2, 4, 8, 16, 32, 64
PATH_SOLO = 128
COUNT_FIELDS = [f for f in STAT_FIELDS if f not in DIAG_FIELDS]

GG_SYMBOLS = [
    "gg_abi_version", "gg_create", "gg_destroy", "gg_last_error", "gg_topology",
    "gg_partition_seeded", "gg_partition_groups", "gg_set_partition", "gg_broadcast", "gg_broadcast_many",
    "gg_lane_of", "gg_step", "gg_topology_part", "gg_topology_part_directed",
    "gg_current_round", "gg_step_device_ms", "gg_run_episodes", "gg_read", "gg_read_bits", "gg_delivery_rounds", "gg_reset",
    "gg_device_bytes",
    "gg_read_bits_nodes", "gg_delivery_rounds_nodes",
    "gg_dist_round_begin", "gg_dist_round_end", "gg_dist_flush", "gg_dist_owned", "gg_dist_info",
    "gg_dist_comm_available", "gg_dist_comm_id", "gg_dist_comm_init", "gg_dist_transport_init", "gg_dist_step",
    "gg_dist_ipc_export", "gg_dist_ipc_import", "gg_dist_ipc_close", "gg_dist_run_episodes",
]

_LIBS: dict[str, C.CDLL] = {}


def load_library(path: str) -> C.CDLL:
    path = os.path.abspath(path)
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise FileNotFoundError(f"engine library {path} is not built (run `make` in {PKG_DIR})")
    # One HIP runtime per process: PyTorch ships its own libamdhip64 (soname
    # libamdhip64.so.7, like /opt/rocm's, but loaded by file name). Loaded after the
    # engine, torch brings a second runtime that finds no GPU; loaded first, the
    # engine binds to torch's by soname. So torch, when installed, goes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P = C.POINTER
    lib.gg_abi_version.restype = C.c_int
    lib.gg_create.argtypes = [P(GGConfig), P(C.c_void_p)]
    lib.gg_destroy.argtypes = [C.c_void_p]
    lib.gg_destroy.restype = None
    lib.gg_last_error.argtypes = [C.c_void_p]
    lib.gg_last_error.restype = C.c_char_p
    lib.gg_topology.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    lib.gg_topology_part.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    lib.gg_topology_part_directed.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    lib.gg_partition_seeded.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_uint64]
    lib.gg_partition_groups.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
    lib.gg_set_partition.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
    lib.gg_broadcast.argtypes = [C.c_void_p, C.c_uint32, C.c_int64, C.c_int64]
    lib.gg_broadcast_many.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    lib.gg_lane_of.argtypes = [C.c_void_p, C.c_int64]
    lib.gg_step.argtypes = [C.c_void_p, C.c_uint32, P(GGRoundStats)]
    lib.gg_step_device_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    lib.gg_run_episodes.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(GGRoundStats)]
    lib.gg_current_round.argtypes = [C.c_void_p]
    lib.gg_current_round.restype = C.c_int64
    lib.gg_read.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, P(C.c_uint64)]
    lib.gg_read_bits.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    lib.gg_delivery_rounds.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64]
    lib.gg_reset.argtypes = [C.c_void_p]
    lib.gg_device_bytes.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64)]
    lib.gg_dist_round_begin.argtypes = [C.c_void_p, P(GGExchange)]
    lib.gg_dist_round_end.argtypes = [C.c_void_p, P(GGRoundStats)]
    lib.gg_dist_flush.argtypes = [C.c_void_p, P(GGRoundStats), C.c_uint64, P(C.c_uint64)]
    lib.gg_dist_owned.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]
    lib.gg_dist_info.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(C.c_uint64)]
    lib.gg_read_bits_nodes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.gg_dist_comm_available.argtypes = [C.c_char_p, C.c_uint64]
    lib.gg_dist_comm_id.argtypes = [C.c_void_p, C.c_void_p]
    lib.gg_dist_comm_init.argtypes = [C.c_void_p, C.c_void_p]
    lib.gg_dist_step.argtypes = [C.c_void_p, C.c_uint32]
    lib.gg_dist_run_episodes.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(GGRoundStats)]
    lib.gg_dist_ipc_export.argtypes = [C.c_void_p, C.c_void_p]
    lib.gg_dist_ipc_import.argtypes = [C.c_void_p, C.c_void_p]
    lib.gg_dist_ipc_close.argtypes = [C.c_void_p]
    lib.gg_dist_transport_init.argtypes = [C.c_void_p, P(GGTransport)]
    lib.gg_delivery_rounds_nodes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    if hasattr(lib, "gg_topology_generate"):
        lib.gg_topology_generate.argtypes = [C.c_void_p, P(GGGenSpec), P(C.c_uint64)]
        lib.gg_topology_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]
    _LIBS[path] = lib
    return lib


class GGError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRNO.get(code, code)}: {msg}")
        self.code = code


@dataclass
class Topology:
    n_nodes: int
    row_ptr: np.ndarray  # int64 [V+1]
    col: np.ndarray  # int32 [nnz]

    @property
    def nnz(self) -> int:
        return int(self.col.size)

    def rows(self) -> list[list[int]]:
        return [self.col[self.row_ptr[v]:self.row_ptr[v + 1]].tolist() for v in range(self.n_nodes)]

    @staticmethod
    def from_rows(rows: list[list[int]]) -> "Topology":
        rp = np.zeros(len(rows) + 1, np.int64)
        for v, r in enumerate(rows):
            rp[v + 1] = rp[v] + len(r)
        col = np.array([x for r in rows for x in r], np.int32)
        return Topology(len(rows), rp, col)


def stats_dict(s: GGRoundStats) -> dict:
    return {f: getattr(s, f) for f in STAT_FIELDS}


class Engine:
    """One engine = every simulated node of one topology (or one shard of it)."""

    def __init__(self, n_nodes: int, n_lanes: int, *, seed: int = 0, sync_base: int = 20,
                 sync_jitter: int = 10, enable_sync: bool = True, track_delivery: bool = False,
                 device: int = -1, rank: int = 0, world: int = 1, lane_groups: int = 1,
                 batch_ticks: int = 0, library: str | None = None):
        self.lib = load_library(library or HIP_LIB)
        self.library = os.path.abspath(library or HIP_LIB)
        cfg = GGConfig(n_nodes, n_lanes, GG_TRACK_DELIVERY if track_delivery else 0, seed,
                       sync_base, sync_jitter, 1 if enable_sync else 0, device, rank, world, lane_groups,
                       batch_ticks)
        h = C.c_void_p()
        rc = self.lib.gg_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise GGError(rc, "gg_create failed")
        self.h = h
        self.V, self.W, self.nw = n_nodes, n_lanes, n_lanes // 64
        self.rank, self.world, self.lane_groups = rank, world, lane_groups
        self.parts = world // max(1, lane_groups)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ok(self, rc: int):
        if rc != 0:
            raise GGError(rc, self.lib.gg_last_error(self.h).decode())
        return rc

    # ---- handler surface ---------------------------------------------------

    def topology(self, topo: Topology):
        rp = np.ascontiguousarray(topo.row_ptr, np.int64)
        col = np.ascontiguousarray(topo.col, np.int32)
        self._ok(self.lib.gg_topology(self.h, rp.ctypes.data, col.ctypes.data, col.size))

    def topology_part(self, part_lo, row_ptr, col):
        """gg_topology_part: this rank's own rows only (row_ptr from 0, global
        column ids) and every part's first node (part_lo, P + 1 entries)."""
        plo = np.ascontiguousarray(part_lo, np.uint64)
        rp = np.ascontiguousarray(row_ptr, np.int64)
        cl = np.ascontiguousarray(col, np.int32)
        self._ok(self.lib.gg_topology_part(self.h, plo.ctypes.data, rp.ctypes.data, cl.ctypes.data, cl.size))

    def topology_part_directed(self, part_lo, row_ptr, col):
        """gg_topology_part_directed: this rank's own rows, which may be directed;
        the in-lists come from the other parts (needs the engine's exchange
        first: dist_comm_init or dist_transport_init)."""
        plo = np.ascontiguousarray(part_lo, np.uint64)
        rp = np.ascontiguousarray(row_ptr, np.int64)
        cl = np.ascontiguousarray(col, np.int32)
        self._ok(self.lib.gg_topology_part_directed(self.h, plo.ctypes.data, rp.ctypes.data, cl.ctypes.data, cl.size))

    def generate(self, kind: str, n: int, k: int = 0, seed: int = 0, a: float = 0.0, b: float = 0.0,
                 c: float = 0.0) -> int:
        """Build a synthetic topology in HBM (gossip_gen.h; HIP library only) and
        install it; the graph equals the host builder's (ggamd.topology.tree /
        random_regular / rmat / grid_links with the same arguments). n = nodes,
        or the grid side. Returns the number of adjacency entries."""
        if not hasattr(self.lib, "gg_topology_generate"):
            raise GGError(-38, f"{self.library} has no on-device generators")
        spec = GGGenSpec(GEN_KINDS[kind], k, n, a, b, c, seed & ((1 << 64) - 1))
        nnz = C.c_uint64(0)
        self._ok(self.lib.gg_topology_generate(self.h, C.byref(spec), C.byref(nnz)))
        return nnz.value

    def export_topology(self) -> Topology:
        """The installed topology as CSR (single engine; in-lists, = rows when symmetric)."""
        n = C.c_uint64(0)
        rp = np.zeros(self.V + 1, np.int64)
        self._ok(self.lib.gg_topology_export(self.h, rp.ctypes.data, None, 0, C.byref(n)))
        col = np.zeros(max(1, n.value), np.int32)
        self._ok(self.lib.gg_topology_export(self.h, rp.ctypes.data, col.ctypes.data, col.size, C.byref(n)))
        return Topology(self.V, rp, col[: n.value])

    def partition_seeded(self, r0: int, r1: int, epoch_seed: int):
        self._ok(self.lib.gg_partition_seeded(self.h, r0, r1, epoch_seed))

    def set_partition(self, r0: int, r1: int, bits):
        """Per-edge window (gg_set_partition): one bit per adjacency entry of the
        installed topology (CSR order; uint64 words), 1 = the link is cut both ways."""
        b = np.ascontiguousarray(bits, np.uint64)
        self._ok(self.lib.gg_set_partition(self.h, r0, r1, b.ctypes.data))

    def partition_groups(self, r0: int, r1: int, groups):
        g = np.ascontiguousarray(groups, np.uint8)
        assert g.size == self.V
        self._ok(self.lib.gg_partition_groups(self.h, r0, r1, g.ctypes.data))

    def broadcast(self, node: int, value: int, rnd: int):
        self._ok(self.lib.gg_broadcast(self.h, node, value, rnd))

    def broadcast_many(self, nodes, values, rounds):
        nodes = np.ascontiguousarray(nodes, np.uint32)
        values = np.ascontiguousarray(values, np.int64)
        rounds = np.ascontiguousarray(np.broadcast_to(rounds, nodes.shape), np.int64)
        self._ok(self.lib.gg_broadcast_many(self.h, nodes.ctypes.data, values.ctypes.data,
                                            rounds.ctypes.data, nodes.size))

    def lane_of(self, value: int) -> int:
        return self.lib.gg_lane_of(self.h, value)

    def step(self, n_rounds: int = 1, raw: bool = False):
        """Run n lockstep rounds; per-round stats as dicts (raw=True: the ctypes
        array, to convert later with stats_dict — keeps timed loops lean)."""
        arr = (GGRoundStats * max(1, n_rounds))()
        self._ok(self.lib.gg_step(self.h, n_rounds, arr))
        if raw:
            return arr
        return [stats_dict(arr[i]) for i in range(n_rounds)]

    def run_episodes(self, n_rounds: int, episodes: int, raw: bool = False):
        """gg_run_episodes: right after reset() and the broadcasts, `episodes`
        episodes of that schedule, n_rounds each, with one host wait; per episode
        its rounds' stats (raw=True: one ctypes array, episode k at k * n_rounds)."""
        arr = (GGRoundStats * (n_rounds * episodes))()
        self._ok(self.lib.gg_run_episodes(self.h, n_rounds, episodes, arr))
        if raw:
            return arr
        return [[stats_dict(arr[k * n_rounds + i]) for i in range(n_rounds)] for k in range(episodes)]

    def step_device_ms(self) -> float:
        """HIP-event device time of the last step() call (whole launch sequence;
        after run_episodes: per episode)."""
        x = C.c_double(0.0)
        self._ok(self.lib.gg_step_device_ms(self.h, C.byref(x)))
        return x.value

    @property
    def round(self) -> int:
        return self.lib.gg_current_round(self.h)

    def read(self, node: int) -> list[int]:
        n = C.c_uint64(0)
        self._ok(self.lib.gg_read(self.h, node, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.int64)
        self._ok(self.lib.gg_read(self.h, node, out.ctypes.data, out.size, C.byref(n)))
        return out[: n.value].tolist()

    def read_bits(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.V if hi is None else hi
        out = np.zeros((hi - lo, self.nw), np.uint64)
        self._ok(self.lib.gg_read_bits(self.h, lo, hi, out.ctypes.data))
        return out

    def delivery_rounds(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.V if hi is None else hi
        out = np.zeros((hi - lo, self.W), np.int32)
        self._ok(self.lib.gg_delivery_rounds(self.h, lo, hi, out.ctypes.data, out.size))
        return out

    def read_bits_nodes(self, nodes) -> np.ndarray:
        nodes = np.ascontiguousarray(nodes, np.uint32)
        out = np.zeros((nodes.size, self.nw), np.uint64)
        self._ok(self.lib.gg_read_bits_nodes(self.h, nodes.ctypes.data, nodes.size, out.ctypes.data))
        return out

    def delivery_rounds_nodes(self, nodes) -> np.ndarray:
        nodes = np.ascontiguousarray(nodes, np.uint32)
        out = np.zeros((nodes.size, self.W), np.int32)
        self._ok(self.lib.gg_delivery_rounds_nodes(self.h, nodes.ctypes.data, nodes.size, out.ctypes.data))
        return out

    def reset(self):
        self._ok(self.lib.gg_reset(self.h))

    def device_bytes(self) -> dict:
        """Device memory this engine holds: total and the streamed-sync part
        (allocated at the first round that can reach a sync timer)."""
        t, s = C.c_uint64(0), C.c_uint64(0)
        self._ok(self.lib.gg_device_bytes(self.h, C.byref(t), C.byref(s)))
        return {"total": t.value, "sync": s.value}

    # ---- sharded rounds ------------------------------------------------------

    def dist_owned(self) -> np.ndarray:
        """Original ids of the nodes this engine owns (sharded mode), in its row order."""
        n = C.c_uint64(0)
        self._ok(self.lib.gg_dist_owned(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.uint32)
        self._ok(self.lib.gg_dist_owned(self.h, out.ctypes.data, out.size, C.byref(n)))
        return out[: n.value]

    def dist_info(self) -> dict:
        a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        self._ok(self.lib.gg_dist_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return {"owned": a.value, "ghosts": b.value, "sent_per_round": c.value}

    def dist_round_begin(self) -> GGExchange:
        x = GGExchange()
        self._ok(self.lib.gg_dist_round_begin(self.h, C.byref(x)))
        return x

    def dist_round_end(self, wait: bool = True) -> dict | None:
        if not wait:
            self._ok(self.lib.gg_dist_round_end(self.h, None))
            return None
        s = GGRoundStats()
        self._ok(self.lib.gg_dist_round_end(self.h, C.byref(s)))
        return stats_dict(s)

    def dist_comm_available(self) -> tuple[bool, str]:
        """Do the RCCL entry points resolve in this process (engine-owned exchange)?"""
        buf = C.create_string_buffer(256)
        rc = self.lib.gg_dist_comm_available(buf, 256)
        return rc == 0, buf.value.decode()

    def dist_comm_id(self) -> bytes:
        """An RCCL id for this engine's lane group (ABI 6: gg_dist_comm_init of an
        engine in another lane group refuses it)."""
        buf = (C.c_uint8 * 128)()
        rc = self.lib.gg_dist_comm_id(self.h, buf)
        if rc:
            raise RuntimeError(f"gg_dist_comm_id failed ({rc})")
        return bytes(buf)

    def dist_ipc_export(self) -> bytes:
        """This part's exchange window as a GG_IPC_BLOB_BYTES blob (device-driven exchange)."""
        buf = (C.c_uint8 * IPC_BLOB_BYTES)()
        self._ok(self.lib.gg_dist_ipc_export(self.h, buf))
        return bytes(buf)

    def dist_ipc_import(self, blobs: bytes) -> None:
        """Map the windows of every part of this lane group (P blobs, part order)."""
        assert len(blobs) == self.parts * IPC_BLOB_BYTES
        buf = (C.c_uint8 * len(blobs)).from_buffer_copy(blobs)
        self._ok(self.lib.gg_dist_ipc_import(self.h, buf))

    def dist_ipc_close(self) -> None:
        """Unmap the peers' windows (collective teardown, first half: every part
        calls it, the caller barriers, then the engines are closed)."""
        if getattr(self, "h", None):
            self._ok(self.lib.gg_dist_ipc_close(self.h))

    def dist_comm_init(self, uid: bytes) -> None:
        assert len(uid) == 128
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._ok(self.lib.gg_dist_comm_init(self.h, buf))

    def dist_transport_init(self, t: "GGTransport") -> None:
        """The engine-driven exchange over the caller's transport (callbacks kept
        alive by the caller for the engine's lifetime)."""
        self._xport = t
        self._ok(self.lib.gg_dist_transport_init(self.h, C.byref(t)))

    def dist_step(self, n_rounds: int) -> None:
        """n sharded rounds with the engine's own RCCL exchange; counters pending (dist_flush)."""
        self._ok(self.lib.gg_dist_step(self.h, n_rounds))

    def dist_run_episodes(self, n_rounds: int, episodes: int) -> list[list[dict]]:
        """gg_dist_run_episodes (device-driven exchange or lane groups only): this
        engine's own stats of every round of every episode, one host wait."""
        arr = (GGRoundStats * (n_rounds * episodes))()
        self._ok(self.lib.gg_dist_run_episodes(self.h, n_rounds, episodes, arr))
        return [[stats_dict(arr[k * n_rounds + i]) for i in range(n_rounds)] for k in range(episodes)]

    def dist_flush(self) -> list[dict]:
        n = C.c_uint64(0)
        self._ok(self.lib.gg_dist_flush(self.h, None, 0, C.byref(n)))
        arr = (GGRoundStats * max(1, n.value))()
        self._ok(self.lib.gg_dist_flush(self.h, arr, n.value, C.byref(n)))
        return [stats_dict(arr[i]) for i in range(n.value)]


def missing_symbols(path: str, extra: tuple = ()) -> list[str]:
    lib = C.CDLL(os.path.abspath(path))
    return [s for s in list(GG_SYMBOLS) + list(extra) if not hasattr(lib, s)]
