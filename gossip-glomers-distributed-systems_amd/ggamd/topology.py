"""Topology builders (libgossip_host.so) returned as `Topology` CSR objects.

The five configs of SURVEY.md §8d; seeds default to the survey's base seed
0x6A09E667F3BCC909 + config number.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .engine import HOST_LIB, Topology

BASE_SEED = 0x6A09E667F3BCC909


class _CSR(C.Structure):
    _fields_ = [("n_nodes", C.c_uint64), ("nnz", C.c_uint64),
                ("row_ptr", C.POINTER(C.c_int64)), ("col", C.POINTER(C.c_int32))]


_lib = None


def host_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(HOST_LIB):
            raise FileNotFoundError(f"{HOST_LIB} not built (run make)")
        _lib = C.CDLL(HOST_LIB)
        P = C.POINTER(_CSR)
        _lib.ggh_tree.argtypes = [C.c_uint64, C.c_uint32, P]
        _lib.ggh_random_regular.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, P]
        _lib.ggh_rmat.argtypes = [C.c_uint64, C.c_uint32, C.c_double, C.c_double, C.c_double,
                                  C.c_uint64, P]
        _lib.ggh_grid_links.argtypes = [C.c_uint64, C.c_uint64, P]
        _lib.ggh_csr_free.argtypes = [P]
        _lib.ggh_is_symmetric.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        _lib.ggh_topology_json.argtypes = [C.c_char_p, C.c_uint64, P]
        _lib.ggh_components.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        _lib.ggh_bfs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
    return _lib


def _take(fn, *args) -> Topology:
    lib = host_lib()
    c = _CSR()
    rc = getattr(lib, fn)(*args, C.byref(c))
    if rc != 0:
        raise RuntimeError(f"{fn} failed: {rc}")
    try:
        V, nnz = c.n_nodes, c.nnz
        rp = np.ctypeslib.as_array(c.row_ptr, shape=(V + 1,)).copy()
        col = np.ctypeslib.as_array(c.col, shape=(max(1, nnz),))[:nnz].copy()
    finally:
        lib.ggh_csr_free(C.byref(c))
    return Topology(int(V), rp, col)


def tree(V: int, k: int = 4) -> Topology:
    """Maelstrom ``tree4``: parent(i) = (i-1)/k."""
    return _take("ggh_tree", V, k)


def random_regular(V: int, d: int = 8, seed: int = BASE_SEED + 3) -> Topology:
    return _take("ggh_random_regular", V, d, seed)


def rmat(V: int, edge_factor: int = 16, a=0.57, b=0.19, c=0.19, seed: int = BASE_SEED + 4) -> Topology:
    return _take("ggh_rmat", V, edge_factor, a, b, c, seed)


def grid_links(side: int, seed: int = BASE_SEED + 5) -> Topology:
    return _take("ggh_grid_links", side, seed)


def from_maelstrom(msg) -> Topology:
    """A Maelstrom `topology` message (JSON text/bytes, or the decoded dict) -> CSR.
    HandleTopology (`broadcast/broadcast.go:36-48`) keeps topology["n<id>"] per node;
    here every row at once, sorted and de-duplicated, missing rows empty."""
    if isinstance(msg, dict):
        import json
        msg = json.dumps(msg)
    if isinstance(msg, str):
        msg = msg.encode()
    return _take("ggh_topology_json", msg, len(msg))


def to_maelstrom(t: Topology) -> dict:
    """CSR -> the `topology` map Maelstrom sends (node "n<i>")."""
    return {f"n{v}": [f"n{int(u)}" for u in t.col[t.row_ptr[v]:t.row_ptr[v + 1]]] for v in range(t.n_nodes)}


def is_symmetric(t: Topology) -> bool:
    return bool(host_lib().ggh_is_symmetric(t.row_ptr.ctypes.data, t.col.ctypes.data, t.n_nodes))


def components(t: Topology) -> np.ndarray:
    """Weak component label (smallest member id) of every node."""
    lab = np.empty(t.n_nodes, np.uint32)
    host_lib().ggh_components(t.row_ptr.ctypes.data, t.col.ctypes.data, t.n_nodes, lab.ctypes.data)
    return lab


def bfs(t: Topology, src: int) -> np.ndarray:
    """Hop distance from src along the rows (-1: unreachable)."""
    d = np.empty(t.n_nodes, np.int32)
    host_lib().ggh_bfs(t.row_ptr.ctypes.data, t.col.ctypes.data, t.n_nodes, src, d.ctypes.data)
    return d
