"""Shared drivers for the parity tests: run one scenario on any engine."""
from __future__ import annotations

import itertools
import os
import random
import socket
from dataclasses import dataclass, field

import numpy as np

from ggamd.engine import COUNT_FIELDS, Engine, Topology


@dataclass
class Scenario:
    topo: Topology
    W: int
    rounds: int
    injections: list  # (node, value, round) in call order
    seed: int = 1
    sync_base: int = 20
    sync_jitter: int = 10
    enable_sync: bool = True
    windows: list = field(default_factory=list)  # ("seeded", r0, r1, epoch) | ("groups", r0, r1, arr)
    #                                              | ("edges", r0, r1, uint64 bit words over the CSR)
    gen: dict | None = None  # the same graph as an on-device generator spec (Engine.generate kwargs)


def apply(eng, sc: Scenario, generate: bool = False):
    """Feed a scenario to an Engine (C ABI) or an O1Network (same method names);
    generate: build the graph with the on-device generator (sc.gen)."""
    if generate:
        eng.generate(**sc.gen)
    else:
        eng.topology(sc.topo if isinstance(eng, Engine) else sc.topo.rows())
    for w in sc.windows:
        if w[0] == "seeded":
            eng.partition_seeded(w[1], w[2], w[3])
        elif w[0] == "edges":
            eng.set_partition(w[1], w[2], w[3])
        else:
            eng.partition_groups(w[1], w[2], w[3])
    for n, v, r in sc.injections:
        eng.broadcast(int(n), int(v), int(r))


def make_engine(lib: str, sc: Scenario, track=True, generate=False, **kw) -> Engine:
    e = Engine(sc.topo.n_nodes, sc.W, seed=sc.seed, sync_base=sc.sync_base,
               sync_jitter=sc.sync_jitter, enable_sync=sc.enable_sync, track_delivery=track,
               library=lib, **kw)
    apply(e, sc, generate)
    return e


def make_o1(sc: Scenario):
    from oracle.o1_literal import O1Network
    o = O1Network(sc.topo.n_nodes, sc.W, sc.seed, sc.sync_base, sc.sync_jitter, sc.enable_sync)
    apply(o, sc)
    return o


def diff_stats(a: list[dict], b: list[dict]) -> list[str]:
    out = []
    for x, y in zip(a, b):
        for f in COUNT_FIELDS:
            if x[f] != y[f]:
                out.append(f"round {x['round']} {f}: {x[f]} != {y[f]}")
    if len(a) != len(b):
        out.append(f"length {len(a)} != {len(b)}")
    return out


def random_scenario(rnd: random.Random, max_v=40, directed_p=0.2, W=None, rounds=50) -> Scenario:
    V = rnd.randrange(2, max_v)
    rows = [set() for _ in range(V)]
    for _ in range(rnd.randrange(0, 3 * V)):
        a, b = rnd.randrange(V), rnd.randrange(V)
        if a != b:
            rows[a].add(b)
            if rnd.random() >= directed_p:
                rows[b].add(a)
    topo = Topology.from_rows([sorted(r) for r in rows])
    W = W or 64 * rnd.randrange(1, 3)
    inj = [(rnd.randrange(V), rnd.randrange(3 * W // 2), rnd.randrange(rounds // 2))
           for _ in range(rnd.randrange(1, W))]
    # keep distinct values <= W
    seen, inj2 = set(), []
    for n, v, r in inj:
        if v in seen or len(seen) < W:
            seen.add(v)
            inj2.append((n, v, r))
    windows = []
    if rnd.random() < 0.7:
        a = rnd.randrange(0, 8)
        windows.append(("seeded", a, a + rnd.randrange(1, 12), rnd.randrange(1 << 30)))
    if rnd.random() < 0.5:
        a = rnd.randrange(22, 30)
        windows.append(("groups", a, a + rnd.randrange(1, 8), np.array(
            [rnd.randrange(3) for _ in range(V)], np.uint8)))
    return Scenario(topo, W, rounds, inj2, seed=rnd.randrange(1 << 40),
                    sync_base=rnd.randrange(1, 7), sync_jitter=rnd.randrange(0, 3),
                    enable_sync=rnd.random() < 0.85, windows=windows)


def bfs_dist(topo: Topology, src: int) -> np.ndarray:
    """Directed hop distance from src along out-lists (row v = who v sends to)."""
    V = topo.n_nodes
    d = np.full(V, -1, np.int64)
    d[src] = 0
    frontier = [src]
    k = 0
    while frontier:
        k += 1
        nxt = []
        for u in frontier:
            for w in topo.col[topo.row_ptr[u]:topo.row_ptr[u + 1]]:
                if d[w] < 0:
                    d[w] = k
                    nxt.append(int(w))
        frontier = nxt
    return d


def c1_scenario(partition=False, rounds=260, seed=0x6A09E667F3BCC909 + 1) -> Scenario:
    """Config C1: 25-node tree4, 10 client ops per round for 200 rounds (~50%
    broadcasts of fresh values at uniform nodes), sync on, then drain."""
    from ggamd import topology as T
    topo = T.tree(25, 4)
    rnd = random.Random(seed)
    inj, val = [], 0
    for r in range(200):
        for _ in range(10):
            if rnd.random() < 0.5:
                inj.append((rnd.randrange(25), val, r))
                val += 1
    W = ((val + 63) // 64) * 64
    windows = [("seeded", 50, 100, seed ^ 0xB15EC7)] if partition else []
    return Scenario(topo, W, rounds, inj, seed=seed, windows=windows)


def symmetric_cut(topo: Topology, rnd: random.Random, p: float) -> np.ndarray:
    """A random set of cut links as gg_set_partition bits: each undirected link
    u-v is cut with probability p, its two adjacency entries together."""
    E = topo.nnz
    words = np.zeros((E + 63) // 64, np.uint64)
    for u in range(topo.n_nodes):
        for k in range(int(topo.row_ptr[u]), int(topo.row_ptr[u + 1])):
            v = int(topo.col[k])
            if v <= u or rnd.random() >= p:
                continue
            kr = int(topo.row_ptr[v]) + int(np.searchsorted(topo.col[topo.row_ptr[v]:topo.row_ptr[v + 1]], u))
            for x in (k, kr):
                words[x >> 6] |= np.uint64(1) << np.uint64(x & 63)
    return words


def symmetric_random_scenario(rnd: random.Random, max_v=60, W=None, rounds=50, edge_windows=2) -> Scenario:
    """random_scenario on a symmetric topology, plus per-edge windows (some
    overlapping its group windows, which they override)."""
    sc = random_scenario(rnd, max_v=max_v, directed_p=0.0, W=W, rounds=rounds)
    wins = list(sc.windows)
    for _ in range(edge_windows):
        a = rnd.randrange(0, 30)
        wins.append(("edges", a, a + rnd.randrange(1, 10), symmetric_cut(sc.topo, rnd, rnd.choice([0.1, 0.3, 0.7]))))
    ok = []
    for w in wins:  # per-edge windows must not overlap each other
        if w[0] == "edges" and any(x[0] == "edges" and w[1] < x[2] and x[1] < w[2] for x in ok):
            continue
        ok.append(w)
    sc.windows = ok
    return sc


_ports = itertools.count()


def free_port() -> int:
    """A rendezvous port below Linux's ephemeral range (32768-60999): a port the
    OS handed out and this process closed again can be handed to one of gloo's
    own outgoing connections before the store binds it (EADDRINUSE, seen once
    in the GPU suite). Ports step per call and per process, and each is checked
    by a bind first."""
    for _ in range(4000):
        p = 20000 + (os.getpid() * 61 + next(_ports) * 7) % 12000
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free rendezvous port")

