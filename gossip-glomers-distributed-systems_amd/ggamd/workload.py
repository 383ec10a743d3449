"""Synthetic workloads of SURVEY.md §8d (seeded; base seed 0x6A09E667F3BCC909 + config#).

A workload = topology + message injections + partition windows + sync
settings. C1 is the reference's own challenge setting (Maelstrom
`--node-count 25 --topology tree4 --rate 100 --latency 100`); C2..C5 are the
scale-up configs of BASELINE.json.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import topology as T
from .engine import Topology

BASE_SEED = 0x6A09E667F3BCC909


@dataclass
class Workload:
    name: str
    topo: Topology
    n_lanes: int
    injections: list  # (node, value, round)
    seed: int
    sync_base: int = 20
    sync_jitter: int = 10
    enable_sync: bool = True
    windows: list = field(default_factory=list)  # ("seeded", r0, r1, epoch_seed)
    max_rounds: int = 400
    gen: dict | None = None  # on-device generator spec of the same graph (Engine.generate kwargs)

    def apply(self, eng):
        if self.topo is None:  # device_gen: the graph is built in HBM (gossip_gen.h)
            eng.generate(**self.gen)
        else:
            eng.topology(self.topo)
        self.apply_events(eng)

    def apply_events(self, eng):
        for w in self.windows:
            if w[0] == "seeded":
                eng.partition_seeded(w[1], w[2], w[3])
            else:
                eng.partition_groups(w[1], w[2], w[3])
        inject(eng, self.injections)


def injection_arrays(injections):
    """(nodes u32, values i64, rounds i64) contiguous arrays of a list of
    (node, value, round) client broadcasts, for repeated inject() calls."""
    a = np.asarray(injections, dtype=np.int64).reshape(-1, 3)
    return (np.ascontiguousarray(a[:, 0], np.uint32), np.ascontiguousarray(a[:, 1]),
            np.ascontiguousarray(a[:, 2]))


def inject(eng, injections):
    """Client broadcasts in call order: a list of (node, value, round) or the
    tuple of arrays from injection_arrays()."""
    if isinstance(injections, tuple) and len(injections) == 3 and isinstance(injections[0], np.ndarray):
        eng.broadcast_many(*injections)
        return
    if not injections:
        return
    eng.broadcast_many(*injection_arrays(injections))


def uniform_injections(V: int, K: int, seed: int, rnd: int = 0) -> list:
    """K fresh values 0..K-1 broadcast by clients at uniform seeded nodes in round `rnd`."""
    rng = np.random.Generator(np.random.PCG64(seed & ((1 << 63) - 1)))
    nodes = rng.integers(0, V, size=K)
    return [(int(nodes[k]), k, rnd) for k in range(K)]


def c1(partition: bool = False, rounds: int = 260, seed: int = BASE_SEED + 1):
    """Config C1, the reference's own test setting (Maelstrom `--node-count 25
    --topology tree4 --rate 100 --latency 100 --time-limit 20`): 10 client ops
    per 100 ms round for 200 rounds, each a broadcast of a fresh value to a
    uniform node with probability 1/2, else a read; sync on; then drain.
    partition: a seeded bisection for rounds [50, 100) (`--nemesis partition`).
    Returns (Workload, number of read ops)."""
    import random
    rnd = random.Random(seed)
    inj, val, reads = [], 0, 0
    for r in range(200):
        for _ in range(10):
            if rnd.random() < 0.5:
                inj.append((rnd.randrange(25), val, r))
                val += 1
            else:
                reads += 1
    W = ((val + 63) // 64) * 64
    windows = [("seeded", 50, 100, seed ^ 0xB15EC7)] if partition else []
    wl = Workload("C1", T.tree(25, 4), W, inj, seed, windows=windows, max_rounds=rounds)
    return wl, reads


# device_gen=True: no host CSR; Workload.apply builds the same graph on the
# device (gossip_gen.h, bit-identical to the host builder)

def c2(V: int = 1 << 20, K: int = 1024, device_gen: bool = False) -> Workload:
    """1M-node tree4, 1024 concurrent messages (1 Kbit sets), sync on, no partitions."""
    seed = BASE_SEED + 2
    gen = dict(kind="tree", n=V, k=4)
    return Workload("C2", None if device_gen else T.tree(V, 4), K, uniform_injections(V, K, seed), seed,
                    gen=gen)


def c3(V: int = 10_000_000, K: int = 1024, device_gen: bool = False) -> Workload:
    """Random 8-regular, seeded random bisection in rounds [2,12) then healed, sync on."""
    seed = BASE_SEED + 3
    gen = dict(kind="random_regular", n=V, k=8, seed=seed)
    return Workload("C3", None if device_gen else T.random_regular(V, 8, seed), K,
                    uniform_injections(V, K, seed), seed, windows=[("seeded", 2, 12, seed ^ 0x5EED)], gen=gen)


def c4(V: int = 100_000_000, K: int = 4096, device_gen: bool = False) -> Workload:
    """R-MAT (.57,.19,.19,.05) edge factor 16, symmetrized; 4096 messages."""
    seed = BASE_SEED + 4
    gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    return Workload("C4", None if device_gen else T.rmat(V, 16, seed=seed), K, uniform_injections(V, K, seed),
                    seed, gen=gen)


def c5(side: int = 32768, K: int = 64, device_gen: bool = False) -> Workload:
    """side^2 grid + 1 long-range link per node (small world); 64 messages."""
    seed = BASE_SEED + 5
    V = side * side
    gen = dict(kind="grid_links", n=side, seed=seed)
    return Workload("C5", None if device_gen else T.grid_links(side, seed), K, uniform_injections(V, K, seed),
                    seed, gen=gen)


def by_name(name: str, **kw) -> Workload:
    return {"C2": c2, "C3": c3, "C4": c4, "C5": c5}[name.upper()](**kw)
