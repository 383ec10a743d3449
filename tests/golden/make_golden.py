#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/.

* c1_tree4.json, c1_tree4_bisect.json — config C1 (25-node tree4, ~1000 client
  broadcasts over 200 rounds, sync on, optional bisection window) run by the
  message-level literal oracle O1: per-round counters + hash, every node's
  final read set, every delivery round.
* c{2,3,4,5}_4k.json — 4096-node variants of configs C2..C5 run by the
  bitset oracle O2 (checked equal to O1 on random cases by
  tests/test_o2_vs_o1.py): per-round counters + hash and a SHA-256 of the
  final node sets and delivery rounds.

The reference has no fixtures of its own; these pin the
oracles against regressions and give the GPU tests a fixed target.
Usage: python tests/golden/make_golden.py   (from the repo root)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"),
                os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

from ggamd import topology as T  # noqa: E402
from ggamd.engine import COUNT_FIELDS  # noqa: E402
from ggamd.workload import uniform_injections  # noqa: E402
from helpers import Scenario, c1_scenario, make_engine, make_o1  # noqa: E402

CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")


def scenario_4k(name: str) -> Scenario:
    V = 4096
    if name == "c2":
        topo, W, win = T.tree(V, 4), 1024, []
    elif name == "c3":
        topo, W, win = T.random_regular(V, 8, seed=3), 1024, [("seeded", 2, 12, 0x5EED)]
    elif name == "c4":
        topo, W, win = T.rmat(V, 16, seed=4), 4096, []
    else:
        topo, W, win = T.grid_links(64, seed=5), 64, []
    inj = uniform_injections(V, W, seed={"c2": 2, "c3": 3, "c4": 4, "c5": 5}[name])
    return Scenario(topo, W, 60, inj, seed=11, windows=win)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stats_rows(st):
    return [{f: int(s[f]) for f in ["round"] + COUNT_FIELDS} for s in st]


def main():
    os.makedirs(HERE, exist_ok=True)
    for name, part in (("c1_tree4", False), ("c1_tree4_bisect", True)):
        sc = c1_scenario(partition=part)
        o1 = make_o1(sc)
        st = o1.step(sc.rounds)
        out = {"config": name, "oracle": "O1", "rounds": sc.rounds, "lanes": sc.W,
               "stats": stats_rows(st),
               "reads": [o1.read(v) for v in range(25)],
               "delivery_rounds": [o1.delivery_rounds(v) for v in range(25)]}
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(name, "ok")
    for name in ("c2", "c3", "c4", "c5"):
        sc = scenario_4k(name)
        e = make_engine(CPU_LIB, sc, track=True)
        st = e.step(sc.rounds)
        out = {"config": name + "_4k", "oracle": "O2", "rounds": sc.rounds, "lanes": sc.W,
               "nodes": sc.topo.n_nodes, "edges": sc.topo.nnz, "stats": stats_rows(st),
               "sets_sha256": digest(e.read_bits()),
               "delivery_sha256": digest(e.delivery_rounds())}
        with open(os.path.join(HERE, name + "_4k.json"), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(name, "ok")


if __name__ == "__main__":
    main()
