"""Maelstrom broadcast-workload checker (ggamd.checker) on config C1 — the
reference's own test setting (25-node tree4, 100 ops/s, 100 ms latency).

CPU: on the oracle engine the report is internally consistent with the
committed C1 golden fixture (message totals = the fixture's per-round counter
sums) and with the analytic facts of the topology: no value lost, every value
in every final read, and without partitions the stable latency of a broadcast
is its source's eccentricity x 100 ms (<= 500 ms on tree4/25).
GPU: the HIP engine produces the identical report.
"""
import json
import os

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.checker import broadcast_report
from ggamd.engine import Engine
from ggamd.workload import c1

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _run(lib, partition, device=-1):
    wl, nreads = c1(partition=partition)
    e = Engine(25, wl.n_lanes, seed=wl.seed, track_delivery=True, library=lib, device=device)
    wl.apply(e)
    st = e.step(wl.max_rounds)
    return broadcast_report(e, wl.injections, nreads, st), st, wl


@pytest.mark.parametrize("partition,gold", [(False, "c1_tree4"), (True, "c1_tree4_bisect")])
def test_c1_report_on_oracle(cpu_lib, partition, gold):
    rep, st, wl = _run(cpu_lib, partition)
    g = json.load(open(os.path.join(GOLD, gold + ".json")))
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in g["stats"])
    assert rep["inter_node_msgs"] == msgs
    assert rep["broadcast_ops"] + rep["read_ops"] == 2000
    assert rep["lost"] == [] and rep["missing_in_final_reads"] == 0
    if not partition:
        topo = T.tree(25, 4)
        ecc = {s: int(T.bfs(topo, s).max()) for s in range(25)}
        first = {}
        for n, v, r in wl.injections:
            first.setdefault(v, n)
        lat = sorted(ecc[n] * 100.0 for n in first.values())
        assert rep["stable_latency_ms"]["max"] == lat[-1] <= 500.0
        assert rep["stable_latency_ms"]["median"] == float(np.median(lat))
        # KAT-2: 24 forwards + 24 acks per broadcast on a 25-node tree, plus sync traffic
        assert rep["gossip_msgs_per_broadcast"] >= 48.0


@pytest.mark.gpu
@pytest.mark.parametrize("partition", [False, True])
def test_c1_report_gpu_equals_oracle(hip_lib, cpu_lib, partition):
    a, _, _ = _run(hip_lib, partition, device=0)
    b, _, _ = _run(cpu_lib, partition)
    assert a == b
