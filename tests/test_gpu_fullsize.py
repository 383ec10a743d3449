"""BASELINE.json's two largest configs at their full size, in the GPU suite
(graphs built in HBM by the on-device generators, gossip_gen.h).

* C5 and C4 against the CPU oracle O2 at full size, round by round: every
  counter and the delivery hash (tests/golden/fullsize_c5.json, fullsize_c4.json,
  made by tests/golden/make_fullsize_golden.py from the host builders' graphs:
  O2 needs minutes of the host's cores there, beyond this suite's budget).
* C5, 2^30 nodes (grid + one long link per node, W = 64): the grid spans
  every node, so each message must reach all V nodes (P1), and before any
  sync timer fires every node forwards each value to all neighbours but its
  claimer, so forwards = K (nnz - (V - 1)) (KAT-3 / P2); every delivered
  broadcast is acked one round later. Checked round by round to quiescence.
* C3, 10^7 nodes (random 8-regular, a seeded bisection in rounds [2, 12),
  healed by the sync timers): connected, so after the heal every message
  reaches all V nodes (P1) and the run quiesces.
* C4, 10^8 nodes (R-MAT, W = 4096): P1 and KAT-3 against the graph's
  connected components (computed on the GPU from the exported graph); and the
  single engine against the two
  lane-group ranks of a 2-GPU strong-scaling job run one after the other on
  this GPU (gg_config.lane_groups: 2048 lanes each, another kernel
  instantiation over another row width): every round's counters and delivery
  hash, summed over the ranks, equal the single engine's.
The reference has no fixtures at all; the properties are size-independent
consequences of broadcast.go's algorithm, and O2 is pinned
against the message-level restatement O1 and the KATs (tests/test_o2_vs_o1.py).
"""
import json
import os

import numpy as np
import pytest

from ggamd.checks import components, expected_from_components
from ggamd.engine import COUNT_FIELDS, Engine
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def _to_quiescence(e, inj, cap=60):
    inject(e, inj)
    out = []
    while True:
        s = e.step(1)[0]
        out.append(s)
        if (s["new_bits"] == 0 and len(out) > 1) or len(out) >= cap:
            return out


def _golden(name):
    """O2's full-size record of a config (tests/golden/make_fullsize_golden.py:
    the host-built graph, every round's counters and delivery hash)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"fullsize_{name}.json")
    with open(path) as f:
        return json.load(f)


def _diff_golden(st, gold):
    """Every round's counters and seen_hash (the fingerprint of every (node, value)
    first-delivery round so far) against O2's record."""
    want = gold["rounds"]
    assert len(st) == len(want), f"quiescence after {len(st)} rounds, O2 after {len(want)}"
    for a, w in zip(st, want):
        bad = [(f, a[f] & M64, w[f]) for f in COUNT_FIELDS if (a[f] & M64) != w[f]]
        assert not bad, f"round {w['round']}: HIP != O2 {bad}"


def test_c5_full_size_equals_o2(hip_lib):
    """C5 at 2^30 nodes against O2 round by round: the device-generated graph
    has the host builder's adjacency count, and every round's counters and
    delivery hash to quiescence equal O2's run on the host-built graph
    (tests/golden/fullsize_c5.json); then P1 / KAT-3 / ACK."""
    gold = _golden("c5")
    side, K = 32768, 64
    V = side * side
    seed = BASE_SEED + 5
    assert (gold["nodes"], gold["lanes"], gold["seed"]) == (V, K, seed)
    e = Engine(V, K, seed=seed, enable_sync=True, library=hip_lib)
    try:
        nnz = e.generate("grid_links", side, seed=seed)
        st = _to_quiescence(e, injection_arrays(uniform_injections(V, K, seed)))
    finally:
        e.close()
    assert nnz == gold["nnz"]
    _diff_golden(st, gold)
    assert st[-1]["new_bits"] == 0, "no quiescence within 60 rounds"
    assert all(s["syncs_fired"] == 0 for s in st), "a sync timer fired before quiescence"
    assert sum(s["new_bits"] for s in st) == V * K  # P1: every message reached every node
    assert sum(s["fwd_sent"] for s in st) == K * (nnz - (V - 1))  # KAT-3 / P2
    for a, b in zip(st, st[1:]):
        assert b["acks"] == a["fwd_delivered"] + a["push_delivered"]
    print(f"C5 2^30: {len(st) - 1} rounds to full delivery, {nnz} adjacency entries")


def test_c3_full_size_heals(hip_lib):
    V, K = 10_000_000, 1024
    seed = BASE_SEED + 3
    e = Engine(V, K, seed=seed, enable_sync=True, library=hip_lib)
    try:
        e.generate("random_regular", V, k=8, seed=seed)
        e.partition_seeded(2, 12, seed ^ 0x5EED)
        inject(e, injection_arrays(uniform_injections(V, K, seed)))
        st = e.step(48)  # the halves go quiet inside the window; the timers (round >= 20) heal it
    finally:
        e.close()
    assert sum(s["dropped"] for s in st) > 0  # the window cut messages
    assert sum(s["new_bits"] for s in st) == V * K  # P1 after the heal
    last = max(s["round"] for s in st if s["new_bits"])
    assert last >= 20  # the heal needed the sync timers
    print(f"C3 10^7: {last} rounds to full delivery")


def test_c3_full_size_equals_o2(hip_lib, cpu_lib):
    """C3 at its full 10^7 nodes against the CPU oracle O2 (16 host threads)
    on the random 8-regular graph the device generator built:
    every round's counters and delivery hash to quiescence (the bisection cuts
    rounds [2, 12), the timers heal it), then every node's set."""
    import time

    from ggamd.workload import c3
    wl = c3(device_gen=True)
    V = 10_000_000
    mk = lambda lib: Engine(V, wl.n_lanes, seed=wl.seed, sync_base=wl.sync_base, sync_jitter=wl.sync_jitter,
                            enable_sync=wl.enable_sync, library=lib)
    g, c = mk(hip_lib), mk(cpu_lib)
    try:
        t0 = time.time()
        wl.apply(g)  # the graph is built in HBM; O2 takes the same CSR exported from it
        c.topology(g.export_topology())
        wl.apply_events(c)
        print(f"C3 vs O2: engines ready in {time.time() - t0:.0f} s", flush=True)
        total, rounds = 0, 0
        for r in range(60):
            a, b = g.step(1)[0], c.step(1)[0]
            bad = [f for f in COUNT_FIELDS if a[f] != b[f]]
            assert not bad, (r, [(f, a[f], b[f]) for f in bad])
            total += a["new_bits"]
            rounds = r + 1
            print(f"C3 vs O2: round {r} new {a['new_bits']} ({time.time() - t0:.0f} s)", flush=True)
            if r > 20 and total == V * wl.n_lanes and a["new_bits"] == 0:
                break
        assert total == V * wl.n_lanes  # P1 after the heal
        for v0 in range(0, V, 1 << 20):
            n = min(1 << 20, V - v0)
            assert np.array_equal(g.read_bits(v0, v0 + n), c.read_bits(v0, v0 + n)), v0
        print(f"C3 10^7 equals O2 over {rounds} rounds in {time.time() - t0:.0f} s")
    finally:
        g.close()
        c.close()


def test_c4_full_size_equals_o2_and_lane_groups(hip_lib):
    """C4 at 10^8 nodes, W = 4096: the single engine's every round (counters and
    delivery hash) against O2's run on the host-built graph
    (tests/golden/fullsize_c4.json: O2 as 4 lane-group engines of 1024 lanes,
    summed); then, on the same engine: P1 (every message reaches exactly its
    source's connected component) and KAT-3 (no timer fires before
    quiescence, so forwards = Σ_m [vol(comp) - (|comp| - 1)]), with the
    components computed from the exported graph."""
    V, K = 100_000_000, 4096
    seed = BASE_SEED + 4
    gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    inj_l = uniform_injections(V, K, seed)
    inj = injection_arrays(inj_l)
    e = Engine(V, K, seed=seed, enable_sync=True, library=hip_lib)
    gold = _golden("c4")
    assert (gold["nodes"], gold["lanes"], gold["seed"]) == (V, K, seed)
    try:
        nnz = e.generate(**gen)
        want = _to_quiescence(e, inj)
        print("C4: episode done, exporting the graph", flush=True)
        topo = e.export_topology()
    finally:
        e.close()
    assert nnz == gold["nnz"]
    _diff_golden(want, gold)  # O2 on the host-built graph, every round
    assert want[-1]["new_bits"] == 0
    assert all(s["syncs_fired"] == 0 for s in want), "a sync timer fired before quiescence"
    lab, size, vol = components(topo.row_ptr, topo.col)
    del topo
    p1, kat3 = expected_from_components(lab, size, vol, [n for n, _, _ in inj_l])
    assert sum(s["new_bits"] for s in want) == p1, "P1: deliveries != sum of source component sizes"
    assert sum(s["fwd_sent"] for s in want) == kat3, "KAT-3: forwards != sum of vol(comp) - (|comp| - 1)"
    for a, b in zip(want, want[1:]):
        assert b["acks"] == a["fwd_delivered"] + a["push_delivered"]
    R = len(want)
    got = None
    for rank in range(2):
        e = Engine(V, K, seed=seed, enable_sync=True, library=hip_lib, rank=rank, world=2, lane_groups=2)
        try:
            e.generate(**gen)
            inject(e, inj)
            st = e.step(R)
        finally:
            e.close()
        if got is None:
            got = [dict(s) for s in st]
        else:
            for g, s in zip(got, st):
                for f in COUNT_FIELDS:
                    g[f] = (g[f] + s[f]) & M64
    for g, w in zip(got, want):
        for f in COUNT_FIELDS:
            assert g[f] == (w[f] & M64), f"round {w['round']} {f}: lane groups {g[f]} != single {w[f]}"
