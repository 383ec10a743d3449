"""Batched gossip (gg_config.batch_ticks).

New semantics, opt-in: the parity mode (batch_ticks = 0) is untouched. A node
keeps what it learns as pending; at the end of every round r with
(r + 1) % B == 0 it sends one message per out-neighbour carrying its pending
values, except to a neighbour that delivered all of them first. Counters
count messages. Pinned here by a message-level Python restatement (below,
sets of values, explicit per-value deliverers and per-neighbour payloads)
against the bitset oracle O2; the HIP engine is checked against O2 on the GPU.
"""
import random

import numpy as np
import pytest

from ggamd.engine import Engine, GGError
from helpers import Scenario, make_engine, random_scenario
from oracle.o1_literal import M64, word_hash


def batched_reference(sc: Scenario, B: int):
    """Message-level restatement: per node a set of values, who delivered each
    pending value first, one message per (sender, neighbour) per send tick."""
    V, W = sc.topo.n_nodes, sc.W
    nw = W // 64
    out = sc.topo.rows()
    lanes = {}
    by_round = {}
    for n, v, r in sc.injections:
        if v not in lanes:
            lanes[v] = len(lanes)
        by_round.setdefault(r, []).append((n, v))
    seen = [set() for _ in range(V)]
    pend = [dict() for _ in range(V)]  # value -> first deliverer ("client" or a node)
    inflight = []  # (sender, receiver, payload) sent last round
    first = {}
    stats, h = [], 0
    for r in range(sc.rounds):
        acks = len(inflight)
        inbox = [[] for _ in range(V)]
        for u, w, pay in inflight:
            inbox[w].append((u, pay))
        new_words = []
        for v in range(V):
            before = set(seen[v])
            for n, val in by_round.get(r, []):
                if n == v and val not in seen[v]:
                    seen[v].add(val)
                    pend[v][val] = "client"
            for u, pay in sorted(inbox[v], key=lambda x: x[0]):
                for val in sorted(pay):
                    if val not in seen[v]:
                        seen[v].add(val)
                        pend[v][val] = u
            words = [0] * nw
            for val in seen[v] - before:
                lane = lanes[val]
                words[lane // 64] |= 1 << (lane % 64)
                first[(v, val)] = r
            new_words.append(words)
        nb = 0
        for v, words in enumerate(new_words):
            for j, x in enumerate(words):
                if x:
                    nb += bin(x).count("1")
                    h = (h + word_hash(v * nw + j, x)) & M64
        sent = []
        if (r + 1) % B == 0:
            for v in range(V):
                if pend[v]:
                    for w in out[v]:
                        pay = {x for x, src in pend[v].items() if src != w}
                        if pay:
                            sent.append((v, w, pay))
                    pend[v] = {}
        inflight = sent
        stats.append({"new_bits": nb, "fwd_sent": len(sent), "fwd_delivered": len(sent), "acks": acks,
                      "pushes": 0, "reads": 0, "read_oks": 0, "dropped": 0, "syncs_fired": 0, "seen_hash": h})
    reads = [sorted(seen[v]) for v in range(V)]
    return stats, reads, first


def _engine(lib, sc, B, **kw):
    sc.enable_sync = False
    return make_engine(lib, sc, batch_ticks=B, **kw)


def _scenarios(seed, n=6, W=128):
    rnd = random.Random(seed)
    out = []
    for _ in range(n):
        sc = random_scenario(rnd, max_v=30, W=W, rounds=24)
        sc.windows = []
        # client broadcasts spread over the first rounds
        sc.injections = [(nd, v, rnd.randrange(0, 8)) for nd, v, _ in sc.injections]
        out.append(sc)
    return out


@pytest.mark.parametrize("B", [1, 2, 3])
def test_o2_batched_equals_message_level(cpu_lib, B):
    for sc in _scenarios(100 + B):
        ref, reads, first = batched_reference(sc, B)
        e = _engine(cpu_lib, sc, B)
        got = e.step(sc.rounds)
        for k, (a, b) in enumerate(zip(ref, got)):
            for f, v in a.items():
                assert b[f] == v, (B, k, f, b[f], v)
        for v in range(sc.topo.n_nodes):
            assert e.read(v) == reads[v]
        dr = e.delivery_rounds()
        lanes = {val: e.lane_of(val) for _, val, _ in sc.injections}
        for (v, val), r in first.items():
            assert dr[v][lanes[val]] == r


def test_batched_fewer_messages_than_parity(cpu_lib):
    """The point of batching: on a tree every value costs E - (N - 1) forwards
    one by one; batched, a node's values of a window share one message."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    topo = T.tree(25, 4)
    inj = [(n, v, v // 10) for n, v, _ in uniform_injections(25, 200, 3)]
    sc = Scenario(topo, 256, 40, inj, seed=4, enable_sync=False)
    parity = make_engine(cpu_lib, sc).step(sc.rounds)
    msgs = {B: sum(s["fwd_sent"] for s in _engine(cpu_lib, sc, B).step(sc.rounds)) for B in (1, 2, 5)}
    p = sum(s["fwd_sent"] for s in parity)
    assert p == 200 * 24  # every value crosses every one of the tree's 24 edges once
    assert msgs[1] < p and msgs[2] < msgs[1] and msgs[5] < msgs[2]


def test_batched_config_rules(cpu_lib):
    with pytest.raises(GGError):
        Engine(10, 64, batch_ticks=2, enable_sync=False, world=2, library=cpu_lib)
    # sync timers and partition windows are part of batched mode
    e = Engine(10, 64, batch_ticks=2, enable_sync=True, library=cpu_lib)
    from ggamd import topology as T
    e.topology(T.tree(10, 2))
    e.partition_seeded(1, 3, 5)


def make_o1b(sc: Scenario, B: int):
    from oracle.o1_batched import O1Batched
    from helpers import apply
    o = O1Batched(sc.topo.n_nodes, sc.W, sc.seed, sc.sync_base, sc.sync_jitter, sc.enable_sync, batch_ticks=B)
    apply(o, sc)
    return o


def _check_vs_o1b(lib, sc, B, **kw):
    o = make_o1b(sc, B)
    e = make_engine(lib, sc, batch_ticks=B, **kw)
    ref, got = o.step(sc.rounds), e.step(sc.rounds)
    for k, (a, b) in enumerate(zip(ref, got)):
        for f, v in a.items():
            assert b[f] == v, (B, k, f, b[f], v)
    for v in range(sc.topo.n_nodes):
        assert e.read(v) == o.read(v), v
    dr = e.delivery_rounds()
    for (v, val), r in o.first_seen.items():
        assert dr[v][e.lane_of(val)] == r


@pytest.mark.parametrize("B", [1, 2, 3])
def test_o1_batched_equals_message_level(B):
    """O1B (oracle/o1_batched.py, the handlers with batched sends) against the
    independent per-value restatement above, where both apply: no sync, no windows."""
    for sc in _scenarios(300 + B):
        ref, reads, first = batched_reference(sc, B)
        sc.enable_sync = False
        o = make_o1b(sc, B)
        got = o.step(sc.rounds)
        for k, (a, b) in enumerate(zip(ref, got)):
            for f, v in a.items():
                assert b[f] == v, (B, k, f, b[f], v)
        assert [o.read(v) for v in range(sc.topo.n_nodes)] == reads
        assert o.first_seen == first


def _sync_scenarios(seed, n=8, W=128):
    """random graphs (directed links included), sync timers from round 1-6,
    seeded and explicit partition windows; every third one symmetric with
    per-edge windows (gg_set_partition) over its group windows"""
    from helpers import symmetric_random_scenario
    rnd = random.Random(seed)
    out = []
    for k in range(n):
        if k % 3 == 2:
            sc = symmetric_random_scenario(rnd, max_v=24, W=W, rounds=40)
        else:
            sc = random_scenario(rnd, max_v=24, W=W, rounds=40)
        sc.enable_sync = True
        sc.injections = [(nd, v, rnd.randrange(0, 12)) for nd, v, _ in sc.injections]
        out.append(sc)
    return out


@pytest.mark.parametrize("B", [1, 2, 3])
def test_o2_batched_sync_partitions_equal_o1b(cpu_lib, B):
    for sc in _sync_scenarios(400 + B):
        _check_vs_o1b(cpu_lib, sc, B)


def test_batched_c1_bisection_loses_nothing(cpu_lib):
    """C1 (25-node tree4, the reference's Maelstrom setting) with a seeded
    bisection window, batched at B = 2 with sync on: every value reaches every
    node (the partition drops batches; the sync pushes repair them), and O2
    equals O1B message for message."""
    from ggamd.workload import c1
    wl, _ = c1(partition=True)
    sc = Scenario(wl.topo, wl.n_lanes, wl.max_rounds, list(wl.injections), seed=wl.seed,
                  enable_sync=True, windows=list(wl.windows))
    _check_vs_o1b(cpu_lib, sc, 2)
    e = make_engine(cpu_lib, sc, batch_ticks=2)
    st = e.step(sc.rounds)
    assert sum(s["dropped"] for s in st) > 0  # the window cut something
    vals = sorted({v for _, v, _ in sc.injections})
    for v in range(sc.topo.n_nodes):
        assert e.read(v) == vals


@pytest.mark.gpu
@pytest.mark.parametrize("W", [64, 128, 1024])
@pytest.mark.parametrize("B", [1, 2, 4])
def test_hip_batched_equals_o2(hip_lib, cpu_lib, W, B):
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    scs = _scenarios(200 + W + B, n=3, W=W)
    scs.append(Scenario(T.tree(3000, 4), W, 30, [(n, v, v % 7) for n, v, _ in uniform_injections(3000, W, 5)],
                        seed=6, enable_sync=False))
    scs.append(Scenario(T.grid_links(40, seed=7), W, 30,
                        [(n, v, v % 5) for n, v, _ in uniform_injections(1600, W // 2, 8)], seed=9,
                        enable_sync=False))
    for sc in scs:
        g = _engine(hip_lib, sc, B, device=0)
        c = _engine(cpu_lib, sc, B)
        gs, cs = g.step(sc.rounds), c.step(sc.rounds)
        from helpers import diff_stats
        d = diff_stats(gs, cs)
        assert not d, d[:10]
        assert np.array_equal(g.read_bits(), c.read_bits())
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())


@pytest.mark.gpu
@pytest.mark.parametrize("W", [64, 128, 512])
@pytest.mark.parametrize("B", [1, 2, 3])
def test_hip_batched_sync_partitions_equal_o2(hip_lib, cpu_lib, W, B):
    """HIP batched rounds with sync timers, pushes, callbacks and partition
    windows (seeded, explicit groups) against O2 (pinned to O1B above)."""
    from helpers import diff_stats
    for sc in _sync_scenarios(500 + W + B, n=6, W=W):
        g = make_engine(hip_lib, sc, batch_ticks=B, device=0)
        c = make_engine(cpu_lib, sc, batch_ticks=B)
        gs, cs = g.step(sc.rounds), c.step(sc.rounds)
        d = diff_stats(gs, cs)
        assert not d, d[:10]
        assert np.array_equal(g.read_bits(), c.read_bits())
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())


@pytest.mark.gpu
def test_hip_batched_c1_bisection_equals_o2(hip_lib, cpu_lib):
    from helpers import diff_stats
    from ggamd.workload import c1
    wl, _ = c1(partition=True)
    sc = Scenario(wl.topo, wl.n_lanes, wl.max_rounds, list(wl.injections), seed=wl.seed,
                  enable_sync=True, windows=list(wl.windows))
    for B in (1, 2, 5):
        g = make_engine(hip_lib, sc, batch_ticks=B, device=0)
        c = make_engine(cpu_lib, sc, batch_ticks=B)
        d = diff_stats(g.step(sc.rounds), c.step(sc.rounds))
        assert not d, (B, d[:10])
        assert np.array_equal(g.read_bits(), c.read_bits())
