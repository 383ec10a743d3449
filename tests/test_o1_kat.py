"""Known-answer tests of the literal oracle O1.

The reference ships no tests or fixtures, so these analytic results are the
anchors that pin O1's reading of `broadcast/broadcast.go` (parity unpinned by
reference tests; see oracle/o1_literal.py header).
"""
import numpy as np
import pytest

from ggamd import topology as T
from ggamd.engine import Topology
from helpers import Scenario, bfs_dist, make_o1
from oracle.o1_literal import O1Network, mix64, sync_interval


def test_mix64_known_values():
    # splitmix64 reference outputs (seed 0 stream: first output of state += golden gamma)
    assert mix64(0) == 0xE220A8397B1DCDAF
    assert mix64(0x9E3779B97F4A7C15) == 0x6E789E6AA1B965F4


def test_sync_interval_range():
    xs = [sync_interval(7, v, k, 20, 10) for v in range(200) for k in range(5)]
    assert min(xs) == 20 and max(xs) == 29
    assert len(set(xs)) == 10


def test_kat1_delivery_round_is_hop_distance():
    topo = T.random_regular(60, 4, seed=3)
    sc = Scenario(topo, 64, 30, [(5, 77, 3)], enable_sync=False)
    o = make_o1(sc)
    o.step(sc.rounds)
    d = bfs_dist(topo, 5)
    for v in range(topo.n_nodes):
        got = o.delivery_rounds(v)[0]
        assert got == (3 + d[v] if d[v] >= 0 else -1)


def test_kat2_tree_one_broadcast_48_messages():
    topo = T.tree(25, 4)
    sc = Scenario(topo, 64, 12, [(17, 1, 0)], enable_sync=False)
    o = make_o1(sc)
    st = o.step(sc.rounds)
    fwd = sum(s["fwd_sent"] for s in st)
    acks = sum(s["acks"] for s in st)
    assert fwd == 24 and acks == 24 and fwd + acks == 48
    assert all(o.read(v) == [1] for v in range(25))


def test_kat3_connected_graph_forwards_E_minus_N_plus_1():
    topo = T.random_regular(50, 6, seed=11)
    E = topo.nnz
    d = bfs_dist(topo, 0)
    assert (d >= 0).all()
    sc = Scenario(topo, 64, 30, [(0, 9, 0)], enable_sync=False)
    o = make_o1(sc)
    st = o.step(sc.rounds)
    fwd = sum(s["fwd_sent"] for s in st)
    assert fwd == E - (topo.n_nodes - 1)
    assert sum(s["acks"] for s in st) == fwd


def test_kat4_single_sync_costs():
    # path 0-1-2; node 1 knows {a}, node 0 knows {b}: one sync of node 1
    rows = [[1], [0, 2], [1]]
    topo = Topology.from_rows(rows)
    o = O1Network(3, 64, seed=0, sync_base=5, sync_jitter=0, enable_sync=True)
    o.topology(rows)
    # only node 1's timer matters for the first 7 rounds: all fire at 5; isolate node 1
    o.broadcast(1, 100, 0)
    st = o.step(4)  # a floods to 0 and 2 by round 1
    assert all(o.read(v) == [100] for v in range(3))
    st = o.step(3)  # rounds 4,5,6: every node fires at 5: reads=deg
    r5 = st[1]
    assert r5["syncs_fired"] == 3 and r5["reads"] == 4
    assert st[2]["read_oks"] == 4
    # all sets equal: no pushes, no forwards from callbacks
    st = o.step(2)
    assert sum(s["pushes"] for s in st) == 0 and sum(s["fwd_sent"] for s in st) == 0


def test_kat4_push_and_callback_forward_counts():
    # star: 0 - {1,2,3}; partition isolates node 1 while 0 learns m; node 1's sync repairs
    rows = [[1, 2, 3], [0], [0], [0]]
    o = O1Network(4, 64, seed=0, sync_base=6, sync_jitter=0, enable_sync=True)
    o.topology(rows)
    o.partition_groups(0, 4, [0, 1, 0, 0])
    o.broadcast(0, 42, 0)
    o.step(6)  # round 5: ...; every node fires at round 6
    assert o.read(1) == [] and o.read(2) == [42]
    st = o.step(3)  # 6: fire (reads), 7: read_oks, 8: callbacks
    cb = st[2]
    # node 0 (deg 3): peer 1 has {}, push 42 to 1; peers 2,3 have {42}: nothing
    # node 1 (deg 1): peer 0 has {42}: new, forwarded to N(1) \ {0} = {} -> 0 forwards
    # nodes 2,3: peer 0 has {42}: nothing new; they push nothing (equal sets)
    assert cb["pushes"] == 1
    assert cb["fwd_sent"] == 0
    assert cb["new_bits"] == 1 and o.read(1) == [42]


def test_kat5_partition_blocks_cross_traffic_until_heal():
    topo = T.random_regular(40, 4, seed=5)
    groups = np.array([v % 2 for v in range(40)], np.uint8)
    sc = Scenario(topo, 64, 60, [(0, 1, 0)], enable_sync=True, sync_base=20, sync_jitter=0,
                  windows=[("groups", 0, 30, groups)])
    o = make_o1(sc)
    o.step(30)
    for v in range(40):
        if groups[v] == 1:
            assert o.read(v) == []
    o.step(30)  # healed at 30; the first sync after that (round 40) repairs
    assert all(o.read(v) == [1] for v in range(40))


def test_read_of_empty_node_is_null():
    """HandleRead's ReadResponse.Messages starts as a nil slice
    (broadcast.go:125): an empty read replies `"messages": null`."""
    o = O1Network(2, 64, enable_sync=False)
    o.topology([[1], [0]])
    assert o.read(0) == []
    assert o.client_read(0, msg_id=5) == {"type": "read_ok", "messages": None, "in_reply_to": 5}
    o.broadcast(1, 9, 0)
    o.step(2)
    assert o.client_read(0)["messages"] == [9]
