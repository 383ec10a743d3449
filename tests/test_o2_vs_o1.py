"""O2 (bitset oracle, C ABI) == O1 (message-level literal) on randomized cases.

Covers directed and symmetric topologies, client broadcasts spread over rounds
(repeated values, several per node), seeded and explicit partition windows, and
sync schedules with short intervals so that reads, read_oks, pushes, callback
forwards, drops and acks all occur. Every round's counters and hash, every
node's read set and every delivery round must be identical.
"""
import random

import numpy as np
import pytest

from helpers import c1_scenario, diff_stats, make_engine, make_o1, random_scenario


def _compare(sc, lib):
    o1 = make_o1(sc)
    o2 = make_engine(lib, sc)
    s1 = o1.step(sc.rounds)
    s2 = o2.step(sc.rounds)
    d = diff_stats(s1, s2)
    assert not d, d[:10]
    for v in range(sc.topo.n_nodes):
        assert o1.read(v) == o2.read(v), v
    dr2 = o2.delivery_rounds()
    for v in range(sc.topo.n_nodes):
        assert o1.delivery_rounds(v) == dr2[v].tolist(), v
    return s1


@pytest.mark.parametrize("seed", range(12))
def test_random_small(cpu_lib, seed):
    rnd = random.Random(1000 + seed)
    tot = {}
    for _ in range(8):
        sc = random_scenario(rnd)
        for s in _compare(sc, cpu_lib):
            for k, v in s.items():
                tot[k] = tot.get(k, 0) + (v if k != "seen_hash" else 0)
    # the cases must exercise every message kind
    for k in ("fwd_sent", "pushes", "acks", "reads", "read_oks", "dropped", "new_bits"):
        assert tot[k] > 0, k


def test_c1_tree_client_workload(cpu_lib):
    sc = c1_scenario(partition=False)
    st = _compare(sc, cpu_lib)
    assert sum(s["new_bits"] for s in st) == 25 * len({v for _, v, _ in sc.injections})


def test_c1_tree_client_workload_bisection(cpu_lib):
    sc = c1_scenario(partition=True)
    st = _compare(sc, cpu_lib)
    assert sum(s["dropped"] for s in st) > 0
    assert sum(s["new_bits"] for s in st) == 25 * len({v for _, v, _ in sc.injections})


def test_sync_disabled_and_no_injection(cpu_lib):
    rnd = random.Random(5)
    sc = random_scenario(rnd)
    sc.enable_sync = False
    _compare(sc, cpu_lib)
    sc.injections = []
    st = _compare(sc, cpu_lib)
    assert all(s["new_bits"] == 0 for s in st)


@pytest.mark.parametrize("seed", range(8))
def test_o2_equals_o1_edge_windows(cpu_lib, seed):
    """gg_set_partition (per-edge windows, overriding overlapping group windows):
    O2 = O1 on random symmetric graphs with sync."""
    from helpers import symmetric_random_scenario
    rnd = random.Random(500 + seed)
    sc = symmetric_random_scenario(rnd)
    o1 = make_o1(sc)
    o2 = make_engine(cpu_lib, sc)
    d = diff_stats(o1.step(sc.rounds), o2.step(sc.rounds))
    assert not d, d[:10]
    for v in range(sc.topo.n_nodes):
        assert o1.read(v) == o2.read(v)


def test_edge_window_rejects_asymmetric(cpu_lib):
    from ggamd.engine import Engine, GGError, Topology
    import numpy as np
    topo = Topology.from_rows([[1], [0, 2], [1]])
    e = Engine(3, 64, library=cpu_lib)
    e.topology(topo)
    with pytest.raises(GGError):
        e.set_partition(0, 5, np.array([0b1], np.uint64))  # cuts 0->1 but not 1->0
    e.set_partition(0, 5, np.array([0b11], np.uint64))      # both entries of link 0-1
    d = Topology.from_rows([[1], [], []])
    e2 = Engine(3, 64, library=cpu_lib)
    e2.topology(d)
    with pytest.raises(GGError):
        e2.set_partition(0, 5, np.array([0b1], np.uint64))  # directed topology
