"""Edge cases of the handler surface: the HIP engine against O2 through the same
C ABI, with sets, counters and error codes compared.

* a single node (`HandleTopology` with an empty neighbour list, `broadcast.go:36-48`):
  broadcasts stay local, sync timers fire with nobody to read;
* a topology without links: every value stays on the node a client gave it to,
  reads of the other nodes are empty (`HandleRead` `:124-132`, `null` on the wire);
* ragged rows (degrees 0 to V-1, one-way links);
* a client re-broadcasting a value the node already holds, and a second node
  receiving it from a client after gossip delivered it (`HandleBroadcast`
  `:59-79`: a seen value is acknowledged and not forwarded);
* calls both libraries must refuse, with the same code: a node out of range, a
  broadcast scheduled in a past round, more distinct values than lanes.
"""
import pytest

from ggamd import topology as T
from ggamd.engine import GGError, Topology
from helpers import Scenario, diff_stats, make_engine

pytestmark = pytest.mark.gpu


def _both(hip_lib, cpu_lib, sc):
    g = make_engine(hip_lib, sc)
    c = make_engine(cpu_lib, sc)
    d = diff_stats(g.step(sc.rounds), c.step(sc.rounds))
    assert not d, d[:10]
    assert (g.read_bits() == c.read_bits()).all()
    assert (g.delivery_rounds() == c.delivery_rounds()).all()
    return g, c


def test_single_node(hip_lib, cpu_lib):
    sc = Scenario(Topology.from_rows([[]]), 64, 12, [(0, 5, 0), (0, 7, 0), (0, 9, 2), (0, 5, 3)], seed=3,
                  sync_base=1, sync_jitter=1)
    g, c = _both(hip_lib, cpu_lib, sc)
    assert g.read(0) == c.read(0) == [5, 7, 9]


def test_no_links(hip_lib, cpu_lib):
    V = 6
    inj = [(v, 100 + v, v % 3) for v in range(0, V, 2)] + [(2, 7, 4)]
    sc = Scenario(Topology.from_rows([[] for _ in range(V)]), 64, 30, inj, seed=4, sync_base=3, sync_jitter=2)
    g, c = _both(hip_lib, cpu_lib, sc)
    for v in range(V):
        assert g.read(v) == c.read(v)
    assert g.read(1) == [] and g.read(2) == [7, 102]


def test_ragged_rows(hip_lib, cpu_lib):
    V = 9
    rows = [[1, 2, 3, 4, 5, 6, 7, 8], [], [0], [0, 4], [3], [0, 6, 7], [5], [], [0]]  # 1 and 7 only receive
    inj = [(0, 1, 0), (3, 2, 0), (6, 3, 1), (1, 4, 2), (7, 5, 5)]
    sc = Scenario(Topology.from_rows(rows), 128, 40, inj, seed=5, sync_base=6, sync_jitter=3)
    _both(hip_lib, cpu_lib, sc)


def test_rebroadcast_of_seen_values(hip_lib, cpu_lib):
    topo = T.tree(20, 4)
    inj = [(0, 11, 0), (0, 11, 3), (7, 11, 4), (19, 11, 6), (5, 12, 1), (5, 12, 1)]
    sc = Scenario(topo, 64, 30, inj, seed=6, sync_base=8, sync_jitter=2)
    g, _ = _both(hip_lib, cpu_lib, sc)
    assert g.read(19) == [11, 12]


def _code(fn):
    try:
        fn()
    except GGError as e:
        return e.code
    return 0


def test_refused_calls_match(hip_lib, cpu_lib):
    codes = []
    for lib in (hip_lib, cpu_lib):
        e = make_engine(lib, Scenario(T.tree(10, 2), 64, 0, []))
        got = [_code(lambda: e.broadcast(10, 1, 0)),  # node out of range
               _code(lambda: e.read(10))]
        e.step(2)
        got.append(_code(lambda: e.broadcast(0, 1, 1)))  # round 1 is past
        for v in range(64):
            e.broadcast(v % 10, 1000 + v, 2)
        got.append(_code(lambda: e.broadcast(0, 5000, 2)))  # a 65th distinct value, W = 64
        got.append(_code(lambda: e.broadcast(0, 1000, 3)))  # a known value still fits
        codes.append(got)
        e.close()
    assert codes[0] == codes[1], codes
    assert all(x != 0 for x in codes[0][:4]) and codes[0][4] == 0, codes
