"""GPU parity of the streamed sync rounds (sync_records + expand_stream_sync):
rounds after the sync timers start, without partition windows, on graphs
without in-hubs, at every row width (W = 64: one word per node, one lane). Every case runs on the default (streamed) path and
on the tile path (GG_SYNC_TILES=1) and must equal the CPU oracle O2 bit for bit
(counters of every round, node sets, delivery rounds). The cases push the
record format to its edges: sparse and dense rounds, more than three
contributing senders (the in-list walk), LAG folds, callbacks, client
broadcasts during sync, directed graphs (out-degree != in-degree).
"""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine, random_scenario

pytestmark = pytest.mark.gpu


def _compare(sc, hip_lib, cpu_lib, path):
    g = make_engine(hip_lib, sc, device=0)
    c = make_engine(cpu_lib, sc)
    gs = g.step(sc.rounds)
    d = diff_stats(gs, c.step(sc.rounds))
    assert not d, d[:10]
    sync = [s for s in gs if s["round"] >= sc.sync_base + 2]
    if path == "stream":  # the tile kernel never runs in sync rounds
        assert sync and all(s["expand_bytes"] == 0 for s in sync)
        assert sum(s["stream_bytes"] for s in sync) > 0
    elif path == "tiles":
        assert sum(s["expand_bytes"] for s in sync) > 0
    assert np.array_equal(g.read_bits(), c.read_bits())
    assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())


@pytest.fixture(params=["stream", "tiles"])
def path(request, monkeypatch):
    monkeypatch.setenv("GG_SYNC_TILES", "1" if request.param == "tiles" else "0")
    return request.param


@pytest.mark.parametrize("W", [64, 128, 1024, 4096])
@pytest.mark.parametrize("directed_p", [0.0, 0.3])
def test_random_sync_rounds(hip_lib, cpu_lib, path, W, directed_p):
    rnd = random.Random(W * 7 + int(directed_p * 10))
    for _ in range(5):
        sc = random_scenario(rnd, max_v=300, W=W, rounds=40, directed_p=directed_p)
        sc.windows = []
        sc.enable_sync = True
        _compare(sc, hip_lib, cpu_lib, path)


@pytest.mark.parametrize("jitter", [0, 1, 6])
def test_synchronous_timers_many_pushers(hip_lib, cpu_lib, path, jitter):
    """Jitter 0: every node fires in the same rounds, so every in-edge pushes and
    most nodes have more than three contributing senders (in-list walk);
    degree 24 and client broadcasts spread over the sync rounds."""
    topo = T.random_regular(2048, 24, seed=77)
    inj = [(n, v, 3 + v % 17) for n, v, _ in uniform_injections(2048, 1000, 78)]
    sc = Scenario(topo, 1024, 30, inj, seed=79, sync_base=2, sync_jitter=jitter)
    _compare(sc, hip_lib, cpu_lib, path)


def test_dense_sync_rounds(hip_lib, cpu_lib, path):
    """Propagation and sync overlap: most nodes active (dense rounds visit every node)."""
    topo = T.random_regular(8192, 8, seed=80)
    sc = Scenario(topo, 256, 24, uniform_injections(8192, 256, 81), seed=82, sync_base=1, sync_jitter=3)
    _compare(sc, hip_lib, cpu_lib, path)


def test_tree_long_sync(hip_lib, cpu_lib, path):
    """C2's shape at 4096 nodes, run far into the sync phase."""
    topo = T.tree(4096, 4)
    inj = uniform_injections(4096, 512, 83) + [(n, 512 + v, 30) for n, v, _ in uniform_injections(4096, 100, 84)]
    sc = Scenario(topo, 1024, 60, inj, seed=85, sync_base=20, sync_jitter=10)
    _compare(sc, hip_lib, cpu_lib, path)


def _digest_scenario():
    """Converges early, then many quiet sync rounds (the saturation digest's
    fast path), with new lanes broadcast late (digest reset), a value
    re-broadcast at another node (same lane: no reset) and a partition-free
    directed sprinkle of hubs-free random edges."""
    topo = T.random_regular(4096, 8, seed=91)
    inj = uniform_injections(4096, 200, 92)
    inj += [(n, 200 + v, 44) for n, v, _ in uniform_injections(4096, 20, 93)]  # new lanes, mid-sync
    inj += [(17, 5, 52), (4000, 210, 57)]  # values already known: no new lane
    inj += [(n, 300 + v, 70) for n, v, _ in uniform_injections(4096, 3, 94)]
    return Scenario(topo, 256, 100, inj, seed=95, sync_base=6, sync_jitter=5)


def test_digest_quiet_rounds(hip_lib, cpu_lib, monkeypatch):
    """Bit-exact with the digest on, and the digest is what saves the work:
    the quiet sync rounds move far fewer bytes than with GG_SYNC_DIGEST=0."""
    sc = _digest_scenario()
    monkeypatch.setenv("GG_SYNC_TILES", "0")
    _compare(sc, hip_lib, cpu_lib, "stream")
    monkeypatch.setenv("GG_SYNC_DIGEST", "0")
    off = make_engine(hip_lib, sc, device=0).step(sc.rounds)
    monkeypatch.delenv("GG_SYNC_DIGEST")
    on = make_engine(hip_lib, sc, device=0).step(sc.rounds)
    assert not diff_stats(on, off)
    late = range(32, 44)  # converged, before the late broadcasts
    b_on = sum(on[r]["stream_bytes"] for r in late)
    b_off = sum(off[r]["stream_bytes"] for r in late)
    assert b_on < 0.5 * b_off, (b_on, b_off)


def test_digest_lane_groups(hip_lib, cpu_lib, monkeypatch):
    """Per lane group the digest counts that group's lanes only: the summed
    counters of 2 and 4 lane groups equal the single engine's."""
    from ggamd.engine import COUNT_FIELDS, Engine
    monkeypatch.setenv("GG_SYNC_TILES", "0")
    sc = _digest_scenario()
    ref = make_engine(cpu_lib, sc).step(sc.rounds)
    for L in (2, 4):
        tot = None
        for r in range(L):
            e = make_engine(hip_lib, sc, track=False, device=0, rank=r, world=L, lane_groups=L)
            st = e.step(sc.rounds)
            e.close()
            if tot is None:
                tot = [dict(s) for s in st]
            else:
                for a, b in zip(tot, st):
                    for f in COUNT_FIELDS:
                        if f != "round":
                            a[f] = (a[f] + b[f]) & ((1 << 64) - 1)
        for a, b in zip(tot, ref):
            for f in COUNT_FIELDS:
                assert a[f] == b[f], (L, a["round"], f, a[f], b[f])


@pytest.mark.parametrize("jitter", [0, 5])
def test_w64_grid_links_sync(hip_lib, cpu_lib, path, jitter):
    """C5's shape (grid + one long link per node, W = 64) run into the sync
    phase, with late broadcasts and synchronous timers: the W = 64 streamed
    sync kernel against O2."""
    topo = T.grid_links(64, seed=96)
    inj = uniform_injections(4096, 40, 97) + [(n, 40 + v, 26 + v % 5) for n, v, _ in uniform_injections(4096, 24, 98)]
    sc = Scenario(topo, 64, 50, inj, seed=99, sync_base=8, sync_jitter=jitter)
    _compare(sc, hip_lib, cpu_lib, path)
