"""GPU parity of the hub path (power-law graphs): nodes with in-degree above the
hub threshold skip the streaming kernel and take hub_chunks + hub_finish (the
ordered (union, first-claimer-reciprocal) scan over in-edge chunks); senders
with out-degree above it are marked by hub_mark. GG_HUB_DEG / GG_HUB_CHUNK
lower the threshold and the chunk size so small graphs exercise many hubs,
multi-chunk scans and chunk boundaries; results must equal the CPU oracle O2
bit for bit (counters of every round, node sets, delivery rounds).
"""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine, random_scenario

pytestmark = pytest.mark.gpu


def _compare(sc, hip_lib, cpu_lib):
    g = make_engine(hip_lib, sc, device=0)
    c = make_engine(cpu_lib, sc)
    d = diff_stats(g.step(sc.rounds), c.step(sc.rounds))
    assert not d, d[:10]
    assert np.array_equal(g.read_bits(), c.read_bits())
    assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())


@pytest.mark.parametrize("deg,chunk", [(16, 7), (40, 1), (8, 1000)])
def test_rmat_hubs(hip_lib, cpu_lib, monkeypatch, deg, chunk):
    monkeypatch.setenv("GG_HUB_DEG", str(deg))
    monkeypatch.setenv("GG_HUB_CHUNK", str(chunk))
    topo = T.rmat(4096, 16, seed=41)
    assert int(np.diff(topo.row_ptr).max()) > 4 * deg  # real hubs
    sc = Scenario(topo, 256, 14, uniform_injections(4096, 256, 42), seed=43, sync_base=9, sync_jitter=2)
    _compare(sc, hip_lib, cpu_lib)


def test_rmat_hubs_wide_rows(hip_lib, cpu_lib, monkeypatch):
    """W = 4096 (C4's lane count): 32 lanes per row in every hub kernel."""
    monkeypatch.setenv("GG_HUB_DEG", "24")
    monkeypatch.setenv("GG_HUB_CHUNK", "13")
    topo = T.rmat(2048, 16, seed=44)
    sc = Scenario(topo, 4096, 10, uniform_injections(2048, 4000, 45), seed=46, enable_sync=False)
    _compare(sc, hip_lib, cpu_lib)


def test_random_with_hub_threshold(hip_lib, cpu_lib, monkeypatch):
    """Directed graphs, partitions, sync: hubs only in lean rounds, the tile
    path everywhere else."""
    monkeypatch.setenv("GG_HUB_DEG", "3")
    monkeypatch.setenv("GG_HUB_CHUNK", "2")
    rnd = random.Random(4242)
    for _ in range(8):
        _compare(random_scenario(rnd, max_v=200, W=128, rounds=45), hip_lib, cpu_lib)


@pytest.mark.parametrize("deg", ["3", "1000000000"])
def test_partition_then_lean_rounds(hip_lib, cpu_lib, monkeypatch, deg):
    """Partition windows without sync: masked (tile-path) rounds hand over to
    streaming rounds, which gather every sender row — so a candidate whose
    senders were all dropped must still clear its stale F row (regression)."""
    monkeypatch.setenv("GG_HUB_DEG", deg)
    monkeypatch.setenv("GG_HUB_CHUNK", "2")
    rnd = random.Random(4242)
    for _ in range(8):
        sc = random_scenario(rnd, max_v=200, W=128, rounds=45)
        sc.enable_sync = False
        _compare(sc, hip_lib, cpu_lib)


@pytest.mark.parametrize("W", [128, 1024, 4096])
def test_masked_streaming_rounds(hip_lib, cpu_lib, monkeypatch, W):
    """Symmetric graphs without hubs stream through partition windows too
    (expand_stream_masked: per-window in-edge bitmaps for drops, delivered
    forwards and dropped acks) — seeded and explicit windows, back to back."""
    monkeypatch.setenv("GG_HUB_DEG", "1000000000")
    rnd = random.Random(W)
    for _ in range(6):
        sc = random_scenario(rnd, max_v=300, W=W, rounds=40, directed_p=0.0)
        sc.enable_sync = False
        sc.windows = [("seeded", 2, 6, rnd.randrange(1 << 30)), ("seeded", 6, 9, rnd.randrange(1 << 30)),
                      ("groups", 12, 20, np.array([rnd.randrange(3) for _ in range(sc.topo.n_nodes)], np.uint8))]
        _compare(sc, hip_lib, cpu_lib)


@pytest.mark.parametrize("W,deg,chunk", [(256, 16, 7), (64, 24, 5), (4096, 40, 1000), (1024, 8, 3)])
def test_rmat_hubs_sync_rounds(hip_lib, cpu_lib, monkeypatch, W, deg, chunk):
    """Sync rounds on a power-law graph with hubs (streamed: hub_sync_chunks /
    hub_sync_finish / hub_sync_push beside sync_records + expand_stream_sync):
    hubs receive pushes, answer reads, run callbacks over many chunks (the
    exclusive prefix across chunks), late client broadcasts reach them, and
    every round equals O2; the tile kernel never runs in those rounds."""
    monkeypatch.setenv("GG_HUB_DEG", str(deg))
    monkeypatch.setenv("GG_HUB_CHUNK", str(chunk))
    monkeypatch.setenv("GG_SYNC_TILES", "0")
    topo = T.rmat(4096, 16, seed=47)
    assert int(np.diff(topo.row_ptr).max()) > 4 * deg
    K = min(W, 200)
    inj = uniform_injections(4096, K // 2, 48) + [(n, K // 2 + v, 9 + v % 7) for n, v, _ in
                                                   uniform_injections(4096, K - K // 2, 49)]
    sc = Scenario(topo, W, 36, inj, seed=50, sync_base=3, sync_jitter=2)
    g = make_engine(hip_lib, sc, device=0)
    c = make_engine(cpu_lib, sc)
    gs = g.step(sc.rounds)
    d = diff_stats(gs, c.step(sc.rounds))
    assert not d, d[:10]
    assert np.array_equal(g.read_bits(), c.read_bits())
    assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())
    sync = [s for s in gs if s["round"] >= sc.sync_base + 2]
    assert sum(s["pushes"] for s in sync) > 0 and sum(s["syncs_fired"] for s in gs) > 0
    assert all(s["expand_bytes"] == 0 for s in sync), [s["expand_bytes"] for s in sync]
