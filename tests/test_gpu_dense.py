"""GPU parity of dense lean rounds (expand_stream visiting every node) on
rows of 8..32 words against the CPU oracle O2, bit for bit: trees (C2's
shape), random regular and directed graphs, R-MAT in-degrees (hubs kept in
the kernel, and hubs split off with a low GG_HUB_DEG), client broadcasts
landing in dense rounds, and node counts that are not a multiple of 64.
"""
import numpy as np
import pytest

from ggamd import topology as T
from ggamd.engine import Topology
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine

pytestmark = pytest.mark.gpu


def _run(sc, hip_lib, cpu_lib, monkeypatch):
    g = make_engine(hip_lib, sc, device=0)
    c = make_engine(cpu_lib, sc)
    gs = g.step(sc.rounds)
    d = diff_stats(gs, c.step(sc.rounds))
    assert not d, d[:10]
    assert np.array_equal(g.read_bits(), c.read_bits())
    assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())
    assert any(s["work_rows"] == sc.topo.n_nodes for s in gs), "no dense round"


def _inj(V, K, seed, late=0):
    inj = uniform_injections(V, K, seed)
    if late:  # more broadcasts while most nodes are busy (dense rounds)
        inj += [(n, K + v, 6) for n, v, _ in uniform_injections(V, late, seed + 1)]
    return inj


@pytest.mark.parametrize("W", [512, 1024, 2048])
@pytest.mark.parametrize("V", [4096, 5003])
def test_tree(hip_lib, cpu_lib, monkeypatch, W, V):
    sc = Scenario(T.tree(V, 4), W, 30, _inj(V, W // 2, 11, late=W // 4), seed=12, sync_base=40)
    _run(sc, hip_lib, cpu_lib, monkeypatch)


@pytest.mark.parametrize("W", [512, 1024, 2048])
def test_random_regular(hip_lib, cpu_lib, monkeypatch, W):
    V = 3001
    sc = Scenario(T.random_regular(V, 8, seed=13), W, 16, _inj(V, W // 2, 14, late=10), seed=15, sync_base=40)
    _run(sc, hip_lib, cpu_lib, monkeypatch)


@pytest.mark.parametrize("hub_deg", [None, "12"])
def test_rmat_hubs(hip_lib, cpu_lib, monkeypatch, hub_deg):
    """Power-law in-degrees: sets with more than 128 senders (the columns past
    two registers come from memory) or, with a low GG_HUB_DEG, hub nodes that
    the hub kernels take."""
    if hub_deg:
        monkeypatch.setenv("GG_HUB_DEG", hub_deg)
    V = 4096
    sc = Scenario(T.rmat(V, 16, seed=16), 1024, 14, _inj(V, 512, 17, late=40), seed=18, sync_base=40)
    _run(sc, hip_lib, cpu_lib, monkeypatch)


def test_directed(hip_lib, cpu_lib, monkeypatch):
    """Out-degree != in-degree (forward counts use the out-lists)."""
    rng = np.random.default_rng(19)
    V = 2500
    rows = [sorted(set(rng.integers(0, V, size=rng.integers(1, 6)).tolist()) - {v}) for v in range(V)]
    topo = Topology.from_rows(rows)
    sc = Scenario(topo, 1024, 20, _inj(V, 300, 20, late=30), seed=21, sync_base=40)
    _run(sc, hip_lib, cpu_lib, monkeypatch)
