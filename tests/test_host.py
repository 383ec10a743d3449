"""Host-side inputs: the Maelstrom topology message loader (HandleTopology,
broadcast/broadcast.go:36-48, TopologyMsgBody :18-20) and the builders."""
import json

import numpy as np
import pytest

from ggamd import topology as T


@pytest.mark.parametrize("topo", [T.tree(25, 4), T.tree(1000, 4), T.grid_links(12, seed=3), T.rmat(512, 8, seed=4)])
def test_maelstrom_round_trip(topo):
    body = {"type": "topology", "msg_id": 1, "topology": T.to_maelstrom(topo)}
    for msg in (body, json.dumps(body), json.dumps(body["topology"]).encode()):
        t = T.from_maelstrom(msg)
        assert t.n_nodes == topo.n_nodes
        assert np.array_equal(t.row_ptr, topo.row_ptr) and np.array_equal(t.col, topo.col)


def test_rows_sorted_dedup_missing_rows_empty():
    t = T.from_maelstrom('{"type": "topology", "topology": {"n3": ["n1", "n0", "n1"], "n0": []}, "extra": [1, {"a": "b"}]}')
    assert t.n_nodes == 4
    assert t.rows() == [[], [], [], [0, 1]]  # n1, n2 never listed a row: empty (:41-42)


@pytest.mark.parametrize("bad", ['{"topology": {"x1": []}}', '{"topology": ["n1"]}', '{"n1": ["n0"', "", "[]"])
def test_malformed_topology_rejected(bad):
    with pytest.raises(RuntimeError):
        T.from_maelstrom(bad)


def test_builders_are_symmetric_and_sorted():
    for t in (T.tree(300, 4), T.random_regular(300, 8, seed=5), T.rmat(256, 16, seed=6), T.grid_links(10, seed=7)):
        assert T.is_symmetric(t)
        for v in range(t.n_nodes):
            row = t.col[t.row_ptr[v]:t.row_ptr[v + 1]]
            assert np.all(np.diff(row) > 0) and v not in row
