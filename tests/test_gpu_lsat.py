"""GPU parity of the lean saturation digest (RoundArgs::lsat, W >= 128): a node
whose set already holds every lane injected so far gathers nothing in lean
rounds (expand_stream*, hub_chunks, hub_finish skip its in-edges). Sets only
grow and hold injected lanes only, so the skip is exact while no new lane is
injected; the host clears the digest after every later injection round, and a
client broadcast to a saturated node still takes the full path (its forwards
and marks need its degree). Every scenario injects again after most nodes have
saturated — some of those values at saturated nodes — and must equal O2 bit for
bit with the digest on and off, stepped and through graph-captured episodes;
with it on, the sender-row gathers (work_gathers) must drop. On graphs with
several components (R-MAT) a node's target is the number of lanes injected into
its component (labels computed at install), since no set ever holds a lane
from another component; a value broadcast twice into one component only makes
that component's target unreachable.
"""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.workload import inject
from helpers import Scenario, diff_stats, make_engine

pytestmark = pytest.mark.gpu


def _late(V, first, later, seed):
    """`first` values at round 0, then (value, round) batches `later` at random nodes."""
    rnd = random.Random(seed)
    inj = [(rnd.randrange(V), v, 0) for v in range(first)]
    v = first
    for n, r in later:
        inj += [(rnd.randrange(V), v + k, r) for k in range(n)]
        v += n
    return inj


def _scenarios():
    return [
        ("regular", {}, Scenario(T.random_regular(3000, 6, seed=7), 128, 34,
                                 _late(3000, 64, [(64, 18)], 1), seed=2, enable_sync=False)),
        ("rmat_hubs", {"GG_HUB_DEG": "16", "GG_HUB_CHUNK": "7"},
         Scenario(T.rmat(4096, 16, seed=41), 256, 24,
                  _late(4096, 128, [(100, 9), (28, 10)], 3) + [(7, 3, 2), (4000, 130, 12)],  # values sent twice
                  seed=43, enable_sync=False)),
        ("tree_db", {"GG_DB": "1"}, Scenario(T.tree(6000, 4), 128, 40, _late(6000, 100, [(28, 26)], 5),
                                             seed=6, enable_sync=False)),
        # wide rows: node groups of 8 and 32 lanes (the group sums cross 16-lane rows)
        ("rmat_w1024", {"GG_HUB_DEG": "24", "GG_HUB_CHUNK": "13"},
         Scenario(T.rmat(2048, 16, seed=44), 1024, 20, _late(2048, 900, [(124, 8)], 7), seed=46,
                  enable_sync=False)),
        ("rmat_w4096", {"GG_HUB_DEG": "24", "GG_HUB_CHUNK": "13"},
         Scenario(T.rmat(2048, 16, seed=45), 4096, 16, _late(2048, 4000, [(96, 7)], 8), seed=47,
                  enable_sync=False)),
    ]


@pytest.mark.parametrize("name", ["regular", "rmat_hubs", "tree_db", "rmat_w1024", "rmat_w4096"])
def test_lsat_equals_oracle_with_late_injections(hip_lib, cpu_lib, monkeypatch, name):
    env, sc = next((e, s) for n, e, s in _scenarios() if n == name)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = make_engine(cpu_lib, sc)
    want = c.step(sc.rounds)
    bits, dr = c.read_bits(), c.delivery_rounds()
    c.close()
    gathers = {}
    for lsat in ("0", "1"):
        monkeypatch.setenv("GG_LSAT", lsat)
        g = make_engine(hip_lib, sc, device=0)
        runs = [g.step(sc.rounds)]
        assert np.array_equal(g.read_bits(), bits), (name, lsat)
        assert np.array_equal(g.delivery_rounds(), dr), (name, lsat)
        g.reset()
        inject(g, sc.injections)
        runs += g.run_episodes(sc.rounds, 2)
        for j, st in enumerate(runs):
            d = diff_stats(want, st)
            assert not d, (name, lsat, j, d[:6])
        gathers[lsat] = sum(s["work_gathers"] for s in runs[0])
        g.close()
    assert gathers["1"] < gathers["0"], (name, gathers)
