"""gg_run_episodes (gossip.h): `episodes` x (gg_reset; the same client
broadcasts; gg_step(n_rounds)) with one host wait. Its result must equal that
loop on the same engine and on the oracle: every round's counters of every
episode, and the sets (and delivery rounds) the last episode leaves."""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.engine import GGError
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine, random_scenario, symmetric_random_scenario


def _loop(eng, sc, episodes):
    out = []
    for k in range(episodes):
        if k:
            eng.reset()
            for n, v, r in sc.injections:
                eng.broadcast(int(n), int(v), int(r))
        out.append(eng.step(sc.rounds))
    return out


def _check(lib_a, lib_b, sc, episodes, track=True):
    """lib_a's run_episodes against lib_b's reset/broadcast/step loop."""
    a = make_engine(lib_a, sc, track=track)
    b = make_engine(lib_b, sc, track=track)
    ea = a.run_episodes(sc.rounds, episodes)
    eb = _loop(b, sc, episodes)
    assert len(ea) == episodes
    for k in range(episodes):
        d = diff_stats(ea[k], eb[k])
        assert not d, (k, d[:10])
    assert a.round == b.round == sc.rounds
    assert np.array_equal(a.read_bits(), b.read_bits())
    if track:
        assert np.array_equal(a.delivery_rounds(), b.delivery_rounds())
    return a, b, ea


def test_o2_episodes_equal_loop(cpu_lib):
    rnd = random.Random(41)
    for _ in range(4):
        _check(cpu_lib, cpu_lib, random_scenario(rnd, max_v=60, rounds=45), 3)


def test_episodes_refuse_bad_calls(cpu_lib):
    sc = random_scenario(random.Random(5), max_v=30, rounds=10)
    e = make_engine(cpu_lib, sc)
    with pytest.raises(GGError):
        e.run_episodes(0, 2)
    with pytest.raises(GGError):
        e.run_episodes(257, 1)
    e.step(1)
    with pytest.raises(GGError):  # not at round 0
        e.run_episodes(5, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_episodes_random_vs_o2(hip_lib, cpu_lib, seed):
    rnd = random.Random(8100 + seed)
    for _ in range(4):
        _check(hip_lib, cpu_lib, random_scenario(rnd, rounds=50), 3)
    # per-edge windows (the masked kernels) and symmetric graphs
    for _ in range(2):
        _check(hip_lib, cpu_lib, symmetric_random_scenario(rnd, rounds=40), 3)


@pytest.mark.gpu
def test_episodes_hip_equal_hip_loop(hip_lib):
    """The one-wait sequence replays exactly what the synchronous calls do."""
    sc = random_scenario(random.Random(17), max_v=200, W=256, rounds=60)
    _check(hip_lib, hip_lib, sc, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_episodes_configs_4k_vs_o2(hip_lib, cpu_lib, name):
    V = 4096
    topo, W, win = {
        "C2": (T.tree(V, 4), 1024, []),
        "C3": (T.random_regular(V, 8, seed=3), 1024, [("seeded", 2, 12, 0x5EED)]),
        "C4": (T.rmat(V, 16, seed=4), 4096, []),
        "C5": (T.grid_links(64, seed=5), 64, []),
    }[name]
    inj = uniform_injections(V, W, seed={"C2": 2, "C3": 3, "C4": 4, "C5": 5}[name])
    sc = Scenario(topo, W, 40, inj, seed=11, windows=win)
    a, _, ea = _check(hip_lib, cpu_lib, sc, 3, track=False)
    assert sum(s["new_bits"] for s in ea[-1]) > 0
    assert a.step_device_ms() > 0.0


@pytest.mark.gpu
def test_episodes_c2_full_size_vs_o2(hip_lib, cpu_lib):
    """The bench's workload: 2^20-node tree4, 1024 messages in round 0, 22 rounds."""
    V, W = 1 << 20, 1024
    inj = uniform_injections(V, W, seed=0x6A09E667F3BCC909 + 2)
    sc = Scenario(T.tree(V, 4), W, 22, inj, seed=0x6A09E667F3BCC909 + 2)
    a = make_engine(hip_lib, sc, track=False)
    c = make_engine(cpu_lib, sc, track=False)
    ea = a.run_episodes(sc.rounds, 4)
    sc_ = c.step(sc.rounds)
    for k in range(4):
        d = diff_stats(ea[k], sc_)
        assert not d, (k, d[:10])
    assert sum(s["new_bits"] for s in ea[-1]) == V * W
    assert np.array_equal(a.read_bits(0, 4096), c.read_bits(0, 4096))
    # and a synchronous step after it starts from the right state
    a.reset()
    c.reset()
    for n, v, r in inj[:7]:
        a.broadcast(int(n), int(v), int(r))
        c.broadcast(int(n), int(v), int(r))
    d = diff_stats(a.step(30), c.step(30))
    assert not d, d[:10]
