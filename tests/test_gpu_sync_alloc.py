"""Streamed-sync buffers allocated lazily (engine.hip alloc_sync / ensure_sync):
the sync records, sender states, digest, reverse edge index and push bytes
exist only once a round that can reach a sync timer (round >= sync_base,
`broadcast/main.go:42-51`) has been enqueued. Where in the episode that
happens must not change any result, so one sync-on scenario runs

  * as one multi-round step (buffers allocated before round 0),
  * as single steps (allocated at round sync_base),
  * as irregular steps that cross sync_base mid-batch,
  * on an engine reused after gg_reset (buffers left from the last episode),
  * on a fresh engine with GG_SYNC_EAGER=1 (allocated with the topology),
  * sharded over 3 ranks (allocated in gg_dist_round_begin at round sync_base),

and every run must equal the CPU oracle O2 in every round's counters, the
final node sets and every delivery round.

The cause of round 3's divergence (single steps and sharded rounds differed
once sync rounds began): the lane history (lanes_through: lanes injected in
rounds <= r, which the saturation digest, the all-full test and expand_stream1's
saturation skip compare set sizes with) was extended lazily from each round's
injection list, and the list was dropped when its round ended. An engine with
the digest asked for round r's count while r ran; without it (before the
buffers existed, or with sync off) only r-1's was asked for, so round r's lanes
were missing once its list was gone and the counts fell short: nodes that
lacked lanes passed for saturated. Now a round's list is dropped only after the
history covers it (engine.hip retire_round).
"""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.engine import Topology
from ggamd.workload import uniform_injections
from helpers import Scenario, diff_stats, make_engine

pytestmark = pytest.mark.gpu


def _scenarios():
    out = []
    # tree (C2's shape): sparse sync rounds, pushes on the few edges that lag
    out.append(Scenario(T.tree(3000, 4), 256, 40,
                        uniform_injections(3000, 200, 5) + [(n, 200 + v, 14) for n, v, _ in
                                                            uniform_injections(3000, 30, 6)],
                        seed=9, sync_base=6, sync_jitter=3))
    # synchronous timers: every in-edge pushes, more than three contributing senders
    out.append(Scenario(T.random_regular(2048, 12, seed=77), 512, 30,
                        [(n, v, 1 + v % 9) for n, v, _ in uniform_injections(2048, 400, 78)],
                        seed=79, sync_base=4, sync_jitter=0))
    # W = 64 grid + long links (C5's shape), late broadcasts during sync
    out.append(Scenario(T.grid_links(48, seed=11), 64, 36,
                        uniform_injections(48 * 48, 40, 6) + [(n, 40 + v, 12 + v % 4) for n, v, _ in
                                                              uniform_injections(48 * 48, 20, 7)],
                        seed=10, sync_base=8, sync_jitter=4))
    # directed random graph (out-lists != in-lists)
    rnd = random.Random(31)
    V = 700
    rows = [set() for _ in range(V)]
    for _ in range(4 * V):
        a, b = rnd.randrange(V), rnd.randrange(V)
        if a != b:
            rows[a].add(b)
            if rnd.random() < 0.7:
                rows[b].add(a)
    topo = Topology.from_rows([sorted(r) for r in rows])
    out.append(Scenario(topo, 128, 34, [(rnd.randrange(V), v, rnd.randrange(12)) for v in range(100)],
                        seed=12, sync_base=5, sync_jitter=2))
    return out


def _check(sc, stats, eng, ref_stats, ref, what):
    d = diff_stats(ref_stats, stats)
    assert not d, (what, d[:8])
    assert np.array_equal(eng.read_bits(), ref.read_bits()), what
    assert np.array_equal(eng.delivery_rounds(), ref.delivery_rounds()), what


@pytest.mark.parametrize("k", range(4))
def test_lazy_sync_buffers_step_granularity(hip_lib, cpu_lib, monkeypatch, k):
    sc = _scenarios()[k]
    monkeypatch.setenv("GG_SYNC_TILES", "0")
    ref = make_engine(cpu_lib, sc)
    want = ref.step(sc.rounds)

    whole = make_engine(hip_lib, sc, device=0)
    assert whole.device_bytes()["sync"] == 0, "sync buffers before any round"
    _check(sc, whole.step(sc.rounds), whole, want, ref, "one step")
    assert whole.device_bytes()["sync"] > 0

    single = make_engine(hip_lib, sc, device=0)
    st = []
    for r in range(sc.rounds):
        st += single.step(1)
        # allocated exactly when the first round >= sync_base is enqueued
        assert (single.device_bytes()["sync"] > 0) == (r >= sc.sync_base), r
    _check(sc, st, single, want, ref, "single steps")

    rnd = random.Random(k)
    irr = make_engine(hip_lib, sc, device=0)
    st, r = [], 0
    while r < sc.rounds:
        n = min(sc.rounds - r, rnd.randrange(1, 7))
        st += irr.step(n)
        r += n
    _check(sc, st, irr, want, ref, "irregular steps")

    # reused after gg_reset: the buffers hold the last episode's records, pushes, digest
    whole.reset()
    for n, v, rr in sc.injections:
        whole.broadcast(int(n), int(v), int(rr))
    st = []
    for r in range(sc.rounds):
        st += whole.step(1)
    _check(sc, st, whole, want, ref, "after reset, single steps")

    monkeypatch.setenv("GG_SYNC_EAGER", "1")
    eager = make_engine(hip_lib, sc, device=0)
    assert eager.device_bytes()["sync"] > 0
    st = []
    for r in range(sc.rounds):
        st += eager.step(1)
    _check(sc, st, eager, want, ref, "eager allocation, single steps")
    for e in (whole, single, irr, eager, ref):
        e.close()


def test_lazy_sync_buffers_sharded(hip_lib, cpu_lib, monkeypatch):
    """3 ranks on one GPU (gloo): every rank allocates its sync buffers at round
    sync_base inside gg_dist_round_begin; summed counters, node sets and delivery
    rounds equal O2."""
    from test_gpu_dist import _run
    scs = _scenarios()
    res = _run(hip_lib, scs, 3, env={"GG_SYNC_TILES": "0"})
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        for rank in range(3):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(want, stats)
            assert not d, (k, rank, d[:8])
            assert np.array_equal(bits, ref.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, ref.delivery_rounds_nodes(owned)), (k, rank)
        ref.close()


@pytest.mark.parametrize("sync", [False, True])
def test_single_steps_injections_every_round(hip_lib, cpu_lib, sync):
    """Client broadcasts in most rounds, run one round per gg_step, W = 64 (the
    saturation skip of expand_stream1) and W = 256 (the all-full test): with
    sync off there is no digest at all, and before the fix the lane counts of
    every round with injections were lost once the round ended."""
    for W, topo in ((64, T.grid_links(40, seed=3)), (256, T.random_regular(1600, 6, seed=4))):
        V = topo.n_nodes
        rnd = random.Random(W)
        inj = [(rnd.randrange(V), v, rnd.randrange(24)) for v in range(W - 3)]
        sc = Scenario(topo, W, 40, inj, seed=21, sync_base=5, sync_jitter=3, enable_sync=sync)
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        e = make_engine(hip_lib, sc, device=0)
        st = [e.step(1)[0] for _ in range(sc.rounds)]
        _check(sc, st, e, want, ref, f"W={W} sync={sync}")
        e.close()
        ref.close()


def test_no_sync_buffers_before_timers(hip_lib):
    """An episode that ends before the first timer (the C4/C5 benchmarks) never
    allocates them; a later step that reaches the timers does."""
    sc = Scenario(T.tree(4096, 4), 128, 10, uniform_injections(4096, 100, 3), seed=4, sync_base=20)
    e = make_engine(hip_lib, sc, device=0)
    e.step(15)
    b = e.device_bytes()
    assert b["sync"] == 0 and b["total"] > 0, b
    e.reset()
    e.step(19)
    assert e.device_bytes()["sync"] == 0
    e.step(1)  # round 19 < 20 still
    assert e.device_bytes()["sync"] == 0
    e.step(1)  # round 20: a timer can fire
    assert e.device_bytes()["sync"] > 0
    e.close()
