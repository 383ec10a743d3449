"""GPU parity: the HIP engine (libgossip_hip.so, via the C ABI) against the
oracles on identical seeded inputs.

Bit-exact on every round's counters (deliveries, forwards sent/delivered,
pushes, acks, reads, read_oks, drops, sync firings, set hash), every node's
read set and every (node, message) delivery round. Small cases are also
compared with the message-level O1; 4K-node variants of C2..C5 and the full
C2 config are compared with O2, plus size-independent properties (delivery
round = hop distance, total deliveries = V*K on a connected graph).
"""
import random

import numpy as np
import pytest

from ggamd import topology as T
from ggamd.workload import uniform_injections
from helpers import (Scenario, bfs_dist, c1_scenario, diff_stats, make_engine, make_o1,
                     random_scenario)

pytestmark = pytest.mark.gpu


def _compare(sc, hip_lib, ref_lib, full=True):
    g = make_engine(hip_lib, sc, track=full)
    c = make_engine(ref_lib, sc, track=full)
    sg = g.step(sc.rounds)
    scpu = c.step(sc.rounds)
    d = diff_stats(sg, scpu)
    assert not d, d[:10]
    assert np.array_equal(g.read_bits(), c.read_bits())
    if full:
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())
    return sg, g


@pytest.mark.parametrize("seed", range(6))
def test_random_small_vs_o2(hip_lib, cpu_lib, seed):
    rnd = random.Random(7000 + seed)
    for _ in range(10):
        _compare(random_scenario(rnd), hip_lib, cpu_lib)


@pytest.mark.parametrize("W", [64, 128, 192, 256, 512, 1024, 2048, 4096, 8192])
def test_lane_widths(hip_lib, cpu_lib, W):
    """Every (lanes-per-node, words-per-lane) kernel instantiation."""
    rnd = random.Random(W)
    for _ in range(3):
        _compare(random_scenario(rnd, max_v=120, W=W, rounds=40), hip_lib, cpu_lib)


def test_random_small_vs_o1(hip_lib):
    rnd = random.Random(99)
    for _ in range(6):
        sc = random_scenario(rnd)
        o1 = make_o1(sc)
        g = make_engine(hip_lib, sc)
        d = diff_stats(o1.step(sc.rounds), g.step(sc.rounds))
        assert not d, d[:10]
        for v in range(sc.topo.n_nodes):
            assert o1.read(v) == g.read(v)


@pytest.mark.parametrize("partition", [False, True])
def test_c1_vs_o1(hip_lib, partition):
    sc = c1_scenario(partition=partition)
    o1 = make_o1(sc)
    g = make_engine(hip_lib, sc)
    d = diff_stats(o1.step(sc.rounds), g.step(sc.rounds))
    assert not d, d[:10]
    dr = g.delivery_rounds()
    for v in range(25):
        assert o1.read(v) == g.read(v)
        assert o1.delivery_rounds(v) == dr[v].tolist()


def _c_small(name):
    V = 4096
    if name == "C2":
        topo, W, win = T.tree(V, 4), 1024, []
    elif name == "C3":
        topo, W, win = T.random_regular(V, 8, seed=3), 1024, [("seeded", 2, 12, 0x5EED)]
    elif name == "C4":
        topo, W, win = T.rmat(V, 16, seed=4), 4096, []
    else:
        topo, W, win = T.grid_links(64, seed=5), 64, []
    inj = uniform_injections(V, W, seed={"C2": 2, "C3": 3, "C4": 4, "C5": 5}[name])
    return Scenario(topo, W, 60, inj, seed=11, windows=win)


@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_config_4k_vs_o2(hip_lib, cpu_lib, name):
    sg, _ = _compare(_c_small(name), hip_lib, cpu_lib)
    assert sum(s["new_bits"] for s in sg) > 0


def test_c2_full_vs_o2(hip_lib, cpu_lib):
    """Config C2 at full size: 2^20-node tree4, 1024 messages in round 0."""
    V, W = 1 << 20, 1024
    topo = T.tree(V, 4)
    inj = uniform_injections(V, W, seed=0x6A09E667F3BCC909 + 2)
    sc = Scenario(topo, W, 26, inj, seed=0x6A09E667F3BCC909 + 2)
    g = make_engine(hip_lib, sc, track=False)
    c = make_engine(cpu_lib, sc, track=False)
    sg, scpu = g.step(sc.rounds), c.step(sc.rounds)
    d = diff_stats(sg, scpu)
    assert not d, d[:10]
    assert sum(s["new_bits"] for s in sg) == V * W  # connected: everyone gets everything
    assert np.array_equal(g.read_bits(0, 4096), c.read_bits(0, 4096))
    assert np.array_equal(g.read_bits(V - 4096, V), c.read_bits(V - 4096, V))


def test_c2_delivery_round_is_hop_distance(hip_lib):
    """KAT-1 at scale: with sync after propagation and no partitions, the round
    message m reaches v is hop_dist(src_m, v) (size-independent property)."""
    V, W = 1 << 16, 256
    topo = T.tree(V, 4)
    inj = uniform_injections(V, W, seed=77)
    sc = Scenario(topo, W, 40, inj, seed=5)
    g = make_engine(hip_lib, sc, track=True)
    g.step(sc.rounds)
    dr = g.delivery_rounds()
    for k in (0, 1, 17, 100, 255):
        src = inj[k][0]
        assert np.array_equal(dr[:, g.lane_of(k)], bfs_dist(topo, src))


def test_reset_repeatable(hip_lib):
    rnd = random.Random(3)
    sc = random_scenario(rnd, max_v=200, W=256, rounds=40)
    g = make_engine(hip_lib, sc)
    a = g.step(sc.rounds)
    g.reset()
    for n, v, r in sc.injections:
        g.broadcast(n, v, r)
    b = g.step(sc.rounds)
    assert not diff_stats(a, b)


def test_batched_steps_equal_single_steps(hip_lib):
    rnd = random.Random(4)
    sc = random_scenario(rnd, max_v=300, W=512, rounds=45)
    a = make_engine(hip_lib, sc).step(sc.rounds)
    e = make_engine(hip_lib, sc)
    b = [e.step(1)[0] for _ in range(sc.rounds)]
    assert not diff_stats(a, b)


def test_launch_cache_replay_and_invalidation(hip_lib, cpu_lib):
    """Episodes replayed from the captured launch sequence match fresh runs; a
    changed injection set or partition window must not reuse the cache."""
    rnd = random.Random(12)
    sc = random_scenario(rnd, max_v=400, W=256, rounds=30)
    g = make_engine(hip_lib, sc)
    c = make_engine(cpu_lib, sc)
    ref = c.step(sc.rounds)
    assert not diff_stats(ref, g.step(sc.rounds))
    for _ in range(2):  # replays
        g.reset()
        for n, v, r in sc.injections:
            g.broadcast(n, v, r)
        assert not diff_stats(ref, g.step(sc.rounds))
    # different injections -> must recompute
    g.reset()
    c.reset()
    inj2 = [(n, v + 7, r) for n, v, r in sc.injections[::2]]
    for eng in (g, c):
        for n, v, r in inj2:
            eng.broadcast(n, v, r)
    assert not diff_stats(c.step(sc.rounds), g.step(sc.rounds))


@pytest.mark.parametrize("shift", [0, 1])
@pytest.mark.parametrize("extra_quiet", [-1, 0, 1, 2])
def test_reset_after_quiet_rounds(hip_lib, cpu_lib, shift, extra_quiet):
    """gg_reset clears only the F/flag buffers that can be dirty: none after two
    quiet rounds, the round r-1 parity after exactly one (where bench episodes
    end; `shift` moves that round's parity), both mid-propagation (-1). The
    next episode must equal a fresh oracle run."""
    topo = T.tree(4096, 4)
    inj = [(n, v, shift) for n, v, _ in uniform_injections(4096, 256, 91)]
    g = make_engine(hip_lib, Scenario(topo, 256, 40, inj, seed=92, enable_sync=False))
    if extra_quiet < 0:
        g.step(3)
    else:
        r = 0
        while True:  # to the first quiet round after the injections
            r += 1
            if g.step(1)[0]["new_bits"] == 0 and r > shift + 1:
                break
        if extra_quiet:
            g.step(extra_quiet)
    g.reset()
    c = make_engine(cpu_lib, Scenario(topo, 256, 30, [], seed=92, enable_sync=False))
    for n, v, _ in uniform_injections(4096, 200, 93):
        g.broadcast(n, v, 0)
        c.broadcast(n, v, 0)
    d = diff_stats(c.step(30), g.step(30))
    assert not d, d[:5]
    assert np.array_equal(c.read_bits(), g.read_bits())


@pytest.mark.parametrize("shift", [0, 1])
def test_reset_after_quiet_sync_round(hip_lib, cpu_lib, shift):
    """As above with the sync timers running when the episode goes quiet (the
    bench's case: the last delivery rounds are sync rounds, whose F rows and
    flags include LAG rows): gg_reset clears only the flagged rows of the dirty
    buffer; the next episode must equal a fresh oracle run."""
    topo = T.tree(4096, 4)
    inj = [(n, v, 16 + shift) for n, v, _ in uniform_injections(4096, 256, 94)]
    g = make_engine(hip_lib, Scenario(topo, 256, 60, inj, seed=95, enable_sync=True))
    r, st = 0, []
    while True:
        r += 1
        st.append(g.step(1)[0])
        if st[-1]["new_bits"] == 0 and r > 18 + shift:
            break
    assert any(s["syncs_fired"] for s in st), "no timer fired before the quiet round"
    g.reset()
    c = make_engine(cpu_lib, Scenario(topo, 256, 40, [], seed=95, enable_sync=True))
    for n, v, _ in uniform_injections(4096, 200, 96):
        g.broadcast(n, v, 0)
        c.broadcast(n, v, 0)
    d = diff_stats(c.step(40), g.step(40))
    assert not d, d[:5]
    assert np.array_equal(c.read_bits(), g.read_bits())


@pytest.mark.parametrize("seed", range(4))
def test_degree_order_vs_o2(hip_lib, cpu_lib, monkeypatch, seed):
    """GG_ORDER=degree: local rows by descending in-degree (the default on
    power-law graphs). Results must not depend on the row order: random
    directed/symmetric graphs with partitions and sync, and an R-MAT with hubs
    through the device generator (gg_topology_generate's reorder), equal O2."""
    monkeypatch.setenv("GG_ORDER", "degree")
    rnd = random.Random(8100 + seed)
    for _ in range(6):
        _compare(random_scenario(rnd, max_v=200, W=128), hip_lib, cpu_lib)
    monkeypatch.setenv("GG_HUB_DEG", "32")
    topo = T.rmat(3000, 16, seed=seed + 5)
    _compare(Scenario(topo, 256, 30, uniform_injections(3000, 256, seed), seed=seed, sync_base=12,
                      sync_jitter=3, windows=[("seeded", 14, 18, 3)]), hip_lib, cpu_lib)


def test_degree_order_device_generated(hip_lib, cpu_lib, monkeypatch):
    """The device reorder of a generated R-MAT equals the host path (and O2),
    and gg_topology_export maps the rows back to the generator's CSR."""
    from ggamd.engine import Engine
    monkeypatch.setenv("GG_HUB_DEG", "48")
    monkeypatch.setenv("GG_ORDER", "degree")
    V, W = 5000, 256
    topo = T.rmat(V, 16, seed=33)
    inj = uniform_injections(V, 200, 4)
    out = []
    for lib, gen in ((hip_lib, True), (cpu_lib, False)):
        e = Engine(V, W, seed=2, sync_base=10, sync_jitter=4, library=lib, track_delivery=True)
        if gen:
            e.generate("rmat", V, k=16, seed=33, a=0.57, b=0.19, c=0.19)
            ex = e.export_topology()
            assert np.array_equal(ex.row_ptr, topo.row_ptr) and np.array_equal(ex.col, topo.col)
        else:
            e.topology(topo)
        for n, v, r in inj:
            e.broadcast(n, v, r)
        out.append((e.step(25), e.read_bits(), e.delivery_rounds()))
    assert not diff_stats(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("seed", range(4))
def test_edge_windows_vs_o2(hip_lib, cpu_lib, seed):
    """gg_set_partition: per-edge windows (overriding overlapping group windows)
    on random symmetric graphs, every lane width class; the masked streaming
    kernel (lean rounds) and the tile kernel (sync rounds) both read the bits."""
    from helpers import symmetric_random_scenario
    rnd = random.Random(9100 + seed)
    for W in (64, 128, 1024):
        sc = symmetric_random_scenario(rnd, max_v=150, W=W, rounds=45)
        _compare(sc, hip_lib, cpu_lib)


def test_edge_window_c3_shape_vs_o2(hip_lib, cpu_lib):
    """A 4K-node random 8-regular graph (C3's shape) with a seeded bisection and
    an overlapping per-edge window that cuts 30% of the links, sync on."""
    from helpers import symmetric_cut
    topo = T.random_regular(4096, 8, seed=3)
    bits = symmetric_cut(topo, random.Random(4), 0.3)
    sc = Scenario(topo, 1024, 40, uniform_injections(4096, 1024, 3), seed=3, sync_base=8, sync_jitter=4,
                  windows=[("seeded", 2, 12, 7), ("edges", 6, 16, bits)])
    st, _ = _compare(sc, hip_lib, cpu_lib)
    assert sum(s["dropped"] for s in st[12:16]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("no_db", [False, True])
@pytest.mark.parametrize("seed", range(3))
def test_lean_rounds_both_kernels_vs_o2(hip_lib, cpu_lib, monkeypatch, seed, no_db):
    """Lean episodes (no sync, no windows) with client broadcasts spread over
    rounds, through the double-buffered kernel (senders' sets of
    r-1, no F rows) and, with GG_NO_DB, through the F-row kernel; then sync
    rounds after the double-buffered ones (materialize_F hands over), against
    O2 per round, with sets and delivery rounds."""
    if no_db:
        monkeypatch.setenv("GG_NO_DB", "1")
    rnd = random.Random(900 + seed)
    for k in range(4):
        sc = random_scenario(rnd, max_v=300, W=rnd.choice([128, 256, 1024]), rounds=40)
        sc.windows = []
        sc.enable_sync = k % 2 == 1
        sc.sync_base = rnd.randrange(3, 12)
        sc.injections = [(n, v, rnd.randrange(0, 10)) for n, v, _ in sc.injections]
        g, c = make_engine(hip_lib, sc), make_engine(cpu_lib, sc)
        d = diff_stats(g.step(sc.rounds), c.step(sc.rounds))
        assert not d, (seed, k, d[:10])
        assert np.array_equal(g.read_bits(), c.read_bits())
        assert np.array_equal(g.delivery_rounds(), c.delivery_rounds())
        # a second episode on the same engines (reset after double-buffered rounds)
        g.reset()
        c.reset()
        for n, v, r in sc.injections:
            g.broadcast(n, v, r)
            c.broadcast(n, v, r)
        d = diff_stats(g.step(sc.rounds), c.step(sc.rounds))
        assert not d, (seed, k, "episode 2", d[:10])
        assert np.array_equal(g.read_bits(), c.read_bits())


@pytest.mark.gpu
@pytest.mark.parametrize("W", [64, 128])
def test_saturated_node_learns_client_broadcast(hip_lib, cpu_lib, W):
    """A node whose set already holds every value broadcast so far skips its
    gathers (expand_stream1, W = 64); a client broadcast of a new value at it
    must still be forwarded to every neighbour (regression: the forward count
    used the skipped in-degree)."""
    for V in (2, 5, 40):
        topo = T.tree(V, 4)
        inj = [(0, 11, 0), (V - 1, 12, 0), (0, 13, 9), (V - 1, 14, 9), (V // 2, 15, 12), (0, 11, 14)]
        sc = Scenario(topo, W, 24, inj, seed=5, enable_sync=False)
        _compare(sc, hip_lib, cpu_lib)


@pytest.mark.parametrize("knobs", ["split", "prep16", "both"])
def test_large_graph_paths_vs_o2(hip_lib, cpu_lib, monkeypatch, knobs):
    """Paths the engine takes by size, forced on 4K-10K-node graphs against O2
    per round: split compaction (GG_COMPACT_SPLIT; by default above 8M nodes:
    per-block counts, offsets, then the list) and round_prep's sparse scan over
    16 nodes per thread (GG_PREP_BLOCKS=1: the capped grid covers fewer than a
    quarter of the nodes, as at 2^26). The C5 shape at W = 64 also takes the
    flags-first gathers of expand_stream1 in its sparse rounds (checked from the
    gather counts); the C2 and C4 shapes the double-buffered and hub kernels;
    lean and with sync timers."""
    if knobs in ("split", "both"):
        monkeypatch.setenv("GG_COMPACT_SPLIT", "1")
    if knobs in ("prep16", "both"):
        monkeypatch.setenv("GG_PREP_BLOCKS", "1")
    cases = [
        (T.grid_links(64, seed=5), 64, False),
        (T.grid_links(100, seed=6), 64, True),
        (T.tree(8192, 4), 1024, False),
        (T.rmat(4096, 16, seed=4), 512, True),
    ]
    for k, (topo, W, sync) in enumerate(cases):
        V = topo.n_nodes
        inj = [(n, v, (3 * v) % 7) for n, v, _ in uniform_injections(V, W, seed=20 + k)]
        sc = Scenario(topo, W, 36, inj, seed=13 + k, sync_base=9, enable_sync=sync)
        sg, _ = _compare(sc, hip_lib, cpu_lib)
        assert sum(s["new_bits"] for s in sg) > 0
        if W == 64:  # flags-first: only senders active in r-1 are gathered (>= 4 in-edges per node)
            assert any(0 < s["work_gathers"] < 2 * s["work_rows"] for s in sg[1:10]), \
                [(s["work_gathers"], s["work_rows"]) for s in sg[:10]]


def test_fresh_injections_replay_vs_o2(hip_lib, cpu_lib):
    """Episodes with fresh injection sets in the same rounds (same lanes per
    round) replay the captured launch sequence, which reads the pairs and each
    round's share from device memory: every episode equals O2, including one
    whose rounds inject different numbers of pairs and one with a round's
    pairs moved to another round."""
    rnd = random.Random(31)
    base = random_scenario(rnd, max_v=500, W=256, rounds=30)
    base.windows = []
    V = base.topo.n_nodes
    g = make_engine(hip_lib, base)
    g.step(base.rounds)
    for ep in range(5):
        rr = random.Random(100 + ep)
        if ep < 3:  # same rounds, same count per round, fresh nodes
            inj = [(rr.randrange(V), v, r) for _, v, r in base.injections]
        elif ep == 3:  # same rounds, other counts per round
            inj = [(rr.randrange(V), v, r) for _, v, r in base.injections for _ in range(rr.randrange(1, 3))]
        else:  # other rounds
            inj = [(rr.randrange(V), v, (r + 1) % 6) for _, v, r in base.injections]
        c = make_engine(cpu_lib, base)
        c.reset()
        g.reset()
        for eng in (g, c):
            for n, v, r in inj:
                eng.broadcast(n, v, r)
        d = diff_stats(c.step(base.rounds), g.step(base.rounds))
        assert not d, (ep, d[:10])
        assert np.array_equal(g.read_bits(), c.read_bits())
