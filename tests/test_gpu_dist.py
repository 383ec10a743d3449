"""Sharded HIP engine on the GPU: world_size 2 and 3, every rank an engine on
the same MI355X (cuda:0), ghost payloads moved by ggamd.dist.ShardedRunner over
gloo (staged through host memory; the multi-GPU runs use RCCL on the same
buffers and stream). Counters summed over ranks, and the node sets and delivery
rounds of every rank's owned nodes, must equal one unsharded HIP engine — which
the other GPU tests pin to the CPU oracle.

Scenarios cover both partition orders (a tree: DFS preorder wins; a grid and
random graphs: native order), directed edges, sync timers, seeded and explicit
partition windows, and the dense (stream) and sparse paths.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import Scenario, c1_scenario, diff_stats, make_engine, random_scenario

pytestmark = pytest.mark.gpu


def _free_port():
    from helpers import free_port
    return free_port()


def _worker(rank, world, port, lib, scenarios, q, lane_groups=1, env=None, generate=False, transport=None,
            kw=None):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    os.environ.update(env or {})
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        for sc in scenarios:
            e = make_engine(lib, sc, rank=rank, world=world, device=0, lane_groups=lane_groups, generate=generate,
                            **(kw or {}))
            r = ShardedRunner(e, dev, transport=transport)
            if transport == "engine" and e.parts > 1:  # gg_dist_step's own sequencing, over gloo
                assert r.host_xport is not None, r.transport
            half = sc.rounds // 2
            stats = r.step(half) + r.step(sc.rounds - half)  # two flushes
            if r.host_xport is not None:
                assert r.host_xport.groups >= sc.rounds, r.host_xport.groups  # one group per round at least
            owned = e.dist_owned()
            out.append((stats, owned, e.read_bits_nodes(owned), e.delivery_rounds_nodes(owned)))
            r.close()  # collective (IPC): every rank leaves the exchange before any engine is destroyed
            e.close()
        q.put((rank, out))
    except BaseException as exc:  # report instead of leaving the parent waiting
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


def _run(lib, scenarios, world, lane_groups=1, env=None, generate=False, transport=None, timeout=150, kw=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, lib, scenarios, q, lane_groups, env, generate,
                                               transport, kw))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = q.get(timeout=timeout)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [res[r] for r in range(world)]


def _scenarios():
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    rnd = random.Random(7)
    out = [random_scenario(random.Random(s), max_v=300, W=128, rounds=50) for s in (3, 4)]
    tree = T.tree(3000, 4)
    out.append(Scenario(tree, 256, 40, uniform_injections(3000, 200, 5), seed=9, sync_base=6,
                        sync_jitter=3, windows=[("seeded", 3, 9, 77)]))
    grid = T.grid_links(48, seed=11)
    out.append(Scenario(grid, 64, 45, uniform_injections(48 * 48, 64, 6), seed=10, sync_base=8,
                        sync_jitter=4))
    rr = T.random_regular(4000, 8, seed=12)
    out.append(Scenario(rr, 1024, 30, uniform_injections(4000, 1000, 7), seed=12, sync_base=10,
                        sync_jitter=5, windows=[("seeded", 2, 7, 5)]))
    out.append(c1_scenario(partition=True, rounds=120))
    from helpers import symmetric_cut
    grid2 = T.grid_links(40, seed=13)
    out.append(Scenario(grid2, 128, 40, uniform_injections(1600, 100, 8), seed=11, sync_base=7, sync_jitter=3,
                        windows=[("seeded", 3, 9, 5), ("edges", 5, 14, symmetric_cut(grid2, rnd, 0.3))]))
    del rnd
    return out


@pytest.mark.parametrize("world,mode", [(2, "static"), (3, "static"), (2, "exact"), (3, "exact")])
def test_sharded_equals_single(hip_lib, world, mode):
    """GG_XCHG_MODE: every exchange direction with static sizes (segment
    capacities) or exact sizes (sizes first, then only the used bytes)."""
    scs = _scenarios()
    res = _run(hip_lib, scs, world, env={"GG_XCHG_MODE": mode})
    for k, sc in enumerate(scs):
        single = make_engine(hip_lib, sc, device=0)
        s1 = single.step(sc.rounds)
        owned_all = []
        for rank in range(world):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(s1, stats)
            assert not d, (k, rank, d[:10])
            assert np.array_equal(bits, single.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, single.delivery_rounds_nodes(owned)), (k, rank)
            owned_all.append(owned)
        allown = np.sort(np.concatenate(owned_all))
        assert np.array_equal(allown, np.arange(sc.topo.n_nodes)), k
        single.close()


def _rmat_scenarios():
    """R-MAT graphs with hubs: with GG_HUB_DEG=24 the high in-degree nodes take
    hub_chunks/hub_finish and the high out-degree senders hub_mark, now with ghost
    senders in their in-lists and ghost receivers in their out-lists."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    rm = T.rmat(4096, 16, seed=21)
    rm2 = T.rmat(3000, 8, seed=22)
    return [Scenario(rm, 256, 24, uniform_injections(4096, 256, 8), seed=13, sync_base=30, sync_jitter=3),
            Scenario(rm2, 128, 40, uniform_injections(3000, 100, 9), seed=14, sync_base=8, sync_jitter=4)]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_rmat_hubs_equals_single(hip_lib, world):
    env = {"GG_HUB_DEG": "24", "GG_XCHG_MODE": "exact"}
    scs = _rmat_scenarios()
    res = _run(hip_lib, scs, world, env=env)
    old = os.environ.get("GG_HUB_DEG")
    os.environ.update(env)
    try:
        for k, sc in enumerate(scs):
            single = make_engine(hip_lib, sc, device=0)
            s1 = single.step(sc.rounds)
            for rank in range(world):
                stats, owned, bits, dr = res[rank][k]
                d = diff_stats(s1, stats)
                assert not d, (k, rank, d[:10])
                assert np.array_equal(bits, single.read_bits_nodes(owned)), (k, rank)
                assert np.array_equal(dr, single.delivery_rounds_nodes(owned)), (k, rank)
            single.close()
    finally:
        if old is None:
            os.environ.pop("GG_HUB_DEG", None)
        else:
            os.environ["GG_HUB_DEG"] = old


@pytest.mark.parametrize("world,groups", [(2, 2), (4, 2), (3, 3)])
def test_lane_groups_equal_single(hip_lib, world, groups):
    """2-D sharding on the GPU (gg_config.lane_groups): lane groups x vertex
    parts. Counters summed over all ranks equal one engine; node sets OR-ed and
    delivery rounds max-ed over a node's owners equal its set and rounds."""
    scs = [sc for sc in _scenarios() + _rmat_scenarios()[:1] if sc.W // 64 >= groups][:4]
    assert len(scs) >= 2
    res = _run(hip_lib, scs, world, lane_groups=groups, env={"GG_HUB_DEG": "24"})
    old = os.environ.get("GG_HUB_DEG")
    os.environ["GG_HUB_DEG"] = "24"
    try:
        for k, sc in enumerate(scs):
            single = make_engine(hip_lib, sc, device=0)
            s1 = single.step(sc.rounds)
            V = sc.topo.n_nodes
            bits = np.zeros((V, sc.W // 64), np.uint64)
            dr = np.full((V, sc.W), -1, np.int32)
            for rank in range(world):
                stats, owned, b, d = res[rank][k]
                assert not diff_stats(s1, stats), (k, rank, diff_stats(s1, stats)[:10])
                o = owned.astype(np.int64)
                bits[o] |= b
                dr[o] = np.maximum(dr[o], d)
            assert np.array_equal(bits, single.read_bits()), k
            assert np.array_equal(dr, single.delivery_rounds()), k
            single.close()
    finally:
        if old is None:
            os.environ.pop("GG_HUB_DEG", None)
        else:
            os.environ["GG_HUB_DEG"] = old


@pytest.mark.parametrize("kind", ["tree", "random_regular"])
def test_exchange_payload_follows_activity(hip_lib, kind):
    """Only first receipts cross (broadcast.go:55,64-76): a rank's payload bytes
    per round are positive while its boundary nodes learn values and exactly 0
    once the network is quiet (no sync: no sets are ever read)."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    V = 3000 if kind == "tree" else 4000
    topo = T.tree(V, 4) if kind == "tree" else T.random_regular(V, 8, seed=12)
    sc = Scenario(topo, 256, 40, uniform_injections(V, 200, 5), seed=9, enable_sync=False)
    res = _run(hip_lib, [sc], 2, env={"GG_XCHG_MODE": "exact"})
    single = make_engine(hip_lib, sc, device=0)
    s1 = single.step(sc.rounds)
    last = max(i for i, s in enumerate(s1) if s["new_bits"])
    for rank in range(2):
        stats = res[rank][0][0]
        assert not diff_stats(s1, stats)
        sent = [s["sent_bytes"] for s in stats]
        assert all(b == 0 for b in sent[last + 1:]), sent
        assert sum(sent[:last + 1]) > 0, sent
    single.close()


def test_lane_group_engine_steps_without_exchange(hip_lib):
    """lane_groups == world: no vertex parts, so every rank steps on its own
    (gg_step, graph-captured batches) and the summed counters equal one engine."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    topo = T.random_regular(5000, 8, seed=3)
    sc = Scenario(topo, 512, 30, uniform_injections(5000, 500, 4), seed=5, sync_base=12, sync_jitter=4)
    single = make_engine(hip_lib, sc, device=0)
    want = single.step(sc.rounds)
    tot = None
    for rank in range(4):
        e = make_engine(hip_lib, sc, device=0, rank=rank, world=4, lane_groups=4)
        st = e.step(sc.rounds)
        if tot is None:
            tot = [dict(x) for x in st]
        else:
            for a, b in zip(tot, st):
                for f in a:
                    if f != "round" and isinstance(a[f], int):
                        a[f] = (a[f] + b[f]) & ((1 << 64) - 1)
        e.close()
    assert not diff_stats(want, tot), diff_stats(want, tot)[:10]
    single.close()


def _gen_worker(rank, world, port, lib, spec, W, inj, rounds, q):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        e = Engine(spec["V"], W, seed=3, sync_base=6, sync_jitter=4, device=0, rank=rank, world=world, library=lib)
        e.generate(**spec["gen"])
        for n, v, r in inj:
            e.broadcast(n, v, r)
        stats = ShardedRunner(e, torch.device("cuda", 0)).step(rounds)
        owned = e.dist_owned()
        q.put((rank, stats, owned, e.read_bits_nodes(owned)))
        e.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["grid_links", "tree"])
def test_sharded_engine_with_device_generated_topology(hip_lib, kind):
    """gg_topology_generate on a sharded engine (device build, host partition
    step) equals one engine given the host builder's CSR."""
    from ggamd import topology as T
    from ggamd.engine import Engine
    from ggamd.workload import uniform_injections
    if kind == "grid_links":
        spec = {"V": 40 * 40, "gen": dict(kind="grid_links", n=40, seed=77)}
        topo = T.grid_links(40, 77)
    else:
        spec = {"V": 3000, "gen": dict(kind="tree", n=3000, k=4)}
        topo = T.tree(3000, 4)
    W, rounds, world = 128, 24, 2
    inj = uniform_injections(spec["V"], 100, 5)
    ref = Engine(spec["V"], W, seed=3, sync_base=6, sync_jitter=4, device=0, library=hip_lib)
    ref.topology(topo)
    for n, v, r in inj:
        ref.broadcast(n, v, r)
    want = ref.step(rounds)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gen_worker, args=(r, world, port, hip_lib, spec, W, inj, rounds, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    stats = res[0][1]
    d = diff_stats(stats, want)
    assert not d, d[:10]
    bits = ref.read_bits()
    for _, _, owned, got in res:
        assert np.array_equal(got, bits[owned])


def test_engine_rccl_plumbing():
    """The engine-owned exchange (gg_dist_comm_*, gg_dist_step) in one process:
    RCCL resolves from the copy torch loaded, a unique id comes back, and the
    error paths hold (a world-1 engine cannot open a communicator; a sharded
    engine without one cannot step). Two ranks on one device are refused by
    RCCL itself (tools/nccl_probe.py), so the grouped send/recv runs only in the
    driver's multi-GPU bench; its segments are the ones the gloo tests above
    move and check."""
    import torch  # noqa: F401  (loads torch's RCCL, as the bench does)

    from ggamd.engine import Engine, GGError, HIP_LIB, Topology
    e1 = Engine(64, 64, device=0, library=HIP_LIB)
    ok, why = e1.dist_comm_available()
    assert ok, why
    uid = e1.dist_comm_id()
    assert len(uid) == 128 and any(uid)
    with pytest.raises(GGError):
        e1.dist_comm_init(uid)
    e2 = Engine(64, 64, device=0, rank=0, world=2, library=HIP_LIB)
    e2.topology(Topology.from_rows([sorted({(v + 1) % 64, (v + 63) % 64}) for v in range(64)]))
    with pytest.raises(GGError, match="no communicator"):
        e2.dist_step(1)
    with pytest.raises(GGError, match="not an id from gg_dist_comm_id"):
        e2.dist_comm_init(bytes(128))
    e1.close()
    e2.close()


def test_comm_id_names_its_lane_group():
    """ABI 6: an RCCL id made by lane group 0's part 0 is refused by a part of
    lane group 1 (2 lane groups x 2 parts), before any RCCL call, instead of
    joining ranks of two groups with equal part numbers in one communicator."""
    import torch  # noqa: F401

    from ggamd.engine import Engine, GGError, HIP_LIB, Topology
    ring = Topology.from_rows([sorted({(v + 1) % 64, (v + 63) % 64}) for v in range(64)])
    engs = [Engine(64, 128, device=0, rank=r, world=4, lane_groups=2, library=HIP_LIB) for r in range(4)]
    for e in engs:
        e.topology(ring)
    uid_g0 = engs[0].dist_comm_id()  # rank 0 = group 0, part 0
    for r in (2, 3):  # group 1
        with pytest.raises(GGError, match="lane group 0 of 2 parts"):
            engs[r].dist_comm_init(uid_g0)
    for e in engs:
        e.close()


def _gen_scenarios():
    """Generated graphs: the same graphs as the host builders (gossip_gen.h)."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    return [
        Scenario(T.grid_links(48, seed=31), 64, 45, uniform_injections(48 * 48, 64, 32), seed=33, sync_base=8,
                 sync_jitter=4, windows=[("seeded", 3, 9, 7)], gen=dict(kind="grid_links", n=48, seed=31)),
        Scenario(T.tree(3001, 4), 256, 40, uniform_injections(3001, 200, 34), seed=35, sync_base=6, sync_jitter=3,
                 gen=dict(kind="tree", n=3001, k=4)),
        Scenario(T.random_regular(4000, 8, seed=36), 1024, 30, uniform_injections(4000, 900, 37), seed=38,
                 sync_base=10, sync_jitter=5, gen=dict(kind="random_regular", n=4000, k=8, seed=36)),
        Scenario(T.rmat(4096, 16, seed=39), 256, 24, uniform_injections(4096, 256, 40), seed=41, sync_base=9,
                 sync_jitter=3, gen=dict(kind="rmat", n=4096, k=16, seed=39, a=0.57, b=0.19, c=0.19)),
    ]


@pytest.mark.parametrize("world,mode", [(2, "static"), (3, "exact"), (4, "static")])
def test_device_partition_equals_single(hip_lib, world, mode):
    """gg_topology_generate on vertex-sharded engines: every rank builds only
    its node range of the generated graph and its ghosts / send lists on the
    device (gg_gen::shard_csr). Counters summed over ranks, and every owned
    node's set and delivery rounds, equal one engine on the host-built graph."""
    scs = _gen_scenarios()
    res = _run(hip_lib, scs, world, env={"GG_XCHG_MODE": mode, "GG_HUB_DEG": "40"}, generate=True)
    for k, sc in enumerate(scs):
        single = make_engine(hip_lib, sc, device=0)
        s1 = single.step(sc.rounds)
        owned_all = []
        for rank in range(world):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(s1, stats)
            assert not d, (k, rank, d[:10])
            assert np.array_equal(bits, single.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, single.delivery_rounds_nodes(owned)), (k, rank)
            owned_all.append(owned)
        assert np.array_equal(np.sort(np.concatenate(owned_all)), np.arange(sc.topo.n_nodes)), k
        single.close()


def test_device_partition_with_lane_groups(hip_lib):
    """2 lane groups x 2 device-built vertex parts (world 4): counters summed
    over all ranks equal one engine; sets OR-ed and delivery rounds max-ed
    over a node's owners equal its own."""
    scs = [sc for sc in _gen_scenarios() if sc.W // 64 >= 2]
    res = _run(hip_lib, scs, 4, lane_groups=2, env={"GG_XCHG_MODE": "exact"}, generate=True)
    for k, sc in enumerate(scs):
        single = make_engine(hip_lib, sc, device=0)
        s1 = single.step(sc.rounds)
        V = sc.topo.n_nodes
        bits = np.zeros((V, sc.W // 64), np.uint64)
        dr = np.full((V, sc.W), -1, np.int32)
        for rank in range(4):
            stats, owned, b, d = res[rank][k]
            assert not diff_stats(s1, stats), (k, rank, diff_stats(s1, stats)[:10])
            o = owned.astype(np.int64)
            bits[o] |= b
            dr[o] = np.maximum(dr[o], d)
        assert np.array_equal(bits, single.read_bits()), k
        assert np.array_equal(dr, single.delivery_rounds()), k
        single.close()


@pytest.mark.parametrize("world,mode", [(2, "exact"), (3, "exact"), (3, "static")])
def test_engine_exchange_sequencing_equals_single(hip_lib, world, mode):
    """gg_dist_step's own sequencing — the exact-size handshake, the peer
    choice, the segment offsets, one host wait per round — run through
    gg_transport callbacks over gloo (ggamd.dist.HostTransport) instead of
    RCCL, which refuses two ranks on one device: bit-exact against one engine,
    host-built and device-built partitions."""
    scs = _scenarios()[:5]
    res = _run(hip_lib, scs, world, env={"GG_XCHG_MODE": mode}, transport="engine")
    gen = _gen_scenarios()
    res_g = _run(hip_lib, gen, world, env={"GG_XCHG_MODE": mode, "GG_HUB_DEG": "40"}, generate=True,
                 transport="engine")
    old = os.environ.get("GG_HUB_DEG")
    for sc_list, rr, hub in ((scs, res, None), (gen, res_g, "40")):
        if hub:
            os.environ["GG_HUB_DEG"] = hub
        try:
            for k, sc in enumerate(sc_list):
                single = make_engine(hip_lib, sc, device=0)
                s1 = single.step(sc.rounds)
                for rank in range(world):
                    stats, owned, bits, dr = rr[rank][k]
                    d = diff_stats(s1, stats)
                    assert not d, (k, rank, d[:10])
                    assert np.array_equal(bits, single.read_bits_nodes(owned)), (k, rank)
                    assert np.array_equal(dr, single.delivery_rounds_nodes(owned)), (k, rank)
                single.close()
        finally:
            if old is None:
                os.environ.pop("GG_HUB_DEG", None)
            else:
                os.environ["GG_HUB_DEG"] = old


def _world8_scenarios():
    """BASELINE's 8-GPU shapes at a size one GPU's eight ranks run in seconds:
    C4 (R-MAT, edge factor 16, hubs on the hub path with GG_HUB_DEG=24) and C5
    (grid + one long link per node, W = 64), each with the sync timers firing
    during propagation so sets cross the cut as well as F rows."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    return [
        Scenario(T.rmat(8192, 16, seed=51), 256, 26, uniform_injections(8192, 256, 52), seed=53, sync_base=6,
                 sync_jitter=3, gen=dict(kind="rmat", n=8192, k=16, seed=51, a=0.57, b=0.19, c=0.19)),
        Scenario(T.grid_links(96, seed=54), 64, 40, uniform_injections(96 * 96, 64, 55), seed=56, sync_base=9,
                 sync_jitter=4, gen=dict(kind="grid_links", n=96, seed=54)),
    ]


def _check_against_oracle(cpu_lib, scs, res, world, lane_groups=1):
    """Summed counters of every round, every node's set and delivery rounds
    (OR / max over a node's lane-group owners) against O2 directly."""
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        V = sc.topo.n_nodes
        bits = np.zeros((V, sc.W // 64), np.uint64)
        dr = np.full((V, sc.W), -1, np.int32)
        seen = np.zeros(V, np.int64)
        for rank in range(world):
            stats, owned, b, d = res[rank][k]
            assert not diff_stats(want, stats), (k, rank, diff_stats(want, stats)[:10])
            o = owned.astype(np.int64)
            bits[o] |= b
            dr[o] = np.maximum(dr[o], d)
            seen[o] += 1
        assert np.all(seen == lane_groups), k  # every node owned once per lane group
        assert np.array_equal(bits, ref.read_bits()), k
        assert np.array_equal(dr, ref.delivery_rounds()), k
        ref.close()


@pytest.mark.parametrize("build", ["host_csr", "device"])
@pytest.mark.parametrize("transport", ["torch", "engine", "ipc"])
def test_world8_equals_oracle(hip_lib, cpu_lib, build, transport):
    """World 8 (BASELINE's GPU count) as 8 ranks on this GPU, vertex-range
    sharded 8 ways, against the CPU oracle O2: the C4 and C5 shapes, host-CSR
    partitions (gg_topology: locality order) and device-built ones
    (gg_topology_generate: native ranges), over the Python all-to-all-v
    sequencing, over the engine's own gg_dist_step sequencing, and over the
    device-driven exchange (IPC-mapped windows, captured batches of rounds)."""
    scs = _world8_scenarios()
    res = _run(hip_lib, scs, 8, env={"GG_HUB_DEG": "24", "GG_XCHG_MODE": "exact"},
               generate=(build == "device"), transport=transport, timeout=240)
    _check_against_oracle(cpu_lib, scs, res, 8)


def test_world8_c4_shape_full_width_equals_oracle(hip_lib, cpu_lib):
    """The C4 shape at BASELINE's width (W = 4096 lanes: 512-byte rows, the
    widest node group of the kernels) on 8 device-built ranks, sync timers firing
    during propagation, over the device-driven exchange, against O2."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    scs = [Scenario(T.rmat(4096, 16, seed=61), 4096, 22, uniform_injections(4096, 4096, 62), seed=63, sync_base=6,
                    sync_jitter=3, gen=dict(kind="rmat", n=4096, k=16, seed=61, a=0.57, b=0.19, c=0.19))]
    res = _run(hip_lib, scs, 8, env={"GG_HUB_DEG": "24"}, generate=True, transport="ipc", timeout=240)
    _check_against_oracle(cpu_lib, scs, res, 8)


@pytest.mark.parametrize("world", [2, 4])
def test_parts_lean_digest_equals_oracle(hip_lib, cpu_lib, world):
    """The lean saturation digest on vertex parts (device-built R-MAT with hubs):
    component labels of the whole generated graph, per-component targets from
    every rank's broadcasts (a later batch of values, two of them re-sent into
    other components) — against O2, and with fewer sender-row gathers than the
    same run without the digest (GG_LSAT=0); and the exchange's need bits
    (expand_kernels.hpp NeedWord) ship fewer payload bytes than the same run
    without them (GG_NEED_BITS=0), against O2 as well."""
    import random as _r

    from ggamd import topology as T
    rnd = _r.Random(71)
    inj = [(rnd.randrange(4096), v, 0) for v in range(200)] + [(rnd.randrange(4096), 200 + v, 9) for v in range(56)]
    inj += [(11, 5, 3), (3000, 201, 10)]
    gen = dict(kind="rmat", n=4096, k=16, seed=72, a=0.57, b=0.19, c=0.19)
    scs = [Scenario(T.rmat(4096, 16, seed=72), 256, 24, inj, seed=73, enable_sync=False, gen=gen),
           Scenario(T.rmat(4096, 16, seed=72), 1024, 20, inj, seed=74, sync_base=11, sync_jitter=2, gen=gen)]
    gathers, sent = {}, {}
    for lsat in ("1", "0", "1-no-need"):
        env = {"GG_HUB_DEG": "16", "GG_HUB_CHUNK": "7"}
        if lsat == "0":
            env["GG_LSAT"] = "0"
        if lsat == "1-no-need":
            env["GG_NEED_BITS"] = "0"
        res = _run(hip_lib, scs, world, env=env, generate=True, transport="ipc", timeout=240)
        _check_against_oracle(cpu_lib, scs, res, world)
        gathers[lsat] = sum(st["work_gathers"] for r in res for st in r[0][0])
        sent[lsat] = sum(st["sent_bytes"] for r in res for k in range(len(scs)) for st in r[k][0])
    assert gathers["1"] < gathers["0"], gathers
    # need bits (the peers skip the F rows of ghosts whose receivers here are all
    # saturated; rounds with client broadcasts in them or the round before keep every row)
    assert sent["1"] < sent["1-no-need"], sent


def test_world8_lane_groups_by_parts_equals_oracle(hip_lib, cpu_lib):
    """2 lane groups x 4 vertex parts (world 8), device-built partitions, the
    engine's exchange sequencing, against O2."""
    scs = [sc for sc in _world8_scenarios() if sc.W >= 128]
    res = _run(hip_lib, scs, 8, lane_groups=2, env={"GG_HUB_DEG": "24"}, generate=True, transport="engine",
               timeout=240)
    _check_against_oracle(cpu_lib, scs, res, 8, lane_groups=2)


def _halves_worker(rank, world, port, lib, scenarios, q, parts, env):
    import torch
    import torch.distributed as dist

    from ggamd.dist import HalvesRunner
    os.environ.update(env or {})
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        g, part = divmod(rank, parts)
        L = world // parts
        for sc in scenarios:
            engs = [make_engine(lib, sc, rank=(2 * g + h) * parts + part, world=2 * world, device=0,
                                lane_groups=2 * L, generate=True) for h in range(2)]
            r = HalvesRunner(engs, dev)
            half = sc.rounds // 2
            stats = r.step(half) + r.step(sc.rounds - half)  # summed over ranks
            owned = engs[0].dist_owned()
            assert np.array_equal(owned, engs[1].dist_owned())
            bits = engs[0].read_bits_nodes(owned) | engs[1].read_bits_nodes(owned)
            dr = np.maximum(engs[0].delivery_rounds_nodes(owned), engs[1].delivery_rounds_nodes(owned))
            out.append((stats, owned, bits, dr))
            r.close()
            for e in engs:
                e.close()
        q.put((rank, out))
    except BaseException as exc:
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,parts,transport", [(2, 2, "engine"), (4, 4, "engine"), (4, 2, "engine"),
                                                  (4, 4, "ipc"), (8, 8, "ipc")])
def test_lane_halves_equal_oracle(hip_lib, cpu_lib, world, parts, transport):
    """ggamd.dist.HalvesRunner: two engines per process over the two halves of
    its lanes, device-built vertex parts, the engines' own exchange over gloo
    (half A's round then half B's) or device-driven (both halves' rounds
    enqueued at once on their own streams): per-rank counters (summed over
    ranks) and every node's set and delivery rounds equal O2."""
    scs = [sc for sc in _world8_scenarios() if sc.W >= 256]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halves_worker, args=(r, world, port, hip_lib, scs, q, parts,
                                                      {"GG_HUB_DEG": "24", "GG_XCHG_MODE": "exact",
                                                       "GG_DIST_TRANSPORT": transport}))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = q.get(timeout=240)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [res[r] for r in range(world)]
    _check_against_oracle(cpu_lib, scs, res, world, lane_groups=world // parts)


def _part_worker(rank, world, port, lib, scenarios, bounds, q, transport):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        for sc, plo in zip(scenarios, bounds):
            t = sc.topo
            lo, hi = int(plo[rank]), int(plo[rank + 1])
            rp = t.row_ptr[lo:hi + 1] - t.row_ptr[lo]  # this rank's rows only
            col = t.col[t.row_ptr[lo]:t.row_ptr[hi]]
            e = Engine(t.n_nodes, sc.W, seed=sc.seed, sync_base=sc.sync_base, sync_jitter=sc.sync_jitter,
                       enable_sync=sc.enable_sync, track_delivery=True, device=0, rank=rank, world=world,
                       library=lib)
            e.topology_part(plo, rp, col)
            for w in sc.windows:
                e.partition_seeded(w[1], w[2], w[3])
            for n, v, r in sc.injections:
                e.broadcast(int(n), int(v), int(r))
            r = ShardedRunner(e, dev, transport=transport)
            stats = r.step(sc.rounds)
            owned = e.dist_owned()
            assert np.array_equal(np.sort(owned), np.arange(lo, hi))  # rows in locality order
            out.append((stats, owned, e.read_bits_nodes(owned), e.delivery_rounds_nodes(owned)))
            r.close()
            e.close()
        q.put((rank, out))
    except BaseException as exc:
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,transport", [(2, "torch"), (3, "engine")])
def test_topology_part_equals_single(hip_lib, world, transport):
    """gg_topology_part: every rank is handed only its own rows (uneven,
    caller-chosen ranges; global column ids) and builds ghosts and send lists
    on the device; no rank sees another's rows. Equal to one engine given the
    whole graph: counters, owned sets and delivery rounds."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    rnd = random.Random(61)
    scs = [Scenario(T.grid_links(40, seed=62), 128, 40, uniform_injections(1600, 100, 63), seed=64, sync_base=7,
                    sync_jitter=3, windows=[("seeded", 3, 8, 9)]),
           Scenario(T.rmat(3000, 8, seed=65), 256, 30, uniform_injections(3000, 200, 66), seed=67, sync_base=9,
                    sync_jitter=4),
           Scenario(T.tree(2500, 4), 64, 30, uniform_injections(2500, 64, 68), seed=69, sync_base=8, sync_jitter=2)]
    bounds = []
    for sc in scs:
        V = sc.topo.n_nodes
        cuts = sorted(rnd.sample(range(1, V), world - 1))
        bounds.append(np.array([0] + cuts + [V], np.uint64))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_part_worker, args=(r, world, port, hip_lib, scs, bounds, q, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = q.get(timeout=150)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, sc in enumerate(scs):
        single = make_engine(hip_lib, sc, device=0)
        s1 = single.step(sc.rounds)
        for rank in range(world):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(s1, stats)
            assert not d, (k, rank, d[:10])
            assert np.array_equal(bits, single.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, single.delivery_rounds_nodes(owned)), (k, rank)
        single.close()


def test_topology_part_refusals(hip_lib):
    """gg_topology_part refuses a non-sharded engine, bad part boundaries, and
    a part whose own links are not listed both ways."""
    from ggamd.engine import Engine, GGError
    e1 = Engine(8, 64, device=0, library=hip_lib)
    with pytest.raises(GGError, match="not a vertex-sharded"):
        e1.topology_part([0, 8], [0, 0], [])
    e1.close()
    e = Engine(8, 64, device=0, rank=0, world=2, library=hip_lib)
    with pytest.raises(GGError, match="from 0 to n_nodes"):
        e.topology_part([0, 4, 7], [0] * 5, [])
    with pytest.raises(GGError, match="symmetric"):  # 0 -> 1 listed, 1 -> 0 missing
        e.topology_part([0, 4, 8], [0, 1, 1, 1, 1], [1])
    e.topology_part([0, 4, 8], [0, 1, 2, 2, 2], [1, 0])
    e.close()


@pytest.mark.parametrize("world,db,mark", [(2, "GG_DB", "1"), (4, "GG_DB", "1"), (2, "GG_DB", "0"),
                                           (2, "GG_NO_DB", "1"), (4, "GG_NO_DB", "1")])
def test_sharded_db_paths_equal_oracle(hip_lib, cpu_lib, world, db, mark):
    """Both lean-round paths of a sharded engine, forced (GG_DB: double-buffered
    sets — ghost senders' F rows from the exchange, pack_ghosts with set_prev,
    materialize_F and clear_stale_ghosts at the hand-over to the sync rounds;
    GG_NO_DB: the F-row kernels), against O2; gg_round_stats.path says which ran.
    Double-buffered rounds on symmetric graphs are marking rounds (the expand
    marks the next round's owned candidates, the exchange's unpack the owned
    receivers of active ghosts: no round_prep) unless GG_NO_MARK=1."""
    from ggamd import topology as T
    from ggamd.engine import PATH_DB, PATH_NO_PREP
    from ggamd.workload import uniform_injections
    scs = [Scenario(T.tree(3000, 4), 256, 34, uniform_injections(3000, 200, 41), seed=42, sync_base=6, sync_jitter=3),
           Scenario(T.random_regular(2500, 8, seed=43), 128, 30,
                    [(n, v, v % 4) for n, v, _ in uniform_injections(2500, 120, 44)], seed=45, sync_base=5,
                    sync_jitter=2),
           Scenario(T.grid_links(44, seed=46), 512, 36, uniform_injections(44 * 44, 300, 47), seed=48, sync_base=9,
                    sync_jitter=4, windows=[("seeded", 12, 16, 3)])]
    res = _run(hip_lib, scs, world, env={db: "1", "GG_NO_MARK": "0" if mark == "1" else "1"})
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        for rank in range(world):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(want, stats)
            assert not d, (k, rank, d[:8])
            assert np.array_equal(bits, ref.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, ref.delivery_rounds_nodes(owned)), (k, rank)
            n_db = sum(1 for s in stats if s["path"] & PATH_DB)
            n_np = sum(1 for s in stats if s["path"] & PATH_NO_PREP)
            if db == "GG_DB":
                assert n_db >= 4, (k, rank, [s["path"] for s in stats])
                assert (n_np >= 3) if mark == "1" else (n_np == 0), (k, rank, [s["path"] for s in stats])
            else:
                assert n_db == 0 and n_np == 0, (k, rank)
        ref.close()


def _ipc_worker(rank, world, port, lib, scenarios, q, lane_groups, env):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from helpers import apply
    os.environ.update(env or {})
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        for sc in scenarios:
            e = make_engine(lib, sc, rank=rank, world=world, device=0, lane_groups=lane_groups)
            r = ShardedRunner(e, dev, transport="ipc")
            assert r.transport.startswith("device-driven"), r.transport
            half = sc.rounds // 2
            first = r.step(half) + r.step(sc.rounds - half)
            owned = e.dist_owned()
            res = (first, owned, e.read_bits_nodes(owned), e.delivery_rounds_nodes(owned))
            # a second episode after gg_reset: the exchange's sequence numbers go on
            e.reset()
            for n, v, rr in sc.injections:
                e.broadcast(int(n), int(v), int(rr))
            again = r.step(sc.rounds)
            out.append(res + (again,))
            r.close()  # collective: every rank unmaps its peers' windows before any window is freed
            e.close()
        q.put((rank, out))
    except BaseException as exc:  # report instead of leaving the parent waiting
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lane_groups", [(2, 1), (3, 1), (4, 2), (8, 1)])
def test_ipc_exchange_equals_oracle(hip_lib, cpu_lib, world, lane_groups):
    """The device-driven exchange (gg_dist_ipc_*): every rank a process with an
    engine on the one GPU, windows mapped with hipIpcOpenMemHandle, segments
    packed straight into the peers' receive buffers and handed over by kernel
    flags — no collective and no host wait per round. Counters of every round,
    node sets and delivery rounds equal O2, and a second episode after gg_reset
    equals the first."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    scs = [Scenario(T.tree(3000, 4), 256, 30, uniform_injections(3000, 200, 5), seed=9, sync_base=6, sync_jitter=3,
                    windows=[("seeded", 3, 9, 77)]),
           Scenario(T.grid_links(40, seed=11), 64, 36, uniform_injections(1600, 64, 6), seed=10, sync_base=8,
                    sync_jitter=4),
           Scenario(T.rmat(2048, 8, seed=22), 128, 26, uniform_injections(2048, 100, 9), seed=14, sync_base=8,
                    sync_jitter=4)]
    scs = [sc for sc in scs if sc.W >= 64 * lane_groups]  # a lane group holds whole 64-lane words
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, world, port, hip_lib, scs, qq, lane_groups, None))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = qq.get(timeout=170)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        tot_own = []
        for rank in range(world):
            stats, owned, bits, dr, again = res[rank][k]
            d = diff_stats(want, stats)
            assert not d, (k, rank, d[:8])
            assert not diff_stats(want, again), (k, rank, "second episode")
            if lane_groups == 1:  # (a lane-group engine holds its own lanes only)
                assert np.array_equal(bits, ref.read_bits_nodes(owned)), (k, rank)
                assert np.array_equal(dr, ref.delivery_rounds_nodes(owned)), (k, rank)
            if rank < world // lane_groups:
                tot_own.append(owned)
        assert np.array_equal(np.sort(np.concatenate(tot_own)), np.arange(sc.topo.n_nodes)), k
        ref.close()


def _slice_bits(words, a, b):
    """Bits [a, b) of a uint64 bit array, re-based to bit 0."""
    n = b - a
    out = np.zeros((n + 63) // 64, np.uint64)
    for k in range(n):
        x = a + k
        if (int(words[x >> 6]) >> (x & 63)) & 1:
            out[k >> 6] |= np.uint64(1) << np.uint64(k & 63)
    return out


def _own_rows_worker(rank, world, port, lib, scenarios, bounds, q, directed):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        for sc, plo in zip(scenarios, bounds):
            t = sc.topo
            lo, hi = int(plo[rank]), int(plo[rank + 1])
            rp = t.row_ptr[lo:hi + 1] - t.row_ptr[lo]  # this rank's rows only
            col = t.col[t.row_ptr[lo]:t.row_ptr[hi]]
            e = Engine(t.n_nodes, sc.W, seed=sc.seed, sync_base=sc.sync_base, sync_jitter=sc.sync_jitter,
                       enable_sync=sc.enable_sync, track_delivery=True, device=0, rank=rank, world=world,
                       library=lib)
            r = ShardedRunner(e, dev, transport="engine")  # the reverse edges travel over it
            if directed:
                e.topology_part_directed(plo, rp, col)
            else:
                e.topology_part(plo, rp, col)
            for w in sc.windows:
                if w[0] == "seeded":
                    e.partition_seeded(w[1], w[2], w[3])
                elif w[0] == "groups":
                    e.partition_groups(w[1], w[2], w[3])
                else:  # per-edge bits over this rank's own rows
                    e.set_partition(w[1], w[2], _slice_bits(w[3], int(t.row_ptr[lo]), int(t.row_ptr[hi])))
            for n, v, rr in sc.injections:
                e.broadcast(int(n), int(v), int(rr))
            stats = r.step(sc.rounds)
            owned = e.dist_owned()
            out.append((stats, owned, e.read_bits_nodes(owned), e.delivery_rounds_nodes(owned)))
            e.close()
        q.put((rank, out))
    except BaseException as exc:
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("directed", [True, False])
def test_own_rows_directed_and_edge_windows_equal_oracle(hip_lib, cpu_lib, directed):
    """Each of 3 ranks holds only its own rows (uneven ranges). Directed rows
    (gg_topology_part_directed): the in-lists come from the other ranks' rows
    through one exchange of reverse edges, with seeded and group windows and sync
    timers. Symmetric rows (gg_topology_part) with per-edge windows whose bits
    each rank gives over its own rows only. Against O2 given the whole graph."""
    from helpers import random_scenario, symmetric_cut, symmetric_random_scenario
    rnd = random.Random(71 + directed)
    world = 3
    scs = []
    for k in range(4):
        if directed:
            sc = random_scenario(rnd, max_v=400, directed_p=0.4, W=128, rounds=45)
            while sc.topo.n_nodes < 30:
                sc = random_scenario(rnd, max_v=400, directed_p=0.4, W=128, rounds=45)
        else:
            sc = symmetric_random_scenario(rnd, max_v=400, W=128, rounds=45, edge_windows=2)
            while sc.topo.n_nodes < 30:
                sc = symmetric_random_scenario(rnd, max_v=400, W=128, rounds=45, edge_windows=2)
        scs.append(sc)
    if not directed:
        assert any(w[0] == "edges" for sc in scs for w in sc.windows)
    bounds = []
    for sc in scs:
        V = sc.topo.n_nodes
        cuts = sorted(rnd.sample(range(1, V), world - 1))
        bounds.append(np.array([0] + cuts + [V], np.uint64))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_own_rows_worker, args=(r, world, port, hip_lib, scs, bounds, q, directed))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = q.get(timeout=170)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        for rank in range(world):
            stats, owned, bits, dr = res[rank][k]
            d = diff_stats(want, stats)
            assert not d, (k, rank, d[:8])
            assert np.array_equal(bits, ref.read_bits_nodes(owned)), (k, rank)
            assert np.array_equal(dr, ref.delivery_rounds_nodes(owned)), (k, rank)
        ref.close()


def _batched_scenarios():
    """Batched gossip across a vertex cut: sync timers firing while batches are
    in flight (pushes and callbacks read ghost sets), seeded and edge windows,
    client broadcasts spread over the rounds."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    from helpers import symmetric_cut
    rnd = random.Random(31)
    grid = T.grid_links(40, seed=32)
    return [
        Scenario(T.tree(3000, 4), 256, 36, [(n, v, v % 9) for n, v, _ in uniform_injections(3000, 200, 33)],
                 seed=34, sync_base=6, sync_jitter=3, windows=[("seeded", 3, 9, 35)]),
        Scenario(grid, 128, 40, [(n, v, v % 5) for n, v, _ in uniform_injections(1600, 100, 36)], seed=37,
                 sync_base=7, sync_jitter=3, windows=[("seeded", 2, 8, 5), ("edges", 5, 14, symmetric_cut(grid, rnd, 0.3))]),
        Scenario(T.random_regular(2500, 6, seed=38), 64, 30, uniform_injections(2500, 64, 39), seed=40,
                 enable_sync=False),
        random_scenario(random.Random(41), max_v=300, W=128, rounds=45),
    ]


@pytest.mark.parametrize("world,transport", [(2, "torch"), (3, "engine"), (3, "ipc")])
@pytest.mark.parametrize("B", [2, 3])
def test_batched_sharded_equals_oracle(hip_lib, cpu_lib, world, transport, B):
    """Batched gossip (gg_config.batch_ticks) on vertex parts: every engine runs
    its ghosts' timers, batches cross the cut as F rows and the sets read by
    pushes and callbacks as kind S into the set buffer of the round. Counters
    of every round, sets and delivery rounds equal the single O2 engine."""
    scs = _batched_scenarios()
    res = _run(hip_lib, scs, world, transport=transport, kw={"batch_ticks": B})
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc, batch_ticks=B)
        want = ref.step(sc.rounds)
        bits = np.zeros((sc.topo.n_nodes, sc.W // 64), np.uint64)
        dr = np.full((sc.topo.n_nodes, sc.W), -1, np.int32)
        for rank in range(world):
            stats, owned, b, d = res[rank][k]
            assert not diff_stats(want, stats), (k, rank, diff_stats(want, stats)[:10])
            bits[owned.astype(np.int64)] = b
            dr[owned.astype(np.int64)] = d
        assert np.array_equal(bits, ref.read_bits()), k
        assert np.array_equal(dr, ref.delivery_rounds()), k
        ref.close()


def test_batched_refuses_lane_groups(hip_lib):
    from ggamd.engine import Engine, GGError
    with pytest.raises(GGError):
        Engine(10, 128, batch_ticks=2, world=2, rank=0, lane_groups=2, library=hip_lib)


def test_ipc_rounded_windows_equal_oracle(hip_lib, cpu_lib, monkeypatch):
    """Windows allocated larger than their exchange needs (GG_IPC_WINDOW_ALIGN_MB=64
    rounds every new window up to 64 MiB, as the engine rounds windows above 1 GiB
    to whole GiB): the same exchange, the same results against O2, at 3 ranks."""
    monkeypatch.setenv("GG_IPC_WINDOW_ALIGN_MB", "64")  # inherited by the spawned ranks
    test_ipc_exchange_equals_oracle(hip_lib, cpu_lib, 3, 1)


def _episodes_worker(rank, world, port, lib, scenarios, q, lane_groups, episodes):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        dev = torch.device("cuda", 0)
        for sc in scenarios:
            e = make_engine(lib, sc, rank=rank, world=world, device=0, lane_groups=lane_groups)
            r = ShardedRunner(e, dev, transport="ipc")
            assert r.can_run_episodes, r.transport
            eps = [r.reduce(ep) for ep in r.run_episodes(sc.rounds, episodes)]
            owned = e.dist_owned()
            bits = e.read_bits_nodes(owned)
            # a synchronous episode after it starts from the state it left
            e.reset()
            for n, v, rr in sc.injections:
                e.broadcast(int(n), int(v), int(rr))
            again = r.step(sc.rounds)
            if os.environ.get("GG_IPC_DEBUG"):
                print(f"episodes worker rank {rank}: synchronous episode done", flush=True)
            # collective teardown (gg_dist_ipc_close on every rank, then a barrier), and
            # the same engines map each other's windows again: the same episode once more
            r.close()
            r = ShardedRunner(e, dev, transport="ipc")
            e.reset()
            for n, v, rr in sc.injections:
                e.broadcast(int(n), int(v), int(rr))
            reimported = r.step(sc.rounds)
            from ggamd.engine import COUNT_FIELDS
            key = lambda st: [[x[f] for f in COUNT_FIELDS] for x in st]  # noqa: E731
            assert key(reimported) == key(again), "an episode after re-import differs"
            out.append((eps, owned, bits, again))
            r.close()
            e.close()
        q.put((rank, out))
    except BaseException as exc:  # report instead of leaving the parent waiting
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lane_groups", [(2, 1), (3, 1), (4, 2)])
def test_ipc_run_episodes_equal_oracle(hip_lib, cpu_lib, world, lane_groups):
    """gg_dist_run_episodes: episodes of the device-driven sharded round queued
    back to back (reset and broadcasts of episode k > 0 on the device, one host
    wait): every episode's summed counters equal O2's episode, the node sets
    after the last one equal O2's, and a synchronous episode after it too."""
    from ggamd import topology as T
    from ggamd.workload import uniform_injections
    scs = [Scenario(T.tree(3000, 4), 256, 30, uniform_injections(3000, 200, 5), seed=9, sync_base=6, sync_jitter=3),
           Scenario(T.grid_links(40, seed=11), 64, 36, uniform_injections(1600, 64, 6), seed=10, sync_base=8,
                    sync_jitter=4),
           Scenario(T.random_regular(2048, 6, seed=3), 128, 26, uniform_injections(2048, 100, 9), seed=14,
                    sync_base=8, sync_jitter=4, windows=[("seeded", 2, 7, 5)])]
    scs = [sc for sc in scs if sc.W >= 64 * lane_groups]
    episodes = 3
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_episodes_worker, args=(r, world, port, hip_lib, scs, qq, lane_groups, episodes))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = qq.get(timeout=170)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, sc in enumerate(scs):
        ref = make_engine(cpu_lib, sc)
        want = ref.step(sc.rounds)
        for rank in range(world):
            eps, owned, bits, again = res[rank][k]
            assert len(eps) == episodes
            for j, ep in enumerate(eps):
                d = diff_stats(want, ep)
                assert not d, (k, rank, j, d[:8])
            assert not diff_stats(want, again), (k, rank, "synchronous episode after")
            if lane_groups == 1:
                assert np.array_equal(bits, ref.read_bits_nodes(owned)), (k, rank)
        ref.close()


def _dead_peer_worker(rank, world, port, lib, q, rounds):
    import time

    import torch
    import torch.distributed as dist

    from ggamd import topology as T
    from ggamd.dist import ShardedRunner
    from ggamd.engine import GGError
    from ggamd.workload import uniform_injections
    os.environ["GG_IPC_SPIN_LIMIT"] = str(1 << 16)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = Scenario(T.tree(3000, 4), 128, 30, uniform_injections(3000, 100, 5), seed=9, enable_sync=False)
        e = make_engine(lib, sc, rank=rank, world=world, device=0)
        r = ShardedRunner(e, torch.device("cuda", 0), transport="ipc")
        t0 = time.perf_counter()
        err1 = err2 = None
        try:
            r.step(rounds[rank], reduce=False)
        except GGError as exc:
            err1 = str(exc)
        t1 = time.perf_counter()
        try:  # a dead exchange stays dead, and its waits no longer spin
            r.step(4, reduce=False) if err1 else None
        except GGError as exc:
            err2 = str(exc)
        t2 = time.perf_counter()
        dist.barrier()  # the short rank keeps its window mapped until the long one is done
        e.close()
        q.put((rank, (err1, err2, t1 - t0, t2 - t1)))
    except BaseException as exc:  # noqa: BLE001
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


def test_ipc_dead_peer_fails_after_one_bound(hip_lib):
    """a peer that stops exchanging costs its partner ONE wait bound.
    Rank 1 runs 4 rounds, rank 0 runs 12 (8 rounds = 16 waits its peer never
    answers). With a lowered bound (GG_IPC_SPIN_LIMIT) rank 0 gets GG_EIO with
    exactly one wait counted as run out (every later wait, pack and unpack saw
    the dead exchange and returned at once), and a further gg_dist_step fails
    at once as well; rank 1 finishes cleanly."""
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, hip_lib, qq, (12, 4))) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, got = qq.get(timeout=120)
        assert not isinstance(got, str), got
        res[r] = got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    err1, err2, t_first, t_again = res[0]
    print(f"dead peer: first failure after {t_first:.3f} s, the next step's after {t_again:.3f} s")
    assert err1 is not None and "EIO" in err1 and "(1 wait(s) ran out" in err1, err1
    assert err2 is not None and "EIO" in err2, err2
    assert t_again < max(0.5, t_first / 2), (t_first, t_again)
    assert res[1][0] is None, res[1]
