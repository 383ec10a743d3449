"""Sharded (N > 1) path on CPU: world_size-2 gloo runs of the sharded round
protocol (ggamd.dist.ShardedRunner over gg_dist_round_begin/end) against the
same scenario on one unsharded engine. Counters summed over ranks, node sets
and delivery rounds of every rank's range must equal the single-engine run.
The engine here is the CPU oracle library; the GPU run of the same
orchestration uses the HIP library with the nccl (RCCL) backend.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import c1_scenario, diff_stats, make_engine, random_scenario


def _free_port():
    from helpers import free_port
    return free_port()


def _worker(rank, world, port, lib, sc, q, lane_groups=1):
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    os.environ["GG_CPU_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        import torch
        e = make_engine(lib, sc, rank=rank, world=world, lane_groups=lane_groups)
        r = ShardedRunner(e, torch.device("cpu"))
        stats = r.step(sc.rounds)
        owned = e.dist_owned()
        bits = e.read_bits_nodes(owned)
        dr = e.delivery_rounds_nodes(owned)
        q.put((rank, stats, owned, bits, dr))
    finally:
        dist.destroy_process_group()


def _run_dist(lib, sc, world=2, lane_groups=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, lib, sc, q, lane_groups)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


def _check(lib, sc, world=2):
    single = make_engine(lib, sc)
    s1 = single.step(sc.rounds)
    res = _run_dist(lib, sc, world)
    for rank, stats, owned, bits, dr in res:
        d = diff_stats(s1, stats)
        assert not d, (rank, d[:10])
        assert np.array_equal(bits, single.read_bits_nodes(owned))
        assert np.array_equal(dr, single.delivery_rounds_nodes(owned))
    allown = np.sort(np.concatenate([x[2] for x in res]))
    assert np.array_equal(allown, np.arange(sc.topo.n_nodes))  # a partition of the nodes


def _check_lanes(lib, sc, world, lane_groups):
    """2-D sharding: lane groups x vertex parts. Counters summed over every rank,
    node sets OR-ed and delivery rounds max-ed over the lane groups of a node's
    owners equal the single engine."""
    single = make_engine(lib, sc)
    s1 = single.step(sc.rounds)
    res = _run_dist(lib, sc, world, lane_groups)
    V = sc.topo.n_nodes
    bits = np.zeros((V, sc.W // 64), np.uint64)
    dr = np.full((V, sc.W), -1, np.int32)
    for rank, stats, owned, b, d in res:
        assert not diff_stats(s1, stats), (rank, diff_stats(s1, stats)[:10])
        o = owned.astype(np.int64)
        bits[o] |= b
        dr[o] = np.maximum(dr[o], d)
    assert np.array_equal(bits, single.read_bits())
    assert np.array_equal(dr, single.delivery_rounds())


@pytest.mark.parametrize("world,groups", [(2, 2), (3, 3), (4, 2)])
def test_lane_groups(cpu_lib, world, groups):
    rnd = random.Random(world * 10 + groups)
    sc = random_scenario(rnd, max_v=200, W=256, rounds=45)
    _check_lanes(cpu_lib, sc, world, groups)


def test_lane_groups_c1_partition(cpu_lib):
    _check_lanes(cpu_lib, c1_scenario(partition=True, rounds=120), 2, 2)


def test_c1_two_ranks(cpu_lib):
    _check(cpu_lib, c1_scenario(partition=True, rounds=120))


@pytest.mark.parametrize("seed", [1, 2])
def test_random_two_ranks(cpu_lib, seed):
    rnd = random.Random(seed)
    sc = random_scenario(rnd, max_v=300, W=128, rounds=50)
    _check(cpu_lib, sc)


def test_random_three_ranks(cpu_lib):
    rnd = random.Random(11)
    sc = random_scenario(rnd, max_v=200, W=64, rounds=45)
    _check(cpu_lib, sc, world=3)


def test_oracle_has_no_rccl(cpu_lib):
    """The CPU oracle exports the engine-owned exchange symbols but has no RCCL:
    each reports GG_EIO, so a caller falls back to its own collective."""
    from ggamd.engine import Engine, GGError
    e = Engine(16, 64, library=cpu_lib, rank=0, world=2)
    ok, why = e.dist_comm_available()
    assert not ok and "no RCCL" in why
    with pytest.raises(RuntimeError):
        e.dist_comm_id()
    with pytest.raises(GGError):
        e.dist_comm_init(bytes(128))
    with pytest.raises(GGError):
        e.dist_step(1)
    e.close()


def test_runner_transport_choice(cpu_lib):
    """ShardedRunner picks the engine-owned exchange only on nccl; gloo moves the
    payloads through the caller; an unknown transport name is an error."""
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    dist.init_process_group("gloo", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_free_port()}")
    try:
        e = Engine(16, 64, library=cpu_lib)
        r = ShardedRunner(e, torch_device_cpu())
        assert not r.engine_comm and r.transport == "gloo via host"
        with pytest.raises(ValueError):
            ShardedRunner(e, torch_device_cpu(), transport="mpi")
        e.close()
    finally:
        dist.destroy_process_group()


def torch_device_cpu():
    import torch
    return torch.device("cpu")


def test_edge_windows_two_ranks(cpu_lib):
    """gg_set_partition windows in a sharded job equal the single engine."""
    from helpers import symmetric_random_scenario
    sc = symmetric_random_scenario(random.Random(77), max_v=200, W=128, rounds=45)
    _check(cpu_lib, sc)
