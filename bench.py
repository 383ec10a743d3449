#!/usr/bin/env python3
"""Benchmark: (node,msg) deliveries/s of the gossip-propagation engine.

One *step* = one full propagation episode of config C2 (BASELINE.json
configs[1]): a 4-ary tree (Maelstrom `tree4`) of 2^20 nodes per GPU, K = 1024
fresh messages broadcast by clients at seeded uniform nodes in round 0, sync
timers on, no partitions; the episode is reset -> inject -> lockstep rounds
until the round after the last delivery (quiescence, fixed during warmup).
`value` = all (node,msg) deliveries of the timed episodes on all ranks / the
max-over-ranks wall time. On N GPUs the tree has N * 2^20 nodes, vertex-range
sharded (locality order), with one exchange of ghost payloads per round ("scaling":
"weak"): the engine's own grouped RCCL send/recv on its stream (checked once
against torch's all_to_all_single during warmup, which it falls back to on a
mismatch; GG_DIST_TRANSPORT=torch forces that), named in config["exchange"].

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
For N > 1 launch under torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "gossip-glomers-distributed-systems_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

METRIC = "(node,msg) deliveries/sec at 1/2/4/8 GPUs; % of HBM roofline; msgs/op"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


KERNELS = {"prep": "round_prep", "expand": "expand_round", "stream": "expand_stream"}
TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic.json")


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/traffic.py: FETCH_SIZE and WRITE_SIZE in separate passes over this
    same bench command, FETCH_SIZE doubled for gfx950). None if not profiled."""
    try:
        import json as _j
        d = _j.load(open(TRAFFIC_JSON))
    except (OSError, ValueError):
        return None, None
    for name, ent in d.get("kernels", {}).items():
        if name.split("(")[0].split("<")[0].split("::")[-1] == kernel:
            return ent["traffic_bytes_per_dispatch"], f'{os.path.relpath(TRAFFIC_JSON, REPO)} ({d.get("source", "")})'
    return None, None


def dense_bytes_per_round(V: int, E: int, nwp: int) -> int:
    """SURVEY.md §8d dense-pull bytes of one round: row_ptr 8(V+1) + col 4E +
    every sender row gathered E*w + read seen, write seen, write F 3*V*w."""
    w = 8 * nwp
    return 8 * (V + 1) + 4 * E + E * w + 3 * V * w


def next_pow2(x: int) -> int:
    p = 1
    while p < x:
        p <<= 1
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--lanes", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-episodes", type=int, default=2)
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 "
                    "(nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ggamd import topology as T
    from ggamd.engine import Engine
    from ggamd.engine import stats_dict
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    if args.backend == "gloo":  # rehearsal: every rank on the one visible GPU
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)

    V = args.nodes_per_gpu * world
    K = args.lanes
    seed = BASE_SEED + 2
    topo = T.tree(V, 4)
    inj = uniform_injections(V, K, seed)
    inj_arr = injection_arrays(inj)  # converted once, outside the timed loop
    eng = Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world)
    eng.topology(topo)
    runner = None
    if world > 1:
        from ggamd.dist import ShardedRunner
        runner = ShardedRunner(eng, device)

    def barrier():
        if world > 1:
            if args.backend == "nccl":
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()
        torch.cuda.synchronize()

    def run_rounds(n):
        if runner is None:
            return eng.step(n, raw=True)  # dicts built after the timed region
        return runner.step(n, reduce=False)

    # warmup 0: find the quiescence round with per-round global counts (sharded:
    # over torch's all_to_all_single, the reference for the engine exchange check)
    engine_xch = runner is not None and runner.engine_comm
    if engine_xch:
        runner.engine_comm = False
    eng.reset()
    inject(eng, inj)
    R = 0
    ref = []
    while True:
        st = runner.step(1)[0] if runner else eng.step(1)[0]
        ref.append(st)
        R += 1
        if st["new_bits"] == 0 and R > 1:
            break
        if R > 400:
            raise RuntimeError("no quiescence within 400 rounds")
    if engine_xch:
        # one episode over the engine-owned RCCL exchange must reproduce every
        # round's global counters; the reduced counts are identical on every
        # rank, so all ranks take the same decision
        from ggamd.engine import COUNT_FIELDS
        runner.engine_comm = True
        eng.reset()
        inject(eng, inj)
        chk = runner.step(R)
        if any(a[f] != b[f] for a, b in zip(ref, chk) for f in COUNT_FIELDS):
            runner.engine_comm = False
            runner.transport = "torch all_to_all_single (engine exchange failed its check)"
            if rank == 0:
                print("bench: engine RCCL exchange disagrees with all_to_all_single; using torch",
                      file=sys.stderr)

    event_ms = []

    def episode():
        eng.reset()
        inject(eng, inj_arr)
        st = run_rounds(R)
        if runner is None:
            event_ms.append(eng.step_device_ms())
        return st

    for _ in range(max(0, args.warmup - 1)):
        episode()
    event_ms.clear()

    barrier()
    t0 = time.perf_counter()
    local_stats = []
    for _ in range(args.steps):
        local_stats.append(episode())
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if runner is None:
        local_stats = [[stats_dict(a[i]) for i in range(R)] for a in local_stats]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_ep = [runner.reduce(s) for s in local_stats]
    else:
        per_ep = local_stats
    deliveries = sum(s["new_bits"] for ep in per_ep for s in ep)
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"]
               for s in per_ep[-1])
    # roofline of the dominant kernel: per-kind device times (first block start
    # to last block end of each launch, stamped by the kernels) and the bytes
    # each launch had to move (counted by the kernels)
    dinfo = eng.dist_info() if world > 1 else None
    if world > 1:
        owned = eng.dist_owned().astype(np.int64)
        n_own = int(owned.size)
        E_own = int((topo.row_ptr[owned + 1] - topo.row_ptr[owned]).sum())
    else:
        n_own, E_own = V, int(topo.nnz)
    nwp = next_pow2(K // 64)
    rounds_local = [s for ep in local_stats for s in ep]
    kinds = {}
    for kind, name in KERNELS.items():
        ms = sum(s[kind + "_ms"] for s in rounds_local)
        by = sum(s[kind + "_bytes"] for s in rounds_local)
        kinds[kind] = {"kernel": name, "launches": len(rounds_local), "total_ms": ms, "bytes": by,
                       "avg_launch_ms": ms / len(rounds_local),
                       "GBps": by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0}
    dom = max(kinds, key=lambda k: kinds[k]["total_ms"])
    D = kinds[dom]
    achieved = D["GBps"]
    traffic, traffic_src = pmc_traffic(D["kernel"])
    round_ms = sum(s["kernel_ms"] for s in rounds_local)
    round_bytes = sum(s["prep_bytes"] + s["expand_bytes"] + s["stream_bytes"] for s in rounds_local)

    if rank == 0:
        value = deliveries / elapsed
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "deliveries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded tree4 topology, seeded client broadcasts)",
            "config": {
                "workload": "C2: tree4 of 2^20 nodes per GPU, 1024 messages broadcast in round 0 "
                            "at seeded uniform nodes, sync on, no partitions; one step = one "
                            "episode to quiescence",
                "nodes": V, "edges": int(topo.nnz), "lanes": K, "rounds_per_step": R,
                "deliveries_per_step": deliveries // args.steps,
                "inter_node_msgs_per_step": msgs,
                "msgs_per_op": msgs / K,
                "parallelism": f"vertex-range x{world}" if world > 1 else "single GPU",
                "exchange": runner.transport if runner is not None else None,
                "shard": dinfo,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": D["kernel"],
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": D["bytes"] / D["launches"],
                "avg_launch_ms": D["avg_launch_ms"],
                "launches": D["launches"],
                "dense_bytes_per_round": dense_bytes_per_round(n_own, E_own, nwp),
                "timing": "per launch: device clock (s_memrealtime) from the first block start to the last "
                          "block end of that kernel, stamped by every block (no-op launches included, as in "
                          "rocprofv3's average); cross-check: HIP events around each step's launch sequence "
                          "on the engine stream",
                "kernels": {k: {kk: v for kk, v in d.items()} for k, d in kinds.items()},
                "round_GBps": round_bytes / (round_ms * 1e-3) / 1e9 if round_ms > 0 else 0.0,
                "event_ms_per_step": (sum(event_ms) / len(event_ms)) if event_ms else None,
                "stamp_ms_per_step": round_ms / args.steps,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(topo, inj, V, K, seed, R, args.cpu_episodes)
        print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()


def cpu_baseline(topo, inj, V, K, seed, R, episodes):
    """The O2 bitset oracle (same semantics, CPU restatement of the reference
    handlers) timed on this host's cores over `episodes` full C2 episodes."""
    from ggamd.engine import Engine
    from ggamd.workload import inject
    lib = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")
    if not os.path.exists(lib):
        return None
    threads = min(16, os.cpu_count() or 1)
    os.environ["GG_CPU_THREADS"] = str(threads)
    e = Engine(V, K, seed=seed, enable_sync=True, library=lib)
    e.topology(topo)
    dl = 0
    t0 = time.perf_counter()
    for _ in range(episodes):
        e.reset()
        inject(e, inj)
        dl += sum(s["new_bits"] for s in e.step(R))
    dt = time.perf_counter() - t0
    return {"value": dl / dt, "unit": "deliveries/s", "cores": threads, "kind": "port",
            "sample": f"{episodes} full C2 episodes ({R} rounds each) of the O2 bitset oracle"}


if __name__ == "__main__":
    main()
