#!/usr/bin/env python3
"""Benchmark: (node,msg) deliveries/s of the gossip-propagation engine.

One *step* = one full propagation episode: reset -> the clients' broadcasts ->
lockstep rounds until the round after the last delivery (quiescence, fixed
during warmup). `value` = all (node,msg) deliveries of the timed episodes on
all ranks / the max-over-ranks wall time.

--config C2 (default; BASELINE.json configs[1]): a 4-ary tree (Maelstrom
  `tree4`) of 2^20 nodes per GPU, K = 1024 fresh messages broadcast by clients
  at seeded uniform nodes in round 0, sync timers on, no partitions. On N GPUs
  the tree has N * 2^20 nodes, vertex-range sharded (locality order) with one
  exchange of ghost payloads per round ("scaling": "weak"): the engine's own
  grouped RCCL send/recv on its stream.
--config C4 (configs[3], the 100M-node config the >= 6x scaling target is
  quoted on): R-MAT (.57,.19,.19,.05), edge factor 16, 10^8 nodes, K = 4096
  messages in round 0. Strong scaling over a 2-D grid of ranks, N = L x P
  (--parts P, default 1): P vertex parts (each rank builds only its node range
  of the graph on its GPU, with ghost copies of the adjacent remote nodes, and
  exchanges one filtered ghost payload per round with the other parts of its
  lane group over RCCL) times L = N / P lane groups (each a slice of the 4096
  message lanes; lane groups never exchange anything). P = 1: every GPU holds
  the whole CSR and 4096/N lanes, no exchange at all. The per-round counters
  are summed with one all_reduce after the timed episodes.

N > 1: after the timed region rank 0 runs one episode of a single unsharded
engine over the whole graph on its own GPU and every round's global counters
must equal it, else the run exits with status 1.

Usage: python bench.py [--config C2|C4] [--parts P] [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
For N > 1 launch under torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gossip-glomers-distributed-systems_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

METRIC = "(node,msg) deliveries/sec at 1/2/4/8 GPUs; % of HBM roofline; msgs/op"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

KERNELS = {"prep": "round_prep", "expand": "expand_round", "stream": "expand_stream"}
# the kernels one round launches exactly one of, per kind (the launch count of a kind)
MAIN_KERNELS = {"prep": ["round_prep"], "expand": ["expand_round", "expand_round_lean"],
                "stream": ["expand_stream", "expand_stream_db", "expand_stream_masked", "expand_stream1",
                           "expand_stream_sync", "expand_batched"]}
# the kernels stamping each kind: a kind's "launch" is one round, so its
# counter traffic per launch is the sum over these kernels' dispatches per round
KIND_KERNELS = {
    "prep": ["round_prep", "compact_round", "mark_injections", "hub_mark", "sync_records"],
    "expand": ["expand_round", "expand_round_lean"],
    "stream": ["expand_stream", "expand_stream_db", "expand_stream_db_mark", "expand_stream_masked", "expand_stream1",
               "expand_stream_sync", "hub_chunks", "hub_finish", "hub_sync_chunks", "hub_sync_finish", "hub_sync_push",
               "expand_batched"],
}
TRAFFIC_JSON = {"C2": os.path.join(REPO, "profiles", "traffic.json"),  # committed PMC passes per config
                "C4": os.path.join(REPO, "profiles", "traffic_C4.json")}
CPU_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so")


def pmc_traffic(kind: str, shape: dict):
    """HBM bytes per round of a kernel kind from the committed rocprofv3 PMC
    passes (tools/traffic.py: FETCH_SIZE and WRITE_SIZE in separate passes over
    this same bench command, FETCH_SIZE doubled for gfx950): the sum over the
    kind's kernels of bytes x dispatches, per dispatch of its main kernel (one
    per round). None unless the passes profiled a run of exactly this shape
    (config, nodes, lanes, world, parts, halves): another run's traffic is not
    this run's."""
    path = TRAFFIC_JSON.get(shape["config"])
    try:
        d = json.load(open(path))
    except (OSError, ValueError, TypeError):
        return None, None
    if d.get("shape") != shape:
        return None, (f"{os.path.relpath(path, REPO)} profiled {d.get('shape')}, not this run's {shape}: "
                      "no counter traffic for this shape")
    base = lambda name: name.split("(")[0].split("<")[0].split("::")[-1]  # noqa: E731
    ents = {}
    for name, ent in d.get("kernels", {}).items():
        b = base(name)
        if b in KIND_KERNELS[kind]:
            e = ents.setdefault(b, [0.0, 0])
            e[0] += ent["traffic_bytes_per_dispatch"] * ent["dispatches"]
            e[1] += ent["dispatches"]
    launches = sum(ents[k][1] for k in MAIN_KERNELS[kind] if k in ents)
    if not launches:
        return None, None
    per_round = sum(v[0] for v in ents.values()) / launches
    return per_round, f'{os.path.relpath(path, REPO)} ({d.get("source", "")}; kernels {sorted(ents)})'


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


def cpu_counts():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return os.cpu_count() or 1, aff or 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=["C2", "C4"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, help="C2: nodes per GPU (2^20); C4: nodes (10^8)")
    ap.add_argument("--lanes", type=int, help="C2: 1024; C4: 4096")
    ap.add_argument("--parts", type=int, default=1, help="C4: vertex parts P (world = lane groups x P)")
    ap.add_argument("--halves", type=int, default=1, choices=[1, 2],
                    help="C4 with --parts > 1: 2 = two engines per GPU over the two halves of its lanes, "
                         "one half's exchange overlapping the other half's kernels (ggamd.dist.HalvesRunner)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fresh-sets", type=int, default=4,
                    help="N = 1: after the timed region, episodes rotating this many distinct seeded injection "
                         "sets (every step re-captures its launch graph and uploads its injections; 0: skip)")
    ap.add_argument("--no-check", action="store_true", help="skip the N > 1 single-engine check")
    ap.add_argument("--xchg", default=os.environ.get("GG_DIST_TRANSPORT", "auto"),
                    choices=["auto", "engine", "ipc", "torch"],
                    help="N > 1 exchange between vertex parts: engine = the engine's grouped RCCL send/recv; "
                         "ipc = device-driven (IPC-mapped peer windows, kernel flags, captured batches of rounds, "
                         "no host wait); torch = torch all_to_all; auto (default) = ipc on RCCL jobs when every "
                         "rank maps its peers and two validation rounds match O2, else engine")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 "
                    "(nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ggamd import topology as T
    from ggamd.engine import COUNT_FIELDS, Engine, stats_dict
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
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

    def barrier():
        if world > 1:
            if args.backend == "nccl":
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()
        torch.cuda.synchronize()

    def allreduce_i64(vals, op=None):
        t = torch.tensor(vals, dtype=torch.int64, device=device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
        return t.cpu().tolist()

    cfg = args.config
    free0 = torch.cuda.mem_get_info(local)[0]
    t_setup = time.perf_counter()

    def setup(xchg):
        runner = None
        if cfg == "C2":
            V = (args.nodes or (1 << 20)) * world
            K = args.lanes or 1024
            seed = BASE_SEED + 2
            topo = T.tree(V, 4)
            gen = None
            E = int(topo.nnz)
            eng = Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world)
            eng.topology(topo)
            engs = [eng]
            if world > 1:
                from ggamd.dist import ShardedRunner
                runner = ShardedRunner(eng, device, transport=xchg if args.backend == "nccl" or xchg == "ipc" else None)
            parallelism = f"vertex-range x{world}" if world > 1 else "single GPU"
            scaling = "weak"
            workload = ("C2: tree4 of 2^20 nodes per GPU, 1024 messages broadcast in round 0 at seeded uniform "
                        "nodes, sync on, no partitions; one step = one episode to quiescence")
        else:
            V = args.nodes or 100_000_000
            K = args.lanes or 4096
            seed = BASE_SEED + 4
            topo = None
            gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
            P = args.parts
            if world % P:
                raise SystemExit(f"--parts {P} does not divide the world size {world}")
            L = world // P
            if args.halves == 2 and P > 1:
                from ggamd.dist import HalvesRunner
                g, q = divmod(rank, P)
                engs = [Engine(V, K, seed=seed, enable_sync=True, device=local, rank=(2 * g + h) * P + q,
                               world=2 * world, lane_groups=2 * L) for h in range(2)]
                E = engs[0].generate(**gen)
                engs[1].generate(**gen)
                eng = engs[0]
                runner = HalvesRunner(engs, device, transport=xchg)
            else:
                eng = Engine(V, K, seed=seed, enable_sync=True, device=local, rank=rank, world=world,
                             lane_groups=L)
                E = eng.generate(**gen)  # this rank's rows of the graph, built in its GPU's HBM (gossip_gen.h)
                engs = [eng]
                if P > 1:
                    from ggamd.dist import ShardedRunner
                    runner = ShardedRunner(eng, device, transport=xchg if args.backend == "nccl" or xchg == "ipc" else "engine")
            if world == 1:
                parallelism = "single GPU"
            elif P == 1:
                parallelism = f"message lanes x{world} (every GPU: whole graph, {K // world} lanes)"
            else:
                parallelism = (f"{L} lane groups x {P} vertex parts (each GPU: 1/{P} of the nodes + ghosts, "
                               f"{K // L} lanes" + (", as two engines of half the lanes each, exchange of one "
                                                    "overlapping the other's kernels)" if len(engs) == 2 else ")"))
            scaling = "strong"
            workload = (f"C4: R-MAT (.57,.19,.19,.05) edge factor 16, symmetrized, {V} nodes, {K} messages "
                        "broadcast in round 0 at seeded uniform nodes, sync on, no partitions; graph built "
                        "in HBM by the on-device generator; one step = one episode to quiescence")

        return runner, V, K, seed, topo, gen, E, eng, engs, parallelism, scaling, workload

    # N > 1 exchange: "auto" = the device-driven one (no host wait, captured rounds)
    # if every rank can map its peers and two validation rounds through it finish
    # (their global counters equal O2's where tests/golden/bench_c2.json has them),
    # else the engine's RCCL send/recv, rebuilt from scratch on every rank
    xchg = args.xchg
    xchg_note = None
    if xchg == "auto":
        xchg = "ipc" if (world > 1 and (cfg == "C2" or args.parts > 1)) else "engine"
    if args.xchg == "auto" and xchg == "ipc":
        ok, built, got = 1, None, [0, 0]
        try:  # (every rank makes the same collective calls whatever fails)
            built = setup("ipc")
            rn, V0, K0, seed0, _, _, _, _, engs0, _, _, _ = built
            arr0 = injection_arrays(uniform_injections(V0, K0, seed0))
            for e in engs0:
                e.reset()
                inject(e, arr0)
            got = [s["new_bits"] for s in rn.step(2, reduce=False)]
            if os.environ.get("GG_BENCH_IPC_FAIL") == str(rank):  # test hook: the fallback path
                raise RuntimeError("GG_BENCH_IPC_FAIL")
        except Exception as exc:  # noqa: BLE001 — any failure: every rank falls back
            ok = 0
            print(f"bench: rank {rank}: device-driven exchange unavailable ({exc!r}); falling back", file=sys.stderr)
        v = allreduce_i64([1 - ok] + [int(x) for x in got])
        ok = v[0] == 0 and sum(v[1:]) > 0
        gold_p = os.path.join(REPO, "tests", "golden", "bench_c2.json")
        if ok and cfg == "C2" and os.path.exists(gold_p):
            g = next((g for g in json.load(open(gold_p))["runs"].values()
                      if g["nodes"] == built[1] and g["lanes"] == built[2]), None)
            if g is not None and v[1:] != [g["rounds"][0]["new_bits"], g["rounds"][1]["new_bits"]]:
                ok = False
                if rank == 0:
                    print(f"bench: device-driven validation rounds differ from O2: {v[1:]}; falling back",
                          file=sys.stderr)
        if ok:
            runner, V, K, seed, topo, gen, E, eng, engs, parallelism, scaling, workload = built
        else:
            if built is not None:
                for e in built[8]:
                    e.close()
            built = None
            torch.cuda.synchronize()
            xchg = "engine"
            xchg_note = "device-driven exchange failed its setup or validation on some rank: fell back to --xchg engine"
            runner, V, K, seed, topo, gen, E, eng, engs, parallelism, scaling, workload = setup(xchg)
    else:
        runner, V, K, seed, topo, gen, E, eng, engs, parallelism, scaling, workload = setup(xchg)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    inj = uniform_injections(V, K, seed)
    inj_arr = injection_arrays(inj)  # converted once, outside the timed loop

    def run_rounds(n):
        if runner is None:
            return eng.step(n, raw=True)  # dicts built after the timed region
        return runner.step(n, reduce=False)

    # warmup 0: the quiescence round R from per-round global counts
    for e in engs:
        e.reset()
        inject(e, inj_arr)
    R = 0
    while True:
        st = runner.step(1, reduce=False)[0] if runner else eng.step(1)[0]
        nb = st["new_bits"]
        if world > 1:  # sum over the ranks
            nb = allreduce_i64([nb])[0]
        R += 1
        if nb == 0 and R > 1:
            break
        if R > 400:
            raise RuntimeError("no quiescence within 400 rounds")
    torch.cuda.synchronize()
    # after the first episode: the engine's second set buffer (double-buffered
    # rounds) is allocated at its first step
    hbm_bytes = free0 - torch.cuda.mem_get_info(local)[0]

    event_ms = []

    def episode():
        for e in engs:
            e.reset()
            inject(e, inj_arr)
        st = run_rounds(R)
        if runner is None:
            event_ms.append(eng.step_device_ms())
        return st

    def quiescence_rounds(arrs):  # single engine: rounds to the round after the last delivery
        eng.reset()
        inject(eng, arrs)
        n = 0
        while True:
            n += 1
            if eng.step(1)[0]["new_bits"] == 0 and n > 1:
                return n
            if n > 400:
                raise RuntimeError("no quiescence within 400 rounds")

    for _ in range(max(0, args.warmup - 1)):
        episode()
    event_ms.clear()

    # one engine per rank (no vertex parts): the K episodes go back to back through
    # gg_run_episodes — each still a reset, the same client broadcasts and R rounds,
    # its counters read back and checked like the loop's — with one host wait, so
    # no host round trip idles the GPU between episodes (the loop of synchronous
    # reset/broadcast/step calls is timed beside it: per_call_ms_per_step)
    # (vertex parts: gg_dist_run_episodes over the device-driven exchange, every rank alike)
    dist_pipe = (runner is not None and getattr(runner, "can_run_episodes", False)
                 and os.environ.get("GG_BENCH_DIST_EPISODES", "1") != "0")
    pipelined = runner is None or dist_pipe
    if pipelined and args.warmup > 0:  # (its counter ring is allocated here)
        eng.reset()
        inject(eng, inj_arr)
        if dist_pipe:
            fail = 0
            try:
                runner.run_episodes(R, args.steps)
            except Exception as exc:  # noqa: BLE001 — every rank agrees below, then falls back
                fail = 1
                print(f"bench: rank {rank}: gg_dist_run_episodes failed ({exc!r}); timing synchronous calls",
                      file=sys.stderr)
            if allreduce_i64([fail])[0]:
                dist_pipe = False
                pipelined = False
        else:
            eng.run_episodes(R, args.steps, raw=True)
    barrier()
    t0 = time.perf_counter()
    local_stats = []
    if dist_pipe:
        eng.reset()
        inject(eng, inj_arr)
        local_stats = runner.run_episodes(R, args.steps)
    elif pipelined:
        eng.reset()
        inject(eng, inj_arr)
        arr = eng.run_episodes(R, args.steps, raw=True)
    else:
        for _ in range(args.steps):
            local_stats.append(episode())
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    per_call_ms = None
    if pipelined:
        if not dist_pipe:
            local_stats = [[arr[k * R + i] for i in range(R)] for k in range(args.steps)]
        ev_pipe = [eng.step_device_ms()] * args.steps
        barrier()
        c0 = time.perf_counter()
        for _ in range(args.steps):
            episode()
        barrier()
        per_call_ms = (time.perf_counter() - c0) / args.steps * 1e3
        event_ms[:] = ev_pipe
        if world > 1:
            per_call_ms = float(allreduce_i64([int(per_call_ms * 1e6)], dist.ReduceOp.MAX)[0]) / 1e6

    # fresh episodes (N = 1): every step broadcasts a different seeded value set, as
    # in a workload whose clients keep sending new values: the injections and each
    # round's offsets into them are uploaded again; the captured launch sequence
    # names neither, so it replays as long as the same rounds inject the same number
    # of lanes (a set with another round pattern would capture once more)
    fresh = None
    if world == 1 and args.fresh_sets > 0:
        sets = [injection_arrays(uniform_injections(V, K, seed + 7919 * (i + 1))) for i in range(args.fresh_sets)]
        rounds_of = [quiescence_rounds(a) for a in sets]
        n_fresh = max(args.fresh_sets, min(args.steps, 2 * args.fresh_sets))
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        fdl = 0
        for k in range(n_fresh):
            i = k % args.fresh_sets
            eng.reset()
            inject(eng, sets[i])
            st = eng.step(rounds_of[i], raw=True)
            fdl += sum(st[j].new_bits for j in range(rounds_of[i]))
        torch.cuda.synchronize()
        fdt = time.perf_counter() - f0
        fresh = {"sets": args.fresh_sets, "steps": n_fresh, "rounds_per_set": rounds_of,
                 "ms_per_step": fdt / n_fresh * 1e3, "deliveries_per_s": fdl / fdt,
                 "note": "each step uploads its own injection pairs and round offsets, then replays the "
                         "captured launch sequence, which reads both from device memory (the timed `value` "
                         "repeats one set, whose pairs stay resident)"}
    if runner is None:
        local_stats = [[stats_dict(a[i]) for i in range(R)] for a in local_stats]
    if world > 1:
        elapsed = float(allreduce_i64([int(elapsed * 1e9)], dist.ReduceOp.MAX)[0]) / 1e9
        per_ep = [reduce_counts(s, allreduce_i64, COUNT_FIELDS) for s in local_stats]
    else:
        per_ep = local_stats
    deliveries = sum(s["new_bits"] for ep in per_ep for s in ep)
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in per_ep[-1])

    # roofline of the dominant kernel: per-kind device times (first block start
    # to last block end of each launch, stamped by the kernels) and the bytes
    # each launch had to move (counted by the kernels); this rank's
    dinfo = None
    if runner is not None:
        dinfo = eng.dist_info()
        n_own = dinfo["owned"]
        if topo is not None:
            owned = eng.dist_owned().astype(np.int64)
            E_own = int((topo.row_ptr[owned + 1] - topo.row_ptr[owned]).sum())
        else:
            E_own = E  # generate() returned this rank's adjacency entries
    else:
        n_own, E_own = V, E
    nwp = next_pow2(K // 64 // (world // args.parts * len(engs) if cfg == "C4" else 1))
    rounds_local = [s for ep in local_stats for s in ep]
    kinds = {}
    for kind, name in KERNELS.items():
        ms = sum(s[kind + "_ms"] for s in rounds_local)
        by = sum(s[kind + "_bytes"] for s in rounds_local)
        if kind == "stream":  # one of the two per lean round (double-buffered rounds)
            name = "expand_stream / expand_stream_db"
        kinds[kind] = {"kernel": name, "launches": len(rounds_local), "total_ms": ms, "bytes": by,
                       "avg_launch_ms": ms / len(rounds_local),
                       "GBps": by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0}
    dom = max(kinds, key=lambda k: kinds[k]["total_ms"])
    D = kinds[dom]
    achieved = D["GBps"]
    shape = {"config": cfg, "nodes": V // world if cfg == "C2" else V, "lanes": K, "world": world,
             "parts": args.parts if cfg == "C4" else world, "halves": len(engs)}
    traffic, traffic_src = pmc_traffic(dom, shape)
    round_ms = sum(s["kernel_ms"] for s in rounds_local)
    round_bytes = sum(s["prep_bytes"] + s["expand_bytes"] + s["stream_bytes"] for s in rounds_local)
    xbytes = None
    if runner is not None:  # payload bytes this rank sent per round (mean over the timed rounds)
        xbytes = sum(s["sent_bytes"] for s in rounds_local) / len(rounds_local)

    # N > 1: the sharded job must reproduce one unsharded engine, round by round
    check = None
    if world > 1 and not args.no_check:
        bad = 0
        if rank == 0:
            for e in engs:
                e.close()  # free this rank's shard before building the whole graph
            ref = Engine(V, K, seed=seed, enable_sync=True, device=local)
            if gen is None:
                ref.topology(topo)
            else:
                ref.generate(**gen)
            inject(ref, inj_arr)
            want = ref.step(R)
            ref.close()
            diffs = [f"round {a['round']} {f}: sharded {a[f]} != single {b[f]}"
                     for a, b in zip(per_ep[-1], want) for f in COUNT_FIELDS if a[f] != b[f]]
            bad = len(diffs)
            if diffs:
                print("bench: sharded run differs from the single engine:", diffs[:8], file=sys.stderr)
        bad = allreduce_i64([bad])[0]
        check = "every round's global counters equal one unsharded engine" if bad == 0 else "FAILED"
        if bad:
            if world > 1:
                dist.destroy_process_group()
            raise SystemExit(1)

    # every timed episode's global counters against the CPU oracle O2's run of the
    # same workload (tests/golden/bench_c2.json, made by make_bench_golden.py for
    # 2^20 x N nodes); a differing episode fails the run
    oracle_check = None
    gold_p = os.path.join(REPO, "tests", "golden", "bench_c2.json")
    if cfg == "C2" and K == 1024 and seed == BASE_SEED + 2 and os.path.exists(gold_p):
        gold = next((g for g in json.load(open(gold_p))["runs"].values() if g["nodes"] == V and g["lanes"] == K),
                    None)
        if gold is not None:
            want = gold["rounds"]
            M = (1 << 64) - 1
            diffs = [f"episode {k} round {j} {f}: {ep[j][f] & M} != O2 {want[j][f] & M}"
                     for k, ep in enumerate(per_ep) for j in range(min(len(ep), len(want))) for f in COUNT_FIELDS
                     if (ep[j][f] & M) != (want[j][f] & M)]
            if len(want) != R:
                diffs.append(f"quiescence round count {R} != O2 {len(want)}")
            if diffs:
                if rank == 0:
                    print("bench: counters differ from O2:", diffs[:8], file=sys.stderr)
                if world > 1:
                    dist.destroy_process_group()
                raise SystemExit(1)
            oracle_check = (f"all {len(per_ep)} timed episodes: every round's global counters and delivery hash "
                            f"equal O2's run of this workload (tests/golden/bench_c2.json, {V} nodes)")

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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic (seeded {'tree4' if cfg == 'C2' else 'R-MAT'} topology, seeded client broadcasts)",
            "config": {
                "workload": workload,
                "nodes": V, "edges": E, "lanes": K, "rounds_per_step": R,
                "deliveries_per_step": deliveries // args.steps,
                "inter_node_msgs_per_step": msgs,
                "msgs_per_op": msgs / K,
                "parallelism": parallelism,
                "exchange": (runner.transport if runner is not None else
                             ("none: lane groups never exchange; one all_reduce of the counters "
                              "after the timed episodes" if world > 1 else None)),
                "exchange_note": xchg_note,
                "lane_groups": world // args.parts if cfg == "C4" else 1,
                "vertex_parts": args.parts if cfg == "C4" else world,
                "exchange_bytes_per_round_rank0": xbytes,
                "shard": dinfo,
                "hbm_bytes_rank0": hbm_bytes,
                "setup_s_rank0": setup_s,
                "check": check,
                "oracle_check": oracle_check,
                "timed_loop": (("gg_dist_run_episodes" if dist_pipe else "gg_run_episodes") + ": the K episodes (each a reset, the same client broadcasts and "
                               "R rounds, its counters read back) queued back to back, one host wait; "
                               "roofline.per_call_ms_per_step times the same episodes as K synchronous "
                               "reset/broadcast/step calls" if pipelined else
                               "one synchronous reset/broadcast/step call sequence per episode"),
                "fresh_injections": fresh,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": D["kernel"],
                "kind": dom,
                "kind_kernels": "every kernel stamping this kind per round: " + ", ".join(KIND_KERNELS[dom]),
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
                "kernels": {k: dict(d) for k, d in kinds.items()},
                "round_GBps": round_bytes / (round_ms * 1e-3) / 1e9 if round_ms > 0 else 0.0,
                "event_ms_per_step": (sum(event_ms) / len(event_ms)) if event_ms else None,
                "per_call_ms_per_step": per_call_ms,
                "stamp_ms_per_step": round_ms / args.steps,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline and os.path.exists(CPU_LIB):
            out["cpu_baseline"] = cpu_baseline(cfg, topo, inj, V, K, seed, R)
        print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()


def reduce_counts(stats, allreduce_i64, fields):
    """Sum one episode's per-round counters over the ranks (seen_hash mod 2^64)."""
    M = (1 << 64) - 1
    flat = []
    for s in stats:
        for f in fields:
            v = s[f] & M
            flat.append(v - (1 << 64) if v >= (1 << 63) else v)
    tot = allreduce_i64(flat)
    out, k = [], 0
    for s in stats:
        d = dict(s)
        for f in fields:
            d[f] = tot[k] & M
            k += 1
        out.append(d)
    return out


def cpu_baseline(cfg, topo, inj, V, K, seed, R):
    """The oracle restatements on this host's cores (reported beside the GPU
    number, not the target). Legs: O2 (bitset, C++) on the box's CPU share, O2
    on one thread, and O1 (message-level literal restatement of the handlers,
    Python) on C1 per inter-node message — the cost of the reference's own
    per-message Send/handler path in kind. Each leg is a bounded sample."""
    from ggamd import topology as T
    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, uniform_injections
    host_cpus, affinity = cpu_counts()
    # the CPU share this process is given: the runtime's declared thread budget
    # (OMP_NUM_THREADS: the GPU box's per-GPU share of its host cores), else every
    # core this process may run on
    share = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(int(share), affinity)) if share and share.isdigit() else affinity
    basis = "OMP_NUM_THREADS (the declared per-GPU CPU share)" if share and share.isdigit() else \
        "sched_getaffinity (every core this process may use)"

    def o2_episodes(topo_, inj_, V_, K_, seed_, thr, budget_s, rounds=None):
        os.environ["GG_CPU_THREADS"] = str(thr)
        e = Engine(V_, K_, seed=seed_, enable_sync=True, library=CPU_LIB)
        e.topology(topo_)
        dl, eps, t0 = 0, 0, time.perf_counter()
        while True:
            e.reset()
            inject(e, inj_)
            if rounds is None:  # to quiescence
                r = 0
                while True:
                    s = e.step(1)[0]
                    dl += s["new_bits"]
                    r += 1
                    if s["new_bits"] == 0 and r > 1:
                        break
                rounds = r
            else:
                dl += sum(s["new_bits"] for s in e.step(rounds))
            eps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        dt = time.perf_counter() - t0
        e.close()
        return dl / dt, eps, rounds, dt

    if cfg == "C2":
        v_all, n_all, r_all, _ = o2_episodes(topo, inj, V, K, seed, threads, 8.0, R)
        sample_all = f"{n_all} full C2 episodes ({r_all} rounds each)"
        v_one, n_one, r_one, _ = o2_episodes(topo, inj, V, K, seed, 1, 6.0, R)
        sample_one = f"{n_one} full C2 episode(s) on one thread"
    else:  # C4: R-MAT samples of the same generator (the 10^8-node graph needs ~150 GB of host state)
        Va = 1 << 20
        ta = T.rmat(Va, 16, seed=seed)
        v_all, n_all, r_all, _ = o2_episodes(ta, uniform_injections(Va, K, seed), Va, K, seed, threads, 1.0)
        sample_all = f"{n_all} episode(s) to quiescence ({r_all} rounds) of the same R-MAT generator at 2^20 nodes"
        V1 = 1 << 17
        t1 = T.rmat(V1, 16, seed=seed)
        v_one, n_one, r_one, _ = o2_episodes(t1, uniform_injections(V1, K, seed), V1, K, seed, 1, 1.0)
        sample_one = f"{n_one} episode(s) ({r_one} rounds) of the R-MAT generator at 2^17 nodes on one thread"
    o1 = o1_c1_leg()
    return {"value": v_all, "unit": "deliveries/s", "cores": threads, "kind": "port",
            "sample": f"O2 bitset oracle (oracle/o2_bitset.cpp, -O3, AVX-512 host) on {threads} threads: "
                      f"{sample_all}",
            "host_cpus": host_cpus, "affinity_cpus": affinity, "cores_basis": basis,
            "single_thread": {"value": v_one, "unit": "deliveries/s", "cores": 1, "sample": sample_one},
            "o1_per_message": o1}


def o1_c1_leg():
    """O1 (oracle/o1_literal.py: every Send/Reply/RPC a message object through an
    in-memory network, handlers restated statement by statement) on config C1:
    inter-node messages and deliveries per second of one thread."""
    sys.path.insert(0, REPO)
    from oracle.o1_literal import O1Network
    from ggamd.workload import c1
    wl, _ = c1()
    o = O1Network(25, wl.n_lanes, wl.seed, wl.sync_base, wl.sync_jitter, wl.enable_sync)
    o.topology(wl.topo.rows())
    for n, v, r in wl.injections:
        o.broadcast(int(n), int(v), int(r))
    t0 = time.perf_counter()
    st = o.step(wl.max_rounds)
    dt = time.perf_counter() - t0
    msgs = sum(s["fwd_sent"] + s["pushes"] + s["acks"] + s["reads"] + s["read_oks"] for s in st)
    dl = sum(s["new_bits"] for s in st)
    return {"value": msgs / dt, "unit": "inter-node messages/s", "cores": 1,
            "deliveries_per_s": dl / dt, "messages": msgs, "seconds": dt,
            "sample": f"C1 (25-node tree4, {len(wl.injections)} client broadcasts over 200 rounds, sync on), "
                      f"{wl.max_rounds} rounds through O1's message-level network"}


if __name__ == "__main__":
    main()
