#!/usr/bin/env python3
"""C4's exchange payload over the device-driven exchange, with and without
need bits (expand_kernels.hpp NeedWord), on ONE GPU: world = parts ranks (one
process each, gloo rendezvous), every rank a device-built vertex part of the
R-MAT graph, windows IPC-mapped, tile segments. Per round and rank: the payload
bytes it packed into its peers' windows (sent_bytes). The kernels of the ranks
share the GPU here, so their times are not the N-GPU times (tools/c4_rehearsal.py
times them one rank at a time); the bytes are exact. Every round's counters,
summed over the ranks, are checked against one unsharded engine.

Output JSON: per round the largest per-rank payload with and without need bits,
and the densest round's; tools/project_c4.py --payload-json takes the "need"
payloads in place of its rehearsal's.

Usage: python tools/c4_ipc_payload.py --nodes 16777216 --parts 8 --out profiles/r6/c4_ipc_payload_2p24_p8.json
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gossip-glomers-distributed-systems_amd")
sys.path[:0] = [REPO, PKG]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, args, need, q):
    os.environ["GG_NEED_BITS"] = "1" if need else "0"
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        V, K = args.nodes, args.lanes
        seed = BASE_SEED + 4
        eng = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=rank, world=world)
        eng.generate(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
        runner = ShardedRunner(eng, dev, transport="ipc")
        inject(eng, injection_arrays(uniform_injections(V, K, seed)))
        rounds = []
        for _ in range(args.rounds):
            st = runner.step(1, reduce=False)[0]
            rounds.append(st)
        info = eng.dist_info()
        runner.close()
        eng.close()
        q.put((rank, {"rounds": rounds, "info": info}))
    except BaseException as exc:  # report instead of leaving the parent waiting
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


def run(args, need):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, args.parts, port, args, need, q)) for r in range(args.parts)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(args.parts):
        r, got = q.get(timeout=900)
        if isinstance(got, str):
            raise SystemExit(got)
        res[r] = got
    for p in procs:
        p.join(timeout=120)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1 << 24)
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    t0 = time.time()
    from ggamd.engine import COUNT_FIELDS
    runs = {}
    for need in (True, False):
        runs["need" if need else "all"] = run(args, need)
        print(f"{'need bits' if need else 'every F row'}: done ({time.time() - t0:.0f} s)", flush=True)
    # the single engine (this process; the ranks have exited)
    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections
    seed = BASE_SEED + 4
    e = Engine(args.nodes, args.lanes, seed=seed, enable_sync=True, device=0)
    e.generate(kind="rmat", n=args.nodes, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    inject(e, injection_arrays(uniform_injections(args.nodes, args.lanes, seed)))
    single = e.step(args.rounds)
    e.close()
    M = (1 << 64) - 1
    bad = []
    for name, res in runs.items():
        for i in range(args.rounds):
            for f in COUNT_FIELDS:
                tot = sum(res[k]["rounds"][i][f] for k in range(args.parts)) & M
                if tot != (single[i][f] & M):
                    bad.append(f"{name}: round {i} {f}: sharded {tot} != single {single[i][f]}")
    per_round = []
    for i in range(args.rounds):
        row = {"round": i, "new_bits": single[i]["new_bits"]}
        for name, res in runs.items():
            xs = [res[k]["rounds"][i]["sent_bytes"] for k in range(args.parts)]
            row[f"payload_bytes_max_{name}"] = max(xs)
            row[f"payload_bytes_sum_{name}"] = sum(xs)
        per_round.append(row)
    dens = {name: max(r[f"payload_bytes_max_{name}"] for r in per_round) for name in runs}
    out = {"config": {"nodes": args.nodes, "lanes": args.lanes, "parts": args.parts, "rounds": args.rounds,
                      "exchange": "device-driven (IPC windows, tile segments), ranks sharing one GPU",
                      "graph": "R-MAT (.57,.19,.19,.05) ef16 (C4's generator), lean digest with component targets"},
           "check": "every round's counters summed over ranks equal the single engine, with and without need bits"
                    if not bad else bad[:10],
           "densest_round_payload_bytes_per_rank": dens,
           "total_payload_bytes": {name: sum(r[f"payload_bytes_sum_{name}"] for r in per_round) for name in runs},
           "per_round": per_round}
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        open(args.out, "w").write(s)
    if bad:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
