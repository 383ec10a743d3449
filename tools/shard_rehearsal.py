#!/usr/bin/env python3
"""Vertex-sharded rehearsal on ONE GPU: N ranks (torch.distributed.run, gloo:
payloads staged through host memory) each build only their node range of a
generated graph on the device (gg_topology_generate -> gg_gen::shard_csr), run
one episode, and rank 0 then runs the same episode on one unsharded engine and
compares every round's counters (summed over ranks; seen_hash fingerprints
every node's set). Reports per rank: topology setup seconds, peak host RSS,
owned / ghost rows, HBM bytes (free-memory delta of its setup; the ranks set
up one at a time), payload bytes sent per round, and the episode time; and the
single engine's HBM bytes (BASELINE configs[4]: "HBM footprint per GPU").

Usage: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
         --master-addr 127.0.0.1 --master-port P tools/shard_rehearsal.py [--side 8192] [--json out.json]
"""
import argparse
import json
import os
import resource
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ggamd.dist import ShardedRunner  # noqa: E402
from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, uniform_injections  # noqa: E402


def rss_mb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=8192)
    ap.add_argument("--lanes", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=0, help="0: until the first quiet round (single engine)")
    ap.add_argument("--json")
    args = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    side, K = args.side, args.lanes
    V = side * side
    seed = BASE_SEED + 5
    gen = dict(kind="grid_links", n=side, seed=seed)
    inj = uniform_injections(V, K, seed)
    # the reference run first (rank 0): its round count bounds the sharded episode
    R = args.rounds
    want = None
    hbm1 = 0
    if rank == 0:
        torch.cuda.synchronize()
        f0 = torch.cuda.mem_get_info(0)[0]
        e1 = Engine(V, K, seed=seed, enable_sync=True, device=0)
        e1.generate(**gen)
        torch.cuda.synchronize()
        hbm1 = f0 - torch.cuda.mem_get_info(0)[0]
        print(f"single engine: {hbm1 / 2**30:.1f} GiB", flush=True)
        for n, v, r in inj:
            e1.broadcast(int(n), int(v), int(r))
        if not R:
            want = []
            while True:
                s = e1.step(1)[0]
                want.append(s)
                if s["new_bits"] == 0 and len(want) > 1:
                    break
            R = len(want)
        else:
            want = e1.step(R)
        e1.close()
        torch.cuda.synchronize()
    t = torch.tensor([R], dtype=torch.int64)
    dist.broadcast(t, 0)
    R = int(t.item())
    rss0 = rss_mb()
    e, setup_s, hbm = None, 0.0, 0
    for k in range(world):  # one rank at a time: a clean free-memory delta per rank
        if k == rank:
            torch.cuda.synchronize()
            f0 = torch.cuda.mem_get_info(0)[0]
            t0 = time.perf_counter()
            e = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=rank, world=world)
            e.generate(**gen)
            torch.cuda.synchronize()
            setup_s = time.perf_counter() - t0
            hbm = f0 - torch.cuda.mem_get_info(0)[0]
            print(f"rank {rank}: set up in {setup_s:.1f} s, {hbm / 2**30:.2f} GiB", flush=True)
        dist.barrier()
    info = e.dist_info()
    n_own, n_ghost, n_send = info["owned"], info["ghosts"], info["sent_per_round"]
    for n, v, r in inj:
        e.broadcast(int(n), int(v), int(r))
    runner = ShardedRunner(e, torch.device("cuda", 0))
    dist.barrier()
    t1 = time.perf_counter()
    got, sent = [], []
    for r in range(R):
        local = runner.step(1, reduce=False)
        sent.append(local[0]["sent_bytes"])
        got += runner.reduce(local)
        if rank == 0:
            print(f"round {r}: new {got[-1]['new_bits']}, rank 0 sent {sent[-1]} B", flush=True)
    episode_s = time.perf_counter() - t1
    me = {"rank": rank, "owned": n_own, "ghosts": n_ghost, "send_entries": n_send, "setup_s": setup_s,
          "hbm_bytes": hbm, "peak_rss_MB": rss_mb(), "rss_before_setup_MB": rss0, "episode_s": episode_s,
          "payload_bytes_per_round": sent, "payload_bytes_max_round": max(sent) if sent else 0}
    allr = [None] * world
    dist.all_gather_object(allr, me)
    if rank == 0:
        diffs = [f"round {a['round']} {f}" for a, b in zip(got, want) for f in COUNT_FIELDS if a[f] != b[f]]
        out = {"nodes": V, "lanes": K, "ranks": world, "rounds": R, "single_engine_hbm_bytes": hbm1,
               "per_rank": allr,
               "counters_equal_single": not diffs, "first_diffs": diffs[:5],
               "deliveries": sum(s["new_bits"] for s in got), "transport": "gloo (host-staged, one GPU)"}
        print(json.dumps(out), flush=True)
        if args.json:
            json.dump(out, open(args.json, "w"), indent=1)
        if diffs:
            sys.exit(1)
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
