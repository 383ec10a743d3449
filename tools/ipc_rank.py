#!/usr/bin/env python3
"""One rank of a sharded run on the one GPU of a box, started per rank from the
shell (so one rank can run under rocprofv3 as the program itself): world W
vertex parts of C2's tree (2^20 nodes per rank) or C4's R-MAT (--config C4,
--nodes), W = 2 by default, gloo for the rendezvous only. Each episode is one
gg_dist_step over R rounds (R = the single engine's quiescence round count)
and one flush. Prints, per transport, the host time to enqueue the episode
(gg_dist_step's return), the wall time to its end (flush) and the rank's
kernel time (device stamps), so a host wait per round shows as enqueue time
that grows with R.

Usage (one per rank):
  python tools/ipc_rank.py --rank 0 --world 2 --port 29612 [--transport ipc|engine] [--config C2|C4]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--port", type=int, default=29612)
    ap.add_argument("--transport", default="ipc", choices=["ipc", "engine"])
    ap.add_argument("--config", default="C2", choices=["C2", "C4"])
    ap.add_argument("--nodes", type=int, default=0)
    ap.add_argument("--episodes", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ggamd import topology as T
    from ggamd.dist import ShardedRunner
    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{args.port}", rank=args.rank,
                            world_size=args.world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W = args.world
    if args.config == "C2":
        V, K, seed = (args.nodes or (1 << 20)) * W, 1024, BASE_SEED + 2
        e = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=args.rank, world=W)
        e.topology(T.tree(V, 4))
    else:
        V, K, seed = args.nodes or (1 << 22), 4096, BASE_SEED + 4
        e = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=args.rank, world=W)
        e.generate(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    runner = ShardedRunner(e, dev, transport=args.transport if args.transport == "ipc" else "engine")
    inj = injection_arrays(uniform_injections(V, K, seed))

    def episode(R):
        e.reset()
        inject(e, inj)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        e.dist_step(R)
        t1 = time.perf_counter()
        st = e.dist_flush()
        t2 = time.perf_counter()
        return st, (t1 - t0) * 1e3, (t2 - t0) * 1e3

    # rounds to quiescence: single rounds until the global new-bit count is zero
    e.reset()
    inject(e, inj)
    R = 0
    while True:
        st = runner.step(1)
        R += 1
        if st[0]["new_bits"] == 0 and R > 1:
            break
    out = []
    for k in range(args.episodes + 1):
        st, enq, wall = episode(R)
        if k == 0:
            continue  # the first episode captures the launch sequence
        out.append({"enqueue_ms": enq, "wall_ms": wall, "kernel_ms": sum(s["kernel_ms"] for s in st),
                    "sent_bytes": sum(s["sent_bytes"] for s in st)})
    res = {"rank": args.rank, "world": W, "config": args.config, "nodes": V, "lanes": K, "rounds": R,
           "transport": runner.transport, "episodes": out,
           "enqueue_ms_per_round": min(o["enqueue_ms"] for o in out) / R,
           "wall_ms_per_episode": min(o["wall_ms"] for o in out)}
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    dist.barrier()
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
