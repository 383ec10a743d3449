#!/usr/bin/env python3
"""C4 sharded rehearsal on ONE GPU: world = lane_groups x parts ranks, every
rank an engine on cuda:0 holding one vertex range of the R-MAT graph (built
on the device, gg_topology_generate) for its lane group's lanes, the ghost
payloads moved through host memory with gloo. Measures what the 8-GPU job's
round time is made of and projects it:

  * per round and rank: kernel time (device clock stamps of the rank's own
    kernels; the ranks' kernels run one rank at a time, so no rank's time is
    inflated by another sharing the GPU), payload bytes sent and received;
  * per rank: owned rows, ghost rows, HBM bytes (free-memory delta of its
    setup, ranks set up one at a time);
  * the single engine over the whole graph on the same GPU: per-round kernel
    time, and every round's counters (summed over ranks) must equal it.

Projection: round r on N GPUs takes
    T_r = max_rank C_r + X_r / B          exchange after compute
    T_r = max(max_rank C_r, X_r / B)      exchange overlapped (lane halves)
with X_r the largest per-rank payload (max of sent, received) and B the
per-GPU exchange bandwidth over the P-1 peer links (--link-gbs per link and
direction). Printed as JSON.

Usage: python tools/c4_rehearsal.py --nodes 8388608 --parts 4 --lane-groups 2
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


def _worker(rank, world, port, args, q):
    import torch
    import torch.distributed as dist

    from ggamd.dist import ShardedRunner
    from ggamd.engine import COUNT_FIELDS, Engine
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections
    os.environ["GG_XCHG_MODE"] = "exact"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        V, K = args.nodes, args.lanes
        seed = BASE_SEED + 4
        gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
        hbm = 0
        eng = None
        for k in range(world):  # one rank at a time: a clean free-memory delta per rank
            if k == rank:
                torch.cuda.synchronize()
                f0 = torch.cuda.mem_get_info(0)[0]
                eng = Engine(V, K, seed=seed, enable_sync=True, device=0, rank=rank, world=world,
                             lane_groups=args.lane_groups)
                nnz = eng.generate(**gen)
                torch.cuda.synchronize()
                hbm = f0 - torch.cuda.mem_get_info(0)[0]
                print(f"rank {rank}: {hbm / 2**30:.2f} GiB, {eng.dist_info()}", flush=True)
            dist.barrier()
        info = eng.dist_info()
        runner = ShardedRunner(eng, dev, transport="torch")
        inject(eng, injection_arrays(uniform_injections(V, K, seed)))
        rounds = []
        while True:
            x = None
            for k in range(world):  # the ranks' kernels one rank at a time
                if k == rank:
                    x = eng.dist_round_begin()
                    torch.cuda.synchronize()
                dist.barrier()
            runner.exchange(x)
            recv = sum(int(x.recv_bytes[i]) for i in range(world))
            st = eng.dist_round_end(wait=True)
            st["recv_bytes"] = recv
            rounds.append(st)
            nb = torch.tensor([st["new_bits"]], dtype=torch.int64)
            dist.all_reduce(nb)
            if rank == 0:
                print(f"round {len(rounds) - 1}: new {int(nb)}, rank 0: {st['kernel_ms']:.2f} ms, "
                      f"sent {st['sent_bytes']} B, received {recv} B", flush=True)
            if (int(nb) == 0 and len(rounds) > 1) or len(rounds) >= args.max_rounds:
                break
        q.put((rank, {"rounds": rounds, "info": info, "hbm": hbm, "nnz_rank": nnz,
                      "fields": COUNT_FIELDS}))
        eng.close()
    except BaseException as exc:  # report instead of leaving the parent waiting
        q.put((rank, f"rank {rank} failed: {exc!r}"))
        raise
    finally:
        dist.destroy_process_group()


def _single(args, R):
    import torch

    from ggamd.engine import Engine
    from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections
    V, K = args.nodes, args.lanes
    seed = BASE_SEED + 4
    torch.cuda.synchronize()
    f0 = torch.cuda.mem_get_info(0)[0]
    e = Engine(V, K, seed=seed, enable_sync=True, device=0)
    nnz = e.generate(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    torch.cuda.synchronize()
    hbm = f0 - torch.cuda.mem_get_info(0)[0]
    inject(e, injection_arrays(uniform_injections(V, K, seed)))
    st = [e.step(1)[0] for _ in range(R)]  # round by round: per-round stamps
    e.close()
    return st, nnz, hbm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1 << 23)
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--parts", type=int, default=4)
    ap.add_argument("--lane-groups", type=int, default=2)
    ap.add_argument("--max-rounds", type=int, default=40)
    ap.add_argument("--link-gbs", type=float, default=64.0,
                    help="xGMI bandwidth per link and direction used in the projection (GB/s)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--single-only", type=int, default=0,
                    help="run only the single engine for this many rounds and print its per-round times")
    args = ap.parse_args()
    if args.single_only:
        st, nnz, hbm = _single(args, args.single_only)
        print(json.dumps({"nodes": args.nodes, "lanes": args.lanes, "order": os.environ.get("GG_ORDER", "auto"),
                          "nnz": nnz, "hbm_bytes": hbm, "round_ms": [s["kernel_ms"] for s in st],
                          "new_bits": [s["new_bits"] for s in st]}))
        return
    import torch.multiprocessing as mp
    world = args.parts * args.lane_groups
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t0 = time.time()
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got = q.get(timeout=1800)
        if isinstance(got, str):
            raise SystemExit(got)
        res[r] = got
        print(f"rank {r} done ({time.time() - t0:.0f} s)", flush=True)
    for p in procs:
        p.join(timeout=120)
    fields = res[0]["fields"]
    R = len(res[0]["rounds"])
    single, nnz, hbm1 = _single(args, R)
    M = (1 << 64) - 1
    bad = []
    for i in range(R):
        for f in fields:
            tot = sum(res[k]["rounds"][i][f] for k in range(world)) & M
            if tot != (single[i][f] & M):
                bad.append(f"round {i} {f}: sharded {tot} != single {single[i][f]}")
    B = args.link_gbs * 1e9 * min(7, max(1, args.parts - 1))
    per_round = []
    t1 = tn_seq = tn_ovl = 0.0
    for i in range(R):
        c1 = single[i]["kernel_ms"]
        cr = [res[k]["rounds"][i]["kernel_ms"] for k in range(world)]
        xs = [max(res[k]["rounds"][i]["sent_bytes"], res[k]["rounds"][i]["recv_bytes"]) for k in range(world)]
        xms = max(xs) / B * 1e3
        t1 += c1
        tn_seq += max(cr) + xms
        tn_ovl += max(max(cr), xms)
        per_round.append({"round": i, "new_bits": single[i]["new_bits"], "single_ms": c1,
                          "rank_ms_max": max(cr), "rank_ms_mean": sum(cr) / world,
                          "payload_bytes_max": max(xs), "payload_bytes_mean": sum(xs) / world,
                          "exchange_ms_at_B": xms})
    out = {
        "config": {"nodes": args.nodes, "lanes": args.lanes, "parts": args.parts, "lane_groups": args.lane_groups,
                   "world": world, "nnz": nnz, "graph": "R-MAT (.57,.19,.19,.05) ef16 (C4's generator)"},
        "check": "every round's counters summed over ranks equal the single engine" if not bad else bad[:10],
        "rounds": R,
        "ranks": [{"rank": k, **res[k]["info"], "hbm_bytes": res[k]["hbm"], "adjacency_entries": res[k]["nnz_rank"],
                   "payload_bytes_total": sum(s["sent_bytes"] for s in res[k]["rounds"])} for k in range(world)],
        "single_hbm_bytes": hbm1,
        "per_round": per_round,
        "projection": {
            "link_GBps_per_direction": args.link_gbs, "exchange_GBps_per_gpu": B / 1e9,
            "single_ms": t1, "sharded_ms_exchange_after_compute": tn_seq, "sharded_ms_overlapped": tn_ovl,
            "speedup_exchange_after_compute": t1 / tn_seq if tn_seq else None,
            "speedup_overlapped": t1 / tn_ovl if tn_ovl else None,
        },
    }
    js = json.dumps(out, indent=1)
    print(js)
    if args.out:
        with open(args.out, "w") as f:
            f.write(js)
    if bad:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
