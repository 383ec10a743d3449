#!/usr/bin/env python3
"""Emulate the ranks of an N-GPU lane-group job on one GPU, one after another.

With gg_config.lane_groups = N (bench.py --config C4) the ranks never exchange
anything during an episode: rank r holds the whole graph and lane words
[nw*r/N, nw*(r+1)/N) of every node, and the per-round counters are summed once
at the end. So an N-GPU episode takes max over ranks of the rank's own
episode time (plus one all_reduce of a few KB), and each rank can be timed on
its own here. Checks that the summed counters of the N ranks equal the N = 1
run round by round, and prints each rank's episode time, the emulated N-GPU
time and the speed-up over N = 1.

Usage: tools/lane_scaling.py [--nodes V] [--lanes K] [--ranks 1,2,4,8] [--steps S]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402


def run_rank(V, K, rank, world, steps, gen, inj, R=None):
    e = Engine(V, K, seed=BASE_SEED + 4, enable_sync=True, device=0, rank=rank, world=world,
               lane_groups=world)
    t = time.perf_counter()
    e.generate(**gen)
    gen_s = time.perf_counter() - t
    if R is None:
        inject(e, inj)
        R = 0
        while True:
            s = e.step(1)[0]
            R += 1
            if s["new_bits"] == 0 and R > 1:
                break
    e.reset()
    inject(e, inj)
    ref = e.step(R)
    times = []
    for _ in range(steps):
        e.reset()
        inject(e, inj)
        t = time.perf_counter()
        e.step(R, raw=True)
        times.append(time.perf_counter() - t)
    if os.environ.get("LANE_ROUNDS"):
        for s in ref:
            print(f"  r{s['round']:2d} new {s['new_bits']:12d} rows {s['work_rows']:10d} gathers {s['work_gathers']:11d} "
                  f"stream {s['stream_ms']:8.2f} ms {s['stream_bytes'] / 1e9:8.2f} GB prep {s['prep_ms']:.2f} ms",
                  flush=True)
    stream_ms = sum(s["stream_ms"] for s in ref)
    stream_b = sum(s["stream_bytes"] for s in ref)
    e.close()
    return R, ref, min(times), sum(times) / len(times), gen_s, stream_b / (stream_ms * 1e-3) / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000_000)
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--only-rank", type=int, help="time just this rank of each N (profiling)")
    ap.add_argument("--json")
    args = ap.parse_args()
    V, K = args.nodes, args.lanes
    gen = dict(kind="rmat", n=V, k=16, seed=BASE_SEED + 4, a=0.57, b=0.19, c=0.19)
    inj = injection_arrays(uniform_injections(V, K, BASE_SEED + 4))
    out = {"nodes": V, "lanes": K, "runs": {}}
    base = None
    R = None
    for N in [int(x) for x in args.ranks.split(",")]:
        tot, per = None, []
        for r in ([args.only_rank] if args.only_rank is not None else range(N)):
            R, st, best, mean, gen_s, gbps = run_rank(V, K, r, N, args.steps, gen, inj, R)
            per.append({"rank": r, "episode_s": mean, "best_s": best, "gen_s": gen_s, "stream_GBps": gbps})
            print(f"N={N} rank {r}: episode {mean * 1e3:.1f} ms (best {best * 1e3:.1f}), stream {gbps:.0f} GB/s, "
                  f"graph {gen_s:.1f} s", flush=True)
            if tot is None:
                tot = [dict(s) for s in st]
            else:
                for a, b in zip(tot, st):
                    for f in COUNT_FIELDS:
                        if f != "round":
                            a[f] = (a[f] + b[f]) & ((1 << 64) - 1)
        if args.only_rank is not None:
            continue
        if base is None:
            base = (tot, max(p["episode_s"] for p in per))
        diffs = [f"round {a['round']} {f}" for a, b in zip(tot, base[0]) for f in COUNT_FIELDS if a[f] != b[f]]
        t_n = max(p["episode_s"] for p in per)
        dl = sum(s["new_bits"] for s in tot)
        out["runs"][N] = {"ranks": per, "episode_s": t_n, "deliveries": dl, "deliveries_per_s": dl / t_n,
                          "speedup_vs_1": base[1] / t_n, "counters_equal_N1": not diffs}
        print(f"N={N}: emulated episode {t_n * 1e3:.1f} ms, {dl / t_n:.3e} deliveries/s, speed-up "
              f"{base[1] / t_n:.2f}x, counters {'equal' if not diffs else 'DIFFER ' + str(diffs[:4])}", flush=True)
    print(json.dumps(out))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
