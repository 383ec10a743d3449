#!/usr/bin/env python3
"""Per-round device times of one episode of a generated bench leg (C3/C4/C5 at
any size), single engine, from the kernels' own stamps: where a leg's episode
goes, round by round (kernel ms, prep / stream split, new bits, active rows,
gathers, the round's path bits).

Usage: python tools/leg_rounds.py C5 [--side 32768] [--rounds 19]
       python tools/leg_rounds.py C4 [--nodes 100000000] [--rounds 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gossip-glomers-distributed-systems_amd")]
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=["C4", "C5"])
    ap.add_argument("--side", type=int, default=32768)
    ap.add_argument("--nodes", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=None)
    args = ap.parse_args()
    if args.leg == "C5":  # bench.py's legs
        side = args.side
        V, K, seed = side * side, 64, BASE_SEED + 5
        gen = dict(kind="grid_links", n=side, seed=seed)
    else:
        V, K, seed = args.nodes, 4096, BASE_SEED + 4
        gen = dict(kind="rmat", n=V, k=16, seed=seed, a=0.57, b=0.19, c=0.19)
    args.rounds = args.rounds or (19 if args.leg == "C5" else 10)
    e = Engine(V, K, seed=seed, enable_sync=True, device=0)
    e.generate(**gen)
    inj = injection_arrays(uniform_injections(V, K, seed))
    for _ in range(2):
        e.reset()
        inject(e, inj)
        st = e.step(args.rounds)
    tot = 0.0
    for s in st:
        tot += s["kernel_ms"]
        print(f'r{s["round"]:3d} ms={s["kernel_ms"]:8.3f} prep={s["prep_ms"]:7.3f} stream={s["stream_ms"]:8.3f} '
              f'new={s["new_bits"]:>12d} active={s["work_rows"]:>11d} gathers={s["work_gathers"]:>11d} '
              f'sGB={s["stream_bytes"] / 1e9:7.2f} path={s.get("path", 0):#x}', flush=True)
    print(f"total kernel ms {tot:.3f}")
    e.close()


if __name__ == "__main__":
    main()
