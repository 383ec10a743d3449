#!/usr/bin/env python3
"""Per-round device time of sync rounds against dense lean rounds, streamed
(sync_records + expand_stream_sync, hub_sync_* on hub graphs) vs the tile path
(GG_SYNC_TILES=1), on the C4 generator (R-MAT, hubs) and the C5 generator
(grid + long links, W = 64), each run past the first sync timers. Both paths
must give the same counters every round.

Usage: python tools/sync_rounds.py [--rmat-nodes 2097152] [--grid-side 8192] [--rounds 34] [--json out]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))

from ggamd.engine import COUNT_FIELDS, Engine  # noqa: E402
from ggamd.workload import BASE_SEED, inject, injection_arrays, uniform_injections  # noqa: E402


def run(gen, V, K, rounds, tiles):
    os.environ["GG_SYNC_TILES"] = "1" if tiles else "0"
    e = Engine(V, K, seed=BASE_SEED + 4, enable_sync=True, device=0)
    e.generate(**gen)
    inject(e, injection_arrays(uniform_injections(V, K, BASE_SEED + 4)))
    st = [e.step(1)[0] for _ in range(rounds)]  # round by round: per-round stamps
    e.close()
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rmat-nodes", type=int, default=1 << 21)
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--grid-side", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=34)
    ap.add_argument("--json")
    args = ap.parse_args()
    out = {}
    cases = [("C4 R-MAT", dict(kind="rmat", n=args.rmat_nodes, k=16, seed=BASE_SEED + 4, a=0.57, b=0.19, c=0.19),
              args.rmat_nodes, args.lanes),
             ("C5 grid+links", dict(kind="grid_links", n=args.grid_side, seed=BASE_SEED + 5),
              args.grid_side ** 2, 64)]
    for name, gen, V, K in cases:
        res = {}
        for tiles in (False, True):
            res["tiles" if tiles else "streamed"] = run(gen, V, K, args.rounds, tiles)
        a, b = res["streamed"], res["tiles"]
        diffs = [f"round {x['round']} {f}" for x, y in zip(a, b) for f in COUNT_FIELDS if x[f] != y[f]]
        dense = [x["kernel_ms"] for x in a if x["syncs_fired"] == 0 and x["new_bits"] > 0]
        sync = [i for i, x in enumerate(a) if i >= 22]
        rec = {"nodes": V, "lanes": K, "same_counters": not diffs, "diffs": diffs[:5],
               "max_lean_round_ms": max(dense) if dense else None,
               "rounds": [{"round": i, "new_bits": a[i]["new_bits"], "syncs_fired": a[i]["syncs_fired"],
                           "pushes": a[i]["pushes"], "streamed_ms": a[i]["kernel_ms"], "tiles_ms": b[i]["kernel_ms"]}
                          for i in range(len(a))],
               "sync_rounds_streamed_ms_max": max(a[i]["kernel_ms"] for i in sync) if sync else None,
               "sync_rounds_tiles_ms_max": max(b[i]["kernel_ms"] for i in sync) if sync else None}
        out[name] = rec
        print(name, json.dumps({k: v for k, v in rec.items() if k != "rounds"}), flush=True)
        for r in rec["rounds"]:
            print(f"  round {r['round']:3d} new {r['new_bits']:>14d} fired {r['syncs_fired']:>9d} "
                  f"streamed {r['streamed_ms']:8.3f} ms  tiles {r['tiles_ms']:8.3f} ms", flush=True)
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
