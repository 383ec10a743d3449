#!/usr/bin/env python3
"""rocprofv3 PMC passes -> profiles/traffic.json (read by bench.py).

Usage: tools/traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <source note> [out] [config] [shape]

shape: JSON of the bench run the passes profiled, {"config", "nodes" (per GPU for
C2), "lanes", "world", "parts", "halves"}; bench.py uses the file only for a run
of exactly that shape (any other run reports traffic null).

FETCH_SIZE and WRITE_SIZE come from separate passes of the same command (they
cannot share a pass on gfx950). Per MI355X_MICROARCH.md (HBM section),
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950, so HBM
bytes per dispatch = 2 * FETCH_SIZE + WRITE_SIZE (kB = 1024 B).
"""
import collections
import csv
import json
import sys


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    f, w = load(sys.argv[1]), load(sys.argv[2])
    out = sys.argv[4] if len(sys.argv) > 4 else "profiles/traffic.json"
    ker = {}
    for k in f:
        fk = sum(f[k]) / len(f[k])
        wl = w.get(k, [])
        wk = sum(wl) / len(wl) if wl else 0.0
        ker[k] = {"dispatches": len(f[k]), "fetch_kB": fk, "write_kB": wk,
                  "traffic_bytes_per_dispatch": (2.0 * fk + wk) * 1024.0}
    cfg = sys.argv[5] if len(sys.argv) > 5 else "C2"
    default = {"C2": {"nodes": 1 << 20, "lanes": 1024}, "C4": {"nodes": 100_000_000, "lanes": 4096}}.get(cfg, {})
    shape = dict(config=cfg, world=1, parts=1, halves=1, **default)
    if len(sys.argv) > 6:
        shape.update(json.loads(sys.argv[6]))
    json.dump({"source": sys.argv[3], "config": cfg, "shape": shape,
               "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950)", "kernels": ker}, open(out, "w"), indent=1)
    for k, v in sorted(ker.items(), key=lambda kv: -kv[1]["traffic_bytes_per_dispatch"] * kv[1]["dispatches"]):
        print(f'{v["dispatches"]:5d} {v["traffic_bytes_per_dispatch"] / 1e6:10.2f} MB  {k[:90]}')


if __name__ == "__main__":
    main()
