#!/usr/bin/env python3
"""rocprofv3 PMC passes -> profiles/traffic*.json (read by bench.py).

Usage: tools/traffic.py FETCH_CSV WRITE_CSV SOURCE_NOTE [OUT] [CONFIG] [SHAPE_JSON] [--req REQ_CSV]

FETCH_CSV / WRITE_CSV: counter_collection.csv of a `--pmc FETCH_SIZE` and a
`--pmc WRITE_SIZE` pass over the same bench command (they cannot share a pass
on gfx950). REQ_CSV (optional): a third pass with `--pmc TCC_EA0_RDREQ_sum
TCC_EA0_WRREQ_sum` — the L2's memory-side read and write requests, the unit
of the random-row request ceiling (tools/gather_bench.hip; bench.py's
line_frac).

shape: JSON of the bench run the passes profiled, {"config", "nodes" (per GPU for
C2), "lanes", "world", "parts", "halves"}; bench.py uses the file only for a run
of exactly that shape (any other run reports traffic null).

Per MI355X_MICROARCH.md (HBM section), FETCH_SIZE reports half the bytes of
wide coalesced reads on gfx950, so HBM bytes per dispatch = 2 * FETCH_SIZE +
WRITE_SIZE (kB = 1024 B).
"""
import collections
import csv
import json
import sys


def load(path, counter=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter is None or r.get("Counter_Name", "").startswith(counter):
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(xs):
    return sum(xs) / len(xs) if xs else 0.0


def main():
    argv = list(sys.argv[1:])
    req = None
    if "--req" in argv:
        i = argv.index("--req")
        req = argv[i + 1]
        del argv[i:i + 2]
    f, w = load(argv[0]), load(argv[1])
    out = argv[3] if len(argv) > 3 else "profiles/traffic.json"
    rd = load(req, "TCC_EA0_RDREQ") if req else {}
    wr = load(req, "TCC_EA0_WRREQ") if req else {}
    ker = {}
    for k in f:
        fk = mean(f[k])
        wk = mean(w.get(k, []))
        ker[k] = {"dispatches": len(f[k]), "fetch_kB": fk, "write_kB": wk,
                  "traffic_bytes_per_dispatch": (2.0 * fk + wk) * 1024.0}
        if req:
            ker[k]["rd_requests_per_dispatch"] = mean(rd.get(k, []))
            ker[k]["wr_requests_per_dispatch"] = mean(wr.get(k, []))
    cfg = argv[4] if len(argv) > 4 else "C2"
    default = {"C2": {"nodes": 1 << 20, "lanes": 1024}, "C3": {"nodes": 10_000_000, "lanes": 1024},
               "C4": {"nodes": 100_000_000, "lanes": 4096},
               "C5": {"nodes": 1 << 30, "lanes": 64}}.get(cfg, {})
    shape = dict(config=cfg, world=1, parts=1, halves=1, **default)
    if len(argv) > 5:
        shape.update(json.loads(argv[5]))
    doc = {"source": argv[2], "config": cfg, "shape": shape,
           "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950)", "kernels": ker}
    if req:
        doc["requests"] = "TCC_EA0_RDREQ_sum / TCC_EA0_WRREQ_sum per dispatch (memory-side requests of the L2)"
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in sorted(ker.items(), key=lambda kv: -kv[1]["traffic_bytes_per_dispatch"] * kv[1]["dispatches"]):
        extra = (f'  rd {v["rd_requests_per_dispatch"] / 1e6:9.2f} M wr {v["wr_requests_per_dispatch"] / 1e6:9.2f} M'
                 if req else "")
        print(f'{v["dispatches"]:5d} {v["traffic_bytes_per_dispatch"] / 1e6:10.2f} MB{extra}  {k[:80]}')


if __name__ == "__main__":
    main()
