#!/usr/bin/env python3
"""C1 (the reference's own Maelstrom setting: 25-node tree4, 100 ms ticks,
~10 client ops per tick for 20 s) in batched gossip mode (gg_config.batch_ticks,
DESIGN.md §2b) for several batch periods, beside the parity mode, reported the
way Maelstrom's broadcast workload does (messages per operation, stable latency
quantiles, lost values) — the Gossip Glomers 3d/3e trade-off (README.md:17).
Usage: tools/batched_report.py [--cpu] [--json out] [--ticks 1,2,3,5,8]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gossip-glomers-distributed-systems_amd"))
from ggamd.checker import broadcast_report  # noqa: E402
from ggamd.engine import Engine  # noqa: E402
from ggamd.workload import c1  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cpu", action="store_true", help="the CPU oracle library instead of the HIP engine")
ap.add_argument("--ticks", default="1,2,3,5,8")
ap.add_argument("--json")
args = ap.parse_args()
lib = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so") if args.cpu else None
dev = -1 if args.cpu else 0
rows = {}
for part in (False, True):
    wl, nreads = c1(partition=part)
    tag = " + bisection [50,100)" if part else ""
    e = Engine(25, wl.n_lanes, seed=wl.seed, track_delivery=True, library=lib, device=dev)
    wl.apply(e)
    rows[f"parity (sync on){tag}"] = broadcast_report(e, wl.injections, nreads, e.step(wl.max_rounds))
    # batched without sync loses what a partition drops; with sync the pushes repair it
    for sync in ((False, True) if part else (False,)):
        for B in [int(x) for x in args.ticks.split(",")]:
            e = Engine(25, wl.n_lanes, seed=wl.seed, track_delivery=True, library=lib, device=dev,
                       enable_sync=sync, batch_ticks=B)
            wl.apply(e)
            rows[f"batched B={B} ({B * 100} ms), sync {'on' if sync else 'off'}{tag}"] = broadcast_report(
                e, wl.injections, nreads, e.step(wl.max_rounds))
for name, r in rows.items():
    lat = r["stable_latency_ms"]
    print(f"{name:58s} msgs/op {r['msgs_per_op']:6.2f}  latency median {lat['median']:6.0f} ms  "
          f"max {lat['max']:6.0f} ms  lost {len(r['lost'])}", flush=True)
print(json.dumps(rows, indent=1))
if args.json:
    json.dump(rows, open(args.json, "w"), indent=1)
