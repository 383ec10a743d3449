#!/usr/bin/env python3
"""C1 (the reference's own Maelstrom setting) through the engine, reported the
way Maelstrom's broadcast workload reports it: stable latency quantiles,
messages per operation, lost values. Usage: tools/maelstrom_report.py [--cpu] [--json out]"""
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
ap.add_argument("--cpu", action="store_true", help="run the CPU oracle library instead of the HIP engine")
ap.add_argument("--json")
args = ap.parse_args()
lib = os.path.join(REPO, "oracle", "_build", "libgossip_cpu.so") if args.cpu else None
out = {}
for part in (False, True):
    wl, nreads = c1(partition=part)
    e = Engine(25, wl.n_lanes, seed=wl.seed, track_delivery=True, library=lib, device=-1 if args.cpu else 0)
    wl.apply(e)
    st = e.step(wl.max_rounds)
    out["partition" if part else "no_partition"] = broadcast_report(e, wl.injections, nreads, st)
print(json.dumps(out, indent=1))
if args.json:
    json.dump(out, open(args.json, "w"), indent=1)
