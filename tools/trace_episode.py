#!/usr/bin/env python3
"""One bench episode from a rocprofv3 kernel_trace.csv: the dispatches between
two reset_state launches (the last complete episode), each with its duration
and the idle gap before it, and per-kernel sums; the episode's wall span versus
its summed kernel time shows how much of a step is launch gaps.
Usage: tools/trace_episode.py kernel_trace.csv|results.db [episode index from the end, default 2]"""
import csv
import sys
from collections import defaultdict

if sys.argv[1].endswith(".db"):  # rocprofv3's default SQLite output: its `kernels` view
    import sqlite3
    db = sqlite3.connect(sys.argv[1])
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in db.execute("select name, start, end from kernels")]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
resets = [i for i, r in enumerate(rows) if "reset_state" in r["Kernel_Name"]]
if len(resets) < back + 1:
    sys.exit(f"only {len(resets)} reset_state dispatches")
i0, i1 = resets[-back - 1], resets[-back]
ep = rows[i0:i1]
t0 = int(ep[0]["Start_Timestamp"])
span = (int(ep[-1]["End_Timestamp"]) - t0) / 1e3
busy = 0.0
per = defaultdict(lambda: [0, 0.0])
prev_end = None
for r in ep:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d = (e - s) / 1e3
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e
    busy += d
    name = r["Kernel_Name"].split("(")[0][:60]
    per[name][0] += 1
    per[name][1] += d
    print(f"{(s - t0) / 1e3:9.2f} {d:8.2f} us  gap {gap:6.2f}  {name}")
print(f"\nepisode: {len(ep)} dispatches, span {span:.1f} us, kernel time {busy:.1f} us, gaps {span - busy:.1f} us")
for name, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:9.2f} us {n:4d}x  {100 * t / busy:5.1f}%  {name}")
