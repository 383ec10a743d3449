#!/usr/bin/env python3
"""HIP API calls of a rocprofv3 run (SQLite output, --hip-trace): counts per
call name, and the calls of the last timed episode of tools/ipc_rank.py — the
window from the last reset_state dispatch's enqueue to the end of the trace's
last kernel — in order, consecutive repeats folded. Shows whether a multi-round
gg_dist_step waits on the host (stream/event synchronisation, blocking copies)
between its rounds.
Usage: tools/hip_api_summary.py results.db"""
import sqlite3
import sys
from collections import Counter

db = sqlite3.connect(sys.argv[1])
views = {n for (n,) in db.execute("select name from sqlite_master where type='view'")}
regions = [(n, s, e) for n, s, e in db.execute("select name, start, end from regions order by start")]
kernels = [(n, s, e) for n, s, e in db.execute("select name, start, end from kernels order by start")]
print(f"{len(regions)} HIP API calls, {len(kernels)} kernel dispatches")
cnt = Counter(n for n, _, _ in regions)
for n, c in cnt.most_common(40):
    print(f"{c:8d}  {n}")
# the last episode: from the enqueue of the last reset_state (the last hipLaunchKernel
# before that kernel started) to the end of the last kernel
resets = [s for n, s, _ in kernels if "reset_state" in n]
if len(resets) >= 1:
    t_reset = resets[-1]
    launches = [s for n, s, _ in regions if "LaunchKernel" in n and s <= t_reset]
    t0 = launches[-1] if launches else t_reset
    t1 = kernels[-1][2]
    win = [(n, s) for n, s, _ in regions if t0 <= s <= t1]
    ks = [k for k in kernels if t0 <= k[1] <= t1]
    print(f"\nlast episode: {len(win)} HIP calls, {len(ks)} kernels, {(t1 - t0) / 1e6:.3f} ms")
    folded = []
    for n, _ in win:
        if folded and folded[-1][0] == n:
            folded[-1][1] += 1
        else:
            folded.append([n, 1])
    for n, c in folded:
        print(f"  {n}" + (f" x{c}" if c > 1 else ""))
    syncs = [n for n, _ in win if any(w in n for w in ("Synchronize", "Memcpy", "EventQuery", "StreamQuery"))]
    print(f"synchronising calls in the episode window: {Counter(syncs)}")
