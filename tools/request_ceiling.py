#!/usr/bin/env python3
"""The random-row request ceiling in the L2's memory-side requests ->
profiles/request_ceiling.json (bench.py's line_frac denominator).

Usage: tools/request_ceiling.py GATHER_STDOUT REQ_COUNTER_CSV [OUT]

GATHER_STDOUT: `tools/gather_bench --calibrate` run without a profiler (rows/s
per row size, HIP events); REQ_COUNTER_CSV: counter_collection.csv of the same
command under `rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum` (requests
per dispatch; rows per dispatch from the stdout). Requests/s at the ceiling =
rows/s x requests per row; the file keeps every row size and takes the highest
rate as the ceiling (the least flattering denominator).
"""
import collections
import csv
import json
import re
import sys


def main():
    rows = {}
    for line in open(sys.argv[1]):
        m = re.match(r"calibrate rows\s+(\d+) B G=\s*(\d+) rows_per_dispatch (\d+) rows_per_s (\S+)", line)
        if m:
            rows[int(m.group(2))] = {"row_bytes": int(m.group(1)), "rows_per_dispatch": int(m.group(3)),
                                     "rows_per_s": float(m.group(4))}
    req = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        m = re.search(r"gather<(\d+),\s*(\d+)>", r["Kernel_Name"])
        if m:
            req[(int(m.group(1)), r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    per_g = collections.defaultdict(list)
    for (g, _), vals in req.items():
        per_g[g].append(sum(vals))  # rd + wr of one dispatch
    out = {"source": "tools/gather_bench.hip --calibrate (8 GiB table, uniformly random rows, K = 8, 4096 blocks) "
                     "timed with HIP events; requests per dispatch from rocprofv3 --pmc TCC_EA0_RDREQ_sum "
                     "TCC_EA0_WRREQ_sum over the same command", "rows": []}
    for g, r in sorted(rows.items()):
        if g not in per_g:
            continue
        rq = sum(per_g[g]) / len(per_g[g])
        per_row = rq / r["rows_per_dispatch"]
        out["rows"].append(dict(r, requests_per_row=per_row, requests_per_s=r["rows_per_s"] * per_row))
    if not out["rows"]:
        raise SystemExit("no gather dispatches matched")
    out["requests_per_s"] = max(x["requests_per_s"] for x in out["rows"])
    json.dump(out, open(sys.argv[3] if len(sys.argv) > 3 else "profiles/request_ceiling.json", "w"), indent=1)
    for x in out["rows"]:
        print(f'{x["row_bytes"]:4d} B rows: {x["rows_per_s"] / 1e9:6.2f} G rows/s x {x["requests_per_row"]:.3f} '
              f'requests/row = {x["requests_per_s"] / 1e9:6.2f} G requests/s')
    print(f'ceiling {out["requests_per_s"] / 1e9:.2f} G requests/s')


if __name__ == "__main__":
    main()
