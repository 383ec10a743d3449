#!/usr/bin/env python3
"""The random-row request ceiling in the L2's memory-side requests ->
profiles/request_ceiling.json (bench.py's line_frac denominator).

Usage: tools/request_ceiling.py GATHER_STDOUT REQ_COUNTER_CSV [OUT]

GATHER_STDOUT: `tools/gather_bench --calibrate` run without a profiler (rows/s
per row size, HIP events); REQ_COUNTER_CSV: counter_collection.csv of the same
command under `rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum` (requests
per dispatch; rows per dispatch from the stdout). Requests/s at the ceiling =
rows/s x requests per row, per direction: reads from the random-row gathers,
writes from the random-row stores and the coalesced sweep; the file keeps every
shape and takes each direction's highest rate as its ceiling (the least
flattering denominator).
"""
import collections
import csv
import json
import re
import sys


def main():
    rows, wrows, seq = {}, {}, None
    for line in open(sys.argv[1]):
        m = re.match(r"calibrate (rows|writes)\s+(\d+) B G=\s*(\d+) rows_per_dispatch (\d+) rows_per_s (\S+)", line)
        if m:
            d = rows if m.group(1) == "rows" else wrows
            d[int(m.group(3))] = {"row_bytes": int(m.group(2)), "rows_per_dispatch": int(m.group(4)),
                                  "rows_per_s": float(m.group(5))}
        m = re.match(r"calibrate seqwrite bytes_per_dispatch (\d+) bytes_per_s (\S+)", line)
        if m:
            seq = {"bytes_per_dispatch": int(m.group(1)), "bytes_per_s": float(m.group(2))}
    req = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, G) -> dispatch -> requests
    for r in csv.DictReader(open(sys.argv[2])):
        name = r["Kernel_Name"]
        m = re.search(r"(gather|scatter)<(\d+),\s*(\d+)>", name)
        key = (m.group(1), int(m.group(2))) if m else (("seqwrite", 0) if "seqwrite" in name else None)
        if key:
            req[key][(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])

    def per_dispatch(key, counter):
        vals = collections.defaultdict(float)
        for (disp, cname), v in req[key].items():
            if cname.startswith(counter):
                vals[disp] += v
        return sum(vals.values()) / len(vals) if vals else None

    out = {"source": "tools/gather_bench.hip --calibrate (8 GiB table, uniformly random rows, K = 8, 4096 blocks; "
                     "random-row stores scatter<G, 8>; a coalesced 2 GiB store sweep) timed with HIP events; "
                     "requests per dispatch from rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum over the same "
                     "command", "rows": [], "write_rows": []}
    for g, r in sorted(rows.items()):
        rq = per_dispatch(("gather", g), "TCC_EA0_RDREQ")
        if rq is None:
            continue
        per_row = rq / r["rows_per_dispatch"]
        out["rows"].append(dict(r, requests_per_row=per_row, requests_per_s=r["rows_per_s"] * per_row))
    for g, r in sorted(wrows.items()):
        rq = per_dispatch(("scatter", g), "TCC_EA0_WRREQ")
        if rq is None:
            continue
        per_row = rq / r["rows_per_dispatch"]
        out["write_rows"].append(dict(r, requests_per_row=per_row, requests_per_s=r["rows_per_s"] * per_row))
    if seq is not None:
        rq = per_dispatch(("seqwrite", 0), "TCC_EA0_WRREQ")
        if rq is not None:
            seq["requests_per_dispatch"] = rq
            seq["requests_per_s"] = rq / (seq["bytes_per_dispatch"] / seq["bytes_per_s"])
            out["write_sweep"] = seq
    if not out["rows"]:
        raise SystemExit("no gather dispatches matched")
    # the least flattering denominators: the highest rate of each direction
    out["requests_per_s"] = max(x["requests_per_s"] for x in out["rows"])
    w = [x["requests_per_s"] for x in out["write_rows"]] + ([seq["requests_per_s"]] if seq and "requests_per_s" in seq
                                                             else [])
    out["write_requests_per_s"] = max(w) if w else None
    json.dump(out, open(sys.argv[3] if len(sys.argv) > 3 else "profiles/request_ceiling.json", "w"), indent=1)
    for x in out["rows"]:
        print(f'reads  {x["row_bytes"]:4d} B rows: {x["rows_per_s"] / 1e9:6.2f} G rows/s x {x["requests_per_row"]:.3f} '
              f'requests/row = {x["requests_per_s"] / 1e9:6.2f} G requests/s')
    for x in out["write_rows"]:
        print(f'writes {x["row_bytes"]:4d} B rows: {x["rows_per_s"] / 1e9:6.2f} G rows/s x {x["requests_per_row"]:.3f} '
              f'requests/row = {x["requests_per_s"] / 1e9:6.2f} G requests/s')
    if seq and "requests_per_s" in seq:
        print(f'writes sweep: {seq["bytes_per_s"] / 1e9:.0f} GB/s = {seq["requests_per_s"] / 1e9:.2f} G requests/s')
    print(f'ceilings: reads {out["requests_per_s"] / 1e9:.2f}, writes '
          f'{(out["write_requests_per_s"] or 0) / 1e9:.2f} G requests/s')


if __name__ == "__main__":
    main()
