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

REGIME = {0: "8 GiB table (HBM)", 1: "256 MiB table (Infinity Cache resident)"}

def main():
    rows, wrows, seqs = {}, {}, {}  # (G, regime) -> calibration; regime 0: 8 GiB table, 1: 256 MiB
    for line in open(sys.argv[1]):
        m = re.match(r"calibrate (rows|writes)(_mall)?\s+(\d+) B G=\s*(\d+) rows_per_dispatch (\d+) rows_per_s (\S+)", line)
        if m:
            d = rows if m.group(1) == "rows" else wrows
            t = 1 if m.group(2) else 0
            d[(int(m.group(4)), t)] = {"row_bytes": int(m.group(3)), "table": REGIME[t],
                                       "rows_per_dispatch": int(m.group(5)), "rows_per_s": float(m.group(6))}
        m = re.match(r"calibrate seqwrite(_mall)? bytes_per_dispatch (\d+) bytes_per_s (\S+)", line)
        if m:
            t = 1 if m.group(1) else 0
            seqs[t] = {"table": REGIME[t], "bytes_per_dispatch": int(m.group(2)), "bytes_per_s": float(m.group(3))}
    req = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, G, T) -> dispatch -> requests
    for r in csv.DictReader(open(sys.argv[2])):
        name = r["Kernel_Name"]
        m = re.search(r"(gather|scatter)<(\d+),\s*(\d+)(?:,\s*(\d+))?>", name)
        if m:
            key = (m.group(1), int(m.group(2)), int(m.group(4) or 0))
        else:
            m = re.search(r"seqwrite(?:<(\d+)>)?", name)
            key = ("seqwrite", 0, int(m.group(1) or 0)) if m else None
        if key:
            req[key][(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])

    def per_dispatch(key, counter):
        vals = collections.defaultdict(float)
        for (disp, cname), v in req[key].items():
            if cname.startswith(counter):
                vals[disp] += v
        return sum(vals.values()) / len(vals) if vals else None

    out = {"source": "tools/gather_bench.hip --calibrate (uniformly random rows, K = 8, 4096 blocks, on an 8 GiB "
                     "table in HBM and on a 256 MiB table the Infinity Cache can hold; random-row stores "
                     "scatter<G, 8, T>; coalesced store sweeps of 2 GiB and 256 MiB) timed with HIP events; requests "
                     "per dispatch from rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum over the same command",
           "rows": [], "write_rows": [], "write_sweeps": []}
    for (g, t), r in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        rq = per_dispatch(("gather", g, t), "TCC_EA0_RDREQ")
        if rq is None:
            continue
        per_row = rq / r["rows_per_dispatch"]
        out["rows"].append(dict(r, requests_per_row=per_row, requests_per_s=r["rows_per_s"] * per_row))
    for (g, t), r in sorted(wrows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        rq = per_dispatch(("scatter", g, t), "TCC_EA0_WRREQ")
        if rq is None:
            continue
        per_row = rq / r["rows_per_dispatch"]
        out["write_rows"].append(dict(r, requests_per_row=per_row, requests_per_s=r["rows_per_s"] * per_row))
    for t, sq in sorted(seqs.items()):
        rq = per_dispatch(("seqwrite", 0, t), "TCC_EA0_WRREQ")
        if rq is not None:
            sq["requests_per_dispatch"] = rq
            sq["requests_per_s"] = rq / (sq["bytes_per_dispatch"] / sq["bytes_per_s"])
            out["write_sweeps"].append(sq)
    if not out["rows"]:
        raise SystemExit("no gather dispatches matched")
    # the least flattering denominators: the highest rate of each direction, any table
    out["requests_per_s"] = max(x["requests_per_s"] for x in out["rows"])
    w = [x["requests_per_s"] for x in out["write_rows"] + out["write_sweeps"]]
    out["write_requests_per_s"] = max(w) if w else None
    json.dump(out, open(sys.argv[3] if len(sys.argv) > 3 else "profiles/request_ceiling.json", "w"), indent=1)
    for x in out["rows"]:
        print(f'reads  {x["row_bytes"]:4d} B rows, {x["table"]}: {x["rows_per_s"] / 1e9:6.2f} G rows/s x '
              f'{x["requests_per_row"]:.3f} requests/row = {x["requests_per_s"] / 1e9:6.2f} G requests/s')
    for x in out["write_rows"]:
        print(f'writes {x["row_bytes"]:4d} B rows, {x["table"]}: {x["rows_per_s"] / 1e9:6.2f} G rows/s x '
              f'{x["requests_per_row"]:.3f} requests/row = {x["requests_per_s"] / 1e9:6.2f} G requests/s')
    for x in out["write_sweeps"]:
        print(f'writes sweep, {x["table"]}: {x["bytes_per_s"] / 1e9:.0f} GB/s = {x["requests_per_s"] / 1e9:.2f} G requests/s')
    print(f'ceilings: reads {out["requests_per_s"] / 1e9:.2f}, writes '
          f'{(out["write_requests_per_s"] or 0) / 1e9:.2f} G requests/s')


if __name__ == "__main__":
    main()
