#!/usr/bin/env python3
"""Per-dispatch rocprofv3 --pmc counter values of one kernel, in dispatch order.

Usage: tools/pmc_dispatch.py <kernel-substring> <counter_collection.csv> ...
Counters of several passes are joined by dispatch position within the kernel
(each pass runs the same program, so the k-th dispatch is the same launch).
"""
import collections
import csv
import sys


def main():
    pat, paths = sys.argv[1], sys.argv[2:]
    cols = collections.OrderedDict()
    for path in paths:
        per = collections.defaultdict(float)
        order = []
        for r in csv.DictReader(open(path)):
            if pat not in r["Kernel_Name"]:
                continue
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            if int(r["Dispatch_Id"]) not in order:
                order.append(int(r["Dispatch_Id"]))
            per[key] += float(r["Counter_Value"])
        names = sorted({c for _, c in per})
        for c in names:
            cols[c] = [per[(d, c)] for d in order]
    n = max(len(v) for v in cols.values())
    print("k  " + "  ".join(f"{c:>14s}" for c in cols))
    for k in range(n):
        print(f"{k:<3d}" + "  ".join(f"{(v[k] if k < len(v) else float('nan')):14.4g}" for v in cols.values()))


if __name__ == "__main__":
    main()
