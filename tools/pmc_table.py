#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counters over one or more passes.

Usage: tools/pmc_table.py <counter_collection.csv> ...
Prints, per kernel (heaviest first by dispatches x first counter), the number
of dispatches and each counter's mean value per dispatch.
"""
import collections
import csv
import sys


def main():
    val = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0][:80]
            val[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, cs in val.items():
        n = max(len(v) for v in cs.values())
        rows.append((k, n, {c: sum(v) / len(v) for c, v in cs.items()}))
    rows.sort(key=lambda x: -x[1] * max(x[2].values()))
    for k, n, cs in rows:
        print(f"{k}  dispatches={n}  " + "  ".join(f"{c}={m:.4g}" for c, m in sorted(cs.items())))


if __name__ == "__main__":
    main()
