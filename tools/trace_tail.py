#!/usr/bin/env python3
"""Print the last N dispatches of a rocprofv3 kernel_trace.csv (duration, start)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for r in rows[-n:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{r['Kernel_Name'][:48]:48s} {d:9.2f} us  grid {r['Grid_Size_X']:>9s}  vgpr {r['VGPR_Count']}")
