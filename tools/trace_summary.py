"""Summarise a rocprofv3 kernel_trace.csv: median duration per (kernel, grid) in dispatch order."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seen = collections.OrderedDict()
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    k = (r["Kernel_Name"][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    seen.setdefault(k, []).append(d)
for k, v in seen.items():
    if "at::native" in k[0] or "rocclr" in k[0]:
        continue
    print(f"{k[0]:60s} grid {k[1]:>8}x{k[2]:>4}x{k[3]:>3} n={len(v):3d} med {sorted(v)[len(v) // 2]:8.1f} us")
