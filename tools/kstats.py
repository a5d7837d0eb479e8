"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, with
calls and average microseconds.  usage: python tools/kstats.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{r['Name'][:72]:72s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
          f"{float(r['TotalDurationNs']) / tot * 100:5.1f}%")
print(f"total {tot / 1e6:.2f} ms")
