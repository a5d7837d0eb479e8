"""One training step's kernel timeline from a rocprofv3 kernel-trace CSV.

Usage: python tools/timeline.py <kernel_trace.csv> [step_index_from_end]

Segments the trace at the optimizer kernel (as tools/step_breakdown.py does)
and prints, for one step, every kernel's start / end offset from the step's
first kernel and its duration, in start order — concurrent launches (side
stream branches of the hipGraph) show as overlapping intervals."""
import csv
import sys

from step_breakdown import short


def main(path, back=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt_idx = [i for i, r in enumerate(rows) if "FusedOptimizer" in r["Kernel_Name"]
               or "adam" in r["Kernel_Name"].lower()]
    a, b = opt_idx[-back - 1] + 1, opt_idx[-back] + 1
    t0 = int(rows[a]["Start_Timestamp"])
    busy_end = t0
    gaps = 0.0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > busy_end:
            gaps += (s - busy_end) / 1e3
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {short(r['Kernel_Name'])}")
    print(f"span {(busy_end - t0) / 1e3:.1f} us, idle gaps {gaps:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
