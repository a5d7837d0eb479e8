"""Per-kernel mean of rocprofv3 --pmc counter collections (one or more CSVs).

Usage: python tools/pmc_sq_summary.py <counter_collection.csv> [...]"""
import csv
import sys
from collections import defaultdict


def main(paths):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((path, r["Dispatch_Id"]))
    for k, cs in vals.items():
        nd = len({d for p, d in disp[k]}) or 1
        n_per_file = len(disp[k]) / max(1, len(paths))
        print(k, f"({int(n_per_file)} dispatches)")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {v / n_per_file:16.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
