"""Per-training-step kernel breakdown from a rocprofv3 kernel-trace CSV.

Usage: python tools/step_breakdown.py <run_kernel_trace.csv> [n_steps]

Segments the trace at the optimizer kernel (one per train step), keeps the
last ``n_steps`` segments that precede the forward-only phase, and prints the
average device time per step by kernel, plus the wall span of a step."""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.split("(")[0]
    for pre in ("void ", "sv2n::"):
        name = name.replace(pre, "")
    if name.startswith("Cijk_"):
        return "hipBLASLt:" + name[:40]
    if "at::native" in name:
        return "aten:" + name.split("at::native::")[-1][:50]
    return name[:60]


def main(path, n_steps=20):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt_idx = [i for i, r in enumerate(rows) if "FusedOptimizer" in r["Kernel_Name"]
               or "adam" in r["Kernel_Name"].lower()]
    segs = [(opt_idx[k] + 1, opt_idx[k + 1] + 1) for k in range(len(opt_idx) - 1)]
    segs = segs[-n_steps:]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    spans = []
    for a, b in segs:
        spans.append((int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot[short(r["Kernel_Name"])] += d
            cnt[short(r["Kernel_Name"])] += 1
    ns = len(segs)
    busy = sum(tot.values()) / ns
    print(f"steps analysed: {ns}; wall span/step {sum(spans)/ns:.1f} us; kernel busy/step {busy:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {v/ns:9.1f} us  x{cnt[k]/ns:4.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
