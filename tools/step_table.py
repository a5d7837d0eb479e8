"""Median per-launch duration of every kernel of the C2 training step from a
rocprofv3 kernel trace (tools/c2_step_trace.sh), plus the median step span:
python tools/step_table.py gpurun_out/<dir>/stats/s_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_prep_fwd_all" in r["Kernel_Name"]]
train = [(a, b) for a, b in zip(idx, idx[1:])
         if any("k_adam" in rows[k]["Kernel_Name"] for k in range(a, b))]
acc, spans = collections.defaultdict(list), []
for a, b in train[5:]:
    t0 = int(rows[a]["Start_Timestamp"])
    spans.append((int(rows[b - 1]["End_Timestamp"]) - t0) / 1e3)
    for j, k in enumerate(range(a, b)):
        r = rows[k]
        acc[(j, r["Kernel_Name"][:64])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (j, n), v in sorted(acc.items()):
    v.sort()
    print(f"{j:2d} {v[len(v) // 2]:7.1f}  {n}")
spans.sort()
print(f"training steps {len(spans)}; median span {spans[len(spans) // 2]:.1f} us")
