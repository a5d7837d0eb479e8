"""GPU idle gaps inside the steps of a rocprofv3 kernel trace: per step (a
step starts at each k_prep_fwd_all launch) the span, the summed kernel time
and the largest gaps between consecutive kernels with the kernel after the
gap.  python tools/gap_table.py <kernel_trace.csv> [skip_steps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
starts = [i for i, r in enumerate(rows) if "k_prep_fwd_all" in r["Kernel_Name"]]
spans, busy, gaps = [], [], {}
for a, b in list(zip(starts, starts[1:]))[skip:]:
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    spans.append((t1 - t0) / 1e3)
    busy.append(sum(int(rows[k]["End_Timestamp"]) - int(rows[k]["Start_Timestamp"])
                    for k in range(a, b)) / 1e3)
    prev_end = int(rows[a]["End_Timestamp"])
    for j, k in enumerate(range(a + 1, b + 1)):
        g = (int(rows[k]["Start_Timestamp"]) - prev_end) / 1e3
        key = (j, rows[k]["Kernel_Name"][:60])
        gaps.setdefault(key, []).append(g)
        prev_end = max(prev_end, int(rows[k]["End_Timestamp"]))
med = lambda v: sorted(v)[len(v) // 2]
print(f"steps {len(spans)}: median span {med(spans):.1f} us, kernels {med(busy):.1f} us, "
      f"idle {med(spans) - med(busy):.1f} us")
for (j, n), v in sorted(gaps.items(), key=lambda kv: -med(kv[1]))[:15]:
    print(f"  gap before #{j:2d} {med(v):7.1f} us  {n}")
