"""Median per-launch duration of every kernel of the C2 training step from a
rocprofv3 kernel trace (tools/r5_final.sh), one table per step kind (the
kernel-name sequence from k_prep_fwd_all to k_adam: the covariance-layout
step, the generic-edge step), plus the median step span:
python tools/step_table.py gpurun_out/<dir>/c2t/p_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_prep_fwd_all" in r["Kernel_Name"]]
kinds = collections.defaultdict(list)
for a, b in zip(idx, idx[1:] + [len(rows)]):
    ad = [k for k in range(a, b) if "k_adam" in rows[k]["Kernel_Name"]]
    if not ad:
        continue
    seq = tuple(rows[k]["Kernel_Name"][:64] for k in range(a, ad[-1] + 1))
    kinds[seq].append((a, ad[-1] + 1))
for seq, steps in sorted(kinds.items(), key=lambda kv: -len(kv[1])):
    if len(steps) < 10:
        continue
    steps = steps[5:]
    acc, spans, busy = collections.defaultdict(list), [], []
    for a, b in steps:
        spans.append((int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
        busy.append(sum(int(rows[k]["End_Timestamp"]) - int(rows[k]["Start_Timestamp"])
                        for k in range(a, b)) / 1e3)
        for j, k in enumerate(range(a, b)):
            acc[j].append((int(rows[k]["End_Timestamp"]) - int(rows[k]["Start_Timestamp"])) / 1e3)
    kind = "covariance-layout edges" if any("cv2" in n for n in seq) else "generic edges"
    print(f"== C2 training step, {kind}: {len(steps)} steps")
    for j, n in enumerate(seq):
        v = sorted(acc[j])
        print(f"{j:2d} {v[len(v) // 2]:7.1f}  {n}")
    spans.sort()
    busy.sort()
    print(f"median span {spans[len(spans) // 2]:.1f} us, summed kernels "
          f"{busy[len(busy) // 2]:.1f} us\n")
