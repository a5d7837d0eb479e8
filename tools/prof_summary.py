"""Summarise a rocprofv3 (ROCm 7.2 rocpd SQLite) kernel trace: per-kernel
calls, total and average device time, sorted by total.

usage: python tools/prof_summary.py <results.db> [top]"""
import sqlite3
import sys


def short(name: str) -> str:
    name = name.split("(")[0].replace("void ", "").replace("sv2n::", "")
    if "at::native" in name:
        name = "aten:" + name.split("at::native::")[1][:60]
    return name[:90]


def main(path, top=30):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average from top_kernels"))
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':92s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'%':>6s}")
    for name, calls, total, avg in rows[:top]:
        print(f"{short(name):92s} {calls:6d} {total:10.1f} {avg:9.2f} {100 * total / tot:6.2f}")
    print(f"total device time {tot:.1f} us over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
