"""Summarise a rocprofv3 --kernel-trace CSV by (kernel, grid): share, calls, avg, per-step time.

usage: python tools/prof_summary.py <run_kernel_trace.csv> [steps] [top]
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    g = collections.defaultdict(list)
    for r in rows:
        k = (r["Kernel_Name"][:70], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        g[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in g.values())
    print(f"total {tot / 1e6:.2f} ms, per step {tot / 1e3 / steps:.1f} us")
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v) / tot * 100:5.1f}% n={len(v):4d} avg={sum(v) / len(v) / 1e3:8.2f}us "
              f"per-step={sum(v) / 1e3 / steps:7.1f}us grid={k[1]},{k[2]},{k[3]} {k[0]}")


if __name__ == "__main__":
    main()
