"""Print the kernel sequence of one training step from a rocprofv3 kernel trace.

usage: python tools/prof_step.py <run_kernel_trace.csv> [step_index_from_end]
Steps are delimited by the aux optimizer kernel (adam_small_kernel).
"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ends = [i for i, r in enumerate(rows) if "adam_small_kernel" in r["Kernel_Name"]]
    a, b = ends[-back - 1] + 1, ends[-back] + 1
    t0 = int(rows[a]["Start_Timestamp"])
    tot = 0
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {d:8.2f}us grid={r['Grid_Size_X']},{r['Grid_Size_Y']},"
              f"{r['Grid_Size_Z']} {r['Kernel_Name'][:90]}")
    print(f"sum {tot:.1f} us over {b - a} kernels, span {(int(rows[b - 1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
