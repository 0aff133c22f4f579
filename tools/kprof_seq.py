"""Durations (us) of the last N launches whose kernel name contains PATTERN, in issue order, from a rocprofv3
kernel trace.  usage: python tools/kprof_seq.py <run_kernel_trace.csv> <pattern> [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat, n = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12
seq = [r for r in rows if pat in r["Kernel_Name"]][-n:]
for r in seq:
    print(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f}  grid={r['Grid_Size_X']:>8}  "
          f"{r['Kernel_Name'][:70]}")
print(f"sum {sum((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in seq):.1f} us")
