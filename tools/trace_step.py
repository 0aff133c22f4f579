"""Per-kernel timeline of the last full training step in a rocprofv3 --kernel-trace CSV (step = pack_many
to pack_many), with per-kernel-name totals.  usage: python tools/trace_step.py <run_kernel_trace.csv> [filter]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else None
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pack_many" in r["Kernel_Name"]]
# the last complete step: a pack_many-to-pack_many range whose gaps are all short (the tail after the timed steps
# holds host-side waits and copies)
step = None
for k in range(len(idx) - 1, 0, -1):
    cand = rows[idx[k - 1]:idx[k]]
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(cand, cand[1:])]
    if cand and max(gaps, default=0) < 50_000:
        step = cand
        break
step = step or rows[idx[-2]:idx[-1]]
t0 = int(step[0]["Start_Timestamp"])
end = t0
tot = defaultdict(float)
for r in step:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
    grid = tuple(int(r[f"Grid_Size_{d}"]) // int(r[f"Workgroup_Size_{d}"]) for d in "XYZ")
    tot[name] += (b - a) / 1e3
    if flt is None or flt in name:
        print(f"{(a - t0) / 1e3:8.1f} {(b - a) / 1e3:7.1f}  {name:60s} {grid}")
    end = max(end, b)
print(f"{len(step)} kernels, span {(end - t0) / 1e3:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:8.1f}  {k}")
