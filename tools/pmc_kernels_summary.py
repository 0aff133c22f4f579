"""Average each PMC counter per kernel name over the runs of tools/pmc_kernels.sh.
usage: python tools/pmc_kernels_summary.py gpurun_out/pmck_<tag> [name-substring ...]"""
import collections
import csv
import glob
import sys

prefix, keys = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(prefix + "_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if keys and not any(k in n for k in keys):
            continue
        key = (n[:80], r["Grid_Size"])
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (n, grid), cs in sorted(agg.items()):
    print(f"== {n}  grid={grid}")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
