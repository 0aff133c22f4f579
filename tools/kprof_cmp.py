"""Side-by-side per-kernel totals of two rocprofv3 --stats directories (base vs new)."""
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f))}


a, b = load(sys.argv[1]), load(sys.argv[2])
ta, tb = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
print(f"total  base {ta / 1e6:9.3f} ms   new {tb / 1e6:9.3f} ms   ({(tb / ta - 1) * 100:+.1f} %)")
for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[1], b.get(k, (0, 0))[1]))[:30]:
    ca, da = a.get(k, (0, 0.0))
    cb, db = b.get(k, (0, 0.0))
    avg_a, avg_b = (da / ca if ca else 0) / 1e3, (db / cb if cb else 0) / 1e3
    print(f"{da / 1e6:8.3f} {db / 1e6:8.3f} ms | avg {avg_a:8.2f} {avg_b:8.2f} us | {k[:110]}")
