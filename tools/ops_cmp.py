"""Compare two bench.py --ops-json ledgers launch by launch (same model / config): per-shape time before and
after, grouped by (kind, shape).  usage: python tools/ops_cmp.py A.json B.json [min_us]"""
import collections
import json
import sys

a = json.load(open(sys.argv[1]))["launches"]
b = json.load(open(sys.argv[2]))["launches"]
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
print(f"launches {len(a)} -> {len(b)}; instrumented {sum(l['ms'] for l in a):.3f} -> {sum(l['ms'] for l in b):.3f} ms")


def group(ls):
    g = collections.OrderedDict()
    for l in ls:
        k = (l["kind"], str(l["shape"]))
        e = g.setdefault(k, [0, 0.0, set()])
        e[0] += 1
        e[1] += l["ms"] * 1e3
        e[2].add(l["kernel"][:30])
    return g


ga, gb = group(a), group(b)
for k in ga:
    x, y = ga[k], gb.get(k, [0, 0.0, set()])
    if abs(x[1] - y[1]) >= thr:
        print(f"{k[0][:10]:10s} {k[1][:52]:52s} n={x[0]:2d} {x[1]:8.1f} -> {y[1]:8.1f} us  {'/'.join(sorted(x[2]))[:30]} -> "
              f"{'/'.join(sorted(y[2]))[:30]}")
