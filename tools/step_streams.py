"""Per-queue occupancy of one training step in a rocprofv3 --kernel-trace CSV: each queue's busy time, the union
of all queues' busy intervals, the idle gaps (no kernel on any queue), and the longest main-queue kernels.
usage: python tools/step_streams.py <run_kernel_trace.csv> [top]"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
idx = [i for i, r in enumerate(rows) if "pack_many" in r["Kernel_Name"]]
step = None
for k in range(len(idx) - 1, 0, -1):
    cand = rows[idx[k - 1]:idx[k]]
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(cand, cand[1:])]
    if cand and max(gaps, default=0) < 50_000:
        step = cand
        break
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
busy = defaultdict(float)
cnt = defaultdict(int)
for r in step:
    busy[r["Queue_Id"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[r["Queue_Id"]] += 1
print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
for q in sorted(busy, key=lambda q: -busy[q]):
    print(f"  queue {q}: {cnt[q]:4d} kernels, busy {busy[q]:8.1f} us")
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
union, idle, cur_s, cur_e = 0, [], iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > cur_e:
        union += cur_e - cur_s
        idle.append((s - cur_e, cur_e - t0))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
print(f"union busy {union / 1e3:.1f} us; idle {sum(g for g, _ in idle) / 1e3:.1f} us in {len(idle)} gaps "
      f"(>2us: {sum(1 for g, _ in idle if g > 2000)}, summing {sum(g for g, _ in idle if g > 2000) / 1e3:.1f} us)")
# overlap: time with >= 2 kernels running
ev = sorted([(int(r["Start_Timestamp"]), 1) for r in step] + [(int(r["End_Timestamp"]), -1) for r in step])
lvl, last, multi = 0, t0, 0
for t, d in ev:
    if lvl >= 2:
        multi += t - last
    lvl += d
    last = t
print(f"time with >= 2 kernels in flight: {multi / 1e3:.1f} us")
q0 = max(busy, key=lambda q: busy[q])
main = [r for r in step if r["Queue_Id"] == q0]
name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cai::", "")[:58]
tot = defaultdict(lambda: [0, 0.0])
for r in main:
    k = tot[name(r)]
    k[0] += 1
    k[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"busiest queue {q0} by kernel:")
for n, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"  {n:58s} n={c:3d} {us:8.1f} us")
gaps_main = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(main, main[1:])]
print(f"busiest queue gaps: sum {sum(max(0, g) for g in gaps_main) / 1e3:.1f} us over {len(gaps_main)} "
      f"(median {sorted(gaps_main)[len(gaps_main) // 2] / 1e3:.2f} us)")
