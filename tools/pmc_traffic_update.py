"""Record the HBM traffic of one replayed launch into profiles/pmc_traffic.json (the records bench.py's
roofline `traffic` field looks up by workload / kernel / shape).

usage: python tools/pmc_traffic_update.py <fetch_dir> <write_dir> <replay_log>
  fetch_dir / write_dir: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE outputs of `bench.py --roofline-only --replay
  kind:index --steps R` (tools/pmc_traffic.sh); replay_log: that run's stdout (its JSON line names the launch).
Per launch: read = 2 x FETCH_SIZE (gfx950 counts half the bytes of 16-byte-per-lane reads,
MI355X_MICROARCH.md 'HBM'), write = WRITE_SIZE, both over the last R dispatches of the kernel (the replays);
Infinity-Cache hits are included in both counts."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_dispatches(d, counter, base, n):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if base in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)[-n:]]


def main():
    fetch_dir, write_dir, log = sys.argv[1:4]
    line = [l for l in open(log) if l.startswith("{")][-1]
    rl = json.loads(line)
    kernel, shape = rl["kernel"], rl["launch"].split(": ", 1)[1]
    kind = rl["launch"].split(": ", 1)[0]     # conv_fwd / conv_dgrad / ...: one kernel may serve both directions
    reps = int(rl["timing"].split(",")[1].split()[0])
    base = kernel.split("<")[0].split(" ")[0]
    f = last_dispatches(fetch_dir, "FETCH_SIZE", base, reps)
    w = last_dispatches(write_dir, "WRITE_SIZE", base, reps)
    if not f or not w:
        sys.exit(f"no {base} dispatches with counters")
    f_kib, w_kib = sorted(f)[len(f) // 2], sorted(w)[len(w) // 2]
    rd, wr = 2.0 * f_kib * 1024, w_kib * 1024
    rec = {"workload": rl["workload"], "kernel": kernel, "shape": shape, "kind": kind, "lib_sha256": rl.get("lib_sha256"),
           "dispatches": [len(f), len(w)],
           "fetch_size_kib": round(f_kib, 1), "write_size_kib": round(w_kib, 1),
           "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
           "hbm_bytes_per_launch": round(rd + wr), "algorithmic_bytes_per_launch": rl["algorithmic_bytes_per_launch"],
           "note": "median over the replayed launches; read = 2 x FETCH_SIZE (gfx950 half-count on 16-B loads); "
                   "Infinity-Cache hits counted"}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        recs = json.load(open(path))
    except (OSError, ValueError):
        recs = []
    if isinstance(recs, dict):
        recs = [recs]
    # one record per launch: a re-measurement (of a new build) replaces the old one
    recs = [r for r in recs if not (r.get("workload") == rec["workload"] and r.get("kernel") == kernel
                                     and r.get("shape") == shape and r.get("kind", kind) == kind)]
    recs.append(rec)
    json.dump(recs, open(path, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
