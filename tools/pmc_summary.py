"""Per-launch HBM bytes of the roofline kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir>   -> JSON on stdout

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch.  On gfx950
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced reads, so the
read bytes are 2 x FETCH_SIZE (MI355X_MICROARCH.md, section HBM); WRITE_SIZE
is exact for 16-byte stores.  Infinity-Cache hits are included in both.
"""
import csv
import glob
import json
import os
import sys

KERNEL = "conv_halo_kernel"


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if KERNEL in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    # the first launches are warm-up; all launches have the same shape
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    rd = 2.0 * f_kib * 1024
    wr = w_kib * 1024
    print(json.dumps({"kernel": KERNEL + "<5> g_a[2] fwd", "batch": 16, "size": 256,
                      "dispatches": [len(fetch), len(write)], "fetch_size_kib": round(f_kib, 1),
                      "write_size_kib": round(w_kib, 1), "read_bytes_per_launch": round(rd),
                      "write_bytes_per_launch": round(wr), "hbm_bytes_per_launch": round(rd + wr),
                      "note": "read = 2 x FETCH_SIZE (gfx950 half-count on 16-B loads); Infinity-Cache hits counted"},
                     indent=1))


if __name__ == "__main__":
    main()
