#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/: kernel stats (from --kernel-trace --stats) and HBM traffic per launch
from separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes, corrected per MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores (8-B stores: uncalibrated).

usage: pmc_traffic.py <kernel-substring> <workload> <kt_dir> <fetch_dir> <write_dir> <out_prefix> [timed_steps]
With timed_steps K, the kernel trace's last K launches (bench.py's timed region, after its warmup) are averaged as
well: the stats CSV averages every launch, warmup included.
"""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    kernel, workload, kt, fetch, write, out = sys.argv[1:7]
    # timed_steps: K (the last K launches) or W:K (launches W+1 .. W+K in issue order: bench.py's timed region when
    # more launches follow it, e.g. its steady-state block)
    spec = sys.argv[7] if len(sys.argv) > 7 else "0"
    skip, timed = (int(v) for v in spec.split(":")) if ":" in spec else (None, int(spec))
    stats = [r for r in csv.DictReader(open(kt + "/kt_kernel_stats.csv"))]
    f_kib, nf = per_launch(fetch + "/pmc_counter_collection.csv", kernel, "FETCH_SIZE")
    w_kib, nw = per_launch(write + "/pmc_counter_collection.csv", kernel, "WRITE_SIZE")
    fetch_b = 2 * f_kib * 1024 if f_kib is not None else None
    write_b = w_kib * 1024 if w_kib is not None else None
    k = [r for r in stats if kernel in r["Name"]]
    d = {
        "kernel": k[0]["Name"] if k else kernel,
        "workload": workload,
        "avg_duration_ns": float(k[0]["AverageNs"]) if k else None,
        "calls": int(k[0]["Calls"]) if k else None,
        "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
        "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": (fetch_b + write_b) if fetch_b is not None and write_b is not None else None,
        "correction": "read = 2 x FETCH_SIZE KiB (gfx950 wide-stream halving), write = WRITE_SIZE KiB",
        "launches_sampled": [nf, nw],
    }
    if timed:
        rows = [r for r in csv.DictReader(open(kt + "/kt_kernel_trace.csv")) if kernel in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        dur = dur[-timed:] if skip is None else dur[skip:skip + timed]
        d["timed_region_launches"] = len(dur)
        d["timed_region_avg_duration_ns"] = sum(dur) / len(dur) if dur else None
    json.dump(d, open(out + "_pmc_traffic.json", "w"), indent=1)
    with open(out + "_kernel_stats.csv", "w") as fo:
        fo.write(open(kt + "/kt_kernel_stats.csv").read())
    print(json.dumps(d))


if __name__ == "__main__":
    main()
