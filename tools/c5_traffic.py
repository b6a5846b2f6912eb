#!/usr/bin/env python3
"""C5 (256 Mi bf16, accuracy 1e-6 and 1e-3) HBM traffic per encode from rocprofv3 FETCH_SIZE and WRITE_SIZE passes
over `tools/prof_cases.py c5 --reps R` (each encode = the tile form's count, scan, coder and oversized-tile kernels,
in dispatch order: R encodes at 1e-6, then R at 1e-3), corrected as tools/pmc_traffic.py does (read = 2 x
FETCH_SIZE KiB, write = WRITE_SIZE KiB; MI355X_MICROARCH.md, HBM section). Writes one profiles/*_pmc_traffic.json per
tolerance, in the format bench.py's load_pmc_traffic reads.
usage: c5_traffic.py <fetch_dir> <write_dir> <reps> <out_prefix>"""
import csv
import glob
import json
import sys

KERNELS = ("k_count1d_var_tile", "k_scan_ranges_mw", "k_encode1d_var_tile<", "k_encode1d_var_tile_big")
LABEL = "k_count1d_var_tile + k_scan_ranges_mw + k_encode1d_var_tile (+ k_encode1d_var_tile_big)"


def per_dispatch(d, counter):
    rows = []
    for path in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows if any(k in r["Kernel_Name"] for k in KERNELS)]


def main():
    fetch, write, reps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f = per_dispatch(fetch, "FETCH_SIZE")
    w = per_dispatch(write, "WRITE_SIZE")
    per = len(KERNELS)
    assert len(f) == len(w) == 2 * reps * per, (len(f), len(w))
    for i, tol in enumerate(("1e-6", "1e-3")):
        fs = f[i * reps * per:(i + 1) * reps * per]
        ws = w[i * reps * per:(i + 1) * reps * per]
        rd = 2 * 1024 * sum(v for _, v in fs) / reps
        wr = 1024 * sum(v for _, v in ws) / reps
        by_kernel = {}
        for (k, fv), (_, wv) in zip(fs, ws):
            name = next(x for x in KERNELS if x in k).rstrip("<")
            e = by_kernel.setdefault(name, {"read": 0.0, "write": 0.0})
            e["read"] += 2 * 1024 * fv / reps
            e["write"] += 1024 * wv / reps
        d = {"kernel": LABEL, "workload": "c5_bf16_acc%s_256Mi" % tol, "hbm_read_bytes_per_launch": rd,
             "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr, "per_kernel": by_kernel,
             "correction": "read = 2 x FETCH_SIZE KiB (gfx950 wide-stream halving), write = WRITE_SIZE KiB",
             "encodes_sampled": reps}
        json.dump(d, open("%s_c5_acc%s_pmc_traffic.json" % (out, tol), "w"), indent=1)
        print(json.dumps(d))


if __name__ == "__main__":
    main()
