#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 counters (one JSON object per kernel): usage pmc_summary.py <dir> [<dir> ...] where
each dir holds a pmc_counter_collection.csv (rocprofv3 --pmc ... --output-format csv -o pmc)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
        out[k]["_dispatch_samples"] = max(len(v) for v in cs.values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
