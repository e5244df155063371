#!/usr/bin/env python3
"""Median per-launch value of every counter found under rocprofv3 --pmc
output directories, for kernels whose name contains --kernel.

  pmc_summary.py --kernel k_spmv_xsort DIR [DIR ...] [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--json")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    vals = defaultdict(list)
    for d in a.dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if a.kernel in row.get("Kernel_Name", ""):
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {k: statistics.median(v) for k, v in sorted(vals.items())}
    for k, v in out.items():
        print(f"{k:40s} {v:16.1f}  (n={len(vals[k])})")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"kernel": a.kernel, "median_per_launch": out}, fh, indent=1)


if __name__ == "__main__":
    main()
