#!/usr/bin/env python3
"""Turn rocprofv3 --pmc CSV output into per-launch HBM traffic for one kernel.

Usage:
  pmc_traffic.py --kernel k_spmv_rowsplit --out profiles/pmc_rowsplit.json \
      --fetch <dir of the FETCH_SIZE pass> --write <dir of the WRITE_SIZE pass> \
      [--l2 <dir of the TCC_HIT_sum/TCC_MISS_sum pass>] [--algorithmic BYTES] \
      [--lib s-blas_amd/libsblas.so]

The summary is stamped with the sha256 of the libsblas.so the passes ran
(`lib_sha256`): bench.py reports `roofline.traffic` from it only while the
loaded library has the same hash, and null (with the reason) otherwise.

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  * FETCH_SIZE and WRITE_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
    streaming read (128-B requests tallied as 64 B), so the read side is
    doubled;
  * the counters sit at the L2's memory side, so Infinity-Cache (MALL) hits
    are included -- "traffic" is L2->fabric bytes, an upper bound on HBM.
FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit
one TCC pass together).
"""
import argparse
import csv
import hashlib
import glob
import json
import os
import statistics


def split_kernels(kernel):
    """Split a comma-separated kernel list at top-level commas only: template
    names such as k_rx2_scatter<256, 0, 512> keep theirs."""
    out, depth, cur = [], 0, ""
    for ch in kernel:
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
            continue
        depth += (ch == "<") - (ch == ">")
        cur += ch
    out.append(cur)
    return [k for k in out if k]


def counter_values(d, kernel, name):
    """Per-launch values; `kernel` may list several comma-separated kernels
    that make up one operation (e.g. panel SpMV + its reduce): their medians
    are summed into a single per-operation value."""
    total = []
    for k in split_kernels(kernel):
        vals = []
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if k in row.get("Kernel_Name", "") and row.get("Counter_Name") == name:
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return []
        total.append(statistics.median(vals))
    return [sum(total)]


def file_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--l2")
    ap.add_argument("--algorithmic", type=float)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "libsblas.so"),
                    help="the library the counter passes ran (its sha256 stamps the summary)")
    a = ap.parse_args()
    f = counter_values(a.fetch, a.kernel, "FETCH_SIZE")
    w = counter_values(a.write, a.kernel, "WRITE_SIZE")
    if not f or not w:
        raise SystemExit(f"no counter rows for {a.kernel}: fetch {len(f)} write {len(w)}")
    fetch_kib = statistics.median(f)
    write_kib = statistics.median(w)
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    out = {
        "kernel": a.kernel,
        "launches": {"fetch_pass": len(f), "write_pass": len(w)},
        "FETCH_SIZE_KiB_median": fetch_kib,
        "WRITE_SIZE_KiB_median": write_kib,
        "read_bytes_per_launch": read_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024",
        "lib_sha256": file_sha256(a.lib),
    }
    if a.algorithmic:
        out["algorithmic_bytes_per_launch"] = a.algorithmic
        out["traffic_over_algorithmic"] = (read_b + write_b) / a.algorithmic
    if a.l2:
        hit = counter_values(a.l2, a.kernel, "TCC_HIT_sum")
        miss = counter_values(a.l2, a.kernel, "TCC_MISS_sum")
        if hit and miss:
            h, mm = statistics.median(hit), statistics.median(miss)
            out["TCC_HIT_sum_median"] = h
            out["TCC_MISS_sum_median"] = mm
            out["l2_hit_rate"] = h / (h + mm) if h + mm else None
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
