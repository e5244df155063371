#!/usr/bin/env python3
"""Average duration of the HEADLINE's kernels in a rocprofv3 kernel trace of
`python bench.py` (run_kernel_trace.csv).  The default bench command also runs
xsort on the structured stand-ins (the `structured` leg, after the headline),
so the per-name stats csv mixes those launches into k_spmv_xsort's average;
the headline's launches are the ones before the first launch of the row-split
leg (`rowsplit_beside`, the next leg: k_spmv_panel / k_spmv_rowsplit).

  python headline_kernels.py gpurun_out/r05_end/prof/run_kernel_trace.csv [--out f.json] [--rows-out f.csv]

--rows-out keeps the headline's own trace rows (kernel, start, end, duration)
so the averages can be recomputed from the committed file alone.
"""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    ap.add_argument("--rows-out")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    stop = next((i for i, r in enumerate(rows)
                 if "k_spmv_panel" in r["Kernel_Name"] or "k_spmv_rowsplit" in r["Kernel_Name"]), len(rows))
    head = rows[:stop]
    out = {"trace": a.trace, "headline_dispatches_before": stop}
    for key in ("k_spmv_xsort", "k_xsort_reduce"):
        d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
                      for r in head if key in r["Kernel_Name"]])
        out[key] = {"calls": int(d.size), "avg_us": round(float(d.mean()), 2) if d.size else None,
                    "min_us": round(float(d.min()), 2) if d.size else None,
                    "max_us": round(float(d.max()), 2) if d.size else None}
    if a.rows_out:
        with open(a.rows_out, "w", newline="") as fh:
            wr = csv.writer(fh)
            wr.writerow(["dispatch", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "duration_us"])
            for i, r in enumerate(head):
                if any(key in r["Kernel_Name"] for key in ("k_spmv_xsort", "k_xsort_reduce")):
                    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    wr.writerow([i, r["Kernel_Name"], st, en, round((en - st) * 1e-3, 3)])
        out["rows_file"] = a.rows_out
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
