"""CPU tests of the evidence tools that bench / session scripts rely on."""
import csv
import json
import os
import subprocess
import sys

from conftest import ROOT

TOOLS = os.path.join(ROOT, "s-blas_amd", "tools")


def _trace(path, rows):
    cols = ["Kind", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=cols)
        w.writeheader()
        for name, t0, t1 in rows:
            w.writerow({"Kind": "KERNEL_DISPATCH", "Kernel_Name": name, "Start_Timestamp": t0, "End_Timestamp": t1})


def test_headline_kernels_stops_at_the_next_leg(tmp_path):
    """headline_kernels.py averages only the xsort launches before the first
    row-split launch (the structured leg's later xsort launches are not the
    headline's)."""
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, [("k_spmv_xsort<...>", 1000, 151000), ("k_xsort_reduce<true>", 152000, 157000),
               ("k_spmv_xsort<...>", 200000, 349000), ("k_xsort_reduce<true>", 350000, 355000),
               ("void sblas::k_spmv_panel<false>(...)", 400000, 700000),
               ("k_spmv_xsort<...>", 800000, 930000)])
    out = tmp_path / "h.json"
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "headline_kernels.py"), str(p), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["headline_dispatches_before"] == 4
    assert d["k_spmv_xsort"]["calls"] == 2 and d["k_spmv_xsort"]["avg_us"] == 149.5
    assert d["k_xsort_reduce"]["calls"] == 2 and d["k_xsort_reduce"]["avg_us"] == 5.0
