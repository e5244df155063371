#!/usr/bin/env python3
"""Experiment: xsort layouts on the R-MAT power-law graph (bench.py --matrix rmat).

Half of an R-MAT graph's rows are empty, and xsort's ranges count rows, so an
empty row spends LDS accumulator room.  This times the kernel (cold span after
a 1 GiB read sweep, as bench.py at N = 1) on the graph as generated and, with
--compact, on the same graph with its empty rows dropped (the kernel time a
row map over non-empty rows could reach, without the map's own cost), under
whatever SBLAS_XS_* switches the environment sets.  One JSON line per matrix.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=21)
    ap.add_argument("--algos", default="xsort")
    ap.add_argument("--compact", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()

    import torch
    import sblas

    dev = torch.device("cuda", 0)
    rp, col, val = sblas.gen_rmat(args.scale, 16, seed=50)
    rp = np.asarray(rp, dtype=np.int64)
    n = len(rp) - 1
    mats = [("full", rp)]
    if args.compact:
        lens = np.diff(rp)
        keep = lens > 0
        rpc = np.zeros(int(keep.sum()) + 1, np.int64)
        rpc[1:] = np.cumsum(lens[keep])
        mats.append(("compact", rpc))
    x = torch.from_numpy(sblas.gen_vector(n, 43)).to(dev)
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    algos = {"rowsplit": sblas.ROWSPLIT, "csr5": sblas.CSR5, "panel": sblas.PANEL, "xsort": sblas.XSORT}
    for name, mrp in mats:
        m = len(mrp) - 1
        for a in args.algos.split(","):
            A = sblas.DeviceCSR.upload(0, n, mrp, col, val)
            A.analyse(algos[a])
            y = torch.zeros(m, dtype=torch.float64, device=dev)
            spans = []
            with torch.cuda.stream(stream):
                for _ in range(args.reps + 2):
                    scrub.sum(dtype=torch.int64)
                    torch.cuda.synchronize()
                    spans.append(A.spmv_timed(algos[a], 1.0, x.data_ptr(), 0.5, y.data_ptr(),
                                              stream.cuda_stream))
            A.close()
            us = float(np.median(spans[2:])) * 1e3
            nnz = int(mrp[-1])
            byts = 12 * nnz + 4 * (m + 1) + 8 * n + 16 * m
            print(json.dumps({"tag": args.tag, "matrix": name, "algo": a, "rows": m, "nnz": nnz,
                              "cold_span_us": round(us, 1), "frac_8TBs": round(byts / us / 8e6, 4),
                              "env": {k: v for k, v in os.environ.items() if k.startswith("SBLAS_XS")}}),
                  flush=True)


if __name__ == "__main__":
    main()
