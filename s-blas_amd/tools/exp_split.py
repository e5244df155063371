#!/usr/bin/env python3
"""Experiment (round 4): how fast are config 2's heavy and
light rows on their own, per kernel, and the CSR5 over XCD column panels on the
heavy rows only?  Config 2 = rows < n/8 with 96 nnz (heavy), the rest 9
(light).  Each part is uploaded as its own CSR (n columns) and timed cold
(1 GiB read sweep, sblas_spmv_timed span, median of --reps).  One JSON line per
(part, variant).  Not a product path."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nrows", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--variants", default="csr5,rowsplit,panel,xsort,csr5p2,csr5p4,csr5p8")
    ap.add_argument("--parts", default="full,heavy,light")
    args = ap.parse_args()
    import torch
    import sblas
    n = args.nrows
    rp = sblas.gen_synth_rowptr(n, 96, 9)
    col, val = sblas.gen_synth_rows(n, rp, 0, n)
    x = torch.from_numpy(sblas.gen_vector(n, 43)).cuda()
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device="cuda")
    h = n // 8
    parts = {"full": (0, n), "heavy": (0, h), "light": (h, n)}
    ids = {"csr5": sblas.CSR5, "rowsplit": sblas.ROWSPLIT, "panel": sblas.PANEL, "xsort": sblas.XSORT}
    for pname in args.parts.split(","):
        r0, r1 = parts[pname]
        for v in args.variants.split(","):
            env = {}
            algo = ids.get(v)
            if v.startswith("csr5p"):
                algo = sblas.CSR5
                env = {"SBLAS_CSR5_PANEL": "1", "SBLAS_PANELS": v[5:]}
            for k, val_ in env.items():
                os.environ[k] = val_
            A = sblas.DeviceCSR.upload_slice(0, n, rp, col, val, r0, r1, int(rp[r0]), int(rp[r1]))
            A.analyse(algo)
            for k in env:
                del os.environ[k]
            y = torch.zeros(r1 - r0, dtype=torch.float64, device="cuda")
            spans = []
            for k in range(args.reps + 2):
                scrub.sum(dtype=torch.int64)
                torch.cuda.synchronize()
                spans.append(A.spmv_timed(algo, 1.0, x.data_ptr(), 0.5, y.data_ptr()))
            byts = A.algorithmic_bytes(True)
            us = float(np.median(spans[2:])) * 1e3
            A.close()
            print(json.dumps({"part": pname, "variant": v, "rows": r1 - r0, "nnz": int(rp[r1] - rp[r0]),
                              "cold_us": round(us, 1), "frac_8TBs": round(byts / us / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
