#!/usr/bin/env python3
"""Stress run (evidence, not a unit test): config 2 through AUTO's xsort plan,
--launches back-to-back launches on ONE plan (the self-rearming claim queues
flip parity every launch), every y checked against the oracle's per-row bound;
then the same on a deterministic handle, every y bitwise equal to the first.
Prints one JSON line.  The oracle is the checker only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=1000)
    ap.add_argument("--matrix", default="synth", choices=["synth", "rmat21"])
    a = ap.parse_args()
    import torch
    import sblas
    import orc  # checker only
    if a.matrix == "synth":
        n = 2_000_000
        rp = sblas.gen_synth_rowptr(n, 96, 9)
        col, val = sblas.gen_synth_rows(n, rp, 0, n, 96, 9, prefix=False, seed=42)
    else:
        rp, col, val = sblas.gen_rmat(21, 16, seed=50)
        n = len(rp) - 1
    xh = sblas.gen_vector(n, 43)
    y0 = sblas.gen_vector(n, 44)
    alpha, beta = orc.alpha_beta()
    want = orc.csr_spmv_omp(rp, col, val, xh, alpha, beta, y0.copy())
    bound = orc.spmv_bound(rp, col, val, xh, alpha, beta, y0)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(xh).to(dev)
    y0d = torch.from_numpy(y0).to(dev)
    wantd = torch.from_numpy(want).to(dev)
    boundd = torch.from_numpy(bound).to(dev)
    out = {"matrix": a.matrix, "n": n, "nnz": int(rp[-1]), "launches": a.launches}
    for det in (False, True):
        A = sblas.DeviceCSR.upload(0, n, rp, col, val)
        A.deterministic = det
        assert A.pick() == sblas.XSORT
        A.analyse(sblas.XSORT)
        y = torch.empty_like(y0d)
        first = None
        bad_bound = bad_bits = 0
        worst = -np.inf
        t0 = time.perf_counter()
        for it in range(a.launches):
            y.copy_(y0d)
            A.spmv(sblas.XSORT, alpha, x.data_ptr(), beta, y.data_ptr())
            err = (y - wantd).abs() - boundd   # on the device: <= 0 everywhere when within the bound
            m = float(err.max().item())
            worst = max(worst, m)
            bad_bound += int(m > 0)
            if det:
                if first is None:
                    first = y.clone()
                elif not torch.equal(first, y):
                    bad_bits += 1
        A.close()
        key = "deterministic" if det else "default"
        out[key] = {"launches_over_bound": bad_bound, "max_excess_over_bound": worst,
                    "wall_s": round(time.perf_counter() - t0, 1)}
        if det:
            out[key]["launches_not_bitwise_equal_to_first"] = bad_bits
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
