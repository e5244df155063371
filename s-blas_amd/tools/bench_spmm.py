#!/usr/bin/env python3
"""SpMM benchmark (BASELINE configs[3]), one GPU.

rail4284 is not in the container: synthetic stand-in with its shape, m =
4,284, k = 1,092,610, nnz = 11,279,748 (2,633 nnz/row, uniform-random sorted
columns, seed 44), B k x 64 U[0,1) (seed 45), C0 m x 64 U[0,1) (seed 46),
alpha = -0.7, beta = 0.8 (dspmm_baseline_test.cu:518-519).  B is resident
row-major (our layout); C column-major (ld = m).

Algorithmic bytes: 12*nnz + 4(m+1) + 8*k*n + 16*m*n;
GFLOP/s = 2*nnz*n/t.  The traffic-aware floor is higher: every nonzero pulls
a 512-B row of B (nnz*512 B = 5.8 GB through L2), reported as gbps_l2.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4284)
    ap.add_argument("--k", type=int, default=1_092_610)
    ap.add_argument("--nnz", type=int, default=11_279_748)
    ap.add_argument("--ncols", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--layout", choices=["row", "col"], default="row")
    ap.add_argument("--blocky", type=int, default=0,
                    help="instead of the rail4284 shape: 16-row blocks each dense (~90%%) over "
                         "BLOCKY random columns (an FEM-like matrix where MFMA tiles apply)")
    args = ap.parse_args()
    import torch
    import sblas

    m, k, n = args.m, args.k, args.ncols
    rng = np.random.default_rng(44)
    if args.blocky:
        rows = []
        for _ in range(m // 16):
            cols = np.sort(rng.choice(k, args.blocky, replace=False))
            for _ in range(16):
                rows.append(cols[rng.random(args.blocky) < 0.9])
        m = len(rows)
        lens = np.array([len(r) for r in rows], np.int64)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate(rows).astype(np.int32)
        args.nnz = int(rp[-1])
    else:
        base, extra = divmod(args.nnz, m)
        lens = np.full(m, base, np.int64)
        lens[:extra] += 1
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.empty(args.nnz, np.int32)
        for r in range(m):  # distinct sorted columns per row
            col[rp[r]:rp[r + 1]] = np.sort(rng.choice(k, size=int(lens[r]), replace=False))
    val = np.random.default_rng(45).random(args.nnz)
    dev = torch.device("cuda", 0)
    B = torch.rand((k, n), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(45))
    C0 = torch.rand((n, m), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(46))
    if args.layout == "col":
        Bd, ldb, lay = B.t().contiguous(), k, 0
    else:
        Bd, ldb, lay = B, n, 1
    A = sblas.DeviceCSR.upload(0, k, rp, col, val)
    C = C0.clone()
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        A.spmm(n, -0.7, Bd.data_ptr(), ldb, lay, 0.8, C.data_ptr(), m, s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.steps):
            A.spmm(n, -0.7, Bd.data_ptr(), ldb, lay, 0.8, C.data_ptr(), m, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    # spot check 32 rows against a float64 reference on the host
    Ch = C0.clone()
    with torch.cuda.stream(s):
        A.spmm(n, -0.7, Bd.data_ptr(), ldb, lay, 0.8, Ch.data_ptr(), m, s.cuda_stream)
    torch.cuda.synchronize()
    rows = np.random.default_rng(0).choice(m, 32, replace=False)
    Bh = B.cpu().numpy()
    C0h = C0.cpu().numpy()
    got = Ch.cpu().numpy()
    err = 0.0
    for r in rows:
        a, b_ = rp[r], rp[r + 1]
        want = -0.7 * (val[a:b_] @ Bh[col[a:b_], :]) + 0.8 * C0h[:, r]
        err = max(err, float(np.max(np.abs(got[:, r] - want) / (np.abs(want) + 1e-300))))
    abytes = 12 * args.nnz + 4 * (m + 1) + 8 * k * n + 16 * m * n
    out = {
        "metric": "fp64 CSR SpMM GFLOP/s (2*nnz*n/t), 1 MI355X",
        "value": round(2.0 * args.nnz * n / ms / 1e6, 3), "unit": "GFLOP/s", "n_gpus": 1,
        "steps": args.steps, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "dtype": "f64", "data": "synthetic rail4284-shaped (DESIGN.md)",
        "config": {"workload": "C = -0.7*A*B + 0.8*C", "m": m, "k": k, "nnz": args.nnz, "ncols": n,
                   "b_layout": args.layout, "structure": f"blocky{args.blocky}" if args.blocky
                   else "rail4284-shaped uniform random",
                   "mfma_fill_threshold": os.environ.get("SBLAS_SPMM_MFMA_FILL", "0.25")},
        "roofline": {"bound": "hbm", "achieved": round(abytes / ms / 1e6, 1), "peak": 8000.0,
                     "unit": "GB/s", "frac": round(abytes / ms / 1e6 / 8000.0, 4)},
        "gbps_l2_brow_traffic": round(args.nnz * n * 8 / ms / 1e6, 1),
        "max_rel_err_32_rows": err,
    }
    A.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
