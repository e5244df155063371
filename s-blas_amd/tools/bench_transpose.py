#!/usr/bin/env python3
"""CSR -> CSC transpose benchmark, config-2 matrix.

Single device: DeviceCSR.transpose (resident CSR -> device CSC), HIP events.
Algorithmic bytes 24*nnz + 4*(m+1) + 4*(n+1) (col+val read, rowidx+val
written, both pointer arrays).  Multi-device: sblas_csr2csc_mgpu from host
arrays, reporting the block-transpose and compose phases (blocks wrap onto
the visible GPUs).  Every result is checked bit-exact against the
single-device transpose.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nrows", type=int, default=2_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mgpu", default="1,2,4")
    args = ap.parse_args()
    import torch
    import sblas

    n = args.nrows
    rp = sblas.gen_synth_rowptr(n, 96, 9)
    col, val = sblas.gen_synth_rows(n, rp, 0, n, 96, 9, prefix=False, seed=42)
    nnz = int(rp[-1])
    dev = torch.device("cuda", 0)
    A = sblas.DeviceCSR.upload(0, n, rp, col, val)
    dcp = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    dri = torch.zeros(nnz, dtype=torch.int32, device=dev)
    dcv = torch.zeros(nnz, dtype=torch.float64, device=dev)
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        A.transpose(dcp.data_ptr(), dri.data_ptr(), dcv.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.steps):
            A.transpose(dcp.data_ptr(), dri.data_ptr(), dcv.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    A.close()
    cp, ri, cv = dcp.cpu().numpy(), dri.cpu().numpy(), dcv.cpu().numpy()
    abytes = 24 * nnz + 4 * (n + 1) * 2
    res = {}
    for g in [int(t) for t in args.mgpu.split(",") if t]:
        sblas.csr2csc_mgpu(n, n, rp, col, val, g)  # warm-up
        t1s, t2s = [], []
        for _ in range(3):
            gcp, gri, gcv, t1, t2 = sblas.csr2csc_mgpu(n, n, rp, col, val, g)
            t1s.append(t1)
            t2s.append(t2)
        exact = bool(np.array_equal(gcp, cp) and np.array_equal(gri, ri) and np.array_equal(gcv, cv))
        res[f"blocks{g}"] = {"gpus": min(g, torch.cuda.device_count()),
                             "transpose_ms": round(float(np.median(t1s)), 3),
                             "compose_ms": round(float(np.median(t2s)), 3), "bit_exact": exact}
    out = {"metric": "fp64 CSR->CSC transpose, algorithmic GB/s", "unit": "GB/s",
           "value": round(abytes / ms / 1e6, 1), "ms": round(ms, 4), "n": n, "nnz": nnz,
           "algorithmic_bytes": abytes,
           "roofline": {"bound": "hbm", "achieved": round(abytes / ms / 1e6, 1), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(abytes / ms / 1e6 / 8000.0, 4)},
           "mgpu": res}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
