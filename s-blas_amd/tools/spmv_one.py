#!/usr/bin/env python3
"""Minimal config-2 SpMV driver for profiling passes (rocprofv3 --pmc / kernel
trace): generate the bench.py matrix, upload, analyse one algorithm, run
--reps warm launches on one stream and print the mean HIP-event time.

  python spmv_one.py [--algo xsort|panel|rowsplit|csr5] [--reps 10] [--nrows N] [--cold]
                     [--matrix synth|stencil7|stencil27|rmat --grid G --scale S]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="xsort")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--nrows", type=int, default=2_000_000)
    ap.add_argument("--cols", choices=["random", "prefix"], default="random")
    ap.add_argument("--matrix", choices=["synth", "stencil7", "stencil27", "rmat"], default="synth")
    ap.add_argument("--grid", type=int, default=128, help="stencil mesh edge")
    ap.add_argument("--scale", type=int, default=21, help="R-MAT scale")
    ap.add_argument("--cold", action="store_true", help="1 GiB scrub before every launch")
    ap.add_argument("--scrub", choices=["write", "read"], default="write",
                    help="cold scrub: read+write (add_) or read-only (sum)")
    a = ap.parse_args()
    import torch
    import sblas
    algo = {"rowsplit": 1, "csr5": 2, "panel": 4, "xsort": 5}[a.algo]
    if a.matrix == "synth":
        n = a.nrows
        rp = sblas.gen_synth_rowptr(n)
        col, val = sblas.gen_synth_rows(n, rp, 0, n, prefix=a.cols == "prefix")
    elif a.matrix == "rmat":
        rp, col, val = sblas.gen_rmat(a.scale, 16, seed=50)
        n = len(rp) - 1
    else:
        rp, col, val = sblas.gen_stencil3d(a.grid, a.grid, a.grid, int(a.matrix[7:]), seed=49)
        n = len(rp) - 1
    x = torch.from_numpy(sblas.gen_vector(n, 43)).cuda()
    y = torch.zeros(n, dtype=torch.float64, device="cuda")
    A = sblas.DeviceCSR.upload(0, n, rp, col, val)
    t0 = time.perf_counter()
    A.analyse(algo)
    plan_s = time.perf_counter() - t0
    s = torch.cuda.Stream()
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device="cuda") if a.cold else None
    ms = []
    with torch.cuda.stream(s):
        A.spmv(algo, 0.84, x.data_ptr(), 0.39, y.data_ptr(), s.cuda_stream)
        for _ in range(a.reps):
            if scrub is not None:
                if a.scrub == "write":
                    scrub.add_(1)
                else:
                    scrub.sum(dtype=torch.int64)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            A.spmv(algo, 0.84, x.data_ptr(), 0.39, y.data_ptr(), s.cuda_stream)
            e1.record(s)
            ms.append((e0, e1))
    torch.cuda.synchronize()
    t = [e0.elapsed_time(e1) for e0, e1 in ms]
    abytes = A.algorithmic_bytes(True)
    print(f"{a.matrix} {a.algo} n={n}: plan {plan_s:.2f} s, mean {np.mean(t) * 1e3:.1f} us, "
          f"min {np.min(t) * 1e3:.1f} us, {abytes / (np.mean(t) * 1e-3) / 1e9:.1f} GB/s alg.",
          flush=True)
    A.close()


if __name__ == "__main__":
    main()
