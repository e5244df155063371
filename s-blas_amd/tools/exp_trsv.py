#!/usr/bin/env python3
"""Experiment driver: configs[4]'s SpTRSV (bench.py's integer known-answer
stand-in, n = 5,558,326) under planner test options (sblas.test_options).

For each option set (JSON objects) times --reps cold solves of the pull
executor (algo 1; 1 GiB read sweep, device-side hold, HIP events on the
launch stream -- bench.py's config5 protocol), checks x == x_ref exactly
after every solve, and prints one JSON line.  Experiment tooling only.

  python exp_trsv.py --opts '[{}, {"trsv_xcd": 1}]'
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opts", default="[{}]")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--algo", type=int, default=1)
    a = ap.parse_args()
    import torch
    import sblas
    import bench
    cp, ri, vi, xref, bi = bench.config5_system(sblas)
    n, nnz = len(cp) - 1, len(ri)
    dev = torch.device("cuda", 0)
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    dcp, dri, dv, db = (torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (cp, ri, vi, bi))
    dx = torch.zeros(n, dtype=torch.float64, device=dev)
    T = sblas.DeviceTRSV(0, n, nnz, dcp.data_ptr(), dri.data_ptr(), dv.data_ptr(), 0)
    T.pick()
    for rnd in range(a.rounds):
        for opts in json.loads(a.opts):
            ms, exact = [], True
            with sblas.test_options(**opts):
                with torch.cuda.stream(stream):
                    T.solve(a.algo, db.data_ptr(), dx.data_ptr(), sp)  # warm-up (builds what the form needs)
                torch.cuda.synchronize()
                exact &= bool(np.array_equal(dx.cpu().numpy(), xref))
                for _ in range(a.reps):
                    scrub.sum(dtype=torch.int64)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    with torch.cuda.stream(stream):
                        torch.cuda._sleep(500_000)
                        e0.record(stream)
                        T.solve(a.algo, db.data_ptr(), dx.data_ptr(), sp)
                        e1.record(stream)
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                    exact &= bool(np.array_equal(dx.cpu().numpy(), xref))
            print(json.dumps({"round": rnd, "opts": opts, "mean_ms": round(float(np.mean(ms)), 4),
                              "min_ms": round(float(np.min(ms)), 4), "exact": exact}), flush=True)
    T.close()


if __name__ == "__main__":
    main()
