#!/usr/bin/env python3
"""Experiment driver: SpMV plan variants through the planner test options.

For each matrix (rmat21, synth = config 2, stencil27 128^3, stencil7 160^3)
and each option set (JSON objects, sblas.test_options; "det": 1 runs the
handle in deterministic mode), builds the plan and times --reps cold calls
(1 GiB read sweep, then the call's device span, sblas_spmv_timed -- bench.py's
N = 1 protocol), checks one y against the oracle's per-row bound, and prints
one JSON line.  Experiment tooling only; the oracle is the checker.

  python exp_opts.py --mats rmat21,synth,slice8 --algo 5 --opts '[{}, {"xs_solo": 1}]'
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


def matrix(sblas, name):
    """(rowptr, col, val, ncols): ncols None = square."""
    if name.startswith("slice"):  # rank 0's cyclic slice of config 2 at N = int(name[5:]) (bench.py N > 1)
        import sblas_dist
        n, world = 2_000_000, int(name[5:])
        rp = sblas.gen_synth_rowptr(n, 96, 9)
        plan = sblas_dist.make_cyclic_plan(rp, n, world)
        lrp, col, val = sblas_dist.cyclic_local_csr(
            rp, plan, 0, lambda a, b: sblas.gen_synth_rows(n, rp, a, b, 96, 9, seed=42))
        return lrp, col, val, n
    return matrix_sq(sblas, name) + (None,)


def matrix_sq(sblas, name):
    if name == "rmat21":
        return sblas.gen_rmat(21, 16, seed=50)
    if name == "synth":
        n = 2_000_000
        rp = sblas.gen_synth_rowptr(n, 96, 9)
        col, val = sblas.gen_synth_rows(n, rp, 0, n, 96, 9, prefix=False, seed=42)
        return rp, col, val
    g, pts = {"stencil27": (128, 27), "stencil7": (160, 7)}[name]
    return sblas.gen_stencil3d(g, g, g, pts, seed=49)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mats", default="rmat21")
    ap.add_argument("--algo", type=int, default=5)
    ap.add_argument("--opts", default="[{}]")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=1, help="alternate the option sets this many times")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    import torch
    import sblas
    import orc  # checker only
    dev = torch.device("cuda", 0)
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    alpha, beta = 0.8401877171547095, 0.39438292681909304
    for mname in a.mats.split(","):
        rp, col, val, ncols = matrix(sblas, mname)
        m = len(rp) - 1
        n = ncols or m
        xh = sblas.gen_vector(n, 43)
        y0 = sblas.gen_vector(m, 44)
        x = torch.from_numpy(xh).to(dev)
        want = bound = None
        if not a.no_check:
            want = orc.csr_spmv(rp, col, val, xh, alpha, beta, y0)
            bound = orc.spmv_bound(rp, col, val, xh, alpha, beta, y0)
        for rnd in range(a.rounds):
            for opts in json.loads(a.opts):
                o = dict(opts)
                det = bool(o.pop("det", 0))
                A = sblas.DeviceCSR.upload(0, n, rp, col, val)
                A.deterministic = det
                t0 = time.perf_counter()
                with sblas.test_options(**o):
                    A.analyse(a.algo)
                build_s = time.perf_counter() - t0
                y = torch.from_numpy(y0.copy()).to(dev)
                A.spmv(a.algo, alpha, x.data_ptr(), beta, y.data_ptr(), sp)
                torch.cuda.synchronize()
                ok = None
                if want is not None:
                    ok = bool(np.all(np.abs(y.cpu().numpy() - want) <= bound))
                ts = []
                with torch.cuda.stream(stream):
                    for _ in range(a.reps):
                        scrub.sum(dtype=torch.int64)
                        torch.cuda.synchronize()
                        ts.append(A.spmv_timed(a.algo, alpha, x.data_ptr(), beta, y.data_ptr(), sp))
                abytes = A.algorithmic_bytes(True)
                plan = A.xsort_info() if a.algo == 5 else None
                A.close()
                t = float(np.mean(ts))
                print(json.dumps({"matrix": mname, "round": rnd, "opts": opts, "algo": a.algo, "n": n,
                                  "nnz": int(rp[-1]), "mean_us": round(t * 1e3, 2),
                                  "min_us": round(min(ts) * 1e3, 2), "frac": round(abytes / (t * 1e-3) / 8e12, 4),
                                  "check": ok, "build_s": round(build_s, 2), "plan": plan}), flush=True)


if __name__ == "__main__":
    main()
