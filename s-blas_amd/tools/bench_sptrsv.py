#!/usr/bin/env python3
"""SpTRSV benchmark (BASELINE configs[4]), one GPU.

circuit5M-class stand-in (circuit5M itself is not in the container): n =
5,558,326 unit-lower CSC, 5 off-diagonal rows per column drawn from a band of
80,000 below the diagonal (~985 level sets, nnz 33.35M incl. diagonal), values
(1 + r%10)/(20*row_len) (sblas_gen_lower_banded), x_ref in {1..10}, b = L x_ref.

Reports both executors (0 = CSC push / reference algorithm, 1 = CSR pull) with
HIP-event timing around sblas_trsv_solve, GFLOP/s = 2*nnz/t
(sptrsv_syncfree_cuda.h:604), algorithmic bytes 12*nnz + 4*(n+1) + 16*n, and
the reference's own serial executor (oracle/_ref, sptrsv_syncfree_serialref.h)
timed on one host core as the CPU baseline.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nrows", type=int, default=5_558_326)
    ap.add_argument("--offd", type=int, default=5)
    ap.add_argument("--band", type=int, default=80_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rhs", default="",
                    help="comma list of rhs counts for the SpTRSM executor (x, b n x rhs)")
    ap.add_argument("--no-push-rhs", action="store_true",
                    help="time only the pull executor for --rhs")
    ap.add_argument("--stencil", type=int, default=0,
                    help="instead of the circuit5M-class stand-in: the lower triangle of a 3-D "
                         "stencil on a STENCIL^3 grid (natural order, diagonally dominant; the "
                         "FEM / finite-difference kind, whose dependencies are mostly on the "
                         "previous rows)")
    ap.add_argument("--points", type=int, default=27, choices=[7, 27])
    ap.add_argument("--mgpu", default="",
                    help="comma list of block counts for the multi-device executor "
                         "(blocks wrap onto the visible GPUs; kernel wall time reported)")
    args = ap.parse_args()
    import torch
    import sblas

    n = args.nrows
    if args.stencil:
        g = args.stencil
        srp, scol, sval = sblas.gen_stencil3d(g, g, g, args.points, seed=49)
        n = len(srp) - 1
        srow = np.repeat(np.arange(n, dtype=np.int64), np.diff(srp))
        keep = scol >= srow  # CSR row j's upper part = CSC column j of L (symmetric pattern), diagonal first
        cp = np.zeros(n + 1, np.int32)
        cp[1:] = np.cumsum(np.bincount(srow[keep], minlength=n))
        ri = np.ascontiguousarray(scol[keep]).astype(np.int32)
        v = np.ascontiguousarray(sval[keep])
    else:
        cp, ri, v = sblas.gen_lower_banded(n, args.offd, args.band, 47)
    nnz = len(ri)
    xref = np.floor(sblas.gen_vector(n, 48) * 10.0) + 1.0
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(cp))
    b = np.bincount(ri, weights=v * xref[cols], minlength=n)
    dev = torch.device("cuda", 0)
    dcp, dri, dv, db = (torch.from_numpy(a).to(dev) for a in (cp, ri, v, b))
    dx = torch.zeros(n, dtype=torch.float64, device=dev)
    t0 = time.perf_counter()
    T = sblas.DeviceTRSV(0, n, nnz, dcp.data_ptr(), dri.data_ptr(), dv.data_ptr(), 0)
    setup_s = time.perf_counter() - t0
    levels = T.levels()
    auto_pick = T.pick()
    abytes = 12 * nnz + 4 * (n + 1) + 16 * n
    res = {}
    s = torch.cuda.Stream(device=dev)
    for algo, name in ((1, "pull_csr"), (3, "pull_level_order"), (4, "pull_auto"), (0, "push_csc"),
                       (2, "levelset_csr")):
        with torch.cuda.stream(s):
            T.solve(algo, db.data_ptr(), dx.data_ptr(), s.cuda_stream)  # warm-up
            torch.cuda.synchronize()
            ms = []
            for _ in range(args.steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                T.solve(algo, db.data_ptr(), dx.data_ptr(), s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
        x = dx.cpu().numpy()
        rel = float(np.abs(x - xref).sum() / np.abs(xref).sum())
        t = float(np.median(ms))
        res[name] = {"ms": round(t, 4), "gflops": round(2.0 * nnz / t / 1e6, 3),
                     "gbps_algorithmic": round(abytes / t / 1e6, 1),
                     "rel_l1_vs_xref": rel}
    for r in [int(t) for t in args.rhs.split(",") if t]:
        X = np.floor(np.random.default_rng(r).random((n, r)) * 10.0) + 1.0
        # B = L X on the host, one column at a time
        B = np.empty((n, r))
        for k in range(r):
            B[:, k] = np.bincount(ri, weights=v * X[cols, k], minlength=n)
        dX = torch.from_numpy(X).to(dev)
        dB = torch.from_numpy(B).to(dev)
        dXs = torch.zeros_like(dB)
        # pull executor (natural, level-ordered, AUTO tickets), then the reference's push dataflow with each lane
        # mapping (opt 1 = OPT_WARP_NNZ, 2 = OPT_WARP_RHS, 3 = OPT_WARP_AUTO)
        for name, algo, opt in ((f"trsm_pull_rhs{r}", 1, 0), (f"trsm_pull_level_rhs{r}", 3, 0),
                                (f"trsm_pull_auto_rhs{r}", 4, 0), (f"trsm_push_nnz_rhs{r}", 0, 1),
                                (f"trsm_push_rhs_rhs{r}", 0, 2), (f"trsm_push_auto_rhs{r}", 0, 3)):
            if algo == 0 and args.no_push_rhs:
                continue
            with torch.cuda.stream(s):
                T.solve_rhs_opt(algo, opt, r, dB.data_ptr(), dXs.data_ptr(), s.cuda_stream)
                torch.cuda.synchronize()
                ms = []
                for _ in range(args.steps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    T.solve_rhs_opt(algo, opt, r, dB.data_ptr(), dXs.data_ptr(), s.cuda_stream)
                    e1.record(s)
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
            t = float(np.median(ms))
            res[name] = {
                "ms": round(t, 4), "gflops": round(2.0 * nnz * r / t / 1e6, 3),
                "rel_l1_vs_xref": float((dXs - dX).abs().sum() / dX.abs().sum())}
        del dX, dB, dXs
    T.close()
    for g in [int(t) for t in args.mgpu.split(",") if t]:
        # persistent handle (sblas_trsv_mgpu_create): the host CSC -> CSR and
        # block uploads happen once, reported as build_s; each run uploads b,
        # resets x and solves
        t0 = time.perf_counter()
        H = sblas.TrsvMgpu(cp, ri, v, n, g)
        build_s = time.perf_counter() - t0
        H.run(b)  # warm-up
        ms, wall = [], []
        for _ in range(args.steps):
            t1 = time.perf_counter()
            x, t = H.run(b)
            wall.append((time.perf_counter() - t1) * 1e3)
            ms.append(t)
        H.close()
        t = float(np.median(ms))
        res[f"mgpu_pull_{g}blocks"] = {
            "ms": round(t, 4), "gflops": round(2.0 * nnz / t / 1e6, 3),
            "gpus": min(g, torch.cuda.device_count()),
            "build_s": round(build_s, 3),
            "run_wall_ms_incl_b_upload_and_x_download": round(float(np.median(wall)), 3),
            "rel_l1_vs_xref": float(np.abs(x - xref).sum() / np.abs(xref).sum())}
    out = {
        "metric": "fp64 sync-free SpTRSV GFLOP/s (2*nnz/t), 1 MI355X",
        "value": max(res[k]["gflops"] for k in ("pull_auto", "push_csc")),
        "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps, "higher_is_better": True,
        "dtype": "f64",
        "data": (f"lower triangle of a {args.points}-point 3-D stencil, {args.stencil}^3 grid" if args.stencil
                 else "synthetic circuit5M-class lower triangle (DESIGN.md)"),
        "config": {"workload": "sptrsv forward, lower CSC", "n": n, "nnz": nnz,
                   "offd_per_col": args.offd, "band": args.band, "levels": levels,
                   "auto_pull_order": "level" if auto_pick == 3 else "natural"},
        "executors": res, "algorithmic_bytes": abytes, "setup_s": round(setup_s, 3),
        "roofline": {"bound": "hbm (latency: level chain)", "peak": 8000.0, "unit": "GB/s"},
    }
    if not args.no_cpu_baseline:
        ref = os.path.join(ROOT, "oracle", "_ref", "libsblas_ref.so")
        if os.path.exists(ref):
            lib = C.CDLL(ref)
            f = lib.ref_sptrsv_serial
            f.restype = C.c_int
            f.argtypes = [C.c_void_p] * 3 + [C.c_int] * 4 + [C.c_void_p] * 2
            xs = np.zeros(n)
            t0 = time.perf_counter()
            f(cp.ctypes.data, ri.ctypes.data, v.ctypes.data, n, nnz, 0, 1, b.ctypes.data, xs.ctypes.data)
            ts = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": round(2.0 * nnz / ts / 1e9, 3), "unit": "GFLOP/s",
                                   "cores": 1, "kind": "reference",
                                   "sample": f"reference sptrsv_syncfree_analyser+_executor "
                                             f"(oracle/_ref) on the full matrix: {ts * 1e3:.1f} ms",
                                   "rel_l1_vs_xref": float(np.abs(xs - xref).sum() / np.abs(xref).sum())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
