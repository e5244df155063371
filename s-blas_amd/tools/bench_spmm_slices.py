#!/usr/bin/env python3
"""Per-rank SpMM slice kernels of BASELINE configs[3] at N = 2 / 4 / 8, timed on
one MI355X, with the C all-gather projected per xGMI link rate (VERDICT r04
item 3; the SpMV counterpart is DESIGN.md §7's slice table).

bench.py's config4 leg at N > 1 (sblas_dist.DistSpMM, split "rows") gives
rank d the whole rows [rb[d], rb[d+1]) of A by nnz (row_blocks_by_nnz), B
replicated, C slices all-gathered.  Here every rank's slice of the
rail4284-shaped stand-in (bench_spmm.rail_like: m 4,284, k 1,092,610, nnz
11,279,748, 64 columns of B) is uploaded on the box's one GPU and its
C = -0.7 A B + 0.8 C timed cold (1 GiB read sweep before each call, device-side
hold, HIP events on the launch stream), so the N-GPU step can be projected
without an 8-GPU node:

  step(N) = max_d kernel_d + all-gather(C) + 3 us placement,
  all-gather(C) = (C bytes / N) / link rate   (rank d receives N-1 slices of
                  C/N, one per xGMI link, all links in parallel),

at an assumed 64 and 153 GB/s per link and direction (MI355X_MICROARCH.md:
7 links x ~153 GB/s).  Prints one JSON line per (N, rank) and a summary line
per N.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--ncols", type=int, default=64)
    ap.add_argument("--split", choices=["rows", "cols", "grid"], default="rows",
                    help="rows (north star; DistSpMM split='rows'), cols (the reference's column split) "
                         "or grid (row blocks x column groups, sblas_dist.spmm_grid_shape)")
    args = ap.parse_args()
    import torch
    import sblas
    import sblas_dist
    from bench_spmm import rail_like

    m, k, nnz, n = 4284, 1_092_610, 11_279_748, args.ncols
    rp, col = rail_like(m, k, nnz, 44)
    val = np.random.default_rng(45).random(nnz)
    dev = torch.device("cuda", 0)
    B = torch.rand((k, n), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(45))
    C0 = torch.rand((n, m), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(46))
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    c_bytes = 8 * m * n
    for world in [int(w) for w in args.worlds.split(",")]:
        if args.split == "cols":
            per = cols_slices(args, world, m, k, n, rp, col, val, B, C0, scrub, stream, torch, sblas)
            summary(world, per, c_bytes)
            continue
        if args.split == "grid":
            per = grid_slices(args, world, m, k, n, rp, col, val, B, C0, scrub, stream, torch, sblas,
                              sblas_dist)
            summary(world, per, c_bytes)
            continue
        rb = sblas_dist.row_blocks_by_nnz(rp, world)
        per = []
        for d in range(world):
            r0, r1 = int(rb[d]), int(rb[d + 1])
            A = sblas.DeviceCSR.upload_slice(0, k, rp, col, val, r0, r1, int(rp[r0]), int(rp[r1]))
            stride = max(1, r1 - r0)
            Cl = C0[:, r0:r1].contiguous() if r1 > r0 else torch.zeros((n, 1), dtype=torch.float64, device=dev)
            ts = []
            with torch.cuda.stream(stream):
                for it in range(args.reps + 2):
                    scrub.sum(dtype=torch.int64)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda._sleep(500_000)
                    e0.record(stream)
                    A.spmm(n, -0.7, B.data_ptr(), n, 1, 0.8, Cl.data_ptr(), stride, stream.cuda_stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
            us = float(np.median(ts[2:])) * 1e3
            lnnz = int(rp[r1] - rp[r0])
            abytes = 12 * lnnz + 4 * (r1 - r0 + 1) + 8 * k * n + 16 * (r1 - r0) * n
            per.append(us)
            print(json.dumps({"world": world, "rank": d, "rows": r1 - r0, "nnz": lnnz, "kernel_cold_us": round(us, 1),
                              "algorithmic_bytes": abytes,
                              "roofline_frac": round(abytes / (us * 1e-6) / 8e12, 4)}), flush=True)
            A.close()
        summary(world, per, c_bytes)


def timed_cold(args, torch, stream, scrub, fn):
    ts = []
    with torch.cuda.stream(stream):
        for it in range(args.reps + 2):
            scrub.sum(dtype=torch.int64)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(500_000)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts[2:])) * 1e3


def cols_slices(args, world, m, k, n, rp, col, val, B, C0, scrub, stream, torch, sblas):
    """The reference's own split (dspmm_mgpu_baseline.cu:147-150): A
    replicated, rank d owns B/C columns [d*n/g, (d+1)*n/g) -- its kernel reads
    all of A and its columns' share of every touched B row."""
    A = sblas.DeviceCSR.upload(0, k, rp, col, val)
    per = []
    for d in range(world):
        c0, c1 = d * n // world, (d + 1) * n // world
        Cl = C0[c0:c1].contiguous()
        us = timed_cold(args, torch, stream, scrub,
                        lambda: A.spmm(c1 - c0, -0.7, B.data_ptr() + 8 * c0, n, 1, 0.8, Cl.data_ptr(), m,
                                       stream.cuda_stream))
        nnz = int(rp[-1])
        abytes = 12 * nnz + 4 * (m + 1) + 8 * k * (c1 - c0) + 16 * m * (c1 - c0)
        per.append(us)
        print(json.dumps({"world": world, "rank": d, "split": "cols", "cols": c1 - c0, "kernel_cold_us": round(us, 1),
                          "algorithmic_bytes": abytes,
                          "roofline_frac": round(abytes / (us * 1e-6) / 8e12, 4)}), flush=True)
    A.close()
    return per


def grid_slices(args, world, m, k, n, rp, col, val, B, C0, scrub, stream, torch, sblas, sblas_dist):
    """Row blocks by nnz x column groups (DistSpMM split "grid"): rank d's
    rows of A times its columns of B into its C block (ld = rows)."""
    R, Cg = sblas_dist.spmm_grid_shape(world, n)
    rb = sblas_dist.row_blocks_by_nnz(rp, R)
    per = []
    for d in range(world):
        r0, r1 = int(rb[d // Cg]), int(rb[d // Cg + 1])
        c0, c1 = d % Cg * n // Cg, (d % Cg + 1) * n // Cg
        A = sblas.DeviceCSR.upload_slice(0, k, rp, col, val, r0, r1, int(rp[r0]), int(rp[r1]))
        stride = max(1, r1 - r0)
        Cl = C0[c0:c1, r0:r1].contiguous()
        us = timed_cold(args, torch, stream, scrub,
                        lambda: A.spmm(c1 - c0, -0.7, B.data_ptr() + 8 * c0, n, 1, 0.8, Cl.data_ptr(), stride,
                                       stream.cuda_stream))
        lnnz = int(rp[r1] - rp[r0])
        abytes = 12 * lnnz + 4 * (r1 - r0 + 1) + 8 * k * (c1 - c0) + 16 * (r1 - r0) * (c1 - c0)
        per.append(us)
        print(json.dumps({"world": world, "rank": d, "split": "grid", "shape": [R, Cg], "rows": r1 - r0,
                          "cols": c1 - c0, "nnz": lnnz, "kernel_cold_us": round(us, 1),
                          "algorithmic_bytes": abytes,
                          "roofline_frac": round(abytes / (us * 1e-6) / 8e12, 4)}), flush=True)
        A.close()
    return per


def summary(world, per, c_bytes):
    kmax = max(per)
    proj = {}
    for link in (64.0, 153.0):
        ag = 0.0 if world == 1 else (c_bytes / world) / (link * 1e9) * 1e6
        step = kmax + (ag + 3.0 if world > 1 else 0.0)
        proj[f"{int(link)}GBps"] = {"allgather_us": round(ag, 1), "step_us": round(step, 1)}
    print(json.dumps({"world": world, "summary": True, "kernel_max_us": round(kmax, 1),
                      "kernel_min_us": round(min(per), 1), "c_bytes": c_bytes, "projection": proj}), flush=True)


if __name__ == "__main__":
    main()
