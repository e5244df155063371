#!/usr/bin/env python3
"""Per-GPU SpMV kernel time of ONE rank's share of config 2 at N ranks.

bench.py at N > 1 deals the rows to the ranks in cyclic chunks
(sblas_dist.make_cyclic_plan); this tool builds rank 0's local CSR for N in
--worlds on the single GPU of the box and times each kernel on it alone
(warm back-to-back and cold after a 1 GiB scrub, HIP events on the launch
stream), so the kernel choice per N can be made without an 8-GPU node.
Prints one JSON line per (N, algo).
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
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--algos", default="xsort,panel,rowsplit")
    ap.add_argument("--nrows", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm-x", action="store_true",
                    help="experiment: read x after each scrub (x in the Infinity Cache and L2s "
                         "when the timed span starts; the matrix stays cold)")
    ap.add_argument("--parts", type=int, default=1,
                    help="also time the slice cut into K parts of consecutive local chunks (the "
                         "overlapped exchange's kernels, sblas_ctx_matrix_upload_parts): the K "
                         "launches back to back after a cold sweep, events between them")
    ap.add_argument("--partition", choices=["cyclic", "nnz", "cost"], default="cyclic",
                    help="cyclic (bench.py's default leg), nnz (configs[2]'s spMV_mgpu_v1 split, the "
                         "config3 leg: ranks hold different row classes, so --ranks all) or cost (the "
                         "cost-weighted whole-row split, config3's cost_weighted leg)")
    ap.add_argument("--row-cost", type=float, default=3.0, help="per-row weight of --partition cost")
    ap.add_argument("--ranks", default="0", help="ranks whose slices to time: a list or 'all'")
    ap.add_argument("--floor", action="store_true",
                    help="also time the slice's streaming floor (slice_floor: one cold read-stream "
                         "kernel over the bytes xsort moves for the slice)")
    args = ap.parse_args()

    import torch
    import sblas
    import sblas_dist

    dev = torch.device("cuda", 0)
    n = args.nrows
    rowptr = sblas.gen_synth_rowptr(n, 96, 9)
    x = torch.from_numpy(sblas.gen_vector(n, 43)).to(dev)
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    algos = {"rowsplit": sblas.ROWSPLIT, "csr5": sblas.CSR5, "panel": sblas.PANEL,
             "xsort": sblas.XSORT}
    rows_fn = lambda a, b: sblas.gen_synth_rows(n, rowptr, a, b, 96, 9, seed=42)
    for world in [int(w) for w in args.worlds.split(",")]:
      ranks = range(world) if args.ranks == "all" else [int(r) for r in args.ranks.split(",") if int(r) < world]
      for rank in ranks:
        plan = None
        if args.partition == "cyclic":
            plan = sblas_dist.make_cyclic_plan(rowptr, n, world)
            lrp, col, val = sblas_dist.cyclic_local_csr(rowptr, plan, rank, rows_fn)
        else:  # whole rows of the nnz split (its split rows' shares rounded to whole rows),
               # or of the cost-weighted whole-row split (sblas_partition_cost)
            _, _, sr, er, _ = (sblas.partition_nnz(rowptr, world) if args.partition == "nnz"
                               else sblas.partition_cost(rowptr, world, args.row_cost))
            a, b = int(sr[rank]), int(er[rank]) + 1
            lrp = np.asarray(rowptr[a:b + 1], np.int64) - int(rowptr[a])
            col, val = rows_fn(a, b)
        for name in args.algos.split(","):
            A = sblas.DeviceCSR.upload(0, n, lrp, col, val)
            A.analyse(algos[name])
            y = torch.zeros(len(lrp) - 1, dtype=torch.float64, device=dev)
            out = {}
            with torch.cuda.stream(stream):
                for mode in ("warm", "cold"):
                    ts = []
                    for k in range(args.reps + 2):
                        if mode == "cold":
                            scrub.add_(1)
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(stream)
                        A.spmv(algos[name], 1.0, x.data_ptr(), 0.5, y.data_ptr(), stream.cuda_stream)
                        e1.record(stream)
                        if mode == "cold":
                            torch.cuda.synchronize()
                        ts.append((e0, e1))
                    torch.cuda.synchronize()
                    out[mode + "_us"] = round(float(np.median([a.elapsed_time(b) for a, b in ts[2:]])) * 1e3, 1)
                # cold as bench.py times it at N = 1: read-only 1 GiB sweep,
                # then the call's device span (runtime events at the first
                # kernel's start and the last kernel's end)
                spans = []
                for k in range(args.reps + 2):
                    scrub.sum(dtype=torch.int64)
                    if args.warm_x:
                        x.sum()
                    torch.cuda.synchronize()
                    spans.append(A.spmv_timed(algos[name], 1.0, x.data_ptr(), 0.5, y.data_ptr(),
                                              stream.cuda_stream))
                out["cold_span_us"] = round(float(np.median(spans[2:])) * 1e3, 1)
                out["cold_span_min_us"] = round(float(np.min(spans[2:])) * 1e3, 1)
            if args.parts > 1 and plan is not None:
                out.update(time_parts(args, plan, lrp, col, val, n, algos[name], A.pick() if algos[name] == 0
                                      else algos[name], x, scrub, stream, torch, sblas))
            A.close()
            print(json.dumps({"world": world, "rank": rank, "partition": args.partition,
                              "algo": name, "local_rows": int(len(lrp) - 1),
                              "local_nnz": int(lrp[-1]), **out}), flush=True)
        if args.floor:
            print(json.dumps(slice_floor(args, lrp, col, val, n, x, scrub, stream, torch, sblas, world)), flush=True)


def slice_floor(args, lrp, col, val, n, x, scrub, stream, torch, sblas, world):
    """the streaming floor of a rank's slice -- ONE
    hand-written read-stream kernel (sblas_hbm_probe: 16-B loads, 8 in flight
    per lane) over exactly the bytes the column-sorted kernel must move for
    the slice (its chunk layout incl. padding and wide-range partials, x
    once, y read and written), cold (1 GiB read sweep before each), timed as
    the SpMV spans are (runtime-stamped kernel start / end events), over
    launch shapes (grid-stride or one span per workgroup, plain or
    non-temporal loads, 1-16 workgroups per CU); the best shape is the
    floor."""
    m = len(lrp) - 1
    A = sblas.DeviceCSR.upload(0, n, lrp, col, val)
    A.analyse(sblas.XSORT)
    layout = int(A.plan_bytes(sblas.XSORT))
    A.close()
    nbytes = (layout + 8 * n + 16 * m + 15) // 16 * 16
    buf = torch.ones(nbytes // 8, dtype=torch.float64, device=x.device)
    sink = torch.zeros(2, dtype=torch.float64, device=x.device)
    shapes = {}
    with torch.cuda.stream(stream):
        for mode, name in ((0, "grid"), (1, "grid_nt"), (3, "span"), (4, "span_nt")):
            for wg in (1, 2, 4, 8, 16):
                ts = []
                for k in range(args.reps + 2):
                    scrub.sum(dtype=torch.int64)
                    torch.cuda.synchronize()
                    ts.append(sblas.hbm_probe_timed(mode, buf.data_ptr(), sink.data_ptr(), nbytes, wg,
                                                    stream.cuda_stream))
                shapes[f"{name}_wg{wg}"] = round(float(np.median(ts[2:])) * 1e3, 2)
    del buf
    best = min(shapes, key=shapes.get)
    us = shapes[best]
    return {"world": world, "floor": "cold read stream of the slice's xsort bytes (sblas_hbm_probe_timed)",
            "layout_bytes": layout, "x_bytes": 8 * n, "y_bytes": 16 * m, "bytes": nbytes,
            "best_shape": best, "us": us, "gbps": round(nbytes / us / 1e3, 1), "shapes_us": shapes}


def time_parts(args, plan, lrp, col, val, n, algo, resolved, x, scrub, stream, torch, sblas):
    """The slice in K parts of consecutive local chunks, as the ctx's
    overlapped exchange cuts it (ctx.hip upload_parts): cold sweep, then the
    K launches back to back; per-part event spans (median over reps)."""
    K, R = args.parts, plan.chunk_rows
    lm = len(lrp) - 1
    ncmax = plan.stride // R
    bounds = [min(lm, (p * ncmax // K) * R) for p in range(K + 1)]
    bounds[-1] = lm
    handles = []
    for p in range(K):
        r0, r1 = bounds[p], bounds[p + 1]
        if r1 <= r0:
            continue
        H = sblas.DeviceCSR.upload_slice(0, n, lrp, col, val, r0, r1, int(lrp[r0]), int(lrp[r1]))
        H.analyse(resolved)
        handles.append((H, r0))
    y = torch.zeros(lm, dtype=torch.float64, device=x.device)
    per = []
    with torch.cuda.stream(stream):
        for k in range(args.reps + 2):
            scrub.sum(dtype=torch.int64)
            torch.cuda.synchronize()
            torch.cuda._sleep(500_000)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(handles) + 1)]
            ev[0].record(stream)
            for j, (H, r0) in enumerate(handles):
                H.spmv(resolved, 1.0, x.data_ptr(), 0.5, y.data_ptr() + 8 * r0, stream.cuda_stream)
                ev[j + 1].record(stream)
            torch.cuda.synchronize()
            per.append([ev[j].elapsed_time(ev[j + 1]) for j in range(len(handles))])
    for H, _ in handles:
        H.close()
    med = np.median(np.array(per[2:]), axis=0) * 1e3
    return {"parts": len(handles), "parts_cold_us": [round(float(v), 1) for v in med],
            "parts_total_cold_us": round(float(np.sum(med)), 1)}


if __name__ == "__main__":
    main()
