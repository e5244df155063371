#!/usr/bin/env python3
"""SpMM benchmark (BASELINE configs[3]), 1..N GPUs.

rail4284 is not in the container: synthetic stand-in with its shape, m =
4,284, k = 1,092,610, nnz = 11,279,748 (2,633 nnz/row, uniform-random
distinct sorted columns, seed 44), B k x 64 U[0,1) (seed 45), C0 m x 64
U[0,1) (seed 46), alpha = -0.7, beta = 0.8 (dspmm_baseline_test.cu:518-519).
B is resident row-major; C column-major (ld = m).

  python bench_spmm.py                      # 1 GPU
  torchrun --nproc-per-node N bench_spmm.py # N ranks: rows of A split by nnz,
                                            # B replicated, C slices all-gathered

Algorithmic bytes: 12*nnz + 4(m+1) + 8*k*n + 16*m*n;
GFLOP/s = 2*nnz*n/t.  The traffic-aware bound is the gather of a 512-B B row
per nonzero (nnz*512 B = 5.8 GB through L2), reported as gbps_brow against the
measured random-row gather rates of MI355X_MICROARCH.md (8.6 TB/s from the
Infinity Cache, 5.7 TB/s from HBM).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def rail_like(m, k, nnz, seed):
    rng = np.random.default_rng(seed)
    base, extra = divmod(nnz, m)
    lens = np.full(m, base, np.int64)
    lens[:extra] += 1
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.empty(nnz, np.int32)
    for r in range(m):  # distinct sorted columns per row
        L = int(lens[r])
        c = np.unique(rng.integers(0, k, L + L // 8 + 16))
        while len(c) < L:
            c = np.unique(np.concatenate([c, rng.integers(0, k, L)]))
        col[rp[r]:rp[r + 1]] = np.sort(rng.permutation(c)[:L])
    return rp, col


def blocky(m, k, width, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(m // 16):
        cols = np.sort(rng.choice(k, width, replace=False))
        for _ in range(16):
            rows.append(cols[rng.random(width) < 0.9])
    lens = np.array([len(r) for r in rows], np.int64)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return rp, np.concatenate(rows).astype(np.int32)


def cpu_baseline_spmm(m, n, rp, col, val, B, C0, budget_s=10.0):
    """The oracle's csrmm restatement (orc_spmm_omp, OpenMP over rows; test
    infrastructure, only this leg touches oracle/) on this host's cores."""
    import ctypes as C
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "liboracle.so"))
    f = lib.orc_spmm_omp
    f.restype = None
    f.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                  C.c_int, C.c_double, C.c_void_p, C.c_int, C.c_void_p, C.c_int]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    rp32 = np.ascontiguousarray(rp, np.int32)
    Cw = np.array(C0, np.float64, copy=True, order="F")
    args = (m, n, -0.7, rp32.ctypes.data, col.ctypes.data, val.ctypes.data, B.ctypes.data, n, 1, 0.8,
            Cw.ctypes.data, m, None, threads)
    f(*args)  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        f(*args)
        reps += 1
        el = time.perf_counter() - t0
        if el > budget_s or reps >= 50:
            break
    t = el / reps
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nnz = int(rp[-1])
    return {"value": round(2.0 * nnz * n / t / 1e9, 3), "unit": "GFLOP/s", "cores": threads, "kind": "port",
            "cpu_model": model,
            "sample": f"full config-4 product, orc_spmm_omp (OpenMP over rows, B row-major) x{reps} reps, "
                      f"{t * 1e3:.1f} ms per call"}


def pmc_traffic_spmm():
    """Fabric bytes per call of the C-tile kernels from a committed
    rocprofv3 FETCH/WRITE summary (profiles/pmc_spmm_ctile.json), or None."""
    p = os.path.join(os.path.dirname(os.path.dirname(HERE)), "profiles", "pmc_spmm_ctile.json")
    try:
        with open(p) as fh:
            return float(json.load(fh)["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mrows", type=int, default=4284)
    ap.add_argument("--kcols", type=int, default=1_092_610)
    ap.add_argument("--nnz", type=int, default=11_279_748)
    ap.add_argument("--ncols", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layout", choices=["row", "col"], default="row",
                    help="B layout (1 GPU only; the multi-rank path keeps B row-major)")
    ap.add_argument("--blocky", type=int, default=0,
                    help="instead of the rail4284 shape: 16-row blocks each dense (~90%%) over "
                         "BLOCKY random columns (an FEM-like matrix where MFMA tiles apply)")
    ap.add_argument("--stencil", type=int, default=0,
                    help="instead of the rail4284 shape: a 3-D 27-point stencil on a STENCIL^3 grid "
                         "(sblas_gen_stencil3d; the SuiteSparse-class banded case)")
    ap.add_argument("--points", type=int, default=27, choices=[7, 27])
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 compares EVERY entry of C with the oracle (orc_spmm_omp) under the "
                         "per-entry fp64 bound (DESIGN.md §3), as dspmm_baseline_test.cu:544-549 "
                         "checks every entry; test infrastructure, after the timed steps")
    ap.add_argument("--split", choices=["rows", "cols", "grid"], default="rows",
                    help="rows: whole-row blocks of A by nnz (north star); cols: A replicated, "
                         "B/C columns split (the reference's dspmm_mgpu_baseline.cu:147-150)")
    args = ap.parse_args()
    import torch
    import sblas
    import sblas_dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    m, k, n = args.mrows, args.kcols, args.ncols
    if args.stencil:
        g = args.stencil
        rp, col, _ = sblas.gen_stencil3d(g, g, g, args.points, seed=49)
        m = k = len(rp) - 1
    elif args.blocky:
        rp, col = blocky(m, k, args.blocky, 44)
        m = len(rp) - 1
    else:
        rp, col = rail_like(m, k, args.nnz, 44)
    nnz = int(rp[-1])
    val = np.random.default_rng(45).random(nnz)
    B = torch.rand((k, n), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(45))
    C0 = torch.rand((n, m), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(46))
    s = torch.cuda.Stream(device=dev)
    if world == 1 and args.layout == "col":
        Bd, ldb, lay = B.t().contiguous(), k, 0
    else:
        Bd, ldb, lay = B, n, 1
    op = sblas_dist.DistSpMM(rp, col, val, k, n, world, rank, dev_idx, torch, dist, split=args.split)

    def step(ev=None):
        if ev is not None:
            ev[0].record(s)
        if lay == 1:
            op.kernel(-0.7, Bd, 0.8, s.cuda_stream)
        else:
            op.A.spmm(n, -0.7, Bd.data_ptr(), ldb, 0, 0.8, op.c_local.data_ptr(), op.stride,
                      s.cuda_stream)
        if ev is not None:
            ev[1].record(s)
        op.exchange()

    def sync_barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    with torch.cuda.stream(s):
        op.load_c(C0)
        # the first call builds the plan (C-tile sort, host side) and runs one
        # product: its wall time is the plan-build figure the line reports
        sync_barrier()
        t_first = time.perf_counter()
        step()
        sync_barrier()
        plan_s = time.perf_counter() - t_first
        for _ in range(max(args.warmup - 1, 0)):
            step()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        sync_barrier()
        t0 = time.perf_counter()
        for q in range(args.steps):
            step(evs[q])
        sync_barrier()
        el = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        # one fresh step from C0 for the check
        op.load_c(C0)
        step()
        torch.cuda.synchronize()
    got = op.result().cpu().numpy()
    stats = torch.tensor([el, kern_ms], dtype=torch.float64,
                         device=dev if dist is None or args.dist_backend == "nccl" else "cpu")
    if dist is not None:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    el, kern_max = float(stats[0]), float(stats[1])
    if rank == 0:
        rows = np.random.default_rng(0).choice(m, min(32, m), replace=False)
        Bh = B.cpu().numpy()
        C0h = C0.cpu().numpy()
        err = 0.0
        for r in rows:
            a, b_ = rp[r], rp[r + 1]
            want = -0.7 * (val[a:b_] @ Bh[col[a:b_], :]) + 0.8 * C0h[:, r]
            err = max(err, float(np.max(np.abs(got[:, r] - want) / (np.abs(want) + 1e-300))))
        check = None
        if args.check:
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests"))
            import orc  # oracle: checker only
            want, bound = orc.spmm_checked(m, n, -0.7, rp, col, val, Bh, 0.8, C0h.T)
            diff = np.abs(got.T - want)
            check = {"entries": int(diff.size), "pass": bool(np.all(diff <= bound)),
                     "max_excess_over_bound": float(np.max(diff - bound)),
                     "abs_1e-3": bool(np.all(diff < 1e-3 * np.maximum(1.0, np.abs(want))))}
        ms = el / args.steps * 1e3
        abytes = 12 * nnz + 4 * (m + 1) + 8 * k * n + 16 * m * n
        out = {
            "metric": "fp64 CSR SpMM GFLOP/s (2*nnz*n/t)",
            "value": round(2.0 * nnz * n / ms / 1e6, 3), "unit": "GFLOP/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "kernel_ms_max_over_ranks": round(kern_max, 4),
            "kernel_only_gflops": round(2.0 * nnz * n / kern_max / 1e6, 3),
            "higher_is_better": True, "scaling": "strong", "dtype": "f64",
            "data": "synthetic (DESIGN.md)",
            "config": {"workload": "C = -0.7*A*B + 0.8*C", "m": m, "k": k, "nnz": nnz, "ncols": n,
                       "b_layout": "row" if lay == 1 else "col",
                       "structure": (f"{args.points}-point 3-D stencil {args.stencil}^3" if args.stencil
                                     else f"blocky{args.blocky}" if args.blocky
                                     else "rail4284-shaped uniform random"),
                       "mfma_blocks": int(op.A.spmm_info()[0]) if hasattr(op.A, "spmm_info") else None,
                       "partition": ("single GPU" if world == 1 else
                                     "whole-row blocks by nnz, B replicated, C all-gathered"
                                     if args.split == "rows" else
                                     "row blocks by nnz x B/C column groups, C blocks all-gathered"
                                     if args.split == "grid" else
                                     "A replicated, B/C column slices, C all-gathered"),
                       "mfma_fill_threshold": os.environ.get("SBLAS_SPMM_MFMA_FILL", "0.08")},
            "roofline": {"bound": "hbm", "achieved": round(abytes / kern_max / 1e6, 1), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(abytes / kern_max / 1e6 / 8000.0, 4)},
            "gbps_brow": round(nnz * n * 8 / kern_max / 1e6 / max(world, 1), 1),
            "max_rel_err_32_rows": err,
            "plan_build_s_rank0": round(plan_s, 3),
            "plan_build_note": "wall time of the first call (host plan build + one product)",
        }
        if check is not None:
            out["check_vs_oracle"] = check
        if world == 1 and not args.blocky and not args.stencil and lay == 1:
            out["roofline"]["traffic"] = pmc_traffic_spmm()
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_spmm(m, n, rp, col, val, Bh, C0h.T)
        if world > 1 and args.dist_backend != "nccl":
            out["note"] = f"rehearsal: {world} ranks over gloo"
        print(json.dumps(out), flush=True)
    op.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
