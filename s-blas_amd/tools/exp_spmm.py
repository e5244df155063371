#!/usr/bin/env python3
"""Experiment driver: config 4 SpMM (rail4284-shaped stand-in x 64, B
row-major resident) under planner test options (sblas.test_options).

For each option set (JSON objects) builds the plan, times --reps cold calls
(1 GiB read sweep, device-side hold, HIP events around the call -- bench.py's
config4 protocol at N = 1), checks every C entry once against the oracle's
csrmm restatement under the per-entry bound, and prints one JSON line.
Experiment tooling only; the oracle is the checker.

  python exp_spmm.py --opts '[{}, {"spmm_pipe": 1}, {"spmm_pipe": 1, "spmm_epochs": 32}]'
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
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opts", default="[{}]")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    import torch
    import sblas
    from bench_spmm import rail_like
    m, k, n = 4284, 1_092_610, 64
    alpha, beta = -0.7, 0.8
    rp, col = rail_like(m, k, 11_279_748, 44)
    val = np.random.default_rng(45).random(11_279_748)
    dev = torch.device("cuda", 0)
    B = torch.rand((k, n), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(45))
    C0 = torch.rand((n, m), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(46))
    scrub = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    want = bound = None
    if not a.no_check:
        import orc  # checker only
        want, bound = orc.spmm_checked(m, n, alpha, rp, col, val, B.cpu().numpy(), beta, C0.cpu().numpy().T)
    for rnd in range(a.rounds):
        for opts in json.loads(a.opts):
            A = sblas.DeviceCSR.upload(0, k, rp, col, val)
            C = C0.clone()
            t0 = time.perf_counter()
            with sblas.test_options(**opts):
                with torch.cuda.stream(stream):
                    A.spmm(n, alpha, B.data_ptr(), n, 1, beta, C.data_ptr(), m, sp)
                torch.cuda.synchronize()
            build_s = time.perf_counter() - t0
            ok = None
            if want is not None:
                C.copy_(C0)
                with torch.cuda.stream(stream):
                    A.spmm(n, alpha, B.data_ptr(), n, 1, beta, C.data_ptr(), m, sp)
                torch.cuda.synchronize()
                got = C.cpu().numpy().T
                diff = np.abs(got - want)
                ok = bool(np.all(diff <= bound))
            ts = []
            for _ in range(a.reps):
                scrub.sum(dtype=torch.int64)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):
                    torch.cuda._sleep(500_000)
                    e0.record(stream)
                    A.spmm(n, alpha, B.data_ptr(), n, 1, beta, C.data_ptr(), m, sp)
                    e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            A.close()
            print(json.dumps({"round": rnd, "opts": opts, "mean_us": round(float(np.mean(ts)), 2),
                              "min_us": round(float(np.min(ts)), 2), "check": ok, "build_s": round(build_s, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
