#!/usr/bin/env python3
"""Experiment: column-panel SpMV built from the existing row-split kernel.

Splits the config-2 matrix into P column panels (each a CSR with its own
rowptr), then y = alpha*A_0 x + beta*y; y += alpha*A_p x for p >= 1.  If
x-gathers become L2 hits, the sum of P launches beats one launch.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sblas  # noqa: E402

n = 2_000_000
rp = sblas.gen_synth_rowptr(n)
col, val = sblas.gen_synth_rows(n, rp, 0, n)
x = torch.from_numpy(sblas.gen_vector(n, 43)).cuda()
y = torch.zeros(n, dtype=torch.float64, device="cuda")
rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
s = torch.cuda.Stream()
sp = s.cuda_stream


def run(mats, reps=20):
    with torch.cuda.stream(s):
        for _ in range(3):
            for i, A in enumerate(mats):
                A.spmv(1, 0.84, x.data_ptr(), 0.39 if i == 0 else 1.0, y.data_ptr(), sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            for i, A in enumerate(mats):
                A.spmv(1, 0.84, x.data_ptr(), 0.39 if i == 0 else 1.0, y.data_ptr(), sp)
        e1.record(s)
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for P in [1, 2, 4, 8, 16, 32]:
    W = (n + P - 1) // P
    panel = col // W
    mats = []
    t0 = time.time()
    for p in range(P):
        sel = panel == p
        prow = rows[sel]
        prp = np.zeros(n + 1, np.int64)
        np.add.at(prp, prow + 1, 1)
        prp = np.cumsum(prp)
        A = sblas.DeviceCSR.upload(0, n, prp, np.ascontiguousarray(col[sel]),
                                   np.ascontiguousarray(val[sel]))
        A.analyse(1)
        mats.append(A)
    ms = run(mats)
    print(f"P={P:3d} W={W*8/2**20:6.2f} MiB  {ms*1e3:8.1f} us/SpMV  "
          f"({2*len(col)/ms/1e6:.1f} GFLOP/s)  build {time.time()-t0:.1f}s", flush=True)
    for A in mats:
        A.close()
