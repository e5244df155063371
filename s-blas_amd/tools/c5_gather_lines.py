#!/usr/bin/env python3
"""Host-side count (no GPU) behind profiles/r05/c5light: distinct 128-B x lines
per CSR5 gather instruction (lane l of a tile holds entries 16l..16l+15, so
instruction k gathers entries 16l + k, l = 0..63) on configs[2]'s N = 8
nnz-split heavy rank 0 and light rank 7."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sblas  # noqa: E402

n = 2_000_000
rp = sblas.gen_synth_rowptr(n)
for label, r0, r1 in (("heavy rank 0", 0, 51758), ("light rank 7", n - 552084, n)):
    col, _ = sblas.gen_synth_rows(n, rp, r0, r1)
    T = len(col) // 1024
    lines = (col[:T * 1024] // 16).reshape(T, 64, 16)
    per = [len(np.unique(lines[t, :, k])) for t in range(0, T, 7) for k in range(16)]
    print(f"{label}: rows {r1 - r0}, nnz {len(col)}, distinct x lines per 64-lane gather {np.mean(per):.1f}")
