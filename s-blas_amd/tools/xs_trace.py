#!/usr/bin/env python3
"""Summarise an SBLAS_XS_TRACE timeline of the column-sorted SpMV (xsort.hip):
per launch, item durations vs entries, per-workgroup busy time, the span and
the idle tail.  Debugging aid for DESIGN.md's xsort notes."""
import sys

import numpy as np

launches, cur = [], None
for line in open(sys.argv[1]):
    if line.startswith("#"):
        cur = []
        launches.append(cur)
        continue
    cur.append([int(v) for v in line.split()])
for li, rows in enumerate(launches[-3:]):
    a = np.array(rows, dtype=np.int64)
    item, f, t0, t1 = a.T
    cnt, blk, xcc = f >> 20, (f >> 4) & 0xffff, f & 15
    narrow = (item & 255) == 0
    dur = (t1 - t0) * 10e-3  # 100 MHz -> us
    start = (t0 - t0.min()) * 10e-3
    end = (t1 - t0.min()) * 10e-3
    print(f"launch -{3 - li}: items {len(a)}  span {end.max():.1f} us  "
          f"first start spread {np.sort(start)[min(len(a) - 1, 255)]:.1f} us")
    for name, sel in (("narrow", narrow), ("wide", ~narrow)):
        if sel.any():
            rate = cnt[sel] / np.maximum(dur[sel], 1e-3)
            print(f"  {name:6s} n={sel.sum():4d}  entries med {np.median(cnt[sel]):9.0f}  "
                  f"dur med {np.median(dur[sel]):6.1f} us (min {dur[sel].min():.1f} max {dur[sel].max():.1f})"
                  f"  entries/us med {np.median(rate):7.0f}")
    per_blk = {}
    for b, d in zip(blk, dur):
        per_blk[b] = per_blk.get(b, 0.0) + d
    busy = np.array(list(per_blk.values()))
    print(f"  workgroups {len(busy)}  busy med {np.median(busy):.1f} max {busy.max():.1f} us; "
          f"ends: p50 {np.percentile(end, 50):.1f} p90 {np.percentile(end, 90):.1f} max {end.max():.1f} us")
    print("  xcc histogram", np.bincount(xcc, minlength=8).tolist())
