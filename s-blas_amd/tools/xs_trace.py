#!/usr/bin/env python3
"""Summarise an SBLAS_XS_TRACE timeline of the column-sorted SpMV (xsort.hip).

Rows (100 MHz s_memrealtime ticks): {subA, subB, block<<4|xcc, t0, endA, endB}
per work item, and {-2, -2, block<<4|xcc, entry, exit, 0} per workgroup.
A sub-item is range<<8 | k (k = 0 narrow, k+1 = wide sub-item of XCD k),
-1 = none.  Prints, for the last launches: span, per-kind sub-item durations,
the idle tail and the workgroups' busy fraction.  Debugging aid for DESIGN.md.
"""
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
    wg = a[a[:, 0] == -2]
    it = a[a[:, 0] != -2]
    base = wg[:, 3].min() if len(wg) else it[:, 3].min()
    us = lambda t: (t - base) * 1e-2  # noqa: E731
    span = us(wg[:, 4]).max() if len(wg) else us(it[:, 4:6].max(1)).max()
    print(f"launch -{len(launches[-3:]) - li}: items {len(it)}  workgroups {len(wg)}  span {span:.1f} us")
    durs = {"narrow": [], "wide": []}
    for subcol, endcol in ((0, 4), (1, 5)):
        sub = it[:, subcol]
        ok = sub >= 0
        d = (it[ok, endcol] - it[ok, 3]) * 1e-2
        for kind, sel in (("narrow", (sub[ok] & 255) == 0), ("wide", (sub[ok] & 255) != 0)):
            durs[kind].extend(d[sel].tolist())
    for kind, d in durs.items():
        if d:
            d = np.array(d)
            print(f"  {kind:6s} sub-items {len(d):5d}  dur med {np.median(d):6.1f} us  "
                  f"p10 {np.percentile(d, 10):6.1f}  p90 {np.percentile(d, 90):6.1f}  max {d.max():6.1f}")
    item_end = us(it[:, 4:6].max(1))
    item_dur = (it[:, 4:6].max(1) - it[:, 3]) * 1e-2
    imb = np.abs(it[:, 4] - it[:, 5])[(it[:, 0] >= 0) & (it[:, 1] >= 0)] * 1e-2
    if len(imb):
        print(f"  pair imbalance |endA-endB| med {np.median(imb):.1f} us  p90 {np.percentile(imb, 90):.1f} us")
    print(f"  item ends: p50 {np.percentile(item_end, 50):.1f}  p90 {np.percentile(item_end, 90):.1f}  "
          f"max {item_end.max():.1f} us; item dur med {np.median(item_dur):.1f} us")
    if len(wg):
        busy = {}
        for b, d in zip(it[:, 2] >> 4, item_dur):
            busy[b] = busy.get(b, 0.0) + d
        bb = np.array(list(busy.values()))
        ent = us(wg[:, 3])
        print(f"  wg entry spread p90 {np.percentile(ent, 90):.1f} us; busy med {np.median(bb):.1f} "
              f"max {bb.max():.1f} us ({np.sum(bb) / (len(wg) * span):.0%} of span)")
    print("  xcc histogram", np.bincount(it[:, 2] & 15, minlength=8).tolist())
