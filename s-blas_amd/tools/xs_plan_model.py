#!/usr/bin/env python3
"""Host-side model of the xsort planner (csrc/xsort.hip build_xsort_plan) on
config 2's row structure, used to read the layout experiments of DESIGN.md §6.

It repeats the planner's range cutting (cost = entries + lambda x distinct x
lines, cap grown until the sub-items fit the slots), then counts for every
item (what one workgroup = one CU runs) its L1->L2 line requests: the x lines
its gathers touch (uniform columns: L (1 - exp(-c / L)) per block) plus the
128-B lines of its entry stream (12 B per entry).  Items are dealt to the
CUs in queue order (greedy, as the persistent grid claims them); the model
time is the busiest CU's requests x CYCLES_PER_REQUEST / clock.

No GPU needed.  Usage: python3 xs_plan_model.py [--n 2000000] [--world 1]
"""
import argparse
import heapq
import math
import os
import sys

import numpy as np

CUS = 256
CLOCK = 2.4e9
CYCLES_PER_REQUEST = 4.0  # calibrated on the default layout at N = 1 (131 us)


def config2_rowptr(n, heavy=96, light=9, world=1):
    """Row lengths of rank 0's cyclic share (sblas_dist.make_cyclic_plan:
    8*world equal chunks, chunk j to rank j % world)."""
    lens = np.where(np.arange(n) < n // 8, heavy, light).astype(np.int64)
    if world > 1:
        nch = 8 * world
        cr = (n + nch - 1) // nch
        keep = np.zeros(n, bool)
        for j in range(0, nch, world):
            keep[j * cr:min(n, (j + 1) * cr)] = True
        lens = lens[keep]
    rp = np.zeros(len(lens) + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    return rp


def plan(rp, n, mode="paired", lam=1.0, rows_cap=None, wstar=None, pairing="grid", lsplit=None, k=1, allwide=False):
    """pairing: leftover light sub-items two to an item only as far as the
    grid needs ("grid", the planner since round 3) or always ("always")."""
    m, nnz = len(rp) - 1, int(rp[-1])
    nmib = (n * 8 + (1 << 20) - 1) >> 20
    q = max(1, (math.ceil(n / ((1 << 18) - 1)) + 7) // 8, (nmib + 7) // 8)
    G = 8 * q
    Wg = (n + G - 1) // G
    Lg = max(1.0, Wg / 16.0)
    pair = mode in ("paired", "solo")
    solo = mode == "solo"
    cap_rows = rows_cap or (8192 if pair else 16384)
    ncap_rows = 16384 if solo else cap_rows
    nfac = 2.0 if solo else 1.0
    slots = CUS * (2 if pair else 1) * k  # k: items per CU (SBLAS_XS_K)

    def nc(c):
        return c + lam * G * Lg * (1 - math.exp(-c / (G * Lg)))

    def wc(c):
        ci = c / 8.0
        return ci + lam * q * Lg * (1 - math.exp(-ci / (q * Lg)))

    def cut(r, wide, cap):
        emax = min(m, r + (cap_rows if wide else ncap_rows))
        lo, hi = r + 1, emax
        while lo < hi:
            mid = lo + (hi - lo + 1) // 2
            c = rp[mid] - rp[r]
            if (wc(c) <= cap) if wide else (nc(c) <= nfac * cap):
                lo = mid
            else:
                hi = mid - 1
        return lo, int(rp[lo] - rp[r])

    def build(cap):
        out, r = [], 0
        while r < m:
            e, cnt = cut(r, True, cap)
            wide = cnt > 0 and (allwide or (nc(cnt) > nfac * cap and cnt >= 16 * (e - r)))
            if not wide:
                e, cnt = cut(r, False, cap)
            out.append((e - r, wide, cnt))
            r = e
        return out

    cap = wstar or nc(nnz) / slots
    for _ in range(400):
        ranges = build(cap)
        subs = sum(8 if w else (2 if solo else 1) for _, w, _ in ranges)
        if subs <= slots or wstar:
            break
        cap *= 1.02

    def req(cnt, wide):
        L = q * Lg if wide else G * Lg
        c = cnt / 8.0 if wide else cnt
        return L * (1 - math.exp(-c / L)) + c * 12 / 128

    nsub = [req(c, False) for _, w, c in ranges if not w]
    if lsplit:
        # the light rows re-cut into ranges of R rows, each
        # split S ways by column group (S sub-items over G / S groups, partials
        # added by the reduce).  A sub-item's block density (entries per x
        # line) is R * nnz_row * 16 / n whatever S is: only R (the LDS rows of
        # one team) sets it; S only makes the work units smaller.
        S, R = lsplit
        light = [(r, c) for r, w, c in ranges if not w]
        lrows = sum(r for r, _ in light)
        lnnz = sum(c for _, c in light)
        nr = max(1, math.ceil(lrows / R))
        c = lnnz / nr / S
        L = G * Lg / S
        # + the sub-item's partial stores (8 B per row, 128-B lines)
        one = L * (1 - math.exp(-c / L)) + c * 12 / 128 + (lrows / nr) * 8 / 128
        nsub = [one] * (nr * S)
    wsub = [[req(c, True) for _, w, c in ranges if w] for _ in range(8)]
    # items in queue order (xsort.hip: pairing per XCD, queues interleaved)
    queues = [[] for _ in range(8)]
    if not pair:
        for k in range(8):
            queues[k] += wsub[k]
        for j, v in enumerate(nsub):
            queues[j % 8].append(v)
        for k in range(8):
            queues[k].sort(reverse=True)
    elif solo:
        for j, v in enumerate(nsub):
            queues[j % 8].append(v)
        for k in range(8):
            ws = [wsub[k][j] + (wsub[k][j + 1] if j + 1 < len(wsub[k]) else 0)
                  for j in range(0, len(wsub[k]), 2)]
            mixed = []
            for j in range(max(len(queues[k]), len(ws))):
                if j < len(queues[k]):
                    mixed.append(queues[k][j])
                if j < len(ws):
                    mixed.append(ws[j])
            queues[k] = mixed
    else:
        ni, left = 0, [[] for _ in range(8)]
        for j in range(max(len(w) for w in wsub) if wsub[0] else 0):
            for k in range(8):
                if j >= len(wsub[k]):
                    continue
                if ni < len(nsub):
                    queues[k].append(nsub[ni] + wsub[k][j])
                    ni += 1
                else:
                    left[k].append(wsub[k][j])
        for k in range(8):
            for j in range(0, len(left[k]), 2):
                queues[k].append(left[k][j] + (left[k][j + 1] if j + 1 < len(left[k]) else 0))
        t = 0
        left = len(nsub) - ni
        free = max(0, CUS * k - sum(map(len, queues)))
        npairs = max(0, left - free) if pairing == "grid" else left // 2
        npairs = min(npairs, left // 2)
        while ni < len(nsub):
            if npairs > 0 and ni + 1 < len(nsub):
                queues[t % 8].append(nsub[ni] + nsub[ni + 1])
                ni += 2
                npairs -= 1
            else:
                queues[t % 8].append(nsub[ni])
                ni += 1
            t += 1
    # 32 CUs per XCD claim from their own queue first (greedy list schedule)
    if os.environ.get("XS_MODEL_DEBUG"):
        print("queue totals (k req):", [round(sum(qq) / 1e3) for qq in queues],
              "items:", [len(qq) for qq in queues], "largest items (k):",
              sorted((round(v / 1e3, 1) for qq in queues for v in qq), reverse=True)[:6],
              "wide sub-items per XCD:", [len(w) for w in wsub], "narrow:", len(nsub))
    busiest = 0.0
    for k in range(8):
        heap = [0.0] * (CUS // 8)
        for v in queues[k]:
            heapq.heappush(heap, heapq.heappop(heap) + v)
        busiest = max(busiest, max(heap))
    total_req = sum(nsub) + sum(map(sum, wsub))
    return {"mode": mode + (f" lsplit S={lsplit[0]} R={lsplit[1]}" if lsplit else ""), "rows_cap": cap_rows, "narrow": len(nsub), "wide_ranges": sum(1 for _, w, _ in ranges if w),
            "items": sum(map(len, queues)), "requests_M": round(total_req / 1e6, 2),
            "busiest_cu_k": round(busiest / 1e3, 1),
            # perfect balance: the chip's requests spread evenly over the CUs
            "balanced_k": round(total_req / CUS / 1e3, 1),
            "model_us": round(busiest * CYCLES_PER_REQUEST / CLOCK * 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rmat", type=int, default=0, help="model an R-MAT graph of this scale instead")
    ap.add_argument("--lsplit", action="store_true", help="also model light ranges split S ways by columns")
    args = ap.parse_args()
    rp = config2_rowptr(args.n, world=args.world)
    if args.rmat:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        import sblas
        rp, _, _ = sblas.gen_rmat(args.rmat, 16, seed=50)
        n = len(rp) - 1
        for pairing in ("always", "grid"):
            print(pairing, plan(rp, n, "paired", pairing=pairing))
        return
    for mode, rc in (("paired", None), ("solo", None), ("unpaired", None)):
        print(plan(rp, args.n, mode, rows_cap=rc))
    if args.lsplit:
        # light ranges split S ways by columns at R rows per range (R <= 8192:
        # a team's LDS rows), partial bytes 8 * S per light row written + read
        base = plan(rp, args.n, "paired")
        for S in (1, 2, 4):
            for R in (4096, 6912, 8192):
                r = plan(rp, args.n, "paired", lsplit=(S, R))
                lrows = int(np.sum(np.diff(rp) < 96)) if args.world == 1 else None
                extra = None if lrows is None or S == 1 else round(2 * 8 * S * lrows / 1e6, 1)
                print(r, "partial MB (write + read):", extra,
                      "vs default busiest", base["busiest_cu_k"])


if __name__ == "__main__":
    main()
