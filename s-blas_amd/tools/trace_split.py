#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `python bench.py` into its phases
(warm-up, cold-timed, warm-timed, in launch order) and print per-phase mean
durations of the SpMV kernels, so the trace can be compared with bench.py's
HIP-event kernel_ms.  Usage: trace_split.py run_kernel_trace.csv [warmup steps]"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    warm_up = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = [r for r in csv.DictReader(open(path)) if "sblas::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    main_k = [r for r in rows if "k_spmv_" in r["Kernel_Name"] and "reduce" not in r["Kernel_Name"]]
    red = [r for r in rows if "reduce" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    # bench.py order: warm-up, cold (events), cold (wall clock), warm
    phases = [("warmup", 0, warm_up), ("cold_events", warm_up, warm_up + steps),
              ("cold_wall", warm_up + steps, warm_up + 2 * steps),
              ("warm", warm_up + 2 * steps, warm_up + 3 * steps)]
    for name, a, b in phases:
        if b > len(main_k):
            break
        line = f"{name:12s} {main_k[a]['Kernel_Name'][:40]} mean {st.mean(map(dur, main_k[a:b])):.1f} us"
        if len(red) >= b:
            span = [(int(r2["End_Timestamp"]) - int(r1["Start_Timestamp"])) / 1e3
                    for r1, r2 in zip(main_k[a:b], red[a:b])]
            line += f"; reduce {st.mean(map(dur, red[a:b])):.1f} us; kernel->reduce span {st.mean(span):.1f} us"
        print(line)


if __name__ == "__main__":
    main()
