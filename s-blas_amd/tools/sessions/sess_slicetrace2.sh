#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for w in 8 1; do
rm -f gpurun_out/xs_trace_w$w.txt
SBLAS_XS_TRACE=gpurun_out/xs_trace_w$w.txt timeout -k 10 120 python3 s-blas_amd/tools/bench_slice.py --worlds $w --reps 3 --algos xsort > gpurun_out/slicetrace.log 2>&1 || { tail -5 gpurun_out/slicetrace.log; exit 1; }
echo "== N=$w"; python3 s-blas_amd/tools/xs_trace.py gpurun_out/xs_trace_w$w.txt
done
