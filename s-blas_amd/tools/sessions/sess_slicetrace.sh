#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/xs_slice_trace.txt
SBLAS_XS_TRACE=gpurun_out/xs_slice_trace.txt timeout -k 10 120 python3 s-blas_amd/tools/bench_slice.py --worlds 8 --reps 3 --algos xsort > gpurun_out/slicetrace.log 2>&1 || { tail -5 gpurun_out/slicetrace.log; exit 1; }
python3 s-blas_amd/tools/xs_trace.py gpurun_out/xs_slice_trace.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_slice -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/s-blas_amd/tools/bench_slice.py --worlds 8 --reps 10 --algos xsort,panel > $GRAFT_REPO_ROOT/gpurun_out/prof_slice.log 2>&1 || exit 1
grep -E "sblas" $GRAFT_REPO_ROOT/gpurun_out/prof_slice/run_kernel_stats.csv | cut -d, -f1-5 | sed 's/(sblas::[^"]*//;s/(int const[^"]*//'
