#!/bin/bash
# round 5: rocprofv3 kernel stats of rank 0's N = 8 slice (xsort, cold) and of
# its streaming floor probe -> profiles/r05/slice_floor/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_slicestats
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --ranks 0 --algos xsort --reps 8 --floor > $O/slice8.jsonl 2> $O/slice8.err || { tail -5 $O/slice8.err; exit 1; }
cat $O/slice8.jsonl | cut -c1-400
