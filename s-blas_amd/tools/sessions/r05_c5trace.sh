#!/bin/bash
# round 5: kernel trace of configs[2]'s CSR5 rank slices (N = 8, cost split)
# and of the N = 1 matrix -> profiles/r05/c5trace/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_c5trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 8 --ranks all --algos csr5 --partition cost --reps 4 > $O/slices8.jsonl 2> $O/slices8.err || { tail -5 $O/slices8.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run --output-format csv -- python3 s-blas_amd/tools/bench_slice.py --worlds 1 --algos csr5,rowsplit --reps 4 > $O/slices1.jsonl 2> $O/slices1.err || { tail -5 $O/slices1.err; exit 1; }
