#!/bin/bash
# round 5: kernel trace of the SpMM rank slices (C tile vs reduce) at N = 8,
# rows and grid -> profiles/r05/spmm_grid/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_grid3
mkdir -p $O
for sp in rows grid; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$sp -o run --output-format csv -- python3 s-blas_amd/tools/bench_spmm_slices.py --worlds 8 --reps 4 --split $sp > $O/slices8_$sp.jsonl 2> $O/slices8_$sp.err || { tail -5 $O/slices8_$sp.err; exit 1; }
  head -5 $O/prof_$sp/run_kernel_stats.csv | cut -c1-220
done
