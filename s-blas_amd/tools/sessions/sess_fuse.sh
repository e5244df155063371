#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for r in 1 2; do
for v in "SBLAS_XS_FUSE=0" "SBLAS_XS_FUSE=1"; do
  env $v $T 200 python s-blas_amd/tools/bench_slice.py --worlds 1,8 --algos xsort --reps 10 > gpurun_out/fz.log 2>&1 || { tail -5 gpurun_out/fz.log; exit 1; }
  echo "$v"; grep '^{' gpurun_out/fz.log | cut -c1-200
done
done
