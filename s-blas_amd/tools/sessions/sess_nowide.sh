#!/bin/bash
# xsort layout A/B on config 2 (cold read scrub): default vs all-narrow variants
set -o pipefail
mkdir -p gpurun_out
R="timeout -k 5 90 python3 s-blas_amd/tools/spmv_one.py --reps 30 --cold --scrub read"
for i in 1 2; do
for v in "X=0" "SBLAS_XS_NOWIDE=1" "SBLAS_XS_NOWIDE=1 SBLAS_XS_ROWS=2048" "SBLAS_XS_NOWIDE=1 SBLAS_XS_Q=1" "SBLAS_XS_NOWIDE=1 SBLAS_XS_LAMBDA=2.0"; do
  echo -n "$v: "; env $v $R 2>/dev/null | tail -1 || exit 1
done
done
