#!/bin/bash
# xsort range-row cap and planner lambda at N = 1 (cold read-scrub), current kernel
set -o pipefail
R="timeout -k 5 60 python3 s-blas_amd/tools/spmv_one.py --reps 30 --cold --scrub read"
for v in "" "SBLAS_XS_ROWS=4096" "SBLAS_XS_ROWS=6144" "SBLAS_XS_LAMBDA=0.7" "SBLAS_XS_LAMBDA=1.4" ""; do
  echo -n "${v:-default}: "; env $v $R 2>/dev/null | tail -1 || exit 1
done
