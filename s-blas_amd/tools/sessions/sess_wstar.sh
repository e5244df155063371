#!/bin/bash
# N = 8 slice: sub-item cost cap (SBLAS_XS_WSTAR) above the slot-filling default (~1e4)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 200"
for w in "" 15000 20000 30000 40000 60000; do
  echo "WSTAR=${w:-default}"
  if [ -n "$w" ]; then export SBLAS_XS_WSTAR=$w; else unset SBLAS_XS_WSTAR; fi; $T python3 s-blas_amd/tools/bench_slice.py --worlds 8 --algos xsort --reps 10 || exit 1
done
