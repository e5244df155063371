#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 120"
B="python3 s-blas_amd/tools/bench_slice.py --worlds 8 --reps 10"
echo base; $T $B --algos xsort,panel,rowsplit || exit 1
for v in "SBLAS_XS_ALLWIDE=1" "SBLAS_XS_ALLWIDE=1 SBLAS_XS_Q=1" "SBLAS_XS_NOWIDE=1" "SBLAS_XS_PAIR=0" "SBLAS_XS_WG=512" "SBLAS_XS_ALLWIDE=1 SBLAS_XS_WG=512"; do
  echo "$v"; env $v $T $B --algos xsort || exit 1
done
