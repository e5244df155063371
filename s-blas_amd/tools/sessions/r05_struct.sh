#!/bin/bash
# round 5: xsort's plan on the structured stand-ins (SBLAS_XS_TIMING prints
# ranges / wide / empty wide sub-items) and forced-narrow / other kernels,
# cold -> profiles/r05/struct_plan/
set -o pipefail
O=gpurun_out/r05_struct_plan
mkdir -p $O
T="timeout -k 10 120"
for M in "stencil27 --grid 128" "stencil7 --grid 160" "rmat --scale 21"; do
  set -- $M
  SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/runs.txt 2>&1 || exit 1
  SBLAS_XS_TIMING=1 SBLAS_XS_NOWIDE=1 $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/runs.txt 2>&1 || exit 1
  $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo rowsplit --reps 8 --cold --scrub read >> $O/runs.txt 2>&1 || exit 1
  $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo csr5 --reps 8 --cold --scrub read >> $O/runs.txt 2>&1 || exit 1
done
grep -v "^xsort plan: [a-z0-9]* *[0-9.]* s$" $O/runs.txt
