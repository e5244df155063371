#!/bin/bash
# round 5: R-MAT item sizes -- the trace shows 204 solo narrow items of ~123 us
# and 48 wide pairs of ~40 us, one item per CU, so the wide CUs idle for the
# last two thirds; smaller caps (SBLAS_XS_WSTAR) let the per-XCD queues
# balance -> profiles/r05/rmat/
set -o pipefail
O=gpurun_out/r05_rmat2
mkdir -p $O
T="timeout -k 10 200"
for r in 1 2; do
for c in "def" "60000" "45000" "35000" "25000" "18000"; do
  if [ $c = def ]; then E="SBLAS_XS_DUMMY=0"; else E="SBLAS_XS_WSTAR=$c"; fi
  env $E SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix rmat --scale 21 --algo xsort --reps 8 --cold --scrub read > $O/w${c}_$r.txt 2>&1 || { tail -5 $O/w${c}_$r.txt; exit 1; }
  echo "$c: $(grep 'ranges,' $O/w${c}_$r.txt | cut -c1-140) | $(grep mean $O/w${c}_$r.txt)"
done
done
