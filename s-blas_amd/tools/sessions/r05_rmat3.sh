#!/bin/bash
# round 5: R-MAT narrow-range cost factor (SBLAS_XS_NFAC, experiment knob): solo
# narrow items ran ~3x their modelled cost against the wide pairs -> profiles/r05/rmat/
set -o pipefail
O=gpurun_out/r05_rmat3
mkdir -p $O
T="timeout -k 10 200"
for r in 1 2; do
for c in "def" "1.5" "1.0" "0.7" "0.5"; do
  if [ $c = def ]; then E="SBLAS_XS_DUMMY=0"; else E="SBLAS_XS_NFAC=$c"; fi
  env $E SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix rmat --scale 21 --algo xsort --reps 8 --cold --scrub read > $O/w${c}_$r.txt 2>&1 || { tail -5 $O/w${c}_$r.txt; exit 1; }
  echo "$c: $(grep 'ranges,' $O/w${c}_$r.txt | cut -c1-140) | $(grep mean $O/w${c}_$r.txt)"
done
done
