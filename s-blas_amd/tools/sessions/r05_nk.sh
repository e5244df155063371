#!/bin/bash
# round 5: R-MAT's solo light items run ~3x their modelled cost against the
# wide pairs (profiles/r05/rmat/); SBLAS_XS_NK (experiment knob) scales the
# narrow cost on solo plans -> profiles/r05/nk/
set -o pipefail
O=gpurun_out/r05_nk
mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 300 python -u -m pytest tests/test_spmv_gpu.py -x -q --timeout 200 --timeout-method thread -k "empty or edge or ragged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SBLAS_XS_NK=3 timeout -k 10 300 python -u -m pytest tests/test_spmv_gpu.py -x -q --timeout 200 --timeout-method thread -k "empty or edge or ragged or xsort_solo" > $O/tests_nk3.log 2>&1 || { tail -30 $O/tests_nk3.log; exit 1; }
tail -1 $O/tests_nk3.log
for r in 1 2; do
  for k in 1 1.5 2 3 4; do
    for M in "rmat --scale 21" "rmat --scale 20"; do
      SBLAS_XS_NK=$k SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/k${k}_$r.txt 2>&1 || { tail -5 $O/k${k}_$r.txt; exit 1; }
    done
    echo "nk $k: $(grep -h 'ranges,' $O/k${k}_$r.txt | sed 's/.*plan: //' | cut -c1-50 | tr '\n' '|') $(grep -h mean $O/k${k}_$r.txt | sed 's/.*mean/mean/' | cut -c1-16 | tr '\n' ' ')"
  done
done
