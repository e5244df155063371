#!/bin/bash
# round 5: xsort compact light ranges (solo plans count only non-empty rows
# against the LDS rows; SBLAS_XS_COMPACT=0 is the previous layout): the
# xsort tests, then R-MAT 21 / 20 and config 2 / stencils (no solo: unchanged)
# alternating -> profiles/r05/compact/
set -o pipefail
O=gpurun_out/r05_compact
mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 600 python -u -m pytest tests/test_spmv_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "xsort or compact or empty or edge or ragged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for c in 0 1; do
    for M in "rmat --scale 21" "rmat --scale 20" "stencil27 --grid 128"; do
      SBLAS_XS_COMPACT=$c SBLAS_XS_TIMING=1 $T python s-blas_amd/tools/spmv_one.py --matrix $M --algo xsort --reps 8 --cold --scrub read >> $O/c${c}_$r.txt 2>&1 || { tail -5 $O/c${c}_$r.txt; exit 1; }
    done
    echo "compact $c: $(grep -h 'ranges,' $O/c${c}_$r.txt | sed 's/.*plan: //' | cut -c1-60 | tr '\n' '|') $(grep -h mean $O/c${c}_$r.txt | sed 's/.*mean/mean/' | cut -c1-16 | tr '\n' ' ')"
  done
done
