#!/bin/bash
# round 4: xsort planner switches on the R-MAT graph (scale 21), cold spans
set -o pipefail
O=gpurun_out/r04_rmat2; mkdir -p $O
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --tag $tag >> $O/rmat.jsonl 2>>$O/err.log || return 1
}
run default X=1 && run lam05 SBLAS_XS_LAMBDA=0.5 && run lam2 SBLAS_XS_LAMBDA=2 && run wb05 SBLAS_XS_WBUDGET=0.5 \
  && run rows4096 SBLAS_XS_ROWS=4096 && run q1 SBLAS_XS_Q=1 && run q3 SBLAS_XS_Q=3 && run solo SBLAS_XS_SOLO=1 \
  && run unpaired SBLAS_XS_PAIR=0 && run nowide SBLAS_XS_NOWIDE=1 && run default2 X=1
python3 -c "
import json
for l in open('$O/rmat.jsonl'):
    d=json.loads(l); print(d['tag'], d['cold_span_us'], d['frac_8TBs'])"
