#!/bin/bash
# round 4: xsort on the R-MAT graph (scale 21) as generated and with its empty rows
# dropped (tools/exp_rmat.py), under the planner's layout switches
set -o pipefail
O=gpurun_out/r04_rmat; mkdir -p $O
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --compact --tag $tag >> $O/rmat.jsonl 2>>$O/err.log || return 1
}
run default X=1 && run allwide SBLAS_XS_ALLWIDE=1 && run allwide_k2 SBLAS_XS_ALLWIDE=1 SBLAS_XS_K=2 \
  && run k2 SBLAS_XS_K=2 && run default2 X=1
python3 -c "
import json
for l in open('$O/rmat.jsonl'):
    d=json.loads(l); print(d['tag'], d['matrix'], d['rows'], d['cold_span_us'], d['frac_8TBs'])"
