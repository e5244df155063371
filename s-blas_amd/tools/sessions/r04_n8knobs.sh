#!/bin/bash
# round 4: existing xsort layout switches on the N = 8 slice (and N = 4), cold spans
set -o pipefail
O=gpurun_out/r04_n8knobs; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos xsort > $O/$name.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d['cold_span_us']) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
run default X=1 && run wg512 SBLAS_XS_WG=512 && run unpaired SBLAS_XS_PAIR=0 && run static SBLAS_XS_DYN=0 \
  && run q1 SBLAS_XS_Q=1 && run q3 SBLAS_XS_Q=3 && run rows4096 SBLAS_XS_ROWS=4096 && run default2 X=1
