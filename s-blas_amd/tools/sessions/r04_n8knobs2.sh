#!/bin/bash
# round 4: more xsort switches on the N = 8 slice (and N = 4), cold spans: no wide
# ranges (no reduce launch), fused reduce, 24-bit keys, claim unroll, lambda, ntstore
set -o pipefail
O=gpurun_out/r04_n8knobs2; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos xsort $EXTRA > $O/$name.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d.get('cold_span_us', d)) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
EXTRA=--floor run default X=1 && run nowide SBLAS_XS_NOWIDE=1 && run fuse SBLAS_XS_FUSE=1 && run k24 SBLAS_XS_K24=1 \
  && run u1 SBLAS_XS_U=1 && run u3 SBLAS_XS_U=3 && run lam05 SBLAS_XS_LAMBDA=0.5 && run lam2 SBLAS_XS_LAMBDA=2 \
  && run nt SBLAS_XS_NTSTORE=1 && run nowide_rows4096 SBLAS_XS_NOWIDE=1 SBLAS_XS_ROWS=4096 && run default2 X=1
