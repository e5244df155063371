#!/bin/bash
# round 5: re-tune on the uniform matrix (the rounds 1-4 knobs were set on the
# correlated generator, profiles/r05/gen/): xsort planner knobs at N = 1 / 8,
# and the XCD-panel choice of CSR5 / row split on the slices -> profiles/r05/sweep/
set -o pipefail
O=gpurun_out/r05_sweep
mkdir -p $O
run() { # tag env... -- args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py "$@" --reps 6 > $O/$tag.jsonl 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; return 1; }
  python3 -c "
import json,sys
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$tag', d['world'], d['algo'], d['cold_span_us'])"
}
X="--worlds 1,8 --ranks 0 --algos xsort"
run xs_default -- $X && \
run xs_lam05 SBLAS_XS_LAMBDA=0.5 -- $X && \
run xs_lam2 SBLAS_XS_LAMBDA=2 -- $X && \
run xs_lam4 SBLAS_XS_LAMBDA=4 -- $X && \
run xs_solo SBLAS_XS_SOLO=1 -- $X && \
run xs_unpaired SBLAS_XS_PAIR=0 -- $X && \
run xs_q1 SBLAS_XS_Q=1 -- $X && \
run xs_q4 SBLAS_XS_Q=4 -- $X && \
run xs_u2 SBLAS_XS_U=2 -- $X && \
run xs_wb05 SBLAS_XS_WBUDGET=0.5 -- $X && \
run xs_nowide SBLAS_XS_NOWIDE=1 -- $X && \
run xs_allwide SBLAS_XS_ALLWIDE=1 -- $X && \
run xs_static SBLAS_XS_DYN=0 -- $X || exit 1
C="--worlds 1,2,4,8 --ranks 0 --algos csr5"
R="--worlds 1,2,4,8 --ranks 0 --algos rowsplit"
run c5_plain SBLAS_CSR5_PANEL=0 -- $C && \
run c5_p2 SBLAS_CSR5_PANEL=1 SBLAS_PANELS=2 -- $C && \
run c5_p4 SBLAS_CSR5_PANEL=1 SBLAS_PANELS=4 -- $C && \
run c5_p8 SBLAS_CSR5_PANEL=1 SBLAS_PANELS=8 -- $C && \
run rs_plain SBLAS_RS_PANEL=0 -- $R && \
run rs_p2 SBLAS_RS_PANEL=1 SBLAS_PANELS=2 -- $R && \
run rs_p4 SBLAS_RS_PANEL=1 SBLAS_PANELS=4 -- $R && \
run rs_p8 SBLAS_RS_PANEL=1 SBLAS_PANELS=8 -- $R || exit 1
