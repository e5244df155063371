#!/bin/bash
# round 5: xsort all-wide layout on small slices, U = 2 / q = 1 A/B at N = 1
# (repeated, alternating), and the new 2M-entry panel rule on the slices
# -> profiles/r05/sweep2/
set -o pipefail
O=gpurun_out/r05_sweep2
mkdir -p $O
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py "$@" --reps 6 > $O/$tag.jsonl 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; return 1; }
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$tag', d['world'], d['rank'], d['algo'], d['local_nnz'], d['cold_span_us'])"
}
S="--worlds 2,4,8,16 --ranks 0 --algos xsort"
run xs_def -- $S && run xs_allwide SBLAS_XS_ALLWIDE=1 -- $S || exit 1
for i in 1 2 3; do
  run ab_def$i -- --worlds 1 --algos xsort && run ab_u2_$i SBLAS_XS_U=2 -- --worlds 1 --algos xsort && \
  run ab_q1_$i SBLAS_XS_Q=1 -- --worlds 1 --algos xsort || exit 1
done
run panels_auto -- --worlds 1,2,4,8,16 --ranks 0 --algos csr5,rowsplit && \
run panels_nnz_auto -- --worlds 8,4 --partition nnz --ranks all --algos csr5 && \
run panels_cost3 -- --worlds 8,4 --partition cost --row-cost 3 --ranks all --algos csr5 || exit 1
