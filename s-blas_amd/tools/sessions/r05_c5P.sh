#!/bin/bash
# round 5: XCD-panel counts for CSR5 / row split on configs[2]'s nnz-split rank
# slices (heavy and light) and on small cyclic slices, uniform matrix
# -> profiles/r05/c5P/ (sets build_csr5_plan's / the row split's panel rule)
set -o pipefail
O=gpurun_out/r05_c5P
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
N="--worlds 8,4 --partition nnz --ranks 0,3,7 --algos csr5,rowsplit"
S="--worlds 16,32 --ranks 0 --algos csr5,rowsplit"
for p in 0 2 4 8; do
  if [ $p = 0 ]; then E="SBLAS_CSR5_PANEL=0 SBLAS_RS_PANEL=0"; else E="SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=$p"; fi
  run nnz_p$p $E -- $N || exit 1
  run small_p$p $E -- $S || exit 1
done
run nnz_auto -- $N && run small_auto -- $S || exit 1
