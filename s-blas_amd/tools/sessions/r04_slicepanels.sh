#!/bin/bash
# round 4: the XCD-panel choice on rank-0 slices (N = 2 / 4 / 8), CSR5 and row split,
# forced on and off (the auto rule turns panels on at >= 12M nnz only)
set -o pipefail
O=gpurun_out/r04_slicepanels; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 2,4,8 --algos csr5,rowsplit > $O/$name.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
run auto X=1 && run on SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 && run off SBLAS_CSR5_PANEL=0 SBLAS_RS_PANEL=0
