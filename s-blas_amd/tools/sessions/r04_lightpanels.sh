#!/bin/bash
# round 4: XCD panels on configs[2]'s light-row ranks (nnz split: N = 4 rank 3, N = 8 rank 5)
# and heavy ranks (rank 0), CSR5 and row split, P = 2 / 4 forced vs auto
set -o pipefail
O=gpurun_out/r04_lightpanels; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos csr5,rowsplit --partition nnz --ranks 0,3,5 > $O/$name.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d['rank'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
run auto X=1 && run p2 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=2 && run p4 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=4
