#!/bin/bash
# round 4: panel count on the N = 4 / 8 slices (CSR5 and row split forced onto panels)
set -o pipefail
O=gpurun_out/r04_slicepanelsP; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos csr5,rowsplit > $O/$name.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
run p2 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=2 && run p3 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=3 \
  && run p4 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=4 && run p8 SBLAS_CSR5_PANEL=1 SBLAS_RS_PANEL=1 SBLAS_PANELS=8 \
  && run auto X=1
# configs[2]'s nnz partition: every rank's slice (heavy ranks, a mixed one, light ranks)
timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 4,8 --algos csr5,rowsplit,xsort --partition nnz --ranks all > $O/nnz_ranks.jsonl 2>>$O/err.log || exit 1
python3 -c "import json;print([(d['world'],d['rank'],d['algo'],d['local_rows'],d['cold_span_us']) for d in map(json.loads,open('$O/nnz_ranks.jsonl'))])"
