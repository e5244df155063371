#!/bin/bash
# round 4: CSR5 panel count per slice class: configs[2]'s nnz split, every rank at
# N = 1 / 2 / 4 / 8, plain / P = 2 / P = 4 forced; R-MAT likewise
set -o pipefail
O=gpurun_out/r04_c5P; mkdir -p $O
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2,4,8 --algos csr5 --partition nnz --ranks all > $O/$name.jsonl 2>>$O/err.log || return 1
  env "$@" timeout -k 10 300 python s-blas_amd/tools/exp_rmat.py --algos csr5 --tag $name >> $O/rmat.jsonl 2>>$O/err.log || return 1
  echo "$name $(python3 -c "import json,sys;print([(d['world'],d['rank'],d['cold_span_us']) for d in map(json.loads,open('$O/$name.jsonl'))])")"
}
run plain SBLAS_CSR5_PANEL=0 && run p2 SBLAS_CSR5_PANEL=1 SBLAS_PANELS=2 && run p4 SBLAS_CSR5_PANEL=1 SBLAS_PANELS=4
cat $O/rmat.jsonl | python3 -c "import json,sys;[print(d['tag'],d['cold_span_us'],d['frac_8TBs']) for d in map(json.loads,sys.stdin)]"
