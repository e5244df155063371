#!/bin/bash
# round 4: panel count for the auto XCD panels (row split, CSR5)
set -o pipefail
O=gpurun_out/r04_panelsP; mkdir -p $O
for P in 2 3 4 6; do
  SBLAS_PANELS=$P timeout -k 10 300 python s-blas_amd/tools/bench_slice.py --worlds 1,2 --algos rowsplit,csr5 > $O/slice_P$P.jsonl 2>>$O/err.log || exit 1
  python3 -c "import json;print('P=$P', [(d['world'],d['algo'],d['cold_span_us']) for d in map(json.loads,open('$O/slice_P$P.jsonl'))])"
done
